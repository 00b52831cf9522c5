"""ctypes wrapper of oracle/_build/libmsha_oracle.so (TEST INFRASTRUCTURE / CPU BASELINE).

Used by tests (as a checker) and by bench.py's cpu_baseline leg (timed on the host
cores).  Never imported by the product package.
"""
import ctypes as C
import os

import numpy as np

from . import build_oracle

_libs = {}


def lib(fp64=False):
    """The fp32 restatement (CPU baseline) or, fp64=True, the same source compiled with
    REAL = double (symbols *_f64), the checker of the full-size parity tests."""
    if fp64 not in _libs:
        path = build_oracle.LIB64 if fp64 else build_oracle.LIB
        if not os.path.exists(path):
            build_oracle.build()
        lb = C.CDLL(path)
        P, I64, I = C.c_void_p, C.c_int64, C.c_int
        R = C.c_double if fp64 else C.c_float
        sfx = "_f64" if fp64 else ""
        getattr(lb, "oracle_edge_attention_fwd" + sfx).argtypes = [I64, P, P, I, I, P, P, P, R,
                                                                   P, P, P]
        getattr(lb, "oracle_edge_attention_bwd_rows" + sfx).argtypes = [
            I64, P, P, I, I, P, P, P, P, P, P, P, P, R, P, P, P, P]
        getattr(lb, "oracle_csc_aggregate" + sfx).argtypes = [I64, P, P, P, I, I, P, P, P, P, P]
        getattr(lb, "oracle_num_threads" + sfx).restype = I
        _libs[fp64] = lb
    return _libs[fp64]


def _fn(name, fp64):
    return getattr(lib(fp64), name + ("_f64" if fp64 else ""))


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dt)


def threads():
    return lib().oracle_num_threads()


def edge_attention_fwd(rowptr, col, el, er, hc, slope=0.2, fp64=False, hs=None, colptr=None,
                       csc_row=None, csc_eid=None):
    """u (n, H, F), lse (n, H) of the fused forward; fp64=True: in double precision.
    With hs (and the CSC view colptr / csc_row / csc_eid): also v = att.T @ hs (m, H, F),
    returned third (the OursLayer3 core, Ablation.py:273-274)."""
    dt = np.float64 if fp64 else np.float32
    n, H = el.shape
    m, _, F = hc.shape
    rowptr, col = _c(rowptr, np.int32), _c(col, np.int32)
    el, er, hc = _c(el, dt), _c(er, dt), _c(hc, dt)
    u = np.empty((n, H, F), dt)
    lse = np.empty((n, H), dt)
    att = np.empty((len(col), H), dt) if hs is not None else None
    _fn("oracle_edge_attention_fwd", fp64)(n, _p(rowptr), _p(col), H, F, _p(el), _p(er),
                                           _p(hc), slope, _p(u), _p(lse), _p(att))
    if hs is None:
        return u, lse
    colptr, csc_row, csc_eid = (_c(x, np.int32) for x in (colptr, csc_row, csc_eid))
    v = np.empty((m, H, F), dt)
    _fn("oracle_csc_aggregate", fp64)(m, _p(colptr), _p(csc_row), _p(csc_eid), H, F, _p(att),
                                      None, _p(_c(hs, dt)), _p(v), None)
    return u, lse, v


def edge_attention_bwd(rowptr, col, colptr, csc_row, csc_eid, el, er, hc, lse, u, dU,
                       slope=0.2, fp64=False, hs=None, dV=None):
    """(d_el, d_er, d_hc) of the fused forward's u; fp64=True: in double precision.  With
    hs and dV (the v branch): (d_el, d_er, d_hc, d_hs)."""
    dt = np.float64 if fp64 else np.float32
    n, H = el.shape
    m, _, F = hc.shape
    E = len(col)
    args = [_c(x, np.int32) for x in (rowptr, col, colptr, csc_row, csc_eid)]
    rowptr, col, colptr, csc_row, csc_eid = args
    el, er, hc, lse, u, dU = (_c(x, dt) for x in (el, er, hc, lse, u, dU))
    d_el = np.empty((n, H), dt)
    de = np.empty((E, H), dt)
    att = np.empty((E, H), dt)
    vb = hs is not None and dV is not None
    hs_c, dV_c = (_c(hs, dt), _c(dV, dt)) if vb else (None, None)
    d_hs = np.empty((n, H, F), dt) if vb else None
    _fn("oracle_edge_attention_bwd_rows", fp64)(n, _p(rowptr), _p(col), H, F, _p(el), _p(er),
                                                _p(hc), _p(lse), _p(u), _p(dU), _p(hs_c),
                                                _p(dV_c), slope, _p(d_el), _p(de), _p(att),
                                                _p(d_hs))
    d_hc = np.empty((m, H, F), dt)
    d_er = np.empty((m, H), dt)
    _fn("oracle_csc_aggregate", fp64)(m, _p(colptr), _p(csc_row), _p(csc_eid), H, F, _p(att),
                                      _p(de), _p(dU), _p(d_hc), _p(d_er))
    if vb:
        return d_el, d_er, d_hc, d_hs
    return d_el, d_er, d_hc
