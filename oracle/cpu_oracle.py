"""ctypes wrapper of oracle/_build/libmsha_oracle.so (TEST INFRASTRUCTURE / CPU BASELINE).

Used by tests (as a checker) and by bench.py's cpu_baseline leg (timed on the host
cores).  Never imported by the product package.
"""
import ctypes as C
import os

import numpy as np

from . import build_oracle

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = build_oracle.LIB
        if not os.path.exists(path):
            path = build_oracle.build()
        _lib = C.CDLL(path)
        P, I64, I = C.c_void_p, C.c_int64, C.c_int
        _lib.oracle_edge_attention_fwd.argtypes = [I64, P, P, I, I, P, P, P, C.c_float, P, P]
        _lib.oracle_edge_attention_bwd_rows.argtypes = [I64, P, P, I, I, P, P, P, P, P, P,
                                                        C.c_float, P, P, P]
        _lib.oracle_csc_aggregate.argtypes = [I64, P, P, P, I, I, P, P, P, P, P]
        _lib.oracle_num_threads.restype = I
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dt)


def threads():
    return lib().oracle_num_threads()


def edge_attention_fwd(rowptr, col, el, er, hc, slope=0.2):
    n, H = el.shape
    F = hc.shape[-1]
    rowptr, col = _c(rowptr, np.int32), _c(col, np.int32)
    el, er, hc = _c(el, np.float32), _c(er, np.float32), _c(hc, np.float32)
    u = np.empty((n, H, F), np.float32)
    lse = np.empty((n, H), np.float32)
    lib().oracle_edge_attention_fwd(n, _p(rowptr), _p(col), H, F, _p(el), _p(er), _p(hc), slope,
                                    _p(u), _p(lse))
    return u, lse


def edge_attention_bwd(rowptr, col, colptr, csc_row, csc_eid, el, er, hc, lse, u, dU,
                       slope=0.2):
    n, H = el.shape
    m, _, F = hc.shape
    E = len(col)
    args = [_c(x, np.int32) for x in (rowptr, col, colptr, csc_row, csc_eid)]
    rowptr, col, colptr, csc_row, csc_eid = args
    el, er, hc, lse, u, dU = (_c(x, np.float32) for x in (el, er, hc, lse, u, dU))
    d_el = np.empty((n, H), np.float32)
    de = np.empty((E, H), np.float32)
    att = np.empty((E, H), np.float32)
    lib().oracle_edge_attention_bwd_rows(n, _p(rowptr), _p(col), H, F, _p(el), _p(er), _p(hc),
                                         _p(lse), _p(u), _p(dU), slope, _p(d_el), _p(de),
                                         _p(att))
    d_hc = np.empty((m, H, F), np.float32)
    d_er = np.empty((m, H), np.float32)
    lib().oracle_csc_aggregate(m, _p(colptr), _p(csc_row), _p(csc_eid), H, F, _p(att), _p(de),
                               _p(dU), _p(d_hc), _p(d_er))
    return d_el, d_er, d_hc
