"""The C restatement (CPU baseline) agrees with the numpy oracle pinned to the reference."""
import numpy as np

from oracle import cpu_oracle
from oracle import gnn_oracle as O


def test_c_oracle_matches_numpy_oracle():
    rng = np.random.default_rng(0)
    n, m, H, F = 500, 300, 4, 8
    deg = rng.integers(1, 40, n)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    col = np.concatenate([np.sort(rng.choice(m, d, replace=False)) for d in deg]).astype(np.int32)
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    u, lse = cpu_oracle.edge_attention_fwd(rowptr, col, el, er, hc)
    ref = O.edge_aggregate_fwd(rowptr, col, el.astype(np.float64), er.astype(np.float64),
                               hc.astype(np.float64))
    np.testing.assert_allclose(u, ref["u"], rtol=1e-5, atol=1e-5)
    colptr, perm = O.csr_to_csc(rowptr, col, m)
    rows = O.edge_rows(rowptr)
    d_el, d_er, d_hc = cpu_oracle.edge_attention_bwd(rowptr, col, colptr, rows[perm], perm, el,
                                                     er, hc, lse, u, dU)
    bw = O.edge_aggregate_bwd(rowptr, col, ref, hc.astype(np.float64), dU.astype(np.float64))
    np.testing.assert_allclose(d_el, bw["d_el"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(d_er, bw["d_er"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(d_hc, bw["d_hc"], rtol=1e-4, atol=1e-5)


def test_c_oracle_fp64_matches_numpy_oracle():
    """The fp64 build (REAL = double, the full-size parity checker) agrees with the numpy
    oracle to fp64 rounding, including the backward."""
    rng = np.random.default_rng(1)
    n, m, H, F = 400, 250, 8, 16
    deg = rng.integers(1, 30, n)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    col = np.concatenate([np.sort(rng.choice(m, d, replace=False)) for d in deg]).astype(np.int32)
    el, er = rng.standard_normal((n, H)), rng.standard_normal((m, H))
    hc, dU = rng.standard_normal((m, H, F)), rng.standard_normal((n, H, F))
    u, lse = cpu_oracle.edge_attention_fwd(rowptr, col, el, er, hc, fp64=True)
    assert u.dtype == np.float64
    ref = O.edge_aggregate_fwd(rowptr, col, el, er, hc)
    np.testing.assert_allclose(u, ref["u"], rtol=1e-12, atol=1e-12)
    colptr, perm = O.csr_to_csc(rowptr, col, m)
    rows = O.edge_rows(rowptr)
    d_el, d_er, d_hc = cpu_oracle.edge_attention_bwd(rowptr, col, colptr, rows[perm], perm, el,
                                                     er, hc, lse, u, dU, fp64=True)
    bw = O.edge_aggregate_bwd(rowptr, col, ref, hc, dU)
    for got, want in ((d_el, bw["d_el"]), (d_er, bw["d_er"]), (d_hc, bw["d_hc"])):
        np.testing.assert_allclose(got, want, rtol=1e-10, atol=1e-11)


def test_c_oracle_v_branch_matches_numpy_oracle():
    """The OursLayer3 core with the v branch (u and v = att.T @ hs; the backward's hs . dV
    term and d_hs): the C restatement, fp64 and fp32, against the pinned numpy oracle --
    the bip1m CPU baseline (bench.py cpu_baseline_bip1m)."""
    rng = np.random.default_rng(2)
    n, m, H, F = 600, 32, 2, 16
    deg = rng.integers(1, 9, n)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    col = np.concatenate([np.sort(rng.choice(m, d, replace=False)) for d in deg]).astype(np.int32)
    el, er = rng.standard_normal((n, H)), rng.standard_normal((m, H))
    hc, hs = rng.standard_normal((m, H, F)), rng.standard_normal((n, H, F))
    dU, dV = rng.standard_normal((n, H, F)), rng.standard_normal((m, H, F))
    colptr, perm = O.csr_to_csc(rowptr, col, m)
    rows = O.edge_rows(rowptr)
    ref = O.edge_aggregate_fwd(rowptr, col, el, er, hc, hs=hs)
    bw = O.edge_aggregate_bwd(rowptr, col, ref, hc, dU, hs=hs, dV=dV)
    for fp64, rtol in ((True, 1e-10), (False, 1e-4)):
        cast = (lambda x: x) if fp64 else (lambda x: x.astype(np.float32))
        u, lse, v = cpu_oracle.edge_attention_fwd(rowptr, col, cast(el), cast(er), cast(hc),
                                                  fp64=fp64, hs=cast(hs), colptr=colptr,
                                                  csc_row=rows[perm], csc_eid=perm)
        np.testing.assert_allclose(u, ref["u"], rtol=rtol, atol=rtol)
        np.testing.assert_allclose(v, ref["v"], rtol=rtol, atol=rtol)
        d_el, d_er, d_hc, d_hs = cpu_oracle.edge_attention_bwd(
            rowptr, col, colptr, rows[perm], perm, cast(el), cast(er), cast(hc), lse, u,
            cast(dU), fp64=fp64, hs=cast(hs), dV=cast(dV))
        for got, want in ((d_el, bw["d_el"]), (d_er, bw["d_er"]), (d_hc, bw["d_hc"]),
                          (d_hs, bw["d_hs"])):
            np.testing.assert_allclose(got, want, rtol=rtol, atol=rtol * 10)
