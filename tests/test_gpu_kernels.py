"""GPU parity of the HIP kernels against the CPU oracle (oracle/gnn_oracle.py).

Index/graph outputs are checked bit-exact; attention weights to 1e-5 absolute and
embeddings / gradients to 1e-5 relative (fp32, BASELINE.json north_star), with a
scale-relative absolute floor where magnitudes are large.
"""
import os

import numpy as np
import pytest
import torch

from conftest import golden
from gpu_helpers import bounded_close, edge_abs_terms, random_counts, t, tol_close, virtual_csr
from oracle import gnn_oracle as O

pytestmark = pytest.mark.gpu

ATT_TOL = 1e-5   # attention weights, absolute
EMB_RTOL = 1e-5  # embeddings / aggregates, relative (+ 1e-5 * max|ref| floor)


# ------------------------------------------------------------------ graph build
def _r15_counts():
    g = golden("r15_graph.npz")
    n, m = int(g["n"]), int(g["m"])
    c = np.zeros((n, m), np.float32)
    c[O.edge_rows(g["rowptr"]), g["col"].astype(np.int64)] = g["cnt"]
    return g, c


def test_graph_from_dense_r15_bit_exact(cuda):
    from msha_gnn_amd.graph import Graph

    g, c = _r15_counts()
    gr = Graph.from_dense(t(c, cuda))
    assert gr.n_edges == 91283
    np.testing.assert_array_equal(gr.rowptr.cpu().numpy(), g["rowptr"])
    np.testing.assert_array_equal(gr.col.cpu().numpy(), g["col"].astype(np.int32))
    assert int(gr.rowflag.sum()) == 0
    colptr, perm = O.csr_to_csc(g["rowptr"], g["col"].astype(np.int32), 32)
    np.testing.assert_array_equal(gr.colptr.cpu().numpy(), colptr)
    np.testing.assert_array_equal(gr.csc_eid.cpu().numpy(), perm)
    np.testing.assert_array_equal(gr.csc_row.cpu().numpy(), O.edge_rows(g["rowptr"])[perm])


def test_graph_from_dense_virtual_rows(cuda):
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(1)
    c = random_counts(rng, 700, 90, 12, empty_rows=(0, 5, 699), hot_col=3, full_rows=(7,))
    gr = Graph.from_dense(t(c, cuda))
    rowptr, col, empty = virtual_csr(c)
    np.testing.assert_array_equal(gr.rowptr.cpu().numpy(), rowptr)
    np.testing.assert_array_equal(gr.col.cpu().numpy(), col)
    np.testing.assert_array_equal(gr.rowflag.cpu().numpy().astype(bool), empty)
    colptr, perm = O.csr_to_csc(rowptr, col, 90)
    np.testing.assert_array_equal(gr.colptr.cpu().numpy(), colptr)
    np.testing.assert_array_equal(gr.csc_eid.cpu().numpy(), perm)


def test_inter_adjacency_and_normalize(cuda, msha):
    z = golden("sub512.npz")
    fl = torch.as_tensor(z["flows"], device=cuda)
    adj = msha.inter_adjacency(fl[:, 0], fl[:, 1], 512, 32)
    np.testing.assert_array_equal(adj.cpu().numpy(), z["counts"])
    np.testing.assert_array_equal(msha.normalize_adjacency_matrix(adj).cpu().numpy(),
                                  z["adj_norm"])
    # full 2015 graph: flows expanded from the reference counts, normalised bit-exact
    g, c = _r15_counts()
    rows = O.edge_rows(g["rowptr"])
    src = np.repeat(rows, g["cnt"].astype(np.int64))
    dst = np.repeat(g["col"].astype(np.int64), g["cnt"].astype(np.int64))
    assert len(src) == int(g["n_flows"])
    perm = np.random.default_rng(0).permutation(len(src))
    adj = msha.inter_adjacency(t(src[perm], cuda, torch.int64), t(dst[perm], cuda, torch.int64),
                               int(g["n"]), 32)
    np.testing.assert_array_equal(adj.cpu().numpy(), c)
    norm = msha.normalize_adjacency_matrix(adj).cpu().numpy()
    np.testing.assert_array_equal(norm[c > 0], g["norm"])
    assert np.all(norm[c == 0] == 0)
    e = golden("edge_cases.npz")
    for k in ("norm_rand", "norm_zero_col"):
        out = msha.normalize_adjacency_matrix(t(e[k + "_in"], cuda)).cpu().numpy()
        np.testing.assert_array_equal(out, e[k + "_out"])  # NaN positions compare equal
    with pytest.raises(IndexError):
        msha.inter_adjacency(t([0, 600], cuda, torch.int64), t([0, 1], cuda, torch.int64), 512,
                             32)


def test_dropout_mask_statistics(cuda):
    from msha_gnn_amd import functional as MF

    k = MF.dropout_keep_mask(1 << 20, 0.5, 1234, cuda).cpu().numpy()
    assert abs(k.mean() - 0.5) < 3e-3
    k2 = MF.dropout_keep_mask(1 << 20, 0.5, 1234, cuda).cpu().numpy()
    assert np.array_equal(k, k2)
    k3 = MF.dropout_keep_mask(1 << 20, 0.5, 1235, cuda).cpu().numpy()
    assert abs((k == k3).mean() - 0.5) < 3e-3
    assert MF.dropout_keep_mask(4096, 0.0, 7, cuda).cpu().numpy().all()
    # word masks (the Ours intra masks): word 0 of the block keyed on each element is the
    # per-element mask; the four words are distinct streams of the right rate
    w = [MF.dropout_keep_mask(1 << 20, 0.5, 1234, cuda, offset=3, word=t).cpu().numpy()
         for t in range(4)]
    assert np.array_equal(w[0], MF.dropout_keep_mask(1 << 20, 0.5, 1234, cuda, offset=3)
                          .cpu().numpy())
    for t in range(4):
        assert abs(w[t].mean() - 0.5) < 3e-3
        for u in range(t):
            assert abs((w[t] == w[u]).mean() - 0.5) < 3e-3


# ------------------------------------------------------------- edge attention
def _edge_case(rng, n, m, H, F, max_deg, **kw):
    c = random_counts(rng, n, m, max_deg, **kw)
    rowptr, col, empty = virtual_csr(c)
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    hs = rng.standard_normal((n, H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    dV = rng.standard_normal((m, H, F)).astype(np.float32)
    return c, rowptr, col, empty, el, er, hc, hs, dU, dV


def _keep_mask(E, H, p, seed, dev):
    from msha_gnn_amd import functional as MF

    if p == 0:
        return None
    return MF.dropout_keep_mask(E * H, p, seed, dev).cpu().numpy().reshape(E, H).astype(bool)


CASES = [
    # (n, m, H, F, max_deg, extra)
    (300, 32, 2, 64, 30, dict(empty_rows=(0, 17), hot_col=5)),   # OursLayer3 x2 heads @R15 shape
    (200, 32, 1, 64, 8, dict(empty_rows=(3,))),                   # single head
    (150, 80, 1, 8, 80, dict(empty_rows=(0,), full_rows=(2,))),   # deg 80 > one wavefront
    (400, 400, 8, 16, 70, dict(hot_col=9)),                       # synthetic GAT shape
    (100, 50, 4, 32, 20, dict()),
    (64, 40, 8, 128, 12, dict(empty_rows=(1,))),                  # 1024-wide rows (QPL > 1)
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}m{c[1]}H{c[2]}F{c[3]}")
@pytest.mark.parametrize("p", [0.0, 0.3])
def test_edge_attention_fwd_bwd(cuda, msha, case, p):
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    n, m, H, F, max_deg, kw = case
    rng = np.random.default_rng(n * 7 + H)
    c, rowptr, col, empty, el, er, hc, hs, dU, dV = _edge_case(rng, n, m, H, F, max_deg, **kw)
    graph = Graph.from_dense(t(c, cuda))
    E = graph.n_edges
    seed = 99
    keep = _keep_mask(E, H, p, seed, cuda)
    d64 = lambda x: x.astype(np.float64)  # noqa: E731  fp64 reference on the fp32 inputs
    ref = O.edge_aggregate_fwd(rowptr, col, d64(el), d64(er), d64(hc), hs=d64(hs), keep=keep, p=p,
                               rowflag=empty)
    tel, ter, thc, ths = (t(x, cuda).requires_grad_(True) for x in (el, er, hc, hs))
    u, v = MF.edge_attention(graph, tel, ter, thc, hs=ths, p=p, training=p > 0, seed=seed)
    tol_close(u.detach().cpu().numpy(), ref["u"], EMB_RTOL, 1e-5)
    tol_close(v.detach().cpu().numpy(), ref["v"], EMB_RTOL, 1e-5)
    (u * t(dU, cuda)).sum().add_((v * t(dV, cuda)).sum()).backward()
    bw = O.edge_aggregate_bwd(rowptr, col, ref, d64(hc), d64(dU), hs=d64(hs), dV=d64(dV),
                              keep=keep, p=p)
    # score gradients: the fp32 forward-error bound of their sums (the softmax backward
    # cancels, sum_j att (g - D) = 0 before lrelu'; gpu_helpers.bounded_close)
    A = edge_abs_terms(rowptr, col, ref, hc, dU, hs=hs, dV=dV, keep=keep, p=p)
    bounded_close(tel.grad.cpu().numpy(), bw["d_el"], A["d_el"], A["n_row"], 1e-5, "d_el")
    bounded_close(ter.grad.cpu().numpy(), bw["d_er"], A["d_er"], A["n_col"], 1e-5, "d_er")
    tol_close(thc.grad.cpu().numpy(), bw["d_hc"], EMB_RTOL, 1e-5)
    tol_close(ths.grad.cpu().numpy(), bw["d_hs"], EMB_RTOL, 1e-5)


def _u_only_grads(MF, graph, el, er, hc, dU, p, seed, dev, dtype, fused, rowterms=None):
    """rowterms: True / False force the fused backward's row terms on / off
    (MSHA_ROWTERMS), None leaves the library's per-graph choice."""
    MF.FUSED_BWD = fused
    if rowterms is not None:
        os.environ["MSHA_ROWTERMS"] = "1" if rowterms else "0"
    if not fused:
        # the split backward these tests hold the fused one to, bit for bit: the
        # score-layout row pass (short-row graphs would take the gather-layout one, whose
        # d_el sums in another order; tests/test_gpu_short_rows.py checks that one)
        os.environ["MSHA_BWD_GL"] = "0"
    try:
        tel, ter = (t(x, dev).requires_grad_(True) for x in (el, er))
        thc = t(hc, dev, dtype).requires_grad_(True)
        u = MF.edge_attention(graph, tel, ter, thc, p=p, training=p > 0, seed=seed)
        u.backward(t(dU, dev, dtype))
        return u.detach(), tel.grad, ter.grad, thc.grad
    finally:
        MF.FUSED_BWD = True
        os.environ.pop("MSHA_ROWTERMS", None)
        os.environ.pop("MSHA_BWD_GL", None)


def _same_as_split(got, split, dtype=torch.float32):
    """Fused vs split backward: the per-edge scores and their sums (u, d_el, d_er) are
    the same bits; d_hc adds the same products in another order when the column pass
    runs head-per-lane (narrow heads): within a few ulps of the split sum."""
    for a, b, name in zip(got[:3], split[:3], ("u", "d_el", "d_er")):
        assert torch.equal(a, b), (name, dtype)
    a, b = got[3].float(), split[3].float()
    # a reordered fp32 sum of many terms moves by a few ulps of the largest partial
    # sums; a bf16 table may then round the other way (one bf16 ulp)
    bound = 16 * 2.0 ** -23 * (b.abs() + b.abs().amax())
    if dtype == torch.bfloat16:
        bound = bound + 2.0 ** -7 * b.abs()
    assert bool(((a - b).abs() <= bound).all()), float((a - b).abs().max())


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}m{c[1]}H{c[2]}F{c[3]}")
@pytest.mark.parametrize("p", [0.0, 0.3])
def test_edge_attention_fused_backward(cuda, msha, case, p):
    """u-only backward: msha_edge_attention_bwd_fused (one CSC pass) agrees with
    bwd_rows + csc_aggregate (bitwise but for d_hc's summation order) and the oracle."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    n, m, H, F, max_deg, kw = case
    rng = np.random.default_rng(n * 5 + H)
    c, rowptr, col, empty, el, er, hc, hs, dU, dV = _edge_case(rng, n, m, H, F, max_deg, **kw)
    graph = Graph.from_dense(t(c, cuda))
    seed = 7
    got = _u_only_grads(MF, graph, el, er, hc, dU, p, seed, cuda, torch.float32, True,
                        rowterms=False)
    split = _u_only_grads(MF, graph, el, er, hc, dU, p, seed, cuda, torch.float32, False)
    _same_as_split(got, split)
    keep = _keep_mask(graph.n_edges, H, p, seed, cuda)
    ref = O.edge_aggregate_fwd(rowptr, col, el, er, hc, keep=keep, p=p, rowflag=empty)
    bw = O.edge_aggregate_bwd(rowptr, col, ref, hc, dU, keep=keep, p=p)
    tol_close(got[1].cpu().numpy(), bw["d_el"], 1e-4, 1e-5)
    tol_close(got[2].cpu().numpy(), bw["d_er"], 1e-4, 1e-5)
    tol_close(got[3].cpu().numpy(), bw["d_hc"], EMB_RTOL, 1e-5)
    # row terms forced on (the large-graph path: d_el = dU . uc - D qc in the row pass,
    # no per-edge de): u, d_er, d_hc are the same bits, d_el matches the oracle
    rt = _u_only_grads(MF, graph, el, er, hc, dU, p, seed, cuda, torch.float32, True,
                       rowterms=True)
    for a, b, name in zip(rt, got, ("u", "d_el", "d_er", "d_hc")):
        if name != "d_el":
            assert torch.equal(a, b), name
    tol_close(rt[1].cpu().numpy(), bw["d_el"], 1e-4, 1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_rowterms_multichunk_and_virtual_rows(cuda, msha, dtype):
    """Row terms on the full 2015 graph (multi-chunk columns, virtual rows) with dropout:
    d_el from (uc, qc) within the north_star bar of the de row sum; everything else the
    same bits."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    g, c = _r15_counts()
    rng = np.random.default_rng(12)
    n, m, H, F = int(g["n"]), 32, 2, 64
    graph = Graph.from_dense(t(c, cuda))
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    base = _u_only_grads(MF, graph, el, er, hc, dU, 0.5, 3, cuda, dtype, True, rowterms=False)
    rt = _u_only_grads(MF, graph, el, er, hc, dU, 0.5, 3, cuda, dtype, True, rowterms=True)
    for a, b, name in zip(rt, base, ("u", "d_el", "d_er", "d_hc")):
        if name != "d_el":
            assert torch.equal(a, b), name
    tol_close(rt[1].cpu().numpy(), base[1].cpu().numpy(), 1e-5, 1e-5)


def test_edge_attention_fused_backward_bf16_multichunk(cuda, msha):
    """bf16 tables and the full 2015 graph's multi-chunk columns: fused == split."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    g, c = _r15_counts()
    rng = np.random.default_rng(11)
    n, m, H, F = int(g["n"]), 32, 2, 64
    graph = Graph.from_dense(t(c, cuda))
    assert graph._plan["n_multi"] > 0
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    for dtype in (torch.float32, torch.bfloat16):
        got = _u_only_grads(MF, graph, el, er, hc, dU, 0.5, 3, cuda, dtype, True, rowterms=False)
        split = _u_only_grads(MF, graph, el, er, hc, dU, 0.5, 3, cuda, dtype, False)
        _same_as_split(got, split, dtype)


WIDE_CASES = [
    # (H, F): shapes whose backward column pass takes one edge per wave-instruction
    # (EPI == 1) and so the buffer-load batch of COLS_WIDE_UG rows
    (4, 64),   # fp32: one 16-B quad per lane (QPL 1); bf16: EPI 2 (control)
    (8, 64),   # fp32 QPL 2; bf16 QPL 1
    (2, 128),  # fp32 QPL 1
    (8, 128),  # fp32 QPL 4; bf16 QPL 2
]


@pytest.mark.parametrize("H,F", WIDE_CASES, ids=lambda v: str(v))
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_edge_attention_fused_backward_wide_rows(cuda, msha, H, F, dtype):
    """Wide rows through the column pass's batched buffer loads, with ragged slot
    groups (nvalid < CE in the last group of a chunk: slots past it read 0) and split
    columns (a hot column over several chunks): fused == split, and fp32 == oracle."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(31 * H + F)
    n, m = 700, 48
    c, rowptr, col, empty, el, er, hc, hs, dU, dV = _edge_case(
        rng, n, m, H, F, 9, empty_rows=(2,), hot_col=7)
    graph = Graph.from_dense(t(c, cuda))
    assert graph._plan["n_multi"] > 0  # some column spans more than one chunk
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    for p in (0.0, 0.4):
        got = _u_only_grads(MF, graph, el, er, hc, dU, p, 5, cuda, tdt, True, rowterms=False)
        split = _u_only_grads(MF, graph, el, er, hc, dU, p, 5, cuda, tdt, False)
        _same_as_split(got, split, tdt)
        if dtype == "f32":
            keep = _keep_mask(graph.n_edges, H, p, 5, cuda)
            ref = O.edge_aggregate_fwd(rowptr, col, el, er, hc, keep=keep, p=p, rowflag=empty)
            bw = O.edge_aggregate_bwd(rowptr, col, ref, hc, dU, keep=keep, p=p)
            tol_close(got[1].cpu().numpy(), bw["d_el"], 1e-4, 1e-5)
            tol_close(got[2].cpu().numpy(), bw["d_er"], 1e-4, 1e-5)
            tol_close(got[3].cpu().numpy(), bw["d_hc"], EMB_RTOL, 1e-5)


@pytest.mark.parametrize("H,F", [(8, 16), (2, 64), (8, 64)], ids=lambda v: str(v))
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_edge_attention_fused_backward_pointer_loads(cuda, msha, H, F, dtype):
    """The column pass that tables of 2 GiB or more take (plain pointer loads, no buffer
    descriptors; forced here with MSHA_COLS_NOBUF=1): fused == split and fp32 == oracle,
    with ragged slot groups, an empty row and a column split over chunks."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(17 * H + F)
    n, m = 700, 48
    c, rowptr, col, empty, el, er, hc, hs, dU, dV = _edge_case(
        rng, n, m, H, F, 9, empty_rows=(2,), hot_col=7)
    graph = Graph.from_dense(t(c, cuda))
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    p = 0.4
    os.environ["MSHA_COLS_NOBUF"] = "1"
    try:
        got = _u_only_grads(MF, graph, el, er, hc, dU, p, 5, cuda, tdt, True, rowterms=False)
    finally:
        os.environ.pop("MSHA_COLS_NOBUF", None)
    split = _u_only_grads(MF, graph, el, er, hc, dU, p, 5, cuda, tdt, False)
    _same_as_split(got, split, tdt)
    if dtype == "f32":
        keep = _keep_mask(graph.n_edges, H, p, 5, cuda)
        ref = O.edge_aggregate_fwd(rowptr, col, el, er, hc, keep=keep, p=p, rowflag=empty)
        bw = O.edge_aggregate_bwd(rowptr, col, ref, hc, dU, keep=keep, p=p)
        tol_close(got[1].cpu().numpy(), bw["d_el"], 1e-4, 1e-5)
        tol_close(got[2].cpu().numpy(), bw["d_er"], 1e-4, 1e-5)
        tol_close(got[3].cpu().numpy(), bw["d_hc"], EMB_RTOL, 1e-5)


def test_edge_attention_weights_exported(cuda):
    """attd output of the forward vs oracle attention (absolute 1e-5)."""
    from msha_gnn_amd import _lib
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(3)
    c, rowptr, col, empty, el, er, hc, hs, dU, dV = _edge_case(rng, 500, 32, 2, 64, 30,
                                                               empty_rows=(4,))
    graph = Graph.from_dense(t(c, cuda))
    E, H, F = graph.n_edges, 2, 64
    u = torch.empty(500, H, F, device=cuda)
    lse = torch.empty(500, H, device=cuda)
    attd = torch.empty(E, H, device=cuda)
    tel, ter, thc = t(el, cuda), t(er, cuda), t(hc, cuda)  # keep alive across the launch
    _lib.call("msha_edge_attention_fwd", graph.desc, H, F, 0, tel.data_ptr(), ter.data_ptr(),
              thc.data_ptr(), 0.2, 0.0, 0, 0, u.data_ptr(), None, lse.data_ptr(), attd.data_ptr(),
              _lib.stream_handle())
    torch.cuda.synchronize()
    att, _, _ = O.edge_softmax_fwd(rowptr, col, el, er, rowflag=empty)
    np.testing.assert_allclose(attd.cpu().numpy(), att, rtol=0, atol=ATT_TOL)
    # virtual row: uniform over all 32 recipients
    s, e = rowptr[4], rowptr[5]
    np.testing.assert_allclose(attd.cpu().numpy()[s:e], 1.0 / 32, rtol=0, atol=1e-7)


def test_edge_attention_r15_full_graph(cuda):
    """Full 2015 graph, 2 heads x 64: multi-chunk CSC columns (nnz up to 5735)."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    g, c = _r15_counts()
    rng = np.random.default_rng(5)
    n, m, H, F = int(g["n"]), 32, 2, 64
    graph = Graph.from_dense(t(c, cuda))
    assert graph._plan["n_multi"] > 0
    rowptr, col = g["rowptr"], g["col"].astype(np.int32)
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    hs = rng.standard_normal((n, H, F)).astype(np.float32)
    ref = O.edge_aggregate_fwd(rowptr, col, el, er, hc, hs=hs)
    u, v = MF.edge_attention(graph, t(el, cuda), t(er, cuda), t(hc, cuda), hs=t(hs, cuda))
    tol_close(u.cpu().numpy(), ref["u"], EMB_RTOL, 1e-5)
    tol_close(v.cpu().numpy(), ref["v"], 1e-4, 1e-5)


# ----------------------------------------------------------------------- GAL
@pytest.mark.parametrize("p", [0.0, 0.5])
def test_gal_fwd_bwd(cuda, p):
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(11)
    n, m = 333, 80
    c = random_counts(rng, n, m, 70, empty_rows=(0, 9), full_rows=(3,))
    rowptr, col, empty = virtual_csr(c)
    h = rng.standard_normal((n, m)).astype(np.float32)
    dout = rng.standard_normal((n, m)).astype(np.float32)
    graph = Graph.from_dense(t(c, cuda))
    seed = 5
    keep = None
    if p > 0:
        keep = MF.dropout_keep_mask(n * m, p, seed, cuda).cpu().numpy().reshape(n, m).astype(bool)
    x = np.eye(m, dtype=np.float32)  # gal_fwd(x @ W) with W = h-part: use h directly
    out, _, att = O.gal_fwd(h, x, rowptr, col, keep=keep, p=p)
    th = t(h, cuda).requires_grad_(True)
    y = MF.gal(graph, th, p=p, training=p > 0, seed=seed)
    tol_close(y.detach().cpu().numpy(), out, 1e-6, 1e-6)
    y.backward(t(dout, cuda))
    ref_dh = O.gal_bwd(h, x, h, att, dout)["dh"]
    tol_close(th.grad.cpu().numpy(), ref_dh, 1e-5, 1e-6)


# --------------------------------------------------------------- MFMA projection
@pytest.mark.parametrize("M,N,K,trans_a,trans_b,splits", [
    (1000, 128, 128, False, False, 1), (257, 64, 64, False, False, 1),
    (64, 200, 96, False, True, 1), (128, 128, 20000, True, False, 64),
    (33, 40, 5000, False, False, 8),
    (64, 32, 10001, True, False, 16),  # K % 4 != 0 with row-contiguous operands (dW)
])
def test_gemm_f32(cuda, M, N, K, trans_a, trans_b, splits):
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((K, M) if trans_a else (M, K)).astype(np.float32)
    B = rng.standard_normal((N, K) if trans_b else (K, N)).astype(np.float32)
    tA, tB = t(A, cuda), t(B, cuda)
    tA = tA.t() if trans_a else tA
    tB = tB.t() if trans_b else tB
    C = MF.gemm(tA, tB, splits=splits).cpu().numpy()
    ref = (A.T if trans_a else A).astype(np.float64) @ (B.T if trans_b else B).astype(np.float64)
    tol_close(C, ref, 1e-5, 2e-6 * np.sqrt(K))
    C2 = MF.gemm(tA, tB, out=torch.as_tensor(C, device=cuda), accumulate=True,
                 splits=max(splits, 2)).cpu().numpy()
    tol_close(C2, 2 * ref, 1e-5, 2e-6 * np.sqrt(K))


@pytest.mark.parametrize("M,K,H,F", [(3000, 128, 8, 16), (517, 128, 2, 64), (80, 16, 1, 8),
                                     (300, 64, 4, 32), (200, 32, 1, 128),
                                     # resident-W kernel (skinny.hip): ragged last tile
                                     (5001, 64, 2, 64), (2050, 128, 4, 32),
                                     # the small-table kernel (M <= 256, small.hip) at feat
                                     # % 4 != 0 (its 4-piece score order)
                                     (32, 128, 1, 3), (32, 64, 2, 6), (32, 128, 4, 10),
                                     (32, 128, 2, 50)])
def test_project_scores_fwd_bwd(cuda, M, K, H, F):
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(M)
    X = rng.standard_normal((M, K)).astype(np.float32)
    W = rng.standard_normal((K, H * F)).astype(np.float32) / np.sqrt(K)
    al = rng.standard_normal((H, F)).astype(np.float32)
    ar = rng.standard_normal((H, F)).astype(np.float32)
    dh = rng.standard_normal((M, H * F)).astype(np.float32)
    dl = rng.standard_normal((M, H)).astype(np.float32)
    dr = rng.standard_normal((M, H)).astype(np.float32)
    ts = [t(x, cuda).requires_grad_(True) for x in (X, W, al, ar)]
    h, el, er = MF.project_scores(*ts, heads=H)
    # torch fp64 reference of the same op
    rs = [torch.tensor(x, dtype=torch.float64, requires_grad=True) for x in (X, W, al, ar)]
    rh = rs[0] @ rs[1]
    rel = (rh.view(M, H, F) * rs[2]).sum(-1)
    rer = (rh.view(M, H, F) * rs[3]).sum(-1)
    for got, want in ((h, rh), (el, rel), (er, rer)):
        tol_close(got.detach().cpu().numpy(), want.detach().numpy(), 1e-5, 1e-5)
    (h * t(dh, cuda)).sum().add_((el * t(dl, cuda)).sum()).add_((er * t(dr, cuda)).sum()) \
        .backward()
    ((rh * torch.tensor(dh, dtype=torch.float64)).sum() + (rel * torch.tensor(dl, dtype=torch.float64)).sum()
     + (rer * torch.tensor(dr, dtype=torch.float64)).sum()).backward()
    for got, want in zip(ts, rs):
        tol_close(got.grad.cpu().numpy(), want.grad.numpy(), 1e-4, 1e-5)


@pytest.fixture(params=["s3", "fp32"])
def wgrad_kernel(request, msha):
    """Run under each fp32 weight-gradient kernel: split-bf16 in registers (the default)
    and the exact-fp32 MFMA (msha_wgrad_kernel)."""
    from msha_gnn_amd import _lib

    lib = _lib.load()
    prev = lib.msha_wgrad_kernel({"s3": 3, "fp32": 1}[request.param])
    yield request.param
    lib.msha_wgrad_kernel(prev)


def _wgrad_bound(got, X, tot, name):
    """Every dW element within 4 sqrt(n) u sum_r |X[r, a]| |tot[r, n]| (n = rows + the
    split's six products and the block / slab reduce levels) of the fp64 product."""
    A = np.abs(X.astype(np.float64)).T @ np.abs(tot)
    ref = X.T.astype(np.float64) @ tot
    bounded_close(got, ref, A, X.shape[0] + 64, 0.0, name)


@pytest.mark.parametrize("operand,M,H,F,K,two", [(1, 100000, 8, 16, 128, True),
                                                 (1, 5000, 2, 64, 96, False),
                                                 (1, 50015, 2, 64, 128, True),
                                                 (0, 3000, 8, 16, 128, True),
                                                 (0, 39179, 2, 64, 128, True),
                                                 (0, 4096, 4, 32, 64, False),
                                                 (0, 2048, 1, 64, 64, True),
                                                 (0, 517, 1, 8, 40, False)])
def test_gemm_head_outer(cuda, wgrad_kernel, operand, M, H, F, K, two):
    """dX = (dh + de (x) a) W^T (operand 0) and dW = X^T (dh + de (x) a) (operand 1)
    with the sum folded into the operand loads, vs torch fp64.  Operand 0 with M >= 1024,
    D and the output width in {64, 128} runs the resident-W kernel (skinny.hip
    dx_kernel; one or two heads per lane's 32 columns), the rest the tiled GEMM."""
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(M + operand)
    D = H * F
    dh = rng.standard_normal((M, D)).astype(np.float32)
    de = rng.standard_normal((M, H)).astype(np.float32)
    a = rng.standard_normal((H, F)).astype(np.float32)
    de2 = rng.standard_normal((M, H)).astype(np.float32) if two else None
    a2 = rng.standard_normal((H, F)).astype(np.float32) if two else None
    tot = dh.astype(np.float64) + np.repeat(de, F, 1) * a.reshape(-1)
    if two:
        tot += np.repeat(de2, F, 1) * a2.reshape(-1)
    outer = (H, F, t(de, cuda), t(a, cuda), t(de2, cuda) if two else None,
             t(a2, cuda) if two else None)
    if operand == 0:
        W = rng.standard_normal((K, D)).astype(np.float32)
        got = MF.gemm_head_outer(t(dh, cuda), t(W, cuda).t(), 0, outer).cpu().numpy()
        ref = tot @ W.T.astype(np.float64)
    else:
        X = rng.standard_normal((M, K)).astype(np.float32)
        got = MF.gemm_head_outer(t(X, cuda).t(), t(dh, cuda), 1, outer).cpu().numpy()
        again = MF.gemm_head_outer(t(X, cuda).t(), t(dh, cuda), 1, outer).cpu().numpy()
        assert np.array_equal(got, again)  # block partials added in a fixed order
        ref = X.T.astype(np.float64) @ tot
        _wgrad_bound(got, X, tot, f"dW[{wgrad_kernel}]")
    tol_close(got, ref, 1e-5, 1e-5)


@pytest.mark.parametrize("M,H,F,two", [(100000, 8, 16, True), (1025, 3, 4, True),
                                       (700, 1, 3, False), (513, 4, 512, True), (1, 2, 8, True)])
def test_head_colsum(cuda, M, H, F, two):
    """out[h,f] = sum_r s[r,h] T[r,h*F+f]: float4 path, scalar path (F % 4 != 0),
    column tiles (H*F > 1024), ragged row blocks; deterministic across calls."""
    from msha_gnn_amd import _lib

    rng = np.random.default_rng(M + F)
    T = rng.standard_normal((M, H * F)).astype(np.float32)
    s1 = rng.standard_normal((M, H)).astype(np.float32)
    s2 = rng.standard_normal((M, H)).astype(np.float32) if two else None
    tT, t1 = t(T, cuda), t(s1, cuda)
    t2 = t(s2, cuda) if two else None
    o1 = torch.empty(H, F, device=cuda)
    o2 = torch.empty(H, F, device=cuda) if two else None
    ws = torch.empty(int(_lib.load().msha_head_colsum_workspace_size(M, H, F)) + 16,
                     dtype=torch.uint8, device=cuda)
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for _ in range(2):
        _lib.call("msha_head_colsum", M, H, F, 0, t1.data_ptr(), _lib.ptr(t2), tT.data_ptr(),
                  o1.data_ptr(), _lib.ptr(o2), ws.data_ptr(), ws.numel(), st)
        outs.append([o1.cpu().numpy().copy()] + ([o2.cpu().numpy().copy()] if two else []))
    T3 = T.astype(np.float64).reshape(M, H, F)
    refs = [np.einsum("mh,mhf->hf", s1.astype(np.float64), T3)]
    if two:
        refs.append(np.einsum("mh,mhf->hf", s2.astype(np.float64), T3))
    for got, ref in zip(outs[0], refs):
        tol_close(got, ref, 1e-5, 1e-5)
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)


# ------------------------------------------------------------------ link scoring
def test_link_predictor_matches_reference(cuda, msha):
    from msha_gnn_amd import layers

    z = golden("link.npz")
    # mlp1: num_layers=1 (still two Linears, one applied); other: an unknown predictor
    # string -> sigmoid(x_i * x_j), (B, F) (LLP.py:104-115)
    for mode, pred, nl in (("mlp", "mlp", 2), ("inner", "inner", 2), ("mlp1", "mlp", 1),
                           ("other", "dot", 2)):
        torch.manual_seed(4)
        lp = layers.LinkPredictor(pred, 32, 32, 1, nl, 0.0)
        for k, v in lp.state_dict().items():  # same init as the reference (bitwise)
            assert np.array_equal(v.numpy(), z[f"{mode}.init.{k}"]), k
        # the same module in fp64 torch (LLP.py:104-115 restated) on the same inputs and
        # init: the 1e-5 bar is held against it; the reference's own fp32 outputs and
        # gradients (fixture) pin it, within their fp32 rounding
        W64 = [(torch.tensor(z[f"{mode}.init.lins.{k}.weight"], dtype=torch.float64,
                             requires_grad=True),
                torch.tensor(z[f"{mode}.init.lins.{k}.bias"], dtype=torch.float64,
                             requires_grad=True)) for k in range(len(lp.lins))]
        xi64 = torch.tensor(z["x_i"], dtype=torch.float64, requires_grad=True)
        xj64 = torch.tensor(z["x_j"], dtype=torch.float64, requires_grad=True)
        x64 = xi64 * xj64
        if pred == "mlp":
            for w_, b_ in W64[:-1]:
                x64 = torch.relu(x64 @ w_.T + b_)
        elif pred == "inner":
            x64 = x64.sum(-1)
        y64 = torch.sigmoid(x64)
        y64.backward(torch.tensor(z[f"{mode}.dout"], dtype=torch.float64))
        lp = lp.to(cuda).train()
        xi = t(z["x_i"], cuda).requires_grad_(True)
        xj = t(z["x_j"], cuda).requires_grad_(True)
        y = lp(xi, xj)
        tol_close(y.detach().cpu().numpy(), y64.detach().numpy(), 1e-5, 1e-6)
        tol_close(y.detach().cpu().numpy(), z[f"{mode}.out"], 1e-5, 1e-6)
        y.backward(t(z[f"{mode}.dout"], cuda))
        tol_close(xi.grad.cpu().numpy(), xi64.grad.numpy(), 1e-5, 1e-5)
        tol_close(xj.grad.cpu().numpy(), xj64.grad.numpy(), 1e-5, 1e-5)
        tol_close(xi.grad.cpu().numpy(), z[f"{mode}.grad.x_i"], 1e-4, 1e-5)
        tol_close(xj.grad.cpu().numpy(), z[f"{mode}.grad.x_j"], 1e-4, 1e-5)
        assert y.shape == z[f"{mode}.out"].shape
        if pred == "mlp":
            tol_close(lp.lins[0].weight.grad.cpu().numpy(), W64[0][0].grad.numpy(), 1e-5, 1e-5)
            tol_close(lp.lins[0].bias.grad.cpu().numpy(), W64[0][1].grad.numpy(), 1e-5, 1e-5)
            tol_close(lp.lins[0].weight.grad.cpu().numpy(), z[f"{mode}.grad.lins.0.weight"],
                      1e-4, 1e-5)
            tol_close(lp.lins[0].bias.grad.cpu().numpy(), z[f"{mode}.grad.lins.0.bias"], 1e-4,
                      1e-5)
            assert lp.lins[1].weight.grad is None
        if mode == "other":
            assert all(p.grad is None for p in lp.parameters())


def test_link_predictor_deep_and_dropout(cuda, msha):
    """num_layers=3 (two used Linears) and dropout: vs oracle with the kernel's mask."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd import layers

    torch.manual_seed(0)
    lp = layers.LinkPredictor("mlp", 16, 24, 1, 3, 0.0).to(cuda).eval()
    rng = np.random.default_rng(2)
    xi, xj = (rng.standard_normal((300, 16)).astype(np.float32) for _ in range(2))
    y = lp(t(xi, cuda), t(xj, cuda)).detach().cpu().numpy()
    W0, b0 = lp.lins[0].weight.detach().cpu().numpy(), lp.lins[0].bias.detach().cpu().numpy()
    W1, b1 = lp.lins[1].weight.detach().cpu().numpy(), lp.lins[1].bias.detach().cpu().numpy()
    x = np.maximum((xi * xj) @ W0.T + b0, 0)
    x = np.maximum(x @ W1.T + b1, 0)
    tol_close(y, 1 / (1 + np.exp(-x)), 1e-5, 1e-6)
    # dropout on the fused layer: mask index = row * N + col
    W = t(W0, cuda)
    b = t(b0, cuda)
    out = MF.pair_layer(t(xi, cuda), t(xj, cuda), W, b, p=0.5, training=True, sigmoid=True,
                        seed=77).cpu().numpy()
    keep = MF.dropout_keep_mask(300 * 24, 0.5, 77, cuda).cpu().numpy().reshape(300, 24)
    z = np.maximum((xi * xj) @ W0.T + b0, 0) * keep * 2.0
    tol_close(out, 1 / (1 + np.exp(-z)), 1e-5, 1e-6)


@pytest.mark.parametrize("F", [32, 128])
def test_score_pairs_fused_gather(cuda, F):
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(F)
    n, P, hid = 5000, 20000, 64
    h = rng.standard_normal((n, F)).astype(np.float32)
    src = rng.integers(0, n, P)
    dst = rng.integers(0, n, P)
    W = (rng.standard_normal((hid, F)) / np.sqrt(F)).astype(np.float32)
    b = rng.standard_normal(hid).astype(np.float32)
    th, ts, td = t(h, cuda), t(src, cuda, torch.int64), t(dst, cuda, torch.int64)
    inner = MF.score_pairs(th, ts, td, "inner").cpu().numpy()
    tol_close(inner, O.score_pairs(h, src, dst, "inner"), 1e-5, 1e-6)
    mlp = MF.score_pairs(th, ts, td, "mlp", t(W, cuda), t(b, cuda)).cpu().numpy()
    tol_close(mlp, O.score_pairs(h, src, dst, "mlp", [(W, b), (None, None)]), 1e-5, 1e-6)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_score_pairs_index_rule(cuda, dt):
    """The fused gather follows torch's h[idx] (LLP.py:233): an index n or -(n+1) raises
    IndexError in both 'inner' and 'mlp'; -1 is row n-1; the 'inner' kernel given row
    counts scores a stray pair NaN and sets its error flag instead of reading past h."""
    from msha_gnn_amd import _lib
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(3)
    n, P, F, hid = 3000, 4096, 64, 64
    h = t(rng.standard_normal((n, F)).astype(np.float32), cuda, dt)
    W = t((rng.standard_normal((hid, F)) / 8).astype(np.float32), cuda, dt)
    b = t(rng.standard_normal(hid).astype(np.float32), cuda)
    src = torch.as_tensor(rng.integers(0, n, P), device=cuda)
    dst = torch.as_tensor(rng.integers(0, n, P), device=cuda)
    for mode in ("inner", "mlp"):
        args = (W, b) if mode == "mlp" else ()
        for bad in (n, -(n + 1), 10 * n):
            for which in (0, 1):
                s_, d_ = src.clone(), dst.clone()
                (s_, d_)[which][P // 2] = bad
                with pytest.raises(IndexError, match="out of bounds"):
                    MF.score_pairs(h, s_, d_, mode, *args)
        # negative indices wrap like torch's
        s_, d_ = src.clone(), dst.clone()
        s_[:7] = -1
        d_[100:110] = -torch.arange(1, 11, device=cuda)
        got = MF.score_pairs(h, s_, d_, mode, *args)
        want = MF.score_pairs(h, torch.where(s_ < 0, s_ + n, s_), torch.where(d_ < 0, d_ + n, d_),
                              mode, *args)
        assert torch.equal(got, want)
    # the kernel-side guard of the unchecked 'inner' path
    s_ = src.clone()
    s_[5], s_[77] = n, -1
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    out = torch.empty(P, device=cuda)
    _lib.call("msha_pair_inner_fwd_ex", P, F, MF._code(dt), h.data_ptr(), h.stride(0),
              s_.data_ptr(), n, h.data_ptr(), h.stride(0), dst.data_ptr(), n, err.data_ptr(),
              out.data_ptr(), MF._stream(h))
    assert int(err.item()) == 1
    o = out.cpu()
    assert torch.isnan(o[5]) and torch.isnan(o[77])
    ok = torch.ones(P, dtype=torch.bool)
    ok[[5, 77]] = False
    ref = MF.score_pairs(h, src, dst, "inner").cpu()
    assert torch.equal(o[ok], ref[ok])


# ------------------------------------------------------- BatchNorm + LeakyReLU
@pytest.mark.parametrize("R,C,dtype", [(32, 64, "f32"), (39179, 64, "f32"), (1000, 300, "f32"),
                                       (5000, 64, "bf16")])
def test_bn_lrelu_matches_torch(cuda, msha, R, C, dtype):
    """functional.bn_lrelu vs torch BatchNorm1d + LeakyReLU (train step: output, running
    statistics, num_batches_tracked, grads; then eval)."""
    import torch.nn as nn
    import torch.nn.functional as Fn
    from msha_gnn_amd import functional as MF

    torch.manual_seed(R)
    x0 = (torch.randn(R, C) * 3 + 1.5).to(cuda)
    dy = torch.randn(R, C, device=cuda)
    ref_bn = nn.BatchNorm1d(C).to(cuda).double()
    with torch.no_grad():
        ref_bn.weight.uniform_(0.5, 1.5)
        ref_bn.bias.uniform_(-0.5, 0.5)
    bn = nn.BatchNorm1d(C).to(cuda)
    bn.load_state_dict({k: v.float() for k, v in ref_bn.state_dict().items()})
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    if dtype == "bf16":
        x0 = x0.to(dt).float()
        dy = dy.to(dt).float()
    xr = x0.double().requires_grad_(True)
    yr = Fn.leaky_relu(ref_bn(xr), 0.2)
    yr.backward(dy.double())
    x = x0.to(dt).requires_grad_(True)
    y = MF.bn_lrelu(x, bn, 0.2)
    assert y.dtype == dt
    y.backward(dy.to(dt))
    tol = (1e-2, 1e-2) if dtype == "bf16" else (1e-5, 1e-5)
    tol_close(y.float().detach().cpu().numpy(), yr.detach().cpu().numpy(), *tol)
    tol_close(x.grad.float().cpu().numpy(), xr.grad.cpu().numpy(), *((1e-2, 1e-2) if dtype == "bf16" else (1e-4, 1e-5)))
    tol_close(bn.weight.grad.cpu().numpy(), ref_bn.weight.grad.cpu().numpy(), 1e-4, 1e-5)
    tol_close(bn.bias.grad.cpu().numpy(), ref_bn.bias.grad.cpu().numpy(), 1e-4, 1e-5)
    tol_close(bn.running_mean.cpu().numpy(), ref_bn.running_mean.cpu().numpy(), 1e-5, 1e-6)
    tol_close(bn.running_var.cpu().numpy(), ref_bn.running_var.cpu().numpy(), 1e-5, 1e-6)
    assert int(bn.num_batches_tracked) == int(ref_bn.num_batches_tracked) == 1
    bn.eval()
    ref_bn.eval()
    with torch.no_grad():
        ye = MF.bn_lrelu(x0.to(dt), bn, 0.2)
        yre = Fn.leaky_relu(ref_bn(x0.double()), 0.2)
    tol_close(ye.float().cpu().numpy(), yre.cpu().numpy(), *tol)


@pytest.mark.parametrize("n,m,D,dt", [(500, 32, 128, "f32"), (3000, 700, 64, "f32"),
                                      (800, 40, 32, "bf16")])
def test_spmm_both_directions(cuda, msha, n, m, D, dt):
    """functional.spmm A^T @ X and A @ Y (and their autograd) vs the oracle SpMM."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(n + D)
    c = random_counts(rng, n, m, 60, empty_rows=(1,), hot_col=0)
    adj = (c / np.maximum(c.sum(0, keepdims=True), 1)).astype(np.float32)
    graph = Graph.from_dense(t(adj, cuda))
    vals = graph.values(t(adj, cuda))
    rowptr, col, _ = virtual_csr(c)
    v_np = adj[O.edge_rows(rowptr), col].astype(np.float64)
    tdt = torch.bfloat16 if dt == "bf16" else torch.float32
    X = rng.standard_normal((n, D)).astype(np.float32)
    Y = rng.standard_normal((m, D)).astype(np.float32)
    if dt == "bf16":
        X = torch.as_tensor(X).to(tdt).float().numpy()
        Y = torch.as_tensor(Y).to(tdt).float().numpy()
    tX = t(X, cuda, tdt).requires_grad_(True)
    tY = t(Y, cuda, tdt).requires_grad_(True)
    a = MF.spmm(graph, vals, tX, transpose=True)
    b = MF.spmm(graph, vals, tY, transpose=False)
    tol = (1e-2, 1e-2) if dt == "bf16" else (1e-5, 1e-5)
    ra = O.spmm_t(rowptr, col, v_np, X.astype(np.float64), m)
    rb_ = O.spmm(rowptr, col, v_np, Y.astype(np.float64))
    tol_close(a.float().detach().cpu().numpy(), ra, *tol)
    tol_close(b.float().detach().cpu().numpy(), rb_, *tol)
    ga = rng.standard_normal((m, D)).astype(np.float32)
    gb = rng.standard_normal((n, D)).astype(np.float32)
    (a.float() * t(ga, cuda)).sum().add_((b.float() * t(gb, cuda)).sum()).backward()
    tol_close(tX.grad.float().cpu().numpy(), O.spmm(rowptr, col, v_np, ga.astype(np.float64)), *tol)
    tol_close(tY.grad.float().cpu().numpy(), O.spmm_t(rowptr, col, v_np, gb.astype(np.float64), m), *tol)


def test_edge_attention_fused_backward_slot_order(cuda, msha):
    """A graph whose de scratch (E x H fp32) exceeds 192 MB: with row terms off, the
    fused backward keeps de in CSC slot order (written contiguously, gathered through
    graph.csr_slot by the row sum): same bits as the split backward for u, d_el, d_er;
    d_hc within the reordered-sum bound.  With the library's default at this size (row
    terms on): u, d_er, d_hc the same bits as that, d_el within the fp32 bar of the
    split backward's row sum (it is exactly 0 where the row sum leaves rounding noise)."""
    import bench
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    n, e, H, F = 400_000, 6_400_000, 8, 16
    assert e * 4 * H >= 192 << 20
    rowptr, col = bench.synth_graph(n, e, seed=5)
    graph = Graph.from_csr(rowptr, col, n, cuda)
    assert graph.desc.csr_slot  # the slot map is built with the CSC view
    perm = graph.csr_slot[graph.csc_eid.long()]
    assert torch.equal(perm, torch.arange(e, dtype=torch.int32, device=cuda))
    rng = np.random.default_rng(2)
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((n, H)).astype(np.float32)
    hc = rng.standard_normal((n, H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    assert MF._lib.load().msha_edge_attention_rowterms_preferred(graph.desc, H, F, 0) == 1
    got = _u_only_grads(MF, graph, el, er, hc, dU, 0.2, 5, cuda, torch.float32, True,
                        rowterms=False)
    split = _u_only_grads(MF, graph, el, er, hc, dU, 0.2, 5, cuda, torch.float32, False)
    _same_as_split(got, split)
    rt = _u_only_grads(MF, graph, el, er, hc, dU, 0.2, 5, cuda, torch.float32, True)
    for a, b, name in zip(rt, got, ("u", "d_el", "d_er", "d_hc")):
        if name != "d_el":
            assert torch.equal(a, b), name
    tol_close(rt[1].cpu().numpy(), split[1].cpu().numpy(), 1e-5, 1e-5)


@pytest.mark.parametrize("K,N", [(128, 128), (64, 128), (128, 64), (64, 64)])
def test_pair_linear_resident_w(cuda, msha, K, N):
    """msha_pair_linear on the resident-W kernels (skinny.hip, fp32, both gathers,
    P >= 1024): hadamard of the gathered rows @ W^T + b, ReLU, dropout keyed on p * N + n
    (the library's Philox mask), sigmoid -- vs the oracle with that mask; a ragged last
    tile (P % 16 != 0).  Table row counts given -> pair_roll_kernel (one rolling row
    set, buffer gathers, line-major k order); unknown (0) -> pair_kernel.  Both against
    the oracle; they sum k in different orders, so they agree to rounding, not bits."""
    from msha_gnn_amd import _lib
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(K + N)
    n, P, p, seed = 3000, 4099, 0.5, 123
    h = rng.standard_normal((n, K)).astype(np.float32)
    src, dst = rng.integers(0, n, P), rng.integers(0, n, P)
    src[-1], dst[0] = n - 1, n - 1  # the tables' last rows (the buffer windows' ends)
    W = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    th, ts, td = t(h, cuda), t(src, cuda, torch.int64), t(dst, cuda, torch.int64)
    tW, tb = t(W, cuda), t(b, cuda)
    act = MF.ACT_BIAS | MF.ACT_RELU | MF.ACT_DROPOUT | MF.ACT_SIGMOID
    outs = []
    for rows in (n, 0):
        out = torch.full((P + 16, N), -7.0, device=cuda)  # 16 guard rows past the batch
        _lib.call("msha_pair_linear", P, K, N, th.data_ptr(), K, ts.data_ptr(), th.data_ptr(),
                  K, td.data_ptr(), rows, rows, tW.data_ptr(), tb.data_ptr(), act, p, seed, 0,
                  out.data_ptr(), _lib.stream_handle(cuda))
        o = out.cpu().numpy()
        assert (o[P:] == -7.0).all(), "a store past the batch"
        outs.append(o[:P])
    keep = MF.dropout_keep_mask(P * N, p, seed, cuda).cpu().numpy().reshape(P, N)
    z = np.maximum((h[src].astype(np.float64) * h[dst]) @ W.T.astype(np.float64) + b, 0)
    ref = 1 / (1 + np.exp(-(z * keep / (1 - p))))
    for o in outs:
        tol_close(o, ref, 1e-5, 1e-6)


@pytest.mark.parametrize("M,H,F,two", [(100000, 8, 16, True), (50015, 2, 64, True),
                                       (4096, 8, 16, False), (8191, 1, 128, True)])
def test_gemm_head_outer_colsum(cuda, wgrad_kernel, M, H, F, two):
    """msha_gemm_f32_head_outer_colsum: dW = X^T (dh + de (x) a [+ de2 (x) a2]) and the
    score-vector gradients sum_r de[r,h] T[r,h*F+f] from one pass over the rows, vs
    torch fp64 (1e-5), deterministic across calls; a shape outside the fused kernel
    (K != 128) is refused with nothing written."""
    from msha_gnn_amd import _lib
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(M + H)
    D, K = H * F, 128
    X = rng.standard_normal((M, K)).astype(np.float32)
    dh = rng.standard_normal((M, D)).astype(np.float32)
    T = rng.standard_normal((M, D)).astype(np.float32)
    de = rng.standard_normal((M, H)).astype(np.float32)
    a = rng.standard_normal((H, F)).astype(np.float32)
    de2 = rng.standard_normal((M, H)).astype(np.float32) if two else None
    a2 = rng.standard_normal((H, F)).astype(np.float32) if two else None
    outer = (H, F, t(de, cuda), t(a, cuda), t(de2, cuda) if two else None,
             t(a2, cuda) if two else None)
    runs = [MF._wgrad_colsum(t(X, cuda), t(dh, cuda), outer, t(T, cuda)) for _ in range(2)]
    assert runs[0] is not None
    for x, y in zip(runs[0], runs[1]):
        assert (x is None and y is None) or torch.equal(x, y)
    tot = dh.astype(np.float64) + np.repeat(de, F, 1) * a.reshape(-1)
    if two:
        tot += np.repeat(de2, F, 1) * a2.reshape(-1)
    dW, o1, o2 = runs[0]
    tol_close(dW.cpu().numpy(), X.T.astype(np.float64) @ tot, 1e-5, 1e-5)
    _wgrad_bound(dW.cpu().numpy(), X, tot, f"dW[{wgrad_kernel}]")
    T3 = T.astype(np.float64).reshape(M, H, F)
    tol_close(o1.cpu().numpy(), np.einsum("mh,mhf->hf", de.astype(np.float64), T3), 1e-5, 1e-5)
    if two:
        tol_close(o2.cpu().numpy(), np.einsum("mh,mhf->hf", de2.astype(np.float64), T3), 1e-5,
                  1e-5)
    else:
        assert o2 is None
    # K = 64 columns of X: not the fused kernel's shape
    assert MF._wgrad_colsum(t(X[:, :64], cuda), t(dh, cuda), outer, t(T, cuda)) is None


@pytest.mark.parametrize("M,F", [(1_000_000, 64), (50015, 64), (4096, 64), (50015, 32)])
def test_gemm_head_outer_colsum_w(cuda, msha, M, F):
    """msha_gemm_f32_head_outer_colsum_w: the score-vector gradients as (de^T X) W from the
    rows the weight gradient streams (h = X W never read), two heads: dW and both column
    sums elementwise within the fp32 bound of the fp64 sums over h = X W; deterministic.  Four
    heads (F = 32) are outside the W form: the same call takes the T form over h."""
    from msha_gnn_amd import _lib

    lib = _lib.load()
    prev = lib.msha_wgrad_kernel(3)  # the split kernel at every size (the W form's home)
    try:
        _colsum_w_case(cuda, M, F)
    finally:
        lib.msha_wgrad_kernel(prev)


def _colsum_w_case(cuda, M, F):
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(M + 7)
    H, K = 128 // F, 128
    X = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((K, H * F)) / np.sqrt(K)).astype(np.float32)
    dh = rng.standard_normal((M, H * F)).astype(np.float32)
    de = rng.standard_normal((M, H)).astype(np.float32)
    de2 = rng.standard_normal((M, H)).astype(np.float32)
    a = rng.standard_normal((H, F)).astype(np.float32)
    a2 = rng.standard_normal((H, F)).astype(np.float32)
    outer = (H, F, t(de, cuda), t(a, cuda), t(de2, cuda), t(a2, cuda))
    Xt, Wt = t(X, cuda), t(W, cuda)
    h = Xt @ Wt  # the forward's h (the W form never reads it)
    runs = [MF._wgrad_colsum(Xt, t(dh, cuda), outer, h, Wt) for _ in range(2)]
    for x, y in zip(runs[0], runs[1]):
        assert torch.equal(x, y)
    dW, o1, o2 = (r.cpu().numpy() for r in runs[0])
    tot = dh.astype(np.float64) + np.repeat(de, F, 1) * a.reshape(-1) + np.repeat(de2, F, 1) * a2.reshape(-1)
    _wgrad_bound(dW, X, tot, "dW")
    X64, W64 = X.astype(np.float64), W.astype(np.float64)
    h64 = (X64 @ W64).reshape(M, H, F)
    for e, o, nm in ((de, o1, "dal"), (de2, o2, "dar")):
        ref = np.einsum("mh,mhf->hf", e.astype(np.float64), h64)
        # |terms|: sum_r |e| sum_a |X| |W| (the rearranged sum's own magnitudes)
        A = np.einsum("mh,mhf->hf", np.abs(e).astype(np.float64),
                      (np.abs(X64) @ np.abs(W64)).reshape(M, H, F))
        bounded_close(o.reshape(H, F), ref, A, M + 2 * K, 0.0, nm)
