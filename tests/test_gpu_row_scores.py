"""Scores from the gathered row (msha_edge_attention_fwd_rs / _bwd_fused_rs).

The u-only path given the score vector a_r computes er_j = hc_j . a_r from the rows
its gather lanes hold instead of gathering er per edge (Ablation.py:266-267: a[:F]
scores the aggregated table itself).  Checked against the oracle fed er = hc . a_r
in fp64 on the same stored values -- fp32 at the north_star 1e-5 bar, bf16 at 1e-2 --
over the edge-case graphs (virtual rows, degree > 64, hot columns, multi-chunk
columns), with and without dropout (the kernels' Philox masks injected), with and
without the row terms.  The er tensor passed alongside is deliberately wrong, so a
kernel that read it instead of recomputing would fail.
"""
import os

import numpy as np
import pytest
import torch

from gpu_helpers import t, tol_close
from oracle import gnn_oracle as O
from test_gpu_kernels import CASES, _edge_case, _keep_mask

pytestmark = pytest.mark.gpu
EMB_RTOL = 1e-5


def _rs_grads(MF, graph, el, hc, ar, dU, p, seed, dev, dtype, rowterms, er_hint=None):
    os.environ["MSHA_ROWTERMS"] = "1" if rowterms else "0"
    os.environ["MSHA_ROW_SCORES"] = "1"  # wherever supported (the default; pinned)
    try:
        tel = t(el, dev).requires_grad_(True)
        H, F = ar.shape
        # er handed to autograd: only its gradient matters on the row-score path
        ter = (t(er_hint, dev) if er_hint is not None
               else torch.full((hc.shape[0], H), 1e3, device=dev)).requires_grad_(True)
        thc = t(hc, dev, dtype).requires_grad_(True)
        u = MF.edge_attention(graph, tel, ter, thc, p=p, training=p > 0, seed=seed,
                              ar=t(ar, dev))
        u.backward(t(dU, dev, dtype))
        return u.detach(), tel.grad, ter.grad, thc.grad
    finally:
        os.environ.pop("MSHA_ROWTERMS", None)
        os.environ.pop("MSHA_ROW_SCORES", None)


def _supported(MF, graph, H, F, dtype):
    from msha_gnn_amd import _lib

    return bool(_lib.load().msha_edge_attention_row_scores_supported(
        graph.desc, H, F, 1 if dtype == torch.bfloat16 else 0))


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}m{c[1]}H{c[2]}F{c[3]}")
@pytest.mark.parametrize("p", [0.0, 0.3])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_row_scores_vs_oracle(cuda, msha, case, p, dtype):
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    n, m, H, F, max_deg, kw = case
    rng = np.random.default_rng(n * 3 + H)
    c, rowptr, col, empty, el, _er, hc, _hs, dU, _dV = _edge_case(rng, n, m, H, F, max_deg, **kw)
    ar = rng.standard_normal((H, F)).astype(np.float32)
    graph = Graph.from_dense(t(c, cuda))
    seed = 41
    tol = EMB_RTOL if dtype == torch.float32 else 1e-2
    # the oracle on the values the kernels read (bf16-rounded table), er = hc . a_r
    hc_s = t(hc, cuda, dtype).double().cpu().numpy()
    dU_s = t(dU, cuda, dtype).double().cpu().numpy()
    er64 = np.einsum("mhf,hf->mh", hc_s, ar.astype(np.float64))
    keep = _keep_mask(graph.n_edges, H, p, seed, cuda)
    ref = O.edge_aggregate_fwd(rowptr, col, el.astype(np.float64), er64, hc_s, keep=keep, p=p,
                               rowflag=empty)
    bw = O.edge_aggregate_bwd(rowptr, col, ref, hc_s, dU_s, keep=keep, p=p)
    er32 = er64.astype(np.float32)
    sup = _supported(MF, graph, H, F, dtype)
    # where the row-score kernels apply, the er handed over is never read (a wrong one
    # proves it); elsewhere (QPL > 1 shapes) the op falls back to reading er
    hint = None if sup else er32
    runs = {rt: _rs_grads(MF, graph, el, hc, ar, dU, p, seed, cuda, dtype, rt, er_hint=hint)
            for rt in (False, True)}
    for rt, got in runs.items():
        tol_close(got[0].float().cpu().numpy(), ref["u"], tol, tol)
        tol_close(got[1].cpu().numpy(), bw["d_el"], max(tol, 1e-4), tol)
        tol_close(got[2].cpu().numpy(), bw["d_er"], max(tol, 1e-4), tol)
        tol_close(got[3].float().cpu().numpy(), bw["d_hc"], tol, tol)
    # the row terms change d_el's summation only
    for a, b, name in zip(runs[True], runs[False], ("u", "d_el", "d_er", "d_hc")):
        if name != "d_el":
            assert torch.equal(a, b), name
    if sup:
        # the er-gather kernels fed the recomputed er agree to rounding (same scores up
        # to the dot's summation order)
        MF.ROW_SCORES = False
        try:
            base = _rs_grads(MF, graph, el, hc, ar, dU, p, seed, cuda, dtype, False, er_hint=er32)
        finally:
            MF.ROW_SCORES = True
        tol_close(runs[False][0].float().cpu().numpy(), base[0].float().cpu().numpy(), tol, tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_row_scores_r15_multichunk(cuda, msha, dtype):
    """The full 2015 graph (39k rows of ~2.3 edges, 32 columns split into many CSC
    chunks) with the reference's attention dropout, against the oracle."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph
    from test_gpu_kernels import _r15_counts

    g, c = _r15_counts()
    rng = np.random.default_rng(17)
    n, m, H, F = int(g["n"]), 32, 2, 64
    graph = Graph.from_dense(t(c, cuda))
    assert graph._plan["n_multi"] > 0
    el = rng.standard_normal((n, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    ar = (rng.standard_normal((H, F)) * 0.2).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    tol = EMB_RTOL if dtype == torch.float32 else 1e-2
    got = _rs_grads(MF, graph, el, hc, ar, dU, 0.5, 9, cuda, dtype, True)
    hc_s = t(hc, cuda, dtype).double().cpu().numpy()
    dU_s = t(dU, cuda, dtype).double().cpu().numpy()
    er64 = np.einsum("mhf,hf->mh", hc_s, ar.astype(np.float64))
    mask = c > 0
    rowptr, col = O.dense_to_csr(mask.astype(np.float32))
    keep = _keep_mask(graph.n_edges, H, 0.5, 9, cuda)
    ref = O.edge_aggregate_fwd(rowptr, col, el.astype(np.float64), er64, hc_s, keep=keep, p=0.5)
    bw = O.edge_aggregate_bwd(rowptr, col, ref, hc_s, dU_s, keep=keep, p=0.5)
    tol_close(got[0].float().cpu().numpy(), ref["u"], tol, tol)
    tol_close(got[1].cpu().numpy(), bw["d_el"], max(tol, 1e-4), tol)
    tol_close(got[2].cpu().numpy(), bw["d_er"], max(tol, 1e-4), tol)
    tol_close(got[3].float().cpu().numpy(), bw["d_hc"], tol, tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("H,F", [(8, 16), (2, 64), (4, 32)])
def test_projection_er_is_the_recomputed_er(cuda, msha, dtype, H, F):
    """msha_project_scores' er (row-order epilogue) is bit-identical to the er_j = h_j . a_r
    the row-score kernels recompute from the gathered row: the backward that reads this
    er (the tagged tensor) and the one that recomputes it from a_r (an untagged copy)
    give the same bits everywhere."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    n, K = 3000, 128
    rng = np.random.default_rng(H * F)
    deg = rng.integers(3, 20, n)
    rowptr = np.concatenate([[0], np.cumsum(deg)])
    col = np.concatenate([np.sort(rng.choice(n, d, replace=False)) for d in deg])
    graph = Graph.from_csr(rowptr, col, n, cuda)
    g = torch.Generator().manual_seed(H + F)
    X = torch.rand(n, K, generator=g).to(cuda, dtype)
    W = (torch.randn(K, H * F, generator=g) * K ** -0.5).to(cuda, dtype)
    al = torch.randn(H, F, generator=g).to(cuda)
    ar = torch.randn(H, F, generator=g).to(cuda)
    dU = torch.randn(n, H, F, generator=g).to(cuda, dtype)
    with torch.no_grad():
        h, el, er = MF.project_scores(X, W, al, ar, heads=H)
    assert getattr(er, "_msha_row_order", False)
    os.environ["MSHA_ROW_SCORES"] = "1"
    try:
        runs = []
        for er_in in (er, er.clone()):  # the clone carries no tag: recompute from a_r
            leaves = [el.clone().requires_grad_(True), er_in.requires_grad_(True),
                      h.view(n, H, F).clone().requires_grad_(True)]
            u = MF.edge_attention(graph, *leaves, ar=ar)
            u.backward(dU)
            runs.append([u.detach()] + [x.grad for x in leaves])
            er.requires_grad_(False)
    finally:
        os.environ.pop("MSHA_ROW_SCORES", None)
    for a, b, name in zip(*runs, ("u", "d_el", "d_er", "d_hc")):
        assert torch.equal(a, b), name
