"""bf16 node tables (config C3: the same models in bf16) on the GPU.

Every reference here is fp64 on the SAME bf16-rounded inputs, so the comparison
measures the kernels (fp32 arithmetic, bf16 storage of their table outputs), not the
input quantisation.  Bars (north_star): bf16 tables (h, u, v, dh) within 1e-2
relative with a 1e-2 * max|ref| floor; fp32 outputs of fp32 arithmetic on bf16
inputs (scores, GEMM with fp32 C) to 1e-4.  The full MSHA core (ours_attention) and
the whole bf16 models (tests/test_gpu_parity_full.py) are likewise checked against
fp64 on the bf16-rounded values; no bf16 result is compared with the fp32 kernels."""
import numpy as np
import pytest
import torch

from conftest import golden
from gpu_helpers import t, tol_close, virtual_csr, random_counts
from oracle import gnn_oracle as O

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rb(x):
    """numpy fp32 -> bf16 (round to nearest even) -> fp32."""
    return torch.as_tensor(np.ascontiguousarray(x, dtype=np.float32)).to(BF).float().numpy()


# ------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("M,N,K,ta,tb,splits,cbf", [
    (1000, 128, 136, False, False, 1, True),    # projection: A k-fast, B n-fast
    (517, 64, 128, False, True, 1, False),      # dX: B = W^T (k-fast)
    (128, 128, 20000, True, False, 64, False),  # dW: A = X^T, B n-fast, split-K
    (128, 128, 5000, True, False, 8, True),     # dW, bf16 C
    (264, 72, 40, True, True, 1, False),        # both transposed, ragged tiles
])
def test_gemm_bf16(cuda, M, N, K, ta, tb, splits, cbf):
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(M + N + K)
    A = rb(rng.standard_normal((M, K)))
    B = rb(rng.standard_normal((K, N)))
    tA = t(A.T.copy(), cuda, BF).t() if ta else t(A, cuda, BF)
    tB = t(B.T.copy(), cuda, BF).t() if tb else t(B, cuda, BF)
    got = MF.gemm(tA, tB, splits=splits, out_dtype=BF if cbf else torch.float32)
    assert got.dtype == (BF if cbf else torch.float32)
    ref = A.astype(np.float64) @ B.astype(np.float64)
    if cbf:
        tol_close(got.float().cpu().numpy(), ref, 1e-2, 1e-2)
    else:
        tol_close(got.cpu().numpy(), ref, 1e-4, 1e-5)


@pytest.mark.parametrize("operand", [0, 1])
def test_gemm_bf16_head_outer(cuda, operand):
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(operand + 3)
    M, H, F, K = 3000, 8, 16, 128
    D = H * F
    dh = rb(rng.standard_normal((M, D)))
    de, de2 = rng.standard_normal((M, H)).astype(np.float32), rng.standard_normal((M, H)).astype(np.float32)
    a, a2 = rng.standard_normal((H, F)).astype(np.float32), rng.standard_normal((H, F)).astype(np.float32)
    tot = dh.astype(np.float64) + np.repeat(de, F, 1) * a.reshape(-1) + np.repeat(de2, F, 1) * a2.reshape(-1)
    outer = (H, F, t(de, cuda), t(a, cuda), t(de2, cuda), t(a2, cuda))
    if operand == 0:
        W = rb(rng.standard_normal((K, D)))
        got = MF.gemm_head_outer(t(dh, cuda, BF), t(W, cuda, BF).t(), 0, outer,
                                 out_dtype=torch.float32).cpu().numpy()
        ref = tot @ W.T.astype(np.float64)
    else:
        X = rb(rng.standard_normal((M, K)))
        got = MF.gemm_head_outer(t(X, cuda, BF).t(), t(dh, cuda, BF), 1, outer,
                                 out_dtype=torch.float32).cpu().numpy()
        ref = X.T.astype(np.float64) @ tot
    # the operand sum is rounded to bf16 before the MFMA: 1e-2
    tol_close(got, ref, 1e-2, 1e-2)


@pytest.mark.parametrize("M,K,H,F", [(3000, 128, 8, 16), (517, 128, 2, 64), (200, 64, 1, 128),
                                     (5001, 128, 2, 64), (2049, 64, 4, 16)])
def test_project_scores_bf16(cuda, M, K, H, F):
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(M)
    X = rb(rng.standard_normal((M, K)))
    W = rb(rng.standard_normal((K, H * F)) / np.sqrt(K))
    al = rng.standard_normal((H, F)).astype(np.float32)
    ar = rng.standard_normal((H, F)).astype(np.float32)
    tX, tW = t(X, cuda, BF).requires_grad_(True), t(W, cuda, BF).requires_grad_(True)
    tal, tar = t(al, cuda).requires_grad_(True), t(ar, cuda).requires_grad_(True)
    h, el, er = MF.project_scores(tX, tW, tal, tar, heads=H)
    assert h.dtype == BF and el.dtype == torch.float32
    rh = X.astype(np.float64) @ W.astype(np.float64)
    tol_close(h.float().detach().cpu().numpy(), rh, 1e-2, 1e-2)
    # el / er: the score dots of the STORED bf16 h (the row the edge kernels gather; the
    # skinny epilogue computes them in their order: msha_project_scores_row_order), fp32
    hs_ = h.float().detach().cpu().numpy().astype(np.float64).reshape(M, H, F)
    tol_close(el.detach().cpu().numpy(), (hs_ * al).sum(-1), 1e-5, 1e-6)
    tol_close(er.detach().cpu().numpy(), (hs_ * ar).sum(-1), 1e-5, 1e-6)
    # ... and within the bf16 bar of the exact product's scores
    tol_close(el.detach().cpu().numpy(), (rh.reshape(M, H, F) * al).sum(-1), 1e-2, 1e-2)
    dh = rb(rng.standard_normal((M, H * F)))
    dl = rng.standard_normal((M, H)).astype(np.float32)
    dr = rng.standard_normal((M, H)).astype(np.float32)
    (h.float() * t(dh, cuda)).sum().add_((el * t(dl, cuda)).sum()).add_((er * t(dr, cuda)).sum()) \
        .backward()
    tot = dh.astype(np.float64) + np.repeat(dl, F, 1) * al.reshape(-1) + np.repeat(dr, F, 1) * ar.reshape(-1)
    tol_close(tX.grad.float().cpu().numpy(), tot @ W.T.astype(np.float64), 1e-2, 1e-2)
    tol_close(tW.grad.float().cpu().numpy(), X.T.astype(np.float64) @ tot, 1e-2, 1e-2)
    hb = h.float().detach().cpu().numpy().astype(np.float64).reshape(M, H, F)  # the saved bf16 h
    tol_close(tal.grad.cpu().numpy(), np.einsum("mh,mhf->hf", dl, hb), 1e-4, 1e-5)
    tol_close(tar.grad.cpu().numpy(), np.einsum("mh,mhf->hf", dr, hb), 1e-4, 1e-5)


# ------------------------------------------------------------ edge kernels
EDGE_CASES = [
    (300, 32, 2, 64, 30, dict(empty_rows=(0, 17), hot_col=5)),  # OursLayer3 @R15 shape
    (400, 400, 8, 16, 70, dict(hot_col=9)),                      # synthetic GAT shape (C4)
    (150, 80, 1, 8, 80, dict(empty_rows=(0,), full_rows=(2,))),  # deg > one wavefront, F = 8
    (64, 40, 8, 128, 12, dict(empty_rows=(1,))),                 # 1024-wide rows
]


@pytest.mark.parametrize("case", EDGE_CASES, ids=lambda c: f"n{c[0]}m{c[1]}H{c[2]}F{c[3]}")
@pytest.mark.parametrize("p", [0.0, 0.3])
def test_edge_attention_bf16(cuda, msha, case, p):
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    n, m, H, F, max_deg, kw = case
    rng = np.random.default_rng(n * 11 + H)
    c = random_counts(rng, n, m, max_deg, **kw)
    rowptr, col, empty = virtual_csr(c)
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc, hs = rb(rng.standard_normal((m, H, F))), rb(rng.standard_normal((n, H, F)))
    dU, dV = rb(rng.standard_normal((n, H, F))), rb(rng.standard_normal((m, H, F)))
    graph = Graph.from_dense(t(c, cuda))
    E = graph.n_edges
    seed = 7
    keep = None
    if p > 0:
        keep = MF.dropout_keep_mask(E * H, p, seed, cuda).cpu().numpy().reshape(E, H).astype(bool)
    tel, ter = t(el, cuda).requires_grad_(True), t(er, cuda).requires_grad_(True)
    thc, ths = t(hc, cuda, BF).requires_grad_(True), t(hs, cuda, BF).requires_grad_(True)
    u, v = MF.edge_attention(graph, tel, ter, thc, hs=ths, p=p, training=p > 0, seed=seed)
    assert u.dtype == BF and v.dtype == BF
    ref = O.edge_aggregate_fwd(rowptr, col, el, er, hc, hs=hs, keep=keep, p=p, rowflag=empty)
    tol_close(u.float().detach().cpu().numpy(), ref["u"], 1e-2, 1e-2)
    tol_close(v.float().detach().cpu().numpy(), ref["v"], 1e-2, 1e-2)
    (u.float() * t(dU, cuda)).sum().add_((v.float() * t(dV, cuda)).sum()).backward()
    bw = O.edge_aggregate_bwd(rowptr, col, ref, hc, dU, hs=hs, dV=dV, keep=keep, p=p)
    tol_close(tel.grad.cpu().numpy(), bw["d_el"], 1e-2, 1e-2)
    tol_close(ter.grad.cpu().numpy(), bw["d_er"], 1e-2, 1e-2)
    tol_close(thc.grad.float().cpu().numpy(), bw["d_hc"], 1e-2, 1e-2)
    tol_close(ths.grad.float().cpu().numpy(), bw["d_hs"], 1e-2, 1e-2)


@pytest.mark.parametrize("p", [0.0, 0.3])
def test_ours_attention_bf16_vs_fp64(cuda, msha, p):
    """Full MSHA core (Ours.py:54-101) with bf16 tables against the dense fp64
    restatement on the same bf16-rounded tables and upstream gradients, with the
    kernels' dropout masks: u, v and every input gradient within 1e-2 (north_star)."""
    from test_gpu_ours import check_ours_attention_vs_dense

    check_ours_attention_vs_dense(cuda, p, BF, 1e-2, 1e-2)


# ------------------------------------------------------------------ modules
@pytest.mark.parametrize("mode", ["inner", "mlp"])
def test_score_pairs_bf16(cuda, mode):
    """Fused gather + LinkPredictor (LLP.py:104-115, :233) on a bf16 table (config C5)
    vs fp64 on the same bf16-rounded table/weights: sigmoid outputs within 1e-2."""
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(9)
    n, F, P, hidden = 3000, 128, 20000, 128
    h = rb(rng.standard_normal((n, F)) * 0.2)
    src, dst = rng.integers(0, n, P), rng.integers(0, n, P)
    th = t(h, cuda, BF)
    ts, td = torch.as_tensor(src, device=cuda), torch.as_tensor(dst, device=cuda)
    hd = h.astype(np.float64)
    if mode == "inner":
        got = MF.score_pairs(th, ts, td, "inner").cpu().numpy()
        ref = 1 / (1 + np.exp(-(hd[src] * hd[dst]).sum(1)))
    else:
        W = rb(rng.standard_normal((hidden, F)) / np.sqrt(F))
        b = rng.standard_normal(hidden).astype(np.float32) * 0.1
        got = MF.score_pairs(th, ts, td, "mlp", t(W, cuda, BF), t(b, cuda)).cpu().numpy()
        z = (hd[src] * hd[dst]) @ W.T.astype(np.float64) + b
        ref = 1 / (1 + np.exp(-np.maximum(z, 0)))
        # bf16 scores (what a bf16 LinkPredictor returns): the fp32 epilogue rounded once
        g16 = MF.score_pairs(th, ts, td, "mlp", t(W, cuda, BF), t(b, cuda), out_dtype=BF)
        assert g16.dtype == BF
        assert torch.equal(g16, torch.as_tensor(got, device=cuda).to(BF))
        tol_close(g16.float().cpu().numpy(), ref, 1e-2, 1e-2)
    tol_close(got, ref, 1e-2, 1e-2)


@pytest.mark.parametrize("out_bf16", [False, True])
def test_pair_linear_bf16_resident_w(cuda, out_bf16):
    """msha_pair_linear_bf16_ex on the resident-W bf16 kernel (skinny.hip pair_bf16_kernel,
    P >= 1024, ragged last tile): bf16(x_i * x_j) @ W^T + b, ReLU, the library's dropout
    mask, sigmoid -- vs fp64 on the same bf16 operands, 1e-2 (bf16 scores: one more
    rounding)."""
    from msha_gnn_amd import _lib
    from msha_gnn_amd import functional as MF

    rng = np.random.default_rng(21)
    n, K, N, P, p, seed = 2000, 128, 128, 3001, 0.3, 9
    h = rb(rng.standard_normal((n, K)) * 0.5)
    src, dst = rng.integers(0, n, P), rng.integers(0, n, P)
    W = rb(rng.standard_normal((N, K)) / np.sqrt(K))
    b = rng.standard_normal(N).astype(np.float32) * 0.1
    th = t(h, cuda, BF)
    ts, td = torch.as_tensor(src, device=cuda), torch.as_tensor(dst, device=cuda)
    tW, tb = t(W, cuda, BF), t(b, cuda)
    out = torch.empty(P, N, device=cuda, dtype=BF if out_bf16 else torch.float32)
    act = MF.ACT_BIAS | MF.ACT_RELU | MF.ACT_DROPOUT | MF.ACT_SIGMOID
    _lib.call("msha_pair_linear_bf16_ex", P, K, N, th.data_ptr(), K, ts.data_ptr(),
              th.data_ptr(), K, td.data_ptr(), tW.data_ptr(), tb.data_ptr(), act, p, seed, 0,
              1 if out_bf16 else 0, out.data_ptr(), _lib.stream_handle(cuda))
    keep = MF.dropout_keep_mask(P * N, p, seed, cuda).cpu().numpy().reshape(P, N)
    had = rb(h[src].astype(np.float32) * h[dst].astype(np.float32)).astype(np.float64)
    z = np.maximum(had @ W.T.astype(np.float64) + b, 0) * keep / (1 - p)
    tol_close(out.float().cpu().numpy(), 1 / (1 + np.exp(-z)), 1e-2, 1e-2)
