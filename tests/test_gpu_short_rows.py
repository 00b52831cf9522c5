"""The gather-layout kernels the library picks on short-row graphs (mean degree <= 8:
R15, bip1m): edge_attn_fwd_gl_kernel (er table, with the attention export of the
v-branch) and edge_attn_bwd_rows_gl_kernel (the row half of the backward, v-branch
included).  Against the oracle (fp64 on the stored values; fp32 1e-5, bf16 1e-2) and
against the score-layout kernels they replace (MSHA_FWD_GL=0 / MSHA_BWD_GL=0), with
virtual rows, rows longer than one chunk, hot columns and dropout (the kernels' Philox
masks injected)."""
import os

import numpy as np
import pytest
import torch

from gpu_helpers import random_counts, t, tol_close, virtual_csr
from oracle import gnn_oracle as O
from test_gpu_kernels import _keep_mask

pytestmark = pytest.mark.gpu

SHORT_CASES = [
    # (n, m, H, F, max_deg, extra): degrees uniform in 1..max_deg (mean <= 8)
    (500, 32, 2, 64, 6, dict(empty_rows=(3, 7), hot_col=4)),   # R15 shape
    (400, 32, 2, 64, 12, dict()),                               # many multi-chunk rows
    (300, 40, 8, 16, 5, dict(empty_rows=(0,))),
    (256, 32, 1, 64, 3, dict()),
    (200, 50, 4, 32, 7, dict(hot_col=11)),
    (128, 32, 8, 64, 4, dict(empty_rows=(5,))),                 # fp32 QPL 2: old kernels
]


def _run(MF, graph, el, er, hc, hs, dU, dV, p, seed, dev, dtype, gl):
    os.environ["MSHA_FWD_GL"] = os.environ["MSHA_BWD_GL"] = "1" if gl else "0"
    bip = MF.BIP
    MF.BIP = False  # these cases test the general short-row kernels (test_gpu_bip.py: M <= 32)
    try:
        leaves = [t(el, dev).requires_grad_(True), t(er, dev).requires_grad_(True),
                  t(hc, dev, dtype).requires_grad_(True), t(hs, dev, dtype).requires_grad_(True)]
        u, v = MF.edge_attention(graph, *leaves[:3], hs=leaves[3], p=p, training=p > 0,
                                 seed=seed)
        torch.autograd.backward([u, v], [t(dU, dev, dtype), t(dV, dev, dtype)])
        return [u.detach(), v.detach()] + [x.grad for x in leaves]
    finally:
        MF.BIP = bip
        os.environ.pop("MSHA_FWD_GL", None)
        os.environ.pop("MSHA_BWD_GL", None)


@pytest.mark.parametrize("case", SHORT_CASES, ids=lambda c: f"n{c[0]}m{c[1]}H{c[2]}F{c[3]}d{c[4]}")
@pytest.mark.parametrize("p", [0.0, 0.3])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_short_rows_vs_oracle_and_score_layout(cuda, msha, case, p, dtype):
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    n, m, H, F, max_deg, kw = case
    rng = np.random.default_rng(n + 13 * H + F)
    c = random_counts(rng, n, m, max_deg, **kw)
    rowptr, col, empty = virtual_csr(c)
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    hs = rng.standard_normal((n, H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    dV = rng.standard_normal((m, H, F)).astype(np.float32)
    graph = Graph.from_dense(t(c, cuda))
    assert graph.n_edges <= 8 * n  # the short-row dispatch
    seed = 23
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    got = _run(MF, graph, el, er, hc, hs, dU, dV, p, seed, cuda, dtype, True)
    old = _run(MF, graph, el, er, hc, hs, dU, dV, p, seed, cuda, dtype, False)
    st = lambda x: t(x, cuda, dtype).double().cpu().numpy()  # noqa: E731  stored values
    keep = _keep_mask(graph.n_edges, H, p, seed, cuda)
    ref = O.edge_aggregate_fwd(rowptr, col, el.astype(np.float64), er.astype(np.float64), st(hc),
                               hs=st(hs), keep=keep, p=p, rowflag=empty)
    bw = O.edge_aggregate_bwd(rowptr, col, ref, st(hc), st(dU), hs=st(hs), dV=st(dV), keep=keep,
                              p=p)
    names = ("u", "v", "d_el", "d_er", "d_hc", "d_hs")
    refs = (ref["u"], ref["v"], bw["d_el"], bw["d_er"], bw["d_hc"], bw["d_hs"])
    for name, a, b, r in zip(names, got, old, refs):
        rt = max(tol, 1e-4) if name in ("d_el", "d_er") else tol
        tol_close(a.float().cpu().numpy(), r, rt, tol)
        tol_close(a.float().cpu().numpy(), b.float().cpu().numpy(), rt, tol)
