"""Bipartite small-M kernels (msha_bip_attention_fwd/_bwd, csrc/edge_bip.hip): the
repo's adjacency shape, N sources x M <= 32 recipients (every shipped year; bip1m).
u, v, lse, the attention export and every gradient against the fp64 oracle on the
stored values (fp32 1e-5, bf16 1e-2) and against the general kernels they replace
(functional.BIP = False), with virtual rows, a hot column, full rows, dropout (the
kernels' Philox masks injected) and groups that straddle keep-bit pages."""
import numpy as np
import pytest
import torch

from gpu_helpers import bounded_close, edge_abs_terms, random_counts, t, tol_close, virtual_csr
from oracle import gnn_oracle as O
from test_gpu_kernels import _keep_mask

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["default", "mfma", "mfma_bwd32"])
def bip_path(request, msha, monkeypatch):
    """The library's size-based choice ("default": below 131,072 rows the mask forward and
    the CSR-walk backward) and the large-graph choice forced on every 2 x 64, M <= 32 graph
    ("mfma": msha_bip2_bwd_min_rows(0) with MSHA_BIP3_BWD32=0: the MFMA kernels of
    edge_bip3.hip, but the fp32 backward on edge_bip2.hip's mask kernel; "mfma_bwd32": the
    MFMA backward for fp32 too, the library's large-graph default since round 6)."""
    from msha_gnn_amd import _lib

    monkeypatch.setenv("MSHA_BIP3_BWD32", "1" if request.param == "mfma_bwd32" else "0")
    prev = _lib.fn("msha_bip2_bwd_min_rows")(-1 if request.param == "default" else 0)
    yield request.param
    _lib.fn("msha_bip2_bwd_min_rows")(prev)

CASES = [
    # (n, m, H, F, max_deg, extra); M * H <= 64 (one row's slots fit one group)
    (3000, 32, 2, 64, 6, dict(empty_rows=(3, 7, 2999), hot_col=4)),   # R15 shape
    (700, 32, 2, 64, 32, dict(full_rows=(1, 2, 3, 40))),             # 64-slot rows
    (900, 8, 8, 16, 5, dict(empty_rows=(0,))),                        # C4 head shape
    (400, 17, 1, 64, 4, dict(hot_col=16)),                            # V = 1, odd M
    (300, 16, 2, 128, 7, dict(empty_rows=(5,))),                      # V = 4
    (257, 16, 4, 32, 3, dict()),
    (5000, 32, 2, 64, 2, dict()),                                     # groups capped by rows
    (600, 16, 4, 64, 6, dict(empty_rows=(2,))),                       # four head blocks
]


def _run(MF, graph, el, er, hc, hs, dU, dV, p, seed, dev, dtype, bip):
    old = MF.BIP
    MF.BIP = bip
    try:
        leaves = [t(el, dev).requires_grad_(True), t(er, dev).requires_grad_(True),
                  t(hc, dev, dtype).requires_grad_(True), t(hs, dev, dtype).requires_grad_(True)]
        u, v = MF.edge_attention(graph, *leaves[:3], hs=leaves[3], p=p, training=p > 0,
                                 seed=seed)
        torch.autograd.backward([u, v], [t(dU, dev, dtype), t(dV, dev, dtype)])
        torch.cuda.synchronize()
        return [u.detach(), v.detach()] + [x.grad for x in leaves]
    finally:
        MF.BIP = old


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}m{c[1]}H{c[2]}F{c[3]}d{c[4]}")
@pytest.mark.parametrize("p", [0.0, 0.5])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_bip_vs_oracle_and_general(cuda, msha, bip_path, case, p, dtype):
    from msha_gnn_amd import _lib
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    n, m, H, F, max_deg, kw = case
    rng = np.random.default_rng(n + 7 * H + F)
    c = random_counts(rng, n, m, max_deg, **kw)
    rowptr, col, empty = virtual_csr(c)
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    hs = rng.standard_normal((n, H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    dV = rng.standard_normal((m, H, F)).astype(np.float32)
    graph = Graph.from_dense(t(c, cuda))
    code = 1 if dtype == torch.bfloat16 else 0
    assert _lib.load().msha_bip_supported(graph.desc, H, F, code) == 1
    seed = 31
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    got = _run(MF, graph, el, er, hc, hs, dU, dV, p, seed, cuda, dtype, True)
    gen = _run(MF, graph, el, er, hc, hs, dU, dV, p, seed, cuda, dtype, False)
    st = lambda x: t(x, cuda, dtype).double().cpu().numpy()  # noqa: E731  stored values
    keep = _keep_mask(graph.n_edges, H, p, seed, cuda)
    ref = O.edge_aggregate_fwd(rowptr, col, el.astype(np.float64), er.astype(np.float64), st(hc),
                               hs=st(hs), keep=keep, p=p, rowflag=empty)
    bw = O.edge_aggregate_bwd(rowptr, col, ref, st(hc), st(dU), hs=st(hs), dV=st(dV), keep=keep,
                              p=p)
    names = ("u", "v", "d_el", "d_er", "d_hc", "d_hs")
    refs = (ref["u"], ref["v"], bw["d_el"], bw["d_er"], bw["d_hc"], bw["d_hs"])
    # every element of every output within rtol |ref| + 4 sqrt(n) 2^-24 A (gpu_helpers.
    # bounded_close, A the absolute terms of its sum; no fraction clause)
    A = edge_abs_terms(rowptr, col, ref, st(hc), st(dU), hs=st(hs), dV=st(dV), keep=keep, p=p)
    per = {"u": "n_row", "d_hs": "n_row", "d_el": "n_row", "v": "n_col", "d_hc": "n_col",
           "d_er": "n_col"}
    for name, a, b, r in zip(names, got, gen, refs):
        bounded_close(a.float().cpu().numpy(), r, A[name], A[per[name]], tol, name)
        bounded_close(b.float().cpu().numpy(), r, A[name], A[per[name]], tol, name + " (general)")


def test_bip_raw_abi_lse_attd_deterministic(cuda, msha, bip_path):
    """The C ABI directly: lse and the attention export against the oracle, u-only
    (no hs) forward, and bitwise-identical repeats (wave- and block-ordered sums)."""
    from msha_gnn_amd import _lib
    from msha_gnn_amd.graph import Graph

    n, m, H, F = 5000, 32, 2, 64
    rng = np.random.default_rng(5)
    c = random_counts(rng, n, m, 5, empty_rows=(11,), hot_col=0)
    rowptr, col, empty = virtual_csr(c)
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    hs = rng.standard_normal((n, H, F)).astype(np.float32)
    graph = Graph.from_dense(t(c, cuda))
    g = graph.desc
    L = _lib.load()
    E = graph.n_edges
    ws = torch.empty(int(L.msha_bip_workspace_size(g, H, F)), dtype=torch.uint8, device=cuda)
    s = _lib.stream_handle(cuda)
    el_d, er_d, hc_d, hs_d = t(el, cuda), t(er, cuda), t(hc, cuda), t(hs, cuda)
    outs = []
    for rep in range(2):
        u = torch.empty(n, H, F, device=cuda)
        v = torch.empty(m, H, F, device=cuda)
        lse = torch.empty(n, H, device=cuda)
        attd = torch.empty(E, H, device=cuda)
        _lib.call("msha_bip_attention_fwd", g, H, F, 0, el_d.data_ptr(), er_d.data_ptr(),
                  hc_d.data_ptr(), hs_d.data_ptr(), 0.2, 0.0, 0, 0, u.data_ptr(), None,
                  lse.data_ptr(), attd.data_ptr(), v.data_ptr(), ws.data_ptr(), ws.numel(), s)
        outs.append((u, v, lse, attd))
    u1 = torch.empty(n, H, F, device=cuda)
    lse1 = torch.empty(n, H, device=cuda)
    _lib.call("msha_bip_attention_fwd", g, H, F, 0, el_d.data_ptr(), er_d.data_ptr(),
              hc_d.data_ptr(), None, 0.2, 0.0, 0, 0, u1.data_ptr(), None, lse1.data_ptr(), None,
              None, None, 0, s)
    torch.cuda.synchronize()
    ref = O.edge_aggregate_fwd(rowptr, col, el.astype(np.float64), er.astype(np.float64),
                               hc.astype(np.float64), hs=hs.astype(np.float64), rowflag=empty)
    u, v, lse, attd = (x.cpu().numpy() for x in outs[0])
    tol_close(u, ref["u"], 1e-5, 1e-5)
    tol_close(v, ref["v"], 1e-5, 1e-5)
    np.testing.assert_allclose(attd, ref["att"], atol=1e-5)
    sc = np.where(ref["pre"] > 0, ref["pre"], 0.2 * ref["pre"])
    seg = np.repeat(np.arange(n), np.diff(rowptr))
    sc[empty[seg]] = 0.0  # virtual rows: constant score
    lse_ref = np.zeros((n, H))
    for h in range(H):
        mx = np.full(n, -np.inf)
        np.maximum.at(mx, seg, sc[:, h])
        acc = np.zeros(n)
        np.add.at(acc, seg, np.exp(sc[:, h] - mx[seg]))
        lse_ref[:, h] = mx + np.log(acc)
    np.testing.assert_allclose(lse, lse_ref, rtol=1e-5, atol=1e-5)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    assert torch.equal(u1, outs[0][0]) and torch.equal(lse1, outs[0][2])


@pytest.mark.parametrize("p", [0.0, 0.5])
def test_bip_many_groups_per_wave_vs_general(cuda, msha, bip_path, p):
    """120k rows: every wave walks many 8-row groups, with sub-groups and the next
    group's loads in flight (the small cases above give each wave one or two rows).
    Every output against the general kernels (functional.BIP = False)."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    n, m, H, F = 120_000, 32, 2, 64
    rng = np.random.default_rng(77)
    deg = rng.integers(1, 7, n)
    deg[rng.choice(n, 200, replace=False)] = 32  # full-width rows: their own sub-groups
    rowptr = np.zeros(n + 1, np.int64)
    rowptr[1:] = np.cumsum(deg)
    col = np.concatenate([np.sort(rng.choice(m, d, replace=False)) for d in deg])
    graph = Graph.from_csr(torch.as_tensor(rowptr), torch.as_tensor(col), m, cuda)
    el = rng.standard_normal((n, H)).astype(np.float32)
    er = rng.standard_normal((m, H)).astype(np.float32)
    hc = rng.standard_normal((m, H, F)).astype(np.float32)
    hs = rng.standard_normal((n, H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    dV = rng.standard_normal((m, H, F)).astype(np.float32)
    got = _run(MF, graph, el, er, hc, hs, dU, dV, p, 13, cuda, torch.float32, True)
    gen = _run(MF, graph, el, er, hc, hs, dU, dV, p, 13, cuda, torch.float32, False)
    keep = _keep_mask(graph.n_edges, H, p, 13, cuda)
    d64 = lambda x: x.astype(np.float64)  # noqa: E731
    ref = O.edge_aggregate_fwd(rowptr, col, d64(el), d64(er), d64(hc), hs=d64(hs), keep=keep, p=p)
    bw = O.edge_aggregate_bwd(rowptr, col, ref, d64(hc), d64(dU), hs=d64(hs), dV=d64(dV),
                              keep=keep, p=p)
    A = edge_abs_terms(rowptr, col, ref, hc, dU, hs=hs, dV=dV, keep=keep, p=p)
    refs = dict(u=ref["u"], v=ref["v"], d_el=bw["d_el"], d_er=bw["d_er"], d_hc=bw["d_hc"],
                d_hs=bw["d_hs"])
    for name, a, b in zip(("u", "v", "d_el", "d_er", "d_hc", "d_hs"), got, gen):
        nt = A["n_row"] if name in ("u", "d_hs", "d_el") else A["n_col"]
        bounded_close(a.cpu().numpy(), refs[name], A[name], nt, 1e-5, name)
        bounded_close(b.cpu().numpy(), refs[name], A[name], nt, 1e-5, name + " (general)")


def test_shipped_graph_models_run_on_the_bipartite_kernels(cuda, msha):
    """ablation3 on the full shipped 2015 graph (39,179 x 32) takes the bipartite kernels
    both ways -- not the general edge kernels -- and its train-step forward stays a
    normalised distribution per row."""
    from conftest import golden
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd import layers

    g = golden("r15_graph.npz")
    n = int(g["n"])
    c = np.zeros((n, 32), np.float32)
    c[O.edge_rows(g["rowptr"]), g["col"].astype(np.int64)] = g["cnt"]
    gdp = {i: float(x) for i, x in enumerate(g["gdp"])}
    torch.manual_seed(0)
    model = layers.ablation3(128, 64, 32, 2, 0.5, gdp, n, 32).to(cuda)
    adj = msha.normalize_adjacency_matrix(torch.as_tensor(c, device=cuda))
    model.train()
    MF.KERNEL_EVENTS = {}
    try:
        out = model(adj, None, None, None)
        out[:64].sum().backward()
        torch.cuda.synchronize()
        names = set(MF.KERNEL_EVENTS)
    finally:
        MF.KERNEL_EVENTS = None
    assert {"bip_attention_fwd", "bip_attention_bwd"} <= names, names
    assert not names & {"edge_attention_fwd", "edge_attention_bwd_rows", "csc_aggregate"}, names
    assert torch.allclose(out.detach().exp().sum(1), torch.ones(n, device=cuda), atol=1e-4)


@pytest.fixture
def mask_bwd_everywhere(msha, monkeypatch):
    """Route every M <= 32, 2 x 64 graph through the MFMA kernels (edge_bip3.hip, the fp32
    backward included), not only those above the 131,072-row cut (msha_bip2_bwd_min_rows)."""
    from msha_gnn_amd import _lib

    monkeypatch.setenv("MSHA_BIP3_BWD32", "1")
    prev = _lib.fn("msha_bip2_bwd_min_rows")(0)
    yield
    _lib.fn("msha_bip2_bwd_min_rows")(prev)


@pytest.mark.parametrize("p", [0.0, 0.4])
def test_ours_attention_mask_backward(cuda, msha, mask_bwd_everywhere, p):
    """Ours (row_coef, with and without dropout) through the MFMA kernels: the COEF / DROP
    variants of bip3_bwd_kernel against the dense fp64 restatement."""
    from test_gpu_ours import check_ours_attention_vs_dense

    check_ours_attention_vs_dense(cuda, p)
