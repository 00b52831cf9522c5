"""Full MSHA layer (Ours.OursLayer, Ours.py:29-167) on the GPU.

Module level: against the reference's own outputs / gradients (tests/golden/ours_small.npz,
fp32 case as the reference runs and an fp64 case with a repeated batch source and a
source without flows).  Kernel level: against a dense fp64 torch restatement of
Ours.py:64-101 (the torch reference of a floating-point op) on a larger random graph,
with and without dropout (the kernels' Philox masks injected into the reference).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden
from gpu_helpers import t, tol_close

pytestmark = pytest.mark.gpu


def _layer_case(msha, cuda, tag):
    from msha_gnn_amd import layers

    z = golden("ours_small.npz")
    counts = z[tag + "counts"] if tag + "counts" in z.files else z["counts"]
    torch.manual_seed(10)
    layer = layers.OursLayer(16, 8, 0.0)
    for k, v in layer.state_dict().items():
        assert np.array_equal(v.numpy(), z[f"init.{k}"]), k  # bit-identical init
    layer = layer.to(cuda)
    inter = msha.normalize_adjacency_matrix(t(counts, cuda))
    city = torch.as_tensor((z["city"][:, None] == z["city"][None, :]).astype(np.float32),
                           device=cuda)
    prov = torch.as_tensor((z["prov"][:, None] == z["prov"][None, :]).astype(np.float32),
                           device=cuda)
    S = t(z[tag + "S"], cuda).requires_grad_(True)
    R = t(z[tag + "R"], cuda).requires_grad_(True)
    src = torch.as_tensor(z[tag + "source_index"], device=cuda)
    return z, layer, inter, city, prov, S, R, src


@pytest.mark.parametrize("tag", ["", "B."])
def test_ours_layer_matches_reference(cuda, msha, tag):
    z, layer, inter, city, prov, S, R, src = _layer_case(msha, cuda, tag)
    layer.eval()
    with torch.no_grad():
        y = layer(S, R, inter, city, prov, src, False)
    tol_close(y.cpu().numpy(), z[tag + "out_eval"], 1e-5, 1e-5)
    layer.train()
    y = layer(S, R, inter, city, prov, src, False)
    tol_close(y.detach().cpu().numpy(), z[tag + "out"], 1e-5, 1e-5)
    y.backward(t(z[tag + "dout"], cuda))
    tol_close(S.grad.cpu().numpy(), z[tag + "grad.S"], 1e-5, 1e-5)
    tol_close(R.grad.cpu().numpy(), z[tag + "grad.R"], 1e-5, 1e-5)
    for k, p in layer.named_parameters():
        key = f"{tag}grad.{k}"
        if key in z.files:
            tol_close(p.grad.cpu().numpy(), z[key], 1e-5, 1e-5)
        else:
            assert p.grad is None, k


def _dense_ours_core(el, er, h1, h2, a3s, a4s, mask, city, prov, src, keep_e=None,
                     keep3=None, keep4=None, p=0.0):
    """fp64 dense restatement of Ours.py:64-101 (one head): returns (u, v)."""
    e12 = F.leaky_relu(el[:, None] + er[None, :], 0.2)
    att = torch.softmax(torch.where(mask, e12, torch.full_like(e12, -9e15)), dim=1)
    if keep_e is not None:
        att = att * keep_e / (1 - p)
    hb = h2[src]
    e3 = F.leaky_relu(hb @ a3s, 0.2)
    e4 = F.leaky_relu(hb @ a4s, 0.2)
    m3 = city[src][:, None] == city[None, :]
    m4 = prov[src][:, None] == prov[None, :]
    neg = torch.full(m3.shape, -9e15, dtype=torch.float64)
    x3 = torch.where(m3, e3[:, None].expand(m3.shape), neg)
    x4 = torch.where(m4, e4[:, None].expand(m4.shape), neg)
    SUM = torch.exp(x3).sum(1, keepdim=True) + torch.exp(x4).sum(1, keepdim=True) + \
        torch.exp(att[src]).sum(1, keepdim=True)
    a3 = torch.exp(x3) / SUM
    a4 = torch.exp(x4) / SUM
    if keep3 is not None:
        a3 = a3 * keep3 / (1 - p)
        a4 = a4 * keep4 / (1 - p)
    u = att @ h1 + a3.t() @ hb + a4.t() @ hb
    v = att.t() @ h2
    return u, v


def check_ours_attention_vs_dense(cuda, p, dtype=torch.float32, tol_out=1e-5, tol_grad=1e-4):
    """ours_attention (u, v and every input gradient) against the dense fp64 restatement
    with the kernels' dropout masks; ``dtype`` = storage of the node tables h1 / h2 (bf16:
    the reference is fed the same bf16-rounded tables and upstream gradients)."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph, Groups

    rng = np.random.default_rng(21)
    n, m, H, Fd, B = 1500, 32, 2, 64, 48
    counts = np.zeros((n, m), np.float32)
    for i in range(n):
        k = int(rng.integers(1, 8))
        counts[i, rng.choice(m, k, replace=False)] = 1
    counts[[7, 100]] = 0  # virtual rows (uniform attention)
    city = rng.integers(0, 60, n)
    prov = city // 10  # provinces contain cities
    src = rng.integers(0, n, B)
    src[:4] = [7, 7, 100, 3]  # repeats + virtual rows in the batch
    el = rng.standard_normal((n, H))
    er = rng.standard_normal((m, H))
    h1 = rng.standard_normal((m, H, Fd)) * 0.3
    h2 = rng.standard_normal((n, H, Fd)) * 0.3
    a3s = rng.standard_normal((H, Fd)) * 0.2
    a4s = rng.standard_normal((H, Fd)) * 0.2
    dU = rng.standard_normal((n, H, Fd))
    dV = rng.standard_normal((m, H, Fd))
    if dtype != torch.float32:  # the values the bf16 kernels read
        rnd = lambda x: torch.as_tensor(x).to(dtype).double().numpy()  # noqa: E731
        h1, h2, dU, dV = rnd(h1), rnd(h2), rnd(dU), rnd(dV)
    graph = Graph.from_dense(t(counts, cuda))
    groups = Groups(city, prov, cuda)
    seed = 5
    tg = [t(x, cuda).requires_grad_(True) for x in (el, er, h1, h2, a3s, a4s)]
    tg[2] = t(h1, cuda, dtype).requires_grad_(True)
    tg[3] = t(h2, cuda, dtype).requires_grad_(True)
    u, v = MF.ours_attention(graph, groups, torch.as_tensor(src, device=cuda), *tg, p=p,
                             training=p > 0, seed=seed)
    assert u.dtype == dtype and v.dtype == dtype
    (u.float() * t(dU, cuda)).sum().add_((v.float() * t(dV, cuda)).sum()).backward()
    # dense fp64 reference, head by head, with the kernels' masks (edge ids follow the
    # CSR with virtual full rows; the reference's scores use the real mask: an empty
    # row is the softmax of all -9e15 = uniform)
    mask = torch.as_tensor(counts > 0)
    mask[~mask.any(1)] = True
    rows, cols = torch.nonzero(mask, as_tuple=True)
    E = len(rows)
    keep_all = None
    if p > 0:
        keep_all = MF.dropout_keep_mask(E * H, p, seed, cuda).cpu().numpy().reshape(E, H)
    for h in range(H):
        rs = [torch.tensor(x[:, h], dtype=torch.float64, requires_grad=True)
              for x in (el, er, h1, h2)]
        ra3 = torch.tensor(a3s[h], dtype=torch.float64, requires_grad=True)
        ra4 = torch.tensor(a4s[h], dtype=torch.float64, requires_grad=True)
        ke = k3 = k4 = None
        if p > 0:
            ke = torch.zeros(n, m, dtype=torch.float64)
            ke[rows, cols] = torch.as_tensor(keep_all[:, h], dtype=torch.float64)
            # intra masks: head pair h // 2 at offset 1 + h // 2, word 2 (h % 2) + kind
            k3 = torch.as_tensor(MF.dropout_keep_mask(B * n, p, seed, cuda, offset=1 + h // 2,
                                                      word=2 * (h % 2))
                                 .cpu().numpy().reshape(B, n), dtype=torch.float64)
            k4 = torch.as_tensor(MF.dropout_keep_mask(B * n, p, seed, cuda, offset=1 + h // 2,
                                                      word=2 * (h % 2) + 1)
                                 .cpu().numpy().reshape(B, n), dtype=torch.float64)
        ru, rv = _dense_ours_core(*rs, ra3, ra4, torch.as_tensor(counts > 0), torch.as_tensor(city),
                                  torch.as_tensor(prov), torch.as_tensor(src), ke, k3, k4, p)
        tol_close(u[:, h].detach().float().cpu().numpy(), ru.detach().numpy(), tol_out, tol_out)
        tol_close(v[:, h].detach().float().cpu().numpy(), rv.detach().numpy(), tol_out, tol_out)
        ((ru * torch.tensor(dU[:, h])).sum() + (rv * torch.tensor(dV[:, h])).sum()).backward()
        for got, ref in ((tg[0].grad[:, h], rs[0].grad), (tg[1].grad[:, h], rs[1].grad),
                         (tg[2].grad[:, h], rs[2].grad), (tg[3].grad[:, h], rs[3].grad),
                         (tg[4].grad[h], ra3.grad), (tg[5].grad[h], ra4.grad)):
            tol_close(got.float().cpu().numpy(), ref.numpy(), tol_grad, 1e-5 if tol_grad < 1e-3
                      else tol_grad)


@pytest.mark.parametrize("p", [0.0, 0.4])
def test_ours_attention_kernels_vs_dense(cuda, msha, p):
    check_ours_attention_vs_dense(cuda, p)


def test_ours_model_record_and_train_step(cuda, msha):
    """Ours model (2 fused heads) trains (finite loss, grads everywhere the reference
    has them) and record mode fills the attention dump like Ours.py:92-96."""
    from msha_gnn_amd import layers
    from msha_gnn_amd.data import GroupAdjacency

    z = golden("ours_small.npz")
    n, m = z["counts"].shape
    gdp = {i: 0.1 * i for i in range(n)}
    torch.manual_seed(0)
    model = layers.Ours(16, 8, m, 2, 0.5, gdp, n, m).to(cuda)
    inter = msha.normalize_adjacency_matrix(t(z["counts"], cuda))
    city = GroupAdjacency(torch.as_tensor(z["city"], device=cuda))
    prov = GroupAdjacency(torch.as_tensor(z["prov"], device=cuda))
    src = torch.as_tensor(z["source_index"], device=cuda)
    model.train()
    out = model(inter, city, prov, src)
    loss = F.nll_loss(out[src], torch.zeros_like(src))
    loss.backward()
    assert torch.isfinite(loss)
    for k, p in model.named_parameters():
        if "a3" in k or "a4" in k or k.endswith("W1") or k.endswith("W2"):
            assert p.grad is not None and torch.isfinite(p.grad).all(), k
    model.eval()
    C12 = torch.zeros(n, m, device=cuda)
    C3 = torch.zeros(n, n, device=cuda)
    C4 = torch.zeros(n, n, device=cuda)
    with torch.no_grad():
        model(inter, city, prov, src, True, C12, C3, C4)
    assert bool((C12 == 0).all())  # as Ours.py:92-96: the argument is never written
    c12new = layers.record_state.Coeff12new
    assert torch.allclose(c12new.sum(1), torch.ones(n, device=cuda), atol=1e-5)
    same = torch.as_tensor(z["city"][z["source_index"]][:, None] == z["city"][None, :],
                           device=cuda)
    r3 = C3[src]
    assert bool((r3[~same] == 0).all()) and bool((r3[same] > 0).all())


def test_ours_record_dump_matches_reference(cuda, msha):
    """Record() (train.py:284-291: eval, batches of sources) through OursLayer with
    record=True vs the reference's own dump (ours_record.npz from Ours.OursLayer):
    train.Coeff12new after each batch, Coeff3 / Coeff4 after both, Coeff12 untouched."""
    import sys
    import types

    from msha_gnn_amd import layers

    z, layer, inter, city, prov, S, R, _ = _layer_case(msha, cuda, "")
    r = golden("ours_record.npz")
    n, m = z["counts"].shape
    layer.eval()
    C12 = torch.full((n, m), -1.0, device=cuda)
    C3 = torch.full((n, n), -1.0, device=cuda)
    C4 = torch.full((n, n), -1.0, device=cuda)
    sink = types.ModuleType("train")  # the module Ours.py:5 imports as `train`
    sys.modules["train"] = sink
    try:
        for k, si in enumerate((np.arange(0, 32), np.arange(32, 64))):
            with torch.no_grad():
                layer(S, R, inter, city, prov, torch.as_tensor(si, device=cuda), True, C12, C3,
                      C4)
            tol_close(sink.Coeff12new.cpu().numpy(), r[f"rec.coeff12new.{k}"], 1e-5, 1e-6)
            assert sink.Coeff12new is layers.record_state.Coeff12new
    finally:
        del sys.modules["train"]
    assert bool((C12 == -1).all())
    tol_close(C3.cpu().numpy(), r["rec.coeff3"], 1e-5, 1e-6)
    tol_close(C4.cpu().numpy(), r["rec.coeff4"], 1e-5, 1e-6)


@pytest.mark.parametrize("n", [3000, 200_000])
def test_ours_packed_intra_draws_bitwise(cuda, msha, n):
    """The intra forward's packed dropout draws (msha_ours_pack_draws 1: matched (entry,
    node) pairs of consecutive nodes share one Philox draw per <= 64 pairs) give the
    per-node form's bits.  n = 200k puts ~24 nodes on every wave; half the batch sits in
    one province, so its nodes carry 32+ matches and the 64-pair groups split."""
    from msha_gnn_amd import _lib
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph, Groups

    rng = np.random.default_rng(3)
    m, H, Fd, B = 32, 2, 64, 64
    counts = np.zeros((n, m), np.float32)
    counts[np.arange(n), rng.integers(0, m, n)] = 1
    city = rng.integers(0, 400, n)
    prov = city // 40
    src = rng.integers(0, n, B)
    src[: B // 2] = rng.choice(np.flatnonzero(prov == 0), B // 2)
    graph = Graph.from_dense(t(counts, cuda))
    groups = Groups(city, prov, cuda)
    ins = [t(rng.standard_normal(s) * 0.3, cuda) for s in ((n, H), (m, H), (m, H, Fd),
                                                           (n, H, Fd), (H, Fd), (H, Fd))]
    lib = _lib.load()
    outs = []
    try:
        for mode in (1, 0):
            lib.msha_ours_pack_draws(mode)
            u, _ = MF.ours_attention(graph, groups, torch.as_tensor(src, device=cuda), *ins,
                                     p=0.5, training=True, seed=11)
            outs.append(u.detach().clone())
    finally:
        lib.msha_ours_pack_draws(1)
    assert torch.equal(outs[0], outs[1])
    assert (outs[0] != 0).any()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("n", [3000, 140_000])
def test_ours_deferred_reduce_bitwise(cuda, msha, n, dtype):
    """The bipartite forward's v reduce and backward's d_hc / d_er reduce run as extra blocks
    of the intra prep / stage-1 finish launches (msha_bip_defer_reduce): u, v and every
    gradient equal the separate-launch form's bits.  n = 140k takes the MFMA / mask kernels
    (>= 131,072 rows), n = 3000 the CSR walk; with dropout and the Ours row coefficients."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph, Groups

    rng = np.random.default_rng(5)
    m, H, Fd, B = 32, 2, 64, 64
    counts = np.zeros((n, m), np.float32)
    for k in range(3):
        counts[np.arange(n), rng.integers(0, m, n)] = 1
    city = rng.integers(0, 300, n)
    prov = city // 30
    src = torch.as_tensor(rng.integers(0, n, B), device=cuda)
    graph = Graph.from_dense(t(counts, cuda))
    groups = Groups(city, prov, cuda)
    base = [t(rng.standard_normal(s) * 0.3, cuda) for s in ((n, H), (m, H), (m, H, Fd),
                                                            (n, H, Fd), (H, Fd), (H, Fd))]
    base[2], base[3] = base[2].to(dtype), base[3].to(dtype)
    dU = t(rng.standard_normal((n, H, Fd)), cuda).to(dtype)
    dV = t(rng.standard_normal((m, H, Fd)), cuda).to(dtype)
    res = []
    try:
        for defer in (True, False):
            MF.BIP_DEFER_REDUCE = defer
            ins = [x.detach().clone().requires_grad_(True) for x in base]
            u, v = MF.ours_attention(graph, groups, src, *ins, p=0.3, training=True, seed=5)
            torch.autograd.backward([u, v], [dU, dV])
            torch.cuda.synchronize()
            res.append([u.detach().clone(), v.detach().clone()] + [x.grad.clone() for x in ins])
    finally:
        MF.BIP_DEFER_REDUCE = True
    for a, b in zip(*res):
        assert torch.equal(a, b)
    assert (res[0][1] != 0).any() and (res[0][4] != 0).any()
