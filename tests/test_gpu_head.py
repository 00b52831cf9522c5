"""Model head (msha_head_fwd / msha_head_bwd) vs an fp64 torch restatement of the
reference's tail (Ablation.py:273-277 per head + :298-301; GAT.py:20-35 for out_att),
with the kernels' own Philox dropout masks injected into the reference.

fp32 bar: 1e-5 relative to each tensor's scale (north_star); bf16 tables: 1e-2 against
the fp64 reference evaluated on the same bf16-rounded inputs.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from gpu_helpers import tol_close

pytestmark = pytest.mark.gpu


def _graph(n, m, seed, dev):
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(seed)
    cnt = np.zeros((n, m), np.float32)
    for i in range(n):
        d = int(rng.integers(0, 6))
        if d:
            cnt[i, rng.choice(m, d, replace=False)] = 1
    cnt[:3] = 0  # empty rows: virtual full rows, uniform 1/M attention
    cnt[3] = 1   # a full row
    g = Graph.from_dense(torch.as_tensor(cnt, device=dev))
    mask = cnt > 0
    mask[~mask.any(1)] = True
    return g, torch.as_tensor(mask)


def _bns(H, F, dev, seed):
    gen = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(H):
        pair = []
        for _ in range(2):
            bn = torch.nn.BatchNorm1d(F).to(dev)
            with torch.no_grad():
                bn.weight.copy_(torch.rand(F, generator=gen) + 0.5)
                bn.bias.copy_(torch.randn(F, generator=gen) * 0.1)
                bn.running_mean.copy_(torch.randn(F, generator=gen) * 0.1)
                bn.running_var.copy_(torch.rand(F, generator=gen) + 0.5)
            pair.append(bn)
        out.append(tuple(pair))  # (bn2 u side, bn1 v side)
    return out


def _reference(u, v, bns, W, mask, keep_x, keep_g, p, training, dout):
    """fp64 restatement on CPU; returns (out, grads dict) with autograd."""
    N, H, F_ = u.shape
    M = v.shape[0]
    u = u.detach().double().cpu().requires_grad_(True)
    v = v.detach().double().cpu().requires_grad_(True)
    W = W.detach().double().cpu().requires_grad_(True)
    prm = []
    for bu, bv in bns:
        prm.append([t.detach().double().cpu().requires_grad_(True)
                    for t in (bu.weight, bu.bias, bv.weight, bv.bias)])
    runs = [[t.detach().double().cpu().clone() for t in (bu.running_mean, bu.running_var,
                                                          bv.running_mean, bv.running_var)]
            for bu, bv in bns]
    scale = 1.0 / (1.0 - p) if p > 0 else 1.0
    cs = []
    for h in range(H):
        wu, bu_, wv, bv_ = prm[h]
        rmu, rvu, rmv, rvv = runs[h]
        uo = F.leaky_relu(F.batch_norm(u[:, h], rmu, rvu, wu, bu_, training, 0.1, 1e-5), 0.2)
        vo = F.leaky_relu(F.batch_norm(v[:, h], rmv, rvv, wv, bv_, training, 0.1, 1e-5), 0.2)
        cs.append(F.elu(uo @ vo.t()))
    x = torch.cat(cs, 1)
    if training and p > 0:
        x = x * keep_x.double().view(N, H * M) * scale
    hg = x @ W
    deg = mask.sum(1, keepdim=True).double()
    att = mask.double() / deg
    if training and p > 0:
        att = att * keep_g.double().view(N, M) * scale
    out = F.log_softmax(F.elu(F.elu(att * hg)), dim=1)
    grads = {}
    if dout is not None:
        out.backward(dout.double().cpu())
        grads = {"u": u.grad, "v": v.grad, "W": W.grad,
                 "uw": [q[0].grad for q in prm], "ub": [q[1].grad for q in prm],
                 "vw": [q[2].grad for q in prm], "vb": [q[3].grad for q in prm]}
    return out.detach(), grads, runs


def _run(cuda, n, m, H, F_, p, training, dtype=torch.float32, sparse=True, seed=0):
    from msha_gnn_amd import functional as MF

    g, mask = _graph(n, m, seed, cuda)
    gen = torch.Generator().manual_seed(seed + 1)
    u = (torch.randn(n, H, F_, generator=gen)).to(cuda, dtype)
    v = (torch.randn(m, H, F_, generator=gen)).to(cuda, dtype)
    W = (torch.randn(H * m, m, generator=gen) * (H * m) ** -0.5).to(cuda)
    a = torch.zeros(2 * m, 1, device=cuda)
    bns = _bns(H, F_, cuda, seed + 2)
    for pair in bns:
        for bn in pair:
            bn.train(training)
    ref_bns = _bns(H, F_, cuda, seed + 2)  # same values, untouched by the kernel
    sx, sa = 1234 + seed, 5678 + seed
    pp = p if training else 0.0
    u_ = u.clone().requires_grad_(True)
    v_ = v.clone().requires_grad_(True)
    W_ = W.clone().requires_grad_(True)
    params = ([b[0].weight for b in bns] + [b[0].bias for b in bns] + [b[1].weight for b in bns]
              + [b[1].bias for b in bns] + [a])
    with torch.set_grad_enabled(training):
        out = MF._ModelHead.apply(u_, v_, W_, g, bns, training, 1e-5, 0.1, 0.2, pp, sx, pp, sa,
                                  *params)
    keep_x = MF.dropout_keep_mask(n * H * m, pp, sx, cuda, flat4=True).cpu().bool() if pp > 0 else None
    keep_g = MF.dropout_keep_mask(n * m, pp, sa, cuda, flat4=True).cpu().bool() if pp > 0 else None
    dout = None
    if training:
        dout = torch.zeros(n, m)
        rows = torch.randint(0, n, (64,), generator=gen) if sparse else torch.arange(n)
        dout.index_put_((rows,), torch.randn(len(rows), m, generator=gen), accumulate=True)
        out.backward(dout.to(cuda, dtype))
    ref, grads, runs = _reference(u, v, ref_bns, W, mask, keep_x, keep_g, pp, training, dout)
    return out, ref, grads, runs, (u_, v_, W_, bns)


@pytest.mark.parametrize("p", [0.0, 0.5])
@pytest.mark.parametrize("sparse", [True, False])
def test_head_train_matches_fp64(cuda, msha, p, sparse):
    """R15's shape (2 heads x 64, 32 recipients) with empty / full rows: output, every
    gradient and the BatchNorm running statistics within 1e-5."""
    out, ref, gr, runs, (u, v, W, bns) = _run(cuda, 3000, 32, 2, 64, p, True, sparse=sparse)
    tol_close(out.detach().cpu().numpy(), ref.numpy(), 1e-5, 1e-5)
    tol_close(u.grad.cpu().numpy(), gr["u"].numpy(), 1e-5, 1e-5)
    tol_close(v.grad.cpu().numpy(), gr["v"].numpy(), 1e-5, 1e-5)
    tol_close(W.grad.cpu().numpy(), gr["W"].numpy(), 1e-5, 1e-5)
    for h, (bu, bv) in enumerate(bns):
        tol_close(bu.weight.grad.cpu().numpy(), gr["uw"][h].numpy(), 1e-5, 1e-5)
        tol_close(bu.bias.grad.cpu().numpy(), gr["ub"][h].numpy(), 1e-5, 1e-5)
        tol_close(bv.weight.grad.cpu().numpy(), gr["vw"][h].numpy(), 1e-5, 1e-5)
        tol_close(bv.bias.grad.cpu().numpy(), gr["vb"][h].numpy(), 1e-5, 1e-5)
        for t, r in zip((bu.running_mean, bu.running_var, bv.running_mean, bv.running_var),
                        runs[h]):
            tol_close(t.cpu().numpy(), r.numpy(), 1e-5, 1e-6)
        # the kernel advanced every BatchNorm's step counter once (nn.BatchNorm1d's +1)
        assert int(bu.num_batches_tracked) == 1 and int(bv.num_batches_tracked) == 1


def test_head_wide_recipients(cuda, msha):
    """80 recipients (two 64-lane column passes per row), 2 heads x 16."""
    out, ref, gr, _, (u, v, W, _) = _run(cuda, 700, 80, 2, 16, 0.3, True, seed=3)
    tol_close(out.detach().cpu().numpy(), ref.numpy(), 1e-5, 1e-5)
    tol_close(u.grad.cpu().numpy(), gr["u"].numpy(), 1e-5, 1e-5)
    tol_close(W.grad.cpu().numpy(), gr["W"].numpy(), 1e-5, 1e-5)


def test_head_eval_running_stats(cuda, msha):
    out, ref, _, _, _ = _run(cuda, 1000, 32, 2, 64, 0.5, False, seed=5)
    tol_close(out.detach().cpu().numpy(), ref.numpy(), 1e-5, 1e-5)


def test_head_eval_with_autograd_refuses(cuda, msha):
    """The head's backward is the training-mode BatchNorm's: the public model_head
    refuses eval-mode gradients instead of returning wrong ones (the models route eval
    with autograd to the unfused tail), and eval without running statistics."""
    from msha_gnn_amd import functional as MF

    g, _ = _graph(300, 32, 3, cuda)
    bns = _bns(2, 64, cuda, 4)
    for pair in bns:
        for bn in pair:
            bn.eval()
    u = torch.randn(300, 2, 64, device=cuda, requires_grad=True)
    v = torch.randn(32, 2, 64, device=cuda)
    W = torch.randn(64, 32, device=cuda)
    a = torch.zeros(64, 1, device=cuda)
    with pytest.raises(NotImplementedError):
        MF.model_head(g, u, v, bns, W, a, training=False)
    with torch.no_grad():
        out = MF.model_head(g, u, v, bns, W, a, training=False)
    assert torch.isfinite(out).all()
    nb = _bns(2, 64, cuda, 4)
    for pair in nb:
        for bn in pair:
            bn.eval()
            bn.running_mean = bn.running_var = None
    with torch.no_grad(), pytest.raises(ValueError):
        MF.model_head(g, u, v, nb, W, a, training=False)


def test_head_bf16_vs_fp64(cuda, msha):
    """bf16 tables (u, v, out, du, dv): 1e-2 against fp64 on the same rounded inputs."""
    out, ref, gr, _, (u, v, W, _) = _run(cuda, 2000, 32, 2, 64, 0.0, True, torch.bfloat16,
                                         seed=7)
    tol_close(out.detach().float().cpu().numpy(), ref.numpy(), 1e-2, 1e-2)
    tol_close(u.grad.float().cpu().numpy(), gr["u"].numpy(), 1e-2, 1e-2)
    tol_close(v.grad.float().cpu().numpy(), gr["v"].numpy(), 1e-2, 1e-2)
    tol_close(W.grad.cpu().numpy(), gr["W"].numpy(), 1e-2, 1e-2)


def test_models_use_the_fused_head(cuda, msha):
    """ablation3 / Ours route their tail through the model head in training (eager and
    inside the replay path's captured forward) and under no_grad; eval with autograd
    takes the per-head launches."""
    from msha_gnn_amd import layers

    class Probe:
        calls = 0
        captured = 0

    orig = layers.MF.model_head

    def probe(*a, **k):
        Probe.calls += 1
        Probe.captured += int(torch.cuda.is_current_stream_capturing())
        return orig(*a, **k)

    from msha_gnn_amd import replay

    g, _ = _graph(200, 32, 11, cuda)
    gdp = {i: 0.1 for i in range(200)}
    torch.manual_seed(0)
    model = layers.ablation3(128, 64, 32, 2, 0.5, gdp, 200, 32).to(cuda)
    layers.MF.model_head = probe
    prev = replay.REPLAY
    try:
        model.train()
        replay.REPLAY = False  # eager training forward: one head call
        model(g, None, None, torch.arange(4, device=cuda)).sum().backward()
        assert Probe.calls == 1 and Probe.captured == 0
        replay.REPLAY = True  # replay path: the head is inside the captured forward
        src = torch.arange(4, device=cuda)
        model(g, None, None, src).sum().backward()
        assert model.__dict__.get("_msha_graphs"), "replay path not taken"
        assert Probe.captured == 1, "captured forward did not route through the model head"
        before = Probe.calls
        model(g, None, None, src).sum().backward()  # pure replay: no Python head call
        assert Probe.calls == before
        model.eval()
        with torch.no_grad():
            model(g, None, None, None)
        assert Probe.calls == before + 1
        model(g, None, None, None)
        assert Probe.calls == before + 1
    finally:
        replay.REPLAY = prev
        layers.MF.model_head = orig


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("intra", [False, True])
def test_pack_heads_matches_cat_and_stack(cuda, msha, intra, dtype):
    """One-launch parameter packing == torch.cat / stack / sum of the heads' parameters,
    and its backward == autograd's gradients of that torch formulation (bit-exact: copies
    and one add).  bf16 parameters: W packed in bf16, score halves (and the a3/a4 half
    sums) in fp32, gradients cast back to bf16 in the same launch."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd import layers

    torch.manual_seed(0)
    cls = layers.OursLayer if intra else layers.OursLayer3
    heads = [cls(128, 64, 0.0).to(cuda, dtype) for _ in range(2)]
    packed = MF.pack_heads(heads, intra)
    ref = [torch.cat([h.W1 for h in heads], 1), torch.cat([h.W2 for h in heads], 1)]
    halves = layers._score_halves(heads, "a").float()
    ref += [halves[:, 0], halves[:, 1]]
    if intra:
        ref += [layers._score_halves(heads, "a3").float().sum(1),
                layers._score_halves(heads, "a4").float().sum(1)]
    assert [t.dtype for t in packed] == [dtype] * 2 + [torch.float32] * (len(packed) - 2)
    assert len(packed) == len(ref)
    gen = torch.Generator(device=cuda).manual_seed(1)
    ws = [torch.randn(r.shape, device=cuda, generator=gen) for r in ref]
    for got, want in zip(packed, ref):
        assert torch.equal(got, want)
    params = [p for h in heads for p in h.parameters()]
    g_ref = torch.autograd.grad(sum((r * w).sum() for r, w in zip(ref, ws)), params,
                                allow_unused=True)
    g_got = torch.autograd.grad(sum((r * w).sum() for r, w in zip(packed, ws)), params,
                                allow_unused=True)
    for a, b in zip(g_got, g_ref):
        assert (a is None) == (b is None)
        if a is not None:
            torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_feature_dropout_masks_and_grad(cuda, msha, dtype):
    """Both feature tables dropped in one launch with the Philox masks
    (msha_dropout_keep_mask of the same seed), gradients masked the same way (bf16
    tables: the same masks, x * 2 exact in bf16)."""
    from msha_gnn_amd import functional as MF

    gen = torch.Generator(device=cuda).manual_seed(2)
    S = torch.rand(1000, 128, device=cuda, generator=gen).to(dtype).requires_grad_(True)
    R = torch.rand(32, 128, device=cuda, generator=gen).to(dtype).requires_grad_(True)
    So, Ro = MF._FeatureDropout.apply(S, R, 0.5, 77, 78)
    kS = MF.dropout_keep_mask(S.numel(), 0.5, 77, cuda, flat4=True).view_as(S).bool()
    kR = MF.dropout_keep_mask(R.numel(), 0.5, 78, cuda, flat4=True).view_as(R).bool()
    assert 0.45 < kS.float().mean() < 0.55
    # word 0 of block q is the per-element generator at index q
    assert torch.equal(kS.view(-1)[::4], MF.dropout_keep_mask(S.numel() // 4, 0.5, 77, cuda)
                       .bool())
    assert torch.equal(So, torch.where(kS, S * 2.0, torch.zeros_like(S)))
    assert torch.equal(Ro, torch.where(kR, R * 2.0, torch.zeros_like(R)))
    (So.sum() + 3 * Ro.sum()).backward()
    assert S.grad.dtype == dtype and So.dtype == dtype
    assert torch.equal(S.grad, (kS.float() * 2.0).to(dtype))
    assert torch.equal(R.grad, (kR.float() * 6.0).to(dtype))


@pytest.mark.parametrize("intra", [False, True])
def test_model_prologue_matches_separate_launches(cuda, msha, intra):
    """model_prologue (feature dropout + head packing in one launch each way, one autograd
    node) == feature_dropout then pack_heads with the same seeds: outputs and every
    gradient bit-identical (the same segment records, one batch)."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd import layers

    torch.manual_seed(0)
    cls = layers.OursLayer if intra else layers.OursLayer3
    heads = [cls(128, 64, 0.5).to(cuda) for _ in range(2)]
    gen = torch.Generator(device=cuda).manual_seed(5)
    S = torch.rand(1000, 128, device=cuda, generator=gen).requires_grad_(True)
    R = torch.rand(32, 128, device=cuda, generator=gen).requires_grad_(True)
    params = [S, R] + [p for h in heads for p in h.parameters()]
    torch.manual_seed(11)
    s1, r1, packed = MF.model_prologue(S, R, 0.5, True, heads, intra)
    torch.manual_seed(11)
    s2, r2 = MF.feature_dropout(S, R, 0.5, True)
    ref = MF.pack_heads(heads, intra)
    outs1, outs2 = [s1, r1, *packed], [s2, r2, *ref]
    ws = [torch.randn(t.shape, device=cuda, generator=gen) for t in outs1]
    for a, b in zip(outs1, outs2):
        assert torch.equal(a, b)
    g1 = torch.autograd.grad(sum((t * w).sum() for t, w in zip(outs1, ws)), params,
                             allow_unused=True)
    g2 = torch.autograd.grad(sum((t * w).sum() for t, w in zip(outs2, ws)), params,
                             allow_unused=True)
    for a, b in zip(g1, g2):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)


def test_cast_segments_round_to_nearest_even(cuda, msha):
    """msha_segments as a dtype cast (ABI 8): fp32 -> bf16 rounds like torch's .to(),
    bf16 -> fp32 is exact, strided rows, and several pairs in one launch."""
    from msha_gnn_amd import functional as MF

    gen = torch.Generator(device=cuda).manual_seed(3)
    a = torch.randn(37, 129, device=cuda, generator=gen) * 1e3
    b = torch.randn(4096, device=cuda, generator=gen).to(torch.bfloat16)
    a16 = torch.empty(a.shape, device=cuda, dtype=torch.bfloat16)
    b32 = torch.empty(b.shape, device=cuda)
    MF._cast_many([(a, a16), (b, b32)], torch.cuda.current_stream(cuda).cuda_stream)
    assert torch.equal(a16, a.to(torch.bfloat16))
    assert torch.equal(b32, b.float())
    # strided (non-flat) segment path: the first 65 columns of each row of a
    out = torch.zeros(37, 65, device=cuda, dtype=torch.bfloat16)
    MF._segments([(a.data_ptr(), out.data_ptr(), 37, 65, 129, 65, None, 0, 0.0, 0,
                   torch.float32, torch.bfloat16)], torch.cuda.current_stream(cuda).cuda_stream)
    assert torch.equal(out, a[:, :65].to(torch.bfloat16))


@pytest.mark.parametrize("M,K,H,F_", [(32, 128, 2, 64), (200, 64, 1, 128), (7, 128, 8, 16)])
def test_project_small_vs_fp64(cuda, msha, M, K, H, F_):
    """The recipient-side projection (msha_project_small / _bwd, one launch each way):
    h, el, er and every gradient (dX, dW, dal, dar) vs fp64 torch within 1e-5."""
    from msha_gnn_amd import functional as MF

    assert msha._lib.load().msha_project_small_supported(M, K, H, F_) == 1
    gen = torch.Generator().manual_seed(M)
    X = torch.randn(M, K, generator=gen)
    W = torch.randn(K, H * F_, generator=gen) / K ** 0.5
    al = torch.randn(H, F_, generator=gen)
    ar = torch.randn(H, F_, generator=gen)
    dh = torch.randn(M, H * F_, generator=gen)
    dl = torch.randn(M, H, generator=gen)
    dr = torch.randn(M, H, generator=gen)
    ts = [t.to(cuda).requires_grad_(True) for t in (X, W, al, ar)]
    h, el, er = MF.project_scores(*ts, heads=H)
    torch.autograd.backward([h, el, er], [dh.to(cuda), dl.to(cuda), dr.to(cuda)])
    r = [t.double().requires_grad_(True) for t in (X, W, al, ar)]
    h64 = r[0] @ r[1]
    hv = h64.view(M, H, F_)
    el64 = (hv * r[2]).sum(-1)
    er64 = (hv * r[3]).sum(-1)
    torch.autograd.backward([h64, el64, er64], [dh.double(), dl.double(), dr.double()])
    for got, want in ((h, h64), (el, el64), (er, er64)):
        tol_close(got.detach().cpu().numpy(), want.detach().numpy(), 1e-5, 1e-5)
    for got, want in zip(ts, r):
        tol_close(got.grad.cpu().numpy(), want.grad.numpy(), 1e-5, 1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_nll_loss_rows_matches_torch(cuda, msha, dtype):
    """msha_nll_rows_fwd/_bwd == F.nll_loss(logp[rows].float(), cols) and its autograd,
    with repeated (row, col) pairs (accumulated, as index backward does) and a row
    repeated with another column."""
    from msha_gnn_amd import functional as MF

    gen = torch.Generator(device=cuda).manual_seed(4)
    N, M, B = 39179, 32, 64
    logp = torch.log_softmax(torch.randn(N, M, device=cuda, generator=gen), 1).to(dtype)
    rows = torch.randint(0, N, (B,), device=cuda, generator=gen)
    cols = torch.randint(0, M, (B,), device=cuda, generator=gen)
    rows[5], cols[5] = rows[3], cols[3]  # a repeated pair
    rows[9] = rows[3]                    # same row, another column
    a = logp.detach().clone().requires_grad_(True)
    b = logp.detach().clone().requires_grad_(True)
    got = MF.nll_loss_rows(a, rows, cols)
    ref = torch.nn.functional.nll_loss(b[rows].float(), cols)
    tol = 1e-6 if dtype == torch.float32 else 1e-3
    assert abs(float(got) - float(ref)) <= tol * abs(float(ref))
    (3.0 * got).backward()
    (3.0 * ref).backward()
    assert a.grad.dtype == dtype
    assert torch.equal(a.grad, b.grad)
    # out-of-range entries are neither read nor written: NaN loss (torch raises), the
    # backward leaves the table's gradient zero there; an empty batch is NaN (torch's mean)
    bad_r, bad_c = rows.clone(), cols.clone()
    bad_r[0], bad_c[1] = N + 7, M
    c = logp.detach().clone().requires_grad_(True)
    lb = MF.nll_loss_rows(c, bad_r, bad_c)
    assert torch.isnan(lb).item()
    lb.backward()
    assert torch.isfinite(c.grad.float()).all()
    e = torch.empty(0, dtype=torch.int64, device=cuda)
    assert torch.isnan(MF.nll_loss_rows(logp, e, e)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_nll_bwd_row_flags_match_scan(cuda, msha, dtype):
    """msha_nll_rows_bwd_flags: the gradient is the plain backward's, bit for bit, and the
    row flags are the head backward's scan of it (rflag[i] = row i has a nonzero, wmask
    word w bit k = rflag[64 w + k]); a row whose entries cancel to zero is not flagged."""
    from msha_gnn_amd import _lib

    gen = torch.Generator(device=cuda).manual_seed(7)
    N, M, B = 39179, 32, 64
    rows = torch.randint(0, N, (B,), device=cuda, generator=gen)
    cols = torch.randint(0, M, (B,), device=cuda, generator=gen)
    rows[-1] = N - 1  # the last, partial word
    g = torch.tensor([2.5], device=cuda)
    code = 1 if dtype == torch.bfloat16 else 0
    d0 = torch.empty(N, M, device=cuda, dtype=dtype)
    d1 = torch.empty(N, M, device=cuda, dtype=dtype)
    nw = (N + 63) // 64
    rflag = torch.full((N,), 7, device=cuda, dtype=torch.uint8)
    wmask = torch.zeros(nw, device=cuda, dtype=torch.int64)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("msha_nll_rows_bwd", N, M, B, rows.data_ptr(), cols.data_ptr(), g.data_ptr(), code,
              d0.data_ptr(), M, s)
    _lib.call("msha_nll_rows_bwd_flags", N, M, B, rows.data_ptr(), cols.data_ptr(), g.data_ptr(),
              code, d1.data_ptr(), M, rflag.data_ptr(), wmask.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(d0, d1)
    want = (d1.float() != 0).any(1)
    assert torch.equal(rflag.bool(), want)
    bits = want.cpu().numpy()
    words = np.zeros(nw, np.uint64)
    for i in np.nonzero(bits)[0]:
        words[i // 64] |= np.uint64(1) << np.uint64(i % 64)
    assert np.array_equal(wmask.cpu().numpy().view(np.uint64), words)
    # gloss 0: every row zero, nothing flagged
    z = torch.zeros(1, device=cuda)
    _lib.call("msha_nll_rows_bwd_flags", N, M, B, rows.data_ptr(), cols.data_ptr(), z.data_ptr(),
              code, d1.data_ptr(), M, rflag.data_ptr(), wmask.data_ptr(), s)
    torch.cuda.synchronize()
    assert int(rflag.sum()) == 0 and int(wmask.abs().sum()) == 0


def test_head_bwd_takes_the_loss_row_flags(cuda, msha):
    """loss = nll_loss_rows(model head): the head backward takes the loss backward's row flags
    (msha_head_bwd_flagged, no scan launch) and every gradient equals the scanning path's
    bit for bit (MSHA_NLL_FLAGS=0 form)."""
    from msha_gnn_amd import functional as MF

    n, m, H, F_ = 3000, 32, 2, 64
    g, _ = _graph(n, m, 11, cuda)
    gen = torch.Generator().manual_seed(12)
    u0 = torch.randn(n, H, F_, generator=gen).to(cuda)
    v0 = torch.randn(m, H, F_, generator=gen).to(cuda)
    W0 = (torch.randn(H * m, m, generator=gen) * (H * m) ** -0.5).to(cuda)
    rows = torch.randint(0, n, (64,), generator=gen).to(cuda)
    cols = torch.randint(0, m, (64,), generator=gen).to(cuda)
    res = []
    for flags in (True, False):
        MF.NLL_FLAGS = flags
        try:
            bns = _bns(H, F_, cuda, 13)
            a = torch.zeros(2 * m, 1, device=cuda, requires_grad=True)
            u, v, W = (t.clone().requires_grad_(True) for t in (u0, v0, W0))
            params = ([b[0].weight for b in bns] + [b[0].bias for b in bns]
                      + [b[1].weight for b in bns] + [b[1].bias for b in bns] + [a])
            out = MF._ModelHead.apply(u, v, W, g, bns, True, 1e-5, 0.1, 0.2, 0.3, 21, 0.3, 22,
                                      *params)
            before = MF.HEAD_BWD_FLAGGED[0]
            MF.nll_loss_rows(out, rows, cols).backward()
            took = MF.HEAD_BWD_FLAGGED[0] - before
            res.append((took, [t.grad.clone() for t in (u, v, W)] +
                        [p.grad.clone() for p in params[:-1]]))
        finally:
            MF.NLL_FLAGS = True
    assert res[0][0] == 1 and res[1][0] == 0
    for x, y in zip(res[0][1], res[1][1]):
        assert torch.equal(x, y)
