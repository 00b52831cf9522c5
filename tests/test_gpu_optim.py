"""msha_gnn_amd.optim.Adam (msha_adam_step, csrc/optim.hip) against torch.optim.Adam, the
optimizer train.py builds (train.py:207: lr 1e-3, weight_decay 5e-4; stepped at :232).

* the same gradients fed to both for 5 steps: parameters and moments within 1e-6
  relative (fp32; tails of n % 4 != 0 elements included), bf16 parameters within the
  bf16 bar;
* the fused path: an ablation3 train loop where Sfeatures' update reads its feature
  dropout's output gradient and mask (fuse_dropout_grad) against the same loop with
  torch's Adam -- every parameter after 5 steps within 1e-6, Sfeatures.grad never
  allocated;
* the same loop replayed from a HIP graph (device step counts) gives the eager bits.
"""
import numpy as np
import pytest
import torch

from gpu_helpers import random_counts, t, tol_close

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _eager_models(msha):
    """These tests compare optimizers on identically seeded eager models (the same
    Philox seeds, hence the same dropout masks); the drop-in models' graph replay
    (replay.py) draws its masks from a replay counter instead, so it is off here."""
    from msha_gnn_amd import replay

    prev, replay.REPLAY = replay.REPLAY, False
    yield
    replay.REPLAY = prev


def test_adam_matches_torch_on_same_grads(cuda, msha):
    from msha_gnn_amd.optim import Adam

    g = torch.Generator().manual_seed(0)
    shapes = [(5000, 128), (32, 128), (128, 64), (128, 1), (7,), (1, 3), (64, 32)]
    ref = [torch.randn(s, generator=g).to(cuda) for s in shapes]
    ours = [p.clone() for p in ref]
    for p in ref + ours:
        p.requires_grad_(True)
    o_ref = torch.optim.Adam(ref, lr=1e-3, weight_decay=5e-4)
    o_us = Adam(ours, lr=1e-3, weight_decay=5e-4)
    for step in range(5):
        for a, b in zip(ref, ours):
            gr = torch.randn(a.shape, generator=g).to(cuda) * (1 + step)
            a.grad, b.grad = gr.clone(), gr.clone()
        o_ref.step()
        o_us.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, ours):
        tol_close(b.detach().cpu().numpy(), a.detach().cpu().numpy(), 1e-6, 1e-6)
        for k in ("exp_avg", "exp_avg_sq"):
            tol_close(o_us.state[b][k].cpu().numpy(), o_ref.state[a][k].cpu().numpy(), 1e-6,
                      1e-6)
        assert float(o_us.state[b]["step"]) == 5.0


def test_adam_bf16_params(cuda, msha):
    from msha_gnn_amd.optim import Adam

    g = torch.Generator().manual_seed(1)
    ref = [torch.randn(s, generator=g).to(cuda, torch.bfloat16).requires_grad_(True)
           for s in ((300, 128), (13,))]
    ours = [p.detach().clone().requires_grad_(True) for p in ref]
    o_ref = torch.optim.Adam(ref, lr=1e-3, weight_decay=5e-4)
    o_us = Adam(ours, lr=1e-3, weight_decay=5e-4)
    for _ in range(5):
        for a, b in zip(ref, ours):
            gr = torch.randn(a.shape, generator=g).to(cuda, torch.bfloat16)
            a.grad, b.grad = gr.clone(), gr.clone()
        o_ref.step()
        o_us.step()
    for a, b in zip(ref, ours):
        assert b.dtype == torch.bfloat16 and o_us.state[b]["exp_avg"].dtype == torch.bfloat16
        tol_close(b.detach().float().cpu().numpy(), a.detach().float().cpu().numpy(), 1e-2,
                  1e-2)


def _model_and_data(cuda, msha, dropout=0.5):
    from msha_gnn_amd import layers

    rng = np.random.default_rng(5)
    n, m = 600, 32
    c = random_counts(rng, n, m, 6, empty_rows=(4,))
    adj = msha.normalize_adjacency_matrix(t(c, cuda))
    batches = [(torch.as_tensor(rng.integers(0, n, 64), device=cuda),
                torch.as_tensor(rng.integers(0, m, 64), device=cuda)) for _ in range(5)]
    torch.manual_seed(0)
    model = layers.ablation3(128, 64, m, 2, dropout, {i: 0.01 * i for i in range(n)}, n,
                             m).to(cuda)
    return model, adj, batches


def _train(model, opt, adj, batches):
    from msha_gnn_amd import functional as MF

    model.train()
    torch.manual_seed(7)  # the dropout seeds (drawn from torch's CPU generator)
    for si, ri in batches:
        opt.zero_grad(set_to_none=True)
        loss = MF.nll_loss_rows(model(adj, None, None, si), si, ri)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()


def test_fused_feature_dropout_adam_matches_torch(cuda, msha):
    from msha_gnn_amd.optim import Adam

    m_ref, adj, batches = _model_and_data(cuda, msha)
    m_us, _, _ = _model_and_data(cuda, msha)
    o_ref = torch.optim.Adam(m_ref.parameters(), lr=1e-3, weight_decay=5e-4)
    o_us = Adam(m_us.parameters(), lr=1e-3, weight_decay=5e-4)
    o_us.fuse_dropout_grad(m_us.Sfeatures)
    _train(m_ref, o_ref, adj, batches)
    _train(m_us, o_us, adj, batches)
    assert m_us.Sfeatures.grad is None  # its step read the dropout's output gradient
    assert float(o_us.state[m_us.Sfeatures]["step"]) == len(batches)
    for (name, a), (_, b) in zip(m_ref.named_parameters(), m_us.named_parameters()):
        tol_close(b.detach().cpu().numpy(), a.detach().cpu().numpy(), 1e-6, 1e-6)


def test_graphed_fused_adam_matches_eager(cuda, msha):
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.optim import Adam
    from msha_gnn_amd.step import GraphedStep

    params = {}
    for graphed in (False, True):
        # p = 1e-9: every dropout launch runs (the fused feature-dropout update included)
        # but keeps every element with scale 1.0f, so eager and replay see the same bits
        # although the replay draws its masks from frozen seeds + the replay counter
        model, adj, batches = _model_and_data(cuda, msha, dropout=1e-9)
        opt = Adam(model.parameters(), lr=1e-3, weight_decay=5e-4)
        opt.fuse_dropout_grad(model.Sfeatures)
        model.train()
        si_s = torch.empty(64, dtype=torch.int64, device=cuda)
        ri_s = torch.empty(64, dtype=torch.int64, device=cuda)

        def body():
            opt.zero_grad(set_to_none=True)
            loss = MF.nll_loss_rows(model(adj, None, None, si_s), si_s, ri_s)
            loss.backward()
            opt.step()
            return loss

        si_s.copy_(batches[0][0])
        ri_s.copy_(batches[0][1])
        if graphed:
            gs = GraphedStep(body, cuda, warmup=2)
            for k in range(3):
                si_s.copy_(batches[k][0])
                ri_s.copy_(batches[k][1])
                gs.replay()
            gs.close()
        else:
            for k in range(2):  # GraphedStep's warm-up steps
                body()
            for k in range(3):
                si_s.copy_(batches[k][0])
                ri_s.copy_(batches[k][1])
                body()
        torch.cuda.synchronize()
        params[graphed] = [p.detach().clone() for p in model.parameters()]
    for a, b in zip(params[False], params[True]):
        assert torch.equal(a, b)


def test_adam_loads_torch_state_dict_from_cpu(cuda, msha):
    """a torch.optim.Adam state_dict saved and loaded with map_location='cpu'
    (its 'step' a CPU tensor) continues bit-for-bit like torch on the device: the loaded
    step moves to the parameter's device (capturable in the defaults / _state_of)."""
    import io

    from msha_gnn_amd.optim import Adam

    g = torch.Generator().manual_seed(2)
    shapes = [(300, 64), (17,)]
    ref = [torch.randn(s, generator=g).to(cuda).requires_grad_(True) for s in shapes]
    o_ref = torch.optim.Adam(ref, lr=1e-3, weight_decay=5e-4)
    grads = [[torch.randn(s, generator=g).to(cuda) for s in shapes] for _ in range(5)]
    for k in range(3):
        for p, gr in zip(ref, grads[k]):
            p.grad = gr.clone()
        o_ref.step()
    buf = io.BytesIO()
    torch.save(o_ref.state_dict(), buf)
    buf.seek(0)
    sd = torch.load(buf, map_location="cpu", weights_only=True)
    assert sd["state"][0]["step"].device.type == "cpu"
    ours = [p.detach().clone().requires_grad_(True) for p in ref]
    o_us = Adam(ours, lr=1e-3, weight_decay=5e-4)
    o_us.load_state_dict(sd)
    for k in range(3, 5):
        for a, b, gr in zip(ref, ours, grads[k]):
            a.grad, b.grad = gr.clone(), gr.clone()
        o_ref.step()
        o_us.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, ours):
        assert o_us.state[b]["step"].device == b.device
        assert float(o_us.state[b]["step"]) == 5.0
        tol_close(b.detach().cpu().numpy(), a.detach().cpu().numpy(), 1e-6, 1e-6)


def test_adam_fused_param_with_grad_raises(cuda, msha):
    """a fuse_dropout_grad parameter that also received a .grad (a second
    consumer) makes step() raise instead of dropping that gradient."""
    from msha_gnn_amd.optim import Adam

    p = torch.randn(64, 8, device=cuda, requires_grad=True)
    opt = Adam([p], lr=1e-3)
    opt.fuse_dropout_grad(p)
    opt.stash_dropout_grad(p, torch.randn(64, 8, device=cuda), 0.5, 7)
    p.grad = torch.randn(64, 8, device=cuda)
    with pytest.raises(RuntimeError, match="another consumer"):
        opt.step()
