"""HIP-graph capture of a training iteration (step.GraphedStep) and the device replay
counter of the library's dropout (msha_set_rng_counter)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden
from gpu_helpers import random_counts, t

pytestmark = pytest.mark.gpu


def test_rng_counter_fresh_masks_per_replay(cuda, msha):
    """A captured dropout edge-attention replays with new masks after each counter
    increment, and the same counter value reproduces the same mask."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(3)
    c = random_counts(rng, 300, 32, 20)
    graph = Graph.from_dense(t(c, cuda))
    el, er = t(rng.standard_normal((300, 2)), cuda), t(rng.standard_normal((32, 2)), cuda)
    hc = t(rng.standard_normal((32, 2, 64)), cuda)
    ctr = torch.zeros(1, dtype=torch.int64, device=cuda)
    MF.set_rng_counter(ctr)
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            MF.edge_attention(graph, el, er, hc, p=0.5, training=True, seed=5)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ctr.add_(1)
            u = MF.edge_attention(graph, el, er, hc, p=0.5, training=True, seed=5)
        outs = []
        for _ in range(2):
            g.replay()
            outs.append(u.clone())
        assert not torch.equal(outs[0], outs[1])
        ctr.zero_()
        g.replay()  # counter back to 1: the first replay's masks
        assert torch.equal(u, outs[0])
        # eager with the same counter value draws the same masks as the graph
        ctr.fill_(1)
        assert torch.equal(MF.edge_attention(graph, el, er, hc, p=0.5, training=True, seed=5),
                           outs[0])
    finally:
        MF.set_rng_counter(None)


def _ours_model(z, cuda, dropout):
    from msha_gnn_amd import layers

    n, m = z["counts"].shape
    torch.manual_seed(0)
    return layers.Ours(16, 8, m, 2, dropout, {i: 0.1 * i for i in range(n)}, n, m).to(cuda)


def test_graphed_train_step_matches_eager(cuda, msha):
    """Ours train step (forward, nll, backward, capturable Adam) replayed from a HIP
    graph gives the eager losses and parameters (dropout 0: deterministic)."""
    from msha_gnn_amd.data import GroupAdjacency
    from msha_gnn_amd.step import GraphedStep

    z = golden("ours_small.npz")
    inter = msha.normalize_adjacency_matrix(t(z["counts"], cuda))
    city = GroupAdjacency(torch.as_tensor(z["city"], device=cuda))
    prov = GroupAdjacency(torch.as_tensor(z["prov"], device=cuda))
    src = torch.as_tensor(z["source_index"], device=cuda)
    tgt = torch.as_tensor(np.arange(src.numel()) % z["counts"].shape[1], device=cuda)
    runs = {}
    for graphed in (False, True):
        model = _ours_model(z, cuda, 0.0)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=5e-4,
                               capturable=graphed)
        model.train()

        def body():
            opt.zero_grad(set_to_none=True)
            out = model(inter, city, prov, src)
            loss = F.nll_loss(out[src], tgt)
            loss.backward()
            opt.step()
            return loss

        losses = []
        if graphed:
            gs = GraphedStep(body, cuda, warmup=1)
            for _ in range(3):
                losses.append(float(gs.replay().detach()))
            gs.close()
        else:
            body()  # the graphed run's warm-up step
            for _ in range(3):
                losses.append(float(body().detach()))
        runs[graphed] = (losses, {k: p.detach().clone() for k, p in model.named_parameters()})
    np.testing.assert_allclose(runs[True][0], runs[False][0], rtol=1e-6)
    for k, p in runs[False][1].items():
        torch.testing.assert_close(runs[True][1][k], p, rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.parametrize("nbytes", [0, 1, 17, 512, 4099])
def test_feed_step_copies_and_counts(cuda, msha, nbytes):
    """msha_feed_step: dst.copy_(src) and counter += 1 in one launch, any size and
    alignment (uint8 views offset by one byte take the byte path)."""
    from msha_gnn_amd import functional as MF

    for off in (0, 1):
        src = torch.randint(0, 256, (nbytes + off,), dtype=torch.uint8, device=cuda)[off:]
        dst = torch.zeros(nbytes + off, dtype=torch.uint8, device=cuda)[off:]
        ctr = torch.full((1,), 41, dtype=torch.int64, device=cuda)
        MF.feed_step(dst, src, ctr)
        torch.testing.assert_close(dst, src, rtol=0, atol=0)
        assert int(ctr) == 42
        MF.feed_step(dst, src)  # no counter
    with pytest.raises(ValueError):
        MF.feed_step(torch.zeros(4, device=cuda), torch.zeros(5, device=cuda))


def test_graphed_step_feed_matches_separate_copy(cuda, msha):
    """GraphedStep.replay(feed=(dst, src)) (batch copy and replay-counter increment in one
    launch) replays the same steps as a separate copy + replay(): dropout 0.5, so every
    replay's masks depend on the counter."""
    from msha_gnn_amd.data import GroupAdjacency
    from msha_gnn_amd.step import GraphedStep

    z = golden("ours_small.npz")
    inter = msha.normalize_adjacency_matrix(t(z["counts"], cuda))
    city = GroupAdjacency(torch.as_tensor(z["city"], device=cuda))
    prov = GroupAdjacency(torch.as_tensor(z["prov"], device=cuda))
    src0 = torch.as_tensor(z["source_index"], device=cuda)
    n, m = z["counts"].shape
    g = torch.Generator().manual_seed(1)
    batches = [torch.randint(0, n, (src0.numel(),), generator=g).to(cuda) for _ in range(3)]
    tgt = torch.as_tensor(np.arange(src0.numel()) % m, device=cuda)
    runs = {}
    for fused in (False, True):
        model = _ours_model(z, cuda, 0.5)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, capturable=True)
        model.train()
        src_s = batches[0].clone()

        def body():
            opt.zero_grad(set_to_none=True)
            loss = F.nll_loss(model(inter, city, prov, src_s)[src_s], tgt)
            loss.backward()
            opt.step()
            return loss

        torch.manual_seed(0)
        gs = GraphedStep(body, cuda, warmup=1)
        losses = []
        for k in range(4):
            b = batches[k % len(batches)]
            if fused:
                out = gs.replay(feed=(src_s, b))
            else:
                src_s.copy_(b)
                out = gs.replay()
            losses.append(float(out.detach()))
        assert int(gs.counter) == 5
        gs.close()
        runs[fused] = (losses, {k: p.detach().clone() for k, p in model.named_parameters()})
    assert runs[True][0] == runs[False][0]
    for k, p in runs[False][1].items():
        torch.testing.assert_close(runs[True][1][k], p, rtol=0, atol=0, msg=k)


def test_two_graphed_steps_keep_their_counters(cuda, msha):
    """Two live GraphedSteps on one device: each replays fresh masks from its own
    counter; closing the newer one reinstalls the older one's counter (the library keeps
    one slot per device, msha_set_rng_counter), closing both leaves none.  A launch from
    a side stream of the device reads that device's counter."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph
    from msha_gnn_amd.step import GraphedStep

    rng = np.random.default_rng(4)
    c = random_counts(rng, 300, 32, 20)
    graph = Graph.from_dense(t(c, cuda))
    el, er = t(rng.standard_normal((300, 2)), cuda), t(rng.standard_normal((32, 2)), cuda)
    hc = t(rng.standard_normal((32, 2, 64)), cuda)

    def body():
        return MF.edge_attention(graph, el, er, hc, p=0.5, training=True, seed=9)

    assert MF.rng_counter(cuda) is None
    a = GraphedStep(body, cuda, warmup=1)
    b = GraphedStep(body, cuda, warmup=1)
    assert MF.rng_counter(cuda) is b.counter
    outs_a = [a.replay().clone() for _ in range(2)]
    outs_b = [b.replay().clone() for _ in range(2)]
    assert not torch.equal(outs_a[0], outs_a[1]) and not torch.equal(outs_b[0], outs_b[1])
    b.close()
    assert MF.rng_counter(cuda) is a.counter
    # eager draws follow the reinstalled counter (a's), also from a side stream
    side = torch.cuda.Stream(cuda)
    with torch.cuda.stream(side):
        a.counter.fill_(2)
        eager = body()
    side.synchronize()
    a.counter.fill_(1)
    a.replay()  # the graph's first node makes it 2 again
    assert torch.equal(a.out, eager)
    a.close()
    assert MF.rng_counter(cuda) is None
    assert msha._lib.load().msha_get_rng_counter(cuda.index) is None


def test_captured_workspaces_survive_cache_growth(cuda, msha):
    """workspaces recorded into a HIP graph belong to the graph's pool.  Two
    graphs of different workspace needs, captured on one stream, replay the eager results
    after an eager call on that stream grows (replaces) the shared scratch buffer and the
    freed memory is scribbled over."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph

    rng = np.random.default_rng(11)
    s = torch.cuda.Stream()
    cases = []
    for n in (300, 20000):
        c = random_counts(rng, n, 32, 20)
        graph = Graph.from_dense(t(c, cuda))
        el, er = t(rng.standard_normal((n, 2)), cuda), t(rng.standard_normal((32, 2)), cuda)
        hc = t(rng.standard_normal((32, 2, 64)), cuda)
        hs = t(rng.standard_normal((n, 2, 64)), cuda)
        cases.append((graph, el, er, hc, hs))
    s.wait_stream(torch.cuda.current_stream())
    refs, graphs, outs = [], [], []
    with torch.cuda.stream(s):
        for graph, el, er, hc, hs in cases:
            refs.append([x.clone() for x in MF.edge_attention(graph, el, er, hc, hs=hs)])
    for graph, el, er, hc, hs in cases:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            assert torch.cuda.is_current_stream_capturing()
            ws = MF._workspace(cuda, 1 << 20)
            assert all(ws.data_ptr() != w.data_ptr() for w in MF._WS.values())
            outs.append(MF.edge_attention(graph, el, er, hc, hs=hs))
        graphs.append(g)
    with torch.cuda.stream(s):
        big = MF._workspace(cuda, 256 << 20)  # replaces the stream's cached buffer
        big.fill_(0xFF)
        junk = [torch.full((1 << 20,), float("nan"), device=cuda) for _ in range(8)]
    torch.cuda.current_stream().wait_stream(s)
    for g, o, r in zip(graphs, outs, refs):
        g.replay()
        torch.cuda.synchronize()
        for a, b in zip(o, r):
            assert torch.equal(a, b)
    del junk


@pytest.mark.parametrize("kind", ["Ours", "ablation3"])
def test_model_replay_matches_eager(cuda, msha, kind):
    """replay.py: the drop-in model's training forward / backward replayed from its own
    HIP graphs under train.py's loop (torch Adam, F.nll_loss(output[src]), .item())
    gives the eager losses, parameters and BatchNorm running statistics (dropout 0), and
    draws fresh dropout masks per replay (dropout 0.5)."""
    from msha_gnn_amd import layers, replay
    from msha_gnn_amd.data import GroupAdjacency

    z = golden("ours_small.npz")
    inter = msha.normalize_adjacency_matrix(t(z["counts"], cuda))
    city = GroupAdjacency(torch.as_tensor(z["city"], device=cuda))
    prov = GroupAdjacency(torch.as_tensor(z["prov"], device=cuda))
    src = torch.as_tensor(z["source_index"], device=cuda)
    tgt = torch.as_tensor(np.arange(src.numel()) % z["counts"].shape[1], device=cuda)
    n, m = z["counts"].shape
    cls = layers.Ours if kind == "Ours" else layers.ablation3

    def make(p):
        torch.manual_seed(0)
        return cls(16, 8, m, 2, p, {i: 0.1 * i for i in range(n)}, n, m).to(cuda)

    runs = {}
    for rp in (False, True):
        replay.REPLAY = rp
        try:
            model = make(0.0)
            opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=5e-4)
            model.train()
            losses = []
            for _ in range(4):
                opt.zero_grad()
                out = model(inter, city, prov, src)
                loss = F.nll_loss(out[src], tgt)
                losses.append(loss.item())
                loss.backward()
                opt.step()
            if rp:
                assert model.__dict__.get("_msha_graphs"), "replay path not taken"
            runs[rp] = (losses, {k: v.detach().clone() for k, v in model.state_dict().items()})
        finally:
            replay.REPLAY = True
    np.testing.assert_allclose(runs[True][0], runs[False][0], rtol=1e-6)
    for k, v in runs[False][1].items():
        torch.testing.assert_close(runs[True][1][k], v, rtol=1e-5, atol=1e-6, msg=k)
    # dropout: every replay draws new masks
    model = make(0.5)
    model.train()
    outs = [model(inter, city, prov, src).detach().clone() for _ in range(3)]
    assert model.__dict__.get("_msha_graphs")
    assert not torch.equal(outs[1], outs[2]) and torch.isfinite(outs[2]).all()


def _ours_small(cuda, msha, kind="Ours", p=0.0):
    from msha_gnn_amd import layers
    from msha_gnn_amd.data import GroupAdjacency

    z = golden("ours_small.npz")
    inter = msha.normalize_adjacency_matrix(t(z["counts"], cuda))
    city = GroupAdjacency(torch.as_tensor(z["city"], device=cuda))
    prov = GroupAdjacency(torch.as_tensor(z["prov"], device=cuda))
    src = torch.as_tensor(z["source_index"], device=cuda)
    tgt = torch.as_tensor(np.arange(src.numel()) % z["counts"].shape[1], device=cuda)
    n, m = z["counts"].shape
    cls = layers.Ours if kind == "Ours" else layers.ablation3
    torch.manual_seed(0)
    model = cls(16, 8, m, 2, p, {i: 0.1 * i for i in range(n)}, n, m).to(cuda)
    model.train()
    return model, (inter, city, prov), src, tgt


def _grads(model):
    return {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("kind", ["Ours", "ablation3"])
def test_model_replay_accumulates_like_eager(cuda, msha, kind):
    """replay.py keeps torch's gradient semantics: two backward() calls without
    zero_grad() accumulate (the first .grad aliases the static buffer), and
    zero_grad(set_to_none=False) followed by a backward gives the new gradient."""
    from msha_gnn_amd import replay

    res = {}
    for rp in (False, True):
        replay.REPLAY = rp
        try:
            model, consts, src, tgt = _ours_small(cuda, msha, kind)
            for _ in range(2):  # settle the capture first (replay: warm-up + capture)
                model.zero_grad()
                F.nll_loss(model(*consts, src)[src], tgt).backward()
            model.zero_grad()
            F.nll_loss(model(*consts, src)[src], tgt).backward()
            one = _grads(model)
            F.nll_loss(model(*consts, src)[src], tgt).backward()  # no zero_grad: accumulate
            two = _grads(model)
            model.zero_grad(set_to_none=False)
            F.nll_loss(model(*consts, src)[src], tgt).backward()
            again = _grads(model)
            if rp:
                assert model.__dict__.get("_msha_graphs"), "replay path not taken"
            res[rp] = (one, two, again)
        finally:
            replay.REPLAY = True
    # (dropout 0, parameters unchanged: every backward adds the same gradient)
    for rp in (False, True):
        for k in res[rp][0]:
            one, two, again = (r[k] for r in res[rp])
            d2 = float((two - 2 * one).abs().max())
            da = float((again - one).abs().max())
            scale = float(one.abs().max())
            assert d2 <= 1e-6 * scale and da <= 1e-6 * scale, (
                f"replay={rp} {k}: |two - 2 one| {d2:.3g}, |again - one| {da:.3g}, max|one| {scale:.3g}")
    for k in res[False][0]:
        torch.testing.assert_close(res[True][0][k], res[False][0][k], rtol=1e-5, atol=1e-7, msg=k)


def test_model_replay_pending_output_and_stale_backward(cuda, msha):
    """Two forwards before one backward match eager (the second runs eagerly while the
    first output's backward is pending); an output held across iterations keeps its
    values; a backward of an output whose graph replayed a newer forward raises."""
    from msha_gnn_amd import replay

    res = {}
    for rp in (False, True):
        replay.REPLAY = rp
        try:
            model, consts, src, tgt = _ours_small(cuda, msha, "Ours")
            for _ in range(2):
                model.zero_grad()
                F.nll_loss(model(*consts, src)[src], tgt).backward()
            model.zero_grad()
            o1 = model(*consts, src)
            o2 = model(*consts, src)
            (F.nll_loss(o1[src], tgt) + 0.5 * F.nll_loss(o2[src], tgt)).backward()
            res[rp] = (o1.detach().clone(), o2.detach().clone(), _grads(model))
            if rp:
                held = o1.detach()
                snap = held.clone()
                model.zero_grad()
                F.nll_loss(model(*consts, src)[src], tgt).backward()
                assert torch.equal(held, snap), "held output changed by the next replay"
                l1 = F.nll_loss(model(*consts, src)[src], tgt)
                l1.backward(retain_graph=True)
                F.nll_loss(model(*consts, src)[src], tgt).backward()
                with pytest.raises(RuntimeError, match="newer forward"):
                    l1.backward()
        finally:
            replay.REPLAY = True
    torch.testing.assert_close(res[True][0], res[False][0], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(res[True][1], res[False][1], rtol=1e-6, atol=1e-6)
    for k, v in res[False][2].items():
        torch.testing.assert_close(res[True][2][k], v, rtol=1e-5, atol=1e-7, msg=k)


def test_model_replay_follows_replaced_parameter(cuda, msha):
    """A Parameter object replaced on the model is trained: the captured graphs are
    keyed on the current parameter objects, not a cached list."""
    from msha_gnn_amd import replay

    model, consts, src, tgt = _ours_small(cuda, msha, "ablation3")
    for _ in range(3):
        model.zero_grad()
        F.nll_loss(model(*consts, src)[src], tgt).backward()
    name, old = next((k, p) for k, p in model.named_parameters() if p.dim() == 2)
    mod = model
    *path, leaf = name.split(".")
    for a in path:
        mod = getattr(mod, a)
    old_grad = old.grad.detach().clone()
    new = torch.nn.Parameter(old.detach().clone() * 1.5)
    setattr(mod, leaf, new)
    model.zero_grad()
    F.nll_loss(model(*consts, src)[src], tgt).backward()
    assert new.grad is not None and torch.isfinite(new.grad).all()
    assert torch.equal(old.grad, old_grad), "the replaced parameter's gradient moved"
    replay.REPLAY = False
    try:
        model.zero_grad()
        ref = F.nll_loss(model(*consts, src)[src], tgt)
        ref.backward()
        want = new.grad.detach().clone()
    finally:
        replay.REPLAY = True
    model.zero_grad()
    F.nll_loss(model(*consts, src)[src], tgt).backward()
    torch.testing.assert_close(new.grad, want, rtol=1e-5, atol=1e-7)
