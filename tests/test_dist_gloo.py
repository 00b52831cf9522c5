"""Multi-process (world_size 2, gloo on CPU) checks of the sharded link-scoring path
and of the bench's max-over-ranks timing.  The scoring function here is the CPU
oracle (tests only); on the GPU the same ShardedTable feeds functional.score_pairs
over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import msha_loader

        msha_loader.load()
        from msha_gnn_amd import sharding
        from oracle import gnn_oracle as O

        rng = np.random.default_rng(0)
        n, F, P = 1001, 16, 5003  # ragged: n and P not divisible by world
        h = rng.standard_normal((n, F)).astype(np.float32)
        src = rng.integers(0, n, P)
        dst = rng.integers(0, n, P)
        W = rng.standard_normal((8, F)).astype(np.float32)
        b = rng.standard_normal(8).astype(np.float32)
        tab = sharding.ShardedTable(n, F, world, rank, "cpu")
        lo, hi = sharding.row_range(n, world, rank)
        tab.set_local(torch.as_tensor(h[lo:hi]))
        full = tab.gather()
        assert torch.equal(full, torch.as_tensor(h))

        def score(hf, s, d):
            return torch.as_tensor(O.score_pairs(hf.numpy(), s.numpy(), d.numpy(), "mlp",
                                                 [(W, b), (None, None)]))

        plo, phi, sc = sharding.score_sharded(tab, torch.as_tensor(src), torch.as_tensor(dst),
                                              score)
        # reassemble on every rank and compare with the single-process result
        sizes = [sharding.pair_range(P, world, r) for r in range(world)]
        mx = max(b_ - a_ for a_, b_ in sizes)  # gloo all_gather needs equal shapes
        pad = torch.zeros(mx, 8)
        pad[: sc.shape[0]] = sc
        parts = [torch.empty(mx, 8) for _ in sizes]
        dist.all_gather(parts, pad)
        got = torch.cat([pt[: b_ - a_] for pt, (a_, b_) in zip(parts, sizes)]).numpy()
        ref = O.score_pairs(h, src, dst, "mlp", [(W, b), (None, None)])
        ok = np.allclose(got, ref, rtol=1e-6, atol=1e-6) and (plo, phi) == sizes[rank]
        # double-buffered gather/score: a different table per batch (refresh), each batch
        # scored against its own gather
        tab2 = sharding.ShardedTable(n, F, world, rank, "cpu", buffers=2)
        assert tab2.path() == "gloo"
        scale = [1.0, -2.0, 0.5]

        def refresh(k):
            tab2.set_local(torch.as_tensor(h[lo:hi] * scale[k]))

        bsz = [0, 1700, 3400, P]
        batches = [(torch.as_tensor(src[a:b_]), torch.as_tensor(dst[a:b_]))
                   for a, b_ in zip(bsz[:-1], bsz[1:])]
        outs = sharding.PipelinedScorer(tab2, score, refresh).run(batches)
        for k, (s_, d_) in enumerate(batches):
            a_, b_ = sharding.pair_range(s_.numel(), world, rank)
            want = O.score_pairs(h * scale[k], s_.numpy()[a_:b_], d_.numpy()[a_:b_], "mlp",
                                 [(W, b), (None, None)])
            ok = ok and outs[k][:2] == (a_, b_) and np.allclose(outs[k][2].numpy(), want,
                                                                rtol=1e-6, atol=1e-6)
        # a rank-local world-1 table inside this multi-process job: no
        # world-size error, its rows are copied
        solo = sharding.ShardedTable(n, F, 1, 0, "cpu")
        solo.set_local(torch.as_tensor(h))
        ok = ok and solo.path() == "copy" and torch.equal(solo.gather(), torch.as_tensor(h))
        # a world > 1 table that does not match the default group fails at construction
        # with the world-size message, not later in path()
        try:
            sharding.ShardedTable(n, F, world + 1, rank, "cpu")
            ok = False
        except ValueError as ex:
            ok = ok and "process group has" in str(ex)
        # bench.py's timing reduction: the max over ranks
        t = torch.tensor([0.5 + rank])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ok = ok and float(t) == 0.5 + world - 1
        q.put((rank, bool(ok)))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, f"{type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_scorer_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] is True for r in range(world)), res


def test_ranges_cover_exactly():
    import msha_loader

    msha_loader.load()
    from msha_gnn_amd import sharding

    for n, w in [(10, 3), (100000, 8), (7, 8)]:
        rows = [sharding.row_range(n, w, r) for r in range(w)]
        assert rows[0][0] == 0 and rows[-1][1] == n
        assert all(rows[i][1] == rows[i + 1][0] for i in range(w - 1))
        pairs = [sharding.pair_range(n, w, r) for r in range(w)]
        assert sum(b - a for a, b in pairs) == n
        assert max(b - a for a, b in pairs) - min(b - a for a, b in pairs) <= 1
