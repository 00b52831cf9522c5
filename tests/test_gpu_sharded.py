"""configs[4] on the GPU: the sharded link scorer through RCCL.

An in-process ``nccl`` (= RCCL) process group of world size 1 on cuda:0 (FileStore
rendezvous, no re-launch) drives ``ShardedTable``'s ``all_gather_into_tensor``
branch at C5 size (100k x 128 table, 4M pairs: 2M graph-like pairs + 2M uniform
negatives), scored by the HIP pair kernels (``functional.score_pairs``) -- 'mlp'
(hidden 128, the LinkPredictor's one applied Linear, LLP.py:104-115) and 'inner',
fp32 and bf16 tables -- against the oracle on 1,000 sampled pairs (fp64 on the same
storage-rounded inputs: 1e-5 fp32, 1e-2 bf16).  The caller contract is LLP.py:231-236
(h = MLP(x); predictor(h[source_index], h[recipient_index])).

Multi-rank correctness of the same code is covered over gloo (test_dist_gloo.py);
the 2/4/8-GPU RCCL curve is the driver's scaling run of bench.py.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

from gpu_helpers import bounded_close, tol_close
from oracle import gnn_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl1(cuda):
    import torch.distributed as dist

    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    fd, path = tempfile.mkstemp(prefix="msha_rccl1_")
    os.close(fd)
    os.unlink(path)
    store = dist.FileStore(path, 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=cuda)
    try:
        yield dist
    finally:
        dist.destroy_process_group()
        if os.path.exists(path):
            os.unlink(path)


@pytest.fixture(scope="module")
def c5(cuda):
    n, F, P, hidden = 100_000, 128, 4_000_000, 128
    g = torch.Generator().manual_seed(21)
    h = torch.rand(n, F, generator=g)
    rng = np.random.default_rng(22)
    # C5: half the batch graph-like pairs (local degree-2 ring), half uniform negatives
    a = rng.integers(0, n, P // 2)
    pos_s, pos_d = a, (a + rng.integers(1, 3, P // 2)) % n
    src = np.concatenate([pos_s, rng.integers(0, n, P // 2)])
    dst = np.concatenate([pos_d, rng.integers(0, n, P // 2)])
    W = torch.randn(hidden, F, generator=g) * F ** -0.5
    b = torch.randn(hidden, generator=g)
    return dict(n=n, F=F, P=P, h=h, src=torch.as_tensor(src, device=cuda),
                dst=torch.as_tensor(dst, device=cuda), W=W, b=b,
                pick=np.random.default_rng(23).choice(P, 50_000, replace=False))


def _ref(c, hh, mode, W=None, b=None):
    hd = hh.float().cpu().numpy().astype(np.float64)
    s = c["src"].cpu().numpy()[c["pick"]]
    d = c["dst"].cpu().numpy()[c["pick"]]
    lins = [] if W is None else [(W.float().cpu().numpy().astype(np.float64),
                                  b.cpu().numpy().astype(np.float64)), (None, None)]
    return O.score_pairs(hd, s, d, mode, lins)


def _terms(c, hh, mode, W=None, b=None):
    """Absolute terms of each score (sigmoid' <= 1/4 scales them): inner sum |x_i x_j|;
    mlp |x_i x_j| |W|^T + |b| (the hadamard product's rounding rides in the dot)."""
    hd = hh.float().cpu().numpy().astype(np.float64)
    x = np.abs(hd[c["src"].cpu().numpy()[c["pick"]]] * hd[c["dst"].cpu().numpy()[c["pick"]]])
    if mode == "inner":
        return 0.25 * x.sum(1), c["F"] + 1
    Wd = np.abs(W.float().cpu().numpy().astype(np.float64))
    return 0.25 * (x @ Wd.T + np.abs(b.cpu().numpy().astype(np.float64))), c["F"] + 2


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_rccl_world1_sharded_scorer(cuda, rccl1, c5, dt):
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd import sharding

    n, F = c5["n"], c5["F"]
    tab = sharding.ShardedTable(n, F, 1, 0, cuda, dtype=dt)
    assert tab.path() == "rccl"
    hh = c5["h"].to(dt)
    tab.set_local(hh.to(cuda))
    full = tab.gather()
    torch.cuda.synchronize()
    assert torch.equal(full.cpu(), hh)  # the gathered table is bit-exact
    tol = 1e-2 if dt == torch.bfloat16 else 1e-5
    W, b = c5["W"].to(dt).to(cuda), c5["b"].to(cuda)
    for mode in ("inner", "mlp"):
        if mode == "mlp":
            fn = lambda h_, s_, d_: MF.score_pairs(  # noqa: E731
                h_, s_, d_, "mlp", W, b, out_dtype=dt)
        else:
            fn = lambda h_, s_, d_: MF.score_pairs(h_, s_, d_, "inner")  # noqa: E731
        lo, hi, sc = sharding.score_sharded(tab, c5["src"], c5["dst"], fn)
        assert (lo, hi) == (0, c5["P"])
        got = sc.float().cpu().numpy()[c5["pick"]]
        ref = _ref(c5, hh, mode, *((W, b) if mode == "mlp" else ()))
        assert got.shape == ref.shape
        # every sampled score within tol |ref| + 4 sqrt(n) u A (its own terms; no
        # max|ref| floor): fp32 1e-5, bf16 1e-2 (bf16 table and bf16 mlp scores)
        A, nt = _terms(c5, hh, mode, *((W, b) if mode == "mlp" else ()))
        bounded_close(got, ref, A, nt, tol, f"{mode} {dt}")


def test_rccl_world1_pipelined_matches_serial(cuda, rccl1, c5):
    """Double-buffered gather/score (PipelinedScorer): each batch is scored against its
    own gathered table (the local rows change per batch) and the scores are the same
    bits as the serial gather-then-score of that batch."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd import sharding

    n, F = c5["n"], c5["F"]
    tab = sharding.ShardedTable(n, F, 1, 0, cuda, buffers=2)
    base = c5["h"].to(cuda)
    P = 1_000_000
    batches = [(c5["src"][k * P:(k + 1) * P], c5["dst"][k * P:(k + 1) * P]) for k in range(4)]
    W, b = c5["W"].to(cuda), c5["b"].to(cuda)
    fn = lambda h_, s_, d_: MF.score_pairs(h_, s_, d_, "mlp", W, b)  # noqa: E731

    def refresh(k):  # batch k's embeddings: a different table per batch
        tab.set_local(base * (1.0 + 0.25 * k))

    got = sharding.PipelinedScorer(tab, fn, refresh).run(batches)
    for k, (s_, d_) in enumerate(batches):
        refresh(k)
        lo, hi, want = sharding.score_sharded(tab, s_, d_, fn)
        assert got[k][:2] == (lo, hi)
        assert torch.equal(got[k][2], want), k
