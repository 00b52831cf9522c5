"""Benchmark: GAT layer forward+backward edges/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload syn100k|r15]

One step = one full GAT attention layer forward + backward over the whole graph
(SURVEY.md §8d, config C4 "synthetic CSR graph 100k nodes / 2M edges, 128-dim
features, 8 heads"):
    h = X @ W                     (100k x 128 @ 128 x 128, fp32)
    el, er = h . a_l, h . a_r     (per head, 8 heads x 16)
    u = softmax_row(lrelu(el_i + er_j)) @ h      <- msha_edge_attention_fwd (dominant)
    backward of all of it (msha_edge_attention_bwd_rows + msha_csc_aggregate + GEMMs)
Inputs are resident in HBM before the timed region.  For N > 1 GPUs the path
does not shard (SURVEY.md §8e "replicas only"): every rank runs its own replica
and value = total edges over all ranks / max-over-ranks time ("scaling": "weak").

The K timed steps run twice: eagerly, with HIP events around every edge-kernel launch
(the rooflines), then as ONE replay of a HIP graph that holds exactly those K steps
(the headline value: same kernels and work, without the host launch gaps of Python
autograd; ``--eager`` reports the eager pass instead).  Both are bracketed by a
barrier + synchronize and maxed over ranks.

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (HIP
events around every launch of it inside the eager timed region) and the CPU baseline
(the oracle's C restatement, timed on this host's cores, rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "edges/sec GAT fwd+bwd @1 GPU; link-score pairs/sec; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FUSED_ADAM = os.environ.get("MSHA_FUSED_ADAM", "1") != "0"


def synth_graph(n, e, seed=0):
    """C4 generator: e unique (row, col) pairs, rows sorted, cols uniform, deg >= 1."""
    rng = np.random.default_rng(seed)
    keys = np.arange(n, dtype=np.int64) * n + rng.integers(0, n, n)  # one edge per row
    while len(keys) < e:
        need = e - len(keys)
        extra = rng.integers(0, n, int(need * 1.05) + 16) * n + rng.integers(0, n,
                                                                            int(need * 1.05) + 16)
        keys = np.unique(np.concatenate([keys, extra]))
    if len(keys) > e:  # drop surplus without emptying a row
        rows = keys // n
        first = np.ones(len(keys), bool)
        first[1:] = rows[1:] != rows[:-1]
        cand = np.nonzero(~first)[0]
        drop = rng.choice(cand, len(keys) - e, replace=False)
        keys = np.delete(keys, drop)
    rows, col = keys // n, keys % n
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=n), out=rowptr[1:])
    return rowptr, col


def r15_graph():
    g = np.load(os.path.join(ROOT, "tests", "golden", "r15_graph.npz"))
    return g["rowptr"].astype(np.int64), g["col"].astype(np.int64), int(g["n"]), int(g["m"])


WORKLOADS = {
    "syn100k": dict(n=100_000, e=2_000_000, fin=128, heads=8, feat=16),
    "syn100k_f128": dict(n=100_000, e=2_000_000, fin=128, heads=8, feat=128),
    "syn2m": dict(n=2_000_000, e=40_000_000, fin=128, heads=8, feat=16),  # cache-busting
}


def pmc_traffic(H, F, bf16=False, workload="syn100k"):
    """HBM bytes per launch of the forward edge kernel from the newest committed PMC
    summary of this workload (profiles/*/pmc_summary.json, written by
    scripts/profile.sh + summarize_profile.py from separate rocprofv3 --pmc passes:
    FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE).  None if absent."""
    import glob
    import re

    pat = (re.compile(rf"edge_attn_fwd(?:_bat)?_kernelILi{H}ELi{F}EDF16b") if bf16 else
           re.compile(rf"edge_attn_fwd(?:_bat)?_kernel<{H}, {F}(, float)?(, \d+)?(, (true|false))?>"))

    def newest_first(path):  # round1_syn100k_v10 after _v9: compare the numbers
        tag = os.path.basename(os.path.dirname(path))
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", tag)]

    paths = glob.glob(os.path.join(ROOT, "profiles", f"*{workload}_v*", "pmc_summary.json"))
    for path in sorted(paths, key=newest_first, reverse=True):
        try:
            summ = json.load(open(path))
        except (OSError, ValueError):
            continue
        for k, v in summ.items():
            if pat.search(k) and v.get("hbm_bytes_per_launch_corrected"):
                return float(v["hbm_bytes_per_launch_corrected"]), os.path.relpath(path, ROOT)
    return None, None


def bwd_rows_bytes(n, m, e, H, F, s=4):
    """Algorithmic bytes of msha_edge_attention_bwd_rows (no v-branch): per edge col +
    er gather + s*D hc gather + the (de, attd) record; per row rowptr, el, lse, dU, u,
    d_el."""
    D = H * F
    return 4 * (n + 1) + e * (4 + 4 * H + s * D + 8 * H) + n * (12 * H + 2 * s * D)


def csc_bytes(m, e, H, F, n_chunks, s=4):
    """Algorithmic bytes of msha_csc_aggregate (d_hc, d_er): per CSC slot row + eid +
    the (attd, de) record + s*D dU gather; per column the outputs; the chunk plan."""
    D = H * F
    return e * (8 + 8 * H + s * D) + m * (s * D + 4 * H) + 12 * n_chunks + 4 * (m + 1)


def bwd_fused_bytes(n, m, e, H, F, n_chunks, s=4, rowterms=False):
    """Algorithmic bytes of msha_edge_attention_bwd_fused (its three launches):
    row stats (dU, u, el, lse in; the 3H-float row record out); the column pass (per
    CSC slot row + eid + the record gather + s*D dU gather + de write; per column hc,
    er in, d_hc, d_er out; the chunk plan); the row sum (rowptr, slot map, de, d_el).
    rowterms (msha_edge_attention_bwd_fused_ex with uc, qc; large graphs): the row
    stats also read uc (fp32 D floats), qc and the row flag and write d_el; the column
    pass writes no de; no row sum."""
    D = H * F
    stats = n * (2 * s * D + 8 * H + 12 * H)
    cols = e * (8 + 12 * H + s * D) + m * (2 * s * D + 8 * H) + 12 * n_chunks + 4 * (m + 1)
    if rowterms:
        return stats + n * (4 * D + 4 * H + 1 + 4 * H) + cols
    slot_map = 4 if e * 4 * H >= 192 << 20 else 0  # de in slot order (edge_attention.hip)
    rsum = 4 * (n + 1) + e * (4 * H + slot_map) + n * 4 * H
    return stats + cols + e * 4 * H + rsum


def fwd_bytes(n, m, e, H, F, s=4, rowterms=False):
    """Algorithmic bytes of one msha_edge_attention_fwd launch:
    rowptr + col + er gather + el + h gather (s*HF per edge) + u write + lse write;
    s = bytes per table element (4 fp32, 2 bf16); rowterms: + the uc (fp32) and qc
    writes of msha_edge_attention_fwd_ex."""
    rt = 4 * n * H * F + 4 * n * H if rowterms else 0
    return (4 * (n + 1) + 4 * e + 4 * e * H + 4 * n * H + s * e * H * F + s * n * H * F
            + 4 * n * H + rt)


class Layer:
    """The benchmarked GAT layer (one replica)."""

    def __init__(self, dev, rowptr, col, n, m, fin, H, F, seed, dtype=torch.float32, graph=None,
                 dropout=0.0):
        import msha_loader

        msha_loader.load()
        from msha_gnn_amd import functional as MF
        from msha_gnn_amd.graph import Graph

        self.MF = MF
        self.graph = graph if graph is not None else Graph.from_csr(rowptr, col, m, dev)
        g = torch.Generator().manual_seed(seed)
        self.n, self.m, self.H, self.F = n, m, H, F
        # dtype = storage of the feature table, W and the node tables (bf16: config C3)
        self.X = torch.rand(n, fin, generator=g).to(dev, dtype)
        # bipartite graphs (R15: sources x recipients) take a recipient feature table
        self.Xr = torch.rand(m, fin, generator=g).to(dev, dtype) if m != n else None
        self.W = (torch.randn(fin, H * F, generator=g) * fin ** -0.5).to(dev, dtype) \
            .requires_grad_(True)
        self.al = torch.randn(H, F, generator=g).to(dev).requires_grad_(True)
        self.ar = torch.randn(H, F, generator=g).to(dev).requires_grad_(True)
        self.dU = torch.randn(n, H, F, generator=g).to(dev, dtype)
        # attention dropout of the reference's training forward (Ablation.py:271): Philox
        # masks drawn inside the forward and regenerated by the backward
        self.p = dropout
        # the u-only fused backward takes the forward's row terms on large graphs
        # (msha_edge_attention_rowterms_preferred): their bytes enter the rooflines
        from msha_gnn_amd import _lib

        code = 1 if dtype == torch.bfloat16 else 0
        self.rowterms = bool(MF.ROWTERMS and MF.FUSED_BWD and _lib.load()
                             .msha_edge_attention_rowterms_preferred(self.graph.desc, H, F, code))

    def step(self):
        for p in (self.W, self.al, self.ar):
            p.grad = None
        # h = X @ W with the per-head score halves fused into the MFMA epilogue
        if self.Xr is None:
            h, el, er = self.MF.project_scores(self.X, self.W, self.al, self.ar, heads=self.H)
            hc = h.view(self.n, self.H, self.F)
        else:  # OursLayer3 shape (Ablation.py:262-274): h1 = R W (recipients), h2 = S W
            h1, er = self.MF.project_scores(self.Xr, self.W, ar=self.ar, heads=self.H)
            _, el = self.MF.project_scores(self.X, self.W, al=self.al, heads=self.H)
            hc = h1.view(self.m, self.H, self.F)
        u = self.MF.edge_attention(self.graph, el, er, hc, p=self.p, training=self.p > 0)
        u.backward(self.dU)


def link_score_bench(dev, rowptr, col, n, F, world, rank, dist, steps=16, warmup=3,
                     hidden=128, n_pairs=4_000_000, dtype=torch.float32, amortise=8):
    """score P = 4M pairs (2M graph edges + 2M uniform negatives,
    seed 1) against h (n x F) with LinkPredictor 'mlp' (hidden 128) and 'inner'.
    Rank r owns rows [r R, (r+1) R) of h (sharding.ShardedTable); one RCCL
    all_gather_into_tensor per batch rebuilds the full table (inside the timed
    loop), then each rank scores its contiguous P/W slice.  pairs/s over all ranks, with
    the all-gather once per batch (``pairs_per_sec_*``) and once per ``amortise`` batches
    (``pairs_per_sec_*_amortised``: the table is reused by k batches, as when one
    embedding pass is scored against many negative samples)."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd import sharding

    g = torch.Generator().manual_seed(1)
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    pick = np.random.default_rng(1).choice(len(col), n_pairs // 2, replace=False)
    src = np.concatenate([rows[pick], torch.randint(0, n, (n_pairs // 2,), generator=g).numpy()])
    dst = np.concatenate([col[pick], torch.randint(0, n, (n_pairs // 2,), generator=g).numpy()])
    t_src = torch.as_tensor(src, device=dev)
    t_dst = torch.as_tensor(dst, device=dev)
    table = sharding.ShardedTable(n, F, world, rank, dev, dtype=dtype)
    lo, hi = sharding.row_range(n, world, rank)
    table.set_local(torch.rand(hi - lo, F, generator=torch.Generator().manual_seed(10 + rank))
                    .to(dev, dtype))
    W = (torch.randn(hidden, F, generator=g) * F ** -0.5).to(dev, dtype)
    b = torch.randn(hidden, generator=g).to(dev)
    plo, phi = sharding.pair_range(n_pairs, world, rank)
    # a bf16 LinkPredictor returns bf16 scores (torch semantics); fp32 table: fp32
    out_mlp = torch.empty(phi - plo, hidden, device=dev, dtype=dtype)
    out_inner = torch.empty(phi - plo, device=dev)
    if dist:
        import torch.distributed as tdist
    fns = {"mlp": lambda h, s_, d_: MF.score_pairs(h, s_, d_, "mlp", W, b, out=out_mlp),
           "inner": lambda h, s_, d_: MF.score_pairs(h, s_, d_, "inner", out=out_inner)}
    res = {}
    plo_, phi_ = sharding.pair_range(n_pairs, world, rank)
    for mode in ("mlp", "inner"):
        for every, tag in ((1, ""), (amortise, "_amortised")):
            def one(k):
                if k % every == 0:
                    sharding.score_sharded(table, t_src, t_dst, fns[mode])
                else:  # the gathered table of the last all-gather is reused
                    fns[mode](table.full[:n], t_src[plo_:phi_], t_dst[plo_:phi_])
            for k in range(warmup):
                one(k)
            if dist:
                tdist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for k in range(steps):
                one(k)
            if dist:
                tdist.barrier()
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            if dist:
                tt = torch.tensor([dt], device=dev)
                tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
                dt = float(tt.item())
            res[f"pairs_per_sec_{mode}{tag}"] = n_pairs * steps / dt
            res[f"ms_per_batch_{mode}{tag}"] = dt / steps * 1e3
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        table.gather()
    torch.cuda.synchronize(dev)
    res["allgather_ms"] = (time.perf_counter() - t0) / steps * 1e3
    res.update(pairs_per_batch=n_pairs, feat=F, hidden=hidden, world=world,
               amortised_over_batches=amortise,
               dtype="bf16" if dtype == torch.bfloat16 else "f32",
               mlp_scores_dtype="bf16" if dtype == torch.bfloat16 else "f32",
               sharding="h rows all-gathered over RCCL (all_gather_into_tensor), pairs split "
               "contiguously per rank" if dist else "single GPU (no collective)")
    return res


def _year_graph(year):
    """(N, M, flows (F, 2), city ids, prov ids, gdp) of a shipped year; 2016-2018 flows
    are synthesised with the 2015 degree law (seed = year)."""
    import msha_loader

    msha_loader.load()
    from msha_gnn_amd.data import synthetic_flows

    z = np.load(os.path.join(ROOT, "tests", "golden", "r15_graph.npz"))
    yz = np.load(os.path.join(ROOT, "tests", "golden", "years.npz"))
    n, m = int(yz[f"{year}.n"]), int(yz[f"{year}.m"])
    rows15 = np.repeat(np.arange(int(z["n"])), np.diff(z["rowptr"]))
    col15 = z["col"].astype(np.int64)
    if year == "2015":
        cnt = z["cnt"].astype(np.int64)
        flows = np.stack([np.repeat(rows15, cnt), np.repeat(col15, cnt)], 1)
    else:
        deg_hist = np.bincount(np.diff(z["rowptr"]))
        col_w = np.bincount(col15, minlength=m).astype(np.float64)
        flows = synthetic_flows(n, m, deg_hist, col_w, seed=int(year))
    return n, m, flows, yz[f"{year}.city"].astype(np.int64), yz[f"{year}.prov"].astype(
        np.int64), yz[f"{year}.gdp"]


def train_step_leg(dev, year="2015", model_kind="Ours", steps=20, warmup=5,
                   dtype=torch.float32):
    """configs[1]: one train.py iteration (train.py:221-232) on a shipped year's graph:
    full-graph forward of the model (in 128, F 64, 2 heads, dropout 0.5), nll on a
    64-flow batch, backward, Adam(lr 1e-3, wd 5e-4) step.  model_kind: 'Ours' (full
    MSHA, Ours.py) or 'ablation3' (the model train.py:206 builds)."""
    import msha_loader

    msha = msha_loader.load()
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd import layers
    from msha_gnn_amd.data import GroupAdjacency

    n, m, flows, city, prov, gdp_arr = _year_graph(year)
    src_t = torch.as_tensor(flows[:, 0], device=dev)
    dst_t = torch.as_tensor(flows[:, 1], device=dev)
    adj = msha.normalize_adjacency_matrix(msha.inter_adjacency(src_t, dst_t, n, m))
    cadj = GroupAdjacency(torch.as_tensor(city, device=dev))
    padj = GroupAdjacency(torch.as_tensor(prov, device=dev))
    gdp = {i: float(x) for i, x in enumerate(gdp_arr)}
    torch.manual_seed(0)
    cls = layers.Ours if model_kind == "Ours" else layers.ablation3
    g = torch.Generator().manual_seed(0)
    picks = [torch.randint(0, len(flows), (64,), generator=g).to(dev) for _ in range(8)]
    batches = [(src_t[b], dst_t[b]) for b in picks]
    from msha_gnn_amd.graph import graph_for

    e = graph_for(adj).n_edges
    res = dict(model=model_kind, year=year, dtype=str(dtype).replace("torch.", ""), nodes=n,
               recipients=m, edges=e,
               flows="shipped" if year == "2015" else "synthetic (2015 degree law)")
    for mode in ("eager", "hip_graph"):
        torch.manual_seed(0)
        model = cls(128, 64, m, 2, 0.5, gdp, n, m).to(dev, dtype)
        graphed = mode == "hip_graph"
        # train.py's Adam (lr 1e-3, wd 5e-4); fused: one multi-tensor kernel per step
        # instead of ~50 foreach / per-tensor launches (same update rule)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=5e-4,
                               capturable=graphed, fused=FUSED_ADAM)
        model.train()
        si_s = torch.empty(64, dtype=torch.int64, device=dev)
        ri_s = torch.empty(64, dtype=torch.int64, device=dev)

        def body():
            opt.zero_grad(set_to_none=True)
            out = model(adj, cadj, padj, si_s)
            # train.py:229 F.nll_loss(output[source_index], recipient_index) as one launch
            # each way (msha_nll_rows_fwd/_bwd) instead of ~12 ATen launches
            loss = MF.nll_loss_rows(out, si_s, ri_s)
            loss.backward()
            opt.step()
            return loss

        def feed(k):
            si_s.copy_(batches[k % len(batches)][0])
            ri_s.copy_(batches[k % len(batches)][1])

        if graphed:
            from msha_gnn_amd.step import GraphedStep

            feed(0)
            gs = GraphedStep(body, dev, warmup=warmup)

            def one(k):
                feed(k)
                return gs.replay()
        else:
            def one(k):
                feed(k)
                return body()

            for k in range(warmup):
                one(k)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(steps):
            loss = one(k)
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / steps
        if graphed:
            gs.close()
        res[f"ms_per_step_{mode}"] = dt * 1e3
        res[f"loss_{mode}"] = float(loss.detach())
    res["ms_per_step"] = min(res["ms_per_step_eager"], res["ms_per_step_hip_graph"])
    res["edges_per_sec"] = e / (res["ms_per_step"] * 1e-3)
    return res


def cpu_baseline(rowptr, col, n, fin, H, F, budget_s=10.0):
    """Oracle C restatement of the same step (projection via numpy BLAS + edge-softmax
    aggregate fwd/bwd), whole graph, repeated for ~budget_s."""
    from oracle import cpu_oracle
    from oracle import gnn_oracle as O

    rng = np.random.default_rng(0)
    X = rng.random((n, fin), dtype=np.float32)
    W = (rng.standard_normal((fin, H * F)) * fin ** -0.5).astype(np.float32)
    al = rng.standard_normal((H, F)).astype(np.float32)
    ar = rng.standard_normal((H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    colptr, perm = O.csr_to_csc(rowptr, col, n)
    csc_row = O.edge_rows(rowptr)[perm]

    def one():
        h = (X @ W).reshape(n, H, F)
        el = np.einsum("nhf,hf->nh", h, al)
        er = np.einsum("nhf,hf->nh", h, ar)
        u, lse = cpu_oracle.edge_attention_fwd(rowptr, col, el, er, h)
        d_el, d_er, d_hc = cpu_oracle.edge_attention_bwd(rowptr, col, colptr, csc_row, perm, el,
                                                         er, h, lse, u, dU)
        dh = d_hc + d_el[:, :, None] * al[None] + d_er[:, :, None] * ar[None]
        dh = dh.reshape(n, H * F)
        _ = X.T @ dh  # dW

    one()  # warm-up (page-in, thread pool)
    t0 = time.perf_counter()
    reps = 0
    while True:
        one()
        reps += 1
        el_t = time.perf_counter() - t0
        if el_t >= budget_s or reps >= 50:
            break
    return dict(value=len(col) * reps / el_t, unit="edges/s", cores=cpu_oracle.threads(),
                kind="port",
                sample=f"whole graph ({n} rows, {len(col)} edges), {reps} fwd+bwd steps in "
                       f"{el_t:.1f}s: numpy X@W + oracle/edge_attention_cpu.c (OpenMP)")


def host_cpu():
    """lscpu-style host description: CPU model and the threads the CPU legs use."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"model": model, "cpus_visible": os.cpu_count(), "cpus_affinity": avail,
            "torch_threads": torch.get_num_threads()}


def cpu_baseline_r15(budget_s=10.0, dropout=0.5):
    """configs[1] CPU baseline: the reference's train.py iteration on the shipped 2015
    graph (ablation3, in 128, F 64, 2 heads, dropout 0.5, nll on 64 flows, Adam) in the
    reference's own dense formulation (oracle/dense_step.py, pinned to the reference's
    outputs and gradients by tests/test_oracle_golden.py), on this host's cores."""
    from oracle import dense_step as D

    z = np.load(os.path.join(ROOT, "tests", "golden", "r15_graph.npz"))
    n, m = int(z["n"]), int(z["m"])
    adj = torch.zeros(n, m)
    rows = torch.as_tensor(np.repeat(np.arange(n), np.diff(z["rowptr"])))
    adj[rows, torch.as_tensor(z["col"]).long()] = torch.as_tensor(z["norm"])
    p = D.init_params(n, m)
    opt = torch.optim.Adam(D.leaves(p), lr=1e-3, weight_decay=5e-4)
    g = torch.Generator().manual_seed(0)
    src, dst = torch.randint(0, n, (64,), generator=g), torch.randint(0, m, (64,), generator=g)
    D.train_step(p, opt, adj, src, dst, dropout)  # warm-up
    times = []
    t_end = time.perf_counter() + budget_s
    while len(times) < 2 or (time.perf_counter() < t_end and len(times) < 20):
        t0 = time.perf_counter()
        D.train_step(p, opt, adj, src, dst, dropout)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return dict(value=med, unit="s/step", higher_is_better=False, cores=torch.get_num_threads(),
                kind="port", edges_per_sec=len(z["col"]) / med,
                sample=f"ablation3 train step on the full 2015 graph ({n} x {m}), median of "
                       f"{len(times)} steps: oracle/dense_step.py (the reference's dense torch "
                       "formulation, CPU)")


def cpu_baseline_pairs(n, F, budget_s=4.0, hidden=128, n_pairs=1_000_000):
    """C5 CPU baseline: LinkPredictor 'mlp' (hidden 128) and 'inner' with the caller's
    gather (LLP.py:233, :104-115) on this host's cores, over a bounded 1M-pair sample of
    the same batch shape (oracle/dense_step.score_pairs, pinned to the reference's
    LinkPredictor outputs by tests/test_oracle_golden.py)."""
    from oracle import dense_step as D

    g = torch.Generator().manual_seed(1)
    h = torch.rand(n, F, generator=g)
    src = torch.randint(0, n, (n_pairs,), generator=g)
    dst = torch.randint(0, n, (n_pairs,), generator=g)
    W = torch.randn(hidden, F, generator=g) * F ** -0.5
    b = torch.randn(hidden, generator=g)
    res = {}
    with torch.no_grad():
        for mode in ("mlp", "inner"):
            D.score_pairs(h, src, dst, mode, W, b)
            reps, t0 = 0, time.perf_counter()
            while reps < 1 or (time.perf_counter() - t0 < budget_s / 2 and reps < 20):
                D.score_pairs(h, src, dst, mode, W, b)
                reps += 1
            res[f"pairs_per_sec_{mode}"] = n_pairs * reps / (time.perf_counter() - t0)
    res.update(unit="pairs/s", cores=torch.get_num_threads(), kind="port",
               sample=f"{n_pairs} pairs against a ({n}, {F}) fp32 table, hidden {hidden}: "
                      "oracle/dense_step.score_pairs (torch CPU)")
    return res


def launch_ranks(n, argv):
    """``bench.py --gpus N`` without a launcher: start N ranks through torch.distributed.run
    on 127.0.0.1 (this process never initialises the GPU) and return their exit status."""
    import socket
    import subprocess

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
    return subprocess.call(cmd + list(argv))


def dry_run(world, rank):
    """CPU rehearsal of the multi-rank path (gloo): rank launch, the sharded table's
    all-gather, the contiguous pair split and the max-over-ranks timing.  Prints one JSON
    line on rank 0 (n_gpus = ranks that took part)."""
    import torch.distributed as tdist

    from msha_loader import load

    load()
    from msha_gnn_amd import sharding

    if world > 1:
        tdist.init_process_group("gloo")
    n, F, P = 1001, 8, 5003
    tab = sharding.ShardedTable(n, F, world, rank, "cpu")
    lo, hi = sharding.row_range(n, world, rank)
    full_ref = torch.arange(n * F, dtype=torch.float32).view(n, F)
    tab.set_local(full_ref[lo:hi])
    t0 = time.perf_counter()
    ok = bool(torch.equal(tab.gather(), full_ref))
    plo, phi = sharding.pair_range(P, world, rank)
    dt = time.perf_counter() - t0
    cnt = torch.tensor([phi - plo, int(ok), 1], dtype=torch.float64)
    tt = torch.tensor([dt])
    if world > 1:
        tdist.all_reduce(cnt)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_reporting": int(cnt[2]),
                          "pairs_covered": int(cnt[0]), "pairs": P,
                          "table_ok_ranks": int(cnt[1]), "max_rank_s": float(tt)}), flush=True)
    if world > 1:
        tdist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="syn100k", choices=sorted(WORKLOADS) + ["r15"])
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-link-score", action="store_true")
    ap.add_argument("--no-r15", action="store_true")
    ap.add_argument("--no-bf16", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="report the eager launches (no HIP-graph replay of the timed steps)")
    ap.add_argument("--no-dropout-leg", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: rehearse the rank launch and the sharded table exchange over "
                         "gloo on the CPU (tests)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # one process per GPU: launch the ranks (before anything touches the GPU) and exit
        # with their status
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or 1)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if args.dry_run:
        return dry_run(world, rank)
    if dist:
        import torch.distributed as tdist

        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")
    dev = torch.device("cuda", local)

    if args.workload == "r15":
        rowptr, col, n, m = r15_graph()
        fin, H, F = 128, 2, 64
    else:
        w = WORKLOADS[args.workload]
        n, fin, H, F = w["n"], w["fin"], w["heads"], w["feat"]
        m = n
        rowptr, col = synth_graph(n, w["e"], seed=0)
    e = len(col)
    layer = Layer(dev, rowptr, col, n, m, fin, H, F, seed=1 + rank)

    def barrier():
        if dist:
            tdist.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(x):
        if dist:
            tt = torch.tensor([x], device=dev)
            tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
            x = float(tt.item())
        return x

    def timed_graph(lay, steps):
        """Max-over-ranks seconds of ONE replay of a HIP graph holding exactly `steps`
        steps (captured after the eager pass, which warmed every cache; one untimed
        replay first).  Same kernels, same work as the eager steps without the host
        launch gaps (~2-10 us per launch, Python autograd).  None if capture fails."""
        ok, g = 1, None
        try:
            g = torch.cuda.CUDAGraph()
            # thread_local: a communicator's watchdog thread (N > 1) may query its events
            # while this thread captures
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for _ in range(steps):
                    lay.step()
            g.replay()
        except RuntimeError as ex:  # report the eager number instead
            print(f"graph capture failed: {ex}", file=sys.stderr)
            ok = 0
        if dist:  # every rank falls back together (no rank left waiting in a barrier)
            t_ok = torch.tensor([ok], device=dev)
            tdist.all_reduce(t_ok, op=tdist.ReduceOp.MIN)
            ok = int(t_ok.item())
        if not ok:
            return None
        barrier()
        t0 = time.perf_counter()
        g.replay()
        barrier()
        dt_ = max_over_ranks(time.perf_counter() - t0)
        del g
        return dt_

    def timed(lay, steps, warmup):
        """(max-over-ranks seconds for `steps` steps, mean fwd-kernel ms, launches)"""
        for _ in range(warmup):
            lay.step()
        barrier()
        lay.MF.KERNEL_EVENTS = {}
        t0 = time.perf_counter()
        for _ in range(steps):
            lay.step()
        barrier()
        dt_ = time.perf_counter() - t0
        evs = lay.MF.KERNEL_EVENTS
        lay.MF.KERNEL_EVENTS = None
        ms = {name: float(np.mean([a.elapsed_time(b) for a, b in lst]))
              for name, lst in evs.items() if lst}
        events = evs.get("edge_attention_fwd", [])
        k = ms.get("edge_attention_fwd", float("nan"))
        dt_ = max_over_ranks(dt_)
        lay.kernel_ms = ms
        return dt_, k, len(events)

    def edge_kernels(lay, s):
        """Rooflines of the edge kernels of the step (HIP events, same run): the forward
        and either the fused backward or bwd_rows + csc_aggregate."""
        nch = lay.graph._plan["n_chunks"]
        rt = lay.rowterms
        out = []
        for name, nbytes in (("msha_edge_attention_fwd", fwd_bytes(n, m, e, H, F, s, rt)),
                             ("msha_edge_attention_bwd_rows", bwd_rows_bytes(n, m, e, H, F, s)),
                             ("msha_csc_aggregate", csc_bytes(m, e, H, F, nch, s)),
                             ("msha_edge_attention_bwd_fused",
                              bwd_fused_bytes(n, m, e, H, F, nch, s, rt))):
            key = name[len("msha_"):]
            if key not in lay.kernel_ms:
                continue
            us = lay.kernel_ms[key] * 1e3
            gbs = nbytes / (us * 1e-6) / 1e9
            out.append({"kernel": name, "algorithmic_bytes": nbytes, "avg_us": us,
                        "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS,
                        **({"rowterms": True} if rt and "rows" not in name
                           and "csc" not in name else {})})
        return out

    dt_eager, k_ms, n_launch = timed(layer, args.steps, args.warmup)
    dt_graph = None if args.eager else timed_graph(layer, args.steps)
    dt = dt_graph if dt_graph is not None else dt_eager
    timing = ("value: one replay of a HIP graph holding exactly `steps` steps (captured after "
              "the eager pass); roofline: HIP events around every launch over the eager timed "
              "region of the same steps" if dt_graph is not None else
              "value and roofline: eager launches, HIP events around every launch")
    drop_leg = None
    if not args.no_dropout_leg:
        # the reference's training forward drops attention at p = 0.5 (Ablation.py:271):
        # the same step with the Philox mask drawn in the forward and regenerated in the
        # backward (no mask tensor)
        layd = Layer(dev, rowptr, col, n, m, fin, H, F, seed=1 + rank, graph=layer.graph,
                     dropout=0.5)
        dtde, kd, nd = timed(layd, args.steps, args.warmup)
        dtdg = None if args.eager else timed_graph(layd, args.steps)
        dtd = dtdg if dtdg is not None else dtde
        ad = fwd_bytes(n, m, e, H, F, 4, layd.rowterms) / (kd * 1e-3) / 1e9
        drop_leg = {"workload": f"gat_layer_{args.workload}, attention dropout p = 0.5 "
                                "(training forward + backward)",
                    "value": world * e * args.steps / dtd, "unit": "edges/s",
                    "ms_per_step": dtd / args.steps * 1e3,
                    "ms_per_step_eager": dtde / args.steps * 1e3, "dtype": "f32",
                    "roofline": {"kernel": "msha_edge_attention_fwd (p = 0.5)", "bound": "hbm",
                                 "achieved": ad, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": ad / HBM_PEAK_GBS, "avg_launch_us": kd * 1e3,
                                 "launches_timed": nd},
                    "edge_kernels": edge_kernels(layd, 4)}
        del layd
    bf16_leg = None
    if not args.no_bf16:
        # config C3: the same layer with bf16 tables / projection (bf16 MFMA)
        lay16 = Layer(dev, rowptr, col, n, m, fin, H, F, seed=1 + rank, dtype=torch.bfloat16,
                      graph=layer.graph)
        dt16e, k16, n16 = timed(lay16, args.steps, args.warmup)
        dt16g = None if args.eager else timed_graph(lay16, args.steps)
        dt16 = dt16g if dt16g is not None else dt16e
        fb16 = fwd_bytes(n, m, e, H, F, 2, lay16.rowterms)
        a16 = fb16 / (k16 * 1e-3) / 1e9
        tr16, src16 = pmc_traffic(H, F, True, args.workload)
        bf16_leg = {"workload": f"gat_layer_{args.workload} (config C3: bf16 tables, bf16 MFMA "
                                "projection, fp32 scores/softmax)",
                    "value": world * e * args.steps / dt16, "unit": "edges/s",
                    "ms_per_step": dt16 / args.steps * 1e3,
                    "ms_per_step_eager": dt16e / args.steps * 1e3, "dtype": "bf16",
                    "roofline": {"kernel": "msha_edge_attention_fwd<bf16>", "bound": "hbm",
                                 "achieved": a16, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": a16 / HBM_PEAK_GBS, "traffic": tr16,
                                 "traffic_source": src16, "algorithmic_bytes_per_launch": fb16,
                                 "avg_launch_us": k16 * 1e3, "launches_timed": n16}}
        bf16_leg["edge_kernels"] = edge_kernels(lay16, 2)
        del lay16
    link = None
    if not args.no_link_score and args.workload != "r15":
        link = link_score_bench(dev, rowptr, col, n, H * F, world, rank, dist)
        if not args.no_bf16:  # C5 names a bf16 table
            link["bf16"] = link_score_bench(dev, rowptr, col, n, H * F, world, rank, dist,
                                            dtype=torch.bfloat16)
    if rank != 0:
        if dist:
            tdist.destroy_process_group()
        return
    ms_per_step = dt / args.steps * 1e3
    value = world * e * args.steps / dt
    fb = fwd_bytes(n, m, e, H, F, 4, layer.rowterms)
    achieved = fb / (k_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(H, F, False, args.workload)
    out = {
        "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "ms_per_step_eager": dt_eager / args.steps * 1e3, "timing": timing,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": f"gat_layer_{args.workload}", "nodes": n, "cols": m, "edges": e,
                   "in_features": fin, "heads": H, "feat": F, "parallelism": f"replicas{world}"},
        "roofline": {"kernel": "msha_edge_attention_fwd", "bound": "hbm",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "bytes per launch (rocprofv3 PMC, same command)",
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": fb, "avg_launch_us": k_ms * 1e3,
                     "launches_timed": n_launch},
    }
    out["edge_kernels"] = edge_kernels(layer, 4)
    if drop_leg is not None:
        out["dropout_p05"] = drop_leg
    if bf16_leg is not None:
        out["bf16"] = bf16_leg
    if link is not None:
        out["link_score"] = link
    if world == 1 and not args.no_r15:
        out["train_step_configs1"] = {
            "workload": "train.py iteration: full-graph fwd + nll(64 flows) + bwd + Adam; "
                        "in 128, F 64, 2 heads, dropout 0.5, fp32",
            "reference_cpu_s_per_step": "ablation3 @2015: see cpu_baseline.configs1_ablation3 "
                                        "(this host, same run); 1.01-1.27 on the 8-core build "
                                        "container (BASELINE.md)",
            "runs": [train_step_leg(dev, y, "Ours") for y in ("2015", "2016", "2017", "2018")]
            + [train_step_leg(dev, "2015", "ablation3")]}
        if not args.no_bf16:
            out["train_step_configs2"] = {
                "workload": "configs[2]: the same Ours model in bf16 (model.to(bfloat16): bf16 "
                            "parameters and node tables, bf16 MFMA projections, fp32 scores, "
                            "softmax and statistics), same step as configs[1]",
                "runs": [train_step_leg(dev, y, "Ours", dtype=torch.bfloat16)
                         for y in ("2015", "2016", "2017", "2018")]}
    if world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(rowptr, col, n, fin, H, F, args.cpu_budget)
        cb["host"] = host_cpu()
        if not args.no_r15:
            cb["configs1_ablation3"] = cpu_baseline_r15(args.cpu_budget)
        if link is not None:
            cb["link_score"] = cpu_baseline_pairs(n, H * F)
        out["cpu_baseline"] = cb
    print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
