"""Benchmark: GAT layer forward+backward edges/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload syn100k|r15|...]

One step = one full GAT attention layer forward + backward over the whole graph
(SURVEY.md §8d, config C4 "synthetic CSR graph 100k nodes / 2M edges, 128-dim
features, 8 heads"):
    h = X @ W                     (100k x 128 @ 128 x 128, fp32)
    el, er = h . a_l, h . a_r     (per head, 8 heads x 16)
    u = softmax_row(lrelu(el_i + er_j)) @ h      <- msha_edge_attention_fwd (dominant)
    backward of all of it (fused backward + GEMMs)
Inputs are resident in HBM before the timed region.  For N > 1 GPUs the layer does
not shard (SURVEY.md §8e "replicas only"): every rank runs its own replica and value
= total edges over all ranks / max-over-ranks time ("scaling": "weak").

The K timed steps run twice: eagerly, with HIP events around every edge-kernel launch
(the rooflines), then as ONE replay of a HIP graph that holds exactly those K steps
(the headline value: same kernels and work, without the host launch gaps of Python
autograd; ``--eager`` reports the eager pass instead).  Both are bracketed by a
barrier + synchronize and maxed over ranks.

Further legs in the same JSON line (same timing rules):
  * ``bf16``    config C3 at C4 (bf16 tables, bf16 MFMA projection);
  * ``syn2m``   the cache-busting variant (2M nodes, 40M edges: a 1 GB fp32 table
                outside the 256 MB Infinity Cache), fp32 and bf16;
  * ``bip1m``   the repo's adjacency shape at scale: 1M sources x 32 recipients with
                the 2015 degree law and column weights, the OursLayer3 core (in 128,
                2 heads x 64, u = att @ h1 AND v = att.T @ h2, Ablation.py:260-277);
  * ``link_score`` config C5: 4M pairs against a 100k x 128 table through the RCCL
                all-gather of ShardedTable (a world-1 group on one GPU);
  * ``train_step_configs1/2`` the train.py iteration on the shipped graphs.
Rank 0 prints ONE JSON line with the roofline of the dominant kernel (HIP events
around every launch of it inside the eager timed region) and the CPU baseline (the
oracle's C restatement, timed on this host's cores, rank 0, N=1 only).
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
F32_MFMA_TFLOPS = 157.3  # exact-fp32 matrix peak (v_mfma_f32_*x*_f32), MI355X_MICROARCH.md
BF16_MFMA_TFLOPS = 2500.0  # dense bf16 MFMA peak (no sparsity)
FUSED_ADAM = os.environ.get("MSHA_FUSED_ADAM", "1") != "0"
# the train-step legs' optimizer: "msha" = msha_gnn_amd.optim.Adam (one launch, Sfeatures
# updated inside its feature-dropout backward), "torch" = torch.optim.Adam (A/B)
ADAM = os.environ.get("MSHA_ADAM", "msha")


def synth_graph(n, e, seed=0):
    """C4 generator: e unique (row, col) pairs, rows sorted, cols uniform, deg >= 1.
    numpy's PCG64 stream (seed 0), not the torch.Generator SURVEY §8d names: the graph's
    law is the one §8d specifies, the exact edges are this generator's."""
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


def bip_graph(n=1_000_000, seed=1015):
    """SURVEY.md §8d C4's repo-shape bipartite generator: n sources x 32 recipients,
    per-source degree from the shipped 2015 degree histogram, recipients drawn without
    replacement in proportion to the 2015 column nnz (data.synthetic_csr)."""
    import msha_loader

    msha_loader.load()
    from msha_gnn_amd.data import synthetic_csr

    z = np.load(os.path.join(ROOT, "tests", "golden", "r15_graph.npz"))
    m = int(z["m"])
    deg_hist = np.bincount(np.diff(z["rowptr"]))
    col_w = np.bincount(z["col"].astype(np.int64), minlength=m).astype(np.float64)
    rowptr, col = synthetic_csr(n, m, deg_hist, col_w, seed)
    return rowptr, col, n, m


WORKLOADS = {
    "syn100k": dict(n=100_000, e=2_000_000, fin=128, heads=8, feat=16),
    "syn100k_f128": dict(n=100_000, e=2_000_000, fin=128, heads=8, feat=128),
    "syn2m": dict(n=2_000_000, e=40_000_000, fin=128, heads=8, feat=16),  # cache-busting
    "bip1m": dict(n=1_000_000, fin=128, heads=2, feat=64),  # repo shape: 1M x 32
}


def _newest_first(path):  # round1_syn100k_v10 after _v9: compare the numbers
    import re

    tag = os.path.basename(os.path.dirname(path))
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", tag)]


def kernel_source_id() -> str:
    """Identity of the HIP sources the library is built from: sha256 over
    msha--gnn_amd/csrc/*.hip|*.h and include/*.h (sorted).  scripts/profile.sh records it
    with each profile; pmc_lookup attaches PMC traffic only from a profile of the same
    sources (no traffic figure from a different build)."""
    import glob
    import hashlib

    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "msha--gnn_amd", "csrc", "*.hip"))
                   + glob.glob(os.path.join(ROOT, "msha--gnn_amd", "csrc", "*.h"))
                   + glob.glob(os.path.join(ROOT, "include", "*.h")))
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def _source_files():
    import glob

    return sorted(glob.glob(os.path.join(ROOT, "msha--gnn_amd", "csrc", "*.hip"))
                  + glob.glob(os.path.join(ROOT, "msha--gnn_amd", "csrc", "*.h"))
                  + glob.glob(os.path.join(ROOT, "include", "*.h")))


def kernel_source_files() -> dict:
    """Per-file identity of the sources (basename -> sha256[:16]), recorded with each
    profile beside kernel_source_id: a profile stays valid for a kernel while the file
    that defines it and every header are unchanged."""
    import hashlib

    return {os.path.basename(f): hashlib.sha256(open(f, "rb").read()).hexdigest()[:16]
            for f in _source_files()}


def _kernel_defs() -> dict:
    """__global__ kernel name -> the .hip file defining it."""
    import re

    out = {}
    for f in _source_files():
        if f.endswith(".hip"):
            for m in re.finditer(r"__global__[\s\S]{0,200}?\b(\w+_kernel)\s*\(", open(f).read()):
                out.setdefault(m.group(1), os.path.basename(f))
    return out


def _same_sources(meta: dict, kernels) -> bool:
    """Whether a profile (its _meta) measured this build's code for ``kernels`` (profile
    kernel names): the whole-tree id matches, or the per-file ids of every header and of
    the files defining those kernels do."""
    if meta.get("source_id") == kernel_source_id():
        return True
    files = meta.get("source_files")
    if not files:
        return False
    cur, defs = kernel_source_files(), _kernel_defs()
    need = {f for f in cur if f.endswith(".h")}
    for k in kernels:
        hit = [n for n in defs if n in k]
        if not hit:
            return False
        need.add(defs[max(hit, key=len)])
    return all(files.get(f) == cur[f] for f in need)


def pmc_lookup(patterns, glob_pat, profiles_dir=None):
    """HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction) summed over
    the kernels matching ``patterns`` (regexes; each must match a kernel of the same
    summary, several matches of one pattern are averaged) in the newest committed profile matching ``glob_pat``
    (profiles/<glob>/pmc_summary.json, written by scripts/summarize_profile.py from
    separate rocprofv3 --pmc passes) whose recorded source id is this build's
    (kernel_source_id), or whose per-file ids match for the headers and the files that
    define the matched kernels (_same_sources).  (None, None) if absent; (None, note) if
    only profiles of other sources exist."""
    import glob
    import re

    pats = [re.compile(p) for p in patterns]
    stale = None
    pdir = profiles_dir or os.path.join(ROOT, "profiles")
    for path in sorted(glob.glob(os.path.join(pdir, glob_pat, "pmc_summary.json")),
                       key=_newest_first, reverse=True):
        try:
            summ = json.load(open(path))
        except (OSError, ValueError):
            continue
        keys = [k for k in summ if any(p.search(k) for p in pats)]
        if not _same_sources(summ.get("_meta", {}), keys):
            stale = stale or os.path.relpath(path, ROOT)
            continue
        tot, ok = 0.0, True
        for p in pats:
            hit = [v for k, v in summ.items() if p.search(k)
                   and v.get("hbm_bytes_per_launch_corrected")]
            if not hit:
                ok = False
                break
            # (several instances of one pattern, e.g. the u and v aggregates: their mean)
            tot += sum(float(h["hbm_bytes_per_launch_corrected"]) for h in hit) / len(hit)
        if ok:
            return tot, os.path.relpath(path, ROOT)
    if stale is not None:  # the newest profile is of other sources: no traffic figure
        return None, f"none of this build (newest: {stale}, other sources)"
    return None, None


def fwd_kernel_pattern(H, F, bf16, variant="bat", rowterms=None):
    """rocprofv3 name of the forward edge kernel (fp32 demangled, bf16 mangled or
    demangled with the type as "bool _Accum"): variant 'rs' (gather layout, scores from
    the row), 'gl' (gather layout, er table: short rows) or 'bat' (score layout, er
    table); rowterms (None = either) pins the instantiation's row-term flag."""
    rt = "(true|false)" if rowterms is None else ("true" if rowterms else "false")
    rtb = "[01]" if rowterms is None else str(int(bool(rowterms)))
    if variant in ("rs", "gl"):
        rs = "true" if variant == "rs" else "false"
        # <H, F, T, NGI, RT, RS, ATTD, PF>; profiles before the PF flag end at ATTD, and
        # the demangled bf16 names of the PF build show only the last three (RS, ATTD, PF)
        return (rf"edge_attn_fwd_gl_kernel(ILi{H}ELi{F}EDF16bLi\d+ELb{rtb}ELb{int(variant == 'rs')}"
                rf"|<{H}, {F}, bool _Accum, .*, {rt}, {rs}, (true|false)>"
                rf"|<{H}, {F}, bool _Accum, .*E, {rs}, (true|false), (true|false)>)"
                if bf16 else rf"edge_attn_fwd_gl_kernel<{H}, {F}, float, \d+, {rt}, {rs}")
    # <H, F, T, EPL, RT>
    return (rf"edge_attn_fwd(?:_bat)?_kernel(ILi{H}ELi{F}EDF16bLi\d+ELb{rtb}|<{H}, {F}, bool _Accum)"
            if bf16 else rf"edge_attn_fwd(?:_bat)?_kernel<{H}, {F}, float, \d+, {rt}>")


def pmc_traffic(H, F, bf16=False, workload="syn100k", variant="bat", rowterms=None):
    """HBM bytes per launch of the forward edge kernel from the newest committed PMC
    summary of this workload (None if absent)."""
    return pmc_lookup([fwd_kernel_pattern(H, F, bf16, variant, rowterms)], f"*{workload}_v*")


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
    pass writes no de; no row sum.  (With row scores the column pass reads a_r instead
    of er_j: the same 4H bytes per column.)"""
    D = H * F
    stats = n * (2 * s * D + 8 * H + 12 * H)
    cols = e * (8 + 12 * H + s * D) + m * (2 * s * D + 8 * H) + 12 * n_chunks + 4 * (m + 1)
    if rowterms:
        return stats + n * (4 * D + 4 * H + 1 + 4 * H) + cols
    slot_map = 4 if e * 4 * H >= 192 << 20 else 0  # de in slot order (edge_attention.hip)
    rsum = 4 * (n + 1) + e * (4 * H + slot_map) + n * 4 * H
    return stats + cols + e * 4 * H + rsum


def fwd_bytes(n, m, e, H, F, s=4, rowterms=False, row_scores=False, attd=False):
    """Algorithmic bytes of one forward edge-kernel launch:
    rowptr + col + er gather + el + h gather (s*HF per edge) + u write + lse write;
    s = bytes per table element (4 fp32, 2 bf16); rowterms: + the uc (fp32) and qc
    writes; row_scores (msha_edge_attention_fwd_rs): no er gather (er_j comes from the
    gathered row); attd: + the (E, H) post-dropout attention write (v-branch path)."""
    rt = 4 * n * H * F + 4 * n * H if rowterms else 0
    er = 0 if row_scores else 4 * e * H
    return (4 * (n + 1) + 4 * e + er + 4 * n * H + s * e * H * F + s * n * H * F
            + 4 * n * H + rt + (4 * e * H if attd else 0))


def bip_fwd_bytes(n, m, e, H, F, s=4, hs=False, attd=False):
    """Compulsory HBM bytes of msha_bip_attention_fwd (edge_bip.hip): per row rowptr, el,
    the u write and lse (+ the hs read with the v branch); per edge its column (+ the
    attention export); the column side (hc, er; v out) once.  hc_j is read from LDS, not
    gathered per edge, so no per-edge table bytes."""
    D = H * F
    return (4 * (n + 1) + 4 * e + 4 * n * H + s * n * D + 4 * n * H + (s * n * D if hs else 0)
            + (4 * e * H if attd else 0) + m * (s * D + 4 * H) + (s * m * D if hs else 0))


def bip_bwd_bytes(n, m, e, H, F, s=4, hs=False):
    """Compulsory HBM bytes of msha_bip_attention_bwd: per row rowptr, el, lse, dU in,
    d_el out (+ hs in and d_hs out with the v branch); per edge its column; the column
    side (hc, er, dV in; d_hc, d_er out) once."""
    D = H * F
    return (4 * (n + 1) + 4 * e + 8 * n * H + s * n * D + 4 * n * H
            + (2 * s * n * D if hs else 0) + m * (s * D + 4 * H) * 2 + (s * m * D if hs else 0))


class Layer:
    """The benchmarked GAT layer (one replica).  Square graphs (C4, syn2m): h = X W is
    both the gathered table and the score source (u-only).  Bipartite graphs (R15,
    bip1m): the OursLayer3 core, h1 = R W (recipients, gathered), h2 = S W (sources);
    ``v_branch`` also aggregates v = att.T @ h2 (Ablation.py:273)."""

    def __init__(self, dev, rowptr, col, n, m, fin, H, F, seed, dtype=torch.float32, graph=None,
                 dropout=0.0, v_branch=False):
        import msha_loader

        msha_loader.load()
        from msha_gnn_amd import _lib
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
        self.v_branch = bool(v_branch and self.Xr is not None)
        self.dV = torch.randn(m, H, F, generator=g).to(dev, dtype) if self.v_branch else None
        # attention dropout of the reference's training forward (Ablation.py:271): Philox
        # masks drawn inside the forward and regenerated by the backward
        self.p = dropout
        code = 1 if dtype == torch.bfloat16 else 0
        lib = _lib.load()
        # the u-only fused backward takes the forward's row terms on large graphs
        # (msha_edge_attention_rowterms_preferred), and its scores come from the gathered
        # rows (msha_edge_attention_fwd_rs): both enter the rooflines' byte counts
        self.rowterms = bool(not self.v_branch and MF.ROWTERMS and MF.FUSED_BWD
                             and lib.msha_edge_attention_rowterms_preferred(self.graph.desc, H,
                                                                            F, code))
        self.row_scores = bool(not self.v_branch and MF.ROW_SCORES and MF.FUSED_BWD
                               and lib.msha_edge_attention_row_scores_preferred(self.graph.desc,
                                                                                H, F, code))
        short = self.graph.n_edges <= 8 * n and os.environ.get("MSHA_FWD_GL", "1") != "0"
        self.fwd_variant = "rs" if self.row_scores else ("gl" if short else "bat")
        # the repo's adjacency shape (M <= 32 recipients): msha_bip_attention_fwd/_bwd
        self.bip = bool(self.v_branch and MF.bip_ok(self.graph, H, F, dtype))
        if self.bip:
            self.rowterms = self.row_scores = False
            self.fwd_variant = "bip"

    def step(self):
        for p in (self.W, self.al, self.ar):
            p.grad = None
        # h = X @ W with the per-head score halves fused into the MFMA epilogue
        if self.Xr is None:
            h, el, er = self.MF.project_scores(self.X, self.W, self.al, self.ar, heads=self.H)
            hc = h.view(self.n, self.H, self.F)
            hs = None
        else:  # OursLayer3 shape (Ablation.py:262-274): h1 = R W (recipients), h2 = S W
            h1, er = self.MF.project_scores(self.Xr, self.W, ar=self.ar, heads=self.H)
            h2, el = self.MF.project_scores(self.X, self.W, al=self.al, heads=self.H)
            hc = h1.view(self.m, self.H, self.F)
            hs = h2.view(self.n, self.H, self.F) if self.v_branch else None
        # er = hc . a_r: the u-only kernels recompute it from the rows they gather
        out = self.MF.edge_attention(self.graph, el, er, hc, hs=hs, p=self.p,
                                     training=self.p > 0, ar=self.ar)
        if hs is None:
            out.backward(self.dU)
        else:
            torch.autograd.backward(list(out), [self.dU, self.dV])


class Clock:
    """Barrier + synchronize bracketing and max-over-ranks reduction (one per run)."""

    def __init__(self, dev, dist):
        self.dev, self.dist = dev, dist
        if dist:
            import torch.distributed as tdist

            self.tdist = tdist

    def barrier(self):
        if self.dist:
            self.tdist.barrier()
        torch.cuda.synchronize(self.dev)

    def max_over_ranks(self, x):
        if self.dist:
            tt = torch.tensor([x], device=self.dev)
            self.tdist.all_reduce(tt, op=self.tdist.ReduceOp.MAX)
            x = float(tt.item())
        return x

    def timed_graph(self, lay, steps):
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
        if self.dist:  # every rank falls back together (no rank left waiting in a barrier)
            t_ok = torch.tensor([ok], device=self.dev)
            self.tdist.all_reduce(t_ok, op=self.tdist.ReduceOp.MIN)
            ok = int(t_ok.item())
        if not ok:
            return None
        self.barrier()
        t0 = time.perf_counter()
        g.replay()
        self.barrier()
        dt_ = self.max_over_ranks(time.perf_counter() - t0)
        del g
        return dt_

    def timed(self, lay, steps, warmup):
        """(max-over-ranks seconds for `steps` eager steps, mean fwd-kernel ms, launches);
        lay.kernel_ms: mean HIP-event ms of every bracketed edge-kernel launch."""
        for _ in range(warmup):
            lay.step()
        self.barrier()
        lay.MF.KERNEL_EVENTS = {}
        t0 = time.perf_counter()
        for _ in range(steps):
            lay.step()
        self.barrier()
        dt_ = time.perf_counter() - t0
        evs = lay.MF.KERNEL_EVENTS
        lay.MF.KERNEL_EVENTS = None
        ms = {name: float(np.mean([a.elapsed_time(b) for a, b in lst]))
              for name, lst in evs.items() if lst}
        fk = "bip_attention_fwd" if getattr(lay, "bip", False) else "edge_attention_fwd"
        events = evs.get(fk, [])
        k = ms.get(fk, float("nan"))
        dt_ = self.max_over_ranks(dt_)
        lay.kernel_ms = ms
        return dt_, k, len(events)


def bip_kernel_patterns(H, F, bf, hs):
    """rocprofv3 names of the bipartite forward / backward kernels: the MFMA kernels
    (edge_bip3.hip, <T, HS, ATTD, DROP> / <T, HS, COEF, DROP>), the mask kernels
    (edge_bip2.hip, <T, HS, ATTD> / <T, HS, COEF, DROP>) or the CSR-walk ones (edge_bip.hip,
    <H, F, T, HS, ATTD, HT> / <H, F, T, ...>), whichever the library chose; bf16
    instances stay mangled (DF16b) or demangle the type as "bool _Accum"."""
    h = str(bool(hs)).lower()
    if bf:
        fwd = (rf"(bip_fwd_kernel(ILi{H}ELi{F}EDF16bLb{int(hs)}E|<{H}, {F}, bool _Accum, "
               rf"bool, E, false(, \d+)?>)|bip[23]_fwd_kernel(IDF16bLb{int(hs)}E|<bool _Accum|<__bf16, {h}))")
        bwd = (rf"(bip_bwd_kernel(ILi{H}ELi{F}EDF16b|<{H}, {F}, bool _Accum)"
               rf"|bip[23]_bwd_kernel(IDF16bLb{int(hs)}E|<bool _Accum|<__bf16, {h}))")
    else:
        fwd = (rf"(bip_fwd_kernel<{H}, {F}, float, {h}, false(, \d+)?>"
               rf"|bip[23]_fwd_kernel<float, {h}, (true|false)(, false)?>)")
        bwd = rf"(bip_bwd_kernel<{H}, {F}, float|bip[23]_bwd_kernel<float, {h},)"
    return fwd, bwd


def edge_kernels(lay, n, m, e, H, F, s, workload=None):
    """Rooflines of the edge kernels of the step (HIP events, same run): the forward and
    either the fused backward or bwd_rows + csc_aggregate; PMC traffic per launch from
    the newest committed profile of ``workload`` where one covers the kernel."""
    nch = lay.graph._plan["n_chunks"]
    rt, rs = lay.rowterms, lay.row_scores
    bf = s == 2
    # rocprofv3 leaves most bf16 instantiations mangled (DF16b) and demangles some with
    # the bf16 type as "bool _Accum"; fp32 ones are demangled
    tmpl = ((lambda k: rf"{k}(ILi{H}ELi{F}EDF16b|<{H}, {F}, bool _Accum)") if bf else
            (lambda k: rf"{k}<{H}, {F}, float"))
    pats = {
        "msha_edge_attention_fwd": [fwd_kernel_pattern(H, F, bf, lay.fwd_variant, rt)],
        # (bwd_row_stats_kernel<H, F, T, RT>: the flag pins the instantiation where the
        # name keeps it)
        "msha_edge_attention_bwd_fused": [tmpl("bwd_row_stats_kernel")
                                          + (rf"(Lb{int(rt)}E|, {str(rt).lower()}>|, bool, E>)"
                                             if bf else rf", {str(rt).lower()}>"),
                                          tmpl("bwd_cols(_eh)?_kernel")]
        + ([] if rt else [rf"bwd_row_sum_kernel(<{H}>|ILi{H}E)"]),
        "msha_edge_attention_bwd_rows": [tmpl("edge_attn_bwd_rows(_gl)?_kernel")],
        "msha_csc_aggregate": [tmpl("csc_aggregate_kernel")],
        "msha_bip_attention_fwd": [bip_kernel_patterns(H, F, bf, lay.v_branch)[0]],
        "msha_bip_attention_bwd": [bip_kernel_patterns(H, F, bf, lay.v_branch)[1]],
    }
    out = []
    v = lay.v_branch
    for name, nbytes in (("msha_edge_attention_fwd",
                          fwd_bytes(n, m, e, H, F, s, rt, rs, attd=v)),
                         ("msha_edge_attention_bwd_rows", bwd_rows_bytes(n, m, e, H, F, s)),
                         ("msha_csc_aggregate", csc_bytes(m, e, H, F, nch, s)),
                         ("msha_edge_attention_bwd_fused",
                          bwd_fused_bytes(n, m, e, H, F, nch, s, rt)),
                         ("msha_bip_attention_fwd", bip_fwd_bytes(n, m, e, H, F, s, hs=v)),
                         ("msha_bip_attention_bwd", bip_bwd_bytes(n, m, e, H, F, s, hs=v))):
        key = name[len("msha_"):]
        if key not in lay.kernel_ms:
            continue
        us = lay.kernel_ms[key] * 1e3
        gbs = nbytes / (us * 1e-6) / 1e9
        row = {"kernel": name, "algorithmic_bytes": nbytes, "avg_us": us,
               "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS}
        if rt and "rows" not in name and "csc" not in name:
            row["rowterms"] = True
        if rs and name != "msha_csc_aggregate" and "rows" not in name:
            row["row_scores"] = True
        if workload and name in pats:
            tr, src = pmc_lookup(pats[name], f"*{workload}_v*")
            if tr is not None:
                row["traffic"], row["traffic_source"] = tr, src
        out.append(row)
    return out


def layer_leg(clock, dev, label, rowptr, col, n, m, fin, H, F, steps, warmup, world, eager,
              dtype=torch.float32, graph=None, dropout=0.0, v_branch=False, workload=None):
    """One timed layer configuration: edges/s (HIP-graph replay unless eager), the forward
    kernel's roofline and the edge-kernel table.  Returns (dict, layer's graph)."""
    e = len(col)
    s = 2 if dtype == torch.bfloat16 else 4
    lay = Layer(dev, rowptr, col, n, m, fin, H, F, seed=1, dtype=dtype, graph=graph,
                dropout=dropout, v_branch=v_branch)
    dte, k_ms, nl = clock.timed(lay, steps, warmup)
    dtg = None if eager else clock.timed_graph(lay, steps)
    dt = dtg if dtg is not None else dte
    if lay.bip:
        fb = bip_fwd_bytes(n, m, e, H, F, s, hs=lay.v_branch)
        bpat = bip_kernel_patterns(H, F, s == 2, lay.v_branch)[0]
        tr, src = pmc_lookup([bpat], f"*{workload}_v*") if workload else (None, None)
    else:
        fb = fwd_bytes(n, m, e, H, F, s, lay.rowterms, lay.row_scores, attd=lay.v_branch)
        tr, src = (pmc_traffic(H, F, s == 2, workload, lay.fwd_variant, lay.rowterms)
                   if workload else (None, None))
    ach = fb / (k_ms * 1e-3) / 1e9
    res = {"workload": label, "value": world * e * steps / dt, "unit": "edges/s",
           "ms_per_step": dt / steps * 1e3, "ms_per_step_eager": dte / steps * 1e3,
           "dtype": "bf16" if s == 2 else "f32",
           "config": {"nodes": n, "cols": m, "edges": e, "in_features": fin, "heads": H,
                      "feat": F},
           "roofline": {"kernel": ("msha_bip_attention_fwd" if lay.bip else
                                   "msha_edge_attention_fwd" + ("_rs" if lay.row_scores else "")),
                        "variant": lay.fwd_variant,
                        "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBS, "traffic": tr,
                        "traffic_unit": "bytes per launch (rocprofv3 PMC)",
                        "traffic_source": src, "algorithmic_bytes_per_launch": fb,
                        "avg_launch_us": k_ms * 1e3, "launches_timed": nl},
           "edge_kernels": edge_kernels(lay, n, m, e, H, F, s, workload)}
    g = lay.graph
    del lay
    return res, g


def pair_bytes(F, s, mode, hidden):
    """Algorithmic bytes per scored pair: two int64 indices, the two
    gathered rows, the score(s) written (fp32 inner; mlp: hidden scores in the table's
    dtype)."""
    out = 4 if mode == "inner" else s * hidden
    return 16 + 2 * s * F + out


IC_GATHER_PEAK_GBS = 8600.0  # random 1,152-B rows from a 38 MB table (MI355X_MICROARCH.md)


def pair_compulsory_bytes(n, F, s, mode, hidden, P):
    """Compulsory HBM bytes of one pair-scoring launch: every table row read once (the
    table, n x F), the two int64 indices per pair, the scores written (fp32 inner; mlp:
    hidden scores in the table's dtype) and, for mlp, W and the bias."""
    out = 4 if mode == "inner" else s * hidden
    w = (hidden * F * s + 4 * hidden) if mode == "mlp" else 0
    return n * F * s + P * (16 + out) + w


def link_score_bench(dev, rowptr, col, n, F, world, rank, group_ok, steps=16, warmup=3,
                     hidden=128, n_pairs=4_000_000, dtype=torch.float32, amortise=8):
    """score P = 4M pairs (2M graph edges + 2M uniform negatives,
    seed 1) against h (n x F) with LinkPredictor 'mlp' (hidden 128) and 'inner'.
    Rank r owns rows [r R, (r+1) R) of h (sharding.ShardedTable); one RCCL
    all_gather_into_tensor per batch rebuilds the full table (inside the timed loop;
    a world-1 group on one GPU, so the collective path is the one measured), then each
    rank scores its contiguous P/W slice.  pairs/s over all ranks:
      pairs_per_sec_*             gather, then score, per batch;
      pairs_per_sec_*_overlapped  sharding.PipelinedScorer: batch k+1's all-gather on
                                  the communicator's stream while batch k is scored;
      pairs_per_sec_*_amortised   one gather per ``amortise`` batches (the table reused,
                                  as when one embedding pass is scored against many
                                  negative samples).
    ``roofline``: the pair kernel alone (HIP events on its stream): fp32 'mlp' at the
    tightest of its ceilings (bf16 pipe on the split products, IC gather, compulsory HBM)
    with its fp32-equivalent rate beside it, the rest against the IC gather rate on the
    PMC bytes (or compulsory HBM without a profile of this build)."""
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd import sharding

    g = torch.Generator().manual_seed(1)
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    pick = np.random.default_rng(1).choice(len(col), n_pairs // 2, replace=False)
    src = np.concatenate([rows[pick], torch.randint(0, n, (n_pairs // 2,), generator=g).numpy()])
    dst = np.concatenate([col[pick], torch.randint(0, n, (n_pairs // 2,), generator=g).numpy()])
    t_src = torch.as_tensor(src, device=dev)
    t_dst = torch.as_tensor(dst, device=dev)
    table = sharding.ShardedTable(n, F, world, rank, dev, dtype=dtype, buffers=2)
    lo, hi = sharding.row_range(n, world, rank)
    table.set_local(torch.rand(hi - lo, F, generator=torch.Generator().manual_seed(10 + rank))
                    .to(dev, dtype))
    W = (torch.randn(hidden, F, generator=g) * F ** -0.5).to(dev, dtype)
    b = torch.randn(hidden, generator=g).to(dev)
    plo, phi = sharding.pair_range(n_pairs, world, rank)
    # a bf16 LinkPredictor returns bf16 scores (torch semantics); fp32 table: fp32
    outs = {m_: [torch.empty(phi - plo, hidden, device=dev, dtype=dtype),
                 torch.empty(phi - plo, hidden, device=dev, dtype=dtype)] if m_ == "mlp" else
            [torch.empty(phi - plo, device=dev), torch.empty(phi - plo, device=dev)]
            for m_ in ("mlp", "inner")}
    if group_ok:
        import torch.distributed as tdist
    calls = [0]

    def fn(mode):
        def score(h, s_, d_):  # alternate output buffers (the pipelined scorer keeps two)
            o = outs[mode][calls[0] % 2]
            calls[0] += 1
            # the pair batch is index-checked once below (the same arrays every batch)
            if mode == "mlp":
                return MF.score_pairs(h, s_, d_, "mlp", W, b, out=o, check=False)
            return MF.score_pairs(h, s_, d_, "inner", out=o, check=False)
        return score

    def sync_all():
        if group_ok:
            tdist.barrier()
        torch.cuda.synchronize(dev)

    MF.check_pair_indices(t_src, t_dst, n)  # torch's h[idx] rule, once per pair batch
    res = {}
    s = 2 if dtype == torch.bfloat16 else 4
    for mode in ("mlp", "inner"):
        f = fn(mode)
        for variant in ("", "_overlapped", "_amortised"):
            if variant == "_overlapped":
                pipe = sharding.PipelinedScorer(table, f)
                batches = [(t_src, t_dst)] * (steps)

                def run(k_steps):
                    pipe.run(batches[:k_steps])
            else:
                every = amortise if variant == "_amortised" else 1

                def run(k_steps, every=every):
                    for k in range(k_steps):
                        if k % every == 0:
                            sharding.score_sharded(table, t_src, t_dst, f)
                        else:  # the gathered table of the last all-gather is reused
                            f(table.full[:n], t_src[plo:phi], t_dst[plo:phi])
            run(warmup)
            sync_all()
            t0 = time.perf_counter()
            run(steps)
            sync_all()
            dt = time.perf_counter() - t0
            if group_ok and world > 1:
                tt = torch.tensor([dt], device=dev)
                tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
                dt = float(tt.item())
            res[f"pairs_per_sec_{mode}{variant}"] = n_pairs * steps / dt
            res[f"ms_per_batch_{mode}{variant}"] = dt / steps * 1e3
        # the pair kernel alone: HIP events on the stream it is launched on
        full = table.full[:n]
        evs = []
        st = torch.cuda.current_stream(dev)
        for k in range(warmup + steps):
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            f(full, t_src[plo:phi], t_dst[plo:phi])
            z.record(st)
            if k >= warmup:
                evs.append((a, z))
        torch.cuda.synchronize(dev)
        us = float(np.mean([a.elapsed_time(z) for a, z in evs])) * 1e3
        P = phi - plo
        gathered = P * pair_bytes(F, s, mode, hidden)
        comp = pair_compulsory_bytes(n, F, s, mode, hidden, P)
        flops = P * (2 * F * hidden + F) if mode == "mlp" else P * 2 * F
        kname = (("pair_bf16_kernel" if s == 2 else "pair_x3_kernel") if mode == "mlp"
                 else "pair_inner")
        tr, src_ = pmc_lookup([_pair_pattern(mode, s == 2)], "*link*")
        t_s = us * 1e-6
        # memory side: the compulsory HBM bytes (every table row once, the indices, the
        # scores) against the 8 TB/s HBM peak, and -- the table (25-51 MB) being gathered
        # ~80x per batch from the Infinity Cache -- the measured PMC bytes against the
        # guide's random-row Infinity-Cache rate (MI355X_MICROARCH.md "Indexed rows")
        mem = {"compulsory_bytes_per_launch": comp,
               "compulsory_GBs": comp / t_s / 1e9,
               "frac_compulsory_hbm": comp / t_s / 1e9 / HBM_PEAK_GBS,
               "gathered_bytes_per_launch": gathered,
               "gathered_note": "per-pair model: both rows counted for every pair (each row is "
                                f"gathered ~{2 * n_pairs // max(n, 1)}x per batch); not a "
                                "roofline numerator",
               "traffic": tr, "traffic_source": src_,
               "traffic_note": "rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE per launch: L2->fabric "
                               "bytes incl. Infinity-Cache hits"}
        if tr is not None:
            mem.update(traffic_GBs=tr / t_s / 1e9, ic_peak_GBs=IC_GATHER_PEAK_GBS,
                       frac_traffic_ic=tr / t_s / 1e9 / IC_GATHER_PEAK_GBS)
        if mode == "mlp" and s == 4:
            # fp32 'mlp' runs as split-bf16 products (skinny.hip pair_x3_kernel: three bf16
            # terms per operand, six bf16 MFMA products per fp32 product): its ceilings are
            # the bf16 pipe on those products, the Infinity-Cache gather rate on the PMC
            # bytes and the compulsory HBM bytes; the tightest one is the roofline, and the
            # algorithmic fp32 rate against the exact-fp32 spec rides along
            ach = flops / t_s / 1e12
            cands = [{"kernel": kname, "bound": "mfma", "achieved": 6 * ach,
                      "peak": BF16_MFMA_TFLOPS, "unit": "TFLOP/s",
                      "frac": 6 * ach / BF16_MFMA_TFLOPS,
                      "ceiling": "bf16 MFMA pipe on the six split products per fp32 product"},
                     {"kernel": kname, "bound": "hbm", "achieved": comp / t_s / 1e9,
                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": comp / t_s / 1e9 / HBM_PEAK_GBS,
                      "ceiling": "compulsory HBM bytes at 8 TB/s"}]
            if tr is not None:
                cands.append({"kernel": kname, "bound": "ic", "achieved": tr / t_s / 1e9,
                              "peak": IC_GATHER_PEAK_GBS, "unit": "GB/s",
                              "frac": tr / t_s / 1e9 / IC_GATHER_PEAK_GBS,
                              "ceiling": "random-row Infinity-Cache gather rate (8.6 TB/s) "
                                         "on the PMC bytes"})
            roof = max(cands, key=lambda r: r["frac"])
            roof["fp32_equivalent"] = {
                "achieved": ach, "peak": F32_MFMA_TFLOPS, "unit": "TFLOP/s",
                "frac": ach / F32_MFMA_TFLOPS,
                "note": "algorithmic fp32 FLOPs / time against the exact-fp32 MFMA spec; the "
                        "kernel computes each fp32 product as six bf16 products (fp32-level "
                        "error, tests/test_gpu_kernels.py at 1e-5 of fp64)"}
            roof["other_ceilings"] = [{k: c[k] for k in ("bound", "frac")} for c in cands
                                      if c is not roof]
        elif tr is not None:
            roof = {"kernel": kname, "bound": "ic", "achieved": tr / t_s / 1e9,
                    "peak": IC_GATHER_PEAK_GBS, "unit": "GB/s",
                    "frac": tr / t_s / 1e9 / IC_GATHER_PEAK_GBS,
                    "ceiling": "random-row Infinity-Cache gather rate (8.6 TB/s, "
                               "MI355X_MICROARCH.md) on the PMC bytes"}
        else:
            roof = {"kernel": kname, "bound": "hbm", "achieved": comp / t_s / 1e9,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": comp / t_s / 1e9 / HBM_PEAK_GBS,
                    "ceiling": "compulsory HBM bytes at 8 TB/s (no PMC profile of this build)"}
        roof.update(avg_launch_us=us, pairs_per_launch=P, flops_per_launch=flops,
                    kernel_pairs_per_sec=P / t_s, memory=mem)
        res[f"roofline_{mode}"] = roof
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
               sharding=(f"h rows all-gathered over RCCL (all_gather_into_tensor, world "
                         f"{world}), pairs split contiguously per rank"
                         if table.path() == "rccl" else f"{table.path()} (no RCCL group)"))
    return res


def _pair_pattern(mode, bf16):
    """rocprofv3 names of the pair kernels (skinny.hip pair_kernel, scorer.hip inner)."""
    if mode == "mlp":  # skinny.hip pair_bf16_kernel (left mangled) / pair_x3_kernel<K, N, W>
        return r"pair_bf16_kernel" if bf16 else r"sk::pair_x3_kernel<"
    return r"pair_inner_kernelIDF16b" if bf16 else r"pair_inner_kernel<float>"


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
    # one (2, 64) tensor per batch: a step's feed is one device copy (source and
    # recipient rows of the static input together)
    batches = [torch.stack([src_t[b], dst_t[b]]) for b in picks]
    from msha_gnn_amd.graph import graph_for

    e = graph_for(adj).n_edges
    res = dict(model=model_kind, year=year, dtype=str(dtype).replace("torch.", ""), nodes=n,
               recipients=m, edges=e, optimizer=f"{ADAM} Adam",
               flows="shipped" if year == "2015" else "synthetic (2015 degree law)")
    for mode in ("eager", "hip_graph"):
        torch.manual_seed(0)
        model = cls(128, 64, m, 2, 0.5, gdp, n, m).to(dev, dtype)
        graphed = mode == "hip_graph"
        # train.py's Adam (lr 1e-3, wd 5e-4): msha_adam_step, one launch for every
        # parameter, with Sfeatures' update fused into its feature-dropout backward (its
        # 5M-float gradient is never written); MSHA_ADAM=torch: torch's fused multi-tensor
        # Adam (same update rule)
        if ADAM == "msha":
            from msha_gnn_amd.optim import Adam

            opt = Adam(model.parameters(), lr=1e-3, weight_decay=5e-4)
            opt.fuse_dropout_grad(model.Sfeatures)
        else:
            opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=5e-4,
                                   capturable=graphed, fused=FUSED_ADAM)
        model.train()
        sr_s = torch.empty(2, 64, dtype=torch.int64, device=dev)
        si_s, ri_s = sr_s[0], sr_s[1]
        unit = torch.ones((), device=dev)  # dL/dL, made once (not a fill node per step)

        def body():
            opt.zero_grad(set_to_none=True)
            out = model(adj, cadj, padj, si_s)
            # train.py:229 F.nll_loss(output[source_index], recipient_index) as one launch
            # each way (msha_nll_rows_fwd/_bwd) instead of ~12 ATen launches
            loss = MF.nll_loss_rows(out, si_s, ri_s)
            loss.backward(unit)
            opt.step()
            return loss

        def feed(k):
            sr_s.copy_(batches[k % len(batches)])

        if graphed:
            from msha_gnn_amd.step import GraphedStep

            feed(0)
            gs = GraphedStep(body, dev, warmup=warmup)

            def one(k):
                # the batch copy and the dropout replay counter's increment: one launch
                return gs.replay(feed=(sr_s, batches[k % len(batches)]))

            # untimed replays: a graph's first launches carry one-time setup (an occasional
            # ~25 ms first-replay stall put one year's step at 1.9 ms instead of 0.5)
            for k in range(warmup):
                one(k)
        else:
            def one(k):
                feed(k)
                return body()

            for k in range(warmup):
                one(k)
        # three timed windows of `steps` steps each; the step time is the median window
        # (a single host-side hiccup of ~10 ms inside one 20-step window otherwise doubled
        # a year's figure; every window is reported)
        windows = []
        for w in range(3):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for k in range(steps):
                loss = one(w * steps + k)
            torch.cuda.synchronize(dev)
            windows.append((time.perf_counter() - t0) / steps * 1e3)
        if graphed:
            gs.close()
        res[f"ms_per_step_{mode}_windows"] = [round(x, 4) for x in windows]
        res[f"ms_per_step_{mode}"] = sorted(windows)[1]
        res[f"loss_{mode}"] = float(loss.detach())
    res["ms_per_step"] = min(res["ms_per_step_eager"], res["ms_per_step_hip_graph"])
    res["edges_per_sec"] = e / (res["ms_per_step"] * 1e-3)
    return res


def write_train_py_year(d):
    """The shipped 2015 graph (tests/golden) as train.py's anonymous_data files under d."""
    from msha_gnn_amd import trainpy

    z = np.load(os.path.join(ROOT, "tests", "golden", "r15_graph.npz"))
    yz = np.load(os.path.join(ROOT, "tests", "golden", "years.npz"))
    rows = np.repeat(np.arange(int(z["n"])), np.diff(z["rowptr"]))
    flows = np.stack([np.repeat(rows, z["cnt"].astype(np.int64)),
                      np.repeat(z["col"].astype(np.int64), z["cnt"].astype(np.int64))], 1)
    trainpy.write_year(d, "2015", yz["2015.city"], yz["2015.prov"], yz["2015.gdp"], flows,
                       int(z["m"]))
    return dict(nodes=int(z["n"]), recipients=int(z["m"]), edges=int(len(z["col"])),
                flows=int(len(flows)))


def train_py_literal_leg(dev, model_kind="ablation3", steps=20, warmup=5):
    """train.py as written (train.py:180-232, msha_gnn_amd.trainpy): the zero-argument
    HigherDataset over the shipped 2015 data in anonymous_data format, its DataLoader
    (batch 64, shuffle), torch.optim.Adam(lr 1e-3, weight_decay 5e-4) as train.py:207
    builds it, and per step the loop body statement for statement -- next batch from the
    loader, .to(device), zero_grad, the model, F.nll_loss(output[source_index], ...),
    loss.item(), backward, step -- eagerly, no HIP graph.  ms per step = median of three
    windows of ``steps`` iterations (the loader's own time included; reported apart)."""
    import tempfile

    import msha_loader

    msha_loader.load()
    from msha_gnn_amd import trainpy

    res = dict(model=model_kind, year="2015", dtype="float32", optimizer="torch.optim.Adam",
               loss="F.nll_loss(output[source_index], recipient_index)", hip_graph=False)
    with tempfile.TemporaryDirectory(prefix="msha_trainpy_") as d:
        sizes = write_train_py_year(d)
        with trainpy.namespace(d, dev) as ns:
            tp = trainpy.TrainPy(ns, dev, dropout=0.5, model_kind=model_kind)
            state = {"it": iter(tp.train_loader)}

            def next_batch():
                try:
                    return next(state["it"])
                except StopIteration:  # a new epoch of the loader, as train.py's next call
                    state["it"] = iter(tp.train_loader)
                    return next(state["it"])

            for _ in range(warmup):
                tp.iteration(next_batch())
            windows, loader = [], []
            for _ in range(3):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(steps):
                    loss = tp.iteration(next_batch())
                torch.cuda.synchronize(dev)
                windows.append((time.perf_counter() - t0) / steps * 1e3)
            t0 = time.perf_counter()
            for _ in range(steps):
                next_batch()
            loader = (time.perf_counter() - t0) / steps * 1e3
            res.update(sizes)
    res["ms_per_step_windows"] = [round(x, 4) for x in windows]
    res["ms_per_step"] = sorted(windows)[1]
    res["loader_ms_per_batch"] = loader
    res["loss"] = float(loss)
    res["edges_per_sec"] = res["edges"] / (res["ms_per_step"] * 1e-3)
    return res


def cpu_share():
    """CPUs this process may use: its affinity, capped by the cgroup's CPU quota (the GPU
    box grants each GPU a share of a large host; os.cpu_count() reports the host)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            avail = min(avail, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return avail


class _Threads:
    """torch CPU threads = the process's CPU share for the duration of a CPU leg."""

    def __enter__(self):
        self.prev = torch.get_num_threads()
        torch.set_num_threads(cpu_share())
        return self

    def __exit__(self, *a):
        torch.set_num_threads(self.prev)


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
                       f"{el_t:.1f}s: numpy X@W + oracle/edge_attention_cpu.c (OpenMP, "
                       f"{cpu_oracle.threads()} threads = OMP_NUM_THREADS)")


def cpu_baseline_bip1m(rowptr, col, n, m, fin=128, H=2, F=64, budget_s=10.0):
    """bip1m CPU baseline: the same OursLayer3-core step as the bip1m leg (h1 = R W,
    h2 = S W, scores, u = att @ h1 AND v = att.T @ h2, the backward incl. the hs . dV
    term, d_hs, and dW) on this host's cores: numpy BLAS for the projections and
    oracle/edge_attention_cpu.c (OpenMP) for the edge softmax / aggregates, whole graph,
    repeated for ~budget_s."""
    from oracle import cpu_oracle
    from oracle import gnn_oracle as O

    rng = np.random.default_rng(0)
    X = rng.random((n, fin), dtype=np.float32)
    Xr = rng.random((m, fin), dtype=np.float32)
    W = (rng.standard_normal((fin, H * F)) * fin ** -0.5).astype(np.float32)
    al = rng.standard_normal((H, F)).astype(np.float32)
    ar = rng.standard_normal((H, F)).astype(np.float32)
    dU = rng.standard_normal((n, H, F)).astype(np.float32)
    dV = rng.standard_normal((m, H, F)).astype(np.float32)
    colptr, perm = O.csr_to_csc(rowptr, col, m)
    csc_row = O.edge_rows(rowptr)[perm]

    def one():
        h2 = (X @ W).reshape(n, H, F)
        h1 = (Xr @ W).reshape(m, H, F)
        el = np.einsum("nhf,hf->nh", h2, al)
        er = np.einsum("mhf,hf->mh", h1, ar)
        u, lse, v = cpu_oracle.edge_attention_fwd(rowptr, col, el, er, h1, hs=h2, colptr=colptr,
                                                  csc_row=csc_row, csc_eid=perm)
        d_el, d_er, d_hc, d_hs = cpu_oracle.edge_attention_bwd(
            rowptr, col, colptr, csc_row, perm, el, er, h1, lse, u, dU, hs=h2, dV=dV)
        dh2 = (d_hs + d_el[:, :, None] * al[None]).reshape(n, H * F)
        dh1 = (d_hc + d_er[:, :, None] * ar[None]).reshape(m, H * F)
        _ = X.T @ dh2 + Xr.T @ dh1  # dW

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
                sample=f"whole bip1m graph ({n} x {m}, {len(col)} edges), {reps} OursLayer3-core "
                       f"fwd+bwd steps (u and v, d_hs, dW) in {el_t:.1f}s: numpy projections + "
                       f"oracle/edge_attention_cpu.c (OpenMP, {cpu_oracle.threads()} threads)")


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
            "cpu_share": cpu_share(), "torch_threads_cpu_legs": cpu_share(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


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
    with _Threads():
        D.train_step(p, opt, adj, src, dst, dropout)  # warm-up
        D.train_step(p, opt, adj, src, dst, dropout)
        times = []
        t_end = time.perf_counter() + budget_s
        while len(times) < 2 or (time.perf_counter() < t_end and len(times) < 20):
            t0 = time.perf_counter()
            D.train_step(p, opt, adj, src, dst, dropout)
            times.append(time.perf_counter() - t0)
        cores = torch.get_num_threads()
    med = float(np.median(times))
    return dict(value=med, unit="s/step", higher_is_better=False, cores=cores,
                kind="port", edges_per_sec=len(z["col"]) / med,
                sample=f"ablation3 train step on the full 2015 graph ({n} x {m}), median of "
                       f"{len(times)} steps after 2 warm-up: oracle/dense_step.py (the "
                       "reference's dense torch formulation, CPU)")


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
    with torch.no_grad(), _Threads():
        for mode in ("mlp", "inner"):
            D.score_pairs(h, src, dst, mode, W, b)
            reps, t0 = 0, time.perf_counter()
            while reps < 1 or (time.perf_counter() - t0 < budget_s / 2 and reps < 20):
                D.score_pairs(h, src, dst, mode, W, b)
                reps += 1
            res[f"pairs_per_sec_{mode}"] = n_pairs * reps / (time.perf_counter() - t0)
        cores = torch.get_num_threads()
    res.update(unit="pairs/s", cores=cores, kind="port",
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


def rank_census(dist_on, dev):
    """Who took part, recorded in the JSON line so a multi-GPU run proves its own shape:
    the process group's world size and backend (nccl = RCCL on ROCm), and per rank its
    RANK / LOCAL_RANK, device and the device's PCI bus id (all_gather_object over the
    group; one entry without a group)."""
    import socket

    local = int(os.environ.get("LOCAL_RANK", "0"))
    me = {"rank": int(os.environ.get("RANK", "0")), "local_rank": local,
          "host": socket.gethostname(), "device": str(dev)}
    if dev is not None and torch.device(dev).type == "cuda":
        props = torch.cuda.get_device_properties(dev)
        me["device_name"] = props.name
        try:
            me["pci_bus_id"] = (f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:"
                                f"{props.pci_device_id:02x}")
        except AttributeError:
            pass
    if not dist_on:
        return {"world_size": 1, "backend": None, "ranks": [me]}
    import torch.distributed as tdist

    ranks = [None] * tdist.get_world_size()
    tdist.all_gather_object(ranks, me)
    backend = str(tdist.get_backend())
    return {"world_size": tdist.get_world_size(),
            "backend": backend + (" (RCCL)" if backend == "nccl" else ""),
            "ranks": ranks}


def dry_run(world, rank):
    """CPU rehearsal of the multi-rank path (gloo): rank launch, the sharded table's
    all-gather (serial and double-buffered), the contiguous pair split and the
    max-over-ranks timing.  Prints one JSON line on rank 0 (n_gpus = ranks that took
    part)."""
    import torch.distributed as tdist

    from msha_loader import load

    load()
    from msha_gnn_amd import sharding

    if world > 1:
        tdist.init_process_group("gloo")
    n, F, P = 1001, 8, 5003
    tab = sharding.ShardedTable(n, F, world, rank, "cpu", buffers=2)
    lo, hi = sharding.row_range(n, world, rank)
    full_ref = torch.arange(n * F, dtype=torch.float32).view(n, F)
    tab.set_local(full_ref[lo:hi])
    t0 = time.perf_counter()
    ok = bool(torch.equal(tab.gather(), full_ref))
    src = torch.arange(P) % n
    outs = sharding.PipelinedScorer(tab, lambda h, s_, d_: h[s_].sum(1)).run([(src, src)] * 3)
    plo, phi = sharding.pair_range(P, world, rank)
    ok = ok and all(torch.equal(o[2], full_ref[src[plo:phi]].sum(1)) for o in outs)
    dt = time.perf_counter() - t0
    cnt = torch.tensor([phi - plo, int(ok), 1], dtype=torch.float64)
    tt = torch.tensor([dt])
    if world > 1:
        tdist.all_reduce(cnt)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
    census = rank_census(world > 1, torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_reporting": int(cnt[2]),
                          "pairs_covered": int(cnt[0]), "pairs": P,
                          "table_ok_ranks": int(cnt[1]), "max_rank_s": float(tt),
                          "exchange": tab.path(), **census}), flush=True)
    if world > 1:
        tdist.destroy_process_group()


def _world1_group(dev):
    """An in-process world-1 RCCL group (FileStore rendezvous) so the link scorer's
    all-gather runs the collective on a single GPU too.  Returns a cleanup callable, or
    None when RCCL is unavailable."""
    import tempfile

    import torch.distributed as tdist

    fd, path = tempfile.mkstemp(prefix="msha_bench_rccl_")
    os.close(fd)
    os.unlink(path)
    try:
        tdist.init_process_group("nccl", store=tdist.FileStore(path, 1), rank=0, world_size=1,
                                 device_id=dev)
    except Exception as ex:  # noqa: BLE001 - report, fall back to the copy path
        print(f"world-1 RCCL group failed: {ex}", file=sys.stderr)
        return None

    def done():
        tdist.destroy_process_group()
        if os.path.exists(path):
            os.unlink(path)
    return done


LINE_MAX_BYTES = 12 * 1024  # the stdout line; the driver keeps only a tail of stdout


def _finite(o):
    """A copy of ``o`` with every non-finite float replaced by None (strict JSON)."""
    if isinstance(o, float):
        return o if np.isfinite(o) else None
    if isinstance(o, dict):
        return {k: _finite(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_finite(v) for v in o]
    if isinstance(o, (np.floating, np.integer)):
        return _finite(o.item())
    return o


def _sig(x, digits=4):
    """Float rounded to ``digits`` significant digits (None for missing / non-finite)."""
    if x is None:
        return None
    x = float(x)
    if not np.isfinite(x):
        return None
    if x == 0.0:
        return 0.0
    return float(f"{x:.{digits}g}")


def dumps_line(obj) -> str:
    """Strict single-line JSON (no NaN/Infinity tokens)."""
    return json.dumps(_finite(obj), separators=(",", ":"), allow_nan=False)


_KSHORT = {"msha_edge_attention_fwd": "fwd", "msha_edge_attention_bwd_fused": "bwd",
           "msha_edge_attention_bwd_rows": "bwd_rows", "msha_csc_aggregate": "csc",
           "msha_bip_attention_fwd": "bip_fwd", "msha_bip_attention_bwd": "bip_bwd"}


def compact_line(out: dict, detail_path: str) -> dict:
    """The stdout line: the contract keys, the headline roofline and CPU baseline, and a
    compact ``legs`` map (per leg value / ms_per_step / frac / traffic) plus each leg's
    edge-kernel HBM fractions; everything else stays in ``detail_path``."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")
    line = {k: out[k] for k in keep if k in out}
    line["value"], line["ms_per_step"] = _sig(out["value"], 6), _sig(out["ms_per_step"], 5)
    rk = out.get("ranks") or {}
    line["ranks"] = {"world_size": rk.get("world_size"), "backend": rk.get("backend"),
                     "ranks": [{k: r.get(k) for k in ("rank", "local_rank", "device",
                                                      "pci_bus_id") if k in r}
                               for r in rk.get("ranks", [])]}
    ro = out.get("roofline") or {}
    line["roofline"] = {k: (_sig(ro.get(k)) if isinstance(ro.get(k), float) else ro.get(k))
                        for k in ("kernel", "bound", "achieved", "peak", "unit", "frac",
                                  "traffic", "algorithmic_bytes_per_launch", "avg_launch_us")}
    legs, kfrac = {}, {}

    def leg(name, d, unit=None):
        if not d:
            return
        r = d.get("roofline") or {}
        legs[name] = {"value": _sig(d.get("value")), "ms_per_step": _sig(d.get("ms_per_step")),
                      "frac": _sig(r.get("frac"), 3), "traffic": _sig(r.get("traffic"))}
        if unit:
            legs[name]["unit"] = unit
        ks = {_KSHORT.get(k["kernel"], k["kernel"]): _sig(k.get("frac"), 3)
              for k in d.get("edge_kernels", [])}
        if ks:
            kfrac[name] = ks

    leg("c4_f32", out)
    leg("c4_f32_dropout", out.get("dropout_p05"))
    leg("c4_bf16", out.get("bf16"))
    for big in ("syn2m", "bip1m"):
        for tag, d in (out.get(big) or {}).items():
            leg(f"{big}_{tag}", d)
    ls = out.get("link_score")
    for tag, d in (("f32", ls), ("bf16", (ls or {}).get("bf16"))):
        if not d:
            continue
        for mode in ("mlp", "inner"):
            r = d.get(f"roofline_{mode}") or {}
            legs[f"link_{mode}_{tag}"] = {
                "value": _sig(d.get(f"pairs_per_sec_{mode}")),
                "ms_per_step": _sig(d.get(f"ms_per_batch_{mode}")),
                "frac": _sig(r.get("frac"), 3),
                "traffic": _sig((r.get("memory") or {}).get("traffic")), "unit": "pairs/s"}
            for v in ("overlapped", "amortised"):
                legs[f"link_{mode}_{tag}_{v}"] = {
                    "value": _sig(d.get(f"pairs_per_sec_{mode}_{v}")),
                    "ms_per_step": _sig(d.get(f"ms_per_batch_{mode}_{v}")), "unit": "pairs/s"}
        legs[f"link_allgather_{tag}"] = {"ms_per_step": _sig(d.get("allgather_ms")),
                                         "world": d.get("world")}
    for key, tag in (("train_step_configs1", "graphed"), ("train_step_configs2", "graphed")):
        for r in (out.get(key) or {}).get("runs", []):
            dt = "bf16" if "bfloat16" in str(r.get("dtype")) else "f32"
            legs[f"step_{r['model']}_{r['year']}_{dt}"] = {
                "value": _sig(r.get("edges_per_sec")), "ms_per_step": _sig(r.get("ms_per_step")),
                "ms_eager": _sig(r.get("ms_per_step_eager"))}
    for r in (out.get("train_py_literal") or {}).get("runs", []):
        legs[f"trainpy_{r['model']}"] = {"value": _sig(r.get("edges_per_sec")),
                                         "ms_per_step": _sig(r.get("ms_per_step"))}
    line["legs"] = legs
    line["kernel_frac"] = kfrac
    cb = out.get("cpu_baseline")
    if cb:
        c = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "sample")}
        c["value"] = _sig(c["value"])
        c["host"] = (cb.get("host") or {}).get("model")
        other = {}
        if cb.get("configs1_ablation3"):
            other["configs1_ablation3"] = {"value": _sig(cb["configs1_ablation3"]["value"]),
                                           "unit": "s/step"}
        if cb.get("link_score"):
            other["link_mlp"] = {"value": _sig(cb["link_score"]["pairs_per_sec_mlp"]),
                                 "unit": "pairs/s"}
            other["link_inner"] = {"value": _sig(cb["link_score"]["pairs_per_sec_inner"]),
                                   "unit": "pairs/s"}
        if cb.get("bip1m"):
            other["bip1m"] = {"value": _sig(cb["bip1m"]["value"]), "unit": "edges/s"}
        if other:
            c["other"] = other
        line["cpu_baseline"] = c
    line["detail"] = detail_path
    return line


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
    ap.add_argument("--no-syn2m", action="store_true")
    ap.add_argument("--no-bip1m", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="report the eager launches (no HIP-graph replay of the timed steps)")
    ap.add_argument("--no-dropout-leg", action="store_true")
    ap.add_argument("--detail", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="where the full per-leg detail goes (stdout carries the compact line)")
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
    # stdout carries exactly the one JSON line: what libraries write to fd 1 (RCCL's
    # version banner at communicator setup) goes to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if dist:
        import torch.distributed as tdist

        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    clock = Clock(dev, dist)
    census = rank_census(dist, dev)
    if census["world_size"] != world:
        print(f"bench.py: the process group has {census['world_size']} ranks, WORLD_SIZE={world}",
              file=sys.stderr)
        sys.exit(2)

    wl = args.workload
    if wl == "r15":
        rowptr, col, n, m = r15_graph()
        fin, H, F = 128, 2, 64
    elif wl == "bip1m":
        rowptr, col, n, m = bip_graph()
        fin, H, F = 128, 2, 64
    else:
        w = WORKLOADS[wl]
        n, fin, H, F = w["n"], w["fin"], w["heads"], w["feat"]
        m = n
        rowptr, col = synth_graph(n, w["e"], seed=0)
    e = len(col)
    K, Wu = args.steps, args.warmup
    # (bip1m: the OursLayer3 core with its u and v aggregates, as the default run's leg)
    head, graph = layer_leg(clock, dev, f"gat_layer_{wl}", rowptr, col, n, m, fin, H, F, K, Wu,
                            world, args.eager, workload=wl, v_branch=wl == "bip1m")
    drop_leg = None
    if not args.no_dropout_leg:
        # the reference's training forward drops attention at p = 0.5 (Ablation.py:271):
        # the same step with the Philox mask drawn in the forward and regenerated in the
        # backward (no mask tensor)
        drop_leg, _ = layer_leg(clock, dev, f"gat_layer_{wl}, attention dropout p = 0.5 "
                                "(training forward + backward)", rowptr, col, n, m, fin, H, F,
                                K, Wu, world, args.eager, graph=graph, dropout=0.5)
    bf16_leg = None
    if not args.no_bf16:
        # config C3: the same layer with bf16 tables / projection (bf16 MFMA)
        bf16_leg, _ = layer_leg(clock, dev, f"gat_layer_{wl} (config C3: bf16 tables, bf16 "
                                "MFMA projection, fp32 scores/softmax)", rowptr, col, n, m, fin,
                                H, F, K, Wu, world, args.eager, dtype=torch.bfloat16,
                                graph=graph, workload=wl, v_branch=wl == "bip1m")
    link = None
    if not args.no_link_score and wl not in ("r15", "bip1m"):
        done = None if dist else _world1_group(dev)
        group_ok = dist or done is not None
        link = link_score_bench(dev, rowptr, col, n, H * F, world, rank, group_ok)
        if not args.no_bf16:  # C5 names a bf16 table
            link["bf16"] = link_score_bench(dev, rowptr, col, n, H * F, world, rank, group_ok,
                                            dtype=torch.bfloat16)
        if done is not None:
            done()
    del graph
    torch.cuda.empty_cache()
    syn2m = bip1m = cpu_bip1m = None
    if wl == "syn100k" and not args.no_syn2m:
        # the cache-busting variant: a 1 GB fp32 table outside the 256 MB Infinity Cache
        w2 = WORKLOADS["syn2m"]
        rp2, c2 = synth_graph(w2["n"], w2["e"], seed=0)
        syn2m = {}
        g2 = None
        for dt_, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            if dt_ == torch.bfloat16 and args.no_bf16:
                continue
            syn2m[tag], g2 = layer_leg(clock, dev, "gat_layer_syn2m", rp2, c2, w2["n"], w2["n"],
                                       w2["fin"], w2["heads"], w2["feat"], K, Wu, world,
                                       args.eager, dtype=dt_, graph=g2, workload="syn2m")
        del g2, rp2, c2
        torch.cuda.empty_cache()
    if wl == "syn100k" and not args.no_bip1m:
        # the repo's adjacency shape at scale: 1M sources x 32 recipients, OursLayer3 core
        rpb, cb, nb, mb = bip_graph()
        bip1m = {}
        gb = None
        for dt_, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            if dt_ == torch.bfloat16 and args.no_bf16:
                continue
            bip1m[tag], gb = layer_leg(clock, dev, "ourslayer3_bip1m (u and v aggregates)", rpb,
                                       cb, nb, mb, 128, 2, 64, K, Wu, world, args.eager,
                                       dtype=dt_, graph=gb, v_branch=True, workload="bip1m")
        del gb
        torch.cuda.empty_cache()
        if world == 1 and rank == 0 and not args.no_cpu_baseline:
            cpu_bip1m = cpu_baseline_bip1m(rpb, cb, nb, mb, budget_s=args.cpu_budget)
    if rank != 0:
        if dist:
            tdist.destroy_process_group()
        return
    ms_per_step = head["ms_per_step"]
    out = {
        "metric": METRIC, "value": head["value"], "unit": "edges/s", "n_gpus": world,
        "steps": K, "warmup": Wu, "ms_per_step": ms_per_step,
        "ms_per_step_eager": head["ms_per_step_eager"],
        "timing": ("value: one replay of a HIP graph holding exactly `steps` steps (captured "
                   "after the eager pass); roofline: HIP events around every launch over the "
                   "eager timed region of the same steps" if not args.eager else
                   "value and roofline: eager launches, HIP events around every launch"),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": f"gat_layer_{wl}", "nodes": n, "cols": m, "edges": e,
                   "in_features": fin, "heads": H, "feat": F, "parallelism": f"replicas{world}"},
        "ranks": census,
        "roofline": head["roofline"],
        "edge_kernels": head["edge_kernels"],
    }
    if drop_leg is not None:
        out["dropout_p05"] = drop_leg
    if bf16_leg is not None:
        out["bf16"] = bf16_leg
    if syn2m:
        out["syn2m"] = syn2m
    if bip1m:
        out["bip1m"] = bip1m
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
        out["train_py_literal"] = {
            "workload": "train.py:221-232 as written through the drop-in modules (DataLoader, "
                        "torch.optim.Adam, F.nll_loss(output[source_index], ...), loss.item() "
                        "per step, eager, no HIP graph), shipped 2015 graph, fp32",
            "runs": [train_py_literal_leg(dev, k) for k in ("ablation3", "Ours")]}
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
        if cpu_bip1m is not None:
            cb["bip1m"] = cpu_bip1m
        out["cpu_baseline"] = cb
    detail = args.detail
    try:
        os.makedirs(os.path.dirname(os.path.abspath(detail)), exist_ok=True)
        with open(detail, "w") as fh:
            json.dump(_finite(out), fh, indent=1)
    except OSError as ex:
        print(f"bench.py: could not write {detail}: {ex}", file=sys.stderr)
    sys.stdout.flush()
    os.write(json_fd, (dumps_line(compact_line(out, detail)) + "\n").encode())
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
