"""Autograd functions over the HIP kernels (include/msha_gnn.h).

``edge_attention``       Ablation.py:266-274 (OursLayer3 inter attention: scores,
                         masked softmax, dropout, u = att @ h1 and, optionally,
                         v = att.T @ h2), forward AND backward on the GPU.
``gal``                  GAT.py:20-35 GraphAttentionLayer row scale (after x @ W).
``dropout_keep_mask``    the Philox mask the kernels draw (for tests / oracles).
"""
from __future__ import annotations

import ctypes
import functools
import os
import struct

import torch

from . import _lib
from .graph import Graph

NEG_SLOPE = 0.2

# Optional live kernel timing: when a dict is installed here, the forward edge
# kernel launch is bracketed by HIP events on its own stream (bench.py).
KERNEL_EVENTS = None


def _timed(name):
    if KERNEL_EVENTS is None:
        return None
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    KERNEL_EVENTS.setdefault(name, []).append(ev)
    ev[0].record()
    return ev


def _f32c(t):
    return t.to(torch.float32).contiguous() if t is not None else None


BF16 = torch.bfloat16


def _table_dtype(*ts):
    """Storage type of node tables: bf16 when any given table is bf16, else fp32."""
    return BF16 if any(t is not None and t.dtype == BF16 for t in ts) else torch.float32


def _code(dt) -> int:
    """MSHA_DTYPE_* of a torch dtype."""
    return 1 if dt == BF16 else 0


def _tc(t, dt):
    return t.to(dt).contiguous() if t is not None else None


def new_seed() -> int:
    """Per-call dropout seed drawn from torch's CPU generator (no device sync;
    reproducible under torch.manual_seed)."""
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


_RNG_COUNTERS: dict = {}  # device index -> installed counter tensor (kept alive)


def set_rng_counter(counter: torch.Tensor | None, device=None):
    """Install (or remove, None) a device int64 replay counter for every dropout draw
    the library launches on ``device`` (default: the counter's device, else the
    current one; msha_set_rng_counter keeps one slot per device): increment it inside
    a captured HIP graph (``counter.add_(1)``) and each replay draws fresh masks.
    Returns the counter previously installed for that device (None if none), so a
    caller can restore it."""
    if counter is not None:
        _lib.require_cuda(counter)
        if counter.dtype != torch.int64 or counter.numel() < 1:
            raise ValueError("rng counter: a CUDA int64 tensor")
        dev = counter.device.index if device is None else torch.device(device).index
    else:
        dev = torch.device(device).index if device is not None else None
    if dev is None:
        dev = torch.cuda.current_device()
    if counter is not None and counter.device.index != dev:
        raise ValueError(f"rng counter lives on cuda:{counter.device.index}, not cuda:{dev}")
    prev = _RNG_COUNTERS.pop(dev, None)
    if counter is not None:
        _RNG_COUNTERS[dev] = counter
    _lib.call("msha_set_rng_counter", dev, None if counter is None else counter.data_ptr())
    return prev


def rng_counter(device=None):
    """The replay counter installed for ``device`` (default: current), or None."""
    dev = torch.device(device).index if device is not None else None
    return _RNG_COUNTERS.get(torch.cuda.current_device() if dev is None else dev)


def feed_step(dst: torch.Tensor, src: torch.Tensor, counter: torch.Tensor | None = None):
    """``dst.copy_(src)`` plus ``counter += 1`` in one launch (msha_feed_step): the feed of a
    replayed step whose graph leaves its replay-counter increment to the feed
    (``step.GraphedStep.replay(feed=...)``).  Same-size contiguous tensors on one device."""
    _lib.require_cuda(dst)
    if (src.device != dst.device or src.dtype != dst.dtype or src.numel() != dst.numel()
            or not (src.is_contiguous() and dst.is_contiguous())):
        raise ValueError("feed_step: same-shape contiguous tensors of one dtype and device")
    if counter is not None and (counter.dtype != torch.int64 or counter.device != dst.device):
        raise ValueError("feed_step: the counter is an int64 tensor on the feed's device")
    _lib.call("msha_feed_step", dst.data_ptr(), src.data_ptr(), dst.numel() * dst.element_size(),
              None if counter is None else counter.data_ptr(), _lib.stream_handle(dst.device))


def _stream(t):
    return _lib.stream_handle(t.device)


# Host-side caches for the per-call work around each launch (the eager train.py step is
# host-bound: ~40 launches behind ~1 ms of Python per step).
_WS: dict = {}  # (device index, stream) -> uint8 scratch tensor


def _workspace(dev, nbytes: int):
    """A scratch buffer of at least ``nbytes`` for one call's launches, shared by every
    call on the same device and stream (the library's workspaces are transient within a
    call; stream order keeps consecutive users apart).

    Under HIP-graph capture every call gets a fresh buffer from the graph's private pool:
    a cached buffer recorded into a graph could later be replaced (and freed) by a larger
    eager request while replays still write to it, and capture streams are pooled handles
    whose keys can collide with an eager stream's."""
    if torch.cuda.is_current_stream_capturing():
        return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
    key = (dev.index, _lib.stream_handle(dev))
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        t = _WS[key] = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
    return t


def _memo(obj, key, make):
    """Per-object memo (a graph's capability answers and workspace sizes)."""
    d = obj.__dict__.setdefault("_msha_memo", {})
    v = d.get(key)
    if v is None:
        v = d[key] = make()
    return v


class _EdgeAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, el, er, hc, hs, graph: Graph, p: float, seed: int, slope: float, ar=None):
        n, H = el.shape
        m, H2, F = hc.shape
        assert H2 == H and m == graph.n_cols and n == graph.n_rows
        dt = _table_dtype(hc, hs)
        el, er = _f32c(el), _f32c(er)
        hc, hs = _tc(hc, dt), _tc(hs, dt)
        dev = el.device
        s = _stream(el)
        g = graph.desc
        # (u-only with a_r keeps the row-score contract: er is then never read)
        if (hs is not None or ar is None) and bip_ok(graph, H, F, dt):
            # the repo's adjacency shape (M <= 32 recipients): msha_bip_attention_fwd,
            # u and v in one pass over the rows (the column side stays in LDS)
            u = torch.empty(n, H, F, device=dev, dtype=dt)
            lse = torch.empty(n, H, device=dev, dtype=torch.float32)
            v = torch.empty(m, H, F, device=dev, dtype=dt) if hs is not None else None
            ws = _bip_ws(graph, H, F, dev)
            ev = _timed("bip_attention_fwd")
            _lib.call("msha_bip_attention_fwd", g, H, F, _code(dt), el.data_ptr(),
                      er.data_ptr(), hc.data_ptr(), _lib.ptr(hs), slope, p, seed, 0,
                      u.data_ptr(), None, lse.data_ptr(), None, _lib.ptr(v), ws.data_ptr(),
                      ws.numel(), s)
            if ev is not None:
                ev[1].record()
            ctx.graph, ctx.p, ctx.seed, ctx.slope = graph, p, seed, slope
            ctx.has_hs, ctx.bip = hs is not None, True
            ctx.save_for_backward(el, er, hc, hs if hs is not None else el.new_empty(0), lse)
            return u if v is None else (u, v)
        # scores from the gathered row (msha_edge_attention_fwd_rs): er_j = hc_j . a_r is
        # recomputed from the row the kernel gathers anyway, in the forward and in the
        # fused backward's column pass (the same bits in both); u-only path
        rs = (ar is not None and hs is None and ROW_SCORES and FUSED_BWD
              and _lib.load().msha_edge_attention_row_scores_preferred(g, H, F, _code(dt)))
        # er from project_scores in the kernels' order is exactly what the forward
        # recomputes: the backward then reads er per column (no recompute from a_r)
        ctx.er_exact = bool(rs and getattr(er, "_msha_row_order", False))
        ar = ar.detach().to(torch.float32).contiguous().view(H, F) if rs else None
        u = torch.empty(n, H, F, device=dev, dtype=dt)
        # bf16 tables under autograd: keep the rounding residual of u for the backward's
        # D = dU . u (include/msha_gnn.h, u_lo)
        u_lo = torch.empty_like(u) if dt == BF16 and any(ctx.needs_input_grad[:4]) else None
        lse = torch.empty(n, H, device=dev, dtype=torch.float32)
        attd = None
        if hs is not None:
            attd = torch.empty(max(graph.n_edges, 1), H, device=dev, dtype=torch.float32)
        # row terms for the u-only fused backward on large graphs (include/msha_gnn.h
        # msha_edge_attention_fwd_ex): d_el without a per-edge de crossing CSC -> CSR
        uc = qc = None
        if (hs is None and FUSED_BWD and ctx.needs_input_grad[0] and ROWTERMS
                and _lib.load().msha_edge_attention_rowterms_preferred(g, H, F, _code(dt))):
            uc = torch.empty(n, H, F, device=dev, dtype=torch.float32)
            qc = torch.empty(n, H, device=dev, dtype=torch.float32)
        ev = _timed("edge_attention_fwd")
        if rs:
            _lib.call("msha_edge_attention_fwd_rs", g, H, F, _code(dt), el.data_ptr(),
                      ar.data_ptr(), hc.data_ptr(), slope, p, seed, 0, u.data_ptr(),
                      _lib.ptr(u_lo), lse.data_ptr(), _lib.ptr(uc), _lib.ptr(qc), s)
        else:
            _lib.call("msha_edge_attention_fwd_ex", g, H, F, _code(dt), el.data_ptr(),
                      er.data_ptr(), hc.data_ptr(), slope, p, seed, 0, u.data_ptr(),
                      _lib.ptr(u_lo), lse.data_ptr(), _lib.ptr(attd), _lib.ptr(uc),
                      _lib.ptr(qc), s)
        if ev is not None:
            ev[1].record()
        v = None
        if hs is not None:
            v = torch.empty(m, H, F, device=dev, dtype=dt)
            _csc_aggregate(graph, H, F, attd, None, hs, v, None, s)
        ctx.graph, ctx.p, ctx.seed, ctx.slope = graph, p, seed, slope
        ctx.has_hs, ctx.bip = hs is not None, False
        ctx.rowterms = uc is not None
        ctx.rs = bool(rs)
        ctx.save_for_backward(el, er, hc, hs if hs is not None else el.new_empty(0), lse, u,
                              u_lo if u_lo is not None else el.new_empty(0),
                              ar if rs else el.new_empty(0),
                              *((uc, qc) if uc is not None else ()))
        if v is None:
            return u
        return u, v

    @staticmethod
    def backward(ctx, dU, dV=None):
        if ctx.bip:
            return _bip_bwd(ctx, dU, dV)
        el, er, hc, hs, lse, u, u_lo, ar, *rowterms = ctx.saved_tensors
        u_lo = u_lo if u_lo.numel() else None
        ar = ar if ctx.rs and not ctx.er_exact else None
        graph = ctx.graph
        n, H = el.shape
        m, _, F = hc.shape
        dt = hc.dtype
        dev = el.device
        s = _stream(el)
        g = graph.desc
        dU = torch.zeros_like(u) if dU is None else _tc(dU, dt)
        use_dv = ctx.has_hs and dV is not None
        dV = _tc(dV, dt) if use_dv else None
        E = max(graph.n_edges, 1)
        d_el = torch.empty(n, H, device=dev, dtype=torch.float32)
        if not use_dv and FUSED_BWD:
            return _bwd_fused(ctx, el, er, hc, lse, u, u_lo, dU, d_el, hs, rowterms, ar)
        # one (de, attd) record of 2H floats per edge: the column pass reads it as one
        # 64-B segment at C4 (the CSC visits edges in random order)
        rec = torch.empty(E, 2, H, device=dev, dtype=torch.float32)
        de, attd = rec[:, 0], rec[:, 1]
        d_hs = torch.empty(n, H, F, device=dev, dtype=dt) if use_dv else None
        ev = _timed("edge_attention_bwd_rows")
        _lib.call("msha_edge_attention_bwd_rows", g, H, F, _code(dt), el.data_ptr(),
                  er.data_ptr(), hc.data_ptr(), lse.data_ptr(), u.data_ptr(), _lib.ptr(u_lo),
                  dU.data_ptr(),
                  hs.data_ptr() if use_dv else None, _lib.ptr(dV), None, ctx.slope, ctx.p,
                  ctx.seed, 0, d_el.data_ptr(), de.data_ptr(), attd.data_ptr(), 2 * H,
                  _lib.ptr(d_hs), s)
        if ev is not None:
            ev[1].record()
        d_hc = torch.empty(m, H, F, device=dev, dtype=dt)
        d_er = torch.empty(m, H, device=dev, dtype=torch.float32)
        ev = _timed("csc_aggregate")
        _csc_aggregate(graph, H, F, attd, de, dU, d_hc, d_er, s, ld=2 * H)
        if ev is not None:
            ev[1].record()
        if ctx.has_hs and d_hs is None:
            d_hs = torch.zeros_like(hs)
        return d_el, d_er, d_hc, (d_hs if ctx.has_hs else None), None, None, None, None, None


# bipartite small-M kernels (msha_bip_attention_fwd/_bwd) wherever the library covers
# the graph (M * heads * feat <= 4096: every shipped year, bip1m).  Module switch for A/B.
BIP = True


def bip_ok(graph, H, F, dtype) -> bool:
    """The bipartite kernels cover the graph: the library's shape rule (M <= 32,
    M * H <= 64, M * H * F <= 4096) and rows with distinct columns, at most 64 / H each
    (every graph from_dense builds; checked on the host for from_csr)."""
    return bool(BIP and graph.distinct_cols and graph.max_deg * H <= 64 and _memo(
        graph, ("bip", H, F, _code(dtype)),
        lambda: bool(_lib.fn("msha_bip_supported")(graph.desc, H, F, _code(dtype)))))


def _bip_ws(graph, H, F, dev):
    return _workspace(dev, _memo(graph, ("bip_ws", H, F), lambda: int(
        _lib.fn("msha_bip_workspace_size")(graph.desc, H, F))))


def _bip_bwd(ctx, dU, dV):
    """Backward of the bipartite forward: one row pass (msha_bip_attention_bwd) gives
    d_el, d_hs and the column gradients d_hc, d_er through per-wave LDS slabs."""
    el, er, hc, hs, lse = ctx.saved_tensors
    n, H = el.shape
    m, _, F = hc.shape
    dt = hc.dtype
    dev = el.device
    s = _stream(el)
    g = ctx.graph.desc
    dU = torch.zeros(n, H, F, device=dev, dtype=dt) if dU is None else _tc(dU, dt)
    use_dv = ctx.has_hs and dV is not None
    dV = _tc(dV, dt) if use_dv else None
    d_el = torch.empty(n, H, device=dev, dtype=torch.float32)
    d_er = torch.empty(m, H, device=dev, dtype=torch.float32)
    d_hc = torch.empty(m, H, F, device=dev, dtype=dt)
    d_hs = torch.empty(n, H, F, device=dev, dtype=dt) if use_dv else None
    ws = _bip_ws(ctx.graph, H, F, dev)
    ev = _timed("bip_attention_bwd")
    _lib.call("msha_bip_attention_bwd", g, H, F, _code(dt), el.data_ptr(), er.data_ptr(),
              hc.data_ptr(), lse.data_ptr(), dU.data_ptr(), hs.data_ptr() if use_dv else None,
              _lib.ptr(dV), None, ctx.slope, ctx.p, ctx.seed, 0, d_el.data_ptr(),
              d_er.data_ptr(), d_hc.data_ptr(), _lib.ptr(d_hs), ws.data_ptr(), ws.numel(), s)
    if ev is not None:
        ev[1].record()
    if ctx.has_hs and d_hs is None:
        d_hs = torch.zeros_like(hs)
    return d_el, d_er, d_hc, (d_hs if ctx.has_hs else None), None, None, None, None, None


# u-only backward as one column pass (msha_edge_attention_bwd_fused) instead of
# bwd_rows + csc_aggregate; same bits.  Module switch for A/B measurements.
FUSED_BWD = True
# row terms (uc, qc) from the forward where the library prefers them (large graphs);
# module switch for A/B measurements
ROWTERMS = True
# scores from the gathered row when the caller passes a_r (msha_edge_attention_fwd_rs);
# module switch for A/B measurements
ROW_SCORES = True


def _bwd_fused(ctx, el, er, hc, lse, u, u_lo, dU, d_el, hs, rowterms=(), ar=None):
    graph = ctx.graph
    n, H = el.shape
    m, _, F = hc.shape
    dev = el.device
    s = _stream(el)
    g = graph.desc
    if not graph.has_csc:
        raise RuntimeError("graph has no CSC view (build it with_csc=True)")
    uc, qc = rowterms if rowterms else (None, None)
    de = None if uc is not None else torch.empty(max(graph.n_edges, 1), H, device=dev,
                                                 dtype=torch.float32)
    wsb = int(_lib.load().msha_edge_attention_bwd_fused_workspace_size(g, H, F))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    d_hc = torch.empty(m, H, F, device=dev, dtype=hc.dtype)
    d_er = torch.empty(m, H, device=dev, dtype=torch.float32)
    ev = _timed("edge_attention_bwd_fused")
    _lib.call("msha_edge_attention_bwd_fused_rs" if ar is not None else
              "msha_edge_attention_bwd_fused_ex", g, H, F, _code(hc.dtype), el.data_ptr(),
              ar.data_ptr() if ar is not None else er.data_ptr(), hc.data_ptr(), lse.data_ptr(),
              u.data_ptr(), _lib.ptr(u_lo), dU.data_ptr(), ctx.slope, ctx.p, ctx.seed, 0,
              _lib.ptr(uc), _lib.ptr(qc), d_el.data_ptr(), d_er.data_ptr(), d_hc.data_ptr(),
              _lib.ptr(de), ws.data_ptr(), wsb, s)
    if ev is not None:
        ev[1].record()
    d_hs = torch.zeros_like(hs) if ctx.has_hs else None
    return d_el, d_er, d_hc, d_hs, None, None, None, None, None


def _csc_aggregate(graph: Graph, H, F, w, x, table, out, out_x, stream, ld=0):
    if not graph.has_csc:
        raise RuntimeError("graph has no CSC view (build it with_csc=True)")
    assert out.dtype == table.dtype
    g = graph.desc
    wsb = _lib.load().msha_csc_aggregate_workspace_size(g, H, F)
    ws = None
    if graph._plan["n_multi"] > 0:
        ws = torch.empty(int(wsb), dtype=torch.uint8, device=table.device)
    _lib.call("msha_csc_aggregate", g, H, F, _code(table.dtype), w.data_ptr(), _lib.ptr(x), ld,
              table.data_ptr(), out.data_ptr(), _lib.ptr(out_x), _lib.ptr(ws),
              0 if ws is None else ws.numel(), stream)


def edge_attention(graph: Graph, el, er, hc, hs=None, p: float = 0.0, training: bool = False,
                   slope: float = NEG_SLOPE, seed: int | None = None, ar=None):
    """Fused masked edge-softmax + aggregation.

    el (N,H), er (M,H), hc (M,H,F) [, hs (N,H,F)] ->  u (N,H,F)  [, v (M,H,F)]
    with att = softmax_row(lrelu(el_i + er_j)), u = drop(att) @ hc, v = drop(att).T @ hs.
    Tables (hc, hs, u, v and their gradients) are bf16 when hc or hs is bf16 (fp32
    arithmetic, config C3), else fp32; scores and statistics are always fp32.

    ``ar`` (H, F), optional: the score vector er was computed with, er = hc . ar per
    head (Ablation.py:266-267 scores the aggregated table itself).  Then the u-only
    kernels recompute er_j from the gathered rows instead of gathering er per edge
    (msha_edge_attention_fwd_rs / _bwd_fused_rs); the gradient w.r.t. er is returned
    as before and reaches ar / hc through er's producer.
    """
    _lib.require_cuda(el, er, hc, hs)
    F = hc.shape[-1]
    H = el.shape[1]
    if not _lib.load().msha_edge_attention_supported(H, F):
        raise NotImplementedError(f"edge_attention: (heads={H}, feat={F}) not compiled")
    p = float(p) if training else 0.0
    if seed is None:
        seed = new_seed() if p > 0 else 0
    if ar is not None and tuple(ar.shape) not in ((H, F), (H * F,), (H * F, 1)):
        raise ValueError(f"edge_attention: ar must hold heads x feat = {H} x {F} values")
    return _EdgeAttention.apply(el, er, hc, hs, graph, p, seed, slope, ar)


class _GAL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, a, graph: Graph, p: float, seed: int):
        ctx.h_dtype = h.dtype
        h = _f32c(h)
        ctx.a_shape = None if a is None else (a.shape, a.dtype, a.device)
        out = torch.empty_like(h)
        _lib.call("msha_gal_fwd", graph.desc, h.data_ptr(), p, seed, 0, out.data_ptr(),
                  _stream(h))
        ctx.graph, ctx.p, ctx.seed = graph, p, seed
        ctx.save_for_backward(h)
        return out

    @staticmethod
    def backward(ctx, dout):
        (h,) = ctx.saved_tensors
        dout = _f32c(dout)
        dh = torch.empty_like(h)
        _lib.call("msha_gal_bwd", ctx.graph.desc, h.data_ptr(), dout.data_ptr(), ctx.p, ctx.seed,
                  0, dh.data_ptr(), _stream(h))
        da = None
        if ctx.a_shape is not None:
            shape, dtype, dev = ctx.a_shape
            da = torch.zeros(shape, dtype=dtype, device=dev)
        return dh.to(ctx.h_dtype), da, None, None, None


def gal(graph: Graph, h, p: float = 0.0, training: bool = False, seed: int | None = None,
        zero_grad_of=None):
    """``elu(dropout(mask/deg) * h)`` -- GraphAttentionLayer after its projection.

    ``zero_grad_of``: the layer's score vector ``a``; it cannot change the output
    (the score is constant along a row), so it gets an exact zero gradient, which
    keeps optimizers (Adam weight decay) stepping it as in the reference."""
    _lib.require_cuda(h)
    if h.shape != (graph.n_rows, graph.n_cols):
        raise ValueError(f"GAL: h must be (N, M) = {(graph.n_rows, graph.n_cols)}, "
                         f"got {tuple(h.shape)} (the reference needs adj with out_features "
                         f"columns, GAT.py:22-30)")
    p = float(p) if training else 0.0
    if seed is None:
        seed = new_seed() if p > 0 else 0
    return _GAL.apply(h, zero_grad_of, graph, p, seed)


def dropout_keep_mask(n: int, p: float, seed: int, device, offset: int = 0,
                      flat4: bool = False, word: int | None = None) -> torch.Tensor:
    """The kernels' Philox keep mask of n elements (uint8); flat4: the four-words-per-call
    mask of the flat-table dropout (msha_segments, feature dropout); word: word `word` of
    the block keyed on each element (the Ours intra masks)."""
    keep = torch.empty(n, dtype=torch.uint8, device=device)
    if word is not None:
        _lib.call("msha_dropout_keep_mask_word", seed, offset, n, p, word, keep.data_ptr(),
                  _lib.stream_handle(device))
        return keep
    _lib.call("msha_dropout_keep_mask4" if flat4 else "msha_dropout_keep_mask", seed, offset, n,
              p, keep.data_ptr(), _lib.stream_handle(device))
    return keep


# ------------------------------------------------------------------ projections ---
def _splits_for(rows: int, M: int = 128, N: int = 128) -> int:
    """split-K factor for reductions over `rows`: >= 64 rows per split, <= ~1024
    workgroups in all, and the fp32 slab (splits x M x N) within 16 MB."""
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    slab_cap = max(1, (16 << 20) // (4 * M * N))
    return max(1, min(rows // 64, slab_cap, max(1, 1024 // tiles)))


def gemm(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor | None = None,
         accumulate: bool = False, splits: int | None = None, out_dtype=None) -> torch.Tensor:
    """C = A @ B (or C += A @ B) on the MFMA GEMM; A and B may be strided views
    (transposes included).  Long reductions use deterministic split-K.  bf16 operands
    (either one) run the bf16 MFMA kernel; C is then out_dtype (default bf16)."""
    M, K = A.shape
    K2, N = B.shape
    assert K == K2
    if splits is None:
        splits = _splits_for(K, M, N) if K >= 4096 else 1
    if A.dtype == BF16 or B.dtype == BF16:
        assert not accumulate and out is None, "bf16 gemm: no accumulate / out"
        return _gemm_bf16(A, B, splits, out_dtype or BF16, -1, None)
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=torch.float32)
    assert out.stride(1) == 1
    if accumulate and splits == 1:
        splits = 2
    ws = None
    if splits > 1:
        wsb = _lib.load().msha_gemm_workspace_size(M, N, splits)
        ws = torch.empty(int(wsb), dtype=torch.uint8, device=A.device)
    _lib.call("msha_gemm_f32", M, N, K, A.data_ptr(), A.stride(0), A.stride(1), B.data_ptr(),
              B.stride(0), B.stride(1), out.data_ptr(), out.stride(0),
              1.0 if accumulate else 0.0, splits, _lib.ptr(ws), 0 if ws is None else ws.numel(),
              _stream(A))
    return out


def _gemm_bf16(A, B, splits, out_dtype, operand, outer):
    """msha_gemm_bf16: bf16 operands (strided views kept), C in out_dtype."""
    A, B = A.to(BF16), B.to(BF16)
    M, K = A.shape
    N = B.shape[1]
    out = torch.empty(M, N, device=A.device, dtype=out_dtype)
    ws = None
    if splits > 1:
        ws = torch.empty(int(_lib.load().msha_gemm_bf16_workspace_size(M, N, splits)),
                         dtype=torch.uint8, device=A.device)
    H = Fd = 0
    d1 = a1 = d2 = a2 = None
    if outer is not None:
        H, Fd, d1, a1, d2, a2 = outer
        a1, a2 = _f32c(a1), _f32c(a2)
    _lib.call("msha_gemm_bf16", M, N, K, A.data_ptr(), A.stride(0), A.stride(1), B.data_ptr(),
              B.stride(0), B.stride(1), out.data_ptr(), out.stride(0), _code(out_dtype), splits,
              _lib.ptr(ws), 0 if ws is None else ws.numel(), operand, H, Fd, _lib.ptr(d1),
              _lib.ptr(a1), _lib.ptr(d2), _lib.ptr(a2), _stream(A))
    return out


def gemm_head_outer(A: torch.Tensor, B: torch.Tensor, operand: int, outer,
                    out_dtype=None) -> torch.Tensor:
    """A @ B with operand 0 (A) or 1 (B) read as X + de (x) a [+ de2 (x) a2]
    (outer = (heads, feat, de, a, de2, a2)).  fp32: falls back to materialising the
    sum with msha_add_head_outer only when the operand layout cannot take the fused
    loads.  bf16 operands: the bf16 kernel (C in out_dtype, default bf16)."""
    H, Fd, d1, a1, d2, a2 = outer
    M, K = A.shape
    N = B.shape[1]
    splits = _splits_for(K, M, N) if K >= 4096 else 1
    if A.dtype == BF16 or B.dtype == BF16:
        return _gemm_bf16(A, B, splits, out_dtype or BF16, operand, outer)
    out = torch.empty(M, N, device=A.device, dtype=torch.float32)
    ws = None
    if splits > 1:
        ws = torch.empty(int(_lib.load().msha_gemm_workspace_size(M, N, splits)),
                         dtype=torch.uint8, device=A.device)
    rc = _lib.load().msha_gemm_f32_head_outer(
        M, N, K, A.data_ptr(), A.stride(0), A.stride(1), B.data_ptr(), B.stride(0), B.stride(1),
        out.data_ptr(), out.stride(0), 0.0, splits, _lib.ptr(ws), 0 if ws is None else ws.numel(),
        operand, H, Fd, d1.data_ptr(), a1.data_ptr(), _lib.ptr(d2), _lib.ptr(a2), _stream(A))
    if rc == 0:
        return out
    if rc != _lib.MSHA_ERR_UNSUPPORTED:
        _lib.raise_for(rc, "msha_gemm_f32_head_outer")
    X = A if operand == 0 else B
    tot = torch.empty(X.shape, device=X.device, dtype=torch.float32)
    _lib.call("msha_add_head_outer", X.shape[0], H, Fd, _f32c(X).data_ptr(), d1.data_ptr(),
              a1.data_ptr(), _lib.ptr(d2), _lib.ptr(a2), tot.data_ptr(), _stream(X))
    return gemm(tot, B) if operand == 0 else gemm(A, tot)


class _MatMul(torch.autograd.Function):
    """C = A @ B with both products of the backward on the library GEMMs (split-K over
    long reductions, deterministic)."""

    @staticmethod
    def forward(ctx, A, B):
        ctx.save_for_backward(A, B)
        return _mm(A, B)

    @staticmethod
    def backward(ctx, dC):
        A, B = ctx.saved_tensors
        dA = _mm(dC, B.t()).to(A.dtype) if ctx.needs_input_grad[0] else None
        dB = _mm(A.t(), dC).to(B.dtype) if ctx.needs_input_grad[1] else None
        return dA, dB


def _mm(A, B):
    if A.dtype == BF16 or B.dtype == BF16:
        if B.shape[1] % 8 == 0:
            return gemm(A, B)
        # bf16 C needs N % 8 == 0: fp32 operands on the exact-fp32 kernel instead
        return gemm(A.float(), B.float()).to(BF16)
    return gemm(A.float(), B.float())


def matmul(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """Differentiable A @ B on the library GEMMs (fp32, or bf16 when an operand is)."""
    _lib.require_cuda(A, B)
    return _MatMul.apply(A, B)


class _ProjectScores(torch.autograd.Function):
    """h = X @ W, el = h . al, er = h . ar (per head) in one MFMA launch.  fp32 X, W:
    the exact-fp32 MFMA kernel; a bf16 X or W: the bf16 kernel (h bf16, el/er fp32)."""

    @staticmethod
    def forward(ctx, X, W, al, ar, heads: int, feat: int):
        ctx.dtypes = (X.dtype, W.dtype, None if al is None else al.dtype,
                      None if ar is None else ar.dtype)
        dt = _table_dtype(X, W)
        X, W = _tc(X, dt), _tc(W, dt)
        al, ar = _f32c(al), _f32c(ar)
        M, K = X.shape
        dev = X.device
        h = torch.empty(M, heads * feat, device=dev, dtype=dt)
        el = torch.empty(M, heads, device=dev, dtype=torch.float32) if al is not None else None
        er = torch.empty(M, heads, device=dev, dtype=torch.float32) if ar is not None else None
        # a small table (the 32 recipients of R15): one single-workgroup launch each way
        ctx.small = dt == torch.float32 and _project_small(M, K, heads, feat)
        fn = ("msha_project_small" if ctx.small else
              "msha_project_scores_bf16" if dt == BF16 else "msha_project_scores")
        _lib.call(fn, M, K, heads, feat, X.data_ptr(), W.data_ptr(), _lib.ptr(al), _lib.ptr(ar),
                  h.data_ptr(), _lib.ptr(el), _lib.ptr(er), _stream(X))
        ctx.heads, ctx.feat = heads, feat
        ctx.save_for_backward(X, W, al, ar, h)
        outs = [h]
        if el is not None:
            outs.append(el)
        if er is not None:
            outs.append(er)
        return tuple(outs) if len(outs) > 1 else h

    @staticmethod
    def backward(ctx, dh, *dscores):
        X, W, al, ar, h = ctx.saved_tensors
        H, Fd = ctx.heads, ctx.feat
        xdt, wdt, aldt, ardt = ctx.dtypes
        dt = h.dtype
        M = X.shape[0]
        dev = X.device
        s = _stream(X)
        it = iter(dscores)
        d_el = next(it) if al is not None else None
        d_er = next(it) if ar is not None else None
        if ctx.small:
            d_el, d_er = _f32c(d_el), _f32c(d_er)
            dh = None if dh is None else _tc(dh, dt)
            dX = torch.empty_like(X) if ctx.needs_input_grad[0] else None
            dW = torch.empty_like(W) if ctx.needs_input_grad[1] else None
            dal = torch.empty(H, Fd, device=dev) if d_el is not None and ctx.needs_input_grad[2] \
                else None
            dar = torch.empty(H, Fd, device=dev) if d_er is not None and ctx.needs_input_grad[3] \
                else None
            _lib.call("msha_project_small_bwd", M, X.shape[1], H, Fd, X.data_ptr(), W.data_ptr(),
                      _lib.ptr(al), _lib.ptr(ar), h.data_ptr(), _lib.ptr(dh), _lib.ptr(d_el),
                      _lib.ptr(d_er), _lib.ptr(dX), _lib.ptr(dW), _lib.ptr(dal), _lib.ptr(dar), s)
            return (dX, dW, None if dal is None else dal.reshape(al.shape).to(aldt),
                    None if dar is None else dar.reshape(ar.shape).to(ardt), None, None)
        dh = torch.zeros_like(h) if dh is None else _tc(dh, dt)
        terms = [(d, a) for d, a in ((d_el, al), (d_er, ar)) if d is not None]
        dX = dW = dal = dar = None
        kw = {"out_dtype": None}
        if terms:
            # dh + d_el (x) al (+ d_er (x) ar) is folded into the GEMM operand loads
            (d1, a1) = terms[0]
            d2, a2 = terms[1] if len(terms) > 1 else (None, None)
            d1, d2 = _f32c(d1), _f32c(d2)
            outer = (H, Fd, d1, a1, d2, a2)
            if ctx.needs_input_grad[0]:
                kw["out_dtype"] = xdt if dt == BF16 else None
                dX = gemm_head_outer(dh, W.t(), 0, outer, **kw)
            if ctx.needs_input_grad[1]:
                kw["out_dtype"] = wdt if dt == BF16 else None
                if dt == torch.float32 and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3]):
                    # dW, dal, dar in one pass over the rows where the shape allows
                    fused = _wgrad_colsum(X, dh, outer, h, W)
                    if fused is not None:
                        dW, o1, o2 = fused
                        dal, dar = _score_grads(d_el, d_er, o1, o2, al, ar, aldt, ardt)
                        return dX, dW, dal, dar, None, None
                dW = gemm_head_outer(X.t(), dh, 1, outer, **kw)
        else:
            if ctx.needs_input_grad[0]:
                dX = gemm(dh, W.t(), out_dtype=xdt if dt == BF16 else None)
            if ctx.needs_input_grad[1]:
                dW = gemm(X.t(), dh, out_dtype=wdt if dt == BF16 else None)
        if terms and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3]):
            # dal[h,f] = sum_m d_el[m,h] h[m,h,f] (and dar): one pass over h
            (d1, a1) = terms[0]
            d2 = terms[1][0] if len(terms) > 1 else None
            o1 = torch.empty(H, Fd, device=dev, dtype=torch.float32)
            o2 = torch.empty(H, Fd, device=dev, dtype=torch.float32) if d2 is not None else None
            ws = _workspace(dev, int(_lib.fn("msha_head_colsum_workspace_size")(M, H, Fd)))
            d1, d2 = _f32c(d1), _f32c(d2)  # held until the launch (see bn_lrelu)
            _lib.call("msha_head_colsum", M, H, Fd, _code(dt), d1.data_ptr(),
                      _lib.ptr(d2), h.data_ptr(), o1.data_ptr(), _lib.ptr(o2),
                      ws.data_ptr(), ws.numel(), s)
            dal, dar = _score_grads(d_el, d_er, o1, o2, al, ar, aldt, ardt)
        return dX, dW, dal, dar, None, None


def _score_grads(d_el, d_er, o1, o2, al, ar, aldt, ardt):
    """(dal, dar) from the column sums of the present score terms, in order."""
    outs = [o1] + ([o2] if o2 is not None else [])
    dal = dar = None
    k = 0
    if d_el is not None:
        dal = outs[k].reshape(al.shape).to(aldt)
        k += 1
    if d_er is not None:
        dar = outs[k].reshape(ar.shape).to(ardt)
    return dal, dar


def _wgrad_colsum(X, dh, outer, h, W=None):
    """dW = X^T (dh + d1 (x) a1 [+ d2 (x) a2]) and the column sums of d1 (x) h, d2 (x) h
    (msha_gemm_f32_head_outer_colsum: one pass over the rows), or None where the fused
    kernel does not cover the shape (the caller runs the two ops).  With W (h = X @ W, the
    projection's own output) the sums come as (d^T X) W from the rows the weight gradient
    already reads (msha_gemm_f32_head_outer_colsum_w: h is not read) where that kernel
    covers the shape."""
    H, Fd, d1, a1, d2, a2 = outer
    M, K = X.shape
    N = dh.shape[1]
    if M < 4096 or not (dh.is_contiguous() and h.is_contiguous() and h.shape == dh.shape):
        return None
    splits = _splits_for(M, K, N)
    dev = X.device
    dW = torch.empty(K, N, device=dev, dtype=torch.float32)
    # the GEMM's and the colsum's scratch as two aligned parts of the shared workspace
    wsb = (int(_lib.fn("msha_gemm_workspace_size")(K, N, splits)) + 255) // 256 * 256
    cwsb = int(_lib.fn("msha_head_outer_colsum_workspace_size")(N))
    buf = _workspace(dev, wsb + cwsb)
    o1 = torch.empty(H, Fd, device=dev, dtype=torch.float32)
    o2 = torch.empty(H, Fd, device=dev, dtype=torch.float32) if d2 is not None else None
    A = X.t()
    if W is not None and W.dtype == torch.float32 and W.shape == (K, N) and W.stride(1) == 1:
        rc = _lib.fn("msha_gemm_f32_head_outer_colsum_w")(
            K, N, M, A.data_ptr(), A.stride(0), A.stride(1), dh.data_ptr(), dh.stride(0),
            dh.stride(1), dW.data_ptr(), dW.stride(0), splits, buf.data_ptr(), wsb, H, Fd,
            d1.data_ptr(), a1.data_ptr(), _lib.ptr(d2), _lib.ptr(a2), W.data_ptr(), W.stride(0),
            o1.data_ptr(), _lib.ptr(o2), buf.data_ptr() + wsb, cwsb, _stream(X))
        if rc == 0:
            return dW, o1, o2
        if rc != _lib.MSHA_ERR_UNSUPPORTED:
            _lib.raise_for(rc, "msha_gemm_f32_head_outer_colsum_w")
    rc = _lib.fn("msha_gemm_f32_head_outer_colsum")(
        K, N, M, A.data_ptr(), A.stride(0), A.stride(1), dh.data_ptr(), dh.stride(0),
        dh.stride(1), dW.data_ptr(), dW.stride(0), splits, buf.data_ptr(), wsb, H, Fd,
        d1.data_ptr(), a1.data_ptr(), _lib.ptr(d2), _lib.ptr(a2), h.data_ptr(), o1.data_ptr(),
        _lib.ptr(o2), buf.data_ptr() + wsb, cwsb, _stream(X))
    if rc == _lib.MSHA_ERR_UNSUPPORTED:
        return None
    if rc != 0:
        _lib.raise_for(rc, "msha_gemm_f32_head_outer_colsum")
    return dW, o1, o2


@functools.lru_cache(maxsize=256)
def _project_small(M, K, heads, feat) -> bool:
    return bool(_lib.fn("msha_project_small_supported")(M, K, heads, feat))


@functools.lru_cache(maxsize=256)
def _row_order(M, K, heads, feat, code) -> bool:
    return bool(_lib.fn("msha_project_scores_row_order")(M, K, heads, feat, code))


def project_scores(X, W, al=None, ar=None, heads: int = 1, feat: int | None = None):
    """``h = X @ W`` on the MFMA GEMM, with optional fused per-head score halves
    ``el = h . al``, ``er = h . ar`` (al/ar: (heads, feat)).  Returns h or
    (h, el[, er])."""
    _lib.require_cuda(X, W)
    feat = W.shape[1] // heads if feat is None else feat
    if al is not None:
        al = al.reshape(heads, feat)
    if ar is not None:
        ar = ar.reshape(heads, feat)
    out = _ProjectScores.apply(X, W, al, ar, heads, feat)
    if ar is not None:
        # er computed from the stored h in the order the row-score edge kernels recompute
        # it (msha_project_scores_row_order): edge_attention(..., ar=) then reads this er
        # where it needs er_j per column instead of recomputing it (the same bits)
        M, K = X.shape
        out[-1]._msha_row_order = _row_order(M, K, heads, feat, _code(_table_dtype(X, W)))
    return out


# ----------------------------------------------------------------- GCN SpMM ---
class _SpMM(torch.autograd.Function):
    """out = A^T @ table (transpose) or A @ table, A = the graph with edge values
    ``vals``: msha_csc_aggregate over the CSC view or the CSR-as-CSC row view."""

    @staticmethod
    def forward(ctx, table, vals, graph: Graph, transpose: bool):
        ctx.graph, ctx.transpose = graph, transpose
        ctx.save_for_backward(vals)
        return _spmm(graph, vals, table, transpose)

    @staticmethod
    def backward(ctx, dout):
        (vals,) = ctx.saved_tensors
        return _spmm(ctx.graph, vals, dout, not ctx.transpose), None, None, None


def _spmm(graph: Graph, vals, table, transpose):
    view = graph if transpose else graph.row_view()
    dt = _table_dtype(table)
    table = _tc(table, dt)
    D = table.shape[1]
    if table.shape[0] != view.n_rows:
        raise ValueError(f"spmm: table has {table.shape[0]} rows, expected {view.n_rows}")
    out = torch.empty(view.n_cols, D, device=table.device, dtype=dt)
    _csc_aggregate(view, 1, D, _f32c(vals), None, table, out, None, _stream(table))
    return out


def spmm(graph: Graph, vals: torch.Tensor, table: torch.Tensor, transpose: bool = True):
    """GCN propagation (model.py:37): ``A^T @ table`` (transpose) or ``A @ table`` with
    A's values ``vals`` on the graph's CSR edges (Graph.values); deterministic, fp32 or
    bf16 tables; feature width in {8, 16, 32, 64, 128}."""
    _lib.require_cuda(table, vals)
    if not _lib.load().msha_edge_attention_supported(1, table.shape[1]):
        raise NotImplementedError(f"spmm: width {table.shape[1]} not compiled")
    return _SpMM.apply(table, vals, graph, transpose)


# --------------------------------------------------- BatchNorm + LeakyReLU ---
class _BnLRelu(torch.autograd.Function):
    """lrelu(batch_norm(x)) with training batch statistics (Ablation.py:273-274)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, slope, momentum):
        dt = _table_dtype(x)
        x = _tc(x, dt)
        R, C = x.shape
        dev = x.device
        w32, b32 = _f32c(weight), _f32c(bias)
        rm = rv = None
        if running_mean is not None:
            rm, rv = _f32c(running_mean), _f32c(running_var)
        mean = torch.empty(C, device=dev, dtype=torch.float32)
        invstd = torch.empty(C, device=dev, dtype=torch.float32)
        y = torch.empty_like(x)
        wsb = int(_lib.load().msha_bn_workspace_size(R, C))
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)
        _lib.call("msha_bn_lrelu_fwd", R, C, _code(dt), x.data_ptr(), _lib.ptr(w32),
                  _lib.ptr(b32), eps, slope, 1, momentum, _lib.ptr(rm), _lib.ptr(rv),
                  mean.data_ptr(), invstd.data_ptr(), y.data_ptr(), ws.data_ptr(), ws.numel(),
                  _stream(x))
        if rm is not None and rm.data_ptr() != running_mean.data_ptr():
            running_mean.copy_(rm)  # non-fp32 / strided buffers: write the update back
            running_var.copy_(rv)
        ctx.slope = slope
        ctx.pdtypes = (None if weight is None else weight.dtype, None if bias is None else bias.dtype)
        ctx.save_for_backward(x, w32, b32, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w32, b32, mean, invstd = ctx.saved_tensors
        R, C = x.shape
        dev = x.device
        dy = _tc(dy, x.dtype)
        dx = torch.empty_like(x)
        dw = torch.empty(C, device=dev, dtype=torch.float32) if w32 is not None else None
        db = torch.empty(C, device=dev, dtype=torch.float32) if b32 is not None else None
        wsb = int(_lib.load().msha_bn_workspace_size(R, C))
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)
        _lib.call("msha_bn_lrelu_bwd", R, C, _code(x.dtype), x.data_ptr(), dy.data_ptr(),
                  _lib.ptr(w32), _lib.ptr(b32), mean.data_ptr(), invstd.data_ptr(), ctx.slope,
                  dx.data_ptr(), _lib.ptr(dw), _lib.ptr(db), ws.data_ptr(), ws.numel(),
                  _stream(x))
        wdt, bdt = ctx.pdtypes
        return (dx, None if dw is None else dw.to(wdt), None if db is None else db.to(bdt),
                None, None, None, None, None)


def bn_lrelu(x: torch.Tensor, bn: torch.nn.BatchNorm1d, slope: float,
             count: bool = True) -> torch.Tensor:
    """``lrelu(bn(x), slope)`` for a (rows, C) table on the fused kernels: batch
    statistics and the running-statistics update as torch.nn.BatchNorm1d in training
    mode (momentum set; num_batches_tracked advanced on the device -- by the caller
    when ``count`` is False, e.g. one foreach add for all heads), running
    statistics in eval mode."""
    _lib.require_cuda(x)
    if x.dim() != 2 or bn.momentum is None:
        # cumulative-average momentum needs the host-side batch count: torch's path
        return torch.nn.functional.leaky_relu(bn(x), slope)
    use_batch = bn.training or not bn.track_running_stats
    if not use_batch:
        if torch.is_grad_enabled() and (x.requires_grad or bn.weight.requires_grad):
            return torch.nn.functional.leaky_relu(bn(x), slope)  # eval with autograd
        dt = _table_dtype(x)
        xc = _tc(x, dt)
        R, C = xc.shape
        y = torch.empty_like(xc)
        # fp32 views/copies held in locals until the launch: a temporary freed after
        # data_ptr() can be handed to the next copy by the caching allocator (bf16 models:
        # weight and bias copies would share one block)
        rm, rv = _f32c(bn.running_mean), _f32c(bn.running_var)
        w32, b32 = _f32c(bn.weight), _f32c(bn.bias)
        _lib.call("msha_bn_lrelu_fwd", R, C, _code(dt), xc.data_ptr(), _lib.ptr(w32),
                  _lib.ptr(b32), bn.eps, slope, 0, 0.0, rm.data_ptr(), rv.data_ptr(),
                  None, None, y.data_ptr(), None, 0, _stream(xc))
        return y
    track = bn.training and bn.track_running_stats
    if track and count:
        bn.num_batches_tracked.add_(1)
    return _BnLRelu.apply(x, bn.weight, bn.bias, bn.running_mean if track else None,
                          bn.running_var if track else None, bn.eps, slope,
                          float(bn.momentum))


# ------------------------------------------------------------------ link scoring ---
ACT_BIAS, ACT_RELU, ACT_DROPOUT, ACT_SIGMOID = 1, 2, 4, 8


class _PairInner(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_i, x_j):
        x_i, x_j = _f32c(x_i), _f32c(x_j)
        B, Fd = x_i.shape
        out = torch.empty(B, device=x_i.device, dtype=torch.float32)
        _lib.call("msha_pair_inner_fwd", B, Fd, x_i.data_ptr(), Fd, None, x_j.data_ptr(), Fd,
                  None, out.data_ptr(), _stream(x_i))
        ctx.save_for_backward(x_i, x_j, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        x_i, x_j, out = ctx.saved_tensors
        B, Fd = x_i.shape
        dxi, dxj = torch.empty_like(x_i), torch.empty_like(x_j)
        _lib.call("msha_pair_inner_bwd", B, Fd, x_i.data_ptr(), Fd, None, x_j.data_ptr(), Fd,
                  None, out.data_ptr(), _f32c(dout).data_ptr(), dxi.data_ptr(), dxj.data_ptr(),
                  _stream(x_i))
        return dxi, dxj


class _PairLayer(torch.autograd.Function):
    """y = [sigmoid](dropout(relu(x @ W^T + b))) with x = x_i * x_j (first layer,
    fused) or x = x_i (deeper layers, x_j None)."""

    @staticmethod
    def forward(ctx, x_i, x_j, W, b, p: float, seed: int, sigmoid: bool):
        x_i, x_j, W, b = _f32c(x_i), _f32c(x_j), _f32c(W), _f32c(b)
        B, K = x_i.shape
        N = W.shape[0]
        act = ACT_BIAS | ACT_RELU | (ACT_DROPOUT if p > 0 else 0) | (ACT_SIGMOID if sigmoid else 0)
        out = torch.empty(B, N, device=x_i.device, dtype=torch.float32)
        _lib.call("msha_pair_linear", B, K, N, x_i.data_ptr(), K, None, _lib.ptr(x_j), K, None,
                  B, B, W.data_ptr(), b.data_ptr(), act, p, seed, 0, out.data_ptr(),
                  _stream(x_i))
        ctx.p, ctx.sigmoid = p, sigmoid
        ctx.has_xj = x_j is not None
        ctx.save_for_backward(x_i, x_j if x_j is not None else x_i.new_empty(0), W, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        x_i, x_j, W, out = ctx.saved_tensors
        B, K = x_i.shape
        N = W.shape[0]
        s = _stream(x_i)
        dz = torch.empty_like(out)
        _lib.call("msha_pair_mlp_dz", B * N, out.data_ptr(), _f32c(dout).data_ptr(), ctx.p,
                  1 if ctx.sigmoid else 0, dz.data_ptr(), s)
        if ctx.has_xj:
            x = torch.empty_like(x_i)
            _lib.call("msha_pair_hadamard", B, K, x_i.data_ptr(), K, None, x_j.data_ptr(), K, None,
                      None, x.data_ptr(), None, s)
        else:
            x = x_i
        dW = gemm(dz.t(), x)                      # (N, K) = dz^T x
        one = torch.ones(1, device=x_i.device, dtype=torch.float32)
        db = gemm(one.as_strided((1, B), (0, 0)), dz).view(N)  # column sums of dz
        dx = gemm(dz, W)                          # (B, K)
        if ctx.has_xj:
            dxi, dxj = torch.empty_like(x_i), torch.empty_like(x_j)
            _lib.call("msha_pair_hadamard", B, K, x_i.data_ptr(), K, None, x_j.data_ptr(), K, None,
                      dx.data_ptr(), dxi.data_ptr(), dxj.data_ptr(), s)
            return dxi, dxj, dW, db, None, None, None
        return dx, None, dW, db, None, None, None


class _PairHadamardSigmoid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_i, x_j):
        x_i, x_j = _f32c(x_i), _f32c(x_j)
        B, Fd = x_i.shape
        y = torch.empty_like(x_i)
        _lib.call("msha_pair_hadamard_sigmoid", B, Fd, x_i.data_ptr(), Fd, None, x_j.data_ptr(),
                  Fd, None, None, None, y.data_ptr(), None, _stream(x_i))
        ctx.save_for_backward(x_i, x_j, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x_i, x_j, y = ctx.saved_tensors
        B, Fd = x_i.shape
        dxi, dxj = torch.empty_like(x_i), torch.empty_like(x_j)
        _lib.call("msha_pair_hadamard_sigmoid", B, Fd, x_i.data_ptr(), Fd, None, x_j.data_ptr(),
                  Fd, None, y.data_ptr(), _f32c(dy).data_ptr(), dxi.data_ptr(), dxj.data_ptr(),
                  _stream(x_i))
        return dxi, dxj


def pair_hadamard_sigmoid(x_i, x_j):
    """LinkPredictor with any predictor other than 'mlp' / 'inner' (LLP.py:104-115):
    ``sigmoid(x_i * x_j)``, (B, F)."""
    _lib.require_cuda(x_i, x_j)
    if x_i.shape != x_j.shape or x_i.dim() != 2:
        raise ValueError(f"pair_hadamard_sigmoid: x_i {tuple(x_i.shape)} vs x_j "
                         f"{tuple(x_j.shape)}")
    return _PairHadamardSigmoid.apply(x_i, x_j)


def pair_inner(x_i, x_j):
    """'inner' LinkPredictor head: sigmoid(sum(x_i * x_j, -1))  (LLP.py:112-115)."""
    _lib.require_cuda(x_i, x_j)
    return _PairInner.apply(x_i, x_j)


def pair_layer(x_i, x_j, W, b, p=0.0, training=False, sigmoid=False, seed=None):
    _lib.require_cuda(x_i, x_j, W, b)
    p = float(p) if training else 0.0
    if seed is None:
        seed = new_seed() if p > 0 else 0
    return _PairLayer.apply(x_i, x_j, W, b, p, seed, sigmoid)


def check_pair_indices(src, dst, rows: int, rows2: int | None = None):
    """torch's ``h[idx]`` index rule for a fused pair gather (LLP.py:233): an index
    outside [-rows, rows) raises IndexError; negative ones inside are wrapped to
    rows + idx.  One device pass (``msha_pair_index_check``) and one flag read (a
    stream sync).  Returns the (possibly wrapped) int64 index tensors."""
    rows2 = rows if rows2 is None else rows2
    src = src.to(torch.int64).contiguous()
    dst = dst.to(torch.int64).contiguous()
    if src.numel() != dst.numel():
        raise ValueError(f"pair indices differ in length: {src.numel()} vs {dst.numel()}")
    flags = torch.zeros(2, dtype=torch.int32, device=src.device)
    _lib.call("msha_pair_index_check", src.numel(), src.data_ptr(), int(rows), dst.data_ptr(),
              int(rows2), flags.data_ptr(), _stream(src))
    oob, neg = flags.tolist()
    if oob:
        for idx, n in ((src, rows), (dst, rows2)):
            bad = idx[(idx >= n) | (idx < -n)]
            if bad.numel():
                raise IndexError(f"index {int(bad[0])} is out of bounds for dimension 0 "
                                 f"with size {n}")
    if neg:
        src = torch.where(src < 0, src + rows, src)
        dst = torch.where(dst < 0, dst + rows2, dst)
    return src, dst


def score_pairs(h, src, dst, mode="inner", W=None, b=None, out=None, out_dtype=None,
                check=True):
    """Fused caller gather + predictor (LLP.py:233 + LLP.py:104-115), inference:
    ``predictor(h[src], h[dst])`` without materialising the gathered rows.
    'inner' -> (P,), 'mlp' (one used Linear W (hidden, F), b) -> (P, hidden).
    A bf16 ``h`` runs the bf16 kernels (bf16 MFMA for 'mlp'; fp32 scores, or bf16
    'mlp' scores with ``out_dtype=torch.bfloat16``, as a bf16 LinkPredictor returns).
    ``check`` (default) applies torch's ``h[idx]`` rule first (``check_pair_indices``:
    IndexError outside [-n, n), negative indices wrapped; one stream sync).  With
    ``check=False`` the caller vouches for indices in [0, n) (a pipelined scorer whose
    batch was checked once); the 'inner' kernel still bounds every row and scores a
    stray pair NaN, the fp32 'mlp' gather reads zeros for it."""
    _lib.require_cuda(h, src, dst)
    dt = _table_dtype(h)
    h = _tc(h, dt)
    bf = dt == BF16
    if check:
        src, dst = check_pair_indices(src, dst, h.shape[0])
    src = src.to(torch.int64).contiguous()
    dst = dst.to(torch.int64).contiguous()
    P, Fd = src.numel(), h.shape[1]
    s = _stream(h)
    if mode == "inner":
        out = torch.empty(P, device=h.device, dtype=torch.float32) if out is None else out
        _lib.call("msha_pair_inner_fwd_ex", P, Fd, _code(dt), h.data_ptr(),
                  h.stride(0), src.data_ptr(), h.shape[0], h.data_ptr(), h.stride(0),
                  dst.data_ptr(), h.shape[0], None, out.data_ptr(), s)
        return out
    W, b = _tc(W, dt), _f32c(b)
    N = W.shape[0]
    if bf and (out_dtype == BF16 or (out is not None and out.dtype == BF16)):
        out = torch.empty(P, N, device=h.device, dtype=BF16) if out is None else out
        _lib.call("msha_pair_linear_bf16_ex", P, Fd, N, h.data_ptr(), h.stride(0),
                  src.data_ptr(), h.data_ptr(), h.stride(0), dst.data_ptr(), W.data_ptr(),
                  b.data_ptr(), ACT_BIAS | ACT_RELU | ACT_SIGMOID, 0.0, 0, 0, 1,
                  out.data_ptr(), s)
        return out
    out = torch.empty(P, N, device=h.device, dtype=torch.float32) if out is None else out
    rows = (h.shape[0], h.shape[0]) if not bf else ()  # the fp32 entry takes the row counts
    _lib.call("msha_pair_linear_bf16" if bf else "msha_pair_linear", P, Fd, N, h.data_ptr(),
              h.stride(0), src.data_ptr(), h.data_ptr(), h.stride(0), dst.data_ptr(), *rows,
              W.data_ptr(), b.data_ptr(), ACT_BIAS | ACT_RELU | ACT_SIGMOID, 0.0, 0, 0,
              out.data_ptr(), s)
    return out


# --------------------------------------------------------- full MSHA layer (Ours) ---
# the bipartite kernels' block-partial reduce rides in the Ours layer's prep / finish
# launches (msha_bip_defer_reduce; one graph node fewer each way); MSHA_BIP_DEFER=0: separate
# reduce launches (A/B)
BIP_DEFER_REDUCE = os.environ.get("MSHA_BIP_DEFER", "1") != "0"


class _OursAttention(torch.autograd.Function):
    """Ours.py:54-101 core: inter attention (u, v) + batch intra attention added to u."""

    @staticmethod
    def forward(ctx, el, er, h1, h2, a3s, a4s, graph: Graph, groups, src, p: float, seed: int,
                slope: float):
        n, H = el.shape
        m, _, Fd = h1.shape
        dt = _table_dtype(h1, h2)
        el, er, h1, h2 = _f32c(el), _f32c(er), _tc(h1, dt), _tc(h2, dt)
        a3s, a4s = _f32c(a3s), _f32c(a4s)
        src = src.to(torch.int64).contiguous()
        B = src.numel()
        dev = el.device
        s = _stream(el)
        g = graph.desc
        u_inter = torch.empty(n, H, Fd, device=dev, dtype=dt)
        bip = bip_ok(graph, H, Fd, dt)
        u_lo = (torch.empty_like(u_inter) if dt == BF16 and not bip
                and any(ctx.needs_input_grad[:4]) else None)
        lse = torch.empty(n, H, device=dev, dtype=torch.float32)
        attd = torch.empty(max(graph.n_edges, 1), H, device=dev, dtype=torch.float32)
        v = torch.empty(m, H, Fd, device=dev, dtype=dt)
        bstat = torch.empty(max(B, 1), H, 8, device=dev, dtype=torch.float32)
        u = torch.empty_like(u_inter)
        defer = bip and BIP_DEFER_REDUCE
        try:
            if bip:
                # u, v and the attention export in one pass (msha_bip_attention_fwd); its v
                # reduce runs inside the intra launch below (msha_bip_defer_reduce)
                ws = _bip_ws(graph, H, Fd, dev)
                if defer:
                    _lib.call("msha_bip_defer_reduce", 1)
                _lib.call("msha_bip_attention_fwd", g, H, Fd, _code(dt), el.data_ptr(),
                          er.data_ptr(), h1.data_ptr(), h2.data_ptr(), slope, p, seed, 0,
                          u_inter.data_ptr(), None, lse.data_ptr(), attd.data_ptr(),
                          v.data_ptr(), ws.data_ptr(), ws.numel(), s)
            else:
                _lib.call("msha_edge_attention_fwd", g, H, Fd, _code(dt), el.data_ptr(),
                          er.data_ptr(), h1.data_ptr(), slope, p, seed, 0, u_inter.data_ptr(),
                          _lib.ptr(u_lo), lse.data_ptr(), attd.data_ptr(), s)
                _csc_aggregate(graph, H, Fd, attd, None, h2, v, None, s)
            _lib.call("msha_ours_intra_fwd", g, groups.desc, B, src.data_ptr(), H, Fd,
                      _code(dt), h2.data_ptr(), a3s.data_ptr(), a4s.data_ptr(), el.data_ptr(),
                      er.data_ptr(), lse.data_ptr(), u_inter.data_ptr(), slope, p, seed, 0,
                      bstat.data_ptr(), u.data_ptr(), s)
        finally:
            if defer:
                _lib.call("msha_bip_defer_reduce", 0)  # (launches it if still pending)
        ctx.bip = bip
        ctx.graph, ctx.groups, ctx.p, ctx.seed, ctx.slope = graph, groups, p, seed, slope
        ctx.save_for_backward(el, er, h1, h2, a3s, a4s, lse, u_inter, bstat, src,
                              u_lo if u_lo is not None else el.new_empty(0))
        # post-dropout inter attention and batch statistics: outputs for record mode
        ctx.mark_non_differentiable(attd, bstat)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for attd / bstat
        return u, v, attd, bstat

    @staticmethod
    def backward(ctx, dU, dV, _attd=None, _bstat=None):
        el, er, h1, h2, a3s, a4s, lse, u_inter, bstat, src, u_lo = ctx.saved_tensors
        u_lo = u_lo if u_lo.numel() else None
        graph, groups = ctx.graph, ctx.groups
        n, H = el.shape
        m, _, Fd = h1.shape
        B = src.numel()
        dev = el.device
        s = _stream(el)
        g, gr = graph.desc, groups.desc
        dt = h1.dtype
        dU = torch.zeros_like(u_inter) if dU is None else _tc(dU, dt)
        dV = torch.zeros(m, H, Fd, device=dev, dtype=dt) if dV is None else _tc(dV, dt)
        G = torch.empty(max(B, 1), 2, H * Fd, device=dev, dtype=torch.float32)
        bgrad = torch.empty(max(B, 1), H, 4, device=dev, dtype=torch.float32)
        row_coef = torch.empty(n, H, device=dev, dtype=torch.float32)  # zeroed by stage 0
        da3s = torch.empty(H, Fd, device=dev, dtype=torch.float32)
        da4s = torch.empty(H, Fd, device=dev, dtype=torch.float32)
        args = (g, gr, B, src.data_ptr(), H, Fd, _code(dt), h2.data_ptr(), a3s.data_ptr(),
                a4s.data_ptr(),
                bstat.data_ptr(), dU.data_ptr())
        ws = _workspace(dev, _memo(groups, ("ours_ws", B, H, Fd), lambda: int(
            _lib.fn("msha_ours_workspace_size")(gr, B, H, Fd))))
        _lib.call("msha_ours_intra_bwd", *args, 0, ctx.slope, ctx.p, ctx.seed, 0, G.data_ptr(),
                  bgrad.data_ptr(), row_coef.data_ptr(), da3s.data_ptr(), da4s.data_ptr(), None,
                  ws.data_ptr(), ws.numel(), s)
        E = max(graph.n_edges, 1)
        d_el = torch.empty(n, H, device=dev, dtype=torch.float32)
        d_hs = torch.empty(n, H, Fd, device=dev, dtype=dt)
        d_hc = torch.empty(m, H, Fd, device=dev, dtype=dt)
        d_er = torch.empty(m, H, device=dev, dtype=torch.float32)
        if ctx.bip:
            # row and column gradients of the inter attention in one pass; its d_hc / d_er
            # reduce runs inside the intra stage-1 launch (msha_bip_defer_reduce)
            ws = _bip_ws(graph, H, Fd, dev)
            defer = BIP_DEFER_REDUCE
            try:
                if defer:
                    _lib.call("msha_bip_defer_reduce", 1)
                _lib.call("msha_bip_attention_bwd", g, H, Fd, _code(dt), el.data_ptr(),
                          er.data_ptr(), h1.data_ptr(), lse.data_ptr(), dU.data_ptr(),
                          h2.data_ptr(), dV.data_ptr(), row_coef.data_ptr(), ctx.slope, ctx.p,
                          ctx.seed, 0, d_el.data_ptr(), d_er.data_ptr(), d_hc.data_ptr(),
                          d_hs.data_ptr(), ws.data_ptr(), ws.numel(), s)
                _lib.call("msha_ours_intra_bwd", *args, 1, ctx.slope, ctx.p, ctx.seed, 0,
                          G.data_ptr(), bgrad.data_ptr(), None, None, None, d_hs.data_ptr(),
                          None, 0, s)
            finally:
                if defer:
                    _lib.call("msha_bip_defer_reduce", 0)
            return d_el, d_er, d_hc, d_hs, da3s, da4s, None, None, None, None, None, None
        rec = torch.empty(E, 2, H, device=dev, dtype=torch.float32)  # (de, attd) per edge
        de, attd = rec[:, 0], rec[:, 1]
        _lib.call("msha_edge_attention_bwd_rows", g, H, Fd, _code(dt), el.data_ptr(), er.data_ptr(),
                  h1.data_ptr(), lse.data_ptr(), u_inter.data_ptr(), _lib.ptr(u_lo), dU.data_ptr(),
                  h2.data_ptr(), dV.data_ptr(), row_coef.data_ptr(), ctx.slope, ctx.p, ctx.seed,
                  0, d_el.data_ptr(), de.data_ptr(), attd.data_ptr(), 2 * H, d_hs.data_ptr(), s)
        _lib.call("msha_ours_intra_bwd", *args, 1, ctx.slope, ctx.p, ctx.seed, 0, G.data_ptr(),
                  bgrad.data_ptr(), None, None, None, d_hs.data_ptr(), None, 0, s)
        _csc_aggregate(graph, H, Fd, attd, de, dU, d_hc, d_er, s, ld=2 * H)
        return d_el, d_er, d_hc, d_hs, da3s, da4s, None, None, None, None, None, None


def ours_attention(graph: Graph, groups, src, el, er, h1, h2, a3s, a4s, p: float = 0.0,
                   training: bool = False, slope: float = NEG_SLOPE, seed: int | None = None,
                   return_aux: bool = False):
    """Full MSHA attention core (Ours.py:54-101): returns (u, v), u = inter + intra;
    with return_aux also (attd (E, H) post-dropout inter attention, bstat (B, H, 8))."""
    _lib.require_cuda(el, er, h1, h2, a3s, a4s, src)
    H, Fd = el.shape[1], h1.shape[-1]
    if not _lib.load().msha_edge_attention_supported(H, Fd):
        raise NotImplementedError(f"ours_attention: (heads={H}, feat={Fd}) not compiled")
    if H * Fd > 512:
        raise NotImplementedError("ours_attention: heads*feat must be <= 512")
    p = float(p) if training else 0.0
    if seed is None:
        seed = new_seed() if p > 0 else 0
    u, v, attd, bstat = _OursAttention.apply(el, er, h1, h2, a3s, a4s, graph, groups, src, p,
                                             seed, slope)
    return (u, v, attd, bstat) if return_aux else (u, v)


# ------------------------------------------------------------------ model head ---
HEAD_TAPS = None  # tests: a list here collects each model-head forward's inputs and statistics
def head_supported(graph: Graph, heads: int, feat: int) -> bool:
    return bool(_lib.load().msha_head_supported(graph.n_cols, heads, feat))


_HP_CACHE: dict = {}


def _head_params(H, F, eps, momentum, slope, ptrs, dyn=None):
    """msha_head_params from pointer lists: the ``ptrs`` part is built once per distinct
    set of pointers (the parameters and buffers stay put across steps) and copied; the
    ``dyn`` part (this call's gradient outputs) is written into the copy."""
    key = (H, F, eps, momentum, slope, tuple((k, None if v is None else tuple(v))
                                            for k, v in ptrs.items()))
    base = _HP_CACHE.get(key)
    if base is None:
        if len(_HP_CACHE) > 64:
            _HP_CACHE.clear()
        base = _lib.MshaHeadParams()
        base.heads, base.feat, base.eps, base.momentum, base.slope = H, F, eps, momentum, slope
        for name, lst in ptrs.items():
            arr = getattr(base, name)
            for h in range(len(lst) if lst is not None else H):
                arr[h] = lst[h] if lst is not None else None
        _HP_CACHE[key] = base
    hp = _lib.MshaHeadParams.from_buffer_copy(base)
    for name, lst in (dyn or {}).items():
        arr = getattr(hp, name)
        for h, v in enumerate(lst):
            arr[h] = v
    return hp


# the loss backward flags its gradient's nonzero rows for the model head's backward
# (msha_nll_rows_bwd_flags -> msha_head_bwd_flagged: one launch fewer per step);
# MSHA_NLL_FLAGS=0 keeps the head's own row scan (A/B).  HEAD_BWD_FLAGGED counts the head
# backwards that took the flags (tests).
NLL_FLAGS = os.environ.get("MSHA_NLL_FLAGS", "1") != "0"
HEAD_BWD_FLAGGED = [0]


class _ModelHead(torch.autograd.Function):
    """msha_head_fwd / msha_head_bwd: the heads' BatchNorm + LeakyReLU epilogues,
    elu(u_out @ v_out.T), cat, dropout, out_att (GraphAttentionLayer), elu, log_softmax
    (Ablation.py:273-277 + :298-301; Ours.py:100-109 + :163-167).  ``params``: the heads'
    bn2 (u side) weights, bn2 biases, bn1 (v side) weights, bn1 biases, then out_att.a."""

    @staticmethod
    def forward(ctx, u, v, W, graph: Graph, bns, training, eps, momentum, slope, px, sx, pa,
                sa, *params):
        N, H, F = u.shape
        M = graph.n_cols
        dt = _table_dtype(u, v)
        u, v = _tc(u, dt), _tc(v, dt)
        a_out = params[4 * H]
        dev = u.device
        s = _stream(u)
        # fp32 views of W, the BatchNorm affine parameters and running statistics: the
        # tensors themselves when fp32, else fp32 copies made in ONE cast launch (and the
        # updated running statistics cast back in one launch after the head)
        cast_in, cast_out = [], []

        def f32_of(t):
            if t.dtype == torch.float32 and t.is_contiguous():
                return t
            c = torch.empty(t.shape, device=t.device, dtype=torch.float32)
            cast_in.append((t.contiguous(), c))
            return c

        W32 = f32_of(W)
        p32 = [f32_of(p) for p in params[:4 * H]]  # held until the launches (see bn_lrelu)
        run = {}
        for side, k in (("u", 0), ("v", 1)):
            rm, rv = [], []
            for bu_bv in bns:
                bn = bu_bv[k]
                if training and bn.track_running_stats and bn.running_mean is not None:
                    for buf, lst in ((bn.running_mean, rm), (bn.running_var, rv)):
                        b32 = f32_of(buf)
                        if b32 is not buf:
                            cast_out.append((b32, buf))
                        lst.append(b32)
                elif not training:
                    rm.append(f32_of(bn.running_mean))
                    rv.append(f32_of(bn.running_var))
                else:
                    rm.append(None)
                    rv.append(None)
            run[side] = (rm, rv)
        _cast_many(cast_in, s)
        ptr = lambda lst: [_lib.ptr(t) for t in lst]  # noqa: E731
        hp = _head_params(H, F, eps, momentum, slope, {
            "u_weight": ptr(p32[0:H]), "u_bias": ptr(p32[H:2 * H]),
            "u_running_mean": ptr(run["u"][0]), "u_running_var": ptr(run["u"][1]),
            "v_weight": ptr(p32[2 * H:3 * H]), "v_bias": ptr(p32[3 * H:4 * H]),
            "v_running_mean": ptr(run["v"][0]), "v_running_var": ptr(run["v"][1]),
            # the kernel advances the BatchNorms' step counters (nn.BatchNorm1d's +1)
            "num_batches_tracked": [
                _lib.ptr(bn.num_batches_tracked)
                if training and bn.track_running_stats and bn.num_batches_tracked is not None
                and bn.num_batches_tracked.is_cuda else None
                for pair in bns for bn in pair]})
        stats = torch.empty(4 * H * F + H * F * M, device=dev, dtype=torch.float32)
        out = torch.empty(N, M, device=dev, dtype=dt)
        g = graph.desc
        ws = _workspace(dev, _memo(graph, ("head_ws", H, F), lambda: int(
            _lib.fn("msha_head_workspace_size")(g, H, F))) if training else 0)
        _lib.call("msha_head_fwd", g, C_byref(hp), _code(dt), u.data_ptr(), v.data_ptr(),
                  W32.data_ptr(), int(training), px, sx, pa, sa, stats.data_ptr(),
                  out.data_ptr(), ws.data_ptr(), ws.numel(), s)
        if HEAD_TAPS is not None:  # tests: the statistics that decide the LeakyReLU branches
            HEAD_TAPS.append({"u": u.detach().clone(), "v": v.detach().clone(),
                              "stats": stats.detach().clone(),
                              "params": [p.detach().clone() for p in p32]})
        _cast_many(cast_out, s)  # non-fp32 running buffers: write the update back
        ctx.graph, ctx.hpar = graph, (H, F, eps, momentum, slope)
        ctx.drop = (px, sx, pa, sa)
        ctx.pdtypes = [p.dtype for p in params[:4 * H]]
        ctx.wdtype = W.dtype
        ctx.a_meta = (a_out.shape, a_out.dtype, a_out.device)
        ctx.save_for_backward(u, v, W32, stats, *p32)
        return out

    @staticmethod
    def backward(ctx, dout):
        u, v, W32, stats, *p32 = ctx.saved_tensors
        H, F, eps, momentum, slope = ctx.hpar
        px, sx, pa, sa = ctx.drop
        graph = ctx.graph
        dev = u.device
        dt = u.dtype
        dout = _tc(dout, dt)
        flags = getattr(dout, "_msha_rowflags", None)  # from _NllRows.backward, if dout is its d
        if flags is not None and (flags[1] != dout.shape[0] or not dout.is_contiguous()):
            flags = None
        du = torch.empty_like(u)
        dv = torch.empty_like(v)
        dW = torch.empty_like(W32)
        dp = torch.empty(4, H, F, device=dev, dtype=torch.float32)
        ptr = lambda lst: [_lib.ptr(t) for t in lst]  # noqa: E731
        base = dp.data_ptr()
        step = 4 * F  # dp (4, H, F): gradient k of head h at base + 4 (k H + h) F
        hp = _head_params(H, F, eps, momentum, slope, {
            "u_weight": ptr(p32[0:H]), "u_bias": ptr(p32[H:2 * H]),
            "v_weight": ptr(p32[2 * H:3 * H]), "v_bias": ptr(p32[3 * H:4 * H]),
            "u_running_mean": None, "u_running_var": None, "v_running_mean": None,
            "v_running_var": None}, dyn={
            name: [base + step * (k * H + h) for h in range(H)]
            for k, name in enumerate(("du_weight", "du_bias", "dv_weight", "dv_bias"))})
        g = graph.desc
        ws = _workspace(dev, _memo(graph, ("head_ws", H, F), lambda: int(
            _lib.fn("msha_head_workspace_size")(g, H, F))))
        shape, adt, adev = ctx.a_meta
        da = torch.empty(shape, dtype=torch.float32, device=adev)  # zeroed by the reduce
        if flags is not None:
            fl, n = flags
            nw = (n + 63) // 64
            HEAD_BWD_FLAGGED[0] += 1
            _lib.call("msha_head_bwd_flagged", g, C_byref(hp), _code(dt), u.data_ptr(),
                      v.data_ptr(), W32.data_ptr(), px, sx, pa, sa, stats.data_ptr(),
                      dout.data_ptr(), fl.data_ptr() + 8 * nw, fl.data_ptr(), du.data_ptr(),
                      dv.data_ptr(), dW.data_ptr(), da.data_ptr(), da.numel(), ws.data_ptr(),
                      ws.numel(), _stream(u))
        else:
            _lib.call("msha_head_bwd", g, C_byref(hp), _code(dt), u.data_ptr(), v.data_ptr(),
                      W32.data_ptr(), px, sx, pa, sa, stats.data_ptr(), dout.data_ptr(),
                      du.data_ptr(), dv.data_ptr(), dW.data_ptr(), da.data_ptr(), da.numel(),
                      ws.data_ptr(), ws.numel(), _stream(u))
        # gradients in the parameters' dtypes: one cast launch for every non-fp32 one
        casts = []

        def as_dtype(g, dtype):
            if g.dtype == dtype:
                return g
            c = torch.empty(g.shape, device=g.device, dtype=dtype)
            casts.append((g, c))
            return c

        grads = [as_dtype(dp[k, h], ctx.pdtypes[k * H + h]) for k in range(4) for h in range(H)]
        dW, da = as_dtype(dW, ctx.wdtype), as_dtype(da, adt)
        _cast_many(casts, _stream(u))
        return (du, dv, dW, None, None, None, None, None, None, None, None, None,
                None, *grads, da)


def C_byref(x):
    import ctypes

    return ctypes.byref(x)


def model_head(graph: Graph, u, v, bns, out_W, out_a, p: float = 0.0, training: bool = False,
               slope: float = 0.2):
    """log_softmax(elu(out_att(dropout(cat_h elu(lrelu(bn2_h(u_h)) @ lrelu(bn1_h(v_h)).T)))))
    for the (N, H, F) / (M, H, F) attention aggregates u, v; ``bns``: per head (bn2, bn1)
    BatchNorm1d modules (u side, v side).  Training: batch statistics (running
    statistics and num_batches_tracked advanced as nn.BatchNorm1d), dropout p on x and on
    the out_att attention; eval: running statistics."""
    _lib.require_cuda(u, v, out_W)
    N, H, F = u.shape
    bn0 = bns[0][0]
    params = ([b[0].weight for b in bns] + [b[0].bias for b in bns] + [b[1].weight for b in bns]
              + [b[1].bias for b in bns] + [out_a])
    if not training:
        # msha_head_bwd differentiates the training-mode BatchNorm (batch statistics);
        # eval normalises with the running statistics, whose backward it does not have
        if torch.is_grad_enabled() and any(t is not None and t.requires_grad
                                           for t in (u, v, out_W, *params)):
            raise NotImplementedError(
                "model_head: gradients through eval-mode BatchNorm (running statistics) are "
                "not implemented; call it under torch.no_grad() or use the unfused tail")
        if any(bn.running_mean is None or bn.running_var is None for pair in bns for bn in pair):
            raise ValueError("model_head: eval needs running statistics "
                             "(BatchNorm1d(track_running_stats=True))")
    px = pa = float(p) if training else 0.0
    sx = new_seed() if px > 0 else 0
    sa = new_seed() if pa > 0 else 0
    return _ModelHead.apply(u, v, out_W, graph, bns, bool(training), float(bn0.eps),
                            float(bn0.momentum), float(slope), px, sx, pa, sa, *params)


# ------------------------------------------------- parameter packing / feature dropout ---
_SEG_FMT = struct.Struct("<QQQqqqqqf4xQQii")  # struct msha_segment (checked at import)
assert _SEG_FMT.size == ctypes.sizeof(_lib.MshaSegment)


def _segments(segs, stream):
    """msha_segments launches: segs = [(a, dst, rows, cols, lda, ldd, b, ldb, p, seed
    [, a_dtype, dst_dtype])] (pointers as ints, a / b may be None; dtypes as torch dtypes,
    fp32 when omitted), MSHA_MAX_SEGMENTS per launch.  The records are packed bytes
    (one struct.pack_into each) viewed as the ctypes array."""
    for lo in range(0, len(segs), _lib.MAX_SEGMENTS):
        part = segs[lo:lo + _lib.MAX_SEGMENTS]
        buf = bytearray(_SEG_FMT.size * len(part))
        for k, sg in enumerate(part):
            a, dst, rows, cols, lda, ldd, b, ldb, p, seed = sg[:10]
            adt, ddt = (sg[10], sg[11]) if len(sg) > 10 else (torch.float32, torch.float32)
            _SEG_FMT.pack_into(buf, k * _SEG_FMT.size, a or 0, b or 0, dst, rows, cols, lda,
                               ldb, ldd, p, seed, 0, 1 if adt == BF16 else 0,
                               1 if ddt == BF16 else 0)
        arr = (_lib.MshaSegment * len(part)).from_buffer(buf)
        _lib.call("msha_segments", len(part), C_byref(arr), stream)


def _cast_segs(pairs):
    """Segments writing dst = src (cast to dst's dtype) for contiguous same-numel pairs."""
    return [(a.data_ptr(), d.data_ptr(), 1, a.numel(), a.numel(), a.numel(), None, 0, 0.0, 0,
             a.dtype, d.dtype) for a, d in pairs if a.numel() > 0]


def _cast_many(pairs, stream):
    """Every (src, dst) pair of contiguous same-numel tensors copied with a dtype cast in
    one launch (the bf16 models' small parameters, gradients and BatchNorm buffers: one
    launch where ``.to(dtype)`` issued one per tensor)."""
    segs = _cast_segs(pairs)
    if segs:
        _segments(segs, stream)


def _fd_fwd(S, R, p, s_seed, r_seed):
    """Segments + outputs of dropout(S), dropout(R) (one Philox mask each)."""
    S, R = S.contiguous(), R.contiguous()
    So, Ro = torch.empty_like(S), torch.empty_like(R)
    segs = [(S.data_ptr(), So.data_ptr(), S.shape[0], S.shape[1], S.shape[1], S.shape[1],
             None, 0, p, s_seed, S.dtype, S.dtype),
            (R.data_ptr(), Ro.data_ptr(), R.shape[0], R.shape[1], R.shape[1], R.shape[1],
             None, 0, p, r_seed, R.dtype, R.dtype)]
    return segs, So, Ro


def _fd_bwd(leaves, grads, p, seeds, needs):
    """Segments + gradients of the two feature dropouts (the masks regenerated).  A leaf
    registered with ``optim.Adam.fuse_dropout_grad`` gets no gradient: its optimizer step
    reads the output gradient and the mask seed instead."""
    from .optim import fused_optimizer_of

    segs, outs = [], []
    for k, (d, seed) in enumerate(zip(grads, seeds)):
        leaf = leaves[k]
        opt = fused_optimizer_of(leaf) if d is not None else None
        if opt is not None and needs[k]:
            opt.stash_dropout_grad(leaf, d, p, seed)
            d = None
        if d is None:
            outs.append(None)
            continue
        d = d.contiguous()
        g = torch.empty_like(d)
        segs.append((d.data_ptr(), g.data_ptr(), d.shape[0], d.shape[1], d.shape[1],
                     d.shape[1], None, 0, p, seed, d.dtype, d.dtype))
        outs.append(g)
    return segs, outs


class _FeatureDropout(torch.autograd.Function):
    """dropout(Sfeatures), dropout(Rfeatures) (Ablation.py:296-297, Ours.py:161-162) in one
    launch; the backward regenerates both Philox masks in one launch.  A table registered
    with ``optim.Adam.fuse_dropout_grad`` gets no gradient: the backward hands the
    dropout's output gradient and mask seed to that optimizer, whose step reads them."""

    @staticmethod
    def forward(ctx, S, R, p, s_seed, r_seed):
        ctx.params = (S, R)  # the leaves themselves (a fused optimizer updates them)
        segs, So, Ro = _fd_fwd(S, R, p, s_seed, r_seed)
        _segments(segs, _stream(S))
        ctx.p, ctx.seeds = p, (s_seed, r_seed)
        return So, Ro

    @staticmethod
    def backward(ctx, dSo, dRo):
        segs, outs = _fd_bwd(ctx.params, (dSo, dRo), ctx.p, ctx.seeds, ctx.needs_input_grad)
        if segs:
            _segments(segs, _stream(outs[0] if outs[0] is not None else outs[1]))
        return outs[0], outs[1], None, None, None


def feature_dropout(S, R, p: float, training: bool):
    """(dropout(S, p), dropout(R, p)) for the models' two feature tables: one launch each
    way for fp32 / bf16 tables (Philox masks, seeds from torch's CPU generator; bf16
    outputs rounded once from the fp32 product), F.dropout otherwise."""
    if not training or p <= 0:
        return S, R
    if not _fd_ok(S, R):
        return (torch.nn.functional.dropout(S, p, training=True),
                torch.nn.functional.dropout(R, p, training=True))
    _lib.require_cuda(S, R)
    return _FeatureDropout.apply(S, R, float(p), new_seed(), new_seed())


def _fd_ok(S, R):
    ok = (torch.float32, BF16)
    return S.dtype in ok and R.dtype in ok and S.dim() == 2 and R.dim() == 2


def _ph_fwd(H, intra, params):
    """Segments + outputs of the head packing: W1 / W2 (K, H*F) in the parameters' dtype,
    a_r / a_l (H, F) fp32 [, a3s, a4s = a3[:F] + a3[F:], a4[:F] + a4[F:]]."""
    W1s, W2s, As = params[:H], params[H:2 * H], params[2 * H:3 * H]
    K, Fd = W1s[0].shape
    dev = W1s[0].device
    pdt = W1s[0].dtype
    es = W1s[0].element_size()
    W1 = torch.empty(K, H * Fd, device=dev, dtype=pdt)
    W2 = torch.empty(K, H * Fd, device=dev, dtype=pdt)
    ar = torch.empty(H, Fd, device=dev)
    al = torch.empty(H, Fd, device=dev)
    outs = [W1, W2, ar, al]
    f32 = torch.float32
    segs = []
    w1p, w2p, arp, alp = W1.data_ptr(), W2.data_ptr(), ar.data_ptr(), al.data_ptr()
    for h in range(H):
        segs.append((W1s[h].data_ptr(), w1p + es * h * Fd, K, Fd, Fd, H * Fd, None, 0, 0.0, 0,
                     pdt, pdt))
        segs.append((W2s[h].data_ptr(), w2p + es * h * Fd, K, Fd, Fd, H * Fd, None, 0, 0.0, 0,
                     pdt, pdt))
        pa = As[h].data_ptr()
        segs.append((pa, arp + 4 * h * Fd, 1, Fd, Fd, Fd, None, 0, 0.0, 0, pdt, f32))
        segs.append((pa + es * Fd, alp + 4 * h * Fd, 1, Fd, Fd, Fd, None, 0, 0.0, 0, pdt, f32))
    if intra:
        a3s = torch.empty(H, Fd, device=dev)
        a4s = torch.empty(H, Fd, device=dev)
        outs += [a3s, a4s]
        for h in range(H):
            for src, dst in ((params[3 * H + h], a3s), (params[4 * H + h], a4s)):
                pa = src.data_ptr()
                segs.append((pa, dst.data_ptr() + 4 * h * Fd, 1, Fd, Fd, Fd, pa + es * Fd, Fd,
                             0.0, 0, pdt, f32))
    return segs, outs, (H, intra, K, Fd, pdt)


def _ph_bwd(meta, dW1, dW2, dar, dal, da3s=None, da4s=None):
    """Segments + per-head parameter gradients of the head packing (cast to the
    parameters' dtype); a missing packed gradient writes zeros."""
    H, intra, K, Fd, pdt = meta
    some = next(t for t in (dW1, dW2, dar, dal, da3s, da4s) if t is not None)
    dev = some.device
    c = lambda t: None if t is None else t.contiguous()  # noqa: E731
    dW1, dW2, dar, dal, da3s, da4s = map(c, (dW1, dW2, dar, dal, da3s, da4s))
    # a missing gradient writes zeros (NULL a); its dtype code is then irrelevant
    dty = lambda t: pdt if t is None else t.dtype  # noqa: E731
    ptr = lambda t, off=0: None if t is None else t.data_ptr() + off * t.element_size()  # noqa: E731
    gW1 = [torch.empty(K, Fd, device=dev, dtype=pdt) for _ in range(H)]
    gW2 = [torch.empty(K, Fd, device=dev, dtype=pdt) for _ in range(H)]
    gA = [torch.empty(2 * Fd, 1, device=dev, dtype=pdt) for _ in range(H)]
    ge = gA[0].element_size()
    segs = []
    for h in range(H):
        o = h * Fd
        segs.append((ptr(dW1, o), gW1[h].data_ptr(), K, Fd, H * Fd, Fd, None, 0, 0.0, 0,
                     dty(dW1), pdt))
        segs.append((ptr(dW2, o), gW2[h].data_ptr(), K, Fd, H * Fd, Fd, None, 0, 0.0, 0,
                     dty(dW2), pdt))
        segs.append((ptr(dar, o), gA[h].data_ptr(), 1, Fd, Fd, Fd, None, 0, 0.0, 0,
                     dty(dar), pdt))
        segs.append((ptr(dal, o), gA[h].data_ptr() + ge * Fd, 1, Fd, Fd, Fd, None, 0, 0.0, 0,
                     dty(dal), pdt))
    g3 = g4 = []
    if intra:
        g3 = [torch.empty(2 * Fd, 1, device=dev, dtype=pdt) for _ in range(H)]
        g4 = [torch.empty(2 * Fd, 1, device=dev, dtype=pdt) for _ in range(H)]
        for h in range(H):
            o = h * Fd
            for d, g in ((da3s, g3[h]), (da4s, g4[h])):  # sum backward: both halves
                segs.append((ptr(d, o), g.data_ptr(), 1, Fd, Fd, Fd, None, 0, 0.0, 0,
                             dty(d), pdt))
                segs.append((ptr(d, o), g.data_ptr() + ge * Fd, 1, Fd, Fd, Fd, None, 0, 0.0,
                             0, dty(d), pdt))
    return segs, [*gW1, *gW2, *gA, *g3, *g4], dev


class _PackHeads(torch.autograd.Function):
    """The heads' parameters as the fused launches read them (Ablation.py:262-267,
    Ours.py:58-75): W1 / W2 concatenated along features (K, H*F) in the parameters'
    dtype, the score vector halves a[:F] (recipient side) / a[F:] (source side) as fp32
    (H, F), and for the full MSHA layer a3[:F] + a3[F:], a4[:F] + a4[F:] -- one launch;
    the backward scatters the packed gradients to every head's parameters (cast to their
    dtype) in one launch.  fp32 or bf16 parameters (the scores are fp32 either way)."""

    @staticmethod
    def forward(ctx, H, intra, *params):
        segs, outs, ctx.meta = _ph_fwd(H, intra, params)
        _segments(segs, _stream(outs[0]))
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        segs, gs, dev = _ph_bwd(ctx.meta, *grads)
        _segments(segs, _lib.stream_handle(dev))
        return (None, None, *gs)


def _pack_params(heads, intra):
    names = ["W1", "W2", "a"] + (["a3", "a4"] if intra else [])
    return [getattr(h, n) for n in names for h in heads]


def _ph_ok(H, params):
    pdt = params[0].dtype
    return H <= 4 and pdt in (torch.float32, BF16) and all(
        p.dtype == pdt and p.is_contiguous() and p.is_cuda for p in params)


def pack_heads(heads, intra: bool):
    """(W1 (K, H*F), W2, a_r (H, F), a_l (H, F)[, a3s, a4s]) of the heads' parameters, or
    None when the one-launch packing does not apply (mixed or non-fp32/bf16 dtypes,
    non-contiguous parameters, more than 4 heads)."""
    H = len(heads)
    params = _pack_params(heads, intra)
    if not _ph_ok(H, params):
        return None
    return _PackHeads.apply(H, intra, *params)


class _Prologue(torch.autograd.Function):
    """feature_dropout + pack_heads as ONE launch each way (and one autograd node): the
    models' step starts with both (Ablation.py:296-297 + :262-267, Ours.py:161-162 +
    :58-75) and their segments fit one msha_segments batch."""

    @staticmethod
    def forward(ctx, p, s_seed, r_seed, H, intra, S, R, *params):
        ctx.leaves = (S, R)
        fsegs, So, Ro = _fd_fwd(S, R, p, s_seed, r_seed)
        psegs, outs, ctx.meta = _ph_fwd(H, intra, params)
        _segments(fsegs + psegs, _stream(So))
        ctx.p, ctx.seeds = p, (s_seed, r_seed)
        return (So, Ro, *outs)

    @staticmethod
    def backward(ctx, dSo, dRo, *dpacked):
        fsegs, fouts = _fd_bwd(ctx.leaves, (dSo, dRo), ctx.p, ctx.seeds,
                               ctx.needs_input_grad[5:7])
        if any(d is not None for d in dpacked):
            psegs, gs, dev = _ph_bwd(ctx.meta, *dpacked)
        else:
            psegs, gs = [], [None] * (len(ctx.needs_input_grad) - 7)
        if fsegs or psegs:
            dev = next(t for t in (*fouts, *gs) if t is not None).device
            _segments(fsegs + psegs, _lib.stream_handle(dev))
        return (None, None, None, None, None, fouts[0], fouts[1], *gs)


def model_prologue(S, R, p: float, training: bool, heads, intra: bool):
    """(dropout(S), dropout(R), packed heads) -- feature_dropout and pack_heads in one
    launch each way when both apply (training with dropout, packable heads); otherwise
    the two separately (packed None where pack_heads does not apply)."""
    H = len(heads)
    params = _pack_params(heads, intra)
    if training and p > 0 and _fd_ok(S, R) and _ph_ok(H, params):
        _lib.require_cuda(S, R)
        outs = _Prologue.apply(float(p), new_seed(), new_seed(), H, intra, S, R, *params)
        return outs[0], outs[1], tuple(outs[2:])
    s_in, r_in = feature_dropout(S, R, p, training)
    return s_in, r_in, pack_heads(heads, intra)


# ------------------------------------------------------------- loss on gathered rows ---
class _NllRows(torch.autograd.Function):
    """F.nll_loss(logp[rows], cols) (mean) and its backward, one launch each
    (msha_nll_rows_fwd / _bwd): replaces the row gather, nll forward/backward, the zero
    fill of the (N, M) gradient and the index backward of train.py:227-229."""

    @staticmethod
    def forward(ctx, logp, rows, cols):
        dt = _table_dtype(logp)
        logp = _tc(logp, dt)
        rows = rows.to(torch.int64).contiguous()
        cols = cols.to(torch.int64).contiguous()
        loss = torch.empty((), device=logp.device, dtype=torch.float32)
        _lib.call("msha_nll_rows_fwd", logp.shape[0], logp.shape[1], rows.numel(),
                  rows.data_ptr(), cols.data_ptr(), _code(dt), logp.data_ptr(), logp.stride(0),
                  loss.data_ptr(), _stream(logp))
        ctx.save_for_backward(rows, cols)
        ctx.shape, ctx.dt = tuple(logp.shape), dt
        return loss

    @staticmethod
    def backward(ctx, gloss):
        rows, cols = ctx.saved_tensors
        N, M = ctx.shape
        g = _f32c(gloss.reshape(1))
        d = torch.empty(N, M, device=rows.device, dtype=ctx.dt)
        if NLL_FLAGS:
            # the rows of d with a nonzero, flagged here for the model head's backward (its
            # consumer in every model): msha_head_bwd_flagged then skips its own row scan
            nw = (N + 63) // 64
            fl = torch.empty(8 * nw + N, device=rows.device, dtype=torch.uint8)
            _lib.call("msha_nll_rows_bwd_flags", N, M, rows.numel(), rows.data_ptr(),
                      cols.data_ptr(), g.data_ptr(), _code(ctx.dt), d.data_ptr(), M,
                      fl.data_ptr() + 8 * nw, fl.data_ptr(), _stream(d))
            d._msha_rowflags = (fl, N)
        else:
            _lib.call("msha_nll_rows_bwd", N, M, rows.numel(), rows.data_ptr(), cols.data_ptr(),
                      g.data_ptr(), _code(ctx.dt), d.data_ptr(), M, _stream(d))
        return d, None, None


def nll_loss_rows(logp, rows, cols):
    """``F.nll_loss(logp[rows].float(), cols)`` (mean reduction) for the (N, M) log-probs
    of a model head, train.py:227-229's loss, as one launch forward and one backward."""
    _lib.require_cuda(logp, rows, cols)
    if logp.dim() != 2 or rows.shape != cols.shape:
        raise ValueError("nll_loss_rows: logp (N, M), rows and cols of the same length")
    return _NllRows.apply(logp, rows, cols)
