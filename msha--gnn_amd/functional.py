"""Autograd functions over the HIP kernels (include/msha_gnn.h).

``edge_attention``       Ablation.py:266-274 (OursLayer3 inter attention: scores,
                         masked softmax, dropout, u = att @ h1 and, optionally,
                         v = att.T @ h2), forward AND backward on the GPU.
``gal``                  GAT.py:20-35 GraphAttentionLayer row scale (after x @ W).
``dropout_keep_mask``    the Philox mask the kernels draw (for tests / oracles).
"""
from __future__ import annotations

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


def new_seed() -> int:
    """Per-call dropout seed drawn from torch's CPU generator (no device sync;
    reproducible under torch.manual_seed)."""
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


def _stream(t):
    return _lib.stream_handle(t.device)


class _EdgeAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, el, er, hc, hs, graph: Graph, p: float, seed: int, slope: float):
        n, H = el.shape
        m, H2, F = hc.shape
        assert H2 == H and m == graph.n_cols and n == graph.n_rows
        el, er, hc = _f32c(el), _f32c(er), _f32c(hc)
        hs = _f32c(hs)
        dev = el.device
        s = _stream(el)
        g = graph.desc
        u = torch.empty(n, H, F, device=dev, dtype=torch.float32)
        lse = torch.empty(n, H, device=dev, dtype=torch.float32)
        attd = None
        if hs is not None:
            attd = torch.empty(max(graph.n_edges, 1), H, device=dev, dtype=torch.float32)
        ev = _timed("edge_attention_fwd")
        _lib.call("msha_edge_attention_fwd", g, H, F, el.data_ptr(), er.data_ptr(),
                  hc.data_ptr(), slope, p, seed, 0, u.data_ptr(), lse.data_ptr(),
                  _lib.ptr(attd), s)
        if ev is not None:
            ev[1].record()
        v = None
        if hs is not None:
            v = torch.empty(m, H, F, device=dev, dtype=torch.float32)
            _csc_aggregate(graph, H, F, attd, None, hs, v, None, s)
        ctx.graph, ctx.p, ctx.seed, ctx.slope = graph, p, seed, slope
        ctx.has_hs = hs is not None
        ctx.save_for_backward(el, er, hc, hs if hs is not None else el.new_empty(0), lse, u)
        if v is None:
            return u
        return u, v

    @staticmethod
    def backward(ctx, dU, dV=None):
        el, er, hc, hs, lse, u = ctx.saved_tensors
        graph = ctx.graph
        n, H = el.shape
        m, _, F = hc.shape
        dev = el.device
        s = _stream(el)
        g = graph.desc
        dU = torch.zeros_like(u) if dU is None else _f32c(dU)
        use_dv = ctx.has_hs and dV is not None
        dV = _f32c(dV) if use_dv else None
        E = max(graph.n_edges, 1)
        d_el = torch.empty(n, H, device=dev, dtype=torch.float32)
        de = torch.empty(E, H, device=dev, dtype=torch.float32)
        attd = torch.empty(E, H, device=dev, dtype=torch.float32)
        d_hs = torch.empty(n, H, F, device=dev, dtype=torch.float32) if use_dv else None
        _lib.call("msha_edge_attention_bwd_rows", g, H, F, el.data_ptr(), er.data_ptr(),
                  hc.data_ptr(), lse.data_ptr(), u.data_ptr(), dU.data_ptr(),
                  hs.data_ptr() if use_dv else None, _lib.ptr(dV), ctx.slope, ctx.p, ctx.seed, 0,
                  d_el.data_ptr(), de.data_ptr(), attd.data_ptr(), _lib.ptr(d_hs), s)
        d_hc = torch.empty(m, H, F, device=dev, dtype=torch.float32)
        d_er = torch.empty(m, H, device=dev, dtype=torch.float32)
        _csc_aggregate(graph, H, F, attd, de, dU, d_hc, d_er, s)
        if ctx.has_hs and d_hs is None:
            d_hs = torch.zeros_like(hs)
        return d_el, d_er, d_hc, (d_hs if ctx.has_hs else None), None, None, None, None


def _csc_aggregate(graph: Graph, H, F, w, x, table, out, out_x, stream):
    if not graph.has_csc:
        raise RuntimeError("graph has no CSC view (build it with_csc=True)")
    g = graph.desc
    wsb = _lib.load().msha_csc_aggregate_workspace_size(g, H, F)
    ws = None
    if graph._plan["n_multi"] > 0:
        ws = torch.empty(int(wsb), dtype=torch.uint8, device=table.device)
    _lib.call("msha_csc_aggregate", g, H, F, w.data_ptr(), _lib.ptr(x), table.data_ptr(),
              out.data_ptr(), _lib.ptr(out_x), _lib.ptr(ws), 0 if ws is None else ws.numel(),
              stream)


def edge_attention(graph: Graph, el, er, hc, hs=None, p: float = 0.0, training: bool = False,
                   slope: float = NEG_SLOPE, seed: int | None = None):
    """Fused masked edge-softmax + aggregation.

    el (N,H), er (M,H), hc (M,H,F) [, hs (N,H,F)] ->  u (N,H,F)  [, v (M,H,F)]
    with att = softmax_row(lrelu(el_i + er_j)), u = drop(att) @ hc, v = drop(att).T @ hs.
    """
    _lib.require_cuda(el, er, hc, hs)
    F = hc.shape[-1]
    H = el.shape[1]
    if not _lib.load().msha_edge_attention_supported(H, F):
        raise NotImplementedError(f"edge_attention: (heads={H}, feat={F}) not compiled")
    p = float(p) if training else 0.0
    if seed is None:
        seed = new_seed() if p > 0 else 0
    return _EdgeAttention.apply(el, er, hc, hs, graph, p, seed, slope)


class _GAL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, a, graph: Graph, p: float, seed: int):
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
        return dh, da, None, None, None


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


def dropout_keep_mask(n: int, p: float, seed: int, device, offset: int = 0) -> torch.Tensor:
    keep = torch.empty(n, dtype=torch.uint8, device=device)
    _lib.call("msha_dropout_keep_mask", seed, offset, n, p, keep.data_ptr(),
              _lib.stream_handle(device))
    return keep
