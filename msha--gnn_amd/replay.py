"""Per-model HIP-graph replay of the drop-in models' training forward and backward.

``train.py`` as written (train.py:221-232) runs the model eagerly every iteration:
torch's Adam, ``F.nll_loss(output[source_index], ...)``, ``loss.item()``.  The GPU work of
one ablation3 / Ours iteration is ~0.3-0.4 ms, but ~40 library launches issued from
Python around ~30 autograd nodes cost more than that on the host.  Here the model's
whole training forward is captured ONCE into a HIP graph (torch.cuda.CUDAGraph on a
side stream, static batch buffer), its whole backward into a second graph (static
output-gradient buffer, the parameters' gradients into static buffers), and every
later call is one autograd node whose forward is a 512-byte batch copy + one graph
replay and whose backward is one output-gradient copy + one replay.  train.py's own
statements (the loss, ``.item()``, torch's Adam) run unchanged around it.

* Dropout stays fresh: the library draws its Philox masks at (seed, offset + counter
  << 32); the model's own device counter is installed while its graphs are captured
  (so the captured launches read it) and incremented as the forward graph's first node.
  The backward graph reads the same counter value, so it regenerates the forward's
  masks (include/msha_gnn.h, msha_set_rng_counter).
* The untimed warm-up passes that settle the caches before capture would also move the
  BatchNorm running statistics; those buffers are restored before the first replay, so
  the statistics see exactly one update per iteration, as in the eager model.
* Gradients come back as the static buffers (no copies), written to the parameters'
  ``.grad`` by the node's backward itself: with ``zero_grad()`` setting ``.grad`` to None
  (torch's default, train.py:226) ``.grad`` becomes an alias of the static buffer, as the
  AccumulateGrad nodes of ``torch.cuda.make_graphed_callables`` adopt theirs; an existing
  ``.grad`` is added to.  Accumulation keeps torch's semantics: a ``.grad`` that still
  aliases the static buffer when the next forward or backward replays (two ``backward()``
  calls without ``zero_grad()``, or ``zero_grad(set_to_none=False)``) is first moved to a
  fresh tensor -- the forward graph shares the backward graph's memory pool, so its
  replay would overwrite the buffer -- and the replayed gradient is added to it.  With
  ``zero_grad()`` (set to None) before each forward, as train.py does, no copy is made.  The parameters are not inputs of the
  node, so the engine runs no AccumulateGrad node per parameter (~20 per model: ~0.1 ms
  of host time per backward); one anchor leaf makes the output require grad.  Parameter
  hooks (``register_hook`` / post-accumulate hooks) do not fire on this path.
* The forward hands back a fresh copy of the graph's static output, so an output held
  across iterations keeps its values.  The graph's saved activations serve one pending
  backward at a time: a forward whose graph still has a live, un-run backward (two
  forwards before one ``backward()``) runs the eager path instead, and a backward of an
  output whose graph has replayed a newer forward since raises instead of replaying on
  the newer activations.
* Not replayed (the eager path runs): eval mode, no grad mode, record mode, an outer
  graph capture (``step.GraphedStep``), a parameter registered with
  ``optim.Adam.fuse_dropout_grad``, or ``MSHA_MODEL_REPLAY=0``.
"""
from __future__ import annotations

import os
import weakref
from collections import OrderedDict

import torch

from . import functional as MF

REPLAY = os.environ.get("MSHA_MODEL_REPLAY", "1") != "0"
WARMUP = 2  # eager passes on the side stream before capture (graph views, workspaces)
MAX_GRAPHS = 4  # per model: batch sizes / adjacency versions kept


def eligible(model, source_index) -> bool:
    """Cheap per-call checks; the parameters' fused-optimizer marks are checked when a
    graph is captured (``run`` falls back to the eager forward then)."""
    return bool(REPLAY and model.training and torch.is_grad_enabled()
                and isinstance(source_index, torch.Tensor) and source_index.is_cuda
                and not torch.cuda.is_current_stream_capturing())


class _ModelGraphs:
    """The captured forward / backward of one (model, adjacencies, batch shape)."""

    def __init__(self, fwd, params, buffers, src, keep):
        dev = src.device
        self.params = params
        self.gen = 0  # forward replays so far; a backward replays only the newest
        self.pending = None  # weakref to the newest forward's autograd node until its backward
        self.keep = keep  # the adjacencies the captured launches read: kept alive
        self.src = src.detach().clone()
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        snaps = [b.detach().clone() for b in buffers]
        prev = MF.set_rng_counter(self.counter, dev.index)
        try:
            cur = torch.cuda.current_stream(dev)
            side = torch.cuda.Stream(dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                for _ in range(WARMUP):
                    self.counter.add_(1)
                    out = fwd(self.src)
                    torch.autograd.grad(out, params, torch.zeros_like(out), allow_unused=True)
                    del out
            cur.wait_stream(side)
            for b, s in zip(buffers, snaps):  # undo the warm-ups' BatchNorm updates
                b.copy_(s)
            self.fwd = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.fwd):
                self.counter.add_(1)
                self.out = fwd(self.src)
            self.dout = torch.empty_like(self.out)
            self.bwd = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.bwd, pool=self.fwd.pool()):
                self.grads = torch.autograd.grad(self.out, params, self.dout, allow_unused=True)
        finally:
            MF.set_rng_counter(prev, dev.index)
        self.out = self.out.detach()


class _Replay(torch.autograd.Function):
    @staticmethod
    def forward(ctx, graphs, src, anchor):
        # the forward graph reuses the pool the backward graph's gradient buffers live in:
        # a .grad still aliasing one of them (kept across iterations, no zero_grad) is
        # moved out first, or the replay would overwrite it
        for p, gr in zip(graphs.params, graphs.grads):
            cur = p.grad
            if gr is not None and cur is not None and cur.data_ptr() == gr.data_ptr():
                p.grad = cur.clone()
        graphs.src.copy_(src)
        graphs.fwd.replay()
        graphs.gen += 1
        graphs.pending = weakref.ref(ctx)
        ctx.graphs, ctx.gen = graphs, graphs.gen
        return graphs.out.clone()

    @staticmethod
    def backward(ctx, dout):
        g = ctx.graphs
        if ctx.gen != g.gen:
            raise RuntimeError(
                "msha replay: backward of a model output whose captured graph has replayed a "
                "newer forward since; run the backward before the next training forward, or "
                "set MSHA_MODEL_REPLAY=0")
        # a .grad still aliasing its static buffer holds an earlier gradient that the
        # replay would overwrite: move it out, then accumulate as torch would
        for p, gr in zip(g.params, g.grads):
            cur = p.grad
            if gr is not None and cur is not None and cur.data_ptr() == gr.data_ptr():
                p.grad = cur.clone()
        g.dout.copy_(dout)
        g.bwd.replay()
        g.pending = None
        for p, gr in zip(g.params, g.grads):
            if gr is None:
                continue
            cur = p.grad
            if cur is None:
                p.grad = gr.detach()
            else:
                cur.add_(gr)
        return None, None, None


def run(model, fwd, consts, source_index):
    """``fwd(src)`` (the model's eager training forward over the fixed inputs ``consts``:
    adjacencies, group structures) through the model's captured graphs for this set of
    inputs and batch shape (captured on first use)."""
    d = model.__dict__
    cache = d.get("_msha_graphs")
    if cache is None:
        cache = d["_msha_graphs"] = OrderedDict()
    params = [p for p in model.parameters() if p.requires_grad]  # current objects
    key = (tuple((id(c), getattr(c, "_version", None)) for c in consts),
           source_index.shape, source_index.dtype, model.dropout,
           tuple([(id(p), p.data_ptr()) for p in params]))
    g = cache.get(key)
    if g is None:
        if any(getattr(p, "_msha_fused_adam", None) is not None for p in params):
            return fwd(source_index)  # optim.Adam consumes a dropout gradient: eager
        g = _ModelGraphs(fwd, params, list(model.buffers()), source_index, tuple(consts))
        cache[key] = g
        while len(cache) > MAX_GRAPHS:
            cache.popitem(last=False)
    else:
        if g.pending is not None and g.pending() is not None:
            return fwd(source_index)  # its previous output's backward is still to run: eager
        cache.move_to_end(key)
    anchor = d.get("_msha_anchor")
    if anchor is None or anchor.device != source_index.device:
        anchor = d["_msha_anchor"] = torch.zeros((), device=source_index.device, requires_grad=True)
    return _Replay.apply(g, source_index, anchor)
