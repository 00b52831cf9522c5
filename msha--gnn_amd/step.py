"""Whole-iteration HIP-graph capture for the train.py step (train.py:221-232).

The shipped graphs are small (R15: 39k sources, 91k edges), so one training
iteration -- forward, nll, backward, Adam -- is ~160 short launches and its wall
time is host launch overhead, not kernel time.  ``GraphedStep`` captures the
iteration once into a HIP graph (torch.cuda.CUDAGraph over the current HIP stream)
and replays it: the library's kernels and the torch ops around them (BatchNorm,
dropout, the loss, the capturable Adam) all become graph nodes.

Dropout stays fresh across replays: the library's Philox draws take their seeds as
kernel arguments (frozen at capture), so a device replay counter is installed with
``functional.set_rng_counter`` and incremented ahead of every replay
(include/msha_gnn.h, msha_set_rng_counter): by ``replay(feed=(dst, src))``'s batch copy
itself (msha_feed_step, one launch for both), else by a separate add; torch's own dropout
uses its generator's graph-safe offsets.
"""
from __future__ import annotations

from typing import Callable

import torch

from . import functional as MF


class GraphedStep:
    """Capture ``body()`` (one full iteration; it reads its batch from static device
    tensors the caller refills before each replay) and replay it.

    The optimizer must be built with ``capturable=True``; gradients must be None
    before capture (``zero_grad(set_to_none=True)``) so the captured backward writes
    fresh gradient buffers on every replay instead of accumulating."""

    def __init__(self, body: Callable[[], torch.Tensor], device, warmup: int = 3):
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        # this step's counter replaces (and on close() restores) the device's previous one
        self._prev = MF.set_rng_counter(self.counter)
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):  # warm caches (graph views, workspaces) off-graph
            for _ in range(warmup):
                self.counter.add_(1)
                body()
        torch.cuda.current_stream(self.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = body()

    def replay(self, feed=None) -> torch.Tensor:
        """Advance the replay counter and replay.  ``feed=(dst, src)``: copy the next batch
        into the static input ``dst`` in the same launch that advances the counter."""
        if feed is not None:
            MF.feed_step(feed[0], feed[1], self.counter)
        else:
            self.counter.add_(1)
        self.graph.replay()
        return self.out

    def close(self):
        """Drop the graph; reinstall the counter that was installed before this step
        (if this step's counter is still the device's), so other live steps keep drawing
        fresh masks.  The captured kernels keep reading ``self.counter``'s memory, which
        stays alive with this object."""
        if self.graph is None:
            return
        if MF.rng_counter(self.device) is self.counter:
            MF.set_rng_counter(self._prev, self.device)
        self.graph = None
