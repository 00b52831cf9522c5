"""Row/pair sharding of the link scorer across GPUs.

The reference scores pairs on one device (LLP.py:233).  Sharded here: rank r owns
rows [r*R, (r+1)*R) of the node-embedding table (R = ceil(n / W)); ONE RCCL
``all_gather_into_tensor`` per batch rebuilds the whole table on every rank; each
rank scores a contiguous P/W slice of the pair batch.  The scores stay local (the
caller gathers them only for metrics).  This is the only collective of the path;
the GAT layers themselves run as independent replicas.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def rows_per_rank(n: int, world: int) -> int:
    return (n + world - 1) // world


def row_range(n: int, world: int, rank: int):
    r = rows_per_rank(n, world)
    lo = min(n, rank * r)
    return lo, min(n, lo + r)


def pair_range(n_pairs: int, world: int, rank: int):
    """Contiguous slice of the batch; the first (n_pairs % world) ranks take one more."""
    base, extra = divmod(n_pairs, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class ShardedTable:
    """Holds this rank's rows of an (n, F) table and rebuilds the full table."""

    def __init__(self, n: int, feat: int, world: int, rank: int, device, group=None,
                 dtype=torch.float32):
        self.n, self.feat, self.world, self.rank = n, feat, world, rank
        self.group = group
        self.R = rows_per_rank(n, world)
        self.local = torch.zeros(self.R, feat, device=device, dtype=dtype)
        self.full = torch.empty(self.R * world, feat, device=device, dtype=dtype)

    def set_local(self, rows: torch.Tensor):
        lo, hi = row_range(self.n, self.world, self.rank)
        assert rows.shape[0] == hi - lo
        self.local[: hi - lo].copy_(rows)

    def gather(self) -> torch.Tensor:
        """Full (n, F) table on every rank (padding rows of the last shard dropped)."""
        if self.world == 1:
            self.full.copy_(self.local)
        elif self.local.is_cuda:
            dist.all_gather_into_tensor(self.full, self.local, group=self.group)
        else:  # gloo (CPU tests): list form
            parts = list(self.full.view(self.world, self.R, self.feat).unbind(0))
            dist.all_gather(parts, self.local, group=self.group)
        return self.full[: self.n]


def score_sharded(table: ShardedTable, src: torch.Tensor, dst: torch.Tensor, score_fn):
    """Gather the table, then score this rank's slice of (src, dst) with
    ``score_fn(h_full, src_slice, dst_slice)``.  Returns (lo, hi, scores)."""
    h = table.gather()
    lo, hi = pair_range(src.numel(), table.world, table.rank)
    return lo, hi, score_fn(h, src[lo:hi], dst[lo:hi])
