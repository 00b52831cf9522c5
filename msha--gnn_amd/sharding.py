"""Row/pair sharding of the link scorer across GPUs.

The reference scores pairs on one device (LLP.py:233).  Sharded here: rank r owns
rows [r*R, (r+1)*R) of the node-embedding table (R = ceil(n / W)); ONE RCCL
``all_gather_into_tensor`` per batch rebuilds the whole table on every rank; each
rank scores a contiguous P/W slice of the pair batch.  The scores stay local (the
caller gathers them only for metrics).  This is the only collective of the path;
the GAT layers themselves run as independent replicas.

Whenever a process group is initialised the gather is the collective -- world 1
included, so the RCCL path is the one a single-GPU run exercises too; only without a
process group does a single rank copy its rows.  ``PipelinedScorer`` double-buffers
the gathered table: batch k+1's all-gather runs on the communicator's stream while
batch k is scored on the compute stream.
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


def _group_ready(group, world: int) -> bool:
    """Run the collective: a process group is initialised and either one was passed or
    the default group spans exactly this table's world.  (A rank-local world-1 table in
    a multi-process job copies its rows instead of failing the world-size check.)"""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return group is not None or dist.get_world_size() == world


class ShardedTable:
    """Holds this rank's rows of an (n, F) table and rebuilds the full table into one
    of ``buffers`` gathered images (two for the pipelined scorer)."""

    def __init__(self, n: int, feat: int, world: int, rank: int, device, group=None,
                 dtype=torch.float32, buffers: int = 1):
        self.n, self.feat, self.world, self.rank = n, feat, world, rank
        self.group = group
        self.R = rows_per_rank(n, world)
        self.local = torch.zeros(self.R, feat, device=device, dtype=dtype)
        self.fulls = [torch.empty(self.R * world, feat, device=device, dtype=dtype)
                      for _ in range(max(1, buffers))]
        self.cur = 0
        if dist.is_available() and dist.is_initialized() and (group is not None or world > 1):
            # world 1 without a group may copy its rows inside a larger job; any other table
            # must match the group it will gather over
            gw = dist.get_world_size(group)
            if gw != world:
                raise ValueError(f"ShardedTable: world {world} but the process group has {gw}")

    @property
    def full(self) -> torch.Tensor:
        """The gathered image last written (padded to R * world rows)."""
        return self.fulls[self.cur]

    def set_local(self, rows: torch.Tensor):
        lo, hi = row_range(self.n, self.world, self.rank)
        assert rows.shape[0] == hi - lo
        self.local[: hi - lo].copy_(rows)

    def path(self) -> str:
        """Which exchange ``gather`` runs: 'rccl' (all_gather_into_tensor on a CUDA
        group), 'gloo' (list all_gather, CPU tests) or 'copy' (no process group)."""
        if not _group_ready(self.group, self.world):
            if self.world != 1:
                raise RuntimeError("ShardedTable: world > 1 needs an initialised process group")
            return "copy"
        return "rccl" if self.local.is_cuda else "gloo"

    def gather_async(self, buffer: int | None = None):
        """Start rebuilding the full table into image ``buffer`` (default: the current
        one); returns (image[:n], work handle or None).  The RCCL collective runs on the
        communicator's stream, ordered after work already queued on the current stream;
        ``work.wait()`` makes the current stream wait for it."""
        b = self.cur if buffer is None else buffer
        dst = self.fulls[b]
        path = self.path()
        work = None
        if path == "copy":
            dst[: self.R].copy_(self.local)
        elif path == "rccl":
            work = dist.all_gather_into_tensor(dst, self.local, group=self.group, async_op=True)
        else:  # gloo (CPU tests): list form
            parts = list(dst.view(self.world, self.R, self.feat).unbind(0))
            work = dist.all_gather(parts, self.local, group=self.group, async_op=True)
        self.cur = b
        return dst[: self.n], work

    def gather(self, buffer: int | None = None) -> torch.Tensor:
        """Full (n, F) table on every rank (padding rows of the last shard dropped),
        stream-ordered before later work on the current stream."""
        full, work = self.gather_async(buffer)
        if work is not None:
            work.wait()
        return full


def score_sharded(table: ShardedTable, src: torch.Tensor, dst: torch.Tensor, score_fn):
    """Gather the table, then score this rank's slice of (src, dst) with
    ``score_fn(h_full, src_slice, dst_slice)``.  Returns (lo, hi, scores)."""
    h = table.gather()
    lo, hi = pair_range(src.numel(), table.world, table.rank)
    return lo, hi, score_fn(h, src[lo:hi], dst[lo:hi])


class PipelinedScorer:
    """Scores a stream of batches, each against its own all-gather of the table, with
    the gather of batch k+1 overlapped with the scoring of batch k (two gathered
    images; the collective runs on the communicator's stream).

    ``refresh(k)``, if given, writes batch k's local rows into ``table.local`` before
    its gather is issued (e.g. the embedding pass that produced them); the gather of
    batch k+1 is issued after batch k-1's scoring, which read the same image, and the
    compute stream waits for it only before scoring batch k+1."""

    def __init__(self, table: ShardedTable, score_fn, refresh=None):
        if len(table.fulls) < 2:
            raise ValueError("PipelinedScorer needs a ShardedTable with buffers=2")
        self.table, self.score_fn, self.refresh = table, score_fn, refresh

    def run(self, batches):
        """batches: sequence of (src, dst) over the whole pair set; returns this rank's
        [(lo, hi, scores)] per batch."""
        t = self.table
        out = []
        if not batches:
            return out
        if self.refresh is not None:
            self.refresh(0)
        full, work = t.gather_async(0)
        for k, (src, dst) in enumerate(batches):
            if work is not None:
                work.wait()
            nxt = None
            if k + 1 < len(batches):
                if self.refresh is not None:
                    self.refresh(k + 1)
                nxt = t.gather_async((k + 1) % 2)
            lo, hi = pair_range(src.numel(), t.world, t.rank)
            out.append((lo, hi, self.score_fn(full, src[lo:hi], dst[lo:hi])))
            if nxt is not None:
                full, work = nxt
        t.cur = (len(batches) - 1) % 2
        return out
