"""Graph structures on the GPU: the CSR/CSC view of the attention mask ``adj > 0``.

Reference: the layers mask a dense (N, M) adjacency with ``torch.where(adj > 0, e,
-9e15)`` (Ablation.py:268, GAT.py:30) every forward.  Here the mask is turned into
CSR + CSC once per adjacency tensor (cached on the tensor's identity and version)
and every kernel works on edges only.

Also the data-side entry points of the reference path:
  * ``inter_adjacency``            dataset.py:279-296 (flow counts)
  * ``normalize_adjacency_matrix`` model.py:95-100
"""
from __future__ import annotations

import os
import weakref

import numpy as np
import torch

from . import _lib

CSC_CHUNK = 512  # max CSC slots per work chunk of the column aggregate
# fused backward keeps de in CSC slot order (csr_slot map); "0" = CSR edge order (A/B)
DE_SLOT_ORDER = os.environ.get("MSHA_DE_SLOT", "1") != "0"


def csc_chunk_for(n_edges: int) -> int:
    """Slots per CSC chunk: up to CSC_CHUNK, smaller on small graphs so the column
    aggregate has >= ~8k chunk-waves in flight (R15: 91k edges over 32 columns)."""
    c = n_edges // 8192
    return int(min(CSC_CHUNK, max(32, 1 << max(0, c.bit_length() - 1)))) if c > 0 else 32


class Graph:
    """CSR + CSC of an (n_rows x n_cols) mask with virtual full rows for empty rows."""

    def __init__(self, n_rows, n_cols, rowptr, col, rowflag=None, colptr=None, csc_row=None,
                 csc_eid=None, chunk=None):
        self.n_rows, self.n_cols = int(n_rows), int(n_cols)
        self.rowptr, self.col, self.rowflag = rowptr, col, rowflag
        self.colptr, self.csc_row, self.csc_eid = colptr, csc_row, csc_eid
        self.n_edges = int(col.numel())
        self.device = rowptr.device
        self._plan = None
        self._chunk = chunk if chunk is not None else csc_chunk_for(self.n_edges)
        self._desc = None
        # rows with distinct columns and at most max_deg edges (from_dense: by construction,
        # max_deg <= n_cols): what the bipartite kernels require (functional.bip_ok)
        self.distinct_cols, self.max_deg = True, self.n_cols
        if colptr is not None:
            self._build_plan(colptr.cpu().numpy().astype(np.int64))

    # -- CSC work plan: >= 1 chunk per column, long columns split into CSC_CHUNK slots
    def _build_plan(self, colptr):
        cnt = np.diff(colptr)
        nch = np.maximum(1, (cnt + self._chunk - 1) // self._chunk)
        first = np.concatenate([[0], np.cumsum(nch)[:-1]])
        chunk_col = np.repeat(np.arange(self.n_cols), nch)
        k = np.arange(int(nch.sum())) - np.repeat(first, nch)
        start = colptr[chunk_col] + k * self._chunk
        end = np.minimum(start + self._chunk, colptr[chunk_col + 1])
        multi = np.nonzero(nch > 1)[0]
        dev = self.device
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.int32), device=dev)  # noqa: E731
        self._plan = dict(n_chunks=len(chunk_col), chunk_col=t(chunk_col), chunk_start=t(start),
                          chunk_end=t(end), n_multi=len(multi), multi_col=t(multi),
                          multi_first=t(first[multi]), multi_count=t(nch[multi]),
                          max_col=int(cnt.max()) if len(cnt) else 0)

    @property
    def desc(self) -> _lib.MshaGraph:
        if self._desc is None:
            d = _lib.MshaGraph()
            d.n_rows, d.n_cols, d.n_edges = self.n_rows, self.n_cols, self.n_edges
            d.rowptr, d.col = _lib.ptr(self.rowptr), _lib.ptr(self.col)
            d.rowflag = _lib.ptr(self.rowflag)
            if self.colptr is not None:
                d.colptr, d.csc_row, d.csc_eid = (_lib.ptr(self.colptr), _lib.ptr(self.csc_row),
                                                  _lib.ptr(self.csc_eid))
                p = self._plan
                d.n_chunks = p["n_chunks"]
                d.chunk_col, d.chunk_start, d.chunk_end = (_lib.ptr(p["chunk_col"]),
                                                           _lib.ptr(p["chunk_start"]),
                                                           _lib.ptr(p["chunk_end"]))
                d.n_multi = p["n_multi"]
                d.multi_col, d.multi_first, d.multi_count = (_lib.ptr(p["multi_col"]),
                                                             _lib.ptr(p["multi_first"]),
                                                             _lib.ptr(p["multi_count"]))
                if self.csc_eid is not None and self.n_edges > 0 and DE_SLOT_ORDER:
                    # inverse of csc_eid: the fused backward's de scratch in slot order
                    self.csr_slot = torch.empty_like(self.csc_eid)
                    self.csr_slot[self.csc_eid.long()] = torch.arange(
                        self.n_edges, dtype=torch.int32, device=self.device)
                    d.csr_slot = _lib.ptr(self.csr_slot)
            if self.n_cols <= 32 and self.n_rows > 0:
                # per-row column bit masks: what the bipartite kernels walk (ABI 13)
                self.rowmask = torch.empty(self.n_rows, dtype=torch.int32, device=self.device)
                _lib.call("msha_graph_rowmask", d, self.rowmask.data_ptr(),
                          _lib.stream_handle(self.device))
                d.rowmask = _lib.ptr(self.rowmask)
            self._desc = d
        return self._desc

    @property
    def has_csc(self):
        return self.colptr is not None

    def row_view(self) -> "Graph":
        """The CSR presented as a CSC (colptr = rowptr, csc_row = col, csc_eid = NULL:
        slot = edge id) with a chunk plan over the rows: msha_csc_aggregate on it
        computes A @ table instead of A^T @ table (GCN's second layer, the SpMM
        backward)."""
        if getattr(self, "_row_view", None) is None:
            self._row_view = Graph(self.n_cols, self.n_rows, self.colptr, self.csc_row, None,
                                   self.rowptr, self.col, None)
        return self._row_view

    def values(self, adj: torch.Tensor) -> torch.Tensor:
        """fp32 adjacency values on the CSR edges (0 on virtual rows), cached per
        (tensor, version): the weights of the GCN SpMM."""
        key = (id(adj), adj._version)
        if getattr(self, "_vals_key", None) != key:
            rows = torch.repeat_interleave(torch.arange(self.n_rows, device=self.device),
                                           self.deg().long())
            self._vals = adj.detach()[rows, self.col.long()].to(torch.float32).contiguous()
            self._vals_key = key
            self._vals_ref = weakref.ref(adj)
        return self._vals

    def deg(self):
        return self.rowptr[1:] - self.rowptr[:-1]

    # ------------------------------------------------------------------ builders
    @classmethod
    def from_dense(cls, adj: torch.Tensor) -> "Graph":
        """Mask ``adj > 0`` -> CSR/CSC on the GPU (msha_graph_count / msha_graph_fill)."""
        _lib.require_cuda(adj)
        if adj.dim() != 2:
            raise ValueError("adjacency must be 2-D (N, M)")
        a = adj.detach()
        if a.dtype != torch.float32:
            a = (a > 0).to(torch.float32)
        a = a.contiguous()
        n, m = a.shape
        dev = a.device
        s = _lib.stream_handle(dev)
        wsb = _lib.load().msha_graph_workspace_size(n, m)
        ws = torch.empty(max(int(wsb), 16), dtype=torch.uint8, device=dev)
        rowptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
        colptr = torch.empty(m + 1, dtype=torch.int32, device=dev)
        rowflag = torch.empty(n, dtype=torch.uint8, device=dev)
        _lib.call("msha_graph_count", a.data_ptr(), n, m, rowptr.data_ptr(), colptr.data_ptr(),
                  rowflag.data_ptr(), ws.data_ptr(), ws.numel(), s)
        e = int(rowptr[-1].item())  # one sync per adjacency (cached afterwards)
        col = torch.empty(max(e, 1), dtype=torch.int32, device=dev)[:e]
        csc_row = torch.empty(max(e, 1), dtype=torch.int32, device=dev)[:e]
        csc_eid = torch.empty(max(e, 1), dtype=torch.int32, device=dev)[:e]
        _lib.call("msha_graph_fill", a.data_ptr(), n, m, rowptr.data_ptr(), colptr.data_ptr(),
                  rowflag.data_ptr(), col.data_ptr(), csc_row.data_ptr(), csc_eid.data_ptr(),
                  ws.data_ptr(), ws.numel(), s)
        return cls(n, m, rowptr, col, rowflag, colptr, csc_row, csc_eid)

    @classmethod
    def from_csr(cls, rowptr, col, n_cols, device, with_csc=True) -> "Graph":
        """Caller-provided CSR (numpy or tensors, every row degree >= 1).  The CSC
        permutation (stable by row) is prepared on the host."""
        rowptr = np.asarray(rowptr.cpu() if torch.is_tensor(rowptr) else rowptr, np.int64)
        col = np.asarray(col.cpu() if torch.is_tensor(col) else col, np.int64)
        if np.any(np.diff(rowptr) <= 0):
            raise ValueError("from_csr needs every row degree >= 1 (use from_dense for "
                             "virtual full rows)")
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.int32), device=device)  # noqa
        n = len(rowptr) - 1
        rows_of = np.repeat(np.arange(n, dtype=np.int64), np.diff(rowptr))
        distinct = len(np.unique(rows_of * max(int(n_cols), 1) + col)) == len(col)
        max_deg = int(np.diff(rowptr).max()) if n else 0
        if not with_csc:
            g = cls(n, n_cols, t(rowptr), t(col))
            g.distinct_cols, g.max_deg = distinct, max_deg
            return g
        perm = np.argsort(col, kind="stable")
        rows = np.repeat(np.arange(n), np.diff(rowptr))
        colptr = np.zeros(n_cols + 1, np.int64)
        np.cumsum(np.bincount(col, minlength=n_cols), out=colptr[1:])
        g = cls(n, n_cols, t(rowptr), t(col), None, t(colptr), t(rows[perm]), t(perm))
        g.distinct_cols, g.max_deg = distinct, max_deg
        return g


_CACHE: dict = {}


def graph_for(adj: torch.Tensor) -> Graph:
    """Cached Graph of a dense adjacency tensor (keyed on its identity + version)."""
    key = (id(adj), adj.data_ptr(), adj._version, tuple(adj.shape), adj.dtype, str(adj.device))
    hit = _CACHE.get(key)
    if hit is not None:
        ref, g = hit
        if ref() is adj:
            return g
    g = Graph.from_dense(adj)
    for k in [k for k, (r, _) in _CACHE.items() if r() is None]:
        del _CACHE[k]
    _CACHE[key] = (weakref.ref(adj), g)
    return g


def graph_of(adj: torch.Tensor):
    """(Graph, transposed): a transposed view of a cached adjacency (``adj.t()``, as
    GCN's second layer passes it, model.py:62) maps to the base tensor's graph."""
    if (adj.dim() == 2 and adj._base is not None and not adj.is_contiguous()
            and adj.t().is_contiguous() and adj._base.shape == adj.t().shape
            and adj._base.data_ptr() == adj.data_ptr()):
        return graph_for(adj._base), True
    return graph_for(adj), False


def clear_cache():
    _CACHE.clear()


# ---------------------------------------------------------------- data side ---
def inter_adjacency(source: torch.Tensor, recipient: torch.Tensor, n_rows: int,
                    n_cols: int) -> torch.Tensor:
    """Flow-count adjacency (dataset.py:279-288): ``adj[source[k], recipient[k]] += 1``.

    Like the reference's dict lookup, an out-of-range index is an error."""
    _lib.require_cuda(source, recipient)
    src = source.to(torch.int64).contiguous()
    dst = recipient.to(torch.int64).contiguous()
    if src.numel() != dst.numel():
        raise ValueError("source and recipient must have the same length")
    if src.numel():
        lo = torch.stack([src.min(), dst.min()]).min()
        if bool(lo < 0) or bool(src.max() >= n_rows) or bool(dst.max() >= n_cols):
            raise IndexError("flow index out of range")
    adj = torch.empty(n_rows, n_cols, dtype=torch.float32, device=src.device)
    ws = torch.empty(n_rows * n_cols, dtype=torch.int32, device=src.device)
    _lib.call("msha_inter_adjacency", src.data_ptr(), dst.data_ptr(), src.numel(), n_rows, n_cols,
              adj.data_ptr(), ws.data_ptr(), _lib.stream_handle(src.device))
    return adj


def normalize_adjacency_matrix(adjacency_matrix: torch.Tensor) -> torch.Tensor:
    """model.py:95-100: ``adj @ diag(d) @ diag(d)``, ``d = colsum ** -0.5``, computed as
    ``(adj * d) * d`` (bit-identical for finite d; a zero column gives NaN everywhere).
    Group adjacencies (data.GroupAdjacency) pass through: every column of a
    same-group mask has a non-zero sum, so normalising keeps the mask."""
    if not torch.is_tensor(adjacency_matrix) and hasattr(adjacency_matrix, "ids"):
        return adjacency_matrix
    _lib.require_cuda(adjacency_matrix)
    a = adjacency_matrix.detach()
    if a.dtype != torch.float32:
        raise TypeError("normalize_adjacency_matrix: float32 adjacency expected")
    a = a.contiguous()
    n, m = a.shape
    out = torch.empty_like(a)
    ws = torch.empty(m + 1, dtype=torch.float32, device=a.device)
    _lib.call("msha_normalize_adjacency", a.data_ptr(), n, m, out.data_ptr(), ws.data_ptr(),
              _lib.stream_handle(a.device))
    return out


# ----------------------------------------------------------- group adjacency ---
class Groups:
    """City + province membership of the N source nodes as CSR (struct msha_groups).

    The reference passes same-group masks as dense N x N matrices
    (dataset.py:260-277); here a node's group is an id and each group a sorted
    member list, built once (host) and kept on the device."""

    def __init__(self, city_ids, prov_ids, device):
        self.n = int(len(city_ids))
        self.device = torch.device(device)
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.int32), device=self.device)  # noqa
        self._keep = []
        self.max_group = 0
        for ids in (city_ids, prov_ids):
            ids = np.asarray(ids.cpu() if torch.is_tensor(ids) else ids, np.int64)
            _, gid = np.unique(ids, return_inverse=True)
            order = np.argsort(gid, kind="stable")
            gptr = np.zeros(gid.max() + 2 if len(gid) else 1, np.int64)
            sizes = np.bincount(gid, minlength=len(gptr) - 1)
            np.cumsum(sizes, out=gptr[1:])
            self.max_group = max(self.max_group, int(sizes.max()) if len(sizes) else 0)
            self._keep.append((t(gid), t(gptr), t(order)))
        self._desc = None

    @property
    def desc(self) -> _lib.MshaGroups:
        if self._desc is None:
            d = _lib.MshaGroups()
            d.n_nodes = self.n
            (g3, p3, m3), (g4, p4, m4) = self._keep
            d.gid3, d.gptr3, d.gmem3 = g3.data_ptr(), p3.data_ptr(), m3.data_ptr()
            d.gid4, d.gptr4, d.gmem4 = g4.data_ptr(), p4.data_ptr(), m4.data_ptr()
            d.max_group = self.max_group
            self._desc = d
        return self._desc


def _group_ids(adj):
    """Group id per node from a GroupAdjacency or a dense same-group mask (the id of a
    node is the first member of its row: rows of one group are identical)."""
    if hasattr(adj, "ids"):
        return adj.ids
    a = adj.detach()
    if a.dim() != 2 or a.shape[0] != a.shape[1]:
        raise ValueError("group adjacency must be square (N, N) or a GroupAdjacency")
    return (a > 0).to(torch.int8).argmax(dim=1)


_GROUP_CACHE: dict = {}


def groups_for(city_adj, province_adj, device) -> Groups:
    key = (id(city_adj), id(province_adj), str(device))
    hit = _GROUP_CACHE.get(key)
    if hit is not None and hit[0]() is city_adj and hit[1]() is province_adj:
        return hit[2]
    g = Groups(_group_ids(city_adj), _group_ids(province_adj), device)
    try:
        _GROUP_CACHE[key] = (weakref.ref(city_adj), weakref.ref(province_adj), g)
    except TypeError:  # objects without weakref support: no caching
        pass
    return g
