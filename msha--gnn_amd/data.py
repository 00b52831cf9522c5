"""Graph ingestion for the shipped anonymised data.

Replaces the reference's ``HigherDataset`` (dataset.py:208-330), which cannot run
on the shipped files (absolute paths; ``indexMatch{Y}.json`` vs the shipped
``Adjacent{Y}.json``; an O(N^2) Python loop building two dense N x N masks that
also indexes a field the anonymised records lack, dataset.py:260-277).

Same interface as the reference dataset (``__getitem__`` -> (source, recipient),
``__len__``, ``get_count``, ``get_gdp``, ``get_adjacent``), but:
  * the inter adjacency (flow counts, dataset.py:279-288) is accumulated on the GPU
    by ``msha_inter_adjacency`` and returned as the dense (N, M) tensor train.py
    expects;
  * the city / province adjacencies are returned as ``GroupAdjacency`` (one group id
    per source: "same group" is the mask the reference materialises as N x N).
Years without a flow file (2016-2018, .MISSING_LARGE_BLOBS) get synthetic flows
with the 2015 degree law, seeded by the year.
"""
from __future__ import annotations

import csv
import json
import os

import numpy as np
import torch

from .graph import inter_adjacency


class GroupAdjacency:
    """Same-group adjacency (city or province) as group ids: row i and column j are
    adjacent iff ids[i] == ids[j] (dataset.py:267-275 builds this densely).
    ``normalize_adjacency_matrix`` keeps the mask, so it passes these through."""

    def __init__(self, ids: torch.Tensor):
        self.ids = ids

    def to(self, device):
        return GroupAdjacency(self.ids.to(device))

    @property
    def shape(self):
        n = self.ids.numel()
        return (n, n)

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim]

    def dense(self) -> torch.Tensor:
        """The reference's N x N float mask (only for small N / tests)."""
        return (self.ids[:, None] == self.ids[None, :]).to(torch.float32)


def read_year(data_dir: str, year: str):
    """Parse Adjacent{Y}.json, GDP{Y}.json and (if shipped) Flow{Y}.csv."""
    with open(os.path.join(data_dir, f"Adjacent{year}.json"), encoding="utf-8") as f:
        adj = json.load(f)
    src_idx = adj["source_index"]
    n, m = len(src_idx), len(adj["recipient_index"])
    groups = np.asarray([src_idx[str(i)] for i in range(n)], np.int64)  # [city, prov]
    with open(os.path.join(data_dir, f"GDP{year}.json"), encoding="utf-8") as f:
        gdp = json.load(f)["GDP_embedding"]
    flows = None
    path = os.path.join(data_dir, f"Flow{year}.csv")
    if os.path.exists(path):
        with open(path, encoding="gb18030") as f:
            r = csv.reader(f)
            next(r)  # header (names 2 of the 4 columns)
            flows = np.asarray([[int(row[0]), int(row[1])] for row in r if row], np.int64)
    return dict(n=n, m=m, city=groups[:, 0], prov=groups[:, 1], gdp=gdp, flows=flows)


def synthetic_flows(n: int, m: int, deg_hist: np.ndarray, col_weight: np.ndarray,
                    seed: int) -> np.ndarray:
    """One flow per (source, recipient) edge: per-source distinct degree drawn from
    ``deg_hist`` (counts of degree d at index d), recipients drawn without
    replacement with probability proportional to ``col_weight``."""
    rng = np.random.default_rng(seed)
    p_deg = deg_hist / deg_hist.sum()
    degs = rng.choice(len(deg_hist), size=n, p=p_deg)
    degs = np.clip(degs, 1, m)
    w = col_weight / col_weight.sum()
    src, dst = [], []
    for i, d in enumerate(degs):
        cols = rng.choice(m, size=int(d), replace=False, p=w)
        src.append(np.full(len(cols), i))
        dst.append(cols)
    return np.stack([np.concatenate(src), np.concatenate(dst)], 1).astype(np.int64)


def synthetic_csr(n: int, m: int, deg_hist: np.ndarray, col_weight: np.ndarray, seed: int,
                  block: int = 1 << 17):
    """Repo-shape bipartite graph at any size (SURVEY.md §8d C4 'bipartite generator,
    M = 32, 2015 degree law'), vectorised: per-source distinct degree drawn from
    ``deg_hist`` (clipped to [1, m]), recipients drawn without replacement with
    probability proportional to ``col_weight`` (Gumbel top-k: the same law as
    ``synthetic_flows``' sequential draws, not the same stream).  Returns the CSR
    (rowptr (n+1) int64, col int64, ascending within each row)."""
    rng = np.random.default_rng(seed)
    p_deg = np.asarray(deg_hist, np.float64) / np.sum(deg_hist)
    degs = np.clip(rng.choice(len(p_deg), size=n, p=p_deg), 1, m).astype(np.int64)
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(degs, out=rowptr[1:])
    col = np.empty(int(rowptr[-1]), np.int64)
    logw = np.log(np.asarray(col_weight, np.float64) / np.sum(col_weight))
    slots = np.arange(m)[None, :]
    for b0 in range(0, n, block):
        b1 = min(n, b0 + block)
        d = degs[b0:b1, None]
        keys = logw[None, :] - np.log(-np.log(rng.random((b1 - b0, m))))
        order = np.argsort(-keys, axis=1)  # a weighted random permutation per row
        pick = np.where(slots < d, order, m)
        pick.sort(axis=1)  # the row's d columns ascending, then the m sentinels
        col[rowptr[b0]:rowptr[b1]] = pick[slots < d]
    return rowptr, col


class HigherDataset(torch.utils.data.Dataset):
    """Drop-in for dataset.py:208-330 over ``anonymous_data/``."""

    def __init__(self, data_dir: str, year: str = "2015", device=None, base_year: str = "2015"):
        self.year = str(year)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        d = read_year(data_dir, self.year)
        self.N, self.M = d["n"], d["m"]
        self.GDP = d["gdp"]
        self.city, self.province = d["city"], d["prov"]
        flows = d["flows"]
        self.synthetic = flows is None
        if flows is None:
            base = read_year(data_dir, base_year)
            bf = base["flows"]
            mask = np.zeros((base["n"], base["m"]), bool)
            mask[bf[:, 0], bf[:, 1]] = True
            deg_hist = np.bincount(mask.sum(1))
            flows = synthetic_flows(self.N, self.M, deg_hist, mask.sum(0).astype(np.float64),
                                    seed=int(self.year))
        self.source = flows[:, 0]
        self.recipient = flows[:, 1]
        self.count = len(flows)
        self._adj = None

    def __getitem__(self, index):
        return int(self.source[index]), int(self.recipient[index])

    def __len__(self):
        return self.count

    def get_gdp(self):
        return self.GDP

    def get_count(self):
        return self.N, self.M

    def get_adjacent(self):
        if self._adj is None:
            src = torch.as_tensor(self.source, device=self.device)
            dst = torch.as_tensor(self.recipient, device=self.device)
            inter = inter_adjacency(src, dst, self.N, self.M)
            self._adj = (inter, GroupAdjacency(torch.as_tensor(self.city, device=self.device)),
                         GroupAdjacency(torch.as_tensor(self.province, device=self.device)))
        return self._adj
