"""Shared helpers for the GPU parity tests (inputs, oracle adapters)."""
import numpy as np
import torch

from oracle import gnn_oracle as O


def random_counts(rng, n, m, max_deg, empty_rows=(), hot_col=None, full_rows=()):
    c = np.zeros((n, m), np.float32)
    for i in range(n):
        d = int(rng.integers(1, max_deg + 1))
        c[i, rng.choice(m, min(d, m), replace=False)] = rng.integers(1, 4, min(d, m))
    for i in full_rows:
        c[i, :] = 1
    if hot_col is not None:
        c[:, hot_col] = np.maximum(c[:, hot_col], 1)
    for i in empty_rows:
        c[i, :] = 0
    return c


def virtual_csr(counts):
    """Oracle CSR with virtual full rows (what msha_graph_count/fill must produce)."""
    mask = counts > 0
    empty = ~mask.any(axis=1)
    mask = mask.copy()
    mask[empty] = True
    rowptr, col = O.dense_to_csr(mask.astype(np.float32))
    return rowptr, col, empty


def t(x, dev, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(x), device=dev).to(dtype)


def tol_close(a, b, rtol, atol_rel):
    """assert |a-b| <= rtol*|b| + atol_rel*max|b|."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol_rel * scale)
