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


U32 = 2.0 ** -24  # fp32 unit roundoff


STAT_C = 4.0  # standard deviations of the rounding-error random walk allowed


BF16_U = 2.0 ** -8  # bf16 unit roundoff with one extra bit of slack (stored bf16 values)
BF16_STORE = 2.0 ** -9  # one round-to-nearest bf16 storage rounding, relative
# an fp32 value carried as hi + mid bf16 terms (RNE each): |x - hi - mid| <= 2^-18 |x|
BF16_SPLIT2 = 2.0 ** -18


def bounded_close(got, ref, absterms, nterms, rtol, name="", u=U32, store_u=0.0, split_u=0.0):
    """Sums against an fp64 reference, EVERY element (no fraction clause):

        |got - ref| <= rtol |ref| + store_u |ref| + 4 sqrt(n) u A

    A = the sum of the absolute values of the terms (incl. the magnitudes inside each
    term, e.g. |g| + |D| of a score gradient), n = the number of terms plus the ops
    inside a term and the reduce levels (``nterms``, scalar or per element).  The
    rounding errors of an n-term fp32 sum are a random walk of n steps of at most
    u |partial| each, so 4 sqrt(n) u A is a four-sigma statistical bound (the worst-case
    n u A is ~sqrt(n) times looser: 2e-3 A for the 70k-edge bip1m columns).  A small
    element is held to its own terms, never to the tensor's largest.  ``u``: the unit
    roundoff of the accumulation (fp32 2^-24, also on the bf16 paths: their operands are
    exact bf16 values, fed to the reference as such, and they accumulate in fp32);
    ``store_u``: the result's own storage rounding (a bf16 output: 2^-9, BF16_STORE);
    ``split_u``: a deterministic per-term operand error, bound + split_u A (an fp32 operand
    carried as two bf16 terms on the matrix cores: 2^-18, BF16_SPLIT2).
    Returns (max err / bound, fraction within rtol |ref| alone) for reporting."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    A = np.broadcast_to(np.asarray(absterms, np.float64), ref.shape)
    n = np.asarray(nterms, np.float64)
    if n.ndim == 1 and ref.ndim > 1:  # per leading index (row / column)
        n = n.reshape((-1,) + (1,) * (ref.ndim - 1))
    n = np.broadcast_to(n, ref.shape)
    err = np.abs(got - ref)
    bound = (rtol + store_u) * np.abs(ref) + (STAT_C * np.sqrt(n) * u + split_u) * A + 1e-300
    worst = float((err / bound).max()) if err.size else 0.0
    assert np.all(err <= bound), (
        f"{name}: {int((err > bound).sum())} of {err.size} elements beyond "
        f"rtol|ref| + 4 sqrt(n) u A (worst {worst:.3g}x the bound)")
    inside = float(np.mean(err <= rtol * np.abs(ref))) if err.size else 1.0
    print(f"{name}: worst err / bound {worst:.3g}; {inside:.2%} within rtol |ref| alone")
    return worst, inside


def rel_close(got, ref, rtol, floor, name=""):
    """Elementwise relative check above a stated magnitude floor: every element within
    rtol max(|ref|, floor) -- the floor is an absolute magnitude of the quantity (not a
    fraction of the tensor's largest element)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(got - ref)
    bound = rtol * np.maximum(np.abs(ref), floor)
    worst = float((err / bound).max()) if err.size else 0.0
    assert np.all(err <= bound), (f"{name}: {int((err > bound).sum())} of {err.size} elements "
                                  f"beyond {rtol} max(|ref|, {floor}) (worst {worst:.3g}x)")
    return worst


def _row_rms(x):
    """RMS over each row (leading index) of x, broadcast back to x's shape; a 1-D or 0-D x
    is one row."""
    x = np.asarray(x, np.float64)
    if x.ndim <= 1 or x.size == x.shape[0]:  # a vector (also (n, 1)): one row
        return np.full(x.shape, np.sqrt(np.mean(x * x)) if x.size else 0.0)
    r = np.sqrt(np.mean(x.reshape(x.shape[0], -1) ** 2, axis=1))
    return np.broadcast_to(r.reshape((-1,) + (1,) * (x.ndim - 1)), x.shape)


def _row_max(x):
    """max |x| over each row (leading index), broadcast back; a vector: one row."""
    x = np.abs(np.asarray(x, np.float64))
    if x.ndim <= 1 or x.size == x.shape[0]:  # a vector (also (n, 1)): one row
        return np.full(x.shape, x.max() if x.size else 0.0)
    r = x.reshape(x.shape[0], -1).max(axis=1)
    return np.broadcast_to(r.reshape((-1,) + (1,) * (x.ndim - 1)), x.shape)


def ref32_close(got, ref64, ref32, rtol, name="", k=4.0):
    """Against the reference's fp64 run, EVERY element:

        |got - ref64| <= rtol |ref64| + k e_row,

    e_row = the largest |ref32 - ref64| on the element's row: the worst error the
    reference's own fp32 run (the north_star's CPU path, same formulation, parameters
    and LeakyReLU branches) makes on that row.  A cancelled element is held to a few times
    the accuracy fp32 arithmetic reaches on its row, never to a fraction of the tensor's
    largest element (no max|ref| floor, no fraction clause)."""
    got = np.asarray(got, np.float64)
    ref64 = np.asarray(ref64, np.float64)
    e = _row_max(np.asarray(ref32, np.float64) - ref64)
    err = np.abs(got - ref64)
    bound = rtol * np.abs(ref64) + k * e + 1e-300
    worst = float((err / bound).max()) if err.size else 0.0
    print(f"{name}: worst err / bound {worst:.3g} (rtol {rtol}, {k} x the row's largest "
          f"fp32-reference error)")
    assert np.all(err <= bound), (
        f"{name}: {int((err > bound).sum())} of {err.size} elements beyond rtol |ref| + "
        f"{k} x the reference's fp32 row error (worst {worst:.3g}x the bound)")
    return worst


def rms_close(got, ref, rtol, name=""):
    """EVERY element within rtol max(|ref|, RMS of its row of ref): relative above the
    row's typical magnitude, absolute at that magnitude below it (a cancelled element's
    error is set by the size of its terms, of the order of its row's typical element);
    no max|ref| floor."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(got - ref)
    bound = rtol * np.maximum(np.abs(ref), _row_rms(ref)) + 1e-300
    worst = float((err / bound).max()) if err.size else 0.0
    print(f"{name}: worst err / bound {worst:.3g} (rtol {rtol} of max(|ref|, row RMS))")
    assert np.all(err <= bound), (f"{name}: {int((err > bound).sum())} of {err.size} elements "
                                  f"beyond {rtol} max(|ref|, row RMS) (worst {worst:.3g}x)")
    return worst


def _seg_sum(x, ptr):
    """Sums of x over the contiguous segments [ptr[k], ptr[k+1]) of axis 0 (empty ones 0),
    via a running sum (the terms here are non-negative)."""
    cs = np.concatenate([np.zeros((1,) + x.shape[1:]), np.cumsum(x, axis=0)])
    return cs[ptr[1:]] - cs[ptr[:-1]]


def edge_abs_terms(rowptr, col, fwd, hc, dU, hs=None, dV=None, keep=None, p=0.0, slope=0.2):
    """Absolute-term sums A for ``bounded_close`` of the OursLayer3 core (fp64, from the
    oracle's forward dict: att, attd, pre): per row u (att |hc_j|), d_hs (att |dV_j|),
    d_el; per column v (att |hs_i|), d_hc (att |dU_i|), d_er.  The score gradient
    de = att (keep g - D) lrelu' has A_e = att (keep |g|_abs + |D|_abs) |lrelu'| with
    |g|_abs = sum_f |dU_if hc_jf| + |hs_if dV_jf|, |D|_abs = sum_row attd |g|_abs.
    Also n_row / n_col, the term counts for the bound."""
    rowptr = np.asarray(rowptr, np.int64)
    n = len(rowptr) - 1
    m, H, F = hc.shape
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    c64 = np.asarray(col, np.int64)
    perm = np.argsort(c64, kind="stable")
    nnz = np.bincount(c64, minlength=m)
    colptr = np.concatenate([[0], np.cumsum(nnz)])
    att, attd = fwd["att"].astype(np.float64), fwd["attd"].astype(np.float64)
    kf = np.ones_like(att) if keep is None else keep.astype(np.float64) / (1.0 - p)
    dl = np.where(fwd["pre"] > 0, 1.0, slope)
    out = {k: np.zeros(s) for k, s in (("u", (n, H, F)), ("d_hs", (n, H, F)),
                                         ("v", (m, H, F)), ("d_hc", (m, H, F)),
                                         ("d_el", (n, H)), ("d_er", (m, H)))}
    for h in range(H):
        ah, adu = np.abs(hc[:, h].astype(np.float64)), np.abs(dU[:, h].astype(np.float64))
        w = attd[:, h:h + 1]
        hcj, dui = ah[c64], adu[rows]
        gabs = np.einsum("ef,ef->e", dui, hcj)
        out["u"][:, h] = _seg_sum(w * hcj, rowptr)
        out["d_hc"][:, h] = _seg_sum((w * dui)[perm], colptr)
        del hcj
        if hs is not None:
            ahs = np.abs(hs[:, h].astype(np.float64))
            hsi = ahs[rows]
            out["v"][:, h] = _seg_sum((w * hsi)[perm], colptr)
            if dV is not None:
                dvj = np.abs(dV[:, h].astype(np.float64))[c64]
                gabs += np.einsum("ef,ef->e", hsi, dvj)
                out["d_hs"][:, h] = _seg_sum(w * dvj, rowptr)
                del dvj
            del hsi
        del dui
        dabs = _seg_sum(attd[:, h] * gabs, rowptr)
        T = att[:, h] * (kf[:, h] * gabs + dabs[rows]) * dl[:, h]
        out["d_el"][:, h] = _seg_sum(T, rowptr)
        out["d_er"][:, h] = _seg_sum(T[perm], colptr)
    # terms per output: the outer sum, the 2F-term dots inside g, 16 elementwise ops, and
    # up to 80 levels of the wave / block partial reduce
    k_in = 2 * F + 96
    out["n_row"] = np.diff(rowptr).astype(np.float64) + k_in
    out["n_col"] = nnz.astype(np.float64) + k_in
    return out
