"""CPU oracle for the MSHA--GNN attention hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker / the timed CPU baseline.  The
product path (``msha--gnn_amd``) never imports it and fails loudly when its HIP
library is missing.

This is a sparse (CSR) restatement, in numpy, of the dense PyTorch arithmetic of
the reference (Sienna12321/MSHA--GNN @ 2025-01-17).  Each function cites the
reference lines it restates.  It is dtype-generic: called with float64 arrays it
reproduces the reference run in float64 to ~1e-12, with float32 arrays it is the
fp32 checker for the HIP kernels.

Parity pin: ``tests/golden/*.npz`` were produced by importing the reference's own
modules (``GAT.py``, ``Ablation.py``, ``model.py``; ``LLP.LinkPredictor`` and
``Ours.OursLayer`` by AST extraction) in the build container
(``tests/golden/make_golden.py``); ``tests/test_oracle_golden.py`` checks this
module against them.

Conventions (shared with the HIP library, see include/msha_gnn.h):
  * CSR over the (N, M) adjacency mask ``adj > 0``: ``rowptr`` (N+1), ``col`` (E),
    edges in row-major order (== ``torch.nonzero(adj > 0)`` order).
  * Per-edge arrays are (E, H); node tables are (rows, H, F), head-major.
  * ``el`` (N, H) is the source-row score half, ``er`` (M, H) the column half.
    Reference ``Ablation.py:266-267`` multiplies ``a[:F]`` with the RECIPIENT
    (column) features ``h1`` and ``a[F:]`` with the SOURCE (row) features ``h2``.
"""
from __future__ import annotations

import numpy as np

NEG_SLOPE = 0.2  # Ablation.py:267, GAT.py:27 (negative_slope=0.2)


# ----------------------------------------------------------------------------------
# graph construction / preprocessing
# ----------------------------------------------------------------------------------
def inter_adjacency(source, recipient, n_rows, n_cols, dtype=np.float32):
    """Flow-count adjacency.  Restates dataset.py:279-288 (``inter_adjacent``):
    ``adj[source[k], recipient[k]] += 1`` for every flow record k."""
    adj = np.zeros((n_rows, n_cols), dtype=np.int64)
    np.add.at(adj, (np.asarray(source, np.int64), np.asarray(recipient, np.int64)), 1)
    return adj.astype(dtype)


def normalize_adjacency(adj):
    """Restates model.py:95-100 ``normalize_adjacency_matrix``.

    ``adj @ diag(d) @ diag(d)`` with ``d = colsum ** -0.5``.  Each product has a
    single non-zero term per output, so it is exactly ``(adj * d) * d`` in the
    input dtype; a zero column sum gives d = inf, and ``0 * inf`` = NaN then
    spreads through the second product to every entry (every row holds that
    NaN column), which we reproduce explicitly.
    """
    adj = np.asarray(adj)
    deg = adj.sum(axis=0, dtype=adj.dtype)
    with np.errstate(divide="ignore", invalid="ignore"):
        d = (np.asarray(1, adj.dtype) / np.sqrt(deg)).astype(adj.dtype)
        out = (adj * d[None, :]) * d[None, :]
    if not np.all(np.isfinite(d)):
        # first product: column j0 with d=inf holds 0*inf=NaN (or inf) in every row;
        # second product sums X[i,j0]*0 into every output -> NaN everywhere.
        out = np.full_like(out, np.nan)
    return out


def dense_to_csr(adj):
    """Mask ``adj > 0`` in row-major order (Ablation.py:268 ``torch.where(adj > 0, ...)``)."""
    mask = np.asarray(adj) > 0
    n = mask.shape[0]
    deg = mask.sum(axis=1)
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(deg, out=rowptr[1:])
    _, col = np.nonzero(mask)
    return rowptr.astype(np.int32), col.astype(np.int32)


def csr_to_csc(rowptr, col, n_cols):
    """Column view: ``colptr`` (M+1), ``perm`` (E) edge ids ordered by (col, row)."""
    col = np.asarray(col, np.int64)
    perm = np.argsort(col, kind="stable")
    cnt = np.bincount(col, minlength=n_cols)
    colptr = np.zeros(n_cols + 1, np.int64)
    np.cumsum(cnt, out=colptr[1:])
    return colptr.astype(np.int32), perm.astype(np.int32)


def edge_rows(rowptr):
    deg = np.diff(np.asarray(rowptr, np.int64))
    return np.repeat(np.arange(len(deg)), deg)


# ----------------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------------
def lrelu(x, slope=NEG_SLOPE):
    return np.where(x > 0, x, x * np.asarray(slope, x.dtype))


def lrelu_grad(x, slope=NEG_SLOPE):
    # torch leaky_relu_backward: grad * (self > 0 ? 1 : negval)
    return np.where(x > 0, np.asarray(1, x.dtype), np.asarray(slope, x.dtype))


def elu(x):
    return np.where(x > 0, x, np.expm1(np.minimum(x, 0)))


def elu_grad(x):
    return np.where(x > 0, np.asarray(1, x.dtype), np.exp(np.minimum(x, 0)))


def _seg_reduce(values, rowptr, ufunc, empty):
    """Segmented reduction over CSR rows along axis 0 (rows with deg 0 get ``empty``)."""
    rowptr = np.asarray(rowptr, np.int64)
    n = len(rowptr) - 1
    out = np.full((n,) + values.shape[1:], empty, dtype=values.dtype)
    nz = np.nonzero(np.diff(rowptr) > 0)[0]
    if len(nz):
        out[nz] = ufunc.reduceat(values, rowptr[nz], axis=0)
    return out


# ----------------------------------------------------------------------------------
# fused edge-softmax + aggregate (OursLayer3 inter attention, Ablation.py:260-277)
# ----------------------------------------------------------------------------------
def edge_softmax_fwd(rowptr, col, el, er, slope=NEG_SLOPE, rowflag=None):
    """Per-row masked softmax of ``lrelu(el_i + er_j)`` over the CSR row.

    Restates Ablation.py:266-270: ``e12 = lrelu(cat(h1_j, h2_i) @ a)``,
    ``where(adj > 0, e12, -9e15)``, ``softmax(dim=1)``.  Returns (att (E,H),
    pre (E,H), empty-row mask).  Empty rows are uniform over all M columns (the
    softmax of an all -9e15 row) and are handled by the callers, or, when
    ``rowflag`` marks rows stored as virtual full rows (every column an edge),
    by a constant score on those rows.
    """
    rows = edge_rows(rowptr)
    col = np.asarray(col, np.int64)
    pre = el[rows] + er[col]
    s = lrelu(pre, slope)
    if rowflag is not None:
        s = np.where(np.asarray(rowflag, bool)[rows][:, None], np.asarray(0, s.dtype), s)
    m = _seg_reduce(s, rowptr, np.maximum, -np.inf)
    ex = np.exp(s - m[rows])
    den = _seg_reduce(ex, rowptr, np.add, 0)
    att = ex / den[rows]
    empty = np.diff(np.asarray(rowptr, np.int64)) == 0
    return att, pre, empty


def edge_aggregate_fwd(rowptr, col, el, er, hc, hs=None, keep=None, p=0.0,
                       slope=NEG_SLOPE, rowflag=None):
    """Forward of the OursLayer3 inter-attention core (Ablation.py:266-274).

    hc (M,H,F): column (recipient) table, gathered per edge -> ``u = att @ h1``.
    hs (N,H,F): optional row (source) table -> ``v = att.T @ h2`` (Ablation.py:273).
    keep (E,H) bool / None: dropout keep mask on edges (Ablation.py:271); the dense
    reference also drops entries of empty rows, which are represented here as
    virtual full rows (see ``empty_row_keep``).
    Returns dict(att, attd, u, v, lse, pre).
    """
    dt = hc.dtype
    n = len(rowptr) - 1
    m_cols, H, F = hc.shape
    att, pre, empty = edge_softmax_fwd(rowptr, col, el, er, slope, rowflag)
    scale = np.asarray(1.0 / (1.0 - p) if p > 0 else 1.0, dt)
    attd = att if keep is None else att * keep * scale
    rows = edge_rows(rowptr)
    col64 = np.asarray(col, np.int64)
    u = np.zeros((n, H, F), dt)
    np.add.at(u, rows, attd[:, :, None] * hc[col64])
    # isolated rows: uniform 1/M over every column (softmax of an all -9e15 row)
    if empty.any():
        u[empty] = hc.mean(axis=0, dtype=dt)[None] if keep is None else u[empty]
    v = None
    if hs is not None:
        v = np.zeros((m_cols, H, F), dt)
        np.add.at(v, col64, attd[:, :, None] * hs[rows])
        if empty.any() and keep is None:
            v += hs[empty].sum(axis=0) / np.asarray(m_cols, dt)
    return dict(att=att, attd=attd, u=u, v=v, pre=pre, empty=empty, rowflag=rowflag)


def edge_aggregate_bwd(rowptr, col, fwd, hc, dU, hs=None, dV=None, keep=None, p=0.0,
                       slope=NEG_SLOPE):
    """Backward of ``edge_aggregate_fwd`` (autograd of Ablation.py:266-274).

    Returns dict(d_el (N,H), d_er (M,H), d_hc (M,H,F), d_hs (N,H,F) or None).
    Rows without edges contribute only through their uniform attention (no score
    gradient), matching the reference's ``where`` mask.
    """
    dt = hc.dtype
    n = len(rowptr) - 1
    m_cols, H, F = hc.shape
    rows = edge_rows(rowptr)
    col64 = np.asarray(col, np.int64)
    att, attd, pre = fwd["att"], fwd["attd"], fwd["pre"]
    g = np.einsum("ehf,ehf->eh", dU[rows], hc[col64])
    if dV is not None:
        g = g + np.einsum("ehf,ehf->eh", dV[col64], hs[rows])
    if keep is not None:
        g = g * keep * np.asarray(1.0 / (1.0 - p), dt)
    dot = _seg_reduce(att * g, rowptr, np.add, 0)
    ds = att * (g - dot[rows])
    de = ds * lrelu_grad(pre, slope)
    if fwd.get("rowflag") is not None:
        de = np.where(np.asarray(fwd["rowflag"], bool)[rows][:, None], np.asarray(0, de.dtype), de)
    d_el = _seg_reduce(de, rowptr, np.add, 0)
    d_er = np.zeros((m_cols, H), dt)
    np.add.at(d_er, col64, de)
    d_hc = np.zeros((m_cols, H, F), dt)
    np.add.at(d_hc, col64, attd[:, :, None] * dU[rows])
    empty = fwd["empty"]
    if empty.any() and keep is None:
        d_hc += dU[empty].sum(axis=0) / np.asarray(m_cols, dt)
    d_hs = None
    if dV is not None:
        d_hs = np.zeros((n, H, F), dt)
        np.add.at(d_hs, rows, attd[:, :, None] * dV[col64])
        if empty.any() and keep is None:
            d_hs[empty] = dV.sum(axis=0) / np.asarray(m_cols, dt)
    return dict(d_el=d_el, d_er=d_er, d_hc=d_hc, d_hs=d_hs, de=de)


# ----------------------------------------------------------------------------------
# GraphAttentionLayer (GAT.py:20-35, Ablation.py:100-115)
# ----------------------------------------------------------------------------------
def gal_attention(rowptr, n_cols):
    """The GAL's attention is ``mask / deg`` (score is constant along a row:
    GAT.py:24-27 concatenates h_i with itself); empty rows are uniform 1/M."""
    deg = np.diff(np.asarray(rowptr, np.int64))
    return deg


def gal_fwd(x, W, rowptr, col, keep=None, p=0.0):
    """``elu(dropout(mask/deg) * (x @ W))`` (GAT.py:21-35).  Returns (out, h, att_dense)."""
    h = x @ W
    n, m = h.shape
    dt = h.dtype
    rows = edge_rows(rowptr)
    deg = np.diff(np.asarray(rowptr, np.int64))
    att = np.zeros((n, m), dt)
    inv = np.asarray(1, dt) / np.maximum(deg, 1).astype(dt)
    att[rows, np.asarray(col, np.int64)] = inv[rows]
    att[deg == 0] = np.asarray(1, dt) / np.asarray(m, dt)
    if keep is not None:
        att = att * keep * np.asarray(1.0 / (1.0 - p), dt)
    z = att * h
    return elu(z), h, att


def gal_bwd(x, W, h, att, dout):
    z = att * h
    dz = dout * elu_grad(z)
    dh = dz * att
    return dict(dx=dh @ W.T, dW=x.T @ dh, dh=dh)


# ----------------------------------------------------------------------------------
# OursLayer3 / ablation3 (Ablation.py:235-301), full forward (dense epilogue)
# ----------------------------------------------------------------------------------
def batchnorm_train(x, gamma, beta, eps=1e-5):
    mu = x.mean(axis=0)
    var = x.var(axis=0)  # biased, as BatchNorm1d normalises with
    return (x - mu) / np.sqrt(var + np.asarray(eps, x.dtype)) * gamma + beta


def batchnorm_eval(x, gamma, beta, rmean, rvar, eps=1e-5):
    return (x - rmean) / np.sqrt(rvar + np.asarray(eps, x.dtype)) * gamma + beta


def ours_layer3_fwd(S, R, p, rowptr, col, training, slope=NEG_SLOPE):
    """OursLayer3.forward restated (Ablation.py:260-277), dropout off.

    ``p`` holds W1, W2, a, bn1_*, bn2_* numpy arrays.  Returns dict with u_pre,
    v_pre (the BatchNorm inputs), att, out.
    """
    h1 = R @ p["W1"]
    h2 = S @ p["W2"]
    F = h1.shape[1]
    a = p["a"].reshape(-1)
    er = (h1 @ a[:F])[:, None]
    el = (h2 @ a[F:])[:, None]
    fw = edge_aggregate_fwd(rowptr, col, el, er, h1[:, None, :], hs=h2[:, None, :],
                            slope=slope)
    u_pre = fw["u"][:, 0, :]
    v_pre = fw["v"][:, 0, :]
    if training:
        v = batchnorm_train(v_pre, p["bn1_weight"], p["bn1_bias"])
        u = batchnorm_train(u_pre, p["bn2_weight"], p["bn2_bias"])
    else:
        v = batchnorm_eval(v_pre, p["bn1_weight"], p["bn1_bias"], p["bn1_running_mean"],
                           p["bn1_running_var"])
        u = batchnorm_eval(u_pre, p["bn2_weight"], p["bn2_bias"], p["bn2_running_mean"],
                           p["bn2_running_var"])
    out = elu(lrelu(u, slope) @ lrelu(v, slope).T)
    return dict(h1=h1, h2=h2, el=el, er=er, att=fw["att"][:, 0], u_pre=u_pre,
                v_pre=v_pre, out=out)


def log_softmax(x, axis=1):
    m = x.max(axis=axis, keepdims=True)
    z = x - m
    return z - np.log(np.exp(z).sum(axis=axis, keepdims=True))


def ablation3_fwd(Sf, Rf, heads, out_W, rowptr, col, training):
    """ablation3.forward restated (Ablation.py:295-301) with dropout off."""
    xs = [ours_layer3_fwd(Sf, Rf, hp, rowptr, col, training)["out"] for hp in heads]
    x = np.concatenate(xs, axis=1)
    y, _, _ = gal_fwd(x, out_W, rowptr, col)
    return log_softmax(elu(y))


def gat_fwd(feat, head_Ws, out_W, rowptr, col):
    """GAT.forward restated (GAT.py:53-58) with dropout off."""
    x = np.concatenate([gal_fwd(feat, W, rowptr, col)[0] for W in head_Ws], axis=1)
    y, _, _ = gal_fwd(x, out_W, rowptr, col)
    return log_softmax(elu(y))


# ----------------------------------------------------------------------------------
# LinkPredictor (LLP.py:86-115) and the caller's pair gather (LLP.py:233)
# ----------------------------------------------------------------------------------
def link_predict(x_i, x_j, mode, lins=(), keep=None, p=0.0):
    """``sigmoid(relu(x_i*x_j @ W0.T + b0))`` for 'mlp' (lins[:-1] only: LLP.py:107-111,
    the last Linear is never applied), ``sigmoid(sum(x_i*x_j))`` for 'inner', and
    ``sigmoid(x_i*x_j)`` (B, F) for any other predictor string (LLP.py:104-115)."""
    x = x_i * x_j
    if mode == "mlp":
        for li, (W, b) in enumerate(lins[:-1]):
            x = np.maximum(x @ W.T + b, 0)
            if keep is not None:
                x = x * keep[li] * np.asarray(1.0 / (1.0 - p), x.dtype)
    elif mode == "inner":
        x = x.sum(axis=-1)
    return 1.0 / (1.0 + np.exp(-x))


def score_pairs(h, src, dst, mode, lins=()):
    """Fused caller gather + predictor: ``predictor(h[src], h[dst])`` (LLP.py:233)."""
    h = np.asarray(h)
    return link_predict(h[np.asarray(src, np.int64)], h[np.asarray(dst, np.int64)], mode,
                        lins)


def link_predict_bwd(x_i, x_j, mode, lins, dout):
    """Gradients of ``link_predict`` (no dropout) w.r.t. x_i, x_j and the used Linear."""
    x = x_i * x_j
    if mode == "inner":
        s = 1.0 / (1.0 + np.exp(-x.sum(axis=-1)))
        dz = dout * s * (1 - s)
        dx = dz[:, None] * np.ones_like(x)
        return dict(dx_i=dx * x_j, dx_j=dx * x_i)
    if mode != "mlp":  # neither branch (LLP.py:106-113): y = sigmoid(x_i * x_j)
        s = 1.0 / (1.0 + np.exp(-x))
        dx = dout * s * (1 - s)
        return dict(dx_i=dx * x_j, dx_j=dx * x_i)
    W, b = lins[0]
    z = x @ W.T + b
    r = np.maximum(z, 0)
    s = 1.0 / (1.0 + np.exp(-r))
    dr = dout * s * (1 - s)
    dz = dr * (z > 0)
    dx = dz @ W
    return dict(dx_i=dx * x_j, dx_j=dx * x_i, dW=dz.T @ x, db=dz.sum(axis=0))


# ----------------------------------------------------------------------------------
# Ours.OursLayer (full MSHA: inter + city/province intra attention), Ours.py:54-109
# ----------------------------------------------------------------------------------
def ours_intra(h2, a3, a4, src, city, prov, attd_rows, n_cols, keep3=None, keep4=None, p=0.0,
               slope=NEG_SLOPE):
    """Intra-source attention of a batch (Ours.py:71-99), one head.

    e3_b = lrelu(h2_b . (a3[:F] + a3[F:])) is constant along n (Ours.py:74-75 concatenate
    h2_b with itself); the mask is "same city" (Ours.py:81).  SUM_b (Ours.py:84-86) adds,
    WITHOUT max subtraction, exp of the masked scores and exp of the batch row's
    post-dropout inter attention over ALL n_cols columns (non-edges give exp(0) = 1).
    attd_rows: (B, n_cols) dense post-dropout inter attention of rows src.
    Returns dict(intra (N,F), w3, w4, SUM, pre3, pre4)."""
    dt = h2.dtype
    F = h2.shape[1]
    a3 = a3.reshape(-1)
    a4 = a4.reshape(-1)
    hb = h2[np.asarray(src, np.int64)]
    pre3 = hb @ (a3[:F] + a3[F:]) if False else hb @ a3[:F] + hb @ a3[F:]
    pre4 = hb @ a4[:F] + hb @ a4[F:]
    E3, E4 = np.exp(lrelu(pre3, slope)), np.exp(lrelu(pre4, slope))
    m3 = (np.asarray(city)[np.asarray(src)][:, None] == np.asarray(city)[None, :]).astype(dt)
    m4 = (np.asarray(prov)[np.asarray(src)][:, None] == np.asarray(prov)[None, :]).astype(dt)
    SUM = m3.sum(1) * E3 + m4.sum(1) * E4 + np.exp(attd_rows).sum(1)
    att3 = m3 * (E3 / SUM)[:, None]
    att4 = m4 * (E4 / SUM)[:, None]
    if keep3 is not None:
        s = np.asarray(1.0 / (1.0 - p), dt)
        att3 = att3 * keep3 * s
        att4 = att4 * keep4 * s
    intra = att3.T @ hb + att4.T @ hb
    return dict(intra=intra, w3=E3 / SUM, w4=E4 / SUM, SUM=SUM, pre3=pre3, pre4=pre4,
                att3=att3, att4=att4)


def ours_layer_fwd(S, R, p, rowptr, col, city, prov, src, training, rowflag=None,
                   slope=NEG_SLOPE):
    """OursLayer.forward restated (Ours.py:54-109) with dropout off."""
    h1 = R @ p["W1"]
    h2 = S @ p["W2"]
    F = h1.shape[1]
    a = p["a"].reshape(-1)
    er = (h1 @ a[:F])[:, None]
    el = (h2 @ a[F:])[:, None]
    m_cols = h1.shape[0]
    fw = edge_aggregate_fwd(rowptr, col, el, er, h1[:, None, :], hs=h2[:, None, :],
                            slope=slope, rowflag=rowflag)
    rows = edge_rows(rowptr)
    dense = np.zeros((len(rowptr) - 1, m_cols), h1.dtype)
    dense[rows, np.asarray(col, np.int64)] = fw["attd"][:, 0]
    it = ours_intra(h2, p["a3"], p["a4"], src, city, prov, dense[np.asarray(src)], m_cols,
                    slope=slope)
    u_pre = fw["u"][:, 0, :] + it["intra"]
    v_pre = fw["v"][:, 0, :]
    if training:
        v = batchnorm_train(v_pre, p["bn1_weight"], p["bn1_bias"])
        u = batchnorm_train(u_pre, p["bn2_weight"], p["bn2_bias"])
    else:
        v = batchnorm_eval(v_pre, p["bn1_weight"], p["bn1_bias"], p["bn1_running_mean"],
                           p["bn1_running_var"])
        u = batchnorm_eval(u_pre, p["bn2_weight"], p["bn2_bias"], p["bn2_running_mean"],
                           p["bn2_running_var"])
    out = elu(lrelu(u, slope) @ lrelu(v, slope).T)
    return dict(out=out, u_pre=u_pre, v_pre=v_pre, intra=it)


# ------------------------------------------------------------------------- GCN ---
def spmm_t(rowptr, col, vals, table, n_cols):
    """``A^T @ table`` over the CSR edges with values ``vals`` (model.py:37)."""
    rows = edge_rows(rowptr)
    out = np.zeros((n_cols, table.shape[1]), table.dtype)
    np.add.at(out, col, vals[:, None] * table[rows])
    return out


def spmm(rowptr, col, vals, table):
    """``A @ table`` over the CSR edges (model.py:37 with adj.t(), model.py:62)."""
    rows = edge_rows(rowptr)
    out = np.zeros((len(rowptr) - 1, table.shape[1]), table.dtype)
    np.add.at(out, rows, vals[:, None] * table[col])
    return out


def gcn_fwd(features, W1, b1, W2, b2, rowptr, col, vals, n_cols):
    """model.py:57-64 (dropout 0): relu(A^T (X W1) + b1) -> relu(A (x W2) + b2) ->
    log_softmax; b1 / b2 are the reference's scalar biases (model.py:23)."""
    x = np.maximum(spmm_t(rowptr, col, vals, features @ W1, n_cols) + b1, 0)
    x = np.maximum(spmm(rowptr, col, vals, x @ W2) + b2, 0)
    return log_softmax(x, axis=1)
