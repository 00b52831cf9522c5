"""Pin the CPU oracle (oracle/gnn_oracle.py) against the reference's golden vectors.

The fixtures were produced by running the reference's own modules
(tests/golden/make_golden.py).  fp64 runs of the reference must be reproduced to
~1e-10 by the oracle run in fp64; fp32 to the fp32 rounding level.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import gnn_oracle as O


def _heads(z, prefix, n_heads, dt):
    heads = []
    for h in range(n_heads):
        p = {}
        for k in ("W1", "W2", "a"):
            p[k] = z[f"{prefix}attention_{h}.{k}"].astype(dt)
        for bn in ("bn1", "bn2"):
            for k in ("weight", "bias", "running_mean", "running_var"):
                p[f"{bn}_{k}"] = z[f"{prefix}attention_{h}.{bn}.{k}"].astype(dt)
        heads.append(p)
    return heads


def _heads_eval(z, heads, tag, dt):
    """eval() ran after the train forward, so BN running stats had moved once."""
    for h, p in enumerate(heads):
        for bn in ("bn1", "bn2"):
            for k in ("running_mean", "running_var"):
                p[f"{bn}_{k}"] = z[f"after{tag}.attention_{h}.{bn}.{k}"].astype(dt)
    return heads


def _sub512_inputs(z, dt):
    rowptr, col = O.dense_to_csr(z["adj_norm"])
    return rowptr, col, z["init.Sfeatures"].astype(dt), z["init.Rfeatures"].astype(dt)


def test_r15_graph_counts_and_normalize():
    g = golden("r15_graph.npz")
    n, m = int(g["n"]), int(g["m"])
    rowptr, col, cnt = g["rowptr"], g["col"].astype(np.int32), g["cnt"].astype(np.float32)
    assert n == 39179 and m == 32 and len(col) == 91283 and int(g["n_flows"]) == 233887
    dense = np.zeros((n, m), np.float32)
    dense[O.edge_rows(rowptr), col] = cnt
    # oracle CSR == reference mask order (row-major nonzero)
    r2, c2 = O.dense_to_csr(dense)
    np.testing.assert_array_equal(r2, rowptr)
    np.testing.assert_array_equal(c2, col)
    # reference normalize_adjacency_matrix values, bit-exact
    norm = O.normalize_adjacency(dense)
    np.testing.assert_array_equal(norm[dense > 0], g["norm"])
    assert np.all(norm[dense == 0] == 0)
    assert np.diff(rowptr).min() >= 1 and np.diff(rowptr).max() == 30


def test_inter_adjacency_counts_match_reference():
    z = golden("sub512.npz")
    fl = z["flows"]
    adj = O.inter_adjacency(fl[:, 0], fl[:, 1], 512, 32)
    np.testing.assert_array_equal(adj, z["counts"])


def test_normalize_edge_cases():
    e = golden("edge_cases.npz")
    np.testing.assert_array_equal(O.normalize_adjacency(e["norm_rand_in"]), e["norm_rand_out"])
    out = O.normalize_adjacency(e["norm_zero_col_in"])
    assert np.isnan(e["norm_zero_col_out"]).all() and np.isnan(out).all()
    np.testing.assert_array_equal(O.normalize_adjacency(e["counts"]), e["adj_norm32"])


@pytest.mark.parametrize("dt,tol", [(np.float64, 1e-10), (np.float32, 2e-5)])
def test_ours_layer3_intermediates(dt, tol):
    z = golden("sub512.npz")
    rowptr, col, S, R = _sub512_inputs(z, dt)
    tag = "64" if dt == np.float64 else "32"
    for h, p in enumerate(_heads(z, "init.", 2, dt)):
        r = O.ours_layer3_fwd(S, R, p, rowptr, col, training=True)
        np.testing.assert_allclose(r["u_pre"], z[f"bn{tag}.h{h}_u_pre"], rtol=tol, atol=tol)
        vref = z[f"bn{tag}.h{h}_v_pre"]
        np.testing.assert_allclose(r["v_pre"], vref, rtol=tol, atol=tol * np.abs(vref).max())
        if dt == np.float32:
            att = np.zeros((512, 32), dt)
            att[O.edge_rows(rowptr), col] = r["att"]
            np.testing.assert_allclose(att, z[f"sm32.h{h}_att"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dt,tol", [(np.float64, 1e-9), (np.float32, 1e-4)])
def test_ablation3_forward(dt, tol):
    z = golden("sub512.npz")
    rowptr, col, S, R = _sub512_inputs(z, dt)
    heads = _heads(z, "init.", 2, dt)
    W = z["init.out_att.W"].astype(dt)
    tag = "64" if dt == np.float64 else "32"
    out = O.ablation3_fwd(S, R, heads, W, rowptr, col, training=True)
    np.testing.assert_allclose(out, z[f"out{tag}"], rtol=tol, atol=tol)
    heads = _heads_eval(z, heads, tag, dt)
    out_eval = O.ablation3_fwd(S, R, heads, W, rowptr, col, training=False)
    np.testing.assert_allclose(out_eval, z[f"out_eval{tag}"], rtol=tol, atol=tol)


def test_gat_forward():
    z = golden("gat_sub512.npz")
    s = golden("sub512.npz")
    rowptr, col = O.dense_to_csr(s["adj_norm"])
    out = O.gat_fwd(z["init.features"], [z["init.attention_0.W"], z["init.attention_1.W"]],
                    z["init.out_att.W"], rowptr, col)
    np.testing.assert_allclose(out, z["out"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("tag", ["32", "64"])
def test_edge_cases_layer(tag):
    e = golden("edge_cases.npz")
    dt = np.float64 if tag == "64" else np.float32
    tol = 1e-9 if tag == "64" else 2e-4
    adj = e[f"adj_norm{tag}"]
    rowptr, col = O.dense_to_csr(adj)
    deg = np.diff(rowptr)
    assert deg[0] == 0 and deg[1] == 1 and deg[2] == 80 and deg[3] == 65
    p = {k: e[f"ol3.init.{k}"].astype(dt) for k in ("W1", "W2", "a")}
    for bn in ("bn1", "bn2"):
        for k in ("weight", "bias", "running_mean", "running_var"):
            p[f"{bn}_{k}"] = e[f"ol3.init.{bn}.{k}"].astype(dt)
    S, R = e[f"ol3.S{tag}"], e[f"ol3.R{tag}"]
    r = O.ours_layer3_fwd(S, R, p, rowptr, col, training=True)
    att = np.zeros(adj.shape, dt)
    att[O.edge_rows(rowptr), col] = r["att"]
    att[deg == 0] = 1.0 / adj.shape[1]
    np.testing.assert_allclose(att, e[f"ol3.att{tag}"], rtol=1e-6, atol=1e-7)
    ref = e[f"ol3.out{tag}"]
    np.testing.assert_allclose(r["out"], ref, rtol=tol, atol=tol * np.abs(ref).max())
    r = O.ours_layer3_fwd(S, R, p, rowptr, col, training=False)
    ref = e[f"ol3.out_eval{tag}"]
    np.testing.assert_allclose(r["out"], ref, rtol=tol, atol=tol * np.abs(ref).max())
    # GAL over the same 80-column adjacency (degree 0 / 1 / 80 / 65 rows)
    x = e[f"gal.x{tag}"]
    W = e["gal.init.W"].astype(dt)
    out, h, attd = O.gal_fwd(x, W, rowptr, col)
    np.testing.assert_allclose(out, e[f"gal.out{tag}"], rtol=tol, atol=tol)
    g = O.gal_bwd(x, W, h, attd, e[f"gal.dout{tag}"].astype(dt))
    np.testing.assert_allclose(g["dx"], e[f"gal.grad{tag}.x"], rtol=tol, atol=tol)
    np.testing.assert_allclose(g["dW"], e[f"gal.grad{tag}.W"], rtol=tol, atol=tol)
    assert np.abs(e[f"gal.grad{tag}.a"]).max() < 1e-5  # reference grad of GAL.a is ~0


def test_link_predictor():
    z = golden("link.npz")
    xi, xj = z["x_i"], z["x_j"]
    for mode, pred in (("mlp", "mlp"), ("inner", "inner"), ("mlp1", "mlp"), ("other", "dot")):
        lins = [(z[f"{mode}.init.lins.0.weight"], z[f"{mode}.init.lins.0.bias"]),
                (z[f"{mode}.init.lins.1.weight"], z[f"{mode}.init.lins.1.bias"])]
        y = O.link_predict(xi, xj, pred, lins)
        assert y.shape == z[f"{mode}.out"].shape
        np.testing.assert_allclose(y, z[f"{mode}.out"], rtol=1e-6, atol=1e-6)
        g = O.link_predict_bwd(xi, xj, pred, lins, z[f"{mode}.dout"])
        np.testing.assert_allclose(g["dx_i"], z[f"{mode}.grad.x_i"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g["dx_j"], z[f"{mode}.grad.x_j"], rtol=1e-5, atol=1e-6)
        if pred == "mlp":
            np.testing.assert_allclose(g["dW"], z[f"{mode}.grad.lins.0.weight"], rtol=1e-5,
                                       atol=1e-6)
            np.testing.assert_allclose(g["db"], z[f"{mode}.grad.lins.0.bias"], rtol=1e-5,
                                       atol=1e-6)


def test_llp_teacher_fixtures():
    """LLP.py's teacher GAT (forward(input, adj), LLP.py:148-168) and
    Teacher_LinkPredictor (LLP.py:170-198) as the reference computed them (llp.npz):
    the oracle's GAT / link-predictor restatements reproduce them."""
    z = golden("llp.npz")
    s = golden("sub512.npz")
    rowptr, col = O.dense_to_csr(s["adj_norm"])
    out = O.gat_fwd(z["gat.input"], [z["gat.init.attention_0.W"], z["gat.init.attention_1.W"]],
                    z["gat.init.out_att.W"], rowptr, col)
    np.testing.assert_allclose(out, z["gat.out"], rtol=1e-5, atol=1e-5)
    xi, xj = z["tlp.x_i"], z["tlp.x_j"]
    for mode, pred, nl in (("mlp", "mlp", 2), ("mlp3", "mlp", 3), ("inner", "inner", 2),
                           ("other", "cos", 2)):
        lins = [(z[f"tlp.{mode}.init.lins.{i}.weight"], z[f"tlp.{mode}.init.lins.{i}.bias"])
                for i in range(nl)]
        y = O.link_predict(xi, xj, pred, lins)
        assert y.shape == z[f"tlp.{mode}.out"].shape
        np.testing.assert_allclose(y, z[f"tlp.{mode}.out"], rtol=1e-6, atol=1e-6)


def _dense_core_torch(rowptr, col, el, er, hc, hs, n_cols):
    """Dense torch restatement of the masked-softmax core for autograd (fp64)."""
    n = len(rowptr) - 1
    mask = torch.zeros(n, n_cols, dtype=torch.bool)
    mask[torch.as_tensor(O.edge_rows(rowptr)), torch.as_tensor(col, dtype=torch.long)] = True
    e = torch.nn.functional.leaky_relu(el[:, None, :] + er[None, :, :], 0.2)  # (N,M,H)
    e = torch.where(mask[:, :, None], e, torch.full_like(e, -9e15))
    att = torch.softmax(e, dim=1)
    u = torch.einsum("nmh,mhf->nhf", att, hc)
    v = torch.einsum("nmh,nhf->mhf", att, hs)
    return u, v


def test_edge_aggregate_bwd_matches_autograd():
    rng = np.random.default_rng(0)
    e = golden("edge_cases.npz")
    rowptr, col = O.dense_to_csr(e["counts"])
    n, m, H, F = 40, 80, 2, 3
    el, er = rng.standard_normal((n, H)), rng.standard_normal((m, H))
    hc, hs = rng.standard_normal((m, H, F)), rng.standard_normal((n, H, F))
    dU, dV = rng.standard_normal((n, H, F)), rng.standard_normal((m, H, F))
    fw = O.edge_aggregate_fwd(rowptr, col, el, er, hc, hs=hs)
    bw = O.edge_aggregate_bwd(rowptr, col, fw, hc, dU, hs=hs, dV=dV)
    t = [torch.tensor(x, requires_grad=True) for x in (el, er, hc, hs)]
    u, v = _dense_core_torch(rowptr, col, *t, m)
    np.testing.assert_allclose(fw["u"], u.detach().numpy(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(fw["v"], v.detach().numpy(), rtol=1e-12, atol=1e-12)
    ((u * torch.tensor(dU)).sum() + (v * torch.tensor(dV)).sum()).backward()
    for name, ref in zip(("d_el", "d_er", "d_hc", "d_hs"), t):
        np.testing.assert_allclose(bw[name], ref.grad.numpy(), rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("tag,tol", [("", 2e-4), ("B.", 1e-9)])
def test_ours_layer_forward(tag, tol):
    """Full MSHA layer (Ours.py:54-109): inter + same-city / same-province attention."""
    z = golden("ours_small.npz")
    dt = np.float64 if tag else np.float32
    counts = z[tag + "counts"] if tag + "counts" in z.files else z["counts"]
    mask = counts > 0
    empty = ~mask.any(1)
    mask[empty] = True
    rowptr, col = O.dense_to_csr(mask.astype(np.float32))
    p = {k: z[f"init.{k}"].astype(dt) for k in ("W1", "W2", "a", "a3", "a4")}
    for bn in ("bn1", "bn2"):
        for k in ("weight", "bias", "running_mean", "running_var"):
            p[f"{bn}_{k}"] = z[f"init.{bn}.{k}"].astype(dt)
    S, R, src = z[tag + "S"].astype(dt), z[tag + "R"].astype(dt), z[tag + "source_index"]
    for training, key in ((True, "out"), (False, "out_eval")):
        r = O.ours_layer_fwd(S, R, p, rowptr, col, z["city"], z["prov"], src, training,
                             rowflag=empty)
        ref = z[tag + key]
        np.testing.assert_allclose(r["out"], ref, rtol=tol, atol=tol * np.abs(ref).max())


def test_gcn_oracle_matches_reference():
    """model.GCN (model.py:48-64) on the sub512 graph: oracle SpMM restatement vs the
    reference's own dense forward (fixture from make_golden.py)."""
    z = golden("gcn_sub512.npz")
    s = golden("sub512.npz")
    adj = s["adj_norm"].astype(np.float64)
    rowptr, col = O.dense_to_csr((s["counts"] > 0).astype(np.float32))
    rows = O.edge_rows(rowptr)
    vals = adj[rows, col]
    out = O.gcn_fwd(z["init.features"].astype(np.float64), z["init.gc1.weight"].astype(np.float64),
                    float(z["init.gc1.bias"]), z["init.gc2.weight"].astype(np.float64),
                    float(z["init.gc2.bias"]), rowptr, col, vals, adj.shape[1])
    np.testing.assert_allclose(out, z["out"], rtol=1e-4, atol=1e-5)


def _torch_heads(z, prefix, n_heads):
    return [{k: torch.as_tensor(v) for k, v in h.items()}
            for h in _heads(z, prefix, n_heads, np.float64)]


def test_dense_ref_matches_reference():
    """tests/dense_ref.py (the fp64 torch restatement the full-size GPU tests use for
    gradients) reproduces the reference's fp64 runs: ablation3 train forward, loss and
    parameter gradients (sub512), OursLayer train/eval outputs and gradients (ours_small
    case B)."""
    import dense_ref as D

    z = golden("sub512.npz")
    mask = torch.as_tensor(z["adj_norm"] > 0)
    heads = _torch_heads(z, "init.", 2)
    for p in heads:
        for k in ("W1", "W2", "a", "bn1_weight", "bn1_bias", "bn2_weight", "bn2_bias"):
            p[k].requires_grad_(True)
    Sf = torch.as_tensor(z["init.Sfeatures"], dtype=torch.float64).requires_grad_(True)
    Rf = torch.as_tensor(z["init.Rfeatures"], dtype=torch.float64).requires_grad_(True)
    oW = torch.as_tensor(z["init.out_att.W"], dtype=torch.float64).requires_grad_(True)
    out = D.model(Sf, Rf, heads, oW, mask, True)
    np.testing.assert_allclose(out.detach().numpy(), z["out64"], rtol=1e-10, atol=1e-10)
    si = torch.as_tensor(z["source_index"])
    loss = torch.nn.functional.nll_loss(out[si], torch.as_tensor(z["recipient_index"]))
    assert abs(float(loss.detach()) - float(z["loss64"])) < 1e-12
    loss.backward()
    np.testing.assert_allclose(Rf.grad.numpy(), z["grad64.Rfeatures"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(oW.grad.numpy(), z["grad64.out_att.W"], rtol=1e-9, atol=1e-12)
    for h, p in enumerate(heads):
        for k in ("W1", "W2", "a", "bn1_weight", "bn1_bias", "bn2_weight", "bn2_bias"):
            ref = z[f"grad64.attention_{h}.{k.replace('_', '.')}"]
            np.testing.assert_allclose(p[k].grad.numpy(), ref, rtol=1e-8,
                                       atol=1e-10 * np.abs(ref).max())

    o = golden("ours_small.npz")
    p = {k: torch.as_tensor(o[f"init.{k}"], dtype=torch.float64).requires_grad_(True)
         for k in ("W1", "W2", "a", "a3", "a4")}
    for bn in ("bn1", "bn2"):
        for k in ("weight", "bias", "running_mean", "running_var"):
            p[f"{bn}_{k}"] = torch.as_tensor(o[f"init.{bn}.{k}"], dtype=torch.float64)
        p[f"{bn}_weight"].requires_grad_(True)
        p[f"{bn}_bias"].requires_grad_(True)
    mask = torch.as_tensor(o["B.counts"] > 0)
    city, prov = torch.as_tensor(o["city"]), torch.as_tensor(o["prov"])
    src = torch.as_tensor(o["B.source_index"])
    S = torch.as_tensor(o["B.S"]).requires_grad_(True)
    R = torch.as_tensor(o["B.R"]).requires_grad_(True)
    y = D.ours_layer(S, R, p, mask, city, prov, src, False)
    np.testing.assert_allclose(y.detach().numpy(), o["B.out_eval"], rtol=1e-10, atol=1e-10)
    y = D.ours_layer(S, R, p, mask, city, prov, src, True)
    np.testing.assert_allclose(y.detach().numpy(), o["B.out"], rtol=1e-10, atol=1e-10)
    (y * torch.as_tensor(o["B.dout"])).sum().backward()
    np.testing.assert_allclose(S.grad.numpy(), o["B.grad.S"], rtol=1e-8, atol=1e-12)
    np.testing.assert_allclose(R.grad.numpy(), o["B.grad.R"], rtol=1e-8, atol=1e-12)
    for k in ("W1", "W2", "a", "a3", "a4", "bn1_weight", "bn1_bias", "bn2_weight", "bn2_bias"):
        ref = o[f"B.grad.{k.replace('_', '.')}"]
        np.testing.assert_allclose(p[k].grad.numpy(), ref, rtol=1e-8,
                                   atol=1e-10 * np.abs(ref).max())


def test_record_fixture_semantics():
    """ours_record.npz (Ours.py:92-96 record mode, eval): train.Coeff12new is the dense
    post-softmax inter attention (rows sum to 1 over the edges); Coeff3 / Coeff4 rows of
    the recorded batches are the same-group masks times E/SUM (one value per row)."""
    r = golden("ours_record.npz")
    o = golden("ours_small.npz")
    mask = o["counts"] > 0
    for k in (0, 1):
        c12 = r[f"rec.coeff12new.{k}"]
        np.testing.assert_allclose(c12.sum(1), 1.0, rtol=1e-5)
        assert np.all(c12[~mask] == 0)
    same = o["city"][:, None] == o["city"][None, :]
    c3 = r["rec.coeff3"]
    assert np.all(c3[~same] == 0) and np.all(c3[same] > 0)


def _dense_params(z):
    """oracle/dense_step parameters from the sub512 fixture's initial state."""
    t = lambda k: torch.tensor(z[k]).double().requires_grad_(True)  # noqa: E731
    heads = []
    for h in range(2):
        d = {k: t(f"init.attention_{h}.{k}") for k in ("W1", "W2", "a")}
        for bn in ("bn1", "bn2"):
            for k in ("weight", "bias"):
                d[f"{bn}_{k}"] = t(f"init.attention_{h}.{bn}.{k}")
            for k in ("running_mean", "running_var"):
                d[f"{bn}_{k}"] = torch.tensor(z[f"init.attention_{h}.{bn}.{k}"]).double()
        heads.append(d)
    return {"Sfeatures": t("init.Sfeatures"), "Rfeatures": t("init.Rfeatures"), "heads": heads,
            "out_W": t("init.out_att.W"), "out_a": t("init.out_att.a")}


def test_dense_step_matches_reference_train_step():
    """oracle/dense_step (the CPU baseline of configs[1]) restates the reference's
    ablation3 step: fp64 output, loss, every gradient and the BN running statistics
    after one train forward vs the reference's own fp64 run (dropout 0)."""
    from oracle import dense_step

    z = golden("sub512.npz")
    p = _dense_params(z)
    adj = torch.tensor(z["adj_norm"]).double()
    si, ri = torch.tensor(z["source_index"]), torch.tensor(z["recipient_index"])
    out = dense_step.ablation3(p, adj, 0.0, True)
    np.testing.assert_allclose(out.detach().numpy(), z["out64"], rtol=1e-9, atol=1e-9)
    loss = torch.nn.functional.nll_loss(out[si], ri)
    assert abs(float(loss.detach()) - float(z["loss64"])) < 1e-9
    loss.backward()
    names = {"Sfeatures": p["Sfeatures"], "Rfeatures": p["Rfeatures"], "out_att.W": p["out_W"]}
    for h, d in enumerate(p["heads"]):
        for k in ("W1", "W2", "a"):
            names[f"attention_{h}.{k}"] = d[k]
        for bn in ("bn1", "bn2"):
            names[f"attention_{h}.{bn}.weight"] = d[f"{bn}_weight"]
            names[f"attention_{h}.{bn}.bias"] = d[f"{bn}_bias"]
    for k, v in names.items():
        # the fixture holds the (512, 128) Sfeatures gradient only from the fp32 run
        tol = 1e-7 if f"grad64.{k}" in z.files else 1e-5
        ref = z[f"grad64.{k}"] if f"grad64.{k}" in z.files else z[f"grad32.{k}"]
        np.testing.assert_allclose(v.grad.numpy(), ref, rtol=tol,
                                   atol=tol * max(1e-2, np.abs(ref).max()), err_msg=k)
    for h, d in enumerate(p["heads"]):
        for bn in ("bn1", "bn2"):
            for k in ("running_mean", "running_var"):
                np.testing.assert_allclose(d[f"{bn}_{k}"].numpy(),
                                           z[f"after64.attention_{h}.{bn}.{k}"], rtol=1e-9,
                                           atol=1e-12)


def test_dense_step_score_pairs_matches_reference():
    """oracle/dense_step.score_pairs vs the reference LinkPredictor fixture (eval)."""
    from oracle import dense_step

    z = golden("link.npz")
    h = torch.cat([torch.tensor(z["x_i"]), torch.tensor(z["x_j"])])
    src = torch.arange(256)
    dst = src + 256
    for mode, pred in (("mlp", "mlp"), ("inner", "inner"), ("other", "dot")):
        W = torch.tensor(z[f"{mode}.init.lins.0.weight"])
        b = torch.tensor(z[f"{mode}.init.lins.0.bias"])
        got = dense_step.score_pairs(h, src, dst, pred, W, b).numpy()
        np.testing.assert_allclose(got, z[f"{mode}.out"], rtol=1e-6, atol=1e-7, err_msg=mode)
