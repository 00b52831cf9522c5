"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run in the build container only (the reference is absent on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own modules from /root/reference (GAT.py, Ablation.py,
model.py; LinkPredictor from LLP.py, OursLayer from Ours.py and
HigherDataset.inter_adjacent from dataset.py by AST extraction, because those
files run training scripts / open absolute paths at import), runs them on seeded
inputs and writes inputs, parameters, outputs and gradients as .npz.  Nothing of
the reference's source is written out: only arrays.

Fixtures
  r15_graph.npz   shipped 2015 graph: CSR of the flow-count adjacency produced by
                  the reference's own ``inter_adjacent`` (dataset.py:279-296), the
                  reference ``normalize_adjacency_matrix`` values on the edges
                  (model.py:95-100), group ids and GDP.
  sub512.npz      ablation3 (in 128, F 64, 2 heads) on a 512-source induced subgraph
                  of 2015: seeded init state_dict, train/eval outputs, loss grads,
                  BN inputs and softmax outputs of both heads, in fp32 and fp64.
  gat_sub512.npz  GAT.py GAT (32 features, 2 heads) on the same subgraph.
  link.npz        LLP.LinkPredictor 'mlp' and 'inner': outputs and grads.
  llp.npz         LLP.GAT (teacher, forward(input, adj)) on the 512-source subgraph and
                  LLP.Teacher_LinkPredictor ('mlp' with 2 and 3 layers, 'inner', an
                  unknown predictor): init, outputs, grads.
  edge_cases.npz  OursLayer3 / GAL on a hand-made adjacency: empty row, degree 1,
                  degree 65 and 80 (> one wavefront), one hot column; normalize
                  with a zero column (NaN spread) and on random counts.
  ours_small.npz  Ours.OursLayer (full MSHA with city / province attention).
  ours_record.npz Ours.OursLayer record=True: train.Coeff12new and Coeff3 / Coeff4.
  gcn_sub512.npz  model.GCN (nfeat 64, nhid 128; adj^T @ (X W) + scalar bias) on the
                  512-source subgraph: init, train output, nll loss, grads.
  years.npz       per-year node counts, group ids and GDP (2015-2018).

``python tests/golden/make_golden.py gcn`` regenerates only gcn_sub512.npz; ``... llp``
only llp.npz;
``... round2`` regenerates sub512.npz (adds the fp64 softmax outputs), link.npz (adds
the num_layers=1 and unknown-predictor cases) and ours_record.npz.
"""
from __future__ import annotations

import ast
import contextlib
import io
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.overrides import TorchFunctionMode

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(REF, "anonymous_data")

sys.dont_write_bytecode = True
sys.path.insert(0, REF)
import Ablation  # noqa: E402  (reference)
import GAT as GATmod  # noqa: E402  (reference)
import model as refmodel  # noqa: E402  (reference)


def extract(path, names, extra_globals=None):
    """exec the named top-level ClassDef/FunctionDef nodes of a reference file."""
    tree = ast.parse(open(path, encoding="utf-8", errors="replace").read())
    ns = dict(torch=torch, nn=nn, F=F, np=np, json=json)
    if extra_globals:
        ns.update(extra_globals)
    found = {}
    for node in tree.body:
        if isinstance(node, (ast.ClassDef, ast.FunctionDef)) and node.name in names:
            exec(compile(ast.Module(body=[node], type_ignores=[]), path, "exec"), ns)
            found[node.name] = ns[node.name]
    return found


def extract_method(path, cls, meth, extra_globals):
    tree = ast.parse(open(path, encoding="latin-1").read())
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == cls:
            for b in node.body:
                if isinstance(b, ast.FunctionDef) and b.name == meth:
                    ns = dict(extra_globals)
                    exec(compile(ast.Module(body=[b], type_ignores=[]), path, "exec"), ns)
                    return ns[meth]
    raise KeyError(meth)


class Capture(TorchFunctionMode):
    """Records outputs of F.softmax calls made by the reference forward."""

    def __init__(self):
        super().__init__()
        self.softmax = []

    def __torch_function__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        if func is F.softmax or func is torch.softmax or getattr(func, "__name__", "") == "softmax":
            self.softmax.append(out.detach().clone())
        return out


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def np64(t):
    return t.detach().cpu().numpy().astype(np.float64)


# ------------------------------------------------------------------------------------
def load_2015():
    adj = json.load(open(os.path.join(DATA, "Adjacent2015.json"), encoding="utf-8"))
    src_idx = adj["source_index"]
    n, m = len(src_idx), len(adj["recipient_index"])
    assert list(src_idx.keys()) == [str(i) for i in range(n)]
    city = np.array([v[0] for v in src_idx.values()], np.int32)
    prov = np.array([v[1] for v in src_idx.values()], np.int32)
    gdp = json.load(open(os.path.join(DATA, "GDP2015.json")))["GDP_embedding"]
    gdp_arr = np.array(list(gdp.values()), np.float64)
    rows = open(os.path.join(DATA, "Flow2015.csv"), encoding="gb18030").read().splitlines()[1:]
    flows = np.array([[int(x) for x in r.split(",")[:2]] for r in rows if r.strip()], np.int64)

    # reference inter_adjacent (dataset.py:279-296) with its JSON dump sent to a sink
    class _Sink(io.StringIO):
        pass

    def _open(*a, **k):
        return _Sink()

    inter_adjacent = extract_method(os.path.join(REF, "dataset.py"), "HigherDataset",
                                    "inter_adjacent", dict(torch=torch, json=json, open=_open, year="2015"))

    class _Self:
        pass

    s = _Self()
    s.N, s.M, s.count = n, m, len(flows)
    s.source, s.recipient = flows[:, 0].tolist(), flows[:, 1].tolist()
    with contextlib.redirect_stderr(io.StringIO()):
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            counts = inter_adjacent(s)
    return dict(n=n, m=m, city=city, prov=prov, gdp=gdp_arr, flows=flows, counts=counts)


def csr_of(mask):
    mask = np.asarray(mask)
    deg = mask.sum(1)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    _, col = np.nonzero(mask)
    return rowptr, col.astype(np.int32)


def make_r15(g):
    counts = g["counts"]
    norm = refmodel.normalize_adjacency_matrix(counts)
    mask = (counts > 0).numpy()
    rowptr, col = csr_of(mask)
    cnt = counts.numpy()[mask].astype(np.int32)
    normv = norm.numpy()[mask].astype(np.float32)
    assert np.all(norm.numpy()[~mask] == 0)
    np.savez_compressed(os.path.join(OUT, "r15_graph.npz"), n=g["n"], m=g["m"],
                        rowptr=rowptr, col=col.astype(np.uint8), cnt=cnt.astype(np.uint16),
                        norm=normv, city=g["city"].astype(np.int16),
                        prov=g["prov"].astype(np.int8), gdp=g["gdp"].astype(np.float64),
                        n_flows=len(g["flows"]))
    return mask


def pick_sub(mask, k=512):
    first = sorted({int(np.nonzero(mask[:, j])[0][0]) for j in range(mask.shape[1])})
    rows = set(first)
    i = 0
    while len(rows) < k:
        rows.add(i)
        i += 1
    return np.array(sorted(rows), np.int64)


def flatten_sd(prefix, sd, out):
    for k, v in sd.items():
        out[f"{prefix}{k}"] = v.detach().cpu().numpy()


def run_ablation3(sub_counts, gdp_sub, flows_sub, dtype):
    torch.manual_seed(0)
    gdp = {i: float(x) for i, x in enumerate(gdp_sub)}
    n, m = sub_counts.shape
    model = Ablation.ablation3(in_features=128, out_features=64, n_classes=m, n_heads=2,
                               dropout=0.0, gdp=gdp, Scount=n, Rcount=m)
    init_sd = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(dtype)
    adj = refmodel.normalize_adjacency_matrix(sub_counts.to(dtype))
    g = torch.Generator().manual_seed(1)
    bidx = torch.randperm(len(flows_sub), generator=g)[:64]
    source_index = torch.as_tensor(flows_sub[bidx, 0])
    recipient_index = torch.as_tensor(flows_sub[bidx, 1])
    bn_in = {}
    hooks = []
    for h in range(2):
        att = getattr(model, f"attention_{h}")
        hooks.append(att.bn1.register_forward_pre_hook(
            lambda mod, inp, h=h: bn_in.__setitem__(f"h{h}_v_pre", inp[0].detach().clone())))
        hooks.append(att.bn2.register_forward_pre_hook(
            lambda mod, inp, h=h: bn_in.__setitem__(f"h{h}_u_pre", inp[0].detach().clone())))
    model.train()
    cap = Capture()
    with cap:
        out = model(adj, None, None, source_index)
    loss = F.nll_loss(out[source_index], recipient_index)
    model.zero_grad()
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    sd_after = {k: v.clone() for k, v in model.state_dict().items()}  # BN running stats moved
    model.eval()
    with torch.no_grad():
        out_eval = model(adj, None, None, source_index)
    for hk in hooks:
        hk.remove()
    return dict(init_sd=init_sd, sd_after=sd_after, out=out.detach(), loss=loss.detach(),
                grads=grads, bn_in=bn_in, softmax=cap.softmax, out_eval=out_eval,
                source_index=source_index, recipient_index=recipient_index, adj=adj)


def make_sub512(g, mask):
    rows = pick_sub(mask)
    counts = g["counts"][torch.as_tensor(rows)]
    assert (counts > 0).sum(0).min() > 0
    remap = -np.ones(g["n"], np.int64)
    remap[rows] = np.arange(len(rows))
    fl = g["flows"]
    keep = remap[fl[:, 0]] >= 0
    flows_sub = np.stack([remap[fl[keep, 0]], fl[keep, 1]], 1)
    gdp_sub = g["gdp"][rows]
    r32 = run_ablation3(counts, gdp_sub, flows_sub, torch.float32)
    r64 = run_ablation3(counts, gdp_sub, flows_sub, torch.float64)
    out = dict(rows=rows, counts=counts.numpy().astype(np.float32), gdp=gdp_sub,
               flows=flows_sub.astype(np.int32),
               source_index=r32["source_index"].numpy(),
               recipient_index=r32["recipient_index"].numpy(),
               adj_norm=np32(r32["adj"]))
    flatten_sd("init.", r32["init_sd"], out)
    flatten_sd("after32.", {k: v for k, v in r32["sd_after"].items() if "running" in k}, out)
    flatten_sd("after64.", {k: v for k, v in r64["sd_after"].items()
                            if "running" in k and "bn3" not in k}, out)
    out["out32"] = np32(r32["out"])
    out["loss32"] = np32(r32["loss"])
    out["out_eval32"] = np32(r32["out_eval"])
    out["out64"] = np64(r64["out"])
    out["loss64"] = np64(r64["loss"])
    out["out_eval64"] = np64(r64["out_eval"])
    for k, v in r32["grads"].items():
        out[f"grad32.{k}"] = np32(v)
    for k, v in r64["grads"].items():
        if k != "Sfeatures":
            out[f"grad64.{k}"] = np64(v)
    for k, v in r32["bn_in"].items():
        out[f"bn32.{k}"] = np32(v)
    for k, v in r64["bn_in"].items():
        out[f"bn64.{k}"] = np64(v)
    # softmax outputs captured in call order: head0 inter, head1 inter, out_att GAL
    assert len(r32["softmax"]) == 3, len(r32["softmax"])
    for i, name in enumerate(["h0_att", "h1_att", "gal_att"]):
        out[f"sm32.{name}"] = np32(r32["softmax"][i])
        out[f"sm64.{name}"] = np64(r64["softmax"][i])
    np.savez_compressed(os.path.join(OUT, "sub512.npz"), **out)
    return counts, gdp_sub, flows_sub


def make_gat(counts, gdp_sub, flows_sub):
    torch.manual_seed(1)
    n, m = counts.shape
    gdp = {i: float(x) for i, x in enumerate(gdp_sub)}
    model = GATmod.GAT(n_features=32, n_classes=m, n_heads=2, dropout=0.0, gdp=gdp, N=n)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    adj = refmodel.normalize_adjacency_matrix(counts)
    g = torch.Generator().manual_seed(2)
    bidx = torch.randperm(len(flows_sub), generator=g)[:64]
    si = torch.as_tensor(flows_sub[bidx, 0])
    ri = torch.as_tensor(flows_sub[bidx, 1])
    model.train()
    out = model(adj)
    loss = F.nll_loss(out[si], ri)
    loss.backward()
    res = dict(source_index=si.numpy(), recipient_index=ri.numpy(), out=np32(out),
               loss=np32(loss))
    flatten_sd("init.", sd, res)
    for k, p in model.named_parameters():
        if p.grad is not None:
            res[f"grad.{k}"] = np32(p.grad)
    np.savez_compressed(os.path.join(OUT, "gat_sub512.npz"), **res)


def make_link():
    LP = extract(os.path.join(REF, "LLP.py"), {"LinkPredictor"})["LinkPredictor"]
    res = {}
    g = torch.Generator().manual_seed(3)
    xi = torch.randn(256, 32, generator=g)
    xj = torch.randn(256, 32, generator=g)
    res["x_i"], res["x_j"] = xi.numpy(), xj.numpy()
    # 'mlp1': num_layers=1 still builds two Linears (LLP.py:93-96), so lins[:-1] is one
    # layer as with num_layers=2; 'other': any predictor string besides 'mlp'/'inner'
    # skips both branches and returns sigmoid(x_i * x_j), shape (B, F) (LLP.py:104-115)
    for mode, pred, nl in (("mlp", "mlp", 2), ("inner", "inner", 2), ("mlp1", "mlp", 1),
                           ("other", "dot", 2)):
        torch.manual_seed(4)
        lp = LP(pred, 32, 32, 1, nl, 0.0)
        for k, v in lp.state_dict().items():
            res[f"{mode}.init.{k}"] = v.numpy()
        a = xi.clone().requires_grad_(True)
        b = xj.clone().requires_grad_(True)
        lp.train()
        y = lp(a, b)
        w = torch.randn(y.shape, generator=g)
        (y * w).sum().backward()
        res[f"{mode}.out"] = np32(y)
        res[f"{mode}.dout"] = w.numpy()
        res[f"{mode}.grad.x_i"] = np32(a.grad)
        res[f"{mode}.grad.x_j"] = np32(b.grad)
        for k, p in lp.named_parameters():
            if p.grad is not None:
                res[f"{mode}.grad.{k}"] = np32(p.grad)
    np.savez_compressed(os.path.join(OUT, "link.npz"), **res)


def make_llp():
    """LLP.py's teacher GAT (forward(input, adj), LLP.py:148-168) and
    Teacher_LinkPredictor (LLP.py:170-198), AST-extracted (LLP.py runs its training
    script at import), on the 512-source subgraph of sub512.npz."""
    ns = extract(os.path.join(REF, "LLP.py"),
                 {"GraphAttentionLayer", "GAT", "Teacher_LinkPredictor"})
    z = np.load(os.path.join(OUT, "sub512.npz"))
    counts = torch.as_tensor(z["counts"])
    n, m = counts.shape
    flows = z["flows"].astype(np.int64)
    adj = refmodel.normalize_adjacency_matrix(counts)
    res = {}
    torch.manual_seed(11)
    gat = ns["GAT"](n_features=32, n_classes=m, n_heads=2, dropout=0.0, gdp=None, N=n)
    for k, v in gat.state_dict().items():
        res[f"gat.init.{k}"] = v.numpy()
    g = torch.Generator().manual_seed(12)
    x = torch.randn(n, 32, generator=g).requires_grad_(True)
    bidx = torch.randperm(len(flows), generator=g)[:64]
    si, ri = torch.as_tensor(flows[bidx, 0]), torch.as_tensor(flows[bidx, 1])
    gat.train()
    out = gat(x, adj)
    loss = F.nll_loss(out[si], ri)
    loss.backward()
    res.update({"gat.input": x.detach().numpy(), "gat.source_index": si.numpy(),
                "gat.recipient_index": ri.numpy(), "gat.out": np32(out), "gat.loss": np32(loss),
                "gat.grad.input": np32(x.grad)})
    for k, p_ in gat.named_parameters():
        if p_.grad is not None:
            res[f"gat.grad.{k}"] = np32(p_.grad)
    TL = ns["Teacher_LinkPredictor"]
    xi = torch.randn(200, 32, generator=g)
    xj = torch.randn(200, 32, generator=g)
    res["tlp.x_i"], res["tlp.x_j"] = xi.numpy(), xj.numpy()
    for mode, pred, nl in (("mlp", "mlp", 2), ("mlp3", "mlp", 3), ("inner", "inner", 2),
                           ("other", "cos", 2)):
        torch.manual_seed(13)
        lp = TL(pred, 32, 24, 1, nl, 0.0)
        for k, v in lp.state_dict().items():
            res[f"tlp.{mode}.init.{k}"] = v.numpy()
        a = xi.clone().requires_grad_(True)
        b = xj.clone().requires_grad_(True)
        lp.train()
        y = lp(a, b)
        w = torch.randn(y.shape, generator=g)
        (y * w).sum().backward()
        res[f"tlp.{mode}.out"] = np32(y)
        res[f"tlp.{mode}.dout"] = w.numpy()
        res[f"tlp.{mode}.grad.x_i"] = np32(a.grad)
        res[f"tlp.{mode}.grad.x_j"] = np32(b.grad)
        for k, p_ in lp.named_parameters():
            if p_.grad is not None:
                res[f"tlp.{mode}.grad.{k}"] = np32(p_.grad)
    np.savez_compressed(os.path.join(OUT, "llp.npz"), **res)


def edge_adj():
    """40 x 80 count matrix: row 0 empty; row 1 degree 1; row 2 full (80 > 64);
    row 3 degree 65; rows 4..20 all in column 7 (hot column); the rest random."""
    rng = np.random.default_rng(5)
    n, m = 40, 80
    c = np.zeros((n, m), np.float32)
    c[1, 13] = 2
    c[2, :] = rng.integers(1, 4, m)
    c[3, rng.permutation(m)[:65]] = 1
    c[4:21, 7] = rng.integers(1, 5, 17)
    for i in range(21, n):
        k = rng.integers(1, 9)
        c[i, rng.permutation(m)[:k]] = rng.integers(1, 3, k)
    return c


def make_edge_cases():
    c = edge_adj()
    res = dict(counts=c)
    for dt, tag in ((torch.float32, "32"), (torch.float64, "64")):
        adj = refmodel.normalize_adjacency_matrix(torch.as_tensor(c).to(dt))
        res[f"adj_norm{tag}"] = adj.numpy()
        torch.manual_seed(6)
        layer = Ablation.OursLayer3(16, 8, 0.0)
        for k, v in layer.state_dict().items():
            res[f"ol3.init.{k}"] = v.numpy().astype(np.float32)
        layer = layer.to(dt)
        g = torch.Generator().manual_seed(7)
        S = torch.rand(40, 16, generator=g, dtype=torch.float64).to(dt).requires_grad_(True)
        R = torch.rand(80, 16, generator=g, dtype=torch.float64).to(dt).requires_grad_(True)
        res[f"ol3.S{tag}"], res[f"ol3.R{tag}"] = S.detach().numpy(), R.detach().numpy()
        layer.eval()  # before the train forward: BN running stats still at init
        with torch.no_grad():
            res[f"ol3.out_eval{tag}"] = layer(S, R, adj, None, None, None).numpy()
        layer.train()
        cap = Capture()
        with cap:
            y = layer(S, R, adj, None, None, None)
        w = torch.randn(y.shape, generator=g, dtype=torch.float64).to(dt)
        (y * w).sum().backward()
        res[f"ol3.out{tag}"] = y.detach().numpy()
        res[f"ol3.dout{tag}"] = w.numpy()
        res[f"ol3.att{tag}"] = cap.softmax[0].numpy()
        res[f"ol3.grad{tag}.S"] = S.grad.numpy()
        res[f"ol3.grad{tag}.R"] = R.grad.numpy()
        for k, p in layer.named_parameters():
            if p.grad is not None:
                res[f"ol3.grad{tag}.{k}"] = p.grad.numpy()
        # GAL with out_features == 80 columns of this adjacency
        torch.manual_seed(8)
        gal = Ablation.GraphAttentionLayer(20, 80, 0.0)
        for k, v in gal.state_dict().items():
            res[f"gal.init.{k}"] = v.numpy().astype(np.float32)
        gal = gal.to(dt)
        x = torch.randn(40, 20, generator=g, dtype=torch.float64).to(dt).requires_grad_(True)
        res[f"gal.x{tag}"] = x.detach().numpy()
        gal.train()
        y = gal(x, adj)
        w = torch.randn(y.shape, generator=g, dtype=torch.float64).to(dt)
        (y * w).sum().backward()
        res[f"gal.out{tag}"] = y.detach().numpy()
        res[f"gal.dout{tag}"] = w.numpy()
        res[f"gal.grad{tag}.x"] = x.grad.numpy()
        res[f"gal.grad{tag}.W"] = gal.W.grad.numpy()
        res[f"gal.grad{tag}.a"] = gal.a.grad.numpy()
    # normalize_adjacency_matrix: zero column -> NaN spread; random counts -> exact values
    z = torch.as_tensor(c.copy())
    z[:, 5] = 0
    res["norm_zero_col_in"] = z.numpy()
    res["norm_zero_col_out"] = refmodel.normalize_adjacency_matrix(z).numpy()
    rc = torch.as_tensor(np.random.default_rng(9).integers(0, 7, (300, 45)).astype(np.float32))
    res["norm_rand_in"] = rc.numpy()
    res["norm_rand_out"] = refmodel.normalize_adjacency_matrix(rc).numpy()
    np.savez_compressed(os.path.join(OUT, "edge_cases.npz"), **res)


def make_ours_small(g):
    """Ours.OursLayer on 64 sources of 2015 (city/province groups restricted):
    case A fp32 as the reference runs it; case B fp64 with a repeated source in the
    batch and one source row without flows (uniform inter attention)."""
    O = extract(os.path.join(REF, "Ours.py"), {"OursLayer"})["OursLayer"]
    rows = np.arange(64)
    counts = g["counts"][torch.as_tensor(rows)].clone()
    keepc = (counts > 0).sum(0) > 0
    counts = counts[:, keepc]
    city = g["city"][rows]
    prov = g["prov"][rows]
    res = dict(counts=counts.numpy(), city=city, prov=prov)
    for tag, dt, si_fix, empty_row in (("", torch.float32, None, None),
                                       ("B.", torch.float64, [5, 17, 5, 40, 33, 5, 60, 12], 33)):
        c = counts.clone()
        if empty_row is not None:
            c[empty_row] = 0
            res[tag + "counts"] = c.numpy()
        city_adj = torch.as_tensor((city[:, None] == city[None, :]).astype(np.float32))
        prov_adj = torch.as_tensor((prov[:, None] == prov[None, :]).astype(np.float32))
        inter = refmodel.normalize_adjacency_matrix(c).to(dt)
        city_n = refmodel.normalize_adjacency_matrix(city_adj).to(dt)
        prov_n = refmodel.normalize_adjacency_matrix(prov_adj).to(dt)
        torch.manual_seed(10)
        layer = O(16, 8, 0.0)
        if tag == "":
            for k, v in layer.state_dict().items():
                res[f"init.{k}"] = v.numpy().copy()
        layer = layer.to(dt)
        gg = torch.Generator().manual_seed(11)
        S = torch.rand(64, 16, generator=gg, dtype=torch.float64).to(dt).requires_grad_(True)
        R = torch.rand(c.shape[1], 16, generator=gg, dtype=torch.float64).to(dt).requires_grad_(True)
        si = torch.randperm(64, generator=gg)[:16] if si_fix is None else torch.as_tensor(si_fix)
        res[tag + "S"], res[tag + "R"] = S.detach().numpy(), R.detach().numpy()
        res[tag + "source_index"] = si.numpy()
        layer.eval()  # before the train forward: BN running stats still at init
        with torch.no_grad():
            res[tag + "out_eval"] = layer(S, R, inter, city_n, prov_n, si, False).numpy()
        layer.train()
        y = layer(S, R, inter, city_n, prov_n, si, False)
        w = torch.randn(y.shape, generator=gg, dtype=torch.float64).to(dt)
        (y * w).sum().backward()
        res[tag + "out"], res[tag + "dout"] = y.detach().numpy(), w.numpy()
        res[tag + "grad.S"], res[tag + "grad.R"] = S.grad.numpy(), R.grad.numpy()
        for k, p in layer.named_parameters():
            if p.grad is not None:
                res[f"{tag}grad.{k}"] = p.grad.numpy()
    np.savez_compressed(os.path.join(OUT, "ours_small.npz"), **res)


def make_ours_record(g):
    """Ours.OursLayer with record=True (Ours.py:92-96, eval mode as Record() runs it,
    train.py:284-291): the layer sets ``train.Coeff12new`` to the (N, M) inter attention
    and writes the batch rows of the (B, N) city / province attention into
    Coeff3[source_index] / Coeff4[source_index]; the Coeff12 argument is never
    written.  Same 64-source graph as ours_small.npz."""
    import types

    sink = types.SimpleNamespace()
    O = extract(os.path.join(REF, "Ours.py"), {"OursLayer"}, dict(train=sink))["OursLayer"]
    z = np.load(os.path.join(OUT, "ours_small.npz"))
    counts = torch.as_tensor(z["counts"])
    n, m = counts.shape
    city, prov = z["city"], z["prov"]
    city_adj = torch.as_tensor((city[:, None] == city[None, :]).astype(np.float32))
    prov_adj = torch.as_tensor((prov[:, None] == prov[None, :]).astype(np.float32))
    inter = refmodel.normalize_adjacency_matrix(counts)
    city_n = refmodel.normalize_adjacency_matrix(city_adj)
    prov_n = refmodel.normalize_adjacency_matrix(prov_adj)
    torch.manual_seed(10)
    layer = O(16, 8, 0.0)
    layer.eval()
    S = torch.as_tensor(z["S"])
    R = torch.as_tensor(z["R"])
    res = {}
    C12 = torch.full((n, m), -1.0)
    C3 = torch.full((n, n), -1.0)
    C4 = torch.full((n, n), -1.0)
    for k, si in enumerate((np.arange(0, 32), np.arange(32, 64))):  # Record(): batches
        with torch.no_grad():
            layer(S, R, inter, city_n, prov_n, torch.as_tensor(si), True, C12, C3, C4)
        res[f"rec.coeff12new.{k}"] = np32(sink.Coeff12new)
    res["rec.coeff3"], res["rec.coeff4"] = np32(C3), np32(C4)
    assert bool((C12 == -1).all())  # the argument is never written
    np.savez_compressed(os.path.join(OUT, "ours_record.npz"), **res)


def make_gcn():
    """model.GCN (model.py:11-64) on the sub512 graph: GraphConvolution is
    adj^T @ (X @ W) + b with a SCALAR bias (model.py:23), the second layer runs on
    adj.t() (so adj @ support), log_softmax over nhid (gc3 is built, never used)."""
    z = np.load(os.path.join(OUT, "sub512.npz"))
    counts = torch.as_tensor(z["counts"])
    n, m = counts.shape
    gdp = {i: float(x) for i, x in enumerate(z["gdp"])}
    adj = refmodel.normalize_adjacency_matrix(counts)
    torch.manual_seed(4)
    model = refmodel.GCN(nfeat=64, nhid=128, nclass=m, dropout=0.0, gdp=gdp, N=n)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    si = torch.as_tensor(z["source_index"]).long()
    ri = torch.as_tensor(z["recipient_index"]).long()
    model.train()
    out = model(adj)
    loss = F.nll_loss(out[si], ri)
    loss.backward()
    res = dict(out=np32(out), loss=np32(loss))
    flatten_sd("init.", sd, res)
    for k, p in model.named_parameters():
        if p.grad is not None:
            res[f"grad.{k}"] = np32(p.grad)
    np.savez_compressed(os.path.join(OUT, "gcn_sub512.npz"), **res)


def make_years():
    """Per-year node tables of the shipped 2015-2018 graphs (Adjacent{Y}.json,
    GDP{Y}.json): N, city / province group ids, GDP.  Flows of 2016-2018 are not
    shipped (.MISSING_LARGE_BLOBS); bench.py synthesises them with the 2015 degree
    law (msha_gnn_amd.data.synthetic_flows, seed = year)."""
    res = {}
    for year in ("2015", "2016", "2017", "2018"):
        adj = json.load(open(os.path.join(DATA, f"Adjacent{year}.json"), encoding="utf-8"))
        src = adj["source_index"]
        n = len(src)
        groups = np.array([src[str(i)] for i in range(n)], np.int64)
        gdp = json.load(open(os.path.join(DATA, f"GDP{year}.json")))["GDP_embedding"]
        res[f"{year}.n"] = n
        res[f"{year}.m"] = len(adj["recipient_index"])
        res[f"{year}.city"] = groups[:, 0].astype(np.int16)
        res[f"{year}.prov"] = groups[:, 1].astype(np.int8)
        res[f"{year}.gdp"] = np.array([gdp[str(i)] for i in range(n)], np.float32)
    np.savez_compressed(os.path.join(OUT, "years.npz"), **res)


def main():
    torch.set_num_threads(8)
    if sys.argv[1:] == ["gcn"]:
        make_gcn()
        return
    if sys.argv[1:] == ["llp"]:  # round 3: LLP.GAT / Teacher_LinkPredictor
        make_llp()
        return
    if sys.argv[1:] == ["round2"]:  # link quirks, sub512 fp64 softmax, Ours record dump
        g = load_2015()
        mask = (g["counts"] > 0).numpy()
        make_sub512(g, mask)
        make_link()
        make_ours_record(g)
        return
    g = load_2015()
    mask = make_r15(g)
    counts, gdp_sub, flows_sub = make_sub512(g, mask)
    make_gat(counts, gdp_sub, flows_sub)
    make_link()
    make_llp()
    make_edge_cases()
    make_ours_small(g)
    make_ours_record(g)
    make_gcn()
    make_years()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
