"""Diagnose a wrong S.grad row of OursLayer on a full year graph (GPU): which rows
differ from the dense fp64 reference, their batch membership / groups / degree, and
whether the kernel-level gradients (d_hs, d_el, d_er, d_hc) agree.

    python scripts/debug_ours_rows.py 2017
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import dense_ref as D  # noqa: E402,F401
import test_gpu_parity_full as T  # noqa: E402
import msha_loader  # noqa: E402

msha = msha_loader.load()
from msha_gnn_amd import functional as MF  # noqa: E402
from msha_gnn_amd.graph import Graph, Groups  # noqa: E402

year = sys.argv[1] if len(sys.argv) > 1 else "2017"
cuda = torch.device("cuda:0")
yg = T._year(msha, cuda, year)
n, m = yg["n"], yg["m"]
src = T._batch(yg, seed=int(year))
print("year", year, "n", n, "src", src[:8], "dup", len(src) - len(np.unique(src)))
city, prov = yg["city"], yg["prov"]
deg = np.diff(yg["rowptr"])


def rows_bad(got, ref, tol=1e-5):
    scale = np.abs(ref).max()
    bad = np.abs(got - ref) > tol * np.abs(ref) + tol * scale
    return np.nonzero(bad.any(axis=tuple(range(1, bad.ndim))))[0]


# kernel level: the attention core with leaves (one head, F 64)
rng = np.random.default_rng(0)
H, Fd = 1, 64
el = rng.standard_normal((n, H))
er = rng.standard_normal((m, H))
h1 = rng.standard_normal((m, H, Fd)) * 0.3
h2 = rng.standard_normal((n, H, Fd)) * 0.3
a3s = rng.standard_normal((H, Fd)) * 0.2
a4s = rng.standard_normal((H, Fd)) * 0.2
dU = rng.standard_normal((n, H, Fd))
dV = rng.standard_normal((m, H, Fd))
graph = Graph.from_dense(yg["adj"])
groups = Groups(city, prov, cuda)
t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=cuda).float()  # noqa: E731
import test_gpu_ours as TO  # noqa: E402

for rep in range(2):
    tg = [t(x).requires_grad_(True) for x in (el, er, h1, h2, a3s, a4s)]
    u, v = MF.ours_attention(graph, groups, torch.as_tensor(src, device=cuda), *tg)
    (u * t(dU)).sum().add_((v * t(dV)).sum()).backward()
    rs = [torch.tensor(x[:, 0], dtype=torch.float64, requires_grad=True) for x in (el, er, h1, h2)]
    ra3 = torch.tensor(a3s[0], dtype=torch.float64, requires_grad=True)
    ra4 = torch.tensor(a4s[0], dtype=torch.float64, requires_grad=True)
    ru, rv = TO._dense_ours_core(*rs, ra3, ra4, torch.as_tensor(yg["mask"]), torch.as_tensor(city),
                                 torch.as_tensor(prov), torch.as_tensor(src))
    ((ru * torch.tensor(dU[:, 0])).sum() + (rv * torch.tensor(dV[:, 0])).sum()).backward()
    print("rep", rep, "u bad rows", rows_bad(u[:, 0].detach().cpu().numpy(), ru.detach().numpy()))
    for name, got, ref in (("d_el", tg[0].grad[:, 0], rs[0].grad), ("d_er", tg[1].grad[:, 0], rs[1].grad),
                           ("d_h1", tg[2].grad[:, 0], rs[2].grad), ("d_h2", tg[3].grad[:, 0], rs[3].grad),
                           ("d_a3", tg[4].grad[0], ra3.grad), ("d_a4", tg[5].grad[0], ra4.grad)):
        g_np, r_np = got.cpu().numpy(), ref.numpy()
        if g_np.ndim > 1:
            bad = rows_bad(g_np, r_np)
        else:
            bad = np.nonzero(np.abs(g_np - r_np) > 1e-5 * np.abs(r_np) + 1e-5 * np.abs(r_np).max())[0]
        print(" ", name, "bad", bad[:10], "n_bad", len(bad))
        for r in bad[:4]:
            if name in ("d_el", "d_h2"):
                inb = np.nonzero(src == r)[0]
                print("    row", r, "in batch at", inb, "deg", deg[r], "city", city[r], "|city|",
                      np.sum(city == city[r]), "prov", prov[r], "|prov|", np.sum(prov == prov[r]),
                      "got", g_np[r].ravel()[:3], "ref", r_np[r].ravel()[:3])
