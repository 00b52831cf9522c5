"""Layer-level diagnosis of test_ours_layer_full_graph (GPU): rows of S.grad that differ
from the dense fp64 reference, and their batch / group / degree properties.

    python scripts/debug_ours_layer.py 2017
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import dense_ref as D  # noqa: E402
import test_gpu_parity_full as T  # noqa: E402
import msha_loader  # noqa: E402

msha = msha_loader.load()
from msha_gnn_amd import layers  # noqa: E402

year = sys.argv[1] if len(sys.argv) > 1 else "2017"
cuda = torch.device("cuda:0")
yg = T._year(msha, cuda, year)
n, m = yg["n"], yg["m"]
city, prov = yg["city"], yg["prov"]
deg = np.diff(yg["rowptr"])
torch.manual_seed(0)
layer = layers.OursLayer(128, 64, 0.0)
g = torch.Generator().manual_seed(int(year))
S = torch.rand(n, 128, generator=g)
R = torch.rand(m, 128, generator=g)
dout = torch.randn(n, m, generator=g)
src = T._batch(yg, seed=int(year))
city_adj, prov_adj = T._groups(yg, cuda)
p64 = D.layer_params(layer)
layer = layer.to(cuda).train()
for rep in range(2):
    St, Rt = S.to(cuda).requires_grad_(True), R.to(cuda).requires_grad_(True)
    h2_keep = {}
    y = layer(St, Rt, yg["adj"], city_adj, prov_adj, torch.as_tensor(src, device=cuda), False)
    y.backward(dout.to(cuda))
    S64 = S.double().requires_grad_(True)
    R64 = R.double().requires_grad_(True)
    for v in p64.values():
        if v.grad is not None:
            v.grad = None
    y64 = D.ours_layer(S64, R64, p64, torch.as_tensor(yg["mask"]), torch.as_tensor(city),
                       torch.as_tensor(prov), torch.as_tensor(src), True)
    (y64 * dout.double()).sum().backward()
    got, ref = St.grad.cpu().numpy(), S64.grad.numpy()
    scale = np.abs(ref).max()
    bad = np.nonzero((np.abs(got - ref) > 1e-5 * np.abs(ref) + 1e-5 * scale).any(1))[0]
    print("rep", rep, "y maxerr", float(np.abs(y.detach().cpu().numpy() - y64.detach().numpy()).max()),
          "scale", float(np.abs(y64.detach().numpy()).max()))
    print("  S.grad bad rows", bad, "scale", scale)
    for r in bad[:6]:
        print("   row", r, "batch pos", np.nonzero(src == r)[0], "deg", deg[r], "city", city[r],
              np.sum(city == city[r]), "prov", prov[r], np.sum(prov == prov[r]),
              "maxdiff", float(np.abs(got[r] - ref[r]).max()), "got", got[r][:3], "ref", ref[r][:3])
        same_c = np.nonzero(city[src] == city[r])[0]
        same_p = np.nonzero(prov[src] == prov[r])[0]
        print("     batch entries sharing city", same_c, "prov", same_p)
    for k, name in D.GRAD_KEYS.items():
        gg = dict(layer.named_parameters())[name].grad.cpu().numpy()
        rr = p64[k].grad.numpy()
        print("  ", name, "max rel-to-max err", float(np.abs(gg - rr).max() / np.abs(rr).max()))
    layer.zero_grad()
