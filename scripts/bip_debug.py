"""bip kernels vs the general kernels on a 200k-row bipartite graph (many groups per
wave): per output, the mismatching rows with their degree and in-group position."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import msha_loader  # noqa: E402

msha_loader.load()
from msha_gnn_amd import functional as MF  # noqa: E402
from msha_gnn_amd.graph import Graph  # noqa: E402

dev = torch.device("cuda:0")
n, m, H, F = 200_000, 32, 2, 64
rng = np.random.default_rng(0)
deg = rng.integers(1, 6, n)
rowptr = np.zeros(n + 1, np.int64)
rowptr[1:] = np.cumsum(deg)
col = np.concatenate([np.sort(rng.choice(m, d, replace=False)) for d in deg]).astype(np.int64)
graph = Graph.from_csr(torch.as_tensor(rowptr), torch.as_tensor(col), m, dev)
g = torch.Generator().manual_seed(1)
el, er = torch.randn(n, H, generator=g), torch.randn(m, H, generator=g)
hc, hs = torch.randn(m, H, F, generator=g), torch.randn(n, H, F, generator=g)
dU, dV = torch.randn(n, H, F, generator=g), torch.randn(m, H, F, generator=g)


def run(bip, p):
    MF.BIP = bip
    lv = [x.to(dev).requires_grad_(True) for x in (el, er, hc, hs)]
    u, v = MF.edge_attention(graph, *lv[:3], hs=lv[3], p=p, training=p > 0, seed=5)
    torch.autograd.backward([u, v], [dU.to(dev), dV.to(dev)])
    torch.cuda.synchronize()
    return dict(u=u.detach().cpu(), v=v.detach().cpu(), d_el=lv[0].grad.cpu(),
                d_er=lv[1].grad.cpu(), d_hc=lv[2].grad.cpu(), d_hs=lv[3].grad.cpu())


from msha_gnn_amd import _lib  # noqa: E402
cu = torch.cuda.get_device_properties(0).multi_processor_count
W = cu * 7
for p in (0.0, 0.5):
    a, b = run(True, p), run(False, p)
    for k in a:
        x, y = a[k].double(), b[k].double()
        err = (x - y).abs()
        tol = 1e-4 * y.abs().max().item() + 1e-4 * y.abs()
        bad = (err > tol)
        if bad.dim() > 1:
            bad = bad.reshape(bad.shape[0], -1).any(1)
        nb = int(bad.sum())
        print(f"p={p} {k:5s} bad rows {nb} / {bad.shape[0]}  maxerr {err.max().item():.3g}")
        if nb and k in ("d_el", "d_hs", "u"):
            idx = torch.nonzero(bad).flatten()[:12].numpy()
            wr = [(int(i), int(deg[i]), int((i - (i * W // n) * n // W))) for i in idx]
            print("   rows (row, deg, ~offset in wave range):", wr)
            print("   got", a[k][idx[:3]].flatten()[:6].numpy(), "want", b[k][idx[:3]].flatten()[:6].numpy())

# forward lse: bip vs the general forward (raw ABI)
gd = graph.desc
L = _lib.load()
s = _lib.stream_handle(dev)
el_d, er_d, hc_d, hs_d = (x.to(dev).contiguous() for x in (el, er, hc, hs))
ws = torch.empty(int(L.msha_bip_workspace_size(gd, H, F)), dtype=torch.uint8, device=dev)
u1, v1 = torch.empty(n, H, F, device=dev), torch.empty(m, H, F, device=dev)
lse1 = torch.full((n, H), 7.0, device=dev)
_lib.call("msha_bip_attention_fwd", gd, H, F, 0, el_d.data_ptr(), er_d.data_ptr(), hc_d.data_ptr(),
          hs_d.data_ptr(), 0.2, 0.0, 0, 0, u1.data_ptr(), None, lse1.data_ptr(), None,
          v1.data_ptr(), ws.data_ptr(), ws.numel(), s)
u2 = torch.empty(n, H, F, device=dev)
lse2 = torch.empty(n, H, device=dev)
_lib.call("msha_edge_attention_fwd", gd, H, F, 0, el_d.data_ptr(), er_d.data_ptr(), hc_d.data_ptr(),
          0.2, 0.0, 0, 0, u2.data_ptr(), None, lse2.data_ptr(), None, s)
torch.cuda.synchronize()
bad = ((lse1 - lse2).abs() > 1e-4).any(1).cpu()
idx = torch.nonzero(bad).flatten()[:10].numpy()
print("lse bad rows", int(bad.sum()), [(int(i), int(deg[i]), int((i - (i * W // n) * n // W))) for i in idx])
print("   got", lse1[idx[:4]].cpu().numpy().ravel(), "want", lse2[idx[:4]].cpu().numpy().ravel())
