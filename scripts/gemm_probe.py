"""GEMM probe: the C4 projection (X 100k x 128 @ W 128 x 128 + score epilogue) and the
weight gradient (X^T @ (dh + de (x) a), K = 100k split-K), 20 launches each.
Run under rocprofv3 (--kernel-trace --stats, or one --pmc pass) to attribute time."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
import msha_loader  # noqa: E402

msha_loader.load()
from msha_gnn_amd import functional as MF  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
M, K, H, F = 100000, 128, 8, 16
X = torch.rand(M, K, generator=g).to(dev)
W = (torch.rand(K, H * F, generator=g) - 0.5).to(dev)
al = torch.randn(H, F, generator=g).to(dev)
ar = torch.randn(H, F, generator=g).to(dev)
dh = torch.randn(M, H * F, generator=g).to(dev)
de = torch.randn(M, H, generator=g).to(dev)
de2 = torch.randn(M, H, generator=g).to(dev)
for name, fn in (("proj", lambda: MF.project_scores(X, W, al, ar, heads=H)),
                 ("dW_ho", lambda: MF.gemm_head_outer(X.t(), dh, 1, (H, F, de, al, de2, ar))),
                 ("dW", lambda: MF.gemm(X.t(), dh)),
                 ("dX_ho", lambda: MF.gemm_head_outer(dh, W.t(), 0, (H, F, de, al, de2, ar)))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us/call (host clock)")
