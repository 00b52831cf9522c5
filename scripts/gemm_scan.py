"""Time the fp32 projection GEMM over shapes (HIP events, 20 launches each) to separate
per-block fixed costs from per-k-tile costs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msha_loader  # noqa: E402

msha_loader.load()
from msha_gnn_amd import functional as MF  # noqa: E402

dev = torch.device("cuda:0")
for M, K, N, score in [(100000, 128, 128, True), (100000, 128, 128, False), (100000, 512, 128, False),
                       (400000, 128, 128, False), (100000, 32, 128, False), (100000, 128, 64, False)]:
    X = torch.rand(M, K, device=dev)
    W = torch.rand(K, N, device=dev)
    al = torch.rand(8, N // 8, device=dev)
    f = (lambda: MF.project_scores(X, W, al, al, heads=8)) if score else (lambda: MF.gemm(X, W))
    for _ in range(3):
        f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        f()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 20 * 1e3
    print(f"M={M} K={K} N={N} score={score}: {us:.1f} us, {2*M*K*N/us/1e6:.1f} TFLOP/s, "
          f"{4*(M*K+M*N)/us/1e3:.0f} GB/s")
