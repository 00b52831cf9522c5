"""Projection time vs row count (fixed cost vs per-tile throughput), fp32, C4 shape.

    MSHA_PROJ=1|2|3 python scripts/proj_scan.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msha_loader  # noqa: E402

msha_loader.load()
from msha_gnn_amd import functional as MF  # noqa: E402
from gemm_ab import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    K, H, F = 128, 8, 16
    W = torch.randn(K, H * F, device=dev, generator=g) / K ** 0.5
    al = torch.randn(H, F, device=dev, generator=g)
    ar = torch.randn(H, F, device=dev, generator=g)
    for M in (16384, 32768, 65536, 100000, 131072, 262144, 524288):
        X = torch.rand(M, K, device=dev, generator=g)
        us = timeit(lambda: MF.project_scores(X, W, al, ar, heads=H))
        us0 = timeit(lambda: MF.project_scores(X, W))
        z = torch.zeros_like(X)
        usz = timeit(lambda: MF.project_scores(z, W, al, ar, heads=H))
        print(json.dumps({"proj": os.environ.get("MSHA_PROJ", "3"), "M": M, "us": round(us, 1),
                          "us_noscore": round(us0, 1), "us_zeros": round(usz, 1),
                          "TFs": round(2 * M * K * H * F / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
