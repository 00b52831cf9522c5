"""Time the C4 projection and weight-gradient GEMMs (one JSON line per case).

    MSHA_SKINNY=0 python scripts/gemm_ab.py   # tiled GEMMs (gemm.hip / gemm_bf16.hip)
    python scripts/gemm_ab.py                 # resident-W / whole-tile kernels (skinny.hip)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msha_loader  # noqa: E402

msha_loader.load()
from msha_gnn_amd import functional as MF  # noqa: E402


def timeit(fn, reps=int(os.environ.get("GEMM_AB_REPS", 50)), warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [(100000, 128, 8, 16), (39179, 128, 2, 64)]  # C4, R15 (configs[1])
    if os.environ.get("GEMM_AB_BIP1M"):
        shapes.append((1000000, 128, 2, 64))  # bip1m's source table
    for shape in shapes:
        run_shape(dev, g, *shape)


def run_shape(dev, g, M, K, H, F):
    D = H * F
    for dt in (torch.float32, torch.bfloat16):
        X = torch.rand(M, K, device=dev, generator=g).to(dt)
        W = (torch.randn(K, D, device=dev, generator=g) / K ** 0.5).to(dt)
        al = torch.randn(H, F, device=dev, generator=g)
        ar = torch.randn(H, F, device=dev, generator=g)
        dh = torch.randn(M, D, device=dev, generator=g).to(dt)
        de = torch.randn(M, H, device=dev, generator=g)
        de2 = torch.randn(M, H, device=dev, generator=g)
        outer = (H, F, de, al, de2, ar)
        us_p = timeit(lambda: MF.project_scores(X, W, al, ar, heads=H))
        us_w = timeit(lambda: MF.gemm_head_outer(X.t(), dh, 1, outer))
        us_x = timeit(lambda: MF.gemm_head_outer(dh, W.t(), 0, outer)) if dt == torch.float32 else 0.0
        flop = 2.0 * M * K * D
        if os.environ.get("GEMM_AB_SAVE") and dt == torch.float32:  # bitwise A/B of the outputs
            torch.save({"h": MF.project_scores(X, W, al, ar, heads=H),
                        "dw": MF.gemm_head_outer(X.t(), dh, 1, outer),
                        "dx": MF.gemm_head_outer(dh, W.t(), 0, outer),
                        "dw0": MF.gemm(X.t(), dh)}, os.environ["GEMM_AB_SAVE"] + f".{M}")
        print(json.dumps({"M": M, "heads": H, "dx_us": round(us_x, 1),
                          "skinny": os.environ.get("MSHA_SKINNY", "1"), "dtype": str(dt)[6:],
                          "proj_us": round(us_p, 1), "proj_TFs": round(flop / us_p / 1e6, 1),
                          "wgrad_us": round(us_w, 1), "wgrad_TFs": round(flop / us_w / 1e6, 1)}),
              flush=True)


def cmp(a, b):
    for M in (100000, 39179):
        cmp1(f"{a}.{M}", f"{b}.{M}")


def cmp1(a, b):
    x, y = torch.load(a, weights_only=True, map_location="cpu"), torch.load(b, weights_only=True, map_location="cpu")
    for k in x:
        xa = x[k][0] if isinstance(x[k], tuple) else x[k]
        ya = y[k][0] if isinstance(y[k], tuple) else y[k]
        print(json.dumps({"out": k, "bit_identical": bool(torch.equal(xa, ya)),
                          "max_abs_diff": float((xa - ya).abs().max())}))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "cmp":
        cmp(sys.argv[2], sys.argv[3])
    else:
        main()
