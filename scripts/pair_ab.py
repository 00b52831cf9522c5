"""A/B of the resident-W pair scorer kernels (C5 shape: 4M pairs, 100k x 128 table,
hidden 128): times fp32 / bf16 'mlp' scoring and saves the scores so two builds
(MSHA_GNN_LIB=...) or knob settings can be compared bit for bit.

    MSHA_GNN_LIB=lib/alt/a.so python scripts/pair_ab.py save gpurun_out/pair_a.pt
    MSHA_GNN_LIB=lib/alt/b.so python scripts/pair_ab.py save gpurun_out/pair_b.pt
    python scripts/pair_ab.py cmp gpurun_out/pair_0.pt gpurun_out/pair_1.pt
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def save(path):
    import msha_loader

    msha_loader.load()
    from msha_gnn_amd import _lib
    from msha_gnn_amd import functional as MF
    from gemm_ab import timeit

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    n, F, N, P = 100000, 128, 128, 4_000_000
    res, outs = {"lib": os.environ.get("MSHA_GNN_LIB", "default")}, {}
    for dt in (torch.float32, torch.bfloat16):
        h = torch.randn(n, F, device=dev, generator=g).to(dt)
        W = (torch.randn(N, F, device=dev, generator=g) / F ** 0.5).to(dt)
        b = torch.randn(N, device=dev, generator=g) * 0.1
        src = torch.randint(0, n, (P,), device=dev, generator=g)
        dst = torch.randint(0, n, (P,), device=dev, generator=g)
        tag = "f32" if dt == torch.float32 else "bf16"
        ob = torch.bfloat16 if dt == torch.bfloat16 else None
        outs[tag] = MF.score_pairs(h, src, dst, "mlp", W, b, out_dtype=ob).clone()
        res[tag + "_us"] = round(timeit(lambda: MF.score_pairs(h, src, dst, "mlp", W, b, out_dtype=ob)), 1)
        res[tag + "_Gpairs"] = round(P / res[tag + "_us"] / 1e3, 2)
        # training epilogue: bias + ReLU + dropout (p = 0.5, fixed seed) + sigmoid
        o = torch.empty(P, N, device=dev, dtype=torch.float32)
        fn = "msha_pair_linear_bf16" if ob is not None else "msha_pair_linear"
        s = torch.cuda.current_stream(dev).cuda_stream
        rows = () if ob is not None else (h.shape[0], h.shape[0])
        _lib.call(fn, P, F, N, h.data_ptr(), h.stride(0), src.data_ptr(), h.data_ptr(),
                  h.stride(0), dst.data_ptr(), *rows, W.data_ptr(), b.data_ptr(), 1 | 2 | 4 | 8, 0.5,
                  1234, 7, o.data_ptr(), s)
        outs[tag + "_drop"] = o
    torch.save({k: v.cpu() for k, v in outs.items()}, path)
    print(json.dumps(res), flush=True)


def cmp(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    for k in A:
        d = (A[k].float() - B[k].float()).abs().max().item()
        print(json.dumps({"out": k, "bit_identical": bool(torch.equal(A[k], B[k])), "max_abs_diff": d}))


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if sys.argv[1] == "save":
        save(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
