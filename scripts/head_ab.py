"""Time the model head (msha_head_fwd / _bwd) alone at R15's shape (N 39179, M 32,
2 heads x 64): forward train with / without dropout, eval, and the backward with a
64-row dout (train.py's nll on out[source_index]) -- one JSON line per case."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msha_loader  # noqa: E402

msha_loader.load()
from msha_gnn_amd import functional as MF  # noqa: E402
from msha_gnn_amd.graph import Graph  # noqa: E402


def timeit(fn, reps=20):
    """GPU time per call: `reps` calls captured in one HIP graph, replayed (no host gaps)."""
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    gr.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    dev = torch.device("cuda:0")
    z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests",
                             "golden", "r15_graph.npz"))
    n, m = int(z["n"]), int(z["m"])
    g = Graph.from_csr(z["rowptr"].astype(np.int64), z["col"].astype(np.int64), m, dev)
    H, F = 2, 64
    gen = torch.Generator(device=dev).manual_seed(0)
    u = torch.randn(n, H, F, device=dev, generator=gen)
    v = torch.randn(m, H, F, device=dev, generator=gen)
    W = torch.randn(H * m, m, device=dev, generator=gen) * 0.1
    a = torch.zeros(2 * m, 1, device=dev)
    bns = [(torch.nn.BatchNorm1d(F).to(dev), torch.nn.BatchNorm1d(F).to(dev)) for _ in range(H)]
    params = ([b[0].weight for b in bns] + [b[0].bias for b in bns] + [b[1].weight for b in bns]
              + [b[1].bias for b in bns] + [a])
    res = {}
    for p in (0.0, 0.5):
        res[f"fwd_train_p{p}"] = timeit(lambda: MF._ModelHead.apply(
            u, v, W, g, bns, True, 1e-5, 0.1, 0.2, p, 11, p, 12, *params))
        print(f"fwd_train_p{p}", res[f"fwd_train_p{p}"], flush=True)
    for pair in bns:
        for bn in pair:
            bn.eval()
    res["fwd_eval"] = timeit(lambda: MF._ModelHead.apply(u, v, W, g, bns, False, 1e-5, 0.1, 0.2,
                                                         0.0, 0, 0.0, 0, *params))
    print("fwd_eval", res["fwd_eval"], flush=True)
    if os.environ.get("HEAD_AB_FWD_ONLY"):
        print(json.dumps({k: round(v_, 1) for k, v_ in res.items()}), flush=True)
        return
    for pair in bns:
        for bn in pair:
            bn.train()
    uu = u.clone().requires_grad_(True)
    out = MF._ModelHead.apply(uu, v, W, g, bns, True, 1e-5, 0.1, 0.2, 0.5, 11, 0.5, 12, *params)
    dout = torch.zeros_like(out)
    rows = torch.randint(0, n, (64,), device=dev, generator=gen)
    dout[rows] = torch.randn(64, m, device=dev, generator=gen)
    res["bwd_64rows"] = timeit(lambda: torch.autograd.grad(out, uu, dout, retain_graph=True))
    dout_all = torch.randn_like(out)
    res["bwd_all_rows"] = timeit(lambda: torch.autograd.grad(out, uu, dout_all, retain_graph=True),
                                 reps=4)
    print(json.dumps({k: round(v_, 1) for k, v_ in res.items()}), flush=True)


if __name__ == "__main__":
    main()
