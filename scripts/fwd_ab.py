"""A/B timing of the forward edge-attention kernel variants on C4 shapes (GPU box).

    python scripts/fwd_ab.py [--workloads syn100k,syn2m] [--iters 20]

Runs msha_edge_attention_fwd under each environment variant (MSHA_FWD_BAT = batched
gathers on/off, MSHA_FWD_WAVES = grid cap), reports mean HIP-event time per launch and
the algorithmic GB/s (bench.fwd_bytes), and checks every variant's u / lse bitwise
against the first one.  MSHA_GNN_LIB selects another build of the library.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import msha_loader  # noqa: E402

msha_loader.load()
from msha_gnn_amd import functional as MF  # noqa: E402
from msha_gnn_amd.graph import Graph  # noqa: E402

VARIANTS = [
    {"MSHA_FWD_BAT": "0"},
    {"MSHA_FWD_BAT": "1", "MSHA_FWD_WAVES": "0"},
    {"MSHA_FWD_BAT": "1", "MSHA_FWD_WAVES": "16384"},
    {"MSHA_FWD_BAT": "1", "MSHA_FWD_WAVES": "32768"},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="syn100k,syn2m")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtypes", default="f32,bf16")
    ap.add_argument("--variants", default=None, help="JSON list of env dicts")
    args = ap.parse_args()
    variants = json.loads(args.variants) if args.variants else VARIANTS
    dev = torch.device("cuda:0")
    res = []
    for wl in args.workloads.split(","):
        w = bench.WORKLOADS[wl]
        n, H, F = w["n"], w["heads"], w["feat"]
        rowptr, col = bench.synth_graph(n, w["e"], seed=0)
        g = Graph.from_csr(rowptr, col, n, dev)
        gen = torch.Generator().manual_seed(3)
        el = torch.randn(n, H, generator=gen).to(dev)
        er = torch.randn(n, H, generator=gen).to(dev)
        hc32 = torch.randn(n, H, F, generator=gen).to(dev)
        for dts in args.dtypes.split(","):
            dt = torch.float32 if dts == "f32" else torch.bfloat16
            hc = hc32.to(dt)
            nbytes = bench.fwd_bytes(n, n, len(col), H, F, 4 if dts == "f32" else 2)
            ref = None
            for var in variants:
                os.environ.update(var)
                for _ in range(3):
                    u = MF.edge_attention(g, el, er, hc)
                torch.cuda.synchronize()
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(args.iters)]
                for a, b in evs:
                    a.record()
                    u = MF.edge_attention(g, el, er, hc)
                    b.record()
                torch.cuda.synchronize()
                us = float(np.median([a.elapsed_time(b) for a, b in evs])) * 1e3
                same = None
                if ref is None:
                    ref = u.clone()
                else:
                    same = bool(torch.equal(u, ref))
                r = {"lib": os.path.basename(os.environ.get("MSHA_GNN_LIB", "default")),
                     "workload": wl, "dtype": dts, "variant": var, "us": round(us, 1),
                     "GBs": round(nbytes / us / 1e3, 0), "bitwise_same": same}
                print(json.dumps(r), flush=True)
                res.append(r)
    return res


if __name__ == "__main__":
    main()
