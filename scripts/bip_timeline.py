"""Per-wave timeline of the MFMA bipartite kernels (edge_bip3.hip) in the bip1m / R15
OursLayer3-core step: where a wave's tile time goes.

    MSHA_GNN_LIB=msha--gnn_amd/lib/libmsha_gnn_timeline.so \
        python scripts/bip_timeline.py OUT [bip1m|r15] [f32|bf16]

Needs the diagnostic library (python msha--gnn_amd/build.py --variant timeline).  Lane 0
of every wave stamps (wall clock at 100 MHz, shader clock) at the kernel's marks: entry,
tables staged, per tile (first four tiles of the wave's range) the phase boundaries, loop
end, exit.  Forward phases: softmax (+ lse, keep bits, attd export), attention images,
u (MFMAs + row-piece flush), v MFMAs issued.  Backward phases: att from lse (+ keep bits),
G MFMAs issued, softmax backward (waits for G), d_hc MFMAs issued, d_hs out.

Writes OUT/bip_timeline_<graph>_<dtype>.json and prints per-phase cycle percentiles over
tiles 1-3 of every wave (tile 0 carries the cold start).
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MSHA_GNN_LIB",
                      os.path.join(ROOT, "msha--gnn_amd", "lib", "libmsha_gnn_timeline.so"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import msha_loader  # noqa: E402

msha_loader.load()
from msha_gnn_amd import _lib  # noqa: E402

SLOTS, STRIDE = 8192, 64
PHASES = {0: ["softmax", "images", "u", "v_issue"],
          1: ["att", "G_issue", "softmax_bwd", "d_hc_issue", "d_hs"]}


def pct(a, q=(10, 50, 90)):
    a = np.asarray(a, np.float64)
    return {f"p{p}": round(float(np.percentile(a, p)), 1) for p in q} if len(a) else {}


def decode(raw, bwd):
    half = SLOTS // 2
    rows = raw[bwd * half:(bwd + 1) * half]
    per = len(PHASES[bwd]) + 1
    nm = 2 + per * 4 + 2
    waves = []
    for slot, row in enumerate(rows):
        if row[1] == 0:
            continue
        m = row[2:2 + 2 * nm].reshape(nm, 2).astype(np.int64)
        hw = int(row[0]) & 0xFFFFFFFF
        waves.append(dict(tag=int(row[1]), simd=(hw >> 4) & 3, cu=(hw >> 8) & 15,
                          xcc=int(row[0]) >> 32, wv=slot % 8, rt=m[:, 0], mt=m[:, 1]))
    if not waves:
        return None
    t0 = min(int(w["rt"][0]) for w in waves)
    out = {"waves": len(waves), "tag": waves[0]["tag"]}
    ent = [(w["rt"][0] - t0) * 0.01 for w in waves]
    ex = [(w["rt"][nm - 1] - t0) * 0.01 for w in waves]
    out["entry_us"] = pct(ent, (0, 50, 100))
    out["exit_us"] = pct(ex, (0, 50, 100))
    cyc = lambda w, a, b: int(w["mt"][b] - w["mt"][a])  # noqa: E731
    out["stage_tables_cyc"] = pct([cyc(w, 0, 1) for w in waves])
    ph = {p: [] for p in PHASES[bwd]}
    tiles = []
    for w in waves:
        for it in range(1, 4):
            s = 2 + per * it
            if w["mt"][s + per - 1] == 0 or (it + 1 < 4 and w["mt"][s + per] == 0):
                continue
            nxt = s + per if it + 1 < 4 else None
            for k, p in enumerate(PHASES[bwd]):
                ph[p].append(int(w["mt"][s + k + 1] - w["mt"][s + k]))
            if nxt is not None:
                tiles.append(int(w["mt"][nxt] - w["mt"][s]))
    out["tile_cyc"] = pct(tiles)
    out["phase_cyc"] = {p: pct(v) for p, v in ph.items()}
    lend = 2 + per * 4
    out["loop_cyc"] = pct([cyc(w, 1, lend) for w in waves])
    out["epilogue_cyc"] = pct([cyc(w, lend, lend + 1) for w in waves])
    out["wave_cyc"] = pct([cyc(w, 0, lend + 1) for w in waves])
    # where the spread comes from: the loop by wave of the block (waves w and w + 4 share a
    # SIMD, w + 4 dispatched second) and by XCD
    out["loop_cyc_by_wave"] = {k: pct([cyc(w, 1, lend) for w in waves if w["wv"] == k], (50,))["p50"]
                               for k in range(8)}
    out["loop_cyc_by_xcc"] = {k: pct([cyc(w, 1, lend) for w in waves if w["xcc"] == k], (50,))["p50"]
                              for k in sorted({w["xcc"] for w in waves})}
    out["window_us"] = round(max(ex), 2)
    return out


def main(out, graph="bip1m", dt="f32"):
    os.makedirs(out, exist_ok=True)
    dev = torch.device("cuda:0")
    dtype = torch.bfloat16 if dt == "bf16" else torch.float32
    if graph == "bip1m":
        rowptr, col, n, m = bench.bip_graph()
    else:
        z = np.load(os.path.join(ROOT, "tests", "golden", "r15_graph.npz"))
        rowptr, col, n, m = z["rowptr"].astype(np.int64), z["col"].astype(np.int64), int(z["n"]), int(z["m"])
    lay = bench.Layer(dev, rowptr, col, n, m, 128, 2, 64, 0, dtype=dtype, v_branch=True)
    assert lay.bip, "not a bipartite layer"
    buf = torch.zeros(SLOTS * STRIDE, dtype=torch.int64, device=dev)
    for _ in range(3):
        lay.step()
    torch.cuda.synchronize()
    _lib.call("msha_debug_bip_timeline", buf.data_ptr(), SLOTS)
    lay.step()
    torch.cuda.synchronize()
    _lib.call("msha_debug_bip_timeline", None, 0)
    raw = buf.view(SLOTS, STRIDE).cpu().numpy().view(np.uint64)
    res = {"graph": graph, "dtype": dt, "rows": n,
           "bip3_bwd32": os.environ.get("MSHA_BIP3_BWD32", "0"),
           "fwd": decode(raw, 0), "bwd": decode(raw, 1)}
    path = os.path.join(out, f"bip_timeline_{graph}_{dt}.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else os.path.join(ROOT, "gpurun_out", "bip_tl"), *a[1:3])
