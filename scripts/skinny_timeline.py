"""Per-wave timeline of the skinny fp32 projection and weight gradient at C4 (VERDICT r2,
next-round item 5): where the launch time goes that the MFMA pipe does not use.

    MSHA_GNN_LIB=msha--gnn_amd/lib/libmsha_gnn_timeline.so python scripts/skinny_timeline.py OUT

Needs the diagnostic library (python msha--gnn_amd/build.py --variant timeline): lane 0 of
every wave stamps (wall clock at 100 MHz, shader clock) at the kernel's marks into the
buffer msha_debug_timeline installs.  proj_kernel marks: entry, W resident (after the
block's W copy + barrier), per item (start, MFMAs done), exit.  wgrad_kernel marks:
entry, row loop start, row loop done, block sum done, exit.

Writes OUT/timeline_<kernel>.json (per-wave records and a summary) and prints the summary:
the launch window, when waves start (dispatch ramp), the W fill, MFMA and epilogue cycles
per item, the tail (last wave's exit vs the median), and per-SIMD occupancy of the window.
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
import msha_loader  # noqa: E402

msha_loader.load()
from msha_gnn_amd import _lib  # noqa: E402
from msha_gnn_amd import functional as MF  # noqa: E402

SLOTS, STRIDE = 16384, 64


def capture(fn, buf):
    fn()
    torch.cuda.synchronize()
    buf.zero_()
    _lib.call("msha_debug_timeline", buf.data_ptr(), SLOTS)
    fn()
    torch.cuda.synchronize()
    _lib.call("msha_debug_timeline", None, 0)
    return buf.view(SLOTS, STRIDE).cpu().numpy().view(np.uint64)


def decode(raw, n_marks_fixed):
    """Per wave: location, wall-clock marks (us from the launch's first entry) and shader
    clock marks (cycles from its own entry)."""
    waves = []
    for row in raw:
        if row[1] == 0:
            continue
        hw = int(row[0]) & 0xFFFFFFFF
        xcc = int(row[0]) >> 32
        marks = row[2:]
        k = int(np.nonzero(marks)[0].max()) + 1 if marks.any() else 0
        marks = marks[:k].reshape(-1, 2)
        waves.append(dict(xcc=xcc, se=(hw >> 13) & 7, sh=(hw >> 12) & 1, cu=(hw >> 8) & 15,
                          simd=(hw >> 4) & 3, wave=hw & 15, rt=marks[:, 0].astype(np.int64),
                          mt=marks[:, 1].astype(np.int64)))
    t0 = min(int(w["rt"][0]) for w in waves)
    for w in waves:
        w["us"] = (w["rt"] - t0) * 0.01  # 100 MHz wall clock
        w["cyc"] = w["mt"] - w["mt"][0]
    return waves


def pct(a, q=(0, 10, 50, 90, 100)):
    a = np.asarray(a, np.float64)
    return {f"p{p}": round(float(np.percentile(a, p)), 2) for p in q} if len(a) else {}


def summarize(waves, kind):
    end = max(float(w["us"][-1]) for w in waves)
    s = {"waves": len(waves), "window_us": round(end, 2),
         "entry_us": pct([w["us"][0] for w in waves]),
         "exit_us": pct([w["us"][-1] for w in waves])}
    if kind == "proj":
        s["wfill_cycles"] = pct([w["cyc"][1] for w in waves])
        s["wfill_us"] = pct([w["us"][1] - w["us"][0] for w in waves])
        mf, ep, items = [], [], []
        for w in waves:
            m = w["cyc"]
            n_it = (len(m) - 3) // 2
            items.append(n_it)
            for i in range(n_it):
                st, md = m[2 + 2 * i], m[3 + 2 * i]
                nx = m[4 + 2 * i] if i + 1 < n_it else m[-1]
                mf.append(md - st)
                ep.append(nx - md)
        s["items_per_wave"] = pct(items)
        s["mfma_cycles_per_item"] = pct(mf)
        s["epilogue_cycles_per_item"] = pct(ep)
        s["mfma_share_of_wave_cycles"] = round(float(np.sum(mf)) / float(
            sum(int(w["cyc"][-1]) for w in waves)), 3)
    else:
        s["rows_loop_cycles"] = pct([w["cyc"][2] - w["cyc"][1] for w in waves])
        s["block_sum_cycles"] = pct([w["cyc"][3] - w["cyc"][2] for w in waves])
        s["store_cycles"] = pct([w["cyc"][4] - w["cyc"][3] for w in waves])
        s["loop_share_of_wave_cycles"] = round(float(sum(int(w["cyc"][2] - w["cyc"][1])
                                                         for w in waves)) / float(
            sum(int(w["cyc"][-1]) for w in waves)), 3)
    # per SIMD: union of its waves' lifetimes over the launch window
    simds = {}
    for w in waves:
        simds.setdefault((w["xcc"], w["se"], w["sh"], w["cu"], w["simd"]), []).append(
            (float(w["us"][0]), float(w["us"][-1])))
    busy, first, last = [], [], []
    for iv in simds.values():
        iv.sort()
        tot, cs, ce = 0.0, iv[0][0], iv[0][1]
        for a, b in iv[1:]:
            if a > ce:
                tot += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        tot += ce - cs
        busy.append(tot / end)
        first.append(iv[0][0])
        last.append(max(b for _, b in iv))
    s["simds"] = len(simds)
    s["simd_busy_fraction"] = pct(busy)
    s["simd_first_entry_us"] = pct(first)
    s["simd_last_exit_us"] = pct(last)
    s["launch_without_live_wave"] = round(1.0 - float(np.mean(busy)), 3)
    return s


def main(out, n=100_000, H=8, F=16, kinds=("proj", "wgrad")):
    os.makedirs(out, exist_ok=True)
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    K = 128
    X = torch.rand(n, K, generator=g).to(dev)
    W = (torch.randn(K, H * F, generator=g) * K ** -0.5).to(dev)
    al = torch.randn(H, F, generator=g).to(dev)
    ar = torch.randn(H, F, generator=g).to(dev)
    dh = torch.randn(n, H * F, generator=g).to(dev)
    d1 = torch.randn(n, H, generator=g).to(dev)
    d2 = torch.randn(n, H, generator=g).to(dev)
    buf = torch.zeros(SLOTS * STRIDE, dtype=torch.int64, device=dev)
    res = {}
    T = torch.randn(n, H * F, generator=g).to(dev)
    legs = {"proj": lambda: MF.project_scores(X, W, al, ar, heads=H),
            "wgrad": lambda: MF.gemm_head_outer(X.t(), dh, 1, (H, F, d1, al, d2, ar)),
            # the score-vector column sums fused in (bip1m's and C4's form)
            "wgrad_cs": lambda: MF._wgrad_colsum(X, dh, (H, F, d1, al, d2, ar), T)}
    for kind in kinds:
        fn = legs[kind]
        waves = decode(capture(fn, buf), 0)
        summ = summarize(waves, "wgrad" if kind.startswith("wgrad") else kind)
        res[kind] = summ
        json.dump({"summary": summ,
                   "waves": [{k: (v.tolist() if isinstance(v, np.ndarray) else v)
                              for k, v in w.items() if k not in ("rt", "mt")} for w in waves]},
                  open(os.path.join(out, f"timeline_{kind}.json"), "w"))
        print(kind, json.dumps(summ, indent=1))
    json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    # OUT [rows heads feat kind,kind]: e.g. OUT 1000000 2 64 wgrad_cs (the bip1m shape)
    a = sys.argv[1:]
    main(a[0] if a else os.path.join(ROOT, "gpurun_out", "timeline"),
         *([int(a[1]), int(a[2]), int(a[3])] if len(a) > 3 else []),
         *([tuple(a[4].split(","))] if len(a) > 4 else []))
