"""Per-block timeline of head_bwd_rows2 (the model head's backward row pass, split form)
in the Ours 2015 fp32 train step.  Needs the diagnostic library:

    python msha--gnn_amd/build.py --variant timeline
    MSHA_GNN_LIB=msha--gnn_amd/lib/libmsha_gnn_timeline.so python scripts/head_timeline.py

Marks (lane 0 of each block; wall clock at 100 MHz): 0 entry, 1 flagged-row count done,
2 tables + transposes in LDS, then per row (row located, head_row_fwd done, row done),
30 partials written.  Prints each active block's marks in us from the launch's first entry.
"""
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

dev = torch.device("cuda:0")
buf = torch.zeros(2048 * 64, dtype=torch.int64, device=dev)
_lib.call("msha_debug_head_timeline", buf.data_ptr())
bench.train_step_leg(dev, "2015", "Ours", steps=2, warmup=2)
torch.cuda.synchronize()
_lib.call("msha_debug_head_timeline", None)
raw = buf.view(2048, 64).cpu().numpy().view(np.uint64).astype(np.int64)
t0 = raw[:, 0][raw[:, 0] > 0].min()
act = []
for b in range(1024):  # rows2 slots
    r = raw[b]
    if r[0] == 0:
        continue
    wall = r[0::2]
    marks = {k: (wall[k] - t0) / 100.0 for k in range(32) if wall[k] > 0}
    act.append((b, marks))
idle = [m for b, m in act if 2 not in m]
print(f"blocks stamped {len(act)}, without rows {len(idle)}; "
      f"idle exit (mark 1) median {np.median([m[1] for m in idle]):.2f} us" if idle else "")
for b, m in act:
    if 2 in m and b < 8:
        print(b, " ".join(f"{k}:{v:.2f}" for k, v in sorted(m.items())))

# head_bwd_apply blocks (slots 1024 + block): 0 entry, 1 coefficients loaded, 2 row pass
# issued, 30 exit (block 0: the v side)
ap = raw[1024:]
ap = ap[ap[:, 0] > 0]
if len(ap):
    t0a = ap[:, 0].min()
    w = (ap[:, 0::2] - t0a) / 100.0
    def col(k):
        v = w[:, k][ap[:, 2 * k] > 0]
        return v
    print(f"apply blocks {len(ap)}: entry min/med/max {col(0).min():.2f}/{np.median(col(0)):.2f}/{col(0).max():.2f} us")
    for k in (1, 2, 30):
        v = col(k)
        if len(v):
            print(f"  mark {k}: min/med/max {v.min():.2f}/{np.median(v):.2f}/{v.max():.2f} us (n={len(v)})")
    b0 = raw[1024]
    print("  block 0 (v side):", " ".join(f"{k}:{(b0[2*k]-t0a)/100:.2f}" for k in range(31) if b0[2*k] > 0))
