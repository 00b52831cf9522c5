"""Run only bench.py's configs[1] train-step leg (for profiling)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "Ours"
year = sys.argv[2] if len(sys.argv) > 2 else "2015"
dtype = getattr(torch, sys.argv[3]) if len(sys.argv) > 3 else torch.float32
print(json.dumps(bench.train_step_leg(torch.device("cuda:0"), year, kind, dtype=dtype)))
