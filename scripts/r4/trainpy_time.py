"""train.py-as-written step time (bench.train_py_literal_leg) for ablation3 and Ours on the
2015 graph, plus a torch-profiler table of one window (host time per op) when --prof."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
for kind in ("ablation3", "Ours"):
    print(json.dumps(bench.train_py_literal_leg(dev, kind)), flush=True)
