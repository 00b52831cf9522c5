import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import msha_loader
msha_loader.load()
from msha_gnn_amd import functional as MF, _lib
orig = _lib.call
def call(name, *a):
    if name.startswith("msha_gemm") or name.startswith("msha_project"):
        print(name, [x for x in a[:11] if isinstance(x, int) and abs(x) < 10**9], flush=True)
    return orig(name, *a)
_lib.call = call
orig_load = _lib.load
import bench
r = bench.train_step_leg(torch.device("cuda:0"), "2015", "Ours", steps=1, warmup=0)
print(r)
