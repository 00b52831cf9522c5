"""Build the gfx950 HIP library ``lib/libmsha_gnn.so`` in-tree with hipcc.

    python msha--gnn_amd/build.py [--force]

Each ``csrc/*.hip`` is compiled to an object (cached by mtime against the sources
and headers), then linked into one shared library whose exported symbols are the
``extern "C"`` functions of ``include/msha_gnn.h``.  The library links the HIP
runtime by its soname, so inside a torch process it binds to the runtime torch
already loaded (one HIP runtime per process, shared streams and allocations).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIBDIR = os.path.join(PKG, "lib")
# variants: "" (shipped) or "timeline" (-DSK_TIMELINE: the skinny kernels' per-wave
# timeline, msha_debug_timeline; lib/libmsha_gnn_timeline.so, selected with MSHA_GNN_LIB)
VARIANTS = {"": [], "timeline": ["-DSK_TIMELINE"],
            # gather-layout forward A/Bs (edge_geo.h knobs)
            "nopf": ["-DGL_PREFETCH_F32=0", "-DGL_PREFETCH_BF16=0", "-DGL_EPL_F32=2"],
            # bipartite kernels' streamed bytes per row group (edge_bip.hip grp_rows)
            "bipg16": ["-DBIP_GRP_BYTES=16384"]}
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libmsha_gnn.so")
ARCH = os.environ.get("MSHA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", INCLUDE,
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-parameter",
          "-fvisibility=hidden", "-munsafe-fp-atomics"]


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, objdir=OBJDIR, defines=()):
    obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
    if not _stale(obj, [src] + _headers()):
        return obj, None
    cmd = [HIPCC, *CFLAGS, *defines, "-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    os.replace(obj + ".tmp", obj)
    return obj, None


def build(force: bool = False, jobs: int | None = None, variant: str = "") -> str:
    defines = VARIANTS[variant]
    objdir = OBJDIR + (f"_{variant}" if variant else "")
    lib = LIB.replace(".so", f"_{variant}.so") if variant else LIB
    os.makedirs(objdir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if force:
        for o in glob.glob(os.path.join(objdir, "*.o")):
            os.remove(o)
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda src: _compile(src, objdir, defines), srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if force or _stale(lib, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    v = sys.argv[sys.argv.index("--variant") + 1] if "--variant" in sys.argv else ""
    print(build(force="--force" in sys.argv, variant=v))
