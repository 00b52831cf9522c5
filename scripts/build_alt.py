"""Build an alternative library for A/B runs: one csrc file recompiled from a given
source (default: the working tree's) with extra -D flags, linked with the other
objects of the main build.  Output: msha--gnn_amd/lib/alt/<name>.so

    python scripts/build_alt.py NAME edge_attention [--src FILE] [-DCOLS_NG=4 ...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "msha--gnn_amd"))
import build as B  # noqa: E402


def main():
    name, unit = sys.argv[1], sys.argv[2]
    rest = sys.argv[3:]
    src = os.path.join(B.CSRC, unit + ".hip")
    if "--src" in rest:
        i = rest.index("--src")
        src = rest[i + 1]
        rest = rest[:i] + rest[i + 2:]
    B.build()
    alt = os.path.join(B.LIBDIR, "alt")
    os.makedirs(alt, exist_ok=True)
    obj = os.path.join(alt, f"{name}_{unit}.o")
    subprocess.run([B.HIPCC, *B.CFLAGS, "-I", B.CSRC, *rest, "-c", src, "-o", obj], check=True)
    objs = [os.path.join(B.OBJDIR, f) for f in sorted(os.listdir(B.OBJDIR))
            if f.endswith(".o") and f != unit + ".o"]
    out = os.path.join(alt, name + ".so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", obj, *objs, "-o",
                    out], check=True)
    os.remove(obj)
    print(out)


if __name__ == "__main__":
    main()
