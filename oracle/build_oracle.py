"""Compile the oracle's C restatement (TEST INFRASTRUCTURE / CPU BASELINE ONLY).

    python oracle/build_oracle.py   ->  oracle/_build/libmsha_oracle.so (fp32, CPU baseline)
                                        oracle/_build/libmsha_oracle64.so (fp64 checker)

The reference itself is pure Python (no C/C++ to build), so there is no
oracle/_ref: parity is pinned by golden vectors produced by importing the
reference modules (tests/golden/make_golden.py).
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "edge_attention_cpu.c")
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "libmsha_oracle.so")
LIB64 = os.path.join(OUT_DIR, "libmsha_oracle64.so")  # REAL = double, symbols *_f64


def _build_one(out, defines, force):
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(SRC):
        return out
    cmd = ["gcc", "-O3", "-march=x86-64-v2", "-fopenmp", "-shared", "-fPIC", *defines, SRC,
           "-o", out + ".tmp", "-lm"]
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build(force=False):
    os.makedirs(OUT_DIR, exist_ok=True)
    _build_one(LIB64, ["-DREAL=double", "-DSFX(n)=n##_f64"], force)
    return _build_one(LIB, [], force)


if __name__ == "__main__":
    print(build(force=True))
