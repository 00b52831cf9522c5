"""Compile the oracle's C restatement (TEST INFRASTRUCTURE / CPU BASELINE ONLY).

    python oracle/build_oracle.py   ->  oracle/_build/libmsha_oracle.so

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


def build(force=False):
    os.makedirs(OUT_DIR, exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    cmd = ["gcc", "-O3", "-march=x86-64-v2", "-fopenmp", "-shared", "-fPIC", SRC, "-o",
           LIB + ".tmp", "-lm"]
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True))
