#!/bin/bash
# projection waves per SIMD: shipped (2) vs lib/alt/wps3.so (3), fp32 split / bf16.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
GEMM_AB_BIP1M=1 $T 300 python -u scripts/gemm_ab.py > gpurun_out/r4/wps_ab.log 2>&1 &&
GEMM_AB_BIP1M=1 MSHA_GNN_LIB=$PWD/msha--gnn_amd/lib/alt/wps3.so $T 300 python -u scripts/gemm_ab.py >> gpurun_out/r4/wps_ab.log 2>&1 || { tail -20 gpurun_out/r4/wps_ab.log; exit 1; }
grep '^{' gpurun_out/r4/wps_ab.log
