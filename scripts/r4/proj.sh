#!/bin/bash
# line-major skinny projection: GEMM / projection parity, then A/B of the projection
# (PROJ_LINE=1 shipped vs lib/alt/proj0.so) at C4, R15, bip1m.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_bf16.py \
  -k "proj or gemm or skinny or score" > gpurun_out/r4/proj_tests.log 2>&1 || { tail -30 gpurun_out/r4/proj_tests.log; exit 1; }
tail -2 gpurun_out/r4/proj_tests.log
GEMM_AB_BIP1M=1 $T 300 python -u scripts/gemm_ab.py > gpurun_out/r4/proj_ab.log 2>&1 &&
GEMM_AB_BIP1M=1 MSHA_GNN_LIB=$PWD/msha--gnn_amd/lib/alt/proj0.so $T 300 python -u scripts/gemm_ab.py >> gpurun_out/r4/proj_ab.log 2>&1 || { tail -20 gpurun_out/r4/proj_ab.log; exit 1; }
grep '^{' gpurun_out/r4/proj_ab.log
