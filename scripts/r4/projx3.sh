#!/bin/bash
# split-bf16 fp32 projection: projection / GEMM / model parity, then A/B timing vs the
# exact-fp32 MFMA build (lib/alt/projx0.so), then the C4 headline leg.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_bf16.py \
  tests/test_gpu_parity_full.py tests/test_gpu_head.py tests/test_gpu_ours.py tests/test_gpu_modules.py tests/test_gpu_fullsize.py > gpurun_out/r4/projx3_tests.log 2>&1 || { tail -30 gpurun_out/r4/projx3_tests.log; exit 1; }
tail -1 gpurun_out/r4/projx3_tests.log
GEMM_AB_BIP1M=1 $T 300 python -u scripts/gemm_ab.py > gpurun_out/r4/projx3_ab.log 2>&1 &&
GEMM_AB_BIP1M=1 MSHA_GNN_LIB=$PWD/msha--gnn_amd/lib/alt/projx0.so $T 300 python -u scripts/gemm_ab.py >> gpurun_out/r4/projx3_ab.log 2>&1 || { tail -20 gpurun_out/r4/projx3_ab.log; exit 1; }
grep '^{' gpurun_out/r4/projx3_ab.log | grep float32
$T 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-link-score --no-r15 --no-syn2m --no-bip1m --no-dropout-leg \
  > gpurun_out/r4/c4.json 2> gpurun_out/r4/c4.err || { tail -20 gpurun_out/r4/c4.err; exit 1; }
python scripts/bench_brief.py gpurun_out/r4/c4.json
