#!/bin/bash
# Round-4 parity set: bip kernels, edge-attention / link-predictor / projection kernels,
# Ours (fp32 + bf16 vs fp64), Adam, train.py drop-in, then the bip1m full-size and the
# ablation3 bf16 model tests; bip1m / R15 layer legs and the train.py-literal timing.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bip.py \
  tests/test_gpu_kernels.py tests/test_gpu_ours.py tests/test_gpu_bf16.py tests/test_gpu_optim.py \
  tests/test_dropin.py > gpurun_out/r4/tests_a.log 2>&1 || { tail -60 gpurun_out/r4/tests_a.log; exit 1; }
tail -2 gpurun_out/r4/tests_a.log
$T 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread \
  "tests/test_gpu_parity_full.py::test_bip1m_ourslayer3_core_every_row" \
  "tests/test_gpu_parity_full.py::test_ablation3_bf16_model_vs_fp64" > gpurun_out/r4/tests_b.log 2>&1 \
  || { tail -60 gpurun_out/r4/tests_b.log; exit 1; }
grep -E "bip1m|of elements|passed|failed" gpurun_out/r4/tests_b.log
$T 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline \
  --no-r15 --no-dropout-leg > gpurun_out/r4/bip1m.json 2> gpurun_out/r4/bip1m.err || { tail -20 gpurun_out/r4/bip1m.err; exit 1; }
python scripts/bench_brief.py gpurun_out/r4/bip1m.json
$T 300 python scripts/r4/trainpy_time.py > gpurun_out/r4/trainpy.json 2> gpurun_out/r4/trainpy.err || { tail -20 gpurun_out/r4/trainpy.err; exit 1; }
cat gpurun_out/r4/trainpy.json
