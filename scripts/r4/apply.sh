#!/bin/bash
# model-head backward apply reading dz only for the loss's rows: head / model parity,
# then the R15 step trace
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_head.py \
  tests/test_gpu_modules.py tests/test_gpu_parity_full.py tests/test_gpu_bf16.py > gpurun_out/r4/apply_tests.log 2>&1 \
  || { tail -40 gpurun_out/r4/apply_tests.log; exit 1; }
tail -1 gpurun_out/r4/apply_tests.log
NROWS=16 bash scripts/trace_train_step.sh r4_apply_ours32 Ours 2015 float32
