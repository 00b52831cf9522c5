#!/bin/bash
# Ours intra forward occupancy: Ours parity, then the configs[1] step trace.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ours.py \
  > gpurun_out/r4/ours_tests.log 2>&1 || { tail -30 gpurun_out/r4/ours_tests.log; exit 1; }
tail -1 gpurun_out/r4/ours_tests.log
NROWS=14 bash scripts/trace_train_step.sh r4_ours32c Ours 2015 float32
