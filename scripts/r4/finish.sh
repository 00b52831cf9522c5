#!/bin/bash
# Ours backward finish (mode 0) with its independent loads issued at entry and bgrad in
# LDS: Ours parity (kernels, modules, full-graph steps), then the R15 step trace
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ours.py \
  tests/test_gpu_modules.py tests/test_gpu_parity_full.py tests/test_gpu_bf16.py tests/test_gpu_graph.py > gpurun_out/r4/finish_tests.log 2>&1 \
  || { tail -40 gpurun_out/r4/finish_tests.log; exit 1; }
tail -1 gpurun_out/r4/finish_tests.log
NROWS=16 bash scripts/trace_train_step.sh r4_finish_ours32 Ours 2015 float32
