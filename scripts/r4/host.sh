#!/bin/bash
# host-overhead pass: the prologue / model tests, then the train.py-literal phases.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_head.py \
  tests/test_gpu_optim.py tests/test_gpu_ours.py tests/test_dropin.py tests/test_gpu_graph.py \
  > gpurun_out/r4/host_tests.log 2>&1 || { tail -30 gpurun_out/r4/host_tests.log; exit 1; }
tail -1 gpurun_out/r4/host_tests.log
timeout -k 10 300 python -u scripts/r4/trainpy_time.py --phases > gpurun_out/r4/trainpy_phases.log 2>&1 || { tail -30 gpurun_out/r4/trainpy_phases.log; exit 1; }
grep '^{' gpurun_out/r4/trainpy_phases.log
