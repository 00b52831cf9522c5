#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_optim.py tests/test_gpu_graph.py > gpurun_out/adam_t.log 2>&1
rc=$?; tail -2 gpurun_out/adam_t.log; [ $rc -ne 0 ] && exit $rc
NROWS=12 scripts/trace_train_step.sh r3_adam Ours 2015 float32 2>&1 | tail -14
