#!/bin/bash
# model-head backward rows per wave A/B (MSHA_HEAD_RPW: 16 shipped, 32, 64): head parity at
# 64, then the R15 Ours 2015 fp32 step trace per setting
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
MSHA_HEAD_RPW=64 $T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_head.py \
  tests/test_gpu_modules.py > gpurun_out/r4/headrpw_tests.log 2>&1 || { tail -40 gpurun_out/r4/headrpw_tests.log; exit 1; }
tail -1 gpurun_out/r4/headrpw_tests.log
for RPW in 16 32 64; do
  echo "== MSHA_HEAD_RPW=$RPW"
  MSHA_HEAD_RPW=$RPW NROWS=4 bash scripts/trace_train_step.sh r4_rpw$RPW Ours 2015 float32 || exit 1
  grep -h "head_bwd" gpurun_out/trace_step_r4_rpw$RPW/run_kernel_stats.csv | cut -d, -f1-6 | head -3
done
