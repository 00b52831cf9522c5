#!/bin/bash
# the whole GPU suite on the bf16 row-score default, then the head rows-per-wave A/B
set -o pipefail
mkdir -p gpurun_out/r4f
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4f/gpu_suite_mid.log 2>&1 || { tail -60 gpurun_out/r4f/gpu_suite_mid.log; exit 1; }
tail -1 gpurun_out/r4f/gpu_suite_mid.log
bash scripts/r4/headrpw.sh
