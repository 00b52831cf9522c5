#!/bin/bash
# Whole GPU suite (pytest -m gpu, one process), then the bip1m / R15 legs and the
# train.py-literal timing.  Output under gpurun_out/r4/.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4/gpu_suite.log 2>&1 || { grep -E "passed|failed|Error|error" gpurun_out/r4/gpu_suite.log | tail -30; tail -50 gpurun_out/r4/gpu_suite.log; exit 1; }
grep -E "bip1m|of elements|passed|failed" gpurun_out/r4/gpu_suite.log | tail -30
$T 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline \
  --no-r15 --no-dropout-leg > gpurun_out/r4/bip1m.json 2> gpurun_out/r4/bip1m.err || { tail -20 gpurun_out/r4/bip1m.err; exit 1; }
$T 300 python -u bench.py --workload r15 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/r4/r15.json 2> gpurun_out/r4/r15.err || { tail -20 gpurun_out/r4/r15.err; exit 1; }
python scripts/bench_brief.py gpurun_out/r4/bip1m.json gpurun_out/r4/r15.json
$T 300 python scripts/r4/trainpy_time.py > gpurun_out/r4/trainpy.json 2> gpurun_out/r4/trainpy.err || { tail -20 gpurun_out/r4/trainpy.err; exit 1; }
cat gpurun_out/r4/trainpy.json
