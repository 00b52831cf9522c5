#!/bin/bash
# head-split bipartite forward and backward: bip tests, bip1m every row, Ours/ablation3 models, then
# bip1m / R15 legs with the split on and off.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 700 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_bip.py \
  "tests/test_gpu_parity_full.py::test_bip1m_ourslayer3_core_every_row" tests/test_gpu_ours.py tests/test_gpu_head.py tests/test_gpu_modules.py \
  > gpurun_out/r4/bipsplit_tests.log 2>&1 || { tail -40 gpurun_out/r4/bipsplit_tests.log; exit 1; }
grep -E "bip1m|passed|failed" gpurun_out/r4/bipsplit_tests.log | tail -14
MSHA_BIP_SPLIT=1 $T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bip.py \
  > gpurun_out/r4/bipsplit_off.log 2>&1 || { tail -40 gpurun_out/r4/bipsplit_off.log; exit 1; }
tail -2 gpurun_out/r4/bipsplit_off.log
for SP in 1 0; do
MSHA_BIP_SPLIT=$SP $T 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline \
  --no-r15 --no-dropout-leg > gpurun_out/r4/bip1m_s$SP.json 2> gpurun_out/r4/bip1m_s$SP.err || { tail -20 gpurun_out/r4/bip1m_s$SP.err; exit 1; }
python scripts/bench_brief.py gpurun_out/r4/bip1m_s$SP.json | head -6
done
NROWS=12 bash scripts/trace_train_step.sh r4_split_ours32 Ours 2015 float32
