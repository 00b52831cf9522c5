#!/bin/bash
# bip kernels quick loop: parity (bip tests + bip1m every row), bip1m / R15 legs.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_bip.py \
  "tests/test_gpu_parity_full.py::test_bip1m_ourslayer3_core_every_row" ${EXTRA_TESTS} \
  > gpurun_out/r4/bipq_tests.log 2>&1 || { tail -40 gpurun_out/r4/bipq_tests.log; exit 1; }
grep -E "bip1m|passed|failed" gpurun_out/r4/bipq_tests.log | tail -14
$T 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline \
  --no-r15 --no-dropout-leg > gpurun_out/r4/bip1m.json 2> gpurun_out/r4/bip1m.err || { tail -20 gpurun_out/r4/bip1m.err; exit 1; }
$T 300 python -u bench.py --workload r15 --steps 20 --warmup 5 --no-cpu-baseline --no-dropout-leg \
  > gpurun_out/r4/r15.json 2> gpurun_out/r4/r15.err || { tail -20 gpurun_out/r4/r15.err; exit 1; }
python scripts/bench_brief.py gpurun_out/r4/bip1m.json gpurun_out/r4/r15.json
