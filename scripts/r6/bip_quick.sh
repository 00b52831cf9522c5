#!/bin/bash
# round 6: bipartite parity (test_gpu_bip + test_gpu_ours) then the bip1m leg, shipped library
set -o pipefail
O=gpurun_out/r6_q${TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread ${TESTS:-tests/test_gpu_bip.py tests/test_gpu_ours.py} -m gpu > $O/tests.log 2>&1 \
  || { grep -E "^E |FAILED" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --workload ${WL:-bip1m} --steps 10 --warmup 3 --no-cpu-baseline \
  --no-r15 --no-dropout-leg --detail $O/bench.json > $O/bench.line 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python scripts/bench_brief.py $O/bench.json | grep -E "${GREP:-bip|head}"
