#!/bin/bash
# Whole GPU suite (pytest -m gpu, one process), smoke(), then the driver's default bench
# command (compact line on stdout, detail to gpurun_out/r5/bench_detail.json).
set -o pipefail
O=gpurun_out/r5${TAG:+_$TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
if [ -z "$NOTESTS" ]; then
$T 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/gpu_suite.log 2>&1 || { grep -E "passed|failed|Error|error" $O/gpu_suite.log | tail -30; tail -50 $O/gpu_suite.log; exit 1; }
grep -E "passed|failed" $O/gpu_suite.log | tail -3
fi
$T 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
$T 600 python -u bench.py --detail $O/bench_detail.json ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err \
  || { tail -20 $O/bench.err; exit 1; }
wc -c $O/bench.json
python scripts/bench_brief.py $O/bench_detail.json
