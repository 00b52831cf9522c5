#!/bin/bash
# round 6, MFMA bipartite kernels (edge_bip3.hip): parity subsets, then the bip1m leg (and
# R15) with MSHA_BIP3=1 / 0 for A/B.  Output under gpurun_out/r6_bip${TAG}/.
set -o pipefail
O=gpurun_out/r6_bip${TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
if [ -z "$NOTESTS" ]; then
  $T 600 python -u -m pytest ${TESTS:-tests/test_gpu_bip.py tests/test_gpu_ours.py} -m gpu -x -q \
    --timeout 240 --timeout-method thread -p no:cacheprovider ${PYK:+-k "$PYK"} > $O/tests.log 2>&1 \
    || { grep -E "passed|failed|Error|error|assert" $O/tests.log | tail -30; tail -80 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for v in ${VALS:-1 0}; do
  MSHA_BIP3=$v $T 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline \
    --no-r15 --no-dropout-leg --detail $O/bip1m_$v.json > $O/bip1m_$v.line 2> $O/bip1m_$v.err \
    || { tail -20 $O/bip1m_$v.err; exit 1; }
  echo "== MSHA_BIP3=$v"
  python scripts/bench_brief.py $O/bip1m_$v.json | grep -E "bip|head"
done
