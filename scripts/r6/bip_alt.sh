#!/bin/bash
# round 6: the bip1m leg on the shipped library and on lib/alt/<name>.so variants
# (ALTS="ust0 hst0"); TESTS=1 runs the bipartite parity tests on the shipped library first
set -o pipefail
O=gpurun_out/r6_alt${TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_bip.py tests/test_gpu_ours.py -m gpu > $O/tests.log 2>&1 \
    || { grep -E "^E |FAILED" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for name in main $ALTS; do
  lib=msha--gnn_amd/lib/libmsha_gnn.so
  [ "$name" != main ] && lib=msha--gnn_amd/lib/alt/$name.so
  MSHA_GNN_LIB=$lib timeout -k 10 300 python -u bench.py --workload ${WL:-bip1m} --steps 10 --warmup 3 --no-cpu-baseline \
    --no-r15 --no-dropout-leg --detail $O/$name.json > $O/$name.line 2> $O/$name.err \
    || { tail -20 $O/$name.err; exit 1; }
  echo "== $name"
  python scripts/bench_brief.py $O/$name.json | grep -E "${GREP:-bip|head}"
done
