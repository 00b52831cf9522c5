#!/bin/bash
# round 6: the fp32 MFMA backward with the hs pieces loaded in their own tile
# (lib/alt/hssync.so, BIP3_HSSYNC=1: no spill in the loop) -- bipartite parity with that
# backward forced, then the bip1m leg: mask backward (shipped default) vs MFMA backward
set -o pipefail
O=gpurun_out/r6_ab4${TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
A=msha--gnn_amd/lib/alt/hssync.so
MSHA_GNN_LIB=$A MSHA_BIP3_BWD32=1 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
  tests/test_gpu_bip.py tests/test_gpu_ours.py "tests/test_gpu_parity_full.py::test_bip1m_ourslayer3_core_every_row" -m gpu -p no:cacheprovider \
  > $O/tests.log 2>&1 || { grep -E "^E |FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name lib [env]
  local name=$1 lib=$2; shift 2
  env "$@" MSHA_GNN_LIB=$lib timeout -k 10 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 \
    --no-cpu-baseline --no-r15 --no-dropout-leg --detail $O/$name.json > $O/$name.line 2> $O/$name.err \
    || { tail -20 $O/$name.err; exit 1; }
  echo "== $name"
  python scripts/bench_brief.py $O/$name.json | grep -E "attention_"
}
run mask $A X=1 && run hs32 $A MSHA_BIP3_BWD32=1 && run mask2 $A X=1 && run hs32b $A MSHA_BIP3_BWD32=1
