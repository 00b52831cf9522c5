#!/bin/bash
# round 6: backward row inputs two tiles ahead (lib/alt/apfb.so) against the shipped library,
# and the fp32 MFMA backward (MSHA_BIP3_BWD32=1) against the mask kernel, bip1m leg
set -o pipefail
O=gpurun_out/r6_ab3${TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name lib [env]
  local name=$1 lib=$2; shift 2
  env "$@" MSHA_GNN_LIB=$lib timeout -k 10 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 \
    --no-cpu-baseline --no-r15 --no-dropout-leg --detail $O/$name.json > $O/$name.line 2> $O/$name.err \
    || { tail -20 $O/$name.err; exit 1; }
  echo "== $name"
  python scripts/bench_brief.py $O/$name.json | grep -E "attention_"
}
M=msha--gnn_amd/lib/libmsha_gnn.so
A=msha--gnn_amd/lib/alt/apfb.so
run main $M X=1 && run apfb $A X=1 && run bwd32 $M MSHA_BIP3_BWD32=1 && run main2 $M X=1 && run apfb2 $A X=1 && run bwd32b $M MSHA_BIP3_BWD32=1
