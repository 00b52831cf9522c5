#!/bin/bash
# round 6: the backward's row inputs two tiles ahead (lib/alt/apfb.so, BIP3_APF_B=2) against
# the shipped library (priority turns, spill-free fp32 MFMA backward), bip1m leg, two pairs
set -o pipefail
O=gpurun_out/r6_ab5${TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name lib
  MSHA_GNN_LIB=$2 timeout -k 10 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 \
    --no-cpu-baseline --no-r15 --no-dropout-leg --detail $O/$1.json > $O/$1.line 2> $O/$1.err \
    || { tail -20 $O/$1.err; exit 1; }
  echo "== $1"
  python scripts/bench_brief.py $O/$1.json | grep -E "attention_"
}
M=msha--gnn_amd/lib/libmsha_gnn.so
A=msha--gnn_amd/lib/alt/apfb.so
run main $M && run apfb $A && run main2 $M && run apfb2 $A
