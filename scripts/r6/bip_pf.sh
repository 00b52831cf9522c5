#!/bin/bash
# round 6: the bip1m leg on the shipped library and on lib/alt/pf1.so (BIP3_PF=1: the
# forward's hs fragments one tile ahead instead of two)
set -o pipefail
O=gpurun_out/r6_bippf${TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
for lib in "" msha--gnn_amd/lib/alt/pf1.so; do
  tag=${lib:+pf1}; tag=${tag:-pf2}
  MSHA_GNN_LIB=${lib:-msha--gnn_amd/lib/libmsha_gnn.so} timeout -k 10 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline \
    --no-r15 --no-dropout-leg --detail $O/bip1m_$tag.json > $O/bip1m_$tag.line 2> $O/bip1m_$tag.err \
    || { tail -20 $O/bip1m_$tag.err; exit 1; }
  echo "== $tag"
  python scripts/bench_brief.py $O/bip1m_$tag.json | grep -E "bip|head"
done
