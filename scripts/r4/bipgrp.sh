#!/bin/bash
# bipartite row-group size A/B: the shipped 8 KB groups vs the bipg16 variant
# (-DBIP_GRP_BYTES=16384, lib/libmsha_gnn_bipg16.so): bip tests, bip1m legs, R15 Ours step
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
V=msha--gnn_amd/lib/libmsha_gnn_bipg16.so
MSHA_GNN_LIB=$V $T 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bip.py \
  > gpurun_out/r4/bipg16_tests.log 2>&1 || { tail -40 gpurun_out/r4/bipg16_tests.log; exit 1; }
tail -1 gpurun_out/r4/bipg16_tests.log
for L in "" $V; do
  tag=$([ -z "$L" ] && echo g8 || echo g16)
  MSHA_GNN_LIB=${L:-msha--gnn_amd/lib/libmsha_gnn.so} $T 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 \
    --no-cpu-baseline --no-dropout-leg > gpurun_out/r4/bip1m_$tag.json 2> gpurun_out/r4/bip1m_$tag.err \
    || { tail -20 gpurun_out/r4/bip1m_$tag.err; exit 1; }
  echo "== $tag"; python scripts/bench_brief.py gpurun_out/r4/bip1m_$tag.json | head -12
done
