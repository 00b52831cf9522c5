#!/bin/bash
# A/B of alternative library builds (scripts/build_alt.py -> msha--gnn_amd/lib/alt/*.so)
# on the headline bench legs; each run is its own process under its own time limit,
# stopping at the first failure.  Usage: scripts/lib_ab.sh [workloads] [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
WLS=${1:-syn100k}; shift
: > gpurun_out/lib_ab.log
for W in ${WLS//,/ }; do
  for L in msha--gnn_amd/lib/alt/*.so; do
    echo "== $W $(basename $L)" >> gpurun_out/lib_ab.log
    MSHA_GNN_LIB=$PWD/$L timeout -k 10 240 python -u bench.py --workload $W --steps 20 --warmup 5 \
      --no-cpu-baseline --no-link-score --no-r15 "$@" > gpurun_out/ab_one.log 2>&1 \
      || { echo "failed on $W $L"; tail -20 gpurun_out/ab_one.log; exit 1; }
    python scripts/bench_summary.py gpurun_out/ab_one.log >> gpurun_out/lib_ab.log
  done
done
cat gpurun_out/lib_ab.log
