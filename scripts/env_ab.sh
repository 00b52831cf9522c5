#!/bin/bash
# A/B of environment switches on the headline bench legs (one process per variant,
# own time limit, stop at the first failure).
# Usage: scripts/env_ab.sh <workloads> "<VAR=a VAR2=b>" "<VAR=c>" ... [-- bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
WLS=$1; shift
VARS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done; shift
: > gpurun_out/env_ab.log
for W in ${WLS//,/ }; do
  for V in "${VARS[@]}"; do
    echo "== $W [$V]" >> gpurun_out/env_ab.log
    env $V timeout -k 10 240 python -u bench.py --workload $W --steps 20 --warmup 5 \
      --no-cpu-baseline --no-link-score --no-r15 "$@" > gpurun_out/ab_one.log 2>&1 \
      || { echo "failed on $W $V"; tail -20 gpurun_out/ab_one.log; exit 1; }
    python scripts/bench_summary.py gpurun_out/ab_one.log >> gpurun_out/env_ab.log
  done
done
cat gpurun_out/env_ab.log
