#!/bin/bash
# A/B of library env knobs on the same box: one short bench per setting.
# Usage: scripts/gpu_env_ab.sh <tag> "<bench args>" "ENV1=a ENV2=b" "ENV1=c" ...
TAG=$1; shift; BARGS=$1; shift
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/ab_$TAG"; mkdir -p "$OUT"; cd "$R"
i=0
for SET in "$@"; do
  i=$((i+1))
  echo "== $SET" | tee -a "$OUT/summary.txt"
  env $SET timeout -k 10 300 python -u bench.py $BARGS > "$OUT/run$i.log" 2>&1 || { echo "run $i failed"; tail -20 "$OUT/run$i.log"; exit 3; }
  python3 scripts/bench_brief.py "$OUT/run$i.log" | tee -a "$OUT/summary.txt"
done
