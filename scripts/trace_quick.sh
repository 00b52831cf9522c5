#!/bin/bash
# Kernel-trace stats of a short bench run (per-kernel average durations).
# Usage: scripts/trace_quick.sh <tag> [bench args]
TAG=${1:-q}; shift
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/trace_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-link-score --no-r15 "$@" > "$OUT/bench.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/bench.log"; exit 3; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f'{float(r["AverageNs"])/1e3:9.1f} us x{int(r["Calls"]):4d}  {r["Name"][:110]}')
PY
