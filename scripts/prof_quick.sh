#!/bin/bash
# rocprofv3 kernel trace + stats of one bench configuration.
# Usage: scripts/prof_quick.sh <tag> "<ENV=...>" "<bench args>"
TAG=$1; ENVS=$2; BARGS=$3
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pq_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export $ENVS
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $BARGS > "$OUT/bench.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/bench.log"; exit 3; }
python3 - "$OUT" <<'PY'
import csv, sys
out = sys.argv[1]
rows = list(csv.DictReader(open(f"{out}/trace/run_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e3:10.1f} us {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:110]}')
PY
