#!/bin/bash
# Kernel trace of bench.py's configs[1] train-step leg alone (scripts/train_step_only.py):
# per-kernel totals over the run.  Usage: scripts/trace_train_step.sh <tag> [model] [year]
TAG=${1:-t}; MODEL=${2:-Ours}; YEAR=${3:-2015}; DT=${4:-float32}
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/trace_step_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- python3 "$R/scripts/train_step_only.py" $MODEL $YEAR $DT > "$OUT/run.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/run.log"; exit 3; }
tail -1 "$OUT/run.log"
python3 - "$OUT" ${NROWS:-40} <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} launches")
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f'{float(r["TotalDurationNs"])/1e3:9.1f} us tot {float(r["AverageNs"])/1e3:7.1f} avg x{int(r["Calls"]):5d}  {r["Name"][:100]}')
PY
