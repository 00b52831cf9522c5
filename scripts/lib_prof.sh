#!/bin/bash
# Per-kernel averages (rocprofv3 --kernel-trace --stats) of the headline bench legs for
# every alternative library in msha--gnn_amd/lib/alt/ (one traced process per library).
# Usage: scripts/lib_prof.sh [workload] [kernel regex]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
WL=${1:-syn100k}; RX=${2:-proj|wgrad|gemm|edge_attn|bwd_|colsum}; EXTRA=${3:-}
mkdir -p "$R/gpurun_out"; : > "$R/gpurun_out/lib_prof.log"
cd /tmp && export TMPDIR=/tmp
for L in "$R"/msha--gnn_amd/lib/alt/*.so; do
  N=$(basename $L .so); OUT="$R/gpurun_out/libprof_$N"
  MSHA_GNN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- \
    python3 "$R/bench.py" --workload $WL --steps 20 --warmup 5 --no-cpu-baseline \
    --no-r15 $EXTRA > "$OUT.log" 2>&1 || { echo "failed on $N"; tail -5 "$OUT.log"; exit 3; }
  echo "== $N" >> "$R/gpurun_out/lib_prof.log"
  python3 - "$OUT/run_kernel_stats.csv" "$RX" >> "$R/gpurun_out/lib_prof.log" <<'PY'
import csv, re, sys
rx = re.compile(sys.argv[2])
for r in csv.DictReader(open(sys.argv[1])):
    if rx.search(r["Name"]):
        print(f'  {float(r["AverageNs"]) / 1e3:8.1f} us x{r["Calls"]:>4}  {r["Name"][:90]}')
PY
done
cat "$R/gpurun_out/lib_prof.log"
