#!/bin/bash
# Kernel trace + FETCH_SIZE / WRITE_SIZE passes (separate runs) over the fp32 layer at a
# given workload.  Usage: scripts/pmc_syn2m.sh <tag> [workload]
TAG=${1:-a}; WL=${2:-syn2m}
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_${WL}_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-link-score --no-r15 --no-bf16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 $B > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/trace.log"; exit 3; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "edge_attn|bwd_|proj|wgrad|colsum" -f csv -d "$OUT/pmc_$C" -o run -- python3 $B > "$OUT/bench_$C.log" 2>&1 || { echo "pmc $C failed"; tail -5 "$OUT/bench_$C.log"; exit 3; }
done
echo done
