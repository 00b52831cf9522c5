#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over the headline bench for every edge kernel and GEMM
# (separate --pmc runs).  Usage: scripts/pmc_edges.sh <tag> [bench args]
TAG=${1:-e}; shift
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-link-score --no-r15 --no-bf16 $*"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "edge_attn|csc_|gemm|colsum|slab" -f csv -d "$OUT/pmc_$C" -o run -- python3 $B > "$OUT/bench_$C.log" 2>&1 || { echo "pmc $C failed"; tail -5 "$OUT/bench_$C.log"; exit 3; }
done
echo done
