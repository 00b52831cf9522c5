#!/bin/bash
# Round-3 evidence profiles, one bench workload per directory (kernel instances are shared
# across workloads, so each gets its own runs): a kernel trace + stats pass, then one PMC
# pass per counter (FETCH_SIZE, WRITE_SIZE: separate runs, MI355X_MICROARCH.md).
# Usage: scripts/gpu_r3_prof.sh <tag> <workload|link> [...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for W in "$@"; do
  OUT="$R/gpurun_out/prof_${TAG}_$W"; mkdir -p "$OUT"
  if [ "$W" = link ]; then
    B="$R/bench.py --workload syn100k --steps 4 --warmup 2 --no-cpu-baseline --no-r15 --no-syn2m --no-bip1m --no-dropout-leg"
    RX="pair_|score_|gather"
  else
    B="$R/bench.py --workload $W --steps 6 --warmup 2 --no-cpu-baseline --no-link-score --no-r15 --no-syn2m --no-bip1m --no-dropout-leg"
    RX="edge_attn|bwd_row|bwd_cols|csc_|bip_|proj_kernel|wgrad|head_colsum|segments|ours_|head_|adam"
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 $B > "$OUT/bench_trace.log" 2>&1 \
    || { echo "trace $W failed"; tail -20 "$OUT/bench_trace.log"; exit 2; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$RX" -f csv -d "$OUT/pmc_$C" -o run -- python3 $B > "$OUT/bench_$C.log" 2>&1 \
      || { echo "pmc $C $W failed"; tail -20 "$OUT/bench_$C.log"; exit 3; }
  done
  echo "profile $W done"
done
