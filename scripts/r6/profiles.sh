#!/bin/bash
# Round-6 evidence at HEAD, one workload per step (each rocprofv3 run under its own
# timeout; counters in separate --pmc passes): C4 headline (+ bf16, dropout and link
# legs), syn2m, bip1m (SQ passes: scripts/r6/pmc.sh).
# Usage: scripts/r6/profiles.sh [tag] [a|b]  -> gpurun_out/prof_r6<tag>_*
#   a: C4 + syn2m; b: bip1m + its SQ passes + the configs[1] step traces; c: bip1m alone
TAG=${1:-v1}; SET=${2:-a}
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
KRE="edge_attn|bwd_|proj_kernel|wgrad|colsum|pair_|inner|head_|bip|slab_reduce|gemm"
run() {  # name, bench args
  local OUT="$R/gpurun_out/prof_r6${TAG}_$1"; shift
  mkdir -p "$OUT"
  (cd "$R" && python3 -c "import bench; print(bench.kernel_source_id())") > "$OUT/source_id.txt" || return 2
  (cd "$R" && python3 -c "import bench, json; print(json.dumps(bench.kernel_source_files()))") > "$OUT/source_files.json" || return 2
  local B="$R/bench.py $*"
  (cd /tmp && TMPDIR=/tmp timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 $B) \
    > "$OUT/bench_trace.log" 2>&1 || { echo "$OUT trace failed"; tail -5 "$OUT/bench_trace.log"; return 3; }
  for C in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && TMPDIR=/tmp timeout -k 10 500 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -f csv -d "$OUT/pmc_$C" -o run -- python3 $B) \
      > "$OUT/bench_$C.log" 2>&1 || { echo "$OUT pmc $C failed"; tail -5 "$OUT/bench_$C.log"; return 3; }
  done
  echo "$OUT done"
}
# a progress line a minute (rocprofv3 writes its files only when a pass ends)
( while true; do date > "$R/gpurun_out/prof_r6${TAG}_heartbeat"; sleep 60; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$SET" = c ]; then  # bip1m alone (the R15 legs share its kernel names)
run bip1m --workload bip1m --steps 5 --warmup 2 --no-cpu-baseline --no-dropout-leg --no-r15 &&
echo ALL_DONE
elif [ "$SET" = a ]; then
run syn100k --workload syn100k --steps 10 --warmup 3 --no-cpu-baseline --no-r15 --no-syn2m --no-bip1m &&
run syn2m --workload syn2m --steps 3 --warmup 1 --no-cpu-baseline --no-link-score --no-r15 --no-bip1m --no-dropout-leg &&
echo ALL_DONE
else
run bip1m --workload bip1m --steps 5 --warmup 2 --no-cpu-baseline --no-dropout-leg --no-r15 &&
echo ALL_DONE
fi
