#!/bin/bash
# rocprofv3 passes over the default bench: kernel trace + stats, then one PMC pass
# per counter for the dominant kernel (separate passes, as MI355X_MICROARCH.md asks).
# Usage: scripts/profile.sh <tag> [bench args...]
TAG=${1:-r1}; shift
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline $*"
(cd "$R" && python3 -c "import bench; print(bench.kernel_source_id())") > "$OUT/source_id.txt"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 $B > "$OUT/bench_trace.log" 2>&1 || { echo "trace pass failed"; tail -20 "$OUT/bench_trace.log"; exit 2; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-edge_attn_fwd}" -f csv -d "$OUT/pmc_$C" -o run -- python3 $B > "$OUT/bench_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$OUT/bench_$C.log"; exit 3; }
done
echo "profile $TAG done"; find "$OUT" -name "*.csv" | head -20
