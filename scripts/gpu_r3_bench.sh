#!/bin/bash
# The default bench line (what the driver runs), timed.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_bench${1:-}"; mkdir -p "$OUT"; cd "$R"
T0=$SECONDS; timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
brc=$?; echo "bench wall $((SECONDS - T0)) s rc=$brc"; python3 scripts/bench_brief.py "$OUT/bench.json" 2>/dev/null | head -40
exit $brc
