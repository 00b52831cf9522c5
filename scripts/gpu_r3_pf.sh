#!/bin/bash
# gather-layout forward with the next chunk's gathers prefetched: forward parity tests,
# then the C4 / syn2m bench legs.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_pf${1:-}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity_full.py tests/test_gpu_row_scores.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py tests/test_gpu_bf16.py > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; grep -E "FAILED|Error" "$OUT/tests.log" | head -20
[ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-link-score --no-r15 --no-bip1m > "$OUT/bench.json" 2> "$OUT/bench.err"
brc=$?; python3 scripts/bench_brief.py "$OUT/bench.json" 2>/dev/null | head -30; echo "bench rc=$brc"; exit $brc
