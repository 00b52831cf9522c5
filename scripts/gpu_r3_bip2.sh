#!/bin/bash
# bip kernels: their tests and the tests that route through them, then the bip1m and
# r15 legs of the bench.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_bip2${1:-}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bip.py tests/test_gpu_row_scores.py tests/test_gpu_ours.py tests/test_gpu_modules.py > "$OUT/bip.log" 2>&1
rc=$?; tail -3 "$OUT/bip.log"; grep -E "FAILED|Error|assert" "$OUT/bip.log" | head -20
[ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline --no-dropout-leg > "$OUT/bench_bip1m.json" 2> "$OUT/bench_bip1m.err"
brc=$?; python3 scripts/bench_brief.py "$OUT/bench_bip1m.json" 2>&1 | head -12; [ $brc -ne 0 ] && { tail -5 "$OUT/bench_bip1m.err"; exit $brc; }
timeout -k 10 300 python -u bench.py --workload r15 --steps 10 --warmup 3 --no-cpu-baseline --no-dropout-leg > "$OUT/bench_r15.json" 2> "$OUT/bench_r15.err"
brc=$?; python3 scripts/bench_brief.py "$OUT/bench_r15.json" 2>&1 | head -30
exit $brc
