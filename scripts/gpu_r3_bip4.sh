#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_bip4${1:-}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bip.py tests/test_gpu_parity_full.py tests/test_gpu_ours.py > "$OUT/t.log" 2>&1
rc=$?; tail -2 "$OUT/t.log"; grep -E "^FAILED|Mismatch|Max abs" "$OUT/t.log" | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline --no-dropout-leg > "$OUT/b.json" 2> "$OUT/b.err"
brc=$?; python3 scripts/bench_brief.py "$OUT/b.json" 2>&1 | head -14; exit $brc
