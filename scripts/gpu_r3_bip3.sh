#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_bip3${1:-}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bip.py tests/test_gpu_parity_full.py tests/test_gpu_ours.py tests/test_gpu_modules.py tests/test_gpu_graph.py > "$OUT/t.log" 2>&1
rc=$?; tail -3 "$OUT/t.log"; grep -E "^FAILED|Mismatch|Max abs" "$OUT/t.log" | head -20
exit $rc
