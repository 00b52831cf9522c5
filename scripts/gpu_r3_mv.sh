#!/bin/bash
# MSHA_BIP_MV A/B: bip tests under the variant, then bip1m legs with and without it.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_mv${1:-}"; mkdir -p "$OUT"; cd "$R"
MSHA_BIP_MV=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bip.py tests/test_gpu_ours.py > "$OUT/t.log" 2>&1
rc=$?; tail -2 "$OUT/t.log"; grep -E "^FAILED|Mismatch|Max abs" "$OUT/t.log" | head -10
[ $rc -ne 0 ] && exit $rc
for MV in 1 0; do
  MSHA_BIP_MV=$MV timeout -k 10 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline --no-dropout-leg > "$OUT/b$MV.json" 2> "$OUT/b$MV.err" || exit 4
  echo "MV=$MV"; python3 scripts/bench_brief.py "$OUT/b$MV.json" 2>&1 | head -7
done
