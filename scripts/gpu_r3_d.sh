#!/bin/bash
# tests touching the forward + bip1m parity, then A/B of the forward variants
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_d"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity_full.py::test_bip1m_ourslayer3_core_every_row \
  tests/test_gpu_modules.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -5 "$OUT/pytest.log"; grep -E "FAILED|Error" "$OUT/pytest.log" | head; [ $rc -ne 0 ] && exit $rc
scripts/gpu_env_ab.sh d "--steps 10 --warmup 3 --no-cpu-baseline --no-link-score --no-dropout-leg" "MSHA_FWD_GL=1" "MSHA_FWD_GL=0 MSHA_ROW_SCORES=0"
