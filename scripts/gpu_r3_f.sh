#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_f"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bf16.py tests/test_gpu_optim.py tests/test_gpu_short_rows.py tests/test_gpu_row_scores.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity_full.py tests/test_gpu_ours.py tests/test_gpu_modules.py tests/test_gpu_graph.py tests/test_gpu_head.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; grep -E "FAILED|Error" "$OUT/pytest.log" | head; [ $rc -ne 0 ] && exit $rc
scripts/gpu_env_ab.sh f "--steps 10 --warmup 3 --no-cpu-baseline --no-link-score --no-dropout-leg" "MSHA_BWD_GL=1" "MSHA_BWD_GL=0 MSHA_ADAM=torch"
