#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_h"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_optim.py tests/test_gpu_modules.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; grep -E "FAILED|Error" "$OUT/pytest.log" | head; [ $rc -ne 0 ] && exit $rc
A="--workload r15 --steps 10 --warmup 3 --no-cpu-baseline --no-link-score --no-bf16 --no-dropout-leg"
scripts/prof_quick.sh adam_msha4 "MSHA_ADAM=msha" "$A"
python3 scripts/bench_brief.py gpurun_out/pq_adam_msha4/bench.log | grep train_step
