#!/bin/bash
# Round-3 check: new GPU tests (row scores, RCCL world-1 scorer), then a short bench.
# Usage: scripts/gpu_r3_check.sh <tag> [pytest selection...]
TAG=${1:-a}; shift
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_$TAG"
mkdir -p "$OUT"
cd "$R"
SEL=${*:-"tests/test_gpu_row_scores.py tests/test_gpu_sharded.py"}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $SEL > "$OUT/pytest.log" 2>&1
rc=$?
tail -30 "$OUT/pytest.log"
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-r15 > "$OUT/bench.log" 2>&1
rc=$?
tail -c 3000 "$OUT/bench.log"
exit $rc
