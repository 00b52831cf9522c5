#!/bin/bash
# bip kernels: their tests first (stop on failure), then the whole -m gpu suite, smoke
# and the default bench line.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_bip${1:-}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bip.py > "$OUT/bip.log" 2>&1
rc=$?; tail -5 "$OUT/bip.log"; grep -E "FAILED|Error|assert" "$OUT/bip.log" | head -20
[ $rc -ne 0 ] && { echo "bip tests rc=$rc"; exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; grep -E "FAILED|Error" "$OUT/pytest.log" | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 3; }
tail -1 "$OUT/smoke.log"
T0=$SECONDS; timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
brc=$?; echo "bench wall $((SECONDS - T0)) s"; python3 scripts/bench_brief.py "$OUT/bench.json" 2>/dev/null | head -40; echo "pytest rc=$rc bench rc=$brc"
exit $brc
