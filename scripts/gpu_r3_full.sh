#!/bin/bash
# Round-3 full check: the -m gpu suite, smoke(), then the default bench line.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_full${1:-}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; grep -E "FAILED|Error" "$OUT/pytest.log" | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 3; }
tail -2 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
brc=$?; tail -c 1500 "$OUT/bench.json"; echo "pytest rc=$rc bench rc=$brc"
exit $brc
