#!/bin/bash
# gather-layout forward A/B: the shipped library vs the knob variants (build.py VARIANTS),
# C4 / syn2m legs only; each variant's forward parity tests first.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r3_pfab${1:-}"; mkdir -p "$OUT"; cd "$R"
for V in "" wpe6; do
  L="$R/msha--gnn_amd/lib/libmsha_gnn${V:+_$V}.so"
  MSHA_GNN_LIB="$L" timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity_full.py tests/test_gpu_row_scores.py > "$OUT/tests_$V.log" 2>&1
  rc=$?; echo "[$V] $(tail -1 "$OUT/tests_$V.log")"
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/tests_$V.log" | head; exit $rc; }
  MSHA_GNN_LIB="$L" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-link-score --no-r15 --no-bip1m --no-dropout-leg > "$OUT/bench_$V.json" 2> "$OUT/bench_$V.err" || { echo "bench $V failed"; tail "$OUT/bench_$V.err"; exit 2; }
  echo "[$V]"; python3 scripts/bench_brief.py "$OUT/bench_$V.json" 2>/dev/null | grep -E "^[a-z]|edge_attention_fwd " | head -20
done
