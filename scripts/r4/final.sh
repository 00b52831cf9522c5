#!/bin/bash
# Round-4 closing run: the whole GPU suite (one process), the default bench line (the
# driver's command), smoke(), and the C4 bf16 row-score A/B (MSHA_ROW_SCORES=1 vs default).
set -o pipefail
mkdir -p gpurun_out/r4f
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4f/gpu_suite.log 2>&1 || { tail -60 gpurun_out/r4f/gpu_suite.log; exit 1; }
tail -3 gpurun_out/r4f/gpu_suite.log
$T 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4f/smoke.log 2>&1 \
  || { tail -20 gpurun_out/r4f/smoke.log; exit 1; }
tail -1 gpurun_out/r4f/smoke.log
$T 600 python -u bench.py > gpurun_out/r4f/bench_line.json 2> gpurun_out/r4f/bench.err \
  || { tail -20 gpurun_out/r4f/bench.err; exit 1; }
python scripts/bench_brief.py gpurun_out/r4f/bench_line.json | head -40
for RS in 1 0; do
  MSHA_ROW_SCORES=$RS $T 300 python -u bench.py --workload syn100k --steps 20 --warmup 5 --no-cpu-baseline \
    --no-r15 --no-syn2m --no-bip1m --no-link-score --no-dropout-leg > gpurun_out/r4f/rs$RS.json 2> gpurun_out/r4f/rs$RS.err \
    || { tail -20 gpurun_out/r4f/rs$RS.err; exit 1; }
  echo "== MSHA_ROW_SCORES=$RS"; python scripts/bench_brief.py gpurun_out/r4f/rs$RS.json | grep -i "bf16\|head" | head -6
done
