#!/bin/bash
# the default bench line (the driver's command) and smoke() at HEAD
set -o pipefail
mkdir -p gpurun_out/r4f
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4f/smoke2.log 2>&1 \
  || { tail -20 gpurun_out/r4f/smoke2.log; exit 1; }
tail -1 gpurun_out/r4f/smoke2.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4f/bench_final.json 2> gpurun_out/r4f/bench_final.err \
  || { tail -20 gpurun_out/r4f/bench_final.err; exit 1; }
wc -l gpurun_out/r4f/bench_final.json
python scripts/bench_brief.py gpurun_out/r4f/bench_final.json
