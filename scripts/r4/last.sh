#!/bin/bash
# last closing run at HEAD: the whole GPU suite, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out/r4f
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4f/gpu_suite_last.log 2>&1 || { tail -60 gpurun_out/r4f/gpu_suite_last.log; exit 1; }
tail -1 gpurun_out/r4f/gpu_suite_last.log
$T 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4f/smoke_last.log 2>&1 \
  || { tail -20 gpurun_out/r4f/smoke_last.log; exit 1; }
tail -1 gpurun_out/r4f/smoke_last.log
$T 600 python -u bench.py > gpurun_out/r4f/bench_last.json 2> gpurun_out/r4f/bench_last.err \
  || { tail -20 gpurun_out/r4f/bench_last.err; exit 1; }
wc -l < gpurun_out/r4f/bench_last.json
python scripts/bench_brief.py gpurun_out/r4f/bench_last.json > gpurun_out/r4f/bench_last_brief.txt
grep -E "head|train_step|literal|bip1m|syn2m|bf16 " gpurun_out/r4f/bench_last_brief.txt
