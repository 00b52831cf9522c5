#!/bin/bash
# configs[1] step state: R15 bench leg (graphed steps + train.py-literal), kernel trace of
# the Ours 2015 fp32 graphed step.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --workload r15 --steps 20 --warmup 5 --no-cpu-baseline --no-dropout-leg \
  > gpurun_out/r4/r15.json 2> gpurun_out/r4/r15.err || { tail -20 gpurun_out/r4/r15.err; exit 1; }
python scripts/bench_brief.py gpurun_out/r4/r15.json
NROWS=30 bash scripts/trace_train_step.sh r4_ours32 Ours 2015 float32
