#!/bin/bash
# Round-4 bipartite-kernel check on one GPU: the bip parity tests, then the bip1m and R15
# layer legs (fwd/bwd HIP-event rates in edge_kernels).  Output under gpurun_out/r4/.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bip.py "$@" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r4/bip_tests.log 2>&1 || { tail -40 gpurun_out/r4/bip_tests.log; exit 1; }
tail -3 gpurun_out/r4/bip_tests.log
timeout -k 10 300 python -u bench.py --workload bip1m --steps 10 --warmup 3 --no-cpu-baseline \
  --no-r15 --no-dropout-leg > gpurun_out/r4/bip1m.json 2> gpurun_out/r4/bip1m.err || { tail -20 gpurun_out/r4/bip1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload r15 --steps 20 --warmup 5 --no-cpu-baseline \
  --no-r15 > gpurun_out/r4/r15.json 2> gpurun_out/r4/r15.err || { tail -20 gpurun_out/r4/r15.err; exit 1; }
python scripts/bench_brief.py gpurun_out/r4/bip1m.json && python scripts/bench_brief.py gpurun_out/r4/r15.json
