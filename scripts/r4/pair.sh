#!/bin/bash
# fp32 pair scorer: parity (both kernels), A/B timing roll vs two-set, kernel trace.
set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "pair or link or score" > gpurun_out/r4/pair_tests.log 2>&1 || { tail -30 gpurun_out/r4/pair_tests.log; exit 1; }
tail -2 gpurun_out/r4/pair_tests.log
MSHA_PAIR_ROLL=2 $T 200 python -u scripts/pair_ab.py save gpurun_out/r4/pair_x3.pt > gpurun_out/r4/pair_ab.log 2>&1 &&
MSHA_PAIR_ROLL=1 $T 200 python -u scripts/pair_ab.py save gpurun_out/r4/pair_roll.pt >> gpurun_out/r4/pair_ab.log 2>&1 &&
MSHA_PAIR_ROLL=0 $T 200 python -u scripts/pair_ab.py save gpurun_out/r4/pair_two.pt >> gpurun_out/r4/pair_ab.log 2>&1 &&
python scripts/pair_ab.py cmp gpurun_out/r4/pair_x3.pt gpurun_out/r4/pair_two.pt >> gpurun_out/r4/pair_ab.log 2>&1 || { tail -30 gpurun_out/r4/pair_ab.log; exit 1; }
grep '^{' gpurun_out/r4/pair_ab.log
rm -f gpurun_out/r4/pair_*.pt
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/r4/pair_trace" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/pair_ab.py" save /tmp/p.pt > "$GRAFT_REPO_ROOT/gpurun_out/r4/pair_trace.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/r4/pair_trace.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/r4/pair_trace" -name "*kernel_stats.csv" -exec grep -i "pair" {} \;
