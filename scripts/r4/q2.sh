#!/bin/bash
# bip quick loop (bipq.sh), then the train.py-literal host-phase breakdown.
set -o pipefail
mkdir -p gpurun_out/r4
bash scripts/r4/bipq.sh || exit 1
timeout -k 10 300 python -u scripts/r4/trainpy_time.py --prof > gpurun_out/r4/trainpy_prof.log 2>&1 || { tail -30 gpurun_out/r4/trainpy_prof.log; exit 1; }
grep '^{' gpurun_out/r4/trainpy_prof.log
