#!/bin/bash
# pair scorer A/B (line-major roll vs two-set), bip v3 SQ counters, train.py-literal breakdown.
set -o pipefail
mkdir -p gpurun_out/r4
bash scripts/r4/pair.sh || exit 1
timeout -k 10 300 python -u scripts/r4/trainpy_time.py --prof > gpurun_out/r4/trainpy_prof.log 2>&1 || { tail -30 gpurun_out/r4/trainpy_prof.log; exit 1; }
grep '^{' gpurun_out/r4/trainpy_prof.log
bash scripts/pmc_bip_sq.sh r4v3 > gpurun_out/r4/pmc_bip_v3.txt 2>&1 || { tail -5 gpurun_out/r4/pmc_bip_v3.txt; exit 1; }
grep -A18 "bip_fwd_kernel<2, 64, float, true, false\|bip_bwd_kernel<2, 64, float, true, false" gpurun_out/r4/pmc_bip_v3.txt | head -40
