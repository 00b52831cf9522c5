#!/bin/bash
# skinny W-fill batching + wgrad load depth A/B: GEMM parity tests, gemm_ab over the
# default build and the WG_PD alternates, the C4 timeline.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/r3_j
ALTS="head" bash scripts/gpu_skinny_ab.sh || exit 3
MSHA_GNN_LIB="$R/msha--gnn_amd/lib/libmsha_gnn_timeline.so" timeout -k 10 300 python -u scripts/skinny_timeline.py "$R/gpurun_out/timeline_c4c" > gpurun_out/timeline_c4c.log 2>&1 \
  || { tail -30 gpurun_out/timeline_c4c.log; exit 4; }
python3 -c "
import json; d=json.load(open('gpurun_out/timeline_c4c/summary.json'))
for k,v in d.items(): print(k, {a: b for a, b in v.items() if a in ('window_us','wfill_us','rows_loop_cycles','block_sum_cycles','store_cycles','launch_without_live_wave','mfma_share_of_wave_cycles')})"
