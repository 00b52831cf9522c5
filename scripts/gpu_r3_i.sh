#!/bin/bash
# wgrad block-sum / reduce rework: skinny tests, the C4 timeline, and a C4 kernel trace.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/r3_i
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_bf16.py > gpurun_out/r3_i/pytest.log 2>&1 \
  || { tail -30 gpurun_out/r3_i/pytest.log; exit 3; }
tail -2 gpurun_out/r3_i/pytest.log
MSHA_GNN_LIB="$R/msha--gnn_amd/lib/libmsha_gnn_timeline.so" timeout -k 10 300 python -u scripts/skinny_timeline.py "$R/gpurun_out/timeline_c4b" > gpurun_out/timeline_c4b.log 2>&1 \
  || { tail -30 gpurun_out/timeline_c4b.log; exit 4; }
python3 -c "
import json; d=json.load(open('gpurun_out/timeline_c4b/summary.json'))
for k,v in d.items(): print(k, {a: b for a, b in v.items() if a in ('window_us','rows_loop_cycles','block_sum_cycles','store_cycles','launch_without_live_wave')})"
bash scripts/prof_quick.sh wg_c4 "MSHA_X=0" "--steps 30 --warmup 5" | grep -i "wgrad\|proj_kernel\|edge\|adam"
python3 scripts/bench_brief.py gpurun_out/pq_wg_c4/bench.log
