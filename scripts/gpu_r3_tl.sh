#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
MSHA_GNN_LIB="$R/msha--gnn_amd/lib/libmsha_gnn_timeline.so" timeout -k 10 300 python -u scripts/skinny_timeline.py "$R/gpurun_out/timeline_c4" > gpurun_out/timeline_c4.log 2>&1
rc=$?; tail -80 gpurun_out/timeline_c4.log; exit $rc
