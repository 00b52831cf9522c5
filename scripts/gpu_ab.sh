#!/bin/bash
# A/B of forward-kernel builds (scripts/fwd_ab.py) on the GPU box; each build is a
# separate process under its own time limit, stopping at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
V='[{"MSHA_FWD_BAT": "0"}, {"MSHA_FWD_BAT": "1"}]'
: > gpurun_out/fwd_ab.log
for L in "" msha--gnn_amd/lib/alt/*.so; do
  if [ -n "$L" ]; then export MSHA_GNN_LIB=$PWD/$L; fi
  timeout -k 10 300 python -u scripts/fwd_ab.py --variants "$V" "$@" >> gpurun_out/fwd_ab.log 2>&1 || { echo "failed on $L"; tail -20 gpurun_out/fwd_ab.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/fwd_ab.log
