#!/bin/bash
# configs[1] train step (Ours / ablation3, 2015) for every alternative library build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
: > gpurun_out/lib_step_ab.log
for L in msha--gnn_amd/lib/alt/*.so; do
  for M in Ours ablation3; do
    MSHA_GNN_LIB=$PWD/$L timeout -k 10 240 python -u scripts/train_step_only.py $M 2015 > gpurun_out/step_one.log 2>&1 \
      || { echo "failed on $L"; tail -20 gpurun_out/step_one.log; exit 1; }
    echo "$(basename $L) $M $(grep '^{' gpurun_out/step_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step_hip_graph'], 3), round(d['loss_hip_graph'], 4))")" >> gpurun_out/lib_step_ab.log
  done
done
cat gpurun_out/lib_step_ab.log
