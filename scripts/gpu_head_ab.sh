#!/bin/bash
# head_ab.py on the default library and the alternative builds named in ALTS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
: > gpurun_out/head_ab.log
for A in default ${ALTS:-}; do
  echo "lib=$A" >> gpurun_out/head_ab.log
  if [ "$A" = default ]; then L=""; else L="msha--gnn_amd/lib/alt/$A.so"; fi
  HEAD_AB_FWD_ONLY=1 MSHA_GNN_LIB=${L:-msha--gnn_amd/lib/libmsha_gnn.so} PYTHONPATH=scripts timeout -k 10 200 python -u scripts/head_ab.py >> gpurun_out/head_ab.log 2>&1 || { tail -20 gpurun_out/head_ab.log; exit 2; }
done
grep -v amdgpu.ids gpurun_out/head_ab.log
