#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
: > gpurun_out/proj_scan.log
for P in ${PROJS:-1 3}; do
  MSHA_PROJ=$P PYTHONPATH=scripts timeout -k 10 200 python -u scripts/proj_scan.py >> gpurun_out/proj_scan.log 2>&1 \
    || { tail -20 gpurun_out/proj_scan.log; exit 2; }
done
grep -v amdgpu.ids gpurun_out/proj_scan.log
