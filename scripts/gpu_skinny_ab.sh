#!/bin/bash
# Projection / weight-gradient A/B: GEMM parity tests on the default build, then
# scripts/gemm_ab.py over MSHA_PROJ versions and the alternative libraries named in ALTS
# (msha--gnn_amd/lib/alt/<name>.so).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "gemm or project or proj or pair or score" > gpurun_out/pytest_skinny.log 2>&1 \
  || { tail -40 gpurun_out/pytest_skinny.log; exit 1; }
tail -3 gpurun_out/pytest_skinny.log
: > gpurun_out/skinny_ab.log
for P in ${PROJS:-1}; do
  echo "proj=$P" >> gpurun_out/skinny_ab.log
  MSHA_PROJ=$P timeout -k 10 200 python -u scripts/gemm_ab.py >> gpurun_out/skinny_ab.log 2>&1 \
    || { tail -20 gpurun_out/skinny_ab.log; exit 2; }
done
for A in ${ALTS:-}; do
  echo "alt=$A" >> gpurun_out/skinny_ab.log
  MSHA_GNN_LIB=msha--gnn_amd/lib/alt/$A.so timeout -k 10 200 python -u scripts/gemm_ab.py \
    >> gpurun_out/skinny_ab.log 2>&1 || { tail -20 gpurun_out/skinny_ab.log; exit 2; }
done
grep -v amdgpu.ids gpurun_out/skinny_ab.log
