#!/bin/bash
# GEMM parity tests, then the skinny-vs-tiled A/B (scripts/gemm_ab.py); stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or project" > gpurun_out/pytest_gemm.log 2>&1 || { tail -40 gpurun_out/pytest_gemm.log; exit 1; }
tail -3 gpurun_out/pytest_gemm.log
: > gpurun_out/gemm_ab.log
for S in 0 1; do
  MSHA_SKINNY=$S timeout -k 10 200 python -u scripts/gemm_ab.py >> gpurun_out/gemm_ab.log 2>&1 || { tail -20 gpurun_out/gemm_ab.log; exit 2; }
done
grep -v amdgpu.ids gpurun_out/gemm_ab.log
