#!/bin/bash
# Skinny GEMM A/B: scripts/gemm_ab.py on the default library and on each alternative
# library named in ALTS (msha--gnn_amd/lib/alt/<name>.so), outputs compared bit for bit.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
GEMM_AB_SAVE=gpurun_out/g_0.pt timeout -k 10 200 python -u scripts/gemm_ab.py > gpurun_out/gemm_bits_ab.log 2>&1 || { tail -20 gpurun_out/gemm_bits_ab.log; exit 1; }
for A in ${ALTS:-}; do
  echo "alt=$A" >> gpurun_out/gemm_bits_ab.log
  MSHA_GNN_LIB=msha--gnn_amd/lib/alt/$A.so GEMM_AB_SAVE=gpurun_out/g_$A.pt timeout -k 10 200 python -u scripts/gemm_ab.py >> gpurun_out/gemm_bits_ab.log 2>&1 || { tail -20 gpurun_out/gemm_bits_ab.log; exit 1; }
  timeout -k 10 100 python -u scripts/gemm_ab.py cmp gpurun_out/g_0.pt gpurun_out/g_$A.pt >> gpurun_out/gemm_bits_ab.log 2>&1
done
rm -f gpurun_out/g_*.pt.*
grep -v amdgpu.ids gpurun_out/gemm_bits_ab.log
