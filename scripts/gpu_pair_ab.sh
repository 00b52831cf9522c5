#!/bin/bash
# Pair-scorer A/B (scripts/pair_ab.py): the default library, then each alternative
# library named in ALTS (msha--gnn_amd/lib/alt/<name>.so); scores compared bit for bit.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/pair_ab.py save gpurun_out/pair_0.pt > gpurun_out/pair_ab.log 2>&1 || { tail -20 gpurun_out/pair_ab.log; exit 1; }
for A in ${ALTS:-}; do
  MSHA_GNN_LIB=msha--gnn_amd/lib/alt/$A.so timeout -k 10 200 python -u scripts/pair_ab.py save gpurun_out/pair_$A.pt >> gpurun_out/pair_ab.log 2>&1 || { tail -20 gpurun_out/pair_ab.log; exit 1; }
  timeout -k 10 100 python -u scripts/pair_ab.py cmp gpurun_out/pair_0.pt gpurun_out/pair_$A.pt >> gpurun_out/pair_ab.log 2>&1
  rm -f gpurun_out/pair_$A.pt
done
rm -f gpurun_out/pair_*.pt
grep -v amdgpu.ids gpurun_out/pair_ab.log
