#!/bin/bash
# round 6: per-wave timelines of the MFMA bipartite kernels (scripts/bip_timeline.py) on
# the diagnostic library: bip1m bf16, bip1m fp32 (MFMA backward forced), R15 fp32 (MFMA
# kernels forced below their row cut) -> gpurun_out/r6_tl${TAG}/
set -o pipefail
O=gpurun_out/r6_tl${TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
export MSHA_GNN_LIB=msha--gnn_amd/lib/libmsha_gnn_timeline.so
T="timeout -k 10 240"
$T python -u scripts/bip_timeline.py $O bip1m bf16 > $O/bip1m_bf16.log 2>&1 || { tail -20 $O/bip1m_bf16.log; exit 1; }
MSHA_BIP3_BWD32=1 $T python -u scripts/bip_timeline.py $O bip1m f32 > $O/bip1m_f32.log 2>&1 || { tail -20 $O/bip1m_f32.log; exit 1; }
MSHA_BIP3_BWD32=1 MSHA_BIP2_BWD_MIN_ROWS=0 $T python -u scripts/bip_timeline.py $O r15 f32 > $O/r15_f32.log 2>&1 || { tail -20 $O/r15_f32.log; exit 1; }
echo TL_DONE
