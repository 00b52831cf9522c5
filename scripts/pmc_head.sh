#!/bin/bash
# SQ counter passes (separate runs) over the model-head kernels of the configs[1] train
# step (scripts/train_step_only.py).  Usage: scripts/pmc_head.sh <tag> [model]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmchead_${1:-a}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "head_" -f csv -d "$OUT/pmc$i" -o run -- python3 "$R/scripts/train_step_only.py" ${2:-Ours} 2015 > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/pmc$i.log"; exit 3; }
done
python3 "$R/scripts/pmc_table.py" "$OUT"
