#!/bin/bash
# SQ counter passes (separate runs) over the skinny projection / weight-gradient kernels
# of the fp32 headline layer.  Usage: scripts/pmc_skinny.sh <tag>
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmcsk_${1:-a}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-link-score --no-r15 --eager $2"
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "proj_kernel|wgrad_kernel|edge_attn_fwd_bat|bwd_cols_eh" -f csv -d "$OUT/pmc$i" -o run -- python3 $B > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/pmc$i.log"; exit 3; }
done
python3 "$R/scripts/pmc_table.py" "$OUT"
