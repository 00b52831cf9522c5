#!/bin/bash
# SQ counter passes (separate runs) over the syn2m edge kernels, fp32 and bf16.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmcsq_${1:-a}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload syn2m --steps 2 --warmup 1 --no-cpu-baseline --no-link-score --no-r15 --no-dropout-leg --eager"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES" "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-include-regex "edge_attn_fwd_gl|bwd_cols_eh|bwd_row_stats" -f csv -d "$OUT/pmc$i" -o run -- python3 $B > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc$i.log"; exit 3; }
done
python3 "$R/scripts/pmc_table.py" "$OUT"
