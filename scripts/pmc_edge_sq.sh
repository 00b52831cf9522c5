#!/bin/bash
# SQ counter passes over the headline bench's edge kernels (fp32 + bf16 legs).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmcsq_${1:-a}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-link-score --no-r15"
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "edge_attn_fwd|csc_agg|bwd_rows" -f csv -d "$OUT/pmc$i" -o run -- python3 $B > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/pmc$i.log"; }
done
echo done
