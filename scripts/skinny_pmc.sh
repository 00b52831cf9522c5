#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each) over scripts/gemm_ab.py (skinny kernels).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/gemm_pmc_${1:-sk}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export GEMM_AB_REPS=5
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 "$R/scripts/gemm_ab.py" > "$OUT/trace.log" 2>&1 || exit 2
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 100 rocprofv3 --pmc $C --kernel-include-regex "proj_kernel|wgrad|dx_kernel" -f csv -d "$OUT/pmc$i" -o run -- python3 "$R/scripts/gemm_ab.py" > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc$i.log"; exit 3; }
done
python3 "$R/scripts/pmc_table.py" "$OUT"
