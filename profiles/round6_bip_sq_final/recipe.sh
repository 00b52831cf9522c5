#!/bin/bash
# round 6: SQ counter passes (separate --pmc runs) and the FETCH/WRITE traffic pass over the
# bip1m leg's MFMA bipartite kernels (edge_bip3.hip), fp32 (BF16=1: bf16 only)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$R/gpurun_out/pmcbip3_${1:-a}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload bip1m --steps 3 --warmup 1 --no-cpu-baseline --no-dropout-leg --no-r15"
[ -z "$BF16" ] && B="$B --no-bf16"
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" "FETCH_SIZE" "WRITE_SIZE"; do
  # (one pass per TCC counter: FETCH_SIZE takes 3 of the 4 TCC slots, WRITE_SIZE 2)
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "bip3_(fwd|bwd)" -f csv -d "$OUT/pmc$i" -o run -- python3 $B > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/pmc$i.log"; exit 3; }
done
python3 - "$OUT" <<'PY' | tee "$OUT/sq_counters.txt"
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:26s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
