#!/bin/bash
# round 6: SQ counter passes and the FETCH / WRITE traffic passes (one --pmc run each) plus a
# kernel-trace --stats pass over one bench.py workload, restricted to a kernel-name regex.
#   usage: pmc.sh <tag> <workload> <kernel regex> [extra bench.py args]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$R/gpurun_out/pmc_$1"
WL="$2"; RX="$3"; shift 3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-dropout-leg --no-r15 $*"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 $B > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -3 "$OUT/trace.log"; exit 3; }
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$RX" -f csv -d "$OUT/pmc$i" -o run -- python3 $B > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/pmc$i.log"; exit 3; }
done
python3 - "$OUT" "$RX" <<'PY' | tee "$OUT/counters.txt"
import csv, glob, sys, collections, re
out, rx = sys.argv[1], re.compile(sys.argv[2])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(out + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if rx.search(r["Name"]):
            print(f"stats {r['Name'][:90]}  calls {r['Calls']}  avg {float(r['AverageNs'])/1e3:.1f} us")
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:26s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
