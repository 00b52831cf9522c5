#!/bin/bash
# rocprofv3 kernel stats of bench.py's configs[1] train-step leg alone, once per env case.
# Usage: KIND=Ours YEAR=2015 DT=float32 CASES="A=1|A=0" bash scripts/r5/step_prof.sh
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out/r5_stepprof"
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
IFS='|' read -ra CS <<< "${CASES:-MSHA_X=1}"
i=0
for c in "${CS[@]}"; do
  i=$((i+1))
  export $c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/c$i" -o run -- \
    python3 "$R/scripts/train_step_only.py" ${KIND:-Ours} ${YEAR:-2015} ${DT:-float32} \
    > "$O/c$i.log" 2>&1 || { echo "case $i failed"; tail -20 "$O/c$i.log"; exit 3; }
  timeout -k 10 300 python3 "$R/scripts/train_step_only.py" ${KIND:-Ours} ${YEAR:-2015} ${DT:-float32} \
    > "$O/c$i.plain" 2>&1 || { echo "case $i plain failed"; tail -20 "$O/c$i.plain"; exit 3; }
  echo "== case $i [$c]: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d.get('ms_per_step'), d.get('ms'))" $O/c$i.plain)"
  python3 - "$O/c$i" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:32]:
    print(f'{float(r["AverageNs"])/1e3:9.2f} us x{int(r["Calls"]):5d}  {r["Name"][:100]}')
PY
  unset ${c%%=*}
done
