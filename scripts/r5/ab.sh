#!/bin/bash
# A/B of one env knob on a bench workload: runs bench.py once per value, prints the brief.
# Usage: KNOB=MSHA_BIP2 VALS="1 0" WL=r15 ARGS="..." bash scripts/r5/ab.sh
set -o pipefail
O=gpurun_out/r5_ab_${KNOB}_${WL}
mkdir -p $O
export PYTHONUNBUFFERED=1
i=0
for v in $VALS; do
  i=$((i+1))  # (file names by index: values may hold paths)
  env $KNOB=$v timeout -k 10 400 python -u bench.py --workload $WL --no-cpu-baseline $ARGS \
    --detail $O/d_$i.json > $O/l_$i.line 2> $O/e_$i.err || { tail -20 $O/e_$i.err; exit 1; }
  echo "== $KNOB=$v"
  python scripts/bench_brief.py $O/d_$i.json | grep -E "${GREP:-.}"
done
