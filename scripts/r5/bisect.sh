#!/bin/bash
# one pytest selection under several env settings; stops on anything but pass/fail
# Usage: SEL="tests/x.py::t" CASES="A=1 B=0|C=2|" bash scripts/r5/bisect.sh   (| separates cases)
O=gpurun_out/r5_bisect
mkdir -p $O
export PYTHONUNBUFFERED=1
IFS='|' read -ra CS <<< "$CASES"
i=0
for c in "${CS[@]}"; do
  i=$((i+1))
  env $c timeout -k 10 300 python -u -m pytest $SEL -m gpu -x -q --timeout 240 \
    --timeout-method thread -p no:cacheprovider > $O/case$i.log 2>&1
  rc=$?
  echo "== case $i [$c] rc=$rc: $(tail -1 $O/case$i.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
