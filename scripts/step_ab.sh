#!/bin/bash
# configs[1] train-step leg (scripts/train_step_only.py) under environment variants.
# Usage: scripts/step_ab.sh "<VAR=a>" "<VAR=b>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export PYTHONDONTWRITEBYTECODE=1
: > gpurun_out/step_ab.log
for V in "$@"; do
  for M in Ours ablation3; do
    echo "== $M [$V]" >> gpurun_out/step_ab.log
    env $V timeout -k 10 240 python -u scripts/train_step_only.py $M 2015 > gpurun_out/step_one.log 2>&1 \
      || { echo "failed on $V"; tail -20 gpurun_out/step_one.log; exit 1; }
    grep '^{' gpurun_out/step_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v, 3) if isinstance(v, float) else v for k, v in d.items() if 'ms' in k or 'loss' in k})" >> gpurun_out/step_ab.log
  done
done
cat gpurun_out/step_ab.log
