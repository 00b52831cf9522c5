#!/bin/bash
# rocprofv3 kernel stats of the configs[1] / configs[2] train-step legs at HEAD: Ours 2015
# fp32, ablation3 2015 fp32, Ours 2015 bf16 -> gpurun_out/r5_step_{ours32,abl32,ours16}/
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for spec in "ours32 Ours float32" "abl32 ablation3 float32" "ours16 Ours bfloat16"; do
  set -- $spec
  O="$R/gpurun_out/r5_step_$1"
  mkdir -p "$O"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- \
    python3 "$R/scripts/train_step_only.py" $2 2015 $3 > "$O/trace.log" 2>&1 || { echo "$1 trace failed"; tail -5 "$O/trace.log"; exit 3; }
  timeout -k 10 300 python3 "$R/scripts/train_step_only.py" $2 2015 $3 > "$O/plain.json" 2>&1 || { echo "$1 plain failed"; exit 3; }
  echo "$1: $(tail -1 $O/plain.json | cut -c1-200)"
done
