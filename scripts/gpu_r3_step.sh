#!/bin/bash
# configs[1] / configs[2] Ours 2015 train step alone under rocprofv3 (kernel trace + stats).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
NROWS=30 scripts/trace_train_step.sh r3_ours32 Ours 2015 float32 > gpurun_out/step_ours32.txt 2>&1 && \
NROWS=30 scripts/trace_train_step.sh r3_ours16 Ours 2015 bfloat16 > gpurun_out/step_ours16.txt 2>&1 && \
NROWS=30 scripts/trace_train_step.sh r3_abl32 ablation3 2015 float32 > gpurun_out/step_abl32.txt 2>&1
rc=$?; head -25 gpurun_out/step_ours32.txt; exit $rc
