#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
A="--workload r15 --steps 10 --warmup 3 --no-cpu-baseline --no-link-score --no-bf16 --no-dropout-leg"
scripts/prof_quick.sh adam_msha "MSHA_ADAM=msha" "$A" && scripts/prof_quick.sh adam_torch "MSHA_ADAM=torch" "$A"
