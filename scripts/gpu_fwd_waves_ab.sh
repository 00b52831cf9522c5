#!/bin/bash
# Batched forward with next-row prefetch: R15 forward time vs the grid cap (waves walking
# rows), and C4 with the default grid.  Prints the forward's HIP-event time per setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-link-score --no-dropout-leg --no-r15"
: > gpurun_out/fwd_waves.log
for W in ${WAVES:--1 4096 8192 16384}; do
  MSHA_FWD_WAVES=$W timeout -k 10 200 python -u $B --workload r15 > gpurun_out/fw_$W.json 2> gpurun_out/fw_$W.err || exit 3
  python - "$W" >> gpurun_out/fwd_waves.log <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/fw_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("r15 waves", sys.argv[1], "step", round(d["ms_per_step"], 4), [(k["kernel"][5:], round(k["avg_us"], 1)) for k in d["edge_kernels"]], "bf16", round(d["bf16"]["ms_per_step"], 4), [(k["kernel"][5:], round(k["avg_us"], 1)) for k in d["bf16"]["edge_kernels"]])
PY
done
timeout -k 10 200 python -u $B > gpurun_out/fw_c4.json 2> gpurun_out/fw_c4.err || exit 4
python - >> gpurun_out/fwd_waves.log <<'PY'
import json
d = json.loads(open("gpurun_out/fw_c4.json").read().strip().splitlines()[-1])
print("c4 step", round(d["ms_per_step"], 4), [(k["kernel"][5:], round(k["avg_us"], 1)) for k in d["edge_kernels"]], "bf16", round(d["bf16"]["ms_per_step"], 4), [(k["kernel"][5:], round(k["avg_us"], 1)) for k in d["bf16"]["edge_kernels"]])
PY
cat gpurun_out/fwd_waves.log
