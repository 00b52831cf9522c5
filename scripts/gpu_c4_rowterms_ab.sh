#!/bin/bash
# syn2m rocprofv3 trace + PMC with the row terms (library default there), then the C4
# headline with the row terms forced on vs the default (off below 192 MB of de).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash scripts/pmc_syn2m.sh rt syn2m > gpurun_out/pmc_syn2m_rt.txt 2>&1 || { tail -5 gpurun_out/pmc_syn2m_rt.txt; exit 2; }
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-link-score --no-r15 --no-dropout-leg"
timeout -k 10 300 python -u $B > gpurun_out/c4_def.json 2> gpurun_out/c4_def.err || exit 3
MSHA_ROWTERMS=1 timeout -k 10 300 python -u $B > gpurun_out/c4_rt.json 2> gpurun_out/c4_rt.err || exit 4
python - <<'PY'
import json
for tag in ("def", "rt"):
    d = json.loads(open(f"gpurun_out/c4_{tag}.json").read().strip().splitlines()[-1])
    print(tag, "fp32 ms/step", round(d["ms_per_step"], 4), [(k["kernel"][5:], round(k["avg_us"], 1)) for k in d["edge_kernels"]])
    b = d["bf16"]
    print(tag, "bf16 ms/step", round(b["ms_per_step"], 4), [(k["kernel"][5:], round(k["avg_us"], 1)) for k in b["edge_kernels"]])
PY
