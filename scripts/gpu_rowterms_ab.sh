#!/bin/bash
# Row-term (uc, qc) fused backward: parity tests, then syn2m with and without row terms.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  ${RT_TESTS:+-k "$RT_TESTS"} > gpurun_out/rt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rt_tests.log; [ $rc -eq 0 ] || exit $rc
B="bench.py --workload syn2m --steps 5 --warmup 2 --no-cpu-baseline --no-link-score --no-r15 --no-dropout-leg"
timeout -k 10 300 python -u $B > gpurun_out/rt_on.json 2> gpurun_out/rt_on.err || exit 3
MSHA_ROWTERMS=0 timeout -k 10 300 python -u $B > gpurun_out/rt_off.json 2> gpurun_out/rt_off.err || exit 4
python - <<'PY'
import json
for tag in ("on", "off"):
    d = json.loads(open(f"gpurun_out/rt_{tag}.json").read().strip().splitlines()[-1])
    print(tag, "fp32 ms/step", round(d["ms_per_step"], 3), [(k["kernel"][5:], round(k["avg_us"]), round(k["frac"], 3)) for k in d["edge_kernels"]])
    b = d.get("bf16") or {}
    if b:
        print(tag, "bf16 ms/step", round(b["ms_per_step"], 3), [(k["kernel"][5:], round(k["avg_us"]), round(k["frac"], 3)) for k in b["edge_kernels"]])
PY
