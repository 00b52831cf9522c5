#!/bin/bash
# Column-pass A/B: edge-kernel GPU tests on the default build, then syn2m (true HBM) and
# the headline syn100k on the default library and on each library named in ALTS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "edge or fused or rowterms or parity_full or modules or ours" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for W in syn2m syn100k; do
  B="bench.py --workload $W --steps 10 --warmup 3 --no-cpu-baseline --no-link-score --no-r15 --no-dropout-leg"
  for A in default ${ALTS:-}; do
    O=gpurun_out/ab_${W}_${A}
    if [ "$A" = default ]; then
      timeout -k 10 300 python -u $B > $O.json 2> $O.err || exit 3
    else
      MSHA_GNN_LIB=msha--gnn_amd/lib/alt/$A.so timeout -k 10 300 python -u $B > $O.json 2> $O.err || exit 3
    fi
    python - "$W" "$A" $O.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], "fp32 ms/step", round(d["ms_per_step"], 4), [(k["kernel"][5:], round(k["avg_us"], 1), round(k["frac"], 3)) for k in d["edge_kernels"]])
b = d.get("bf16") or {}
if b:
    print(sys.argv[1], sys.argv[2], "bf16 ms/step", round(b["ms_per_step"], 4), [(k["kernel"][5:], round(k["avg_us"], 1), round(k["frac"], 3)) for k in b["edge_kernels"]])
PY
  done
done
