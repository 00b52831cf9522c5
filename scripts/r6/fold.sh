#!/bin/bash
# round 6: launch folds of the configs[1] step (loss row flags -> head backward; bipartite
# reduce inside the Ours prep / finish launches): parity subsets, then the Ours 2015 fp32
# step with the folds off / on, then the bip1m knob A/B (ALTS)
set -o pipefail
O=gpurun_out/r6_fold${TAG}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_head.py tests/test_gpu_ours.py tests/test_gpu_bip.py tests/test_gpu_graph.py} -m gpu -p no:cacheprovider > $O/tests.log 2>&1 \
  || { grep -E "^E |FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for spec in "off:MSHA_BIP_DEFER=0 MSHA_NLL_FLAGS=0" "on:MSHA_BIP_DEFER=1 MSHA_NLL_FLAGS=1" "off2:MSHA_BIP_DEFER=0 MSHA_NLL_FLAGS=0" "on2:MSHA_BIP_DEFER=1 MSHA_NLL_FLAGS=1"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python -u scripts/train_step_only.py ${KIND:-Ours} 2015 float32 > $O/step_$name.json 2> $O/step_$name.err || { tail -5 $O/step_$name.err; exit 1; }
  echo "$name: $(python -c "import json,sys; d=json.loads(open('$O/step_$name.json').read().strip().splitlines()[-1]); print(d.get('ms_per_step'))")"
done
[ -n "$ALTS" ] && TAG=$TAG bash scripts/r6/bip_alt.sh
exit 0
