#!/bin/bash
# round 6: the headline leg alone under rocprofv3 (C4 fp32, no bf16 / dropout / link / other
# legs): the roofline kernel's rocprof average against the bench's HIP-event duration; then
# the driver's default bench command once more (bip1m traffic now attached)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O=$R/gpurun_out/r6_headline
mkdir -p $O
export PYTHONUNBUFFERED=1
(cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-link-score --no-r15 --no-bf16 \
  --no-syn2m --no-bip1m --no-dropout-leg --detail $O/headline_detail.json) > $O/headline.json 2> $O/headline.err \
  || { tail -20 $O/headline.err; exit 1; }
python -c "import json; d=json.loads(open('$O/headline.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'])"
timeout -k 10 600 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python scripts/bench_brief.py $O/bench_detail.json
