#!/bin/bash
# Round-4 close at HEAD: profiles (C4 / link / syn2m, bip1m alone + its SQ passes),
# summarised into profiles/round4_*_v2 on the box so the bench line's traffic comes from
# them, then the whole GPU suite, smoke() and the default bench line (scripts/r4/final.sh).
set -o pipefail
bash scripts/r4/profiles.sh v2 a && bash scripts/r4/profiles.sh v2 c || exit 1
for w in syn100k syn2m bip1m; do
  python scripts/summarize_profile.py gpurun_out/prof_r4v2_$w profiles/round4_${w}_v2 > /dev/null || exit 1
done
mkdir -p profiles/round4_link_v2 && cp profiles/round4_syn100k_v2/pmc_summary.json profiles/round4_link_v2/
bash scripts/r4/final.sh
