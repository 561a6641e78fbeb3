#!/bin/bash
# Round-5 check of the lane-uniform EST 4 pass: full GPU suite + smoke, then the 14-unit
# engine probe (kernel stats: k_rankB on the full-set pass, k_full_corr).
set -o pipefail
tag=${1:-r5b}
bash scripts/gpu_suite.sh $tag || exit 1
bash scripts/gpu_eng_ab.sh $tag/eng || exit 1
