#!/bin/bash
# Full GPU suite + smoke of the current build, then the 14-unit engine probe.
set -o pipefail
tag=${1:-r5e}
bash scripts/gpu_suite.sh $tag || exit 1
bash scripts/gpu_eng_ab.sh $tag/eng || exit 1
