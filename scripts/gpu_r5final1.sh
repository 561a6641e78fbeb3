#!/bin/bash
# Round-5 build check: full GPU suite + smoke + world-2 rehearsal, then the engine PMC traffic
# of the bench's grid path (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
tag=${1:-r5final1}
bash scripts/gpu_suite.sh $tag || exit 1
JOINED=1 GRID=1 bash scripts/gpu_pmc_engine.sh $tag/pmc || exit 1
