#!/bin/bash
# Round 6 final build: PMC of the bench's engine path (grid), then the bench line + kernel stats,
# each step under its own time limit, stopping at the first failure
set -o pipefail
tag=${1:-r6final}
JOINED=1 GRID=1 bash scripts/gpu_pmc_engine.sh $tag/pmc || exit 1
# bench.py reads profiles/r6_pmc_engine_grid.json: the new build's counts go there first
cp gpurun_out/$tag/pmc/pmc_engine.json profiles/r6_pmc_engine_grid.json
bash scripts/gpu_bench.sh $tag/bench || exit 1
