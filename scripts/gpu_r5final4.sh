#!/bin/bash
# Round-5 final build: full GPU suite + smoke + rehearsal and the engine PMC of the grid path
# (gpu_r5final1.sh), the PMC profile placed where bench.py reads it, then the bench.
set -o pipefail
tag=${1:-r5final4}
bash scripts/gpu_r5final1.sh $tag || exit 1
cp gpurun_out/$tag/pmc/pmc_engine.json profiles/r5_pmc_engine_grid.json || exit 1
bash scripts/gpu_bench.sh $tag/bench || exit 1
