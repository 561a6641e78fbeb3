#!/bin/bash
# HBM traffic of one 14-unit engine call on the bench RDMs (probe_engine_bench.py, REPS=1):
# separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE, summarised per unit with
# the gfx950 FETCH_SIZE x 2 correction (profiles/r2_fetch_calibration.json).
# JOINED=1: the bench's path (shared joins + one joined call per region, 56 units).
# Usage (from the repo root, via gpurun): [JOINED=1] bash scripts/gpu_pmc_engine.sh [tag]
set -o pipefail
tag=${1:-pmc_engine}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST REPS=1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d $out/$c -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$c.log 2>&1 || { echo "$c pass failed"; tail -5 $out/$c.log; exit 1; }
done
units=14; [ "${JOINED:-0}" = 1 ] && units=56
python3 scripts/pmc_engine_summary.py $out $units > $out/pmc_engine.json && cat $out/pmc_engine.json
