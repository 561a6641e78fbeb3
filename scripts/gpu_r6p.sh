#!/bin/bash
# Round 6: the exact form's kernel split on the bench's grid path (56 units, VISREPS_ENGINE_EST=0)
set -o pipefail
out=gpurun_out/r6p
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
VISREPS_ENGINE_EST=0 JOINED=1 GRID=1 REPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/exact -o p \
    --output-format csv -- python scripts/probe_engine_bench.py > $out/exact.log 2>&1 || { tail -20 $out/exact.log; exit 1; }
tail -5 $out/exact.log
