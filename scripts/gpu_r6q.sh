#!/bin/bash
# Round 6: the exact grid walk (k_rankB_gridx): its engine tests, then the exact-form probe timing
set -o pipefail
out=gpurun_out/r6q
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_est.py \
    -k "grid" > $out/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $out/tests.log | head -20; tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
VISREPS_ENGINE_EST=0 JOINED=1 GRID=1 REPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/exact -o p \
    --output-format csv -- python scripts/probe_engine_bench.py > $out/exact.log 2>&1 || { tail -20 $out/exact.log; exit 1; }
grep "ms/unit" $out/exact.log
