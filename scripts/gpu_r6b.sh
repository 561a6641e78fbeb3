#!/bin/bash
# Round 6, second GPU call: prefetching walk with L2 masks on by default (the round-5 fault's
# cause fixed), EST 1 fallback for calls whose EST 3 estimate fails up front, grid flagged
# passes re-run alone: the engine tests, the large-n test, the large-n unit probe.
set -o pipefail
out=gpurun_out/r6b
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST VISREPS_MARGINS=$PWD/$out/parity_margins.jsonl
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_engine_est.py "tests/test_gpu_parity.py::test_bootstrap_masks_large_n_global_path" -m gpu > $out/engine_est.log 2>&1 || { tail -40 $out/engine_est.log; exit 1; }
tail -3 $out/engine_est.log
timeout -k 10 500 python scripts/probe_large_n.py > $out/large_n.log 2>&1 || { tail -20 $out/large_n.log; exit 1; }
cat $out/large_n.log
VISREPS_ENGINE_EST1_FALLBACK=0 SIZES=20500 timeout -k 10 400 python scripts/probe_large_n.py > $out/large_n_noest1.log 2>&1 || { tail -20 $out/large_n_noest1.log; exit 1; }
cat $out/large_n_noest1.log
