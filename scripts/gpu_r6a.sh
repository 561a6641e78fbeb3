#!/bin/bash
# Round 6, first GPU call: the new grid-engine tests (full-size grid parity, L2-mask grid,
# flagged/structured regions leaving the fused set, n = 12,000 / 20,500 forms), smoke, the
# large-n unit probe, then the prefetching walk with L2 masks (abl/xwl2.so, -DVR_XW_L2=1)
# on the round-5 faulting test -- last, so a fault there ends nothing else.
set -o pipefail
out=gpurun_out/r6a
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST VISREPS_MARGINS=$PWD/$out/parity_margins.jsonl
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_engine_est.py -m gpu > $out/engine_est.log 2>&1 || { tail -30 $out/engine_est.log; exit 1; }
tail -3 $out/engine_est.log
timeout -k 10 700 $T "tests/test_benchsize.py::test_bench_grid_walk_full_size" -m gpu > $out/grid_full.log 2>&1 || { tail -30 $out/grid_full.log; exit 1; }
tail -3 $out/grid_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
cat $out/smoke.log
timeout -k 10 400 python scripts/probe_large_n.py > $out/large_n.log 2>&1 || { tail -20 $out/large_n.log; exit 1; }
cat $out/large_n.log
# the round-5 fault: prefetching B walk with masks from L2
VISREPS_AMD_LIB=$PWD/abl/xwl2.so timeout -k 10 300 $T "tests/test_gpu_parity.py::test_bootstrap_masks_large_n_global_path" \
    "tests/test_engine_est.py::test_large_n_engine_forms" -m gpu > $out/xwl2.log 2>&1 || { tail -40 $out/xwl2.log; exit 1; }
tail -5 $out/xwl2.log
ALT_LIB=$PWD/abl/xwl2.so timeout -k 10 400 python scripts/probe_large_n.py > $out/large_n_xwl2.log 2>&1 || { tail -20 $out/large_n_xwl2.log; exit 1; }
cat $out/large_n_xwl2.log
