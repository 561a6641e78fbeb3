#!/bin/bash
# Round 6: Kendall walks with their block-summary partials over the mask LDS (two 16-wave
# blocks per CU at n = 10k) -- Kendall tests, then the unit probe against the previous build
# (abl/kw1blk.so: one block per CU).
set -o pipefail
out=gpurun_out/r6m
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_kendall.py -m gpu > $out/kendall.log 2>&1 || { tail -30 $out/kendall.log; exit 1; }
tail -1 $out/kendall.log
CASES=unit timeout -k 10 300 python scripts/probe_kendall.py > $out/unit_new.log 2>&1 || { tail -10 $out/unit_new.log; exit 1; }
grep -v amdgpu.ids $out/unit_new.log | tail -3
ALT_LIB=$PWD/abl/kw1blk.so CASES=unit timeout -k 10 300 python scripts/probe_kendall.py > $out/unit_old.log 2>&1 || { tail -10 $out/unit_old.log; exit 1; }
grep -v amdgpu.ids $out/unit_old.log | tail -3
