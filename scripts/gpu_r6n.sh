#!/bin/bash
# Round 6: Kendall unit A/B -- masks in LDS with two walk blocks per CU (default) against
# masks from L2 with two (VISREPS_KENDALL_MASKS=global) or three blocks per CU (abl/kw3.so).
set -o pipefail
out=gpurun_out/r6n
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
run() { CASES=unit timeout -k 10 300 python scripts/probe_kendall.py > $out/$1.log 2>&1 || { tail -10 $out/$1.log; exit 1; }; echo "$1: $(grep '^unit' $out/$1.log)"; }
run lds2
VISREPS_KENDALL_MASKS=global run l2_2
VISREPS_KENDALL_MASKS=global ALT_LIB=$PWD/abl/kw3.so run l2_3
ALT_LIB=$PWD/abl/kw3.so run lds_kw3build
