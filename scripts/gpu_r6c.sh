#!/bin/bash
# Round 6: the O(m log m) Kendall form (kendall_full.hip): vector and triangle tests, 73k.
set -o pipefail
out=gpurun_out/r6c
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST VISREPS_MARGINS=$PWD/$out/parity_margins.jsonl
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_kendall.py -m gpu -k "vec or full" > $out/kendall.log 2>&1 || { tail -40 $out/kendall.log; exit 1; }
tail -15 $out/kendall.log
cat $out/parity_margins.jsonl
