#!/bin/bash
# Round 6: Kendall's lowest levels as a list of inverted pairs: the Kendall tests, then the unit
# (V2 x V1, N = 10k, 1001 subsets) with every level walked (0) and with 1 / 2 / 3 listed levels
set -o pipefail
out=gpurun_out/r6u
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kendall.py \
    > $out/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $out/tests.log | head -20; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
export CASES=unit_n2_n
for pl in 0 2 1 3 2 0; do
  VISREPS_KENDALL_PAIR_LEVELS=$pl timeout -k 10 200 python scripts/probe_kendall.py > $out/k.json 2> $out/k.err \
      || { tail -20 $out/k.err; exit 1; }
  echo "pair_levels=$pl $(grep unit_n2_n $out/k.err | tail -1)" | tee -a $out/ab.log
done
