#!/bin/bash
# HBM traffic of the hot kernels: separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
# over the engine probe (one multi call: 14 units of N=10k, REPS=1) and the Gram probe (N=10k, D=43264).
set -o pipefail
tag=${1:-pmc}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  REPS=1 timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $out/eng_$c -o p --output-format csv \
      -- python scripts/probe_engine_multi.py > $out/eng_$c.log 2>&1 || { echo "engine $c failed"; tail $out/eng_$c.log; exit 1; }
  DS=43264 timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $out/gram_$c -o p --output-format csv \
      -- python scripts/probe_gram.py > $out/gram_$c.log 2>&1 || { echo "gram $c failed"; tail $out/gram_$c.log; exit 1; }
done
find $out -name '*counter_collection*'
