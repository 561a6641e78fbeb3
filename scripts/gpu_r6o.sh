#!/bin/bash
# Round 6: the shared join's shapes (scripts/microbench_join.hip): gather vs scatter, 4 arrays
# vs one interleaved 16-B record, with FETCH_SIZE / WRITE_SIZE per kernel (separate passes).
set -o pipefail
out=gpurun_out/r6o
mkdir -p $out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 scripts/microbench_join.hip -o /tmp/mb_join || exit 1
timeout -k 10 120 /tmp/mb_join 49995000 10 2>&1 | tee $out/times.log || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/$c -o p --output-format csv -- /tmp/mb_join 49995000 2 \
      > $out/$c.log 2>&1 || { echo "$c pass failed"; tail -5 $out/$c.log; exit 1; }
done
find $out -name '*counter_collection.csv' | head
