#!/bin/bash
# k_rankB gap probe: the plain row gather in a real B walk's order vs random vs sequential.
set -o pipefail
out=gpurun_out/${1:-walk_probe}
mkdir -p $out /tmp/mbw
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 scripts/microbench_walk.hip -o /tmp/mbw/mb_walk || exit 1
timeout -k 10 300 python scripts/probe_walk_order.py /tmp/mbw/posA.bin conv5_post > $out/order.log 2>&1 || { tail -20 $out/order.log; exit 1; }
cat $out/order.log | tail -2
timeout -k 10 120 /tmp/mbw/mb_walk /tmp/mbw/posA.bin > $out/mb_walk.log 2>&1; rc=$?
cat $out/mb_walk.log
exit $rc
