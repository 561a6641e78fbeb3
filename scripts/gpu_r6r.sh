#!/bin/bash
# Round 6: exact grid A/B on the bench RDMs (56 units, VISREPS_ENGINE_EST=0): fused 4 regions,
# 2 + 2, and the per-region exact calls (VISREPS_ENGINE_GRIDX=0); kernel stats of the first
set -o pipefail
out=gpurun_out/r6r
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST VISREPS_ENGINE_EST=0 JOINED=1 GRID=1 REPS=3
for v in "4 1" "2 1" "4 0"; do
  set -- $v
  VISREPS_ENGINE_GRIDX_MAXR=$1 VISREPS_ENGINE_GRIDX=$2 timeout -k 10 300 python scripts/probe_engine_bench.py \
      > $out/maxr$1_gx$2.log 2>&1 || { tail -20 $out/maxr$1_gx$2.log; exit 1; }
  echo "maxr=$1 gridx=$2: $(grep ms/unit $out/maxr$1_gx$2.log)"
done
