#!/bin/bash
# Bench A/B on one box: the default bench line, then one per variant environment, in
# alternating rounds (no CPU baseline, no EST probe).
#   bash scripts/gpu_bench_ab.sh <tag> <rounds> name:VAR=value ...
set -o pipefail
tag=${1:-benchab}; rounds=${2:-1}; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for r in $(seq 1 $rounds); do
  for spec in default "$@"; do
    name=${spec%%:*}; env=${spec#*:}
    [ "$name" = default ] && env=""
    env $env timeout -k 10 400 python bench.py --no-cpu-baseline --no-est-probe > $out/$name.$r.json 2> $out/$name.$r.err \
        || { echo "$name failed"; tail -20 $out/$name.$r.err; exit 1; }
    python3 - $out/$name.$r.json $name $r <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = b["kernels_per_step"]
print("round", sys.argv[3], sys.argv[2], "value", b["value"], "breakdown",
      {x: b["breakdown_ms_per_step"][x] for x in ("extract", "phase1", "rdms", "units", "engine", "gram")},
      "gram_wide", k["k_gram_wide"]["ms_per_step"], "rankB", k["k_rankB_est"]["ms_per_step"])
PY
  done
done
