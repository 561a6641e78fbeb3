#!/bin/bash
# Grid-walk A/B (mask-multiply, non-temporal) + short benches at extraction batch 128 / 512.
set -o pipefail
tag=${1:-r5l}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_grid_ab.sh $tag/ab abl/mm.so abl/nt0.so || exit 1
for b in 128 512; do
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --batch $b --no-cpu-baseline --no-est-probe --no-extra-legs --no-exact-step \
      > $out/bench_b$b.json 2> $out/bench_b$b.err || { echo "bench b$b failed"; tail -20 $out/bench_b$b.err; exit 1; }
  python3 - $out/bench_b$b.json $b <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("batch", sys.argv[2], "value", b["value"], "breakdown", b["breakdown_ms_per_step"], "roofline", b["roofline"]["frac"], b["roofline"]["avg_launch_us"])
PY
done
