#!/bin/bash
# Extraction batch size A/B inside the bench (breakdown_ms_per_step.extract).
set -o pipefail
out=gpurun_out/${1:-batchab}
mkdir -p $out
for b in 128 256 512; do
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch $b > $out/b$b.json 2> $out/b$b.err \
    || { echo "batch $b failed"; tail -5 $out/b$b.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$out/b$b.json').read().strip().splitlines()[-1]); print($b, d['value'], d['breakdown_ms_per_step'])"
done
