#!/bin/bash
# B-walk work-queue segments per wave: 1 (default) vs 4 (VISREPS_ENGINE_SEGS_B=4): one bench line each
# (no CPU baseline, no extra legs), twice, interleaved. Usage: bash scripts/gpu_segsb_ab.sh <tag>
set -o pipefail
tag=${1:-segsb}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  for sj in 1 4; do
    VISREPS_ENGINE_SEGS_B=$sj timeout -k 10 400 python bench.py --no-cpu-baseline --no-est-probe --no-extra-legs \
        > $out/bench_sj${sj}_$rep.json 2> $out/bench_sj${sj}_$rep.err || { echo "bench sj=$sj failed"; tail -20 $out/bench_sj${sj}_$rep.err; exit 1; }
    python3 - $out/bench_sj${sj}_$rep.json $sj <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = b["kernels_per_step"]
print("SEGS_B=%s value %.4f engine %.1f units %.1f" % (sys.argv[2], b["value"], b["breakdown_ms_per_step"]["engine"],
      b["breakdown_ms_per_step"]["units"]), {n: (v["ms_per_step"], v["avg_us"]) for n, v in k.items() if n.startswith(("k_rankB", "k_rankA", "k_join"))})
PY
  done
done
