#!/bin/bash
# Round-5 check: short bench with the new legs and the exact-form step, the legs' kernel stats
# and bf16 Gram PMC, and the joined engine path's PMC traffic.
set -o pipefail
out=gpurun_out/${1:-r5a}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-est-probe > $out/bench.json 2> $out/bench.err \
    || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python3 - $out/bench.json <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", b["value"], "exact", b.get("exact_form_step_s"))
print("join4", b.get("roofline_join4"))
for k in ("configs4", "configs2_1gpu", "kendall_unit"):
    print(k, json.dumps(b.get(k))[:800])
PY
bash scripts/gpu_legs.sh ${1:-r5a}/legs || exit 1
JOINED=1 bash scripts/gpu_pmc_engine.sh ${1:-r5a}/pmcj || exit 1
