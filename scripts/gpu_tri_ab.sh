#!/bin/bash
# Triangle-order TB (EST 5/6, opt-in VISREPS_ENGINE_TRI=1) vs the default A-order TB + joins:
# engine parity tests, then one bench line of each form (no CPU baseline, no extra legs).
# Usage (via gpurun): bash scripts/gpu_tri_ab.sh <tag> [test files...]
set -o pipefail
tag=${1:-tri}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu "$@" \
      > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest.log | head; tail -30 $out/pytest.log; exit 1; }
  tail -1 $out/pytest.log
fi
for form in 1 0; do
  VISREPS_ENGINE_TRI=$form timeout -k 10 400 python bench.py --no-cpu-baseline --no-est-probe --no-extra-legs \
      > $out/bench_tri$form.json 2> $out/bench_tri$form.err || { echo "bench tri=$form failed"; tail -20 $out/bench_tri$form.err; exit 1; }
  python3 - $out/bench_tri$form.json $form <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = b["kernels_per_step"]
print("TRI=%s value %.4f engine %.1f reruns %s tail %s" % (sys.argv[2], b["value"], b["breakdown_ms_per_step"]["engine"],
      b["est_reruns"], b.get("est_tail_flags")))
print("  ", {n: (v["ms_per_step"], v["avg_us"]) for n, v in k.items() if n.startswith(("k_rank", "k_join", "k_count"))})
PY
done
