#!/bin/bash
# Quick GPU check of a change: the named test files (-m gpu), then one bench line without the
# CPU baseline. Usage (via gpurun): bash scripts/gpu_quick.sh <tag> <test files...>
set -o pipefail
tag=${1:-quick}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" \
      > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest.log | head; tail -30 $out/pytest.log; exit 1; }
  tail -1 $out/pytest.log
fi
timeout -k 10 400 python bench.py --no-cpu-baseline --no-est-probe --no-extra-legs > $out/bench.json 2> $out/bench.err \
    || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python3 - $out/bench.json <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g = b["roofline_gram"]
print("value", b["value"], "gram frac", g["frac"], "gram ms", g["ms_per_step"], "wide", g.get("wide_kernel", {}).get("frac_tile"))
print("kernels", {k: round(v["ms_per_step"], 1) for k, v in b["kernels_per_step"].items()})
print("breakdown", b["breakdown_ms_per_step"])
PY
