#!/bin/bash
# Full GPU parity suite (margins logged), smoke, and the world-2 rehearsal of the multi-rank
# path on one GPU. Usage (via gpurun): bash scripts/gpu_suite.sh [tag]
set -o pipefail
tag=${1:-suite}
out=gpurun_out/$tag
mkdir -p $out
export VISREPS_MARGINS=$out/parity_margins.jsonl
rm -f $VISREPS_MARGINS
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
    > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest.log | head; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
bash scripts/gpu_rehearse.sh $tag/rehearse 4000
