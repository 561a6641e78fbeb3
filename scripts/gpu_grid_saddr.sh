#!/bin/bash
# Grid walk gather-form check: engine EST tests (grid equality included), then the 56-unit
# grid probe for the default build vs the alternative libraries.
set -o pipefail
tag=${1:-gsa}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_engine_est.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
bash scripts/gpu_grid_ab.sh $tag/grid "$@" || exit 1
rm -f $out/grid/*/p_kernel_trace.csv
