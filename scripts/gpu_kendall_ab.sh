#!/bin/bash
# Kendall A/B: parity tests, then per-stream walk times for the default build and each
# alternative library. Usage (via gpurun): bash scripts/gpu_kendall_ab.sh <tag> [lib.so ...]
set -o pipefail
tag=${1:-kab}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_kendall.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
bash scripts/gpu_kendall_levels.sh $tag/klv "$@" || exit 1
