#!/bin/bash
# Whole GPU parity suite (no -x: every failure is listed) + smoke.
# Usage (from the repo root, via gpurun): bash scripts/gpu_suite.sh [tag] [pytest args...]
set -o pipefail
tag=${1:-suite}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -q -rf --timeout 300 --timeout-method thread \
    > $out/pytest_gpu.log 2>&1
rc=$?
tail -15 $out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
exit $rc
