#!/bin/bash
# Run GPU pytest files on the box: bash scripts/gpu_pytest.sh <tag> <files...>
set -o pipefail
tag=${1:-pt}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
timeout -k 10 1000 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $out/pytest.log | sed 's/ PASSED.*/ PASSED/' | tail -80
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "^E " $out/pytest.log | head -40; exit 1; }
