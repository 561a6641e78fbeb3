#!/bin/bash
# A/B session: RDM tests, Gram probe (split and fp32 kernels), engine probe per library build.
set -o pipefail
out=gpurun_out/${1:-ab}; shift
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "rdm" --timeout 200 --timeout-method thread \
    > $out/pytest_rdm.log 2>&1; echo "pytest rc=$?"; tail -2 $out/pytest_rdm.log
DS=43264,4096 timeout -k 10 200 python scripts/probe_gram.py 2>&1 | grep TF || exit 1
VISREPS_GRAM=fp32 DS=43264 timeout -k 10 200 python scripts/probe_gram.py 2>&1 | grep TF || exit 1
for lib in "" "$@"; do  # engine probe per build
  echo "lib=${lib:-default}"
  ALT_LIB=$lib timeout -k 10 200 python scripts/probe_engine_time.py 2>&1 | grep engine || exit 1
done
