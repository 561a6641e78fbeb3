#!/bin/bash
# Engine-only A/B: multi-unit probe (14 units, N=10k) per library build.
set -o pipefail
export TMPDIR=/tmp
for lib in "" "$@"; do
  echo "lib=${lib:-default}"
  ALT_LIB=$lib REPS=2 timeout -k 10 200 python scripts/probe_engine_multi.py 2>&1 | grep engine || exit 1
done
