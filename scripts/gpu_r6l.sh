#!/bin/bash
# Round 6: extraction time vs batch size (MIOpen find NORMAL + cudnn.benchmark, as bench.py),
# and the kernel mix at the default batch 128 vs the best other.
set -o pipefail
out=gpurun_out/r6l
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=NORMAL BENCH=1
for b in 128 256 512 100 200; do
  BATCH=$b timeout -k 10 300 python scripts/probe_extract.py 2>&1 | grep -v amdgpu.ids | tee -a $out/batches.log || exit 1
done
