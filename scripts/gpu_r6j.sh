#!/bin/bash
# Round 6: full-triangle Spearman form choice (bucket, else sort; tables only when named), one-key
# buckets' counts from bucket sizes, distributed count tables (LDS counts for small ranges):
# their GPU tests, then the 73k probe.
set -o pipefail
out=gpurun_out/r6j
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 $T tests/test_gpu_parity.py tests/test_distributed_spearman.py tests/test_kendall.py -m gpu -k "full or distributed or world1 or kendall" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python scripts/probe_full73k.py > $out/full73k.log 2>&1 || { tail -20 $out/full73k.log; exit 1; }
grep "kendall\|spearman" $out/full73k.log
