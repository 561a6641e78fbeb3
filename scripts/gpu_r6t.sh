#!/bin/bash
# Round 6: Kendall unit (V2 x V1 neural RDMs, N = 10k, 1001 subsets) for the default build and
# alternative builds (abl/*.so: two windows per trip off, 64-bit and per-call transposes)
set -o pipefail
out=gpurun_out/r6t
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST CASES=unit_n2_n
for lib in default abl/kwpair0.so abl/xk1.so abl/xk2.so default; do
  for rep in 1 2; do
    if [ $lib = default ]; then
      timeout -k 10 200 python scripts/probe_kendall.py > $out/k.json 2> $out/k.err || { tail -20 $out/k.err; exit 1; }
    else
      ALT_LIB=$lib timeout -k 10 200 python scripts/probe_kendall.py > $out/k.json 2> $out/k.err || { tail -20 $out/k.err; exit 1; }
    fi
    echo "$lib $rep $(grep unit_n2_n $out/k.err | tail -1)" | tee -a $out/ab.log
  done
done
