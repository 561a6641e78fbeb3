#!/bin/bash
# Gram timing of library variants, alternating rounds (probe_gram.py, N = 10k, random rows):
#   bash scripts/gpu_gram_variants.sh <tag> <rounds> name:lib.so | name:VAR=value ...
#   ("default" = the in-tree library, no extra environment)
set -o pipefail
tag=${1:-gramvar}; rounds=${2:-2}; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp DS=${DS:-43264,290400} REPS=${REPS:-5}
for r in $(seq 1 $rounds); do
  for spec in default "$@"; do
    name=${spec%%:*}; lib=${spec#*:}
    if [ "$name" = default ]; then env="";
    elif [[ "$lib" == *=* ]]; then env="$lib";
    else env="ALT_LIB=$PWD/$lib"; fi
    env $env timeout -k 10 200 python scripts/probe_gram.py > $out/$name.$r.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.$r.log; exit 1; }
    echo "round $r $name: $(grep -h 'TF/s' $out/$name.$r.log | tr '\n' ' ')"
  done
done
