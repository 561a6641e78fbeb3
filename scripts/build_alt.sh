#!/bin/bash
# Builds an alternative library with extra defines for A/B timing probes:
#   bash scripts/build_alt.sh <name> "-DVR_X=1 ..."  ->  abl/<name>.so
# (abl/ is git-ignored, not gpurun-ignored: it travels to the GPU box)
set -e
name=$1; flags=$2
cd "$(dirname "$0")/../visreps_amd/csrc"
make -s -j8 BUILD=build_$name OUT=../../abl/$name.so EXTRA="$flags" >/dev/null
echo "abl/$name.so"
