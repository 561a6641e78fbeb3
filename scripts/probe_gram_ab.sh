#!/bin/bash
# Gram A/B across library builds: probe_gram_pipe.py per build (ALT_LIB).
set -o pipefail
for lib in default "$@"; do
  echo "== $lib"
  if [ "$lib" = default ]; then
    timeout -k 10 200 python scripts/probe_gram_pipe.py || exit 1
  else
    VISREPS_AMD_LIB=$PWD/$lib timeout -k 10 200 python scripts/probe_gram_pipe.py || exit 1
  fi
done
