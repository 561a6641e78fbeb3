#!/bin/bash
# Round-1 measurement session: full GPU suite, bench line, rocprof kernel stats of the
# bench, PMC traffic passes of the engine (multi call) and the Gram.
set -o pipefail
bash scripts/gpu_check.sh ${1:-v6} || exit 1
bash scripts/gpu_pmc.sh ${1:-v6}_pmc || exit 1
REPS=2 timeout -k 10 200 python scripts/probe_engine_multi.py || exit 1
