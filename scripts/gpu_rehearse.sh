#!/bin/bash
# Multi-rank rehearsal on a one-GPU box: bench.py at world 2 over gloo (both ranks on
# cuda:0; RCCL refuses two ranks on one device), then world 1 at the same N; the two
# check fields (unit score and CI, phase-1 choices) must be identical: the RDMs are
# bit-identical at every world size (pipeline.py), and the scores exact integer statistics.
# Usage (from the repo root, via gpurun): bash scripts/gpu_rehearse.sh [tag] [n]
set -o pipefail
tag=${1:-rehearse}; n=${2:-4000}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
VISREPS_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --stimuli $n \
    --no-cpu-baseline > $out/w2.json 2> $out/w2.err || { echo "world-2 failed"; tail -30 $out/w2.err; exit 1; }
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --stimuli $n --no-cpu-baseline > $out/w1.json 2> $out/w1.err \
    || { echo "world-1 failed"; tail -30 $out/w1.err; exit 1; }
python3 - $out <<'PY'
import json, sys
def line(f):  # gloo prints its connection lines to stdout too
    return json.loads([l for l in open(f) if l.startswith('{"metric"')][-1])
a = line(sys.argv[1] + "/w2.json"); b = line(sys.argv[1] + "/w1.json")
print("world2", a["value"], a["check"]); print("world1", b["value"], b["check"])
print("check equal:", a["check"] == b["check"])
sys.exit(0 if a["check"] == b["check"] else 1)
PY
