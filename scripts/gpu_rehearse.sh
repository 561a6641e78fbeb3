#!/bin/bash
# Multi-rank rehearsal on a one-GPU box: bench.py at world 2 over gloo (both ranks on
# cuda:0; RCCL refuses two ranks on one device), then world 1 at the same N; the two
# check fields must agree: phase-1 choices equal, unit score and CI within 1e-8 (see below).
# Usage (from the repo root, via gpurun): bash scripts/gpu_rehearse.sh [tag] [n] [world]
set -o pipefail
tag=${1:-rehearse}; n=${2:-4000}; world=${3:-2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
VISREPS_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $world \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $world --steps 1 --warmup 1 --stimuli $n \
    --no-cpu-baseline > $out/w2.json 2> $out/w2.err || { echo "world-$world failed"; tail -30 $out/w2.err; exit 1; }
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --stimuli $n --no-cpu-baseline > $out/w1.json 2> $out/w1.err \
    || { echo "world-1 failed"; tail -30 $out/w1.err; exit 1; }
python3 - $out <<'PY'
import json, sys
def line(f):  # gloo prints its connection lines to stdout too
    return json.loads([l for l in open(f) if l.startswith('{"metric"')][-1])
a = line(sys.argv[1] + "/w2.json"); b = line(sys.argv[1] + "/w1.json")
print("world%s" % a["n_gpus"], a["value"], a["check"]); print("world1", b["value"], b["check"])
# RDMs are bit-identical for identical rows at any world size (tests/test_gpu_distributed.py);
# the extracted features are not: MIOpen / rocBLAS pick kernels by batch shape (a shard's
# last batch differs), so the rows may differ in their last bits between shardings
ca, cb = a["check"], b["check"]
same_phase1 = ca["phase1_best"] == cb["phase1_best"]
d = max(abs(ca["score"] - cb["score"]), *(abs(x - y) for x, y in zip(ca["ci"], cb["ci"])))
print("phase-1 choices equal:", same_phase1, " max |d| score/ci:", d, " bit-equal:", ca == cb)
sys.exit(0 if same_phase1 and d < 1e-8 else 1)
PY
