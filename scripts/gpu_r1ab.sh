set -o pipefail
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
mkdir -p gpurun_out/r1ab
( cd altlib/r1tree && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r1ab/r1 -o p --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r1ab/r1.json 2> $GRAFT_REPO_ROOT/gpurun_out/r1ab/r1.err ) || { echo r1 failed; tail gpurun_out/r1ab/r1.err; exit 1; }
rm -f gpurun_out/r1ab/r1/p_kernel_trace.csv
cat gpurun_out/r1ab/r1.json | python3 -c "import json,sys; print('r1 step', json.loads(sys.stdin.read())['value'])"
grep -h "k_rankB\|k_rankA" gpurun_out/r1ab/r1/p_kernel_stats.csv | cut -d, -f1-4 | cut -c1-40,170-260
