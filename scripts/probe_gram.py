"""Gram-only probe: RDMs of N=10k rows at several D (timed with HIP events)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
if os.environ.get("ALT_LIB"):  # another library build (scripts/build_alt.sh)
    import visreps_amd._lib as _L
    _L.LIB_PATH = os.environ["ALT_LIB"]
from visreps_amd.analysis import rsa as R
dev = torch.device("cuda", 0)
N = int(os.environ.get("N", 10000))
for D in [int(x) for x in os.environ.get("DS", "43264,4096,290400").split(",")]:
    x = torch.randn(N, D, device=dev)
    R.compute_rdm(x); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(int(os.environ.get("REPS", 3))):
        R.compute_rdm(x)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / int(os.environ.get("REPS", 3))
    print(f"N={N} D={D}: {ms:.2f} ms  {N * (N + 1) * D / ms / 1e9:.1f} TF/s", flush=True)
    del x
