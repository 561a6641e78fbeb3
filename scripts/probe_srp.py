"""SRP (phase-1 projection) timing per point width at N=10k, HIP events; checksum per width
(identical across builds: the fmas run in CSR order either way)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from visreps_amd.analysis.sparse_random_projection import SparseProjector, get_srp_transformer
dev = torch.device("cuda", 0)
N = 10000
tot = 0.0
for D in [290400, 186624, 64896, 43264, 4096]:
    P = SparseProjector(get_srp_transformer(D=D, k=min(4096, D), density=None, seed=0,
                                            cache_dir=f"/tmp/visreps_srp_cache_{os.getuid()}"), dev)
    x = torch.randn(N, D, device=dev).relu_()
    y = P(x); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        y = P(x)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 3
    tot += ms * (2 if D != 4096 else 4)
    print(f"D={D}: {ms:.2f} ms  checksum={float(y.double().sum()):.10g}", flush=True)
    del x, y
print(f"bench-equivalent SRP per step (14 points): {tot:.1f} ms")
