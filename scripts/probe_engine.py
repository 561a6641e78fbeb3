"""Engine-only probe: one N=10k unit (1000+1 subsets) for kernel-level profiling."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices
dev = torch.device("cuda", 0)
N = int(os.environ.get("N", 10000))
g = torch.Generator(device=dev); g.manual_seed(0)
A = R.compute_rdm(torch.randn(N, 64, device=dev, generator=g) @ torch.randn(64, 3000, device=dev, generator=g) + 2*torch.randn(N, 3000, device=dev, generator=g))
B = R.compute_rdm(torch.randn(N, 2000, device=dev, generator=g))
pa, pb = R.RankPlan(A), R.RankPlan(B)
idx = torch.from_numpy(bootstrap_indices(42, N, int(0.9 * N), 1000).copy()).to(dev)
for _ in range(int(os.environ.get("REPS", 2))):
    s = R.bootstrap_spearman(pa, pb, idx)
torch.cuda.synchronize()
print("ok", s[:3].tolist())
