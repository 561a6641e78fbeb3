"""Kendall engine timing probe: one N-stimulus unit (point + NB bootstrap subsets)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices
dev = torch.device("cuda", 0)
N = int(os.environ.get("N", 10000)); NB = int(os.environ.get("NB", 1000))
g = torch.Generator(device=dev); g.manual_seed(0)
A = R.compute_rdm(torch.randn(N, 64, device=dev, generator=g) @ torch.randn(64, 3000, device=dev, generator=g) + 2*torch.randn(N, 3000, device=dev, generator=g))
B = R.compute_rdm(torch.randn(N, 2000, device=dev, generator=g))
pa, pb = R.RankPlan(A), R.RankPlan(B)
k = int(0.9 * N)
idx = torch.from_numpy(bootstrap_indices(42, N, k, NB).copy()).to(dev)
s0 = R.bootstrap_kendall(pa, pb, idx); torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(); s = R.bootstrap_kendall(pa, pb, idx); b.record(); torch.cuda.synchronize()
assert torch.equal(s, s0)
print(f"kendall N={N} NB={NB}: {a.elapsed_time(b):.1f} ms/unit  point={s0[0].item():.8f} boot={s0[1:4].tolist()}", flush=True)
