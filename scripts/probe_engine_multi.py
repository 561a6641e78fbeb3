"""Engine probe in the bench's shape: one neural plan against NB model plans (one
vr_bootstrap_spearman_multi call = NB units of N=10k, 1001 subsets each)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
if os.environ.get("ALT_LIB"):  # A/B against another build of the library
    import visreps_amd._lib as _L
    _L.LIB_PATH = os.environ["ALT_LIB"]
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices
dev = torch.device("cuda", 0)
N = int(os.environ.get("N", 10000)); NB = int(os.environ.get("NB", 14))
g = torch.Generator(device=dev); g.manual_seed(0)
neural = R.RankPlan(R.compute_rdm(torch.randn(N, 2000, device=dev, generator=g)))
z = torch.randn(N, 64, device=dev, generator=g)
models = []
for j in range(NB):
    x = torch.relu(z @ torch.randn(64, 1024, device=dev, generator=g) + 2 * torch.randn(N, 1024, device=dev, generator=g))
    models.append(R.RankPlan(R.compute_rdm(x)))
k = int(0.9 * N)
idx = torch.from_numpy(bootstrap_indices(42, N, k, 1000).copy()).to(dev)
ts = []
for _ in range(int(os.environ.get("REPS", 2))):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); s = R.bootstrap_spearman_multi(neural, models, idx); b.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
ms = min(ts) / NB
byt = 8.0 * (N * (N - 1) // 2 + 1000 * (k * (k - 1) // 2))
print(f"engine multi N={N} NB={NB}: {ms:.2f} ms/unit  {byt / ms / 1e6:.0f} GB/s algorithmic  point0={float(s[0, 0]):.12g}", flush=True)
