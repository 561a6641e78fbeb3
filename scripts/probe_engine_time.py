"""Engine timing probe: N=10k unit (1001 subsets), HIP-event time per call and per-kernel
split is left to rocprof. Prints ms per unit and the algorithmic HBM rate."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
if os.environ.get("ALT_LIB"):  # A/B against another build of the library
    import visreps_amd._lib as _L
    _L.LIB_PATH = os.environ["ALT_LIB"]
    for _k in [k for k in _L._PROTOTYPES if "kendall" in k]:
        del _L._PROTOTYPES[_k]
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices
dev = torch.device("cuda", 0)
N = int(os.environ.get("N", 10000))
g = torch.Generator(device=dev); g.manual_seed(0)
A = R.compute_rdm(torch.randn(N, 64, device=dev, generator=g) @ torch.randn(64, 3000, device=dev, generator=g) + 2*torch.randn(N, 3000, device=dev, generator=g))
B = R.compute_rdm(torch.randn(N, 2000, device=dev, generator=g))
pa, pb = R.RankPlan(A), R.RankPlan(B)
k = int(0.9 * N)
idx = torch.from_numpy(bootstrap_indices(42, N, k, 1000).copy()).to(dev)
s0 = R.bootstrap_spearman(pa, pb, idx); torch.cuda.synchronize()
ts = []
for _ in range(int(os.environ.get("REPS", 3))):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); s = R.bootstrap_spearman(pa, pb, idx); b.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
    assert torch.equal(s, s0)
ms = min(ts)
byt = 8.0 * (N * (N - 1) // 2 + 1000 * (k * (k - 1) // 2))
print(f"engine N={N}: {ms:.2f} ms/unit  {byt / ms / 1e6:.0f} GB/s algorithmic  first={s0[:3].tolist()} sum={float(s0.sum()):.17g}", flush=True)
