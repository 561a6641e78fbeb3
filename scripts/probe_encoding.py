"""Encoding-score timing on one MI355X: n_train=NTR (9000), n_test=1000, V=2000 voxels,
layers of D in DIMS (4096,43264), synthetic and seeded, 1000 bootstraps."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from visreps_amd.analysis.alignment import AlignmentData
from visreps_amd.analysis.encoding_score import compute_encoding_score

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
n_tr, n_te, v = int(os.environ.get("NTR", 9000)), 1000, 2000
n = n_tr + n_te
z = torch.randn(n, 64, device=dev, generator=g)
acts = {f"d{d}": torch.relu(z @ (torch.randn(64, d, device=dev, generator=g) / 8)
                            + 2 * torch.randn(n, d, device=dev, generator=g))
        for d in [int(v) for v in os.environ.get("DIMS", "4096,43264").split(",")]}
Y = z @ torch.randn(64, v, device=dev, generator=g) + 3 * torch.randn(n, v, device=dev, generator=g)
tr = AlignmentData({k: a[:n_tr] for k, a in acts.items()}, Y[:n_tr])
te = AlignmentData({k: a[n_tr:] for k, a in acts.items()}, Y[n_tr:])
for it in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    res = compute_encoding_score(tr, te, bootstrap=True, n_bootstrap=1000, seed=42)[0]
    torch.cuda.synchronize()
    print(f"run {it}: {time.perf_counter() - t:.2f} s  layer={res['layer']} score={res['score']:.4f} "
          f"ci=[{res['ci_low']:.4f}, {res['ci_high']:.4f}] sel={[round(s['score'], 4) for s in res['layer_selection_scores']]}",
          flush=True)
