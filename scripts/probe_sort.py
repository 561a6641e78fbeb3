"""Times vr_sort_pairs_u32 (4 LSD passes) on M uniform keys -- the rank-plan sort's size
at N = 10000 (M = N(N-1)/2). VISREPS_AMD_LIB selects an ablation library."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from visreps_amd import _lib
from visreps_amd.analysis.distributed_spearman import RankKernels

m = int(sys.argv[1]) if len(sys.argv) > 1 else 49995000
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
k = torch.randint(-(1 << 31), (1 << 31) - 1, (m,), dtype=torch.int32, device=dev, generator=g)
v = torch.arange(m, dtype=torch.int32, device=dev)
for _ in range(3):
    RankKernels.sort(k, v)
torch.cuda.synchronize()
reps = 20
t0 = time.perf_counter()
for _ in range(reps):
    ks, vs = RankKernels.sort(k, v)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
u = ks.to(torch.int64) & 0xFFFFFFFF
ok = bool(torch.all(u[1:] >= u[:-1]).item())
print(f"{_lib.LIB_PATH.split('/')[-1]}: M={m} sort {dt * 1e3:.3f} ms (incl. 2 clones, "
      f"{4 * m * 4 / dt / 1e9:.0f} GB/s clone-equiv) sorted={ok}")
