"""spearman_full at growing n: A vs -A must be -1, A vs A +1 (probe for the >2^31-pair path)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from visreps_amd.analysis import rsa as R
dev = torch.device("cuda", 0)
for n in [int(v) for v in os.environ.get("NS", "500,3000,40000,65536,66000,73000").split(",")]:
    g = torch.Generator(device=dev).manual_seed(n)
    a = R.compute_rdm(torch.randn(n, 24, device=dev, generator=g))
    print(n, n * (n - 1) // 2, R.spearman_full(a, a), R.spearman_full(a, -a), flush=True)
    del a
    torch.cuda.empty_cache()
