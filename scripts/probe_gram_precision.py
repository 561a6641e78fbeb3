"""Split-Gram RDM error vs fp64 per wide kernel (k_gram3e / k_gram3p) and depth, n = 6000
post-ReLU synthetic rows (the test_rdm_wide_supertiles data)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import rsa_oracle as O
from visreps_amd.analysis import rsa as R
dev = torch.device("cuda", 0)
os.environ["VISREPS_GRAM"] = "split"
n = 6000
for d in (40, 64, 300, 1100, 4096):
    x = torch.from_numpy(O.synthetic_features(n, [d], seed=13, relu=[True])[0]).to(dev)
    xd = x.double()
    xd = xd - xd.mean(1, keepdim=True)
    s = torch.sqrt((xd * xd).mean(1) + 1e-12)
    ref = 1.0 - ((xd @ xd.T / d) / (s[:, None] * s[None, :] + 1e-12)).clamp(-1.0, 1.0)
    ref.fill_diagonal_(0.0)
    errs = {}
    for k in ("e", "p"):
        os.environ["VISREPS_GRAM_KERNEL"] = k
        errs[k] = float((R.compute_rdm(x).double() - ref).abs().max())
    os.environ["VISREPS_GRAM"] = "fp32"
    errs["fp32"] = float((R.compute_rdm(x).double() - ref).abs().max())
    os.environ["VISREPS_GRAM"] = "split"
    print(f"d={d}: " + "  ".join(f"{k} {v:.3g}" for k, v in errs.items()), flush=True)
