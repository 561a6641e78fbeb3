"""Gram accuracy on the bench's own CustomCNN points (N=10k): max |dRDM| on 64 sampled rows
against float64 references, for the split and the exact-fp32 kernels, with the centring
done in float64 and in float32 (the reference's x -= x.mean(1) runs in fp32)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
import torch
from bench import LAYERS, extract
from visreps_amd.analysis import rsa as R
from visreps_amd.dataloaders.synthetic import make_images
from visreps_amd.models.custom_model import CustomCNN
from visreps_amd.models.utils import FeatureExtractor

dev = torch.device("cuda", 0)
N = int(os.environ.get("N", 10000))
torch.manual_seed(0)
model = CustomCNN(num_classes=1000).to(dev).eval()
ex = FeatureExtractor(model, LAYERS, extract_pre_and_post=True)
images = make_images(range(N), device=dev)
feats = extract(ex, images, 128)
del images
rows = torch.randperm(N, device=dev, generator=torch.Generator(device=dev).manual_seed(1))[:64]


def ref_rows(x, f32_centre):
    if f32_centre:
        xc = (x - x.mean(1, keepdim=True)).double()
    else:
        xd = x.double()
        xc = xd - xd.mean(1, keepdim=True)
    s = torch.sqrt((xc * xc).mean(1) + 1e-12)
    g = xc[rows] @ xc.T / x.size(1)
    out = 1.0 - (g / (s[rows, None] * s[None, :] + 1e-12)).clamp(-1, 1)
    out[torch.arange(64, device=dev), rows] = 0.0
    return out


for p in [q for q in os.environ.get("POINTS", ",".join(feats)).split(",")]:
    x = feats[p]
    st = x.std(1) / x.mean(1).abs().clamp_min(1e-30)
    split = R.compute_rdm(x)[rows].double()
    os.environ["VISREPS_GRAM"] = "fp32"
    f32 = R.compute_rdm(x)[rows].double()
    del os.environ["VISREPS_GRAM"]
    r64, r32 = ref_rows(x, False), ref_rows(x, True)
    print(f"{p:11s} D={x.size(1):6d} std/|mean|={float(st.median()):.3g}  split: vs64c {float((split - r64).abs().max()):.2e}"
          f" vs32c {float((split - r32).abs().max()):.2e} | fp32: vs64c {float((f32 - r64).abs().max()):.2e}"
          f" vs32c {float((f32 - r32).abs().max()):.2e} | 32c-64c {float((r32 - r64).abs().max()):.2e}", flush=True)
