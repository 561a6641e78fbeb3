"""Write a real bench unit's B-walk row order (posA_byB: A position of every pair in B
order) to a file for scripts/microbench_walk.hip: the bench's CustomCNN conv5_post RDM (B,
model) against the V1 neural RDM (A), N = 10k, through the product's shared join.

  python scripts/probe_walk_order.py <out.bin> [point]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import LAYERS, extract  # noqa: E402
from visreps_amd.analysis import rsa as R  # noqa: E402
from visreps_amd.dataloaders.synthetic import NSD_ROIS_4, make_images, make_responses  # noqa: E402
from visreps_amd.models.custom_model import CustomCNN  # noqa: E402
from visreps_amd.models.utils import FeatureExtractor  # noqa: E402

dev = torch.device("cuda", 0)
N = 10000
point = sys.argv[2] if len(sys.argv) > 2 else "conv5_post"
torch.manual_seed(0)
model = CustomCNN(num_classes=1000).to(dev).eval()
ex = FeatureExtractor(model, LAYERS, extract_pre_and_post=True)
images = make_images(range(N), device=dev)
y = make_responses(images, range(N), {"V1": NSD_ROIS_4["V1"]})["V1"]
feats = extract(ex, images, 128)
pn = R.RankPlan(R.compute_rdm(y))
pm = R.RankPlan(R.compute_rdm(feats[point]))
pos = R.SharedJoins([pn]).join(pm)[0]
a = pos.cpu().numpy().astype(np.uint32)
a.tofile(sys.argv[1])
d = np.abs(np.diff(a.astype(np.int64)))
print(f"{point} x V1: {a.size} pairs, posA range [{a.min()}, {a.max()}], median |step| {np.median(d):.0f}, "
      f"steps < 4096: {np.mean(d < 4096):.4f}", flush=True)
