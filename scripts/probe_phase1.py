"""Phase-1 cost breakdown on the bench's own data (N=10k CustomCNN features, 4 NSD-shaped
ROIs): pipeline.phase1_select as timed in the bench, then its pieces one by one (row
gather, SRP, selection RDMs, rank plans, engine calls), each bracketed by synchronize."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
import numpy as np
import torch

from bench import LAYERS, extract
from visreps_amd import pipeline as PL
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import LegacyRandomState
from visreps_amd.analysis.sparse_random_projection import SparseProjector, get_srp_transformer
from visreps_amd.dataloaders.synthetic import NSD_ROIS_4, make_images, make_responses
from visreps_amd.models.custom_model import CustomCNN
from visreps_amd.models.utils import FeatureExtractor

dev = torch.device("cuda", 0)
N = 10000
torch.manual_seed(0)
model = CustomCNN(num_classes=1000).to(dev).eval()
ex = FeatureExtractor(model, LAYERS, extract_pre_and_post=True)
points = list(ex.return_nodes)
images = make_images(range(N), device=dev)
responses = make_responses(images, range(N), NSD_ROIS_4)
feats = extract(ex, images, 128)
del images
cache = os.path.join("/tmp", f"visreps_srp_cache_{os.getuid()}")
proj = {}
for p in points:
    d = feats[p].size(1)
    proj[p] = SparseProjector(get_srp_transformer(D=d, k=min(4096, d), density=None, seed=0, cache_dir=cache), dev)


def timed(fn, reps=3):
    best = 1e9
    out = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best * 1e3, out


ms, _ = timed(lambda: PL.phase1_select(feats, proj, responses, points, N, n_select=1000, seed=42))
print(f"phase1_select total {ms:.1f} ms", flush=True)
sel = LegacyRandomState(42).choice(N, 1000, replace=False)
st = torch.as_tensor(sel, device=dev)
ms, rows = timed(lambda: {p: feats[p][st] for p in points})
print(f"row gather (14 points) {ms:.1f} ms")
ms, pr = timed(lambda: {p: proj[p](rows[p]) for p in points})
print(f"SRP (14 points, 1000 rows) {ms:.1f} ms")
ms, rd = timed(lambda: {p: R.compute_rdm(pr[p]) for p in points})
print(f"selection RDMs (14) {ms:.1f} ms")
ms, nr = timed(lambda: {r: R.compute_rdm(y[st]) for r, y in responses.items()})
print(f"neural selection RDMs (4) {ms:.1f} ms")
ms, pl = timed(lambda: [R.RankPlan(rd[p]) for p in points])
print(f"rank plans (14) {ms:.1f} ms")
ms, pn = timed(lambda: {r: R.RankPlan(v) for r, v in nr.items()})
print(f"neural rank plans (4) {ms:.1f} ms")
ms, _ = timed(lambda: [R.bootstrap_spearman_multi(pn[r], pl, None, full_first=True) for r in pn])
print(f"engine point Spearmans (4 calls x 14) {ms:.1f} ms")
