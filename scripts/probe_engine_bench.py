"""Engine probe on the bench's own RDMs: the 14 CustomCNN points (random init, seed 0) of
10k synthetic images against the V1 neural RDM, one vr_bootstrap_spearman_multi call
(14 units x 1001 subsets), timed REPS times. ALT_LIB=path selects another library build.
JOINED=1: the 4 NSD ROI neural plans, shared joins (vr_engine_posmap4 once, vr_engine_join4
per model plan) and one vr_bootstrap_spearman_multi_joined call per region (4 x 14 = 56
units); with GRID=1 one region-fused vr_bootstrap_spearman_grid_joined call instead (the
bench's engine path)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
import torch
if os.environ.get("ALT_LIB"):
    import visreps_amd._lib as _L
    _L.LIB_PATH = os.environ["ALT_LIB"]
from bench import LAYERS, extract
from visreps_amd.analysis import rsa as R
from visreps_amd import _lib
from visreps_amd.analysis._random import bootstrap_indices
from visreps_amd.dataloaders.synthetic import NSD_ROIS_4, make_images, make_responses
from visreps_amd.models.custom_model import CustomCNN
from visreps_amd.models.utils import FeatureExtractor

dev = torch.device("cuda", 0)
N = 10000
torch.manual_seed(0)
model = CustomCNN(num_classes=1000).to(dev).eval()
ex = FeatureExtractor(model, LAYERS, extract_pre_and_post=True)
images = make_images(range(N), device=dev)
JOINED = os.environ.get("JOINED", "0") == "1"
ys = make_responses(images, range(N), NSD_ROIS_4 if JOINED else {"V1": NSD_ROIS_4["V1"]})
feats = extract(ex, images, 128)
del images
neurals = {r: R.RankPlan(R.compute_rdm(y)) for r, y in ys.items()}
neural = neurals["V1"]
models = []
for p in list(feats):
    models.append(R.RankPlan(R.compute_rdm(feats.pop(p))))
torch.cuda.empty_cache()
idx = torch.from_numpy(bootstrap_indices(42, N, int(0.9 * N), 1000).copy()).to(dev)
ts = []


def joined_step():
    sj = R.SharedJoins(list(neurals.values()))
    js = [sj.join(pm) for pm in models]  # js[m][region]
    del sj
    if os.environ.get("GRID", "0") == "1":  # the region-fused call (bootstrap_spearman_grid)
        g = R.bootstrap_spearman_grid(list(neurals.values()), models, idx, js, full_first=True)
        return g.reshape(-1, g.shape[-1])
    out = []
    for i, pn in enumerate(neurals.values()):
        out.append(R.bootstrap_spearman_multi(pn, models, idx, joined=[js[m][i] for m in range(len(models))]))
    return torch.cat(out)


for _ in range(int(os.environ.get("REPS", 2))):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    s = joined_step() if JOINED else R.bootstrap_spearman_multi(neural, models, idx)
    b.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(b) / (len(neurals) if JOINED else 1))
ref_note = ""
if os.environ.get("CHECK_EXACT", "1") == "1" and os.environ.get("VISREPS_ENGINE_EST") == "1":
    os.environ["VISREPS_ENGINE_EST"] = "0"  # the same RDMs in the exact form, same process
    ref = R.bootstrap_spearman_multi(neural, models, idx)
    os.environ["VISREPS_ENGINE_EST"] = "1"
    s0 = s[: len(models)]  # JOINED: the first region's units (V1, the reference's neural plan)
    ref_note = f" exact_equal={bool(torch.equal(ref, s0))} max_diff={float((ref - s0).abs().max()):.3g}"
print(f"engine bench-RDMs NB={len(models)}: {min(ts) / len(models):.2f} ms/unit  "
      f"checksum={float(s.double().sum()):.15g} est_reruns={int(_lib.lib().vr_engine_est_reruns())}{ref_note}",
      flush=True)
