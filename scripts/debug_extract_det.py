"""Is extraction bit-deterministic across calls (the NSD-synthetic driver test re-extracts)?"""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from visreps_amd import utils, evals
from visreps_amd.models import utils as mutils
from visreps_amd.dataloaders.neural import _make_loader, load_nsd_synthetic_test_data

items = ["synthetic.n_test=80", "synthetic.n_train=120", "n_select=60", "n_bootstrap=12",
         "region=[V1,hV4]", "subject_idx=[0,1]", "batchsize=64", "synthetic.nsd_synthetic_n=70",
         "neural_dataset=nsd_synthetic", "mode=eval"]
cfg = utils.validate_config(utils.load_config("configs/eval/base.json", items))
dev = torch.device("cuda", 0)
if len(sys.argv) > 1 and sys.argv[1] == "det":
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = True
    print("deterministic")
cfg = evals._load_cfg(cfg)
data = load_nsd_synthetic_test_data(cfg, [0, 1], ["V1", "hV4"])
outs = []
for trial in range(3):
    model = mutils.configure_feature_extractor(cfg, mutils.load_model(cfg, dev))
    w = [p.detach().float().sum().item() for p in model.parameters()][:3]
    dl = _make_loader(data["stimuli"], None, 64, 0)
    for layer in ["conv5_post", "fc1_post"]:
        a, _ = mutils.extract_single_layer(model, dl, dev, layer, data["test_ids"], keep_on_device=True)
        outs.append((trial, layer, a.float().cpu().numpy(), w))
for layer in ["conv5_post", "fc1_post"]:
    xs = [o for o in outs if o[1] == layer]
    print(layer, "weights", [o[3] for o in xs])
    for o in xs[1:]:
        print(layer, "trial", o[0], "max|diff| vs trial 0:", float(np.max(np.abs(o[2] - xs[0][2]))))
