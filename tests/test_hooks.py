"""Extraction points (reference visreps/models/utils.py:122-230, custom_model.py:140-185,
standard_model.py:5-20). CPU: the forward pass is plumbing here, no HIP kernel is involved.

  * CustomCNN: 7 layers x pre/post = 14 points, each hooked on the module the reference's
    mapping picks (`_pre` the raw Conv2d/Linear, i.e. pre-BN; `_post` the ReLU after BN),
    with the flattened widths of SURVEY §3.5 (290,400 ... 4,096; sum 1,316,544);
  * torchvision AlexNet: every Conv/Linear is followed directly by ReLU(inplace=True), so
    the hook on the Conv stores the tensor the ReLU then overwrites: `_pre == _post`.
"""
import torch
import torch.nn as nn

from visreps_amd.models.custom_model import CustomCNN
from visreps_amd.models.standard_model import AlexNetModule
from visreps_amd.models.utils import FeatureExtractor

LAYERS = ["conv1", "conv2", "conv3", "conv4", "conv5", "fc1", "fc2"]

# SURVEY §3.5 (measured on the reference CustomCNN via forward hooks)
WIDTHS = {"conv1": 290400, "conv2": 186624, "conv3": 64896, "conv4": 64896, "conv5": 43264,
          "fc1": 4096, "fc2": 4096}
# reference module indices (custom_model.py:147-185): features = [Conv, BN, ReLU, (Pool)] x 5,
# classifier = [Dropout, Linear, BN, ReLU, Dropout, Linear, BN, ReLU, Linear]
CUSTOM_PATHS = {
    "conv1": ("features.0", "features.2"), "conv2": ("features.4", "features.6"),
    "conv3": ("features.8", "features.10"), "conv4": ("features.11", "features.13"),
    "conv5": ("features.14", "features.16"), "fc1": ("classifier.1", "classifier.3"),
    "fc2": ("classifier.5", "classifier.7"),
}


def test_custom_cnn_points_modules_and_widths():
    torch.manual_seed(0)
    model = CustomCNN(num_classes=1000).eval()
    ex = FeatureExtractor(model, LAYERS, extract_pre_and_post=True)
    assert list(ex.return_nodes) == [f"{l}_{s}" for l in LAYERS for s in ("pre", "post")]
    mods = dict(model.named_modules())
    for layer, (pre, post) in CUSTOM_PATHS.items():
        assert ex.layer_mapping[f"{layer}_pre"] == pre
        assert ex.layer_mapping[f"{layer}_post"] == post
        assert isinstance(mods[pre], (nn.Conv2d, nn.Linear))
        assert isinstance(mods[post], nn.ReLU)
        bn = mods[pre.rsplit(".", 1)[0] + "." + str(int(pre.rsplit(".", 1)[1]) + 1)]
        assert isinstance(bn, (nn.BatchNorm2d, nn.BatchNorm1d))  # genuine pre-BN point
    with torch.no_grad():
        feats = ex(torch.randn(2, 3, 224, 224))
    widths = {k: v[0].numel() for k, v in feats.items()}
    for layer, d in WIDTHS.items():
        assert widths[f"{layer}_pre"] == d and widths[f"{layer}_post"] == d, (layer, widths)
    assert sum(widths.values()) == 1316544
    # pre-BN and post-ReLU points hold different values on CustomCNN
    for layer in LAYERS:
        assert not torch.equal(feats[f"{layer}_pre"], feats[f"{layer}_post"])
        assert float(feats[f"{layer}_post"].min()) >= 0.0


def test_torchvision_alexnet_pre_equals_post():
    torch.manual_seed(0)
    model = AlexNetModule(1000).eval()
    ex = FeatureExtractor(model, LAYERS, extract_pre_and_post=True)
    mods = dict(model.named_modules())
    for layer in LAYERS:
        pre, post = ex.layer_mapping[f"{layer}_pre"], ex.layer_mapping[f"{layer}_post"]
        assert isinstance(mods[pre], (nn.Conv2d, nn.Linear))
        assert isinstance(mods[post], nn.ReLU) and mods[post].inplace
    with torch.no_grad():
        feats = ex(torch.randn(2, 3, 224, 224))
    for layer in LAYERS:
        a, b = feats[f"{layer}_pre"], feats[f"{layer}_post"]
        assert torch.equal(a, b), layer  # the in-place ReLU mutated the stored Conv output
        assert float(a.min()) >= 0.0
    assert feats["conv1_pre"][0].numel() == 64 * 55 * 55 and feats["fc2_pre"][0].numel() == 4096
