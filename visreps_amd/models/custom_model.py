"""AlexNet-style CNNs whose checkpoints the eval path scores
(reference: visreps/models/custom_model.py: BaseCNN 6-90, TinyCustomCNN 93-137,
CustomCNN 140-185).

The module tree (features / adaptive_pool / classifier Sequentials and their indices)
is the reference's, so a reference state_dict loads unchanged and the feature-extractor
mapping conv1..conv5 / fc1..fc3 lands on the same modules. Layers are generated from a
spec table here rather than spelled out.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence, Tuple

import torch
import torch.nn as nn

# (out_channels, kernel, stride, padding, pool_after(kernel, stride) or None)
_CUSTOM_CONVS: Sequence[Tuple] = (
    (96, 11, 4, 2, (3, 2)),
    (256, 5, 1, 2, (3, 2)),
    (384, 3, 1, 1, None),
    (384, 3, 1, 1, None),
    (256, 3, 1, 1, (3, 2)),
)
_TINY_CONVS: Sequence[Tuple] = (
    (64, 5, 2, 2, (2, 2)),
    (128, 3, 1, 1, None),
    (256, 3, 1, 1, (2, 2)),
    (512, 3, 1, 1, None),
    (512, 3, 1, 1, None),
)


class BaseCNN(nn.Module):
    """Conv-BN-ReLU feature stack + FC-BN-ReLU head (custom_model.py:6-90)."""

    conv_spec: Sequence[Tuple] = ()
    pool_hw: int = 3
    hidden: int = 4096

    def __init__(self, num_classes=1000, trainable_layers=None, dropout=0.5, pooling_type="max"):
        super().__init__()
        self.num_classes = num_classes
        self.dropout = dropout
        self.pooling_type = pooling_type
        # trainable_layers (custom_model.py:36-68) only freezes parameters for training;
        # it is accepted for signature parity and has no effect on the eval path
        del trainable_layers
        self._build_architecture()
        self._initialize_weights()

    def _pool(self, kernel_size=3, stride=2):
        if self.pooling_type == "max":
            return nn.MaxPool2d(kernel_size=kernel_size, stride=stride)
        return nn.AvgPool2d(kernel_size=kernel_size, stride=stride)

    def _build_architecture(self):
        layers = []
        c_in = 3
        for c_out, k, s, p, pool in self.conv_spec:
            layers += [nn.Conv2d(c_in, c_out, kernel_size=k, stride=s, padding=p, bias=False),
                       nn.BatchNorm2d(c_out), nn.ReLU(inplace=True)]
            if pool is not None:
                layers.append(self._pool(*pool))
            c_in = c_out
        self.features = nn.Sequential(*layers)
        self.adaptive_pool = nn.AdaptiveAvgPool2d((self.pool_hw, self.pool_hw))
        flat = c_in * self.pool_hw * self.pool_hw
        n_cls = self.num_classes if self.num_classes is not None else 1000
        self.classifier = nn.Sequential(
            nn.Dropout(p=self.dropout), nn.Linear(flat, self.hidden), nn.BatchNorm1d(self.hidden),
            nn.ReLU(inplace=True), nn.Dropout(p=self.dropout), nn.Linear(self.hidden, self.hidden),
            nn.BatchNorm1d(self.hidden), nn.ReLU(inplace=True), nn.Linear(self.hidden, n_cls),
        )

    def _initialize_weights(self):
        n_cls = self.num_classes if self.num_classes is not None else 1000
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.BatchNorm1d)):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                if m.out_features == n_cls:
                    nn.init.normal_(m.weight, 0, 1.0 / math.sqrt(m.weight.size(1)))
                else:
                    nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.features(x)
        x = self.adaptive_pool(x)
        return self.classifier(torch.flatten(x, 1))


class CustomCNN(BaseCNN):
    """224x224 ImageNet model (custom_model.py:140-185)."""

    conv_spec = _CUSTOM_CONVS
    pool_hw = 3
    hidden = 4096


class TinyCustomCNN(BaseCNN):
    """64x64 Tiny-ImageNet model (custom_model.py:93-137)."""

    conv_spec = _TINY_CONVS
    pool_hw = 4
    hidden = 2048

    def __init__(self, num_classes=200, trainable_layers=None, dropout=0.3, pooling_type="max"):
        super().__init__(num_classes, trainable_layers, dropout, pooling_type)
