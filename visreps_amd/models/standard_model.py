"""torchvision-architecture models used with load_model_from=torchvision
(reference: visreps/models/standard_model.py AlexNet 5-20, ViTBase 82-97).

torchvision is not installed in this image, so both networks are rebuilt here with
torchvision's exact module names and shapes (a torchvision state_dict loads with
strict=True). Pretrained weights cannot be downloaded (no network): `pretrained_dataset`
other than "none" requires a local state_dict file via VISREPS_AMD_WEIGHTS_<NAME>.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import torch
import torch.nn as nn

__all__ = ["AlexNetModule", "VisionTransformer", "AlexNet", "ViTBase"]


class AlexNetModule(nn.Module):
    """torchvision.models.AlexNet layout (features / avgpool / classifier)."""

    def __init__(self, num_classes: int = 1000, dropout: float = 0.5):
        super().__init__()
        spec = [(64, 11, 4, 2, True), (192, 5, 1, 2, True), (384, 3, 1, 1, False),
                (256, 3, 1, 1, False), (256, 3, 1, 1, True)]
        layers, c_in = [], 3
        for c_out, k, s, p, pool in spec:
            layers += [nn.Conv2d(c_in, c_out, kernel_size=k, stride=s, padding=p), nn.ReLU(inplace=True)]
            if pool:
                layers.append(nn.MaxPool2d(kernel_size=3, stride=2))
            c_in = c_out
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d((6, 6))
        self.classifier = nn.Sequential(
            nn.Dropout(p=dropout), nn.Linear(256 * 6 * 6, 4096), nn.ReLU(inplace=True),
            nn.Dropout(p=dropout), nn.Linear(4096, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, num_classes),
        )

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1))


class _MLPBlock(nn.Sequential):
    def __init__(self, dim: int, mlp_dim: int, dropout: float):
        super().__init__(nn.Linear(dim, mlp_dim), nn.GELU(), nn.Dropout(dropout),
                         nn.Linear(mlp_dim, dim), nn.Dropout(dropout))
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.normal_(m.bias, std=1e-6)


class _EncoderBlock(nn.Module):
    def __init__(self, heads: int, dim: int, mlp_dim: int, dropout: float = 0.0,
                 attention_dropout: float = 0.0):
        super().__init__()
        self.ln_1 = nn.LayerNorm(dim, eps=1e-6)
        self.self_attention = nn.MultiheadAttention(dim, heads, dropout=attention_dropout,
                                                    batch_first=True)
        self.dropout = nn.Dropout(dropout)
        self.ln_2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _MLPBlock(dim, mlp_dim, dropout)

    def forward(self, inp):
        x = self.ln_1(inp)
        x, _ = self.self_attention(x, x, x, need_weights=False)
        x = self.dropout(x) + inp
        return x + self.mlp(self.ln_2(x))


class _Encoder(nn.Module):
    def __init__(self, seq_len: int, layers: int, heads: int, dim: int, mlp_dim: int):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq_len, dim).normal_(std=0.02))
        self.dropout = nn.Dropout(0.0)
        self.layers = nn.Sequential(OrderedDict(
            (f"encoder_layer_{i}", _EncoderBlock(heads, dim, mlp_dim)) for i in range(layers)))
        self.ln = nn.LayerNorm(dim, eps=1e-6)

    def forward(self, x):
        return self.ln(self.layers(self.dropout(x + self.pos_embedding)))


class VisionTransformer(nn.Module):
    """torchvision.models.VisionTransformer layout (conv_proj, class_token, encoder, heads)."""

    def __init__(self, image_size=224, patch_size=16, num_layers=12, num_heads=12,
                 hidden_dim=768, mlp_dim=3072, num_classes=1000):
        super().__init__()
        self.image_size, self.patch_size, self.hidden_dim = image_size, patch_size, hidden_dim
        self.conv_proj = nn.Conv2d(3, hidden_dim, kernel_size=patch_size, stride=patch_size)
        seq_len = (image_size // patch_size) ** 2 + 1
        self.class_token = nn.Parameter(torch.zeros(1, 1, hidden_dim))
        self.encoder = _Encoder(seq_len, num_layers, num_heads, hidden_dim, mlp_dim)
        self.heads = nn.Sequential(OrderedDict(head=nn.Linear(hidden_dim, num_classes)))
        fan_in = 3 * patch_size * patch_size
        nn.init.trunc_normal_(self.conv_proj.weight, std=math.sqrt(1 / fan_in))
        nn.init.zeros_(self.conv_proj.bias)
        nn.init.zeros_(self.heads.head.weight)
        nn.init.zeros_(self.heads.head.bias)

    def forward_features(self, x):
        """Token sequence after the encoder (B, 1 + patches, hidden); [:, 0] is the CLS
        token (the timm forward_features contract used by vit_representations.py:34)."""
        n = x.shape[0]
        x = self.conv_proj(x)
        x = x.reshape(n, self.hidden_dim, -1).permute(0, 2, 1)
        x = torch.cat([self.class_token.expand(n, -1, -1), x], dim=1)
        return self.encoder(x)

    def forward(self, x):
        return self.heads(self.forward_features(x)[:, 0])


def _maybe_load(model: nn.Module, name: str, pretrained_dataset: str) -> nn.Module:
    if pretrained_dataset == "none":
        return model
    if pretrained_dataset != "imagenet1k":
        raise ValueError(f"Invalid pretrained dataset: {pretrained_dataset}")
    path = os.environ.get(f"VISREPS_AMD_WEIGHTS_{name.upper()}")
    if not path or not os.path.exists(path):
        raise FileNotFoundError(
            f"{name} imagenet1k weights are not downloadable here; point "
            f"VISREPS_AMD_WEIGHTS_{name.upper()} at a torchvision state_dict file")
    state = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(state, strict=True)
    return model


def AlexNet(pretrained_dataset="imagenet1k", num_classes=1000):
    """standard_model.py:5-20 (torchvision AlexNet, optional head replacement)."""
    model = _maybe_load(AlexNetModule(1000), "alexnet", pretrained_dataset)
    if num_classes != 1000 and num_classes is not None:
        model.classifier[-1] = nn.Linear(4096, num_classes)
        nn.init.xavier_uniform_(model.classifier[-1].weight)
        nn.init.zeros_(model.classifier[-1].bias)
    return model


def ViTBase(pretrained_dataset="imagenet1k", num_classes=1000):
    """standard_model.py:82-97 (torchvision vit_b_16, optional head replacement)."""
    model = _maybe_load(VisionTransformer(), "vit_b_16", pretrained_dataset)
    if num_classes != 1000 and num_classes is not None:
        model.heads.head = nn.Linear(768, num_classes)
        nn.init.xavier_uniform_(model.heads.head.weight)
        nn.init.zeros_(model.heads.head.bias)
    return model


def vit_large_patch16_224(pretrained_dataset: str = "none"):
    """ViT-L/16 at 224 px: the feature-dump default of the reference's
    scripts/extract_representations/vit_representations.py:19,25
    (timm.create_model("vit_large_patch16_224", pretrained=True, num_classes=0)). timm's
    VisionTransformer has this module's semantics -- pre-norm blocks (LayerNorm eps 1e-6,
    qkv bias, GELU MLP), a learned class token and position embedding added to all 197
    tokens, and the final LayerNorm inside forward_features -- at width 1024, 24 blocks, 16
    heads, MLP 4096, so forward_features(x)[:, 0] is the 1024-d CLS row the dump
    normalises. The pretrained weights need timm's download: random init unless
    VISREPS_AMD_WEIGHTS_VIT_L_16 names a state_dict in this layout."""
    model = VisionTransformer(image_size=224, patch_size=16, num_layers=24, num_heads=16, hidden_dim=1024,
                              mlp_dim=4096, num_classes=1000)
    return _maybe_load(model, "vit_l_16", pretrained_dataset)
