"""Feature dumps for downstream RSA (reference: scripts/extract_representations/).

Same contract as the reference scripts: batch forward -> extract_fn (AlexNet fc2 /
ViT CLS token) -> row L2 normalisation -> concatenation in loader order -> one
`features_{model}.npz` holding `{model}_features` (N, D) float32 and `image_names`.

  extract_features   utils.py:31-69 (names from dataset.samples[i][2], mismatch -> ValueError)
  save_features      utils.py:72-78 (datasets/obj_cls/{dataset}/features_{model}.npz)
  alexnet_fc2        alexnet_representations.py:25-27,43-45 (classifier[:6], F.normalize)
  vit_cls            vit_representations.py:25,33-35 (forward_features(x)[:, 0], F.normalize);
                     the script's default model, ViT-L/16 (1024-d CLS), is
                     models.standard_model.vit_large_patch16_224
  clip_image         clip_representations.py:26-38 (encode_image / its norm; CLIP ViT-L/14)
  dino_cls           dino_representations.py:24-38 (forward_features(x)[:, 0], F.normalize)
                     (models/foundation.py; loaders' bicubic preprocessing:
                     dataloaders/obj_cls.clip_transform / dino_transform)

Pretrained weights need a download the reference makes (torchvision / timm / clip); here
the models are the repo's own random-initialised AlexNet / ViT-B/16 / ViT-L/16 unless a
local checkpoint is supplied (models/standard_model.py). The rows are written on the device
in one (N, D) buffer, so a caller can hand them straight to the RDM kernels without the
host round trip of the reference.
"""
from __future__ import annotations

import os
from typing import Callable, Iterable, List, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["extract_features", "save_features", "load_features", "alexnet_fc2", "vit_cls",
           "clip_image", "dino_cls"]


def alexnet_fc2(model: nn.Module) -> Tuple[nn.Module, Callable]:
    """Truncate an AlexNet to its second fully-connected block (classifier[:6]) and return
    (model, extract_fn) with extract_fn = L2-normalised fc2 output."""
    model.classifier = nn.Sequential(*list(model.classifier.children())[:6])

    def extract_fn(m, x):
        return F.normalize(m(x), p=2, dim=-1)

    return model, extract_fn


def vit_cls(model: nn.Module) -> Tuple[nn.Module, Callable]:
    """(model, extract_fn) with extract_fn = L2-normalised CLS token of forward_features."""

    def extract_fn(m, x):
        return F.normalize(m.forward_features(x)[:, 0, :], p=2, dim=-1)

    return model, extract_fn


def clip_image(model: nn.Module) -> Tuple[nn.Module, Callable]:
    """(model, extract_fn) with extract_fn = encode_image(x) / ||encode_image(x)||
    (clip_representations.py:37-39: features / features.norm(dim=-1, keepdim=True))."""

    def extract_fn(m, x):
        f = m.encode_image(x)
        return f / f.norm(dim=-1, keepdim=True)

    return model, extract_fn


def dino_cls(model: nn.Module) -> Tuple[nn.Module, Callable]:
    """(model, extract_fn) with extract_fn = L2-normalised CLS of forward_features
    (dino_representations.py:35-37)."""

    def extract_fn(m, x):
        return F.normalize(m.forward_features(x)[:, 0, :], p=2, dim=-1)

    return model, extract_fn


@torch.no_grad()
def extract_features(model: nn.Module, loader_list: Sequence[Iterable], extract_fn: Callable,
                     device: torch.device, desc: str = "Extracting features",
                     as_numpy: bool = True):
    """Features of every loader's images in loader order, plus image names.

    Returns (features (N, D), image_names). Names come from `dataset.samples[i][2]` when
    the dataset has `samples`; a name/feature count mismatch raises ValueError, as the
    reference does. With as_numpy=False the features stay on the device."""
    chunks: List[torch.Tensor] = []
    names: List[str] = []
    model.eval()
    for loader in loader_list:
        dataset = getattr(loader, "dataset", None)
        sample_idx = 0
        for batch in loader:
            images = batch[0] if isinstance(batch, (tuple, list)) else batch
            images = images.to(device, non_blocking=True)
            feats = extract_fn(model, images)
            for _ in range(images.shape[0]):
                if dataset is not None and hasattr(dataset, "samples"):
                    names.append(dataset.samples[sample_idx][2])
                sample_idx += 1
            chunks.append(feats)
    if not chunks:
        raise ValueError("no batches to extract")
    feats = torch.cat(chunks, dim=0)
    if len(names) != feats.shape[0]:
        raise ValueError(f"Mismatch: {len(names)} names vs {feats.shape[0]} features")
    return (feats.cpu().numpy() if as_numpy else feats), names


def save_features(features, image_names, dataset: str, model_name: str,
                  root: str = "datasets") -> str:
    """np.savez_compressed(root/obj_cls/{dataset}/features_{model_name}.npz) with keys
    `{model_name}_features` and `image_names`; returns the path."""
    if isinstance(features, torch.Tensor):
        features = features.detach().cpu().numpy()
    out_dir = os.path.join(root, "obj_cls", dataset)
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, f"features_{model_name}.npz")
    np.savez_compressed(path, **{f"{model_name}_features": features, "image_names": image_names})
    print(f"Saved {tuple(features.shape)} to {path}")
    return path


def load_features(path: str, model_name: str):
    """Inverse of save_features (no pickle: names are stored as a unicode array)."""
    with np.load(path, allow_pickle=False) as z:
        return z[f"{model_name}_features"], [str(s) for s in z["image_names"]]
