"""Image preprocessing of the eval loaders (reference: visreps/dataloaders/obj_cls.py:18-45)
and the file-backed stimulus loader (neural.py:463-523).

get_transform(ds_stats, data_augment, image_size, preprocess) returns a DeviceTransform:
Resize(256 | 64, bilinear) -> CenterCrop(image_size | 64) -> ToTensor -> Normalize on the
MI355X (vr_transform_u8, csrc/transform.hip), bit-identical to torchvision on PIL images
(Pillow's antialiased fixed-point resample). It takes PIL images / HWC uint8 arrays one at
a time (`t(img)` -> (3, crop, crop)) or as a batch (`t.batch(imgs)` -> (B, 3, crop, crop));
same-size images of a batch go through one kernel launch.

ImageLoader mirrors DataLoader(_StimuliDataset(stimuli, transform), shuffle=False):
sorted keys, each stimulus a path (opened and converted to RGB), an HWC uint8 array or a
PIL image; yields (images on the device, keys).
"""
from __future__ import annotations

from typing import Any, Dict, Iterator, List, Sequence, Tuple

import numpy as np
import torch

from .._lib import check, lib, stream_of, workspace

__all__ = ["DS_MEAN", "DS_STD", "get_transform", "clip_transform", "dino_transform",
           "DeviceTransform", "ImageLoader"]

DS_MEAN = {"tiny-imagenet": [0.480, 0.448, 0.398], "imgnet": [0.485, 0.456, 0.406]}
DS_STD = {"tiny-imagenet": [0.272, 0.265, 0.274], "imgnet": [0.229, 0.224, 0.225]}


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("visreps_amd image transform needs a HIP (MI355X) device")
    return torch.device("cuda", torch.cuda.current_device())


def _as_rgb_u8(img) -> np.ndarray:
    """HWC uint8 RGB array of a PIL image (converted to RGB) or an array."""
    if isinstance(img, np.ndarray):
        a = img.astype(np.uint8, copy=False)
        if a.ndim != 3 or a.shape[2] != 3:
            raise ValueError(f"expected an H x W x 3 uint8 array, got {a.shape}")
        return np.ascontiguousarray(a)
    from PIL import Image

    if isinstance(img, Image.Image):
        return np.asarray(img if img.mode == "RGB" else img.convert("RGB"), dtype=np.uint8)
    raise TypeError(f"Unsupported image type {type(img)}")


class DeviceTransform:
    """Resize(resize) -> CenterCrop(crop) -> ToTensor -> Normalize(mean, std) on the device;
    with preprocess=False only ToTensor (transforms.ToTensor(): HWC uint8 -> CHW / 255)."""

    FILTERS = {"bilinear": 0, "bicubic": 1}

    def __init__(self, resize: int, crop: int, mean: Sequence[float], std: Sequence[float],
                 preprocess: bool = True, interpolation: str = "bilinear"):
        self.resize, self.crop, self.preprocess = int(resize), int(crop), bool(preprocess)
        if interpolation not in self.FILTERS:
            raise ValueError(f"interpolation {interpolation!r}: bilinear or bicubic")
        self.interpolation = interpolation
        self.mean = np.asarray(mean, dtype=np.float32)
        self.std = np.asarray(std, dtype=np.float32)

    def __repr__(self):
        return (f"DeviceTransform(Resize({self.resize}, {self.interpolation}), CenterCrop({self.crop}), "
                f"ToTensor, Normalize({self.mean.tolist()}, {self.std.tolist()}))")

    def __call__(self, img) -> torch.Tensor:
        return self.batch([img])[0]

    def _run(self, arrs: List[np.ndarray], dev: torch.device) -> torch.Tensor:
        B = len(arrs)
        H, W, _ = arrs[0].shape
        src = torch.from_numpy(np.stack(arrs)).to(dev, non_blocking=True)
        if not self.preprocess:  # transforms.ToTensor() only: one fp32 division per value
            return src.permute(0, 3, 1, 2).float().div(255)
        out = torch.empty((B, 3, self.crop, self.crop), dtype=torch.float32, device=dev)
        L = lib()
        f = self.FILTERS[self.interpolation]
        ws = workspace.get(dev, L.vr_transform_workspace(B, H, W, self.resize, self.crop, f), "transform")
        with torch.cuda.device(dev):
            check(L.vr_transform_u8(src.data_ptr(), B, H, W, self.resize, self.crop, f,
                                    self.mean.ctypes.data, self.std.ctypes.data, out.data_ptr(),
                                    ws.data_ptr(), ws.numel(), stream_of(dev)), "vr_transform_u8")
        return out

    def batch(self, images: Sequence[Any], device=None) -> torch.Tensor:
        """(B, 3, crop, crop) fp32 on the device; images of one size share a launch."""
        dev = torch.device(device) if device is not None else _device()
        arrs = [_as_rgb_u8(im) for im in images]
        if not arrs:
            return torch.empty((0, 3, self.crop, self.crop), dtype=torch.float32, device=dev)
        groups: Dict[Tuple[int, int], List[int]] = {}
        for i, a in enumerate(arrs):
            groups.setdefault(a.shape[:2], []).append(i)
        if len(groups) == 1:
            return self._run(arrs, dev)
        if not self.preprocess:
            raise ValueError("ToTensor-only batches need images of one size")
        out = torch.empty((len(arrs), 3, self.crop, self.crop), dtype=torch.float32, device=dev)
        for rows in groups.values():
            out[torch.as_tensor(rows, device=dev)] = self._run([arrs[i] for i in rows], dev)
        return out


def get_transform(ds_stats: str = "imgnet", data_augment: bool = False, image_size: int = 224,
                  preprocess: bool = True) -> DeviceTransform:
    """obj_cls.py:27-45. data_augment adds training-time random flips / rotations, which the
    eval path never uses (training is out of scope): refused."""
    if data_augment:
        raise NotImplementedError("data_augment is training-only (out of scope for the eval build)")
    if ds_stats not in DS_MEAN:
        raise KeyError(ds_stats)
    resize, crop = (64, 64) if ds_stats == "tiny-imagenet" else (256, image_size)
    return DeviceTransform(resize, crop, DS_MEAN[ds_stats], DS_STD[ds_stats], preprocess)


def clip_transform(n_px: int = 224) -> DeviceTransform:
    """clip._transform(n_px) (clip.load's preprocess, clip_representations.py:27):
    Resize(n_px, BICUBIC), CenterCrop(n_px), RGB, ToTensor, Normalize(CLIP stats)."""
    from ..models.foundation import CLIP_MEAN, CLIP_STD

    return DeviceTransform(n_px, n_px, CLIP_MEAN, CLIP_STD, interpolation="bicubic")


def dino_transform(img_size: int = 224, crop_pct: float = 1.0) -> DeviceTransform:
    """timm create_transform(**resolve_model_data_config(dinov3), is_training=False)
    (dino_representations.py:31-32): Resize(int(img_size / crop_pct), BICUBIC),
    CenterCrop(img_size), ImageNet stats. The data config is assumed (timm is absent)."""
    return DeviceTransform(int(img_size / crop_pct), img_size, DS_MEAN["imgnet"], DS_STD["imgnet"],
                           interpolation="bicubic")


class ImageLoader:
    """Batches of (images (B, 3, crop, crop) on the device, keys) in sorted key order."""

    def __init__(self, stimuli: Dict[str, Any], transform: DeviceTransform | None, batch: int):
        self.stimuli = stimuli
        self.keys = sorted(stimuli.keys())
        self.tr = transform or DeviceTransform(0, 0, [0, 0, 0], [1, 1, 1], preprocess=False)
        self.batch = max(1, int(batch))

    def __len__(self) -> int:
        return (len(self.keys) + self.batch - 1) // self.batch

    @staticmethod
    def _load(data_or_path, key):
        if isinstance(data_or_path, str):
            from PIL import Image

            with Image.open(data_or_path) as im:
                return im.convert("RGB")
        if isinstance(data_or_path, np.ndarray):
            return data_or_path.astype(np.uint8)
        from PIL import Image

        if isinstance(data_or_path, Image.Image):
            return data_or_path
        raise TypeError(f"Unsupported data type {type(data_or_path)} for key {key}")

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, List[str]]]:
        for i in range(0, len(self.keys), self.batch):
            keys = self.keys[i:i + self.batch]
            yield self.tr.batch([self._load(self.stimuli[k], k) for k in keys]), keys
