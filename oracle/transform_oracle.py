"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference's get_transform (visreps/dataloaders/obj_cls.py:27-45)
on PIL images: torchvision Resize(size) -> Pillow Image.resize(BILINEAR) (Pillow 12,
libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc, ImagingResample
Horizontal/Vertical_8bpc), CenterCrop (torchvision F.center_crop offsets), ToTensor,
Normalize. Used only as the checker by tests/; tests/test_transform.py pins resample()
against Pillow itself on seeded images (Pillow is importable here; torchvision is not).
"""
from __future__ import annotations

import math

import numpy as np

PREC = 22  # PRECISION_BITS = 32 - 8 - 2


def _filter(kind: str, x: float) -> float:
    """Resample.c bilinear_filter / bicubic_filter (a = -0.5)."""
    x = -x if x < 0.0 else x
    if kind == "bicubic":
        a = -0.5
        if x < 1.0:
            return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
        if x < 2.0:
            return (((x - 5) * x + 8) * x - 4) * a
        return 0.0
    return 1.0 - x if x < 1.0 else 0.0


def _coeffs(in_size: int, out_size: int, kind: str = "bilinear"):
    """(bounds (out, 2) int, kk (out, ksize) int32) of Pillow's filter."""
    scale = float(np.float32(in_size) - np.float32(0.0)) / out_size
    filterscale = max(scale, 1.0)
    support = (2.0 if kind == "bicubic" else 1.0) * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        xmin = max(xmin, 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        for x in range(xmax):
            w.append(_filter(kind, (x + xmin - center + 0.5) * ss))
        ww = sum(w)  # left-to-right double sum, as the C loop
        k = [v / ww if ww != 0.0 else v for v in w]
        for x, v in enumerate(k):
            f = v * (1 << PREC)
            kk[xx, x] = int(-0.5 + f) if v < 0 else int(0.5 + f)
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _pass(a: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """One 8bpc pass along axis (1 = horizontal, 0 = vertical) of an H x W x 3 uint8 image."""
    a = np.moveaxis(a.astype(np.int64), axis, 0)
    out = np.empty((bounds.shape[0],) + a.shape[1:], np.uint8)
    for o, (lo, n) in enumerate(bounds):
        ss = np.full(a.shape[1:], 1 << (PREC - 1), np.int64)
        for i in range(n):
            ss += a[lo + i] * kk[o, i]
        out[o] = np.clip(ss >> PREC, 0, 255)
    return np.moveaxis(out, 0, axis)


def resample(img: np.ndarray, new_w: int, new_h: int, kind: str = "bilinear") -> np.ndarray:
    """Pillow Image.resize((new_w, new_h), BILINEAR | BICUBIC) of an H x W x 3 uint8 image."""
    H, W, _ = img.shape
    out = img
    if new_w != W:
        b, k = _coeffs(W, new_w, kind)
        out = _pass(out, b, k, 1)
    if new_h != H:
        b, k = _coeffs(H, new_h, kind)
        out = _pass(out, b, k, 0)
    return out


def resize_size(H: int, W: int, size: int):
    """torchvision _compute_resized_output_size for an int size: (new_h, new_w)."""
    short, long = (W, H) if W <= H else (H, W)
    new_short, new_long = size, int(size * long / short)
    return (new_long, new_short) if W <= H else (new_short, new_long)


def transform(img: np.ndarray, resize: int, crop: int, mean, std, kind: str = "bilinear") -> np.ndarray:
    """get_transform on one H x W x 3 uint8 image -> 3 x crop x crop float32."""
    H, W, _ = img.shape
    nh, nw = resize_size(H, W, resize)
    r = resample(img, nw, nh, kind)
    top = int(round((nh - crop) / 2.0))
    left = int(round((nw - crop) / 2.0))
    c = r[top:top + crop, left:left + crop]
    x = np.transpose(c, (2, 0, 1)).astype(np.float32) / np.float32(255)
    m = np.asarray(mean, np.float32)[:, None, None]
    s = np.asarray(std, np.float32)[:, None, None]
    return ((x - m) / s).astype(np.float32)
