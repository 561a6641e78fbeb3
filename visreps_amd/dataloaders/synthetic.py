"""Deterministic synthetic stimuli and neural responses (no datasets are reachable).

SURVEY.md §8(d): images of NSD shape (3 x 224 x 224, ImageNet-normalised range) and
region responses Y_r = Z B_r + 3 E_r over a latent Z shared with the images, so model
RDMs and neural RDMs correlate. Every block of `BLOCK` stimuli is generated from its own
seed, so any sharding of the stimulus axis (one GPU or eight) yields bit-identical data.
"""
from __future__ import annotations

from typing import Dict, Sequence

import torch
import torch.nn.functional as F

BLOCK = 64
LATENT_HW = 7  # latent = 3 x 7 x 7 average-pooled image


def _gen(seed: int, device) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def make_images(rows: range, *, seed: int = 20260306, device="cuda",
                dtype=torch.float32) -> torch.Tensor:
    """Images of stimuli `rows` (a contiguous range): smooth random fields, ~N(0,1) per
    channel like ImageNet-normalised inputs."""
    out = torch.empty((len(rows), 3, 224, 224), dtype=dtype, device=device)
    r0 = rows.start
    for b0 in range(rows.start - rows.start % BLOCK, rows.stop, BLOCK):
        g = _gen(seed * 1000003 + b0 // BLOCK, device)
        coarse = torch.randn((BLOCK, 3, 28, 28), generator=g, device=device)
        img = F.interpolate(coarse, size=(224, 224), mode="bilinear", align_corners=False)
        img = img + 0.25 * torch.randn((BLOCK, 3, 224, 224), generator=g, device=device)
        lo, hi = max(b0, rows.start), min(b0 + BLOCK, rows.stop)
        out[lo - r0:hi - r0] = img[lo - b0:hi - b0].to(dtype)
    return out


def latent_of(images: torch.Tensor) -> torch.Tensor:
    """Z: the 3 x 7 x 7 average-pooled image, flattened (147 dims)."""
    return F.adaptive_avg_pool2d(images.float(), LATENT_HW).flatten(1)


def make_responses(images: torch.Tensor, rows: range, voxels: Dict[str, int], *,
                   seed: int = 20260306, noise: float = 3.0) -> Dict[str, torch.Tensor]:
    """Region responses for stimuli `rows` whose images are given: Y_r = Z B_r + noise E_r."""
    z = latent_of(images)
    dev = images.device
    out = {}
    for ri, (region, v) in enumerate(voxels.items()):
        gb = _gen(seed * 7919 + 101 * ri, dev)
        b = torch.randn((z.size(1), v), generator=gb, device=dev) / (z.size(1) ** 0.5)
        y = torch.empty((z.size(0), v), dtype=z.dtype, device=dev)
        r0 = rows.start
        for b0 in range(rows.start - rows.start % BLOCK, rows.stop, BLOCK):
            g = _gen(seed * 15485863 + 31 * ri + 7 * (b0 // BLOCK), dev)
            e = torch.randn((BLOCK, v), generator=g, device=dev)
            lo, hi = max(b0, rows.start), min(b0 + BLOCK, rows.stop)
            # one BLOCK-row GEMM per block (the rows of a partial block padded with zeros):
            # the GEMM shape, and so its summation order, does not depend on the sharding
            zb = torch.zeros((BLOCK, z.size(1)), dtype=z.dtype, device=dev)
            zb[lo - b0:hi - b0] = z[lo - r0:hi - r0]
            y[lo - r0:hi - r0] = (zb @ b)[lo - b0:hi - b0] + noise * e[lo - b0:hi - b0]
        out[region] = y.contiguous()
    return out


NSD_ROIS_4 = {"V1": 2000, "V2": 2000, "V3": 2000, "hV4": 1000}


def shard_rows(n: int, rank: int, world: int) -> range:
    """Contiguous, equal-as-possible stimulus shard of a rank."""
    per, extra = divmod(n, world)
    start = rank * per + min(rank, extra)
    return range(start, start + per + (1 if rank < extra else 0))


def shard_sizes(n: int, world: int) -> Sequence[int]:
    return [len(shard_rows(n, r, world)) for r in range(world)]
