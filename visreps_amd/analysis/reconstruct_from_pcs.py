"""Rank-k PCA reconstruction of activations (reference: visreps/analysis/
reconstruct_from_pcs.py:7-31).

The reference fits sklearn PCA(n_components=min(k, D)) on the (n, D) flattened
activations and returns inverse_transform(fit_transform(X)) = mean + P_k (X - mean), P_k
the projection onto the top-k principal axes, cast back to the input type and device.
Here the same projection is computed on the device in fp64: the top-k eigenvectors of
the smaller of the two centred Grams (n x n when n <= D, else D x D) give
  n <= D:  rec = mean + U_k U_k^T Xc          (U_k: top-k eigenvectors of Xc Xc^T)
  n >  D:  rec = mean + Xc V_k V_k^T          (V_k: top-k eigenvectors of Xc^T Xc)
which is the same subspace sklearn's SVD returns (up to ties in the spectrum). sklearn's
own solver choice ('auto' picks a randomized SVD for large inputs) makes its result
run-dependent at the 1e-6 level; the exact projection is what it approximates.
"""
from __future__ import annotations

from typing import Dict, Union

import numpy as np
import torch

Array = Union[torch.Tensor, np.ndarray]

__all__ = ["reconstruct_from_pcs"]


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("visreps_amd reconstruct_from_pcs needs a HIP (MI355X) device")
    return torch.device("cuda", torch.cuda.current_device())


def _project(flat: torch.Tensor, k: int) -> torch.Tensor:
    """mean + rank-k projection of the centred rows of flat (fp64, on its device)."""
    n, d = flat.shape
    if k > min(n, d):  # sklearn: n_components must be <= min(n_samples, n_features)
        raise ValueError(f"n_components={k} must be between 0 and min(n_samples, n_features)="
                         f"{min(n, d)} with svd_solver='full'")
    mean = flat.mean(dim=0)
    xc = flat - mean
    if k == 0:
        return mean.expand(n, d).clone()
    if n <= d:
        _, U = torch.linalg.eigh(xc @ xc.T)  # ascending eigenvalues
        Uk = U[:, n - k:]
        return mean + Uk @ (Uk.T @ xc)
    _, V = torch.linalg.eigh(xc.T @ xc)
    Vk = V[:, d - k:]
    return mean + (xc @ Vk) @ Vk.T


def reconstruct_from_pcs(acts: Dict[str, Array], k: int) -> Dict[str, Array]:
    """{name: activations reconstructed from their top-k PCs}, each with its input's
    type, dtype and device (numpy in -> numpy out)."""
    out: Dict[str, Array] = {}
    for name, x in acts.items():
        if isinstance(x, torch.Tensor):
            if x.ndim < 2:
                raise ValueError(f"{name}: need ≥2-D tensor")
            dev = x.device if x.is_cuda else _device()
            flat = x.detach().reshape(x.shape[0], -1).to(dev, torch.float64)
            rec = _project(flat, min(int(k), flat.shape[1]))
            out[name] = rec.reshape(x.shape).to(device=x.device, dtype=x.dtype)
        elif isinstance(x, np.ndarray):
            if x.ndim < 2:
                raise ValueError(f"{name}: need ≥2-D array")
            flat = torch.from_numpy(np.ascontiguousarray(x.reshape(x.shape[0], -1), dtype=np.float64))
            rec = _project(flat.to(_device()), min(int(k), flat.shape[1]))
            out[name] = rec.cpu().numpy().reshape(x.shape).astype(x.dtype, copy=False)
        else:
            raise TypeError(f"{name}: expect torch.Tensor or np.ndarray")
    return out
