"""Phase-1 sparse random projection (SRP) of layer activations.

Mirrors visreps/analysis/sparse_random_projection.py:
  * get_srp_transformer(D, k, density, seed, cache_dir) builds sklearn's
    SparseRandomProjection(n_components=k, density=density or 'auto', random_state=seed)
    fitted on one zero row (:49-81) and caches it per (D, k, density, seed) (:83-150);
    a cached entry that fails validation (:10-47) or cannot be read is refitted.
  * The product itself (torch.sparse.mm(P, flat.t()).t(), visreps/models/utils.py:297-336)
    is SparseProjector -> vr_srp_csr_f32 (HIP CSR x dense kernel, visreps_amd/csrc/srp.hip).

Differences, both deliberate:
  * The cache is an .npz of the CSR arrays (loaded with allow_pickle=False) instead of a
    joblib pickle; the file name keeps the reference pattern with a .npz suffix.
  * The returned object is an SRPComponents record carrying the same attributes the
    reference reads (components_, n_components, density_, random_state) rather than the
    sklearn estimator. With seed=None (the reference's default) the matrix is random per
    fit, exactly as in the reference; the cache is what makes a run repeatable.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import scipy.sparse as sp
import torch

from .. import _lib
from ..utils import rprint

__all__ = ["SRPComponents", "get_srp_transformer", "SparseProjector", "srp_cache_path"]


@dataclass
class SRPComponents:
    components_: sp.csr_matrix  # (k, D) float32, values +-sqrt(1/density)/sqrt(k)
    n_components: int
    density_: float
    random_state: Optional[int]

    def transform(self, X: np.ndarray) -> np.ndarray:
        """Host product X @ components_.T (for inspection; the GPU path is SparseProjector)."""
        return np.asarray(self.components_ @ np.asarray(X, dtype=np.float32).T).T


def srp_cache_path(cache_dir: str, D: int, k: int, density: Optional[float], seed: Optional[int]) -> str:
    density_str = f"{density:.4f}" if density is not None else "auto"
    return os.path.join(cache_dir, f"srp_D{D}_k{k}_density{density_str}_seed{seed}.npz")


def _validate(t: SRPComponents, k: int, density: Optional[float], seed: Optional[int]) -> bool:
    """sparse_random_projection.py:10-47."""
    if t.n_components != k:
        rprint(f"Cached transformer k mismatch (Loaded: {t.n_components}, Requested: {k}).", style="warning")
        return False
    if t.density_ is None or not np.isfinite(t.density_):
        rprint("Cached transformer seems invalid (no density_ attribute after fit).", style="warning")
        return False
    if density is not None and not np.isclose(t.density_, density):
        rprint(f"Cached transformer density mismatch (Loaded: {t.density_:.4f}, Requested: {density:.4f}).",
               style="warning")
        return False
    if t.random_state != seed:
        rprint(f"Cached transformer seed mismatch (Loaded: {t.random_state}, Requested: {seed}).", style="warning")
        return False
    return True


def _fit(D: int, k: int, density: Optional[float], seed: Optional[int]) -> Optional[SRPComponents]:
    """sparse_random_projection.py:49-81 (sklearn is the construction, as in the reference)."""
    from sklearn.random_projection import SparseRandomProjection

    rprint(f"🔧 Fitting SRP (D={D}→k={k})", style="info")
    try:
        t = SparseRandomProjection(n_components=k, density=density if density is not None else "auto",
                                   random_state=seed)
        t.fit(np.zeros((1, D), dtype=np.float32))
    except Exception as e:  # noqa: BLE001  (reference reports and returns None)
        rprint(f"Failed to fit SRP transformer: {e}", style="error")
        return None
    return SRPComponents(sp.csr_matrix(t.components_, dtype=np.float32), int(t.n_components),
                         float(t.density_), seed)


def _save(path: str, t: SRPComponents) -> None:
    c = t.components_
    tmp = path + ".tmp.npz"
    np.savez(tmp, indptr=c.indptr.astype(np.int64), indices=c.indices.astype(np.int32),
             data=c.data.astype(np.float32), shape=np.asarray(c.shape, np.int64),
             n_components=np.int64(t.n_components), density=np.float64(t.density_),
             seed=np.int64(-1 if t.random_state is None else t.random_state))
    os.replace(tmp, path)


def _load(path: str) -> SRPComponents:
    with np.load(path, allow_pickle=False) as z:
        shape = tuple(int(v) for v in z["shape"])
        comp = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=shape)
        seed = int(z["seed"])
        return SRPComponents(comp, int(z["n_components"]), float(z["density"]), None if seed < 0 else seed)


def get_srp_transformer(D: int, k: int, density: Optional[float], seed: Optional[int],
                        cache_dir: str) -> Optional[SRPComponents]:
    """sparse_random_projection.py:83-150: cached or freshly fitted SRP for (D, k)."""
    if k <= 0 or D <= 0:
        rprint(f"Invalid dimensions D={D}, k={k}. Cannot create transformer.", style="error")
        return None
    os.makedirs(cache_dir, exist_ok=True)
    path = srp_cache_path(cache_dir, D, k, density, seed)
    t = None
    if os.path.exists(path):
        try:
            loaded = _load(path)
            if _validate(loaded, k, density, seed):
                t = loaded
            else:
                rprint("Cached transformer validation failed. Will refit.", style="warning")
        except Exception as e:  # noqa: BLE001  (corrupt cache: refit, :121-141)
            rprint(f"Error loading cached transformer: {e}. Will refit.", style="warning")
            try:
                os.remove(path)
            except OSError as err:
                rprint(f"Could not remove problematic cache file: {err}", style="warning")
    if t is None:
        t = _fit(D, k, density, seed)
        if t is not None:
            try:
                _save(path, t)
            except Exception as e:  # noqa: BLE001
                rprint(f"Failed to cache transformer: {e}", style="warning")
    return t


class SparseProjector:
    """Device-resident CSR projection: __call__(flat (B, D) fp32 on device) -> (B, k) fp32.

    The HIP kernel accumulates each output in fp32 in CSR order (torch.sparse.mm's order is
    an implementation detail of torch; results agree to fp32 rounding)."""

    def __init__(self, transformer, device: torch.device):
        comp = transformer.components_ if hasattr(transformer, "components_") else transformer
        comp = sp.csr_matrix(comp)
        comp.sort_indices()
        if comp.nnz >= 2**31:
            raise ValueError("SparseProjector: more than 2^31 nonzeros")
        self.k, self.D = (int(v) for v in comp.shape)
        self.device = torch.device(device)
        self.indptr = torch.from_numpy(comp.indptr.astype(np.int32)).to(self.device)
        self.indices = torch.from_numpy(comp.indices.astype(np.int32)).to(self.device)
        self.values = torch.from_numpy(comp.data.astype(np.float32)).to(self.device)

    def __call__(self, flat: torch.Tensor) -> torch.Tensor:
        if flat.dim() != 2 or flat.size(1) != self.D:
            raise ValueError(f"SparseProjector: expected (B, {self.D}), got {tuple(flat.shape)}")
        if flat.device != self.device:
            raise ValueError(f"SparseProjector: input on {flat.device}, projector on {self.device}")
        x = flat if flat.dtype == torch.float32 else flat.float()
        if x.stride(1) != 1:
            x = x.contiguous()
        B = x.size(0)
        out = torch.empty((B, self.k), dtype=torch.float32, device=self.device)
        if B == 0:
            return out
        L = _lib.lib()
        nbytes = L.vr_srp_workspace(B, self.D)
        ws = _lib.workspace.get(self.device, nbytes, "srp")
        rc = L.vr_srp_csr_f32(self.indptr.data_ptr(), self.indices.data_ptr(), self.values.data_ptr(),
                              self.k, self.D, x.data_ptr(), B, x.stride(0), out.data_ptr(), self.k,
                              ws.data_ptr(), ws.numel(), _lib.stream_of(self.device))
        _lib.check(rc, "vr_srp_csr_f32")
        return out
