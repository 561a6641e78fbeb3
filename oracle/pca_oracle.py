"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference's reconstruct_from_pcs (visreps/analysis/
reconstruct_from_pcs.py:7-31: sklearn PCA(n_components=min(k, D)).fit_transform then
inverse_transform on the (n, D) flattened activations), used only by tests/ as the
checker. With the full SVD Xc = U S V^T of the centred rows the reconstruction is
mean + U_k S_k V_k^T; pinned against sklearn.decomposition.PCA(svd_solver="full") in
tests/test_pca.py (sklearn is the library the reference calls).
"""
from __future__ import annotations

import numpy as np


def reconstruct_from_pcs(x: np.ndarray, k: int) -> np.ndarray:
    x = np.asarray(x)
    flat = x.reshape(x.shape[0], -1).astype(np.float64)
    k = min(int(k), flat.shape[1])
    if k > min(flat.shape):
        raise ValueError("n_components must be <= min(n_samples, n_features)")
    mean = flat.mean(0)
    U, S, Vt = np.linalg.svd(flat - mean, full_matrices=False)
    rec = mean + (U[:, :k] * S[:k]) @ Vt[:k]
    return rec.reshape(x.shape)
