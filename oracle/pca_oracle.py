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


# --------------------------------------------------------------------------------------
# batched PCA for the coarse-grained PCA labels
# --------------------------------------------------------------------------------------
def batched_pca(X: np.ndarray, n_components: int, batch_size: int = 10000):
    """Restates scripts/coarsegrain/compute_eigenvectors.py:23-44 line by line: float32
    mean (numpy's own), fp64 covariance summed over row batches of the centred rows,
    / (n - 1), eigh, top components by descending eigenvalue, total variance."""
    n, p = X.shape
    mean = X.mean(axis=0)
    cov = np.zeros((p, p), dtype=np.float64)
    for i in range(0, n, batch_size):
        batch = X[i:i + batch_size].astype(np.float64) - mean
        cov += batch.T @ batch
    cov /= (n - 1)
    vals, vecs = np.linalg.eigh(cov)
    idx = np.argsort(vals)[::-1][:n_components]
    total_var = vals.sum()
    return vecs[:, idx], vals[idx], mean, total_var, cov


def col_sum_sequential(X: np.ndarray) -> np.ndarray:
    """float32 column sums with rows added in row order (what X.sum(axis=0) does for a
    C-order float32 array, and what vr_col_sum_f32 restates)."""
    s = np.zeros(X.shape[1], dtype=np.float32)
    for r in np.asarray(X, dtype=np.float32):
        s = s + r
    return s
