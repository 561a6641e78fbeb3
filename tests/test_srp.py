"""Sparse random projection (phase-1 extraction).

CPU: get_srp_transformer follows sparse_random_projection.py:83-150 (sklearn construction,
per-(D, k, density, seed) cache, refit on a mismatched or corrupt cache entry). With a
fixed seed the matrix equals sklearn's own (same pinned sklearn 1.7.2). The reference's
default seed=None is random per fit, so only seeded matrices are parity-pinned.
GPU: SparseProjector (vr_srp_csr_f32) against the float64 host product P @ X^T."""
import os

import numpy as np
import pytest
import torch

from visreps_amd.analysis import sparse_random_projection as S


def test_fit_matches_sklearn(tmp_path):
    from sklearn.random_projection import SparseRandomProjection

    t = S.get_srp_transformer(D=900, k=128, density=None, seed=5, cache_dir=str(tmp_path))
    ref = SparseRandomProjection(n_components=128, random_state=5).fit(np.zeros((1, 900), np.float32))
    assert (t.components_ != ref.components_).nnz == 0
    assert t.components_.dtype == np.float32
    assert np.isclose(t.density_, 1 / np.sqrt(900))
    vals = np.unique(np.abs(t.components_.data))
    assert np.allclose(vals, np.sqrt(1 / t.density_) / np.sqrt(128))


def test_cache_roundtrip_and_name(tmp_path):
    t1 = S.get_srp_transformer(D=300, k=40, density=None, seed=11, cache_dir=str(tmp_path))
    path = S.srp_cache_path(str(tmp_path), 300, 40, None, 11)
    assert os.path.basename(path) == "srp_D300_k40_densityauto_seed11.npz"
    assert os.path.exists(path)
    t2 = S.get_srp_transformer(D=300, k=40, density=None, seed=11, cache_dir=str(tmp_path))
    assert (t1.components_ != t2.components_).nnz == 0 and t2.random_state == 11


def test_corrupt_cache_is_refitted(tmp_path):
    path = S.srp_cache_path(str(tmp_path), 200, 16, None, 3)
    with open(path, "wb") as f:
        f.write(b"not an npz")
    t = S.get_srp_transformer(D=200, k=16, density=None, seed=3, cache_dir=str(tmp_path))
    assert t is not None and t.components_.shape == (16, 200)
    assert S._load(path).n_components == 16


def test_mismatched_cache_is_refitted(tmp_path):
    t = S.get_srp_transformer(D=200, k=16, density=None, seed=3, cache_dir=str(tmp_path))
    bad = S.SRPComponents(t.components_, 17, t.density_, 3)  # wrong k under the right name
    S._save(S.srp_cache_path(str(tmp_path), 200, 16, None, 3), bad)
    again = S.get_srp_transformer(D=200, k=16, density=None, seed=3, cache_dir=str(tmp_path))
    assert again.n_components == 16 and (again.components_ != t.components_).nnz == 0


def test_invalid_dims_return_none(tmp_path):
    assert S.get_srp_transformer(D=0, k=4, density=None, seed=0, cache_dir=str(tmp_path)) is None
    assert S.get_srp_transformer(D=10, k=0, density=None, seed=0, cache_dir=str(tmp_path)) is None


def test_explicit_density(tmp_path):
    t = S.get_srp_transformer(D=1000, k=64, density=0.1, seed=2, cache_dir=str(tmp_path))
    assert np.isclose(t.density_, 0.1)
    assert os.path.exists(S.srp_cache_path(str(tmp_path), 1000, 64, 0.1, 2))


@pytest.mark.gpu
@pytest.mark.parametrize("B,D,k", [(1, 100, 16), (63, 1000, 64), (65, 4097, 130), (200, 9216, 4096)])
def test_gpu_projector_matches_host(dev, tmp_path, B, D, k):
    t = S.get_srp_transformer(D=D, k=min(k, D), density=None, seed=B, cache_dir=str(tmp_path))
    rng = np.random.default_rng(B)
    X = rng.standard_normal((B, D)).astype(np.float32)
    X[:, ::7] = np.maximum(X[:, ::7], 0)
    proj = S.SparseProjector(t, dev)
    got = proj(torch.from_numpy(X).to(dev)).cpu().numpy()
    ref = (t.components_.astype(np.float64) @ X.T.astype(np.float64)).T
    scale = np.sqrt(np.abs(t.components_).astype(np.float64).power(2) @ (X.T.astype(np.float64) ** 2)).T + 1e-30
    assert got.shape == (B, min(k, D))
    assert np.max(np.abs(got - ref) / scale) < 1e-5


@pytest.mark.gpu
def test_gpu_projector_strided_input(dev, tmp_path):
    t = S.get_srp_transformer(D=500, k=50, density=None, seed=1, cache_dir=str(tmp_path))
    base = torch.randn(10, 800, device=dev)
    view = base[:, 100:600]  # row stride 800
    got = S.SparseProjector(t, dev)(view).cpu().numpy()
    ref = (t.components_.astype(np.float64) @ view.cpu().numpy().T.astype(np.float64)).T
    assert np.allclose(got, ref, atol=1e-4)
    with pytest.raises(ValueError):
        S.SparseProjector(t, dev)(torch.randn(3, 499, device=dev))
