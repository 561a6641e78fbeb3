"""reconstruct_from_pcs (reference: visreps/analysis/reconstruct_from_pcs.py:7-31) on the
device against the numpy oracle, which is pinned to sklearn's PCA here."""
import numpy as np
import pytest

from oracle import pca_oracle as P


def _acts(n, shape, seed, decay=0.7):
    rs = np.random.RandomState(seed)
    d = int(np.prod(shape))
    r = min(n, d)
    # a decaying spectrum so the top components are well separated
    U = np.linalg.qr(rs.randn(n, r))[0]
    V = np.linalg.qr(rs.randn(d, r))[0]
    s = 10.0 * decay ** np.arange(r)
    x = (U * s) @ V.T + 0.5
    return x.reshape((n,) + tuple(shape)).astype(np.float32)


@pytest.mark.parametrize("n,shape,k", [(40, (300,), 1), (40, (6, 5, 5), 3), (200, (30,), 2)])
def test_oracle_matches_sklearn_pca(n, shape, k):
    from sklearn.decomposition import PCA

    x = _acts(n, shape, n + k)
    flat = x.reshape(n, -1).astype(np.float64)
    pca = PCA(n_components=min(k, flat.shape[1]), svd_solver="full")
    ref = pca.inverse_transform(pca.fit_transform(flat)).reshape(x.shape)
    assert np.allclose(P.reconstruct_from_pcs(x, k), ref, rtol=0, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("n,shape,k", [(40, (300,), 1), (40, (6, 5, 5), 3), (200, (30,), 2), (64, (4096,), 5)])
def test_reconstruct_matches_oracle_torch_and_numpy(dev, n, shape, k):
    import torch
    from visreps_amd.analysis.reconstruct_from_pcs import reconstruct_from_pcs

    x = _acts(n, shape, 7 * n + k)
    ref = P.reconstruct_from_pcs(x, k)
    xt = torch.from_numpy(x).to(dev)
    before = xt.clone()
    got = reconstruct_from_pcs({"l": xt, "np": x}, k)
    assert torch.equal(xt, before)  # input untouched
    gt = got["l"]
    assert gt.dtype == torch.float32 and gt.device == xt.device and gt.shape == xt.shape
    tol = 1e-5 * np.abs(ref).max()
    assert np.max(np.abs(gt.cpu().numpy() - ref)) <= tol
    assert isinstance(got["np"], np.ndarray) and got["np"].dtype == np.float32
    assert np.max(np.abs(got["np"] - ref)) <= tol


@pytest.mark.gpu
def test_reconstruct_k_larger_than_rank_raises(dev):
    import torch
    from visreps_amd.analysis.reconstruct_from_pcs import reconstruct_from_pcs

    x = torch.randn(5, 40, device=dev)
    with pytest.raises(ValueError):
        reconstruct_from_pcs({"l": x}, 6)
    with pytest.raises(ValueError):
        reconstruct_from_pcs({"l": torch.randn(5, device=dev)}, 1)
