"""Golden vectors (tests/golden/, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces its committed vectors and the native RNG reproduces the
numpy RandomState streams. GPU: the HIP path against the committed vectors (no oracle
call at run time)."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import rsa_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(pattern):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLD, pattern))):
        with np.load(p, allow_pickle=False) as z:
            out.append((os.path.basename(p), {k: z[k] for k in z.files}))
    return out


@pytest.mark.parametrize("name,z", _load("rdm_*.npz"))
def test_oracle_rdm_golden(name, z):
    assert np.max(np.abs(O.compute_rdm(z["X"]) - z["rdm"])) <= 1e-6


@pytest.mark.parametrize("name,z", _load("spearman_*.npz"))
def test_oracle_spearman_golden(name, z):
    got = O.compute_rdm_correlation(z["A"], z["B"], "Spearman")
    assert np.isclose(got, z["scipy"], atol=1e-12, equal_nan=True)
    assert np.isclose(z["exact"], z["scipy"], atol=1e-12, equal_nan=True)


@pytest.mark.parametrize("name,z", _load("bootstrap_*.npz"))
def test_oracle_bootstrap_golden(name, z):
    point, scores, lo, hi = O.bootstrap_rsa(z["A"], z["B"], n_bootstrap=len(z["scores"]), seed=42)
    assert np.isclose(point, z["point"], atol=1e-12)
    assert np.allclose(scores, z["scores"], atol=1e-12)
    assert np.allclose([lo, hi], z["ci"], atol=1e-12)


def test_native_rng_golden():
    from visreps_amd.analysis._random import LegacyRandomState

    with np.load(os.path.join(GOLD, "rng.npz"), allow_pickle=False) as z:
        for key in z.files:
            ref = z[key]
            if key.startswith("perm_"):
                _, seed, n = key.split("_")
                assert np.array_equal(LegacyRandomState(int(seed)).permutation(int(n)), ref)
                continue
            seed, n, k = (int(t[1:]) for t in key.split("_"))
            rs = LegacyRandomState(seed)
            for row in ref:
                assert np.array_equal(rs.choice(n, k, replace=False), row)


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name,z", _load("rdm_*.npz"))
def test_gpu_rdm_golden(dev, name, z):
    from visreps_amd.analysis import rsa as R

    got = R.compute_rdm(torch.from_numpy(z["X"]).to(dev)).cpu().numpy()
    assert np.max(np.abs(got - z["rdm"])) <= 2e-5
    assert np.array_equal(got, got.T) and np.all(np.diag(got) == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("name,z", _load("spearman_*.npz"))
def test_gpu_spearman_golden(dev, name, z):
    from visreps_amd.analysis import rsa as R

    a, b = torch.from_numpy(z["A"]).to(dev), torch.from_numpy(z["B"]).to(dev)
    got = R.compute_rdm_correlation(a, b, correlation="Spearman")
    assert np.isclose(got, z["exact"], atol=1e-12, equal_nan=True)
    got_p = R.compute_rdm_correlation(a, b, correlation="Pearson")
    assert np.isclose(got_p, z["pearson"], atol=1e-6, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name,z", _load("bootstrap_*.npz"))
def test_gpu_bootstrap_golden(dev, name, z):
    from visreps_amd.analysis import rsa as R
    from visreps_amd.analysis._random import bootstrap_indices

    n = z["A"].shape[0]
    idx = bootstrap_indices(42, n, int(0.9 * n), len(z["scores"]))
    assert np.array_equal(idx, z["idx"]), "bootstrap index draws must be bit-exact"
    point, scores, lo, hi = R.bootstrap_rsa(torch.from_numpy(z["A"]).to(dev),
                                            torch.from_numpy(z["B"]).to(dev),
                                            n_bootstrap=len(z["scores"]), seed=42)
    assert abs(point - z["point"]) <= 1e-12
    assert np.max(np.abs(scores - z["scores"])) <= 1e-12
    assert np.allclose([lo, hi], z["ci"], atol=1e-12)
