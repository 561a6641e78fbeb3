"""Pins the CPU oracle to the reference's own tests (CPU only).

Known-answer and property tests transcribed from /root/reference/tests/test_rsa_bootstrap.py
(line numbers cited per test) plus checks against scipy / numpy, the third-party functions
the reference calls. The oracle is then the checker for every GPU parity test."""
import math

import numpy as np
import pytest
import scipy.stats

from oracle import rsa_oracle as O


def test_rdm_known_values():
    # test_rsa_bootstrap.py:214-225
    x = np.array([[1, 2, 3, 4, 5], [2, 4, 6, 8, 10], [5, 3, 1, -1, -3]], np.float32)
    r = O.compute_rdm(x)
    assert r[0, 1] == pytest.approx(0.0, abs=1e-4)
    assert r[0, 2] == pytest.approx(2.0, abs=1e-4)


def test_rdm_identical_and_negated():
    # :1017-1033
    assert O.compute_rdm(np.array([[1, 2, 3], [1, 2, 3]], np.float32))[0, 1] == pytest.approx(0, abs=1e-5)
    assert O.compute_rdm(np.array([[1, 2, 3], [-1, -2, -3]], np.float32))[0, 1] == pytest.approx(2, abs=1e-4)


def test_rdm_properties():
    # :123-143, :177-196, :227-231
    x = np.random.RandomState(0).randn(50, 20).astype(np.float32)
    r = O.compute_rdm(x)
    assert r.dtype == np.float32 and r.shape == (50, 50)
    assert np.allclose(r, r.T, atol=1e-5)
    assert np.all(np.diag(r) == 0)
    off = r[~np.eye(50, dtype=bool)]
    assert off.min() >= -0.01 and off.max() <= 2.01


def test_rdm_vs_scipy_pairwise():
    # :910-952
    x = np.random.RandomState(42).randn(10, 20).astype(np.float32)
    r = O.compute_rdm(x)
    for i in range(10):
        for j in range(i + 1, 10):
            assert abs(r[i, j] - (1 - scipy.stats.pearsonr(x[i], x[j])[0])) < 0.01
    xs = np.random.RandomState(42).randn(8, 15).astype(np.float32)
    rs = O.compute_rdm(xs, correlation="Spearman")
    for i in range(8):
        for j in range(i + 1, 8):
            assert abs(rs[i, j] - (1 - scipy.stats.spearmanr(xs[i], xs[j])[0])) < 0.02


def test_rdm_zero_variance_and_single():
    # :184-189, :204-212, :1005-1015
    x = np.random.RandomState(1).randn(10, 5).astype(np.float32)
    x[3] = 5.0
    x[7] = -2.0
    r = O.compute_rdm(x)
    assert np.isfinite(r).all() and np.all(np.diag(r) == 0)
    assert O.compute_rdm(np.random.randn(1, 5)).tolist() == [[0.0]]


def test_rdm_permutation_and_subindex():
    # :987-1003, :730-744, :1390-1412
    x = np.random.RandomState(42).randn(30, 20).astype(np.float32)
    r = O.compute_rdm(x)
    perm = np.random.RandomState(1).permutation(30)
    assert np.allclose(O.compute_rdm(x[perm]), r[perm][:, perm], atol=1e-5)
    rng = np.random.RandomState(42)
    for _ in range(10):
        idx = rng.choice(30, size=27, replace=False)
        assert np.allclose(r[idx][:, idx], O.compute_rdm(x[idx]), atol=1e-4)


def test_rank_known():
    # :877-905, :1206-1232
    assert O._rank(np.array([[3.0, 1.0, 2.0]])).tolist() == [[2.0, 0.0, 1.0]]
    assert O._rank(np.array([[1.0, 1.0, 3.0]])).tolist() == [[0.0, 1.0, 2.0]]


def test_invalid_methods():
    with pytest.raises(ValueError):
        O.compute_rdm(np.zeros((3, 3)), correlation="cosine")
    with pytest.raises(ValueError):
        O.compute_rdm_correlation(np.zeros((5, 5)), np.zeros((6, 6)))
    with pytest.raises(ValueError):
        O.compute_rdm_correlation(np.zeros((5, 5)), np.zeros((5, 5)), correlation="cosine")
    assert math.isnan(O.compute_rdm_correlation(np.zeros((1, 1)), np.zeros((1, 1)), correlation="cosine"))


def test_kendall_tau_a_known():
    # :383-394, :1124-1135, :1151-1172, :415-420, :1174-1177
    assert O._kendall_tau_a(np.array([1.0, 2, 3]), np.array([3.0, 1, 2]))[0] == pytest.approx(-1 / 3, abs=1e-5)
    assert O._kendall_tau_a(np.array([1.0, 2, 3, 4]), np.array([1.0, 4, 2, 3]))[0] == pytest.approx(1 / 3, abs=1e-5)
    x = np.array([1.0, 1.0, 2.0, 2.0, 3.0])
    y = np.array([1.0, 2.0, 3.0, 4.0, 5.0])
    tb = scipy.stats.kendalltau(x, y).statistic
    assert O._kendall_tau_a(x, y)[0] == pytest.approx(tb * np.sqrt((10 - 2) * 10) / 10, abs=1e-5)
    assert math.isnan(O._kendall_tau_a(np.ones(4), 2 * np.ones(4))[0])
    assert math.isnan(O._kendall_tau_a(np.array([]), np.array([]))[0])


def test_spearman_equals_exact_midrank():
    # :269-286 (vs scipy) + the exact integer restatement used as the GPU checker
    rng = np.random.RandomState(3)
    for m, levels in [(2, None), (3, None), (50, 5), (1000, 30), (4000, None)]:
        a = rng.rand(m).astype(np.float32)
        b = rng.rand(m).astype(np.float32)
        if levels:
            a = np.floor(a * levels) / levels
            b = np.floor(b * levels) / levels
        s = scipy.stats.spearmanr(a, b).statistic
        e = O.midrank_spearman(a, b)
        if m < 3:
            assert math.isnan(e) or abs(e - s) < 1e-12
        else:
            assert abs(e - s) < 1e-12


def test_subsample_sizes():
    # test_encoding_score.py:1610-1620
    for n, k in [(10, 9), (20, 18), (50, 45), (100, 90), (1000, 900)]:
        assert int(n * 0.9) == k


def test_bootstrap_without_replacement_and_determinism():
    # :761-770, :1333-1358, :586-604
    rs = np.random.RandomState(0).rand(40, 40).astype(np.float32)
    m = np.triu(rs, 1) + np.triu(rs, 1).T
    rn = np.random.RandomState(1).rand(40, 40).astype(np.float32)
    n = np.triu(rn, 1) + np.triu(rn, 1).T
    p1, s1, lo1, hi1 = O.bootstrap_rsa(m, n, n_bootstrap=30, seed=42)
    p2, s2, lo2, hi2 = O.bootstrap_rsa(m, n, n_bootstrap=30, seed=42)
    assert np.array_equal(s1, s2) and lo1 == lo2 and hi1 == hi2
    _, s3, _, _ = O.bootstrap_rsa(m, n, n_bootstrap=30, seed=99)
    assert not np.array_equal(s1, s3)
    assert lo1 <= hi1
