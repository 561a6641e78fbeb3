"""BASELINE configs[1] sizes (N = 10k stimuli, k = 9000, 1000 bootstrap sets) on the GPU,
checked through size-independent properties (the CPU oracle needs ~6 s per N=10k
Spearman, so full-size parity goes through independent GPU code paths instead):

* Gram: fp64 recomputation of 64 sampled rows (<= 5e-6), exact symmetry, zero diagonal.
* Engine subset masking vs an explicit sub-RDM: subset s of the bootstrap call equals the
  triangle Spearman of A[idx_s][:, idx_s] vs B[idx_s][:, idx_s] computed from a rank plan
  of the gathered 9000 x 9000 sub-RDMs (different plan, different pass structure; both
  exact integer sums, so they agree to fp64 rounding).
* Point estimate (subset 0 of the call) == vr_spearman_triu_f32 on the full RDMs.
* Symmetry of Spearman: swapping the RDMs gives the same scores bit for bit.
* Bootstrap index sets == numpy.random.RandomState(42) draws (first and last rows).
"""
import numpy as np
import pytest
import torch

from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices

pytestmark = pytest.mark.gpu

N, K, NB = 10000, 9000, 1000


@pytest.fixture(scope="module")
def rdms(dev):
    g = torch.Generator(device=dev).manual_seed(20260306)
    z = torch.randn(N, 64, device=dev, generator=g)
    xm = torch.relu(z @ (torch.randn(64, 4096, device=dev, generator=g) / 8)
                    + 2 * torch.randn(N, 4096, device=dev, generator=g))
    xn = z @ torch.randn(64, 2000, device=dev, generator=g) + 3 * torch.randn(N, 2000, device=dev, generator=g)
    return xm, R.compute_rdm(xm), R.compute_rdm(xn)


def test_fullsize_gram_rows_vs_fp64(dev, rdms):
    x, rdm, _ = rdms
    rows = torch.randperm(N, device=dev, generator=torch.Generator(device=dev).manual_seed(1))[:64]
    xd = x.double()
    xd = xd - xd.mean(1, keepdim=True)
    s = torch.sqrt((xd * xd).mean(1) + 1e-12)
    ref = 1.0 - ((xd[rows] @ xd.T / x.size(1)) / (s[rows, None] * s[None, :] + 1e-12)).clamp(-1, 1)
    ref[torch.arange(64, device=dev), rows] = 0.0
    assert float((rdm[rows].double() - ref).abs().max()) <= 5e-6
    assert torch.equal(rdm, rdm.T) and torch.all(torch.diagonal(rdm) == 0)


def test_fullsize_bootstrap_matches_explicit_subrdms(dev, rdms):
    _, a, b = rdms
    idx = bootstrap_indices(42, N, K, NB)
    rs = np.random.RandomState(42)
    assert np.array_equal(idx[0], rs.choice(N, K, replace=False))
    pa, pb = R.RankPlan(a), R.RankPlan(b)
    scores = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert scores.shape == (NB + 1,) and np.all(np.isfinite(scores))
    # point estimate: the triangle-Spearman entry point on the full RDMs
    point = R.compute_rdm_correlation(a, b, correlation="Spearman")
    assert abs(scores[0] - point) <= 1e-12
    # swapping the RDMs: same exact sums
    swapped = R.bootstrap_spearman(pb, pa, idx, full_first=True).cpu().numpy()
    assert np.array_equal(scores, swapped)
    # subsets 1, 500, 1000 from explicit gathered sub-RDMs
    for s in (0, 499, NB - 1):
        it = torch.as_tensor(np.array(idx[s]), dtype=torch.long, device=dev)
        sa = a[it][:, it].contiguous()
        sb = b[it][:, it].contiguous()
        ref = R.compute_rdm_correlation(sa, sb, correlation="Spearman")
        assert abs(scores[1 + s] - ref) <= 1e-12, (s, scores[1 + s], ref)
    assert rs.choice(N, K, replace=False).tolist() == idx[1].tolist()
