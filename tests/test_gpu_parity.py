"""HIP path vs the CPU oracle (oracle/rsa_oracle.py) on seeded inputs.

Tolerances
  * RDM entries: |delta| <= 2e-5 (fp32 Gram, different summation order; the reference's
    own torch-CPU sgemm differs from any other fp32 order at this level).
  * Spearman on identical RDM inputs: |delta| <= 1e-12 (both exact midrank arithmetic;
    scipy's float64 corrcoef rounding is ~1e-15).
  * Spearman / RSA scores where each side builds its own RDM: |delta| < 1e-5
    (BASELINE.json north_star tolerance).
  * Bootstrap index sets: bit-exact (legacy MT19937 stream).
"""
import math

import numpy as np
import pytest
import torch

from oracle import rsa_oracle as O
from visreps_amd.analysis import rsa as R

pytestmark = pytest.mark.gpu


def _rand(n, d, seed=0, scale=1.0):
    return np.random.RandomState(seed).randn(n, d).astype(np.float32) * scale


# --------------------------------------------------------------------------- RDM
@pytest.mark.parametrize("n,d", [(1, 5), (2, 3), (3, 7), (17, 33), (130, 257), (300, 1000),
                                 (129, 4100), (64, 1), (200, 6)])
def test_rdm_matches_oracle(dev, n, d):
    x = _rand(n, d, seed=n * 7 + d)
    got = R.compute_rdm(torch.from_numpy(x).to(dev)).cpu().numpy()
    ref = O.compute_rdm(x)
    assert got.dtype == np.float32 and got.shape == (n, n)
    assert np.array_equal(got, got.T), "RDM must be exactly symmetric"
    assert np.all(np.diag(got) == 0.0)
    assert np.max(np.abs(got - ref)) <= 2e-5


def test_rdm_split_k_conv5_shape(dev):
    # cfg1 shape: N=256 stimuli x conv5 D=43264 -> split-K path
    x = np.maximum(_rand(256, 43264, seed=5), 0)
    got = R.compute_rdm(torch.from_numpy(x).to(dev)).cpu().numpy()
    ref = O.compute_rdm(x)
    assert np.array_equal(got, got.T)
    assert np.max(np.abs(got - ref)) <= 2e-5


def test_rdm_cpu_input_returns_cpu(dev):
    x = torch.from_numpy(_rand(20, 10))
    rdm = R.compute_rdm(x)
    assert rdm.device.type == "cpu" and rdm.dtype == torch.float32


def test_rdm_known_values(dev):
    # tests/test_rsa_bootstrap.py:214-225 and 1017-1033
    x = torch.tensor([[1.0, 2.0, 3.0, 4.0, 5.0], [2.0, 4.0, 6.0, 8.0, 10.0],
                      [5.0, 3.0, 1.0, -1.0, -3.0]])
    rdm = R.compute_rdm(x)
    assert rdm[0, 1].item() == pytest.approx(0.0, abs=1e-4)
    assert rdm[0, 2].item() == pytest.approx(2.0, abs=1e-4)
    assert R.compute_rdm(torch.tensor([[1.0, 2.0, 3.0], [1.0, 2.0, 3.0]]))[0, 1].item() == pytest.approx(0.0, abs=1e-5)
    assert R.compute_rdm(torch.tensor([[1.0, 2.0, 3.0], [-1.0, -2.0, -3.0]]))[0, 1].item() == pytest.approx(2.0, abs=1e-4)


def test_rdm_zero_variance_rows_finite(dev):
    x = torch.randn(10, 5)
    x[3] = 5.0
    x[7] = -2.0
    rdm = R.compute_rdm(x)
    assert torch.isfinite(rdm).all()
    assert torch.all(rdm.diag() == 0.0)
    ref = O.compute_rdm(x.numpy())
    assert np.max(np.abs(rdm.numpy() - ref)) <= 2e-5


def test_rdm_spearman_is_pearson_on_ranks(dev):
    x = torch.from_numpy(_rand(12, 20, seed=3))
    a = R.compute_rdm(x, correlation="Spearman")
    b = R.compute_rdm(R._rank(x), correlation="Pearson")
    assert torch.equal(a, b)
    ref = O.compute_rdm(x.numpy(), correlation="Spearman")
    assert np.max(np.abs(a.numpy() - ref)) <= 2e-5


def test_rdm_invalid_method():
    with pytest.raises(ValueError):
        R.compute_rdm(torch.randn(5, 3), correlation="cosine")


def test_rdm_does_not_mutate(dev):
    x = torch.randn(10, 5, device=dev)
    x0 = x.clone()
    R.compute_rdm(x)
    R.compute_rdm(x, correlation="Spearman")
    assert torch.equal(x, x0)


# --------------------------------------------------------------------------- Spearman
def _tied_rdm(n, seed, levels=None):
    rng = np.random.RandomState(seed)
    m = rng.rand(n, n).astype(np.float32)
    if levels:
        m = np.floor(m * levels).astype(np.float32) / levels
    m = np.triu(m, 1)
    return (m + m.T).astype(np.float32)


@pytest.mark.parametrize("n", [2, 3, 4, 5, 16, 63, 64, 65, 257, 1000])
@pytest.mark.parametrize("levels", [None, 7, 1000])
def test_spearman_exact_vs_oracle(dev, n, levels):
    a = _tied_rdm(n, 1 + n, levels)
    b = _tied_rdm(n, 2 + n, levels)
    got = R.compute_rdm_correlation(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev),
                                    correlation="Spearman")
    iu = np.triu_indices(n, 1)
    exact = O.midrank_spearman(a[iu], b[iu])
    ref = O.compute_rdm_correlation(a, b, "Spearman")
    if math.isnan(exact):
        assert math.isnan(got) and math.isnan(ref)
    else:
        assert abs(got - exact) <= 1e-12
        assert abs(got - ref) <= 1e-9


def test_spearman_giant_tie_group_wide_path(dev):
    # a tie group larger than 32767 - 4096 positions forces u32 chunk ranks
    n = 300
    rng = np.random.RandomState(9)
    a = rng.rand(n, n).astype(np.float32)
    a[rng.rand(n, n) < 0.75] = 0.5
    a = np.triu(a, 1)
    a = a + a.T
    b = _tied_rdm(n, 10, levels=50)
    iu = np.triu_indices(n, 1)
    assert np.sum(a[iu] == 0.5) > 30000
    pa, pb = R.RankPlan(torch.from_numpy(a).to(dev)), R.RankPlan(torch.from_numpy(b).to(dev))
    idx = np.stack([rng.choice(n, 270, replace=False) for _ in range(70)]).astype(np.int32)
    got = R.bootstrap_spearman(pa, pb, idx).cpu().numpy()
    assert abs(got[0] - O.midrank_spearman(a[iu], b[iu])) <= 1e-12
    ik = np.triu_indices(270, 1)
    for i in range(70):
        s = idx[i]
        ref = O.midrank_spearman(a[np.ix_(s, s)][ik], b[np.ix_(s, s)][ik])
        assert abs(got[i + 1] - ref) <= 1e-12


def test_spearman_nan_and_constant(dev):
    a = _tied_rdm(10, 1)
    b = a.copy()
    b[2, 5] = b[5, 2] = np.nan
    assert math.isnan(R.compute_rdm_correlation(torch.from_numpy(a), torch.from_numpy(b), correlation="Spearman"))
    c = np.ones((10, 10), np.float32)
    np.fill_diagonal(c, 0)
    assert math.isnan(R.compute_rdm_correlation(torch.from_numpy(a), torch.from_numpy(c), correlation="Spearman"))
    assert math.isnan(R.compute_rdm_correlation(torch.zeros(1, 1), torch.zeros(1, 1), correlation="Spearman"))
    # n=2 -> one pair -> undefined
    assert math.isnan(R.compute_rdm_correlation(torch.from_numpy(a[:2, :2]), torch.from_numpy(a[:2, :2]),
                                                correlation="Spearman"))


def test_spearman_negative_zero_ties(dev):
    a = _tied_rdm(30, 4, levels=5) - 0.4  # negative values and exact zeros
    a[np.abs(a) < 1e-7] = -0.0
    b = _tied_rdm(30, 5, levels=5)
    iu = np.triu_indices(30, 1)
    got = R.compute_rdm_correlation(torch.from_numpy(a), torch.from_numpy(b), correlation="Spearman")
    assert abs(got - O.midrank_spearman(a[iu], b[iu])) <= 1e-12


@pytest.mark.parametrize("n", [3, 15, 200])
def test_pearson_vs_scipy(dev, n):
    a, b = _tied_rdm(n, 7), _tied_rdm(n, 8)
    got = R.compute_rdm_correlation(torch.from_numpy(a), torch.from_numpy(b), correlation="Pearson")
    ref = O.compute_rdm_correlation(a, b, "Pearson")
    assert abs(got - ref) <= 1e-6


def test_correlation_errors():
    with pytest.raises(ValueError):
        R.compute_rdm_correlation(torch.zeros(5, 5), torch.zeros(6, 6))
    with pytest.raises(ValueError):
        R.compute_rdm_correlation(torch.zeros(5, 5), torch.zeros(5, 5), correlation="cosine")


# --------------------------------------------------------------------------- bootstrap
@pytest.mark.parametrize("n,nb", [(10, 20), (64, 50), (130, 70), (256, 130)])
def test_bootstrap_matches_oracle_same_rdms(dev, n, nb):
    x = O.synthetic_features(n, [300, 200], seed=n)
    m_rdm = O.compute_rdm(x[0])
    n_rdm = O.compute_rdm(x[1])
    point, scores, lo, hi = R.bootstrap_rsa(torch.from_numpy(m_rdm).to(dev),
                                            torch.from_numpy(n_rdm).to(dev), n_bootstrap=nb, seed=42)
    rp, rs, rlo, rhi = O.bootstrap_rsa(m_rdm, n_rdm, n_bootstrap=nb, seed=42)
    assert abs(point - rp) <= 1e-12
    assert np.max(np.abs(scores - rs)) <= 1e-12
    assert abs(lo - rlo) <= 1e-12 and abs(hi - rhi) <= 1e-12


def test_bootstrap_end_to_end_tolerance(dev):
    # each side computes its own RDMs from the same features: |dSpearman| < 1e-5
    n = 256
    feats = O.synthetic_features(n, [43264, 2000], seed=11, relu=[True, False], noise=3.0)
    gm = R.compute_rdm(torch.from_numpy(feats[0]).to(dev))
    gn = R.compute_rdm(torch.from_numpy(feats[1]).to(dev))
    point, scores, lo, hi = R.bootstrap_rsa(gm, gn, n_bootstrap=100, seed=42)
    rp, rs, rlo, rhi = O.bootstrap_rsa(O.compute_rdm(feats[0]), O.compute_rdm(feats[1]),
                                       n_bootstrap=100, seed=42)
    assert abs(point - rp) < 1e-5
    assert np.max(np.abs(scores - rs)) < 1e-5
    assert abs(lo - rlo) < 1e-5 and abs(hi - rhi) < 1e-5


def _rdm_f64(x: np.ndarray) -> np.ndarray:
    xc = x.astype(np.float64) - x.astype(np.float64).mean(1, keepdims=True)
    s = np.sqrt((xc * xc).mean(1) + 1e-12)
    c = np.clip((xc @ xc.T) / x.shape[1] / (np.outer(s, s) + 1e-12), -1, 1)
    np.fill_diagonal(c, 1.0)
    return 1.0 - c


@pytest.mark.parametrize("n,d", [(256, 43264), (700, 4096), (130, 257), (1000, 290)])
def test_rdm_split_gram_accuracy_vs_fp64(dev, n, d, monkeypatch):
    # the bf16 hi/lo split Gram (default) and the exact-fp32 MFMA kernel (VISREPS_GRAM=fp32)
    # against an fp64 reference: the split kernel within 5e-6 (observed: 6.7e-7 at n=256,
    # D=43264; 1.8e-6 at D=257), the fp32 kernel within 1e-6 (observed 1.2e-7-1.8e-7),
    # both inside the 2e-5 RDM tolerance
    feats = O.synthetic_features(n, [d], seed=d % 97, relu=[True])[0]
    ref = _rdm_f64(feats)
    x = torch.from_numpy(feats).to(dev)
    monkeypatch.setenv("VISREPS_GRAM", "split")
    split = R.compute_rdm(x).double().cpu().numpy()
    monkeypatch.setenv("VISREPS_GRAM", "fp32")
    exact = R.compute_rdm(x).double().cpu().numpy()
    e_split, e_exact = np.abs(split - ref).max(), np.abs(exact - ref).max()
    assert e_split <= 5e-6 and e_exact <= 1e-6, (e_split, e_exact)
    assert np.array_equal(split, split.T) and np.all(np.diag(split) == 0)


def test_split_gram_end_to_end_spearman_tolerance(dev, monkeypatch):
    # RSA scores from split-kernel RDMs vs the CPU path's own RDMs: |dSpearman| < 1e-5
    monkeypatch.setenv("VISREPS_GRAM", "split")
    n = 1500
    feats = O.synthetic_features(n, [8192, 2000], seed=3, relu=[True, False], noise=3.0)
    gm = R.compute_rdm(torch.from_numpy(feats[0]).to(dev))
    gn = R.compute_rdm(torch.from_numpy(feats[1]).to(dev))
    point, scores, lo, hi = R.bootstrap_rsa(gm, gn, n_bootstrap=8, seed=42)
    rp, rs, _, _ = O.bootstrap_rsa(O.compute_rdm(feats[0]), O.compute_rdm(feats[1]),
                                   n_bootstrap=8, seed=42)
    assert abs(point - rp) < 1e-5
    assert np.max(np.abs(scores - rs)) < 1e-5


@pytest.mark.parametrize("n,d", [(3, 7), (130, 257), (300, 1000)])
def test_rdm_fp32_kernel_matches_oracle(dev, n, d, monkeypatch):
    monkeypatch.setenv("VISREPS_GRAM", "fp32")
    x = np.random.RandomState(n).randn(n, d).astype(np.float32)
    got = R.compute_rdm(torch.from_numpy(x).to(dev)).cpu().numpy()
    assert np.max(np.abs(got - O.compute_rdm(x))) <= 2e-5


@pytest.mark.parametrize("mode", ["split", "fp32"])
@pytest.mark.parametrize("n,d,world", [(300, 70, 3), (1000, 40, 4), (2100, 33, 5), (4000, 64, 2)])
def test_rdm_tile_ranges_assemble_full_rdm(dev, n, d, world, mode, monkeypatch):
    # the block-distributed Gram (band launch order inside each rank's tile range) writes
    # every entry of its range exactly as the one-launch RDM does, with either kernel
    from visreps_amd import pipeline as P

    monkeypatch.setenv("VISREPS_GRAM", mode)
    x = torch.randn(n, d, device=dev)
    full = R.compute_rdm(x)
    acc = torch.zeros(n, n, device=dev)
    for t0, t1 in P.tile_ranges(n, world):
        part = torch.zeros(n, n, device=dev)
        P.rdm_tiles_into(x, part, t0, t1)
        acc += part
    assert torch.equal(acc, full)
    assert torch.equal(full, full.T)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_rdm_tile_ranges_wide_d_match_within_rounding(dev, world):
    # at d = 4096 split-K engages and the one-launch RDM uses the wide kernel, so a tile
    # range may sum in another order: entries agree to fp32 rounding, not bit for bit
    from visreps_amd import pipeline as P

    n, d = 3000, 4096
    g = torch.Generator(device=dev).manual_seed(world)
    x = torch.relu(torch.randn(n, d, device=dev, generator=g))
    full = R.compute_rdm(x)
    acc = torch.zeros(n, n, device=dev)
    for t0, t1 in P.tile_ranges(n, world):
        part = torch.zeros(n, n, device=dev)
        P.rdm_tiles_into(x, part, t0, t1)
        acc += part
        del part
    assert torch.equal(acc, acc.T)
    assert (acc - full).abs().max().item() <= 2e-6


@pytest.mark.parametrize("n,nb,levels_a",[(64, 70, None), (200, 130, None), (150, 64, 6)])
def test_bootstrap_multi_equals_per_unit(dev, n, nb, levels_a):
    # one shared (neural) plan against several model plans: every row bit-equal to the
    # per-unit engine call and within 1e-12 of the oracle; one model RDM tie-heavy
    from visreps_amd.analysis._random import bootstrap_indices

    feats = O.synthetic_features(n, [200, 300, 150, 100], seed=n + 1)
    rdms = [O.compute_rdm(f) for f in feats]
    if levels_a:
        rdms[0] = (np.floor(rdms[0] * levels_a) / levels_a).astype(np.float32)
    rdms[2] = (np.floor(rdms[2] * 7) / 7).astype(np.float32)
    neural = R.RankPlan(torch.from_numpy(rdms[0]).to(dev))
    models = [R.RankPlan(torch.from_numpy(r).to(dev)) for r in rdms[1:]]
    idx = bootstrap_indices(42, n, int(0.9 * n), nb)
    multi = R.bootstrap_spearman_multi(neural, models, idx).cpu().numpy()
    assert multi.shape == (3, nb + 1)
    for j, pm in enumerate(models):
        single = R.bootstrap_spearman(pm, neural, idx).cpu().numpy()
        assert np.array_equal(multi[j], single)
        rp, rs, _, _ = O.bootstrap_rsa(rdms[j + 1], rdms[0], n_bootstrap=nb, seed=42)
        assert abs(multi[j][0] - rp) <= 1e-12
        assert np.max(np.abs(multi[j][1:] - rs)) <= 1e-12


def test_all_units_groups_match_per_unit(dev):
    # the pipeline's grouped engine calls equal independent per-unit bootstrap_rsa runs
    from visreps_amd import pipeline as P

    n = 120
    feats = O.synthetic_features(n, [300, 200, 100, 80, 60], seed=5)
    rdm = {f"p{i}": torch.from_numpy(O.compute_rdm(feats[i])).to(dev) for i in range(3)}
    neural = {"r0": torch.from_numpy(O.compute_rdm(feats[3])).to(dev),
              "r1": torch.from_numpy(O.compute_rdm(feats[4])).to(dev)}
    res = P.all_units_rsa(lambda p: rdm[p], list(rdm), neural, n, n_boot=40, seed=42)
    for (p, r), v in res.items():
        point, scores, lo, hi = R.bootstrap_rsa(rdm[p], neural[r], n_bootstrap=40, seed=42)
        assert v["score"] == point and v["ci_low"] == lo and v["ci_high"] == hi
        assert np.array_equal(np.array(v["bootstrap_scores"]), scores)


def test_bootstrap_masks_large_n_global_path(dev):
    # n > 20k stimuli -> inclusion masks read from global memory instead of LDS
    n = 20500
    rng = np.random.RandomState(0)
    a = torch.rand(n, n, device=dev)
    a = torch.triu(a, 1)
    a = a + a.T
    b = (a * 3).floor() / 3 + 0.01 * torch.rand(n, n, device=dev)
    b = torch.triu(b, 1)
    b = b + b.T
    idx = np.stack([rng.choice(n, 50, replace=False) for _ in range(3)]).astype(np.int32)
    pa, pb = R.RankPlan(a), R.RankPlan(b)
    scores = R.bootstrap_spearman(pa, pb, idx).cpu().numpy()
    an, bn = a.cpu().numpy(), b.cpu().numpy()
    for i in range(3):
        s = idx[i]
        sa, sb = an[np.ix_(s, s)], bn[np.ix_(s, s)]
        iu = np.triu_indices(len(s), 1)
        assert abs(scores[i + 1] - O.midrank_spearman(sa[iu], sb[iu])) <= 1e-12


# --------------------------------------------------------------------------- compute_rsa
def test_compute_rsa_matches_oracle(dev):
    from visreps_amd.analysis.alignment import AlignmentData

    rng = np.random.RandomState(42)
    n_train, n_test, v = 200, 50, 100
    neural_train = rng.randn(n_train, v).astype(np.float32)
    neural_test = rng.randn(n_test, v).astype(np.float32)
    good_train = neural_train + 0.5 * rng.randn(n_train, v).astype(np.float32)
    good_test = neural_test + 0.5 * rng.randn(n_test, v).astype(np.float32)
    bad_train = rng.randn(n_train, v).astype(np.float32)
    bad_test = rng.randn(n_test, v).astype(np.float32)
    cfg = {"compare_method": "spearman"}
    sel = AlignmentData({"good": torch.from_numpy(good_train), "bad": torch.from_numpy(bad_train)},
                        torch.from_numpy(neural_train))
    ev = AlignmentData({"good": torch.from_numpy(good_test), "bad": torch.from_numpy(bad_test)},
                       torch.from_numpy(neural_test))
    got = R.compute_rsa(cfg, sel, ev, n_select=100, bootstrap=True, n_bootstrap=60, seed=42)[0]
    ref = O.compute_rsa(cfg, {"good": good_train, "bad": bad_train}, neural_train,
                        {"good": good_test, "bad": bad_test}, neural_test,
                        n_select=100, bootstrap=True, n_bootstrap=60, seed=42)[0]
    assert got["layer"] == ref["layer"] == "good"
    assert abs(got["score"] - ref["score"]) < 1e-5
    assert np.max(np.abs(np.array(got["bootstrap_scores"]) - np.array(ref["bootstrap_scores"]))) < 1e-5
    for g, r in zip(got["layer_selection_scores"], ref["layer_selection_scores"]):
        assert g["layer"] == r["layer"] and abs(g["score"] - r["score"]) < 1e-5


@pytest.mark.parametrize("mode", ["split", "fp32"])
def test_rdm_generation_tail_split(dev, mode, monkeypatch):
    # n = 4200 -> 33 x 34 / 2 = 561 tiles: one 512-block generation of whole-k tiles plus a
    # 49-tile tail launched split over k (gram_tail). Both launch schemes and the tiles of
    # the tail must agree with an fp64 RDM, and the matrix stays exactly symmetric.
    n, d = 4200, 1100
    feats = O.synthetic_features(n, [d], seed=11, relu=[True])[0]
    x = torch.from_numpy(feats).to(dev)
    monkeypatch.setenv("VISREPS_GRAM", mode)
    tail = R.compute_rdm(x).double()
    monkeypatch.setenv("VISREPS_GRAM_GEN", "0")  # one launch, no tail split
    whole = R.compute_rdm(x).double()
    xd = x.double()
    xd = xd - xd.mean(1, keepdim=True)
    s = torch.sqrt((xd * xd).mean(1) + 1e-12)
    ref = 1.0 - ((xd @ xd.T / d) / (s[:, None] * s[None, :] + 1e-12)).clamp(-1.0, 1.0)
    ref.fill_diagonal_(0.0)
    bound = 5e-6 if mode == "split" else 1e-6
    assert float((tail - ref).abs().max()) <= bound
    assert float((whole - ref).abs().max()) <= bound
    assert torch.equal(tail, tail.T) and torch.all(torch.diagonal(tail) == 0)


@pytest.mark.parametrize("wide,kernel,d", [("1", "e", 1100), ("1", "p", 1100), ("0", "e", 1100),
                                           ("1", "e", 40), ("1", "e", 9000), ("1", "p", 9000)])
def test_rdm_wide_supertiles(dev, wide, kernel, d, monkeypatch):
    # n = 6000: 24 x 25 / 2 = 300 super-tiles of 256; super-tile rows [0, 15) run on the wide
    # kernel (255 super-tiles = one generation; k_gram3e, or k_gram3p with
    # VISREPS_GRAM_KERNEL=p), the 45 super-tiles below on the wide kernel split over k
    # (k_gram_reduce_w) -- the 128-tile rows on k_gram3 when the wide kernel is off. Depths:
    # 35 stages (odd, a ragged last stage), 2 stages, 282 stages (one accumulator flush).
    # Every scheme against fp64 -- within 5e-6, except at d = 40, where the hi/lo split's
    # own precision over so few products reaches 1.2e-5 (both wide kernels alike,
    # profiles/r3_gram_precision.log) and the RDM bound of DESIGN §4 (2e-5) applies; the
    # product never takes the split kernel there (n^2 d < 1e10: the exact-fp32 kernel).
    # Exact symmetry.
    n = 6000
    feats = O.synthetic_features(n, [d], seed=13, relu=[True])[0]
    x = torch.from_numpy(feats).to(dev)
    monkeypatch.setenv("VISREPS_GRAM", "split")
    monkeypatch.setenv("VISREPS_GRAM_WIDE", wide)
    monkeypatch.setenv("VISREPS_GRAM_KERNEL", kernel)
    got = R.compute_rdm(x).double()
    xd = x.double()
    xd = xd - xd.mean(1, keepdim=True)
    s = torch.sqrt((xd * xd).mean(1) + 1e-12)
    ref = 1.0 - ((xd @ xd.T / d) / (s[:, None] * s[None, :] + 1e-12)).clamp(-1.0, 1.0)
    ref.fill_diagonal_(0.0)
    assert float((got - ref).abs().max()) <= (2e-5 if d < 64 else 5e-6)
    assert torch.equal(got, got.T) and torch.all(torch.diagonal(got) == 0)


# --------------------------------------------------------------------------- large n
def _key_range(v: np.ndarray) -> int:
    """Number of fp32 sort keys between the smallest and largest value (f32_sort_key)."""
    u = np.ascontiguousarray(v, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u[u == 0x80000000] = 0
    k = np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    return int(k.max() - k.min() + 1)


@pytest.mark.parametrize("n,levels", [(2, None), (3, None), (700, None), (1500, 5), (3000, 40), (2500, 2000),
                                     (2000, 200000)])
@pytest.mark.parametrize("form", ["bucket", "table", "sort"])
def test_spearman_full_equals_plan_path_and_oracle(dev, n, levels, form, monkeypatch):
    # the plan-free full-triangle Spearman (used above n = 65535) against the rank-plan
    # engine (bit for bit: both exact integer sums) and scipy (tie-heavy RDMs included), in
    # each of its forms (bucketed count tables, plain count tables, radix sort)
    monkeypatch.setenv("VISREPS_FULL_FORM", form)
    if form != "sort":  # room for two tables of 2^30 + 1 keys (the default workspace of a small n
        from visreps_amd._lib import workspace  # is the sort form's, and its tables may not fit)
        workspace.get(dev, 9 << 30, "spearman_full")
    a = O.synthetic_features(n, [40], seed=n)[0]
    b = O.synthetic_features(n, [60], seed=n + 1)[0]
    ra, rb = O.compute_rdm(a), O.compute_rdm(b)
    if levels:
        ra = (np.floor(ra * levels) / levels).astype(np.float32)
    ta, tb = torch.from_numpy(ra).to(dev), torch.from_numpy(rb).to(dev)
    got = R.spearman_full(ta, tb)
    ref = R.compute_rdm_correlation(ta, tb, correlation="Spearman")
    if n < 3:
        assert np.isnan(got) and np.isnan(ref)
        return
    from visreps_amd._lib import lib
    iu = np.triu_indices(n, 1)
    ranges = [_key_range(r[iu]) for r in (ra, rb)]
    used = lib().vr_spearman_full_last_form()
    if form == "bucket" and max(ranges) > (1 << 26):  # keys beyond the bucketed tables (e.g. 0.0 .. 2.0)
        assert used in (1, 2)
    else:
        assert used == ["bucket", "table", "sort"].index(form), (used, ranges)
    assert got == ref
    iu = np.triu_indices(n, 1)
    assert abs(got - O.midrank_spearman(ra[iu], rb[iu])) <= 1e-12
    assert R.spearman_full(tb, ta) == got


def test_spearman_full_wide_key_range_takes_the_sort_form(dev):
    # values far outside [0, 2] (a key range beyond the count tables' 2^30 + 1): the call
    # returns VR_EWORKSPACE on the default workspace and rsa.spearman_full re-runs it on the
    # sort form's; the statistic still equals the rank-plan engine's and scipy's
    n = 900
    g = np.random.default_rng(5)
    ra = np.exp(g.normal(0, 8, (n, n))).astype(np.float32)
    ra = np.where(g.random((n, n)) < 0.3, -ra, ra).astype(np.float32)
    ra = np.triu(ra, 1) + np.triu(ra, 1).T
    rb = (ra + np.exp(g.normal(0, 6, (n, n))).astype(np.float32)).astype(np.float32)
    rb = np.triu(rb, 1) + np.triu(rb, 1).T
    ta, tb = torch.from_numpy(ra).to(dev), torch.from_numpy(rb).to(dev)
    got = R.spearman_full(ta, tb)
    assert got == R.compute_rdm_correlation(ta, tb, correlation="Spearman")
    iu = np.triu_indices(n, 1)
    assert abs(got - O.midrank_spearman(ra[iu], rb[iu])) <= 1e-12
    # n = 30,000: the default workspace (count tables for 2^30 + 1 keys) is smaller than the
    # sort form's, so this call takes the VR_EWORKSPACE retry
    from visreps_amd._lib import lib, workspace
    L = lib()
    n = 30000
    assert L.vr_spearman_full_sort_workspace(n) > L.vr_spearman_full_workspace(n)
    gt = torch.Generator(device=dev).manual_seed(6)

    def wide():
        x = torch.exp(torch.randn(n, n, device=dev, generator=gt) * 8)
        x = torch.where(torch.rand(n, n, device=dev, generator=gt) < 0.3, -x, x).triu(1)
        return x + x.T

    ta = wide()
    tb = ta + wide()
    workspace.release("spearman_full")
    got = R.spearman_full(ta, tb)
    assert workspace.current(dev, "spearman_full") >= L.vr_spearman_full_sort_workspace(n)
    assert got == R.compute_rdm_correlation(ta, tb, correlation="Spearman") and 0.0 < got < 1.0
    workspace.release("spearman_full")


@pytest.mark.parametrize("nkeys", [1, 2, 200, 5000])
def test_spearman_full_few_adjacent_keys(dev, nkeys):
    # values on nkeys consecutive fp32 keys (1.0 + k ulp): a key range of <= 4096 keys puts one
    # key in each bucket (counts = bucket sizes); 5000 keys: W = 2 keys per bucket
    n = 900
    g = np.random.default_rng(nkeys)
    u = (0x3F800000 + g.integers(0, nkeys, (n, n))).astype(np.uint32)
    ra = np.triu(u.view(np.float32), 1)
    ra = (ra + ra.T).astype(np.float32)
    ub = (0x3F800000 + g.integers(0, max(2, nkeys // 3), (n, n))).astype(np.uint32)
    rb = np.triu(ub.view(np.float32), 1)
    rb = (rb + rb.T).astype(np.float32)
    from visreps_amd._lib import lib, workspace
    workspace.get(dev, 1 << 30, "spearman_full")
    ta, tb = torch.from_numpy(ra).to(dev), torch.from_numpy(rb).to(dev)
    got = R.spearman_full(ta, tb)
    assert lib().vr_spearman_full_last_form() == 0
    ref = R.compute_rdm_correlation(ta, tb, correlation="Spearman")
    if nkeys == 1:  # a constant triangle
        assert np.isnan(got) and np.isnan(ref)
        return
    assert got == ref
    iu = np.triu_indices(n, 1)
    assert abs(got - O.midrank_spearman(ra[iu], rb[iu])) <= 1e-12


def test_spearman_full_nan_and_constant(dev):
    a = torch.rand(50, 50, device=dev)
    a = (a + a.T) / 2
    c = torch.ones(50, 50, device=dev)
    assert np.isnan(R.spearman_full(a, c))
    b = a.clone()
    b[3, 7] = float("nan")
    assert np.isnan(R.spearman_full(a, b))


# --------------------------------------------------------------------------- radix sort
@pytest.mark.parametrize("m", [2, 4095, 4096, 4097, 100003, (1 << 20) + 17])
@pytest.mark.parametrize("dist", ["uniform", "few", "equal", "top"])
def test_sort_pairs_stable_vs_numpy(dev, m, dist):
    """vr_sort_pairs_u32 (sort.hip) against numpy's stable argsort: ragged last tiles,
    all-equal digits, few distinct keys (long same-digit runs inside one wave) and keys at
    0xFFFFFFFF (the value the kernel's padding lanes carry). Bit-exact incl. value order."""
    from visreps_amd.analysis.distributed_spearman import RankKernels
    rs = np.random.RandomState(m % 1000 + len(dist))
    if dist == "uniform":
        k = rs.randint(0, 1 << 32, size=m, dtype=np.uint64).astype(np.uint32)
    elif dist == "few":
        k = rs.choice(np.array([0, 7, 0x01000100, 0xFFFFFFFF, 12345678], np.uint32), size=m)
    elif dist == "equal":
        k = np.full(m, 0x5A5A5A5A, np.uint32)
    else:
        k = (0xFFFFFFFF - rs.randint(0, 3, size=m)).astype(np.uint32)
    v = np.arange(m, dtype=np.uint32)[::-1].copy()
    kt = torch.from_numpy(k.view(np.int32)).to(dev)
    vt = torch.from_numpy(v.view(np.int32)).to(dev)
    ks, vs = RankKernels.sort(kt, vt)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(ks.cpu().numpy().view(np.uint32), k[order])
    np.testing.assert_array_equal(vs.cpu().numpy().view(np.uint32), v[order])


# ------------------------------------------------- bootstrap beyond the rank plans (n > 65,535)
def test_bootstrap_full_equals_engine(dev):
    # the plan-free per-draw path (bootstrap_full: sub-RDMs read in place) against the rank-plan
    # engines on the same RDMs and RandomState(42) draws: exact integer statistics, bit for bit,
    # Spearman and Kendall
    from visreps_amd.analysis._random import bootstrap_indices

    n = 2500
    g = torch.Generator(device=dev).manual_seed(5)
    z = torch.randn(n, 16, device=dev, generator=g)
    a = R.compute_rdm(torch.relu(z @ torch.randn(16, 80, device=dev, generator=g) + torch.randn(n, 80, device=dev,
                                                                                            generator=g)))
    b = R.compute_rdm(z + torch.randn(n, 16, device=dev, generator=g))
    idx = bootstrap_indices(42, n, int(0.9 * n), 12)
    for method in ("spearman", "kendall"):
        full = R.bootstrap_full(a, b, idx, method=method).cpu().numpy()
        eng = R._ENGINES[method](R.RankPlan(a), R.RankPlan(b), idx, full_first=True).cpu().numpy()
        assert np.array_equal(full, eng), method


def test_bootstrap_rsa_beyond_rank_plans(dev):
    # n = 70,000 (> 65,535): bootstrap_rsa runs the per-draw plan-free path; a draw's score equals
    # spearman_full on the explicitly materialised sub-RDMs A[idx][:, idx] (the reference's
    # evals.py:362-364 indexing), the point equals spearman_full on the whole RDMs
    from visreps_amd.analysis._random import bootstrap_indices

    n = 70000
    g = torch.Generator(device=dev).manual_seed(70)
    z = torch.randn(n, 24, device=dev, generator=g)
    a = R.compute_rdm(z + 0.7 * torch.randn(n, 24, device=dev, generator=g))
    b = R.compute_rdm(z + 0.7 * torch.randn(n, 24, device=dev, generator=g))
    del z
    idx = bootstrap_indices(42, n, int(0.9 * n), 2)
    point, scores, lo, hi = R.bootstrap_rsa(a, b, idx=idx)
    assert point == R.spearman_full(a, b)
    i = torch.as_tensor(idx[1], dtype=torch.long, device=dev)
    sa = a[i][:, i]
    sb = b[i][:, i]
    assert scores[1] == R.spearman_full(sa, sb)
    assert lo <= hi and 0.0 < point < 1.0


# ------------------------------------------- bf16 features: one MFMA product per k (configs[4])
def _rdm_rows_f64(x, rows):
    xd = x.double()
    xd = xd - xd.mean(1, keepdim=True)
    s = torch.sqrt((xd * xd).mean(1) + 1e-12)
    g = xd[rows] @ xd.T / x.size(1)
    out = 1.0 - (g / (s[rows, None] * s[None, :] + 1e-12)).clamp(-1, 1)
    out[torch.arange(len(rows), device=x.device), rows] = 0.0
    return out


@pytest.mark.parametrize("n,d", [(3000, 4128), (700, 768), (1300, 50000)])
def test_bf16_one_product_rdm(dev, n, d, monkeypatch):
    # bf16 rows: sum x_i x_j on one bf16 MFMA product per k (exact products, fp32 accumulation)
    # and the centring as the epilogue's rank-1 correction; against fp64 rows it must do no
    # worse than the split (hi/lo, 3 products) kernel or the exact-fp32 kernel (the parity bar of
    # tests/test_benchsize.py::test_cfg5_*); exact symmetry and zero diagonal; rows whose mean is
    # large against their spread (mean^2 > 4 var) send the call to the split records, bit-equal
    # to VISREPS_GRAM_ONE=0
    g = torch.Generator(device=dev).manual_seed(n + d)
    z = torch.randn(n, 32, device=dev, generator=g)
    x = (z @ torch.randn(32, d, device=dev, generator=g) / 4 + torch.randn(n, d, device=dev, generator=g)).to(
        torch.bfloat16)
    rows = torch.randperm(n, device=dev, generator=g)[:48]
    ref = _rdm_rows_f64(x.float(), rows)
    one = R.compute_rdm(x)
    monkeypatch.setenv("VISREPS_GRAM_ONE", "0")
    split = R.compute_rdm(x)
    monkeypatch.setenv("VISREPS_GRAM", "fp32")
    fp32 = R.compute_rdm(x.float())
    monkeypatch.delenv("VISREPS_GRAM")
    e1 = float((one[rows].double() - ref).abs().max())
    e3 = float((split[rows].double() - ref).abs().max())
    e32 = float((fp32[rows].double() - ref).abs().max())
    from conftest import record_margin
    record_margin("bf16_one_product_rdm", n=n, d=d, err_one=e1, err_split=e3, err_fp32=e32)
    assert e1 <= max(5e-6, e3, e32), (e1, e3, e32)
    assert torch.all(torch.diagonal(one) == 0) and torch.equal(one, one.T)
    # large means: the split records (flag), the same bits as forcing them
    xm = (x.float() + 8.0).to(torch.bfloat16)
    forced = R.compute_rdm(xm)
    monkeypatch.delenv("VISREPS_GRAM_ONE")
    assert torch.equal(R.compute_rdm(xm), forced)
