"""Parity at the bench's own sizes and precision (BASELINE.json configs[1], [2], [4]).

The bench builds every Gram with the bf16x3 split kernel (n^2 d >= 1e10), so these tests
check that kernel on the bench's own inputs against float64 ground truth:

* configs[1] (N = 10k): the 14 CustomCNN points of the bench (random-init weights,
  synthetic images: exactly bench.py's features, D = 290,400 ... 4,096) and the §8(d)
  synthetic features at D = 290,400 / 186,624 / 43,264:
    - RDM rows vs a float64 recomputation on 64 sampled rows: no worse than the exact-fp32
      kernel's RDM on the same inputs (or 5e-6). Any fp32 Gram, the reference's CPU sgemm
      included, accumulates rounding over D terms; on the bench's post-ReLU points (all
      products positive) the exact-fp32 kernel is off by up to 5.7e-4 and the split kernel,
      whose MFMAs add 16 products per fp32 rounding, by up to 1.9e-4
      (profiles/r2_gram_accuracy.log);
    - point + all 1000 bootstrap Spearman scores (RandomState(42) subsets, evals.py:355-373)
      of the split RDMs vs the same scores of the float64 RDMs rounded to fp32 (the RDM
      an exact reference would produce), and of the exact-fp32 kernel's RDMs
      (VISREPS_GRAM=fp32): |dSpearman| < 1e-5, the north-star tolerance.
* configs[2]: the 73k x 43,264 RDM (one GPU), float64 rows, exact symmetry, zero diagonal.
* configs[4]: ViT-B/16 block tokens (D = 151,296) and the CLS embedding in bf16 at
  N = 50k, RDM straight from the bf16 features (no fp32 copy), float64 rows.

Reference semantics: rsa.py:59-93 (RDM), rsa.py:96-129 (Spearman), evals.py:341-373.
"""
import os

import numpy as np
import pytest
import torch

from conftest import record_margin
from oracle import rsa_oracle as O
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices

pytestmark = pytest.mark.gpu

N, NB = 10000, 1000
SPEARMAN_TOL = 1e-5  # BASELINE.json north_star: |dSpearman| < 1e-5 vs CPU
ROW_TOL = 5e-6       # floor of the row bound; otherwise the exact-fp32 kernel's own error


class gram_mode:
    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        self.old = os.environ.get("VISREPS_GRAM")
        os.environ["VISREPS_GRAM"] = self.mode

    def __exit__(self, *a):
        if self.old is None:
            os.environ.pop("VISREPS_GRAM", None)
        else:
            os.environ["VISREPS_GRAM"] = self.old


def _centred_f64(x):
    xd = x.double()
    xd -= xd.mean(1, keepdim=True)
    s = torch.sqrt((xd * xd).mean(1) + 1e-12)
    return xd, s


def _row_stats_f64(x, chunk=4096):
    """float64 row means and stds of x, without a float64 copy of all of x."""
    m = torch.empty(x.size(0), dtype=torch.float64, device=x.device)
    s = torch.empty_like(m)
    for c0 in range(0, x.size(0), chunk):
        xd = x[c0:c0 + chunk].double()
        m[c0:c0 + chunk] = xd.mean(1)
        xd -= m[c0:c0 + chunk, None]
        s[c0:c0 + chunk] = torch.sqrt((xd * xd).mean(1) + 1e-12)
    return m, s


def rdm_f64_rows(x, rows, chunk=4096):
    """float64 RDM rows `rows` of x (rsa.py:76-92 in exact arithmetic), built from column
    chunks so x is never copied to float64 whole."""
    m, s = _row_stats_f64(x, chunk)
    xr = x[rows].double() - m[rows, None]
    g = torch.empty((len(rows), x.size(0)), dtype=torch.float64, device=x.device)
    for c0 in range(0, x.size(0), chunk):
        xc = x[c0:c0 + chunk].double() - m[c0:c0 + chunk, None]
        g[:, c0:c0 + chunk] = xr @ xc.T
    g /= x.size(1)
    out = 1.0 - (g / (s[rows, None] * s[None, :] + 1e-12)).clamp(-1, 1)
    out[torch.arange(len(rows), device=x.device), rows] = 0.0
    return out


def rdm_f64(x, block=2048):
    """Whole float64 RDM of x, rounded to fp32 (what an exact-arithmetic reference
    compute_rdm would return)."""
    xd, s = _centred_f64(x)
    n = x.size(0)
    out = torch.empty((n, n), dtype=torch.float32, device=x.device)
    for r0 in range(0, n, block):
        r1 = min(n, r0 + block)
        g = xd[r0:r1] @ xd.T / x.size(1)
        c = (g / (s[r0:r1, None] * s[None, :] + 1e-12)).clamp(-1, 1)
        c[torch.arange(r1 - r0, device=x.device), torch.arange(r0, r1, device=x.device)] = 1.0
        out[r0:r1] = (1.0 - c).float()
    del xd
    return out


def _rows(dev, n, seed=1):
    return torch.randperm(n, device=dev, generator=torch.Generator(device=dev).manual_seed(seed))[:64]


def _row_err(rdm, x, rows):
    return float((rdm[rows].double() - rdm_f64_rows(x, rows)).abs().max())


def _fp32_rdm(x):
    with gram_mode("fp32"):
        return R.compute_rdm(x.float())


def _scores(a, b, idx):
    return R.bootstrap_spearman(R.RankPlan(a), R.RankPlan(b), idx, full_first=True).cpu().numpy()


@pytest.fixture(scope="module")
def idx():
    return bootstrap_indices(42, N, int(0.9 * N), NB)


# ----------------------------------------------------------------------------- configs[2]
# (first in the module: they need ~130 GB of device memory before the module-scoped bench
# features are created)
def test_cfg3_73k_rdm(dev):
    n, d = 73000, 43264
    g = torch.Generator(device=dev).manual_seed(7)
    z = torch.randn(n, 64, device=dev, generator=g)
    x = z @ (torch.randn(64, d, device=dev, generator=g) / 8)
    x += 2 * torch.randn(n, d, device=dev, generator=g)
    x.relu_()
    del z
    rdm = R.compute_rdm(x)
    rows = _rows(dev, n, 5)
    err = _row_err(rdm, x, rows)
    err32 = _row_err(_fp32_rdm(x), x, rows)
    assert err <= max(ROW_TOL, err32), (err, err32)
    assert torch.all(torch.diagonal(rdm) == 0)
    cols = _rows(dev, n, 6)
    assert torch.equal(rdm[rows][:, cols], rdm[cols][:, rows].T)  # exact symmetry, sampled
    assert torch.all(rdm[rows] >= 0) and torch.all(rdm[rows] <= 2)
    # configs[2]'s full-triangle Spearman (2.66e9 pairs) on the plan-free path: exact
    # properties of the rank statistic at full size (the arithmetic itself is pinned to the
    # rank-plan engine and scipy at small n, tests/test_gpu_parity.py, and at n = 65535 below)
    del x
    torch.cuda.empty_cache()
    r_aa = R.compute_rdm_correlation(rdm, rdm, correlation="Spearman")
    assert abs(r_aa - 1.0) <= 1e-12
    neg = -rdm  # the reversed order, same ties
    assert abs(R.spearman_full(rdm, neg) + 1.0) <= 1e-12
    del neg
    other = rdm.clone()
    other[:, : n // 2] = other[:, : n // 2].sqrt()  # monotone on half the columns only
    other = torch.minimum(other, other.T)  # symmetric again
    r_ab = R.spearman_full(rdm, other)
    assert R.spearman_full(other, rdm) == r_ab and 0.5 < r_ab < 1.0


def test_spearman_full_equals_engine_at_plan_limit(dev):
    # n = 65535 (2.15e9 pairs), the largest rank plan: the plan-free full Spearman and the
    # rank-plan engine are both exact integer statistics and must agree bit for bit
    n = 65535
    g = torch.Generator(device=dev).manual_seed(11)
    z = torch.randn(n, 32, device=dev, generator=g)
    a = R.compute_rdm(z + 0.5 * torch.randn(n, 32, device=dev, generator=g))
    b = R.compute_rdm(z + 0.5 * torch.randn(n, 32, device=dev, generator=g))
    del z
    full = R.spearman_full(a, b)
    eng = R.compute_rdm_correlation(a, b, correlation="Spearman")
    assert full == eng and 0.0 < full < 1.0


# ------------------------------------------------------------------------ bench features
@pytest.fixture(scope="module")
def bench(dev):
    """bench.py's inputs: random-init CustomCNN (seed 0), 10k synthetic images, the 14
    flattened points, and the V1 responses."""
    import os

    # bench.py switches on cudnn.benchmark and MIOpen's find mode at import; the later
    # modules' exact-equality tests extract twice and need one fixed algorithm per shape
    prev = torch.backends.cudnn.benchmark, os.environ.get("MIOPEN_FIND_MODE")
    from bench import LAYERS, extract
    torch.backends.cudnn.benchmark = prev[0]
    if prev[1] is None:
        os.environ.pop("MIOPEN_FIND_MODE", None)
    else:
        os.environ["MIOPEN_FIND_MODE"] = prev[1]
    from visreps_amd.dataloaders.synthetic import NSD_ROIS_4, make_images, make_responses
    from visreps_amd.models.custom_model import CustomCNN
    from visreps_amd.models.utils import FeatureExtractor

    torch.manual_seed(0)
    model = CustomCNN(num_classes=1000).to(dev).eval()
    ex = FeatureExtractor(model, LAYERS, extract_pre_and_post=True)
    images = make_images(range(N), device=dev)
    ys = make_responses(images, range(N), NSD_ROIS_4)  # the bench's 4 regions (V1 first)
    y = ys["V1"]
    feats = extract(ex, images, 128)
    del images
    neural_split = R.compute_rdm(y)
    neural_64 = rdm_f64(y)
    with gram_mode("fp32"):
        neural_32 = R.compute_rdm(y)
    return feats, neural_split, neural_64, neural_32, y, ys


POINTS = [f"{l}_{s}" for l in ["conv1", "conv2", "conv3", "conv4", "conv5", "fc1", "fc2"]
          for s in ("pre", "post")]


@pytest.mark.parametrize("point", POINTS)
def test_bench_point_split_gram_parity(dev, bench, idx, point):
    feats, neural_split, neural_64, neural_32 = bench[:4]
    x = feats[point]
    assert x.size(0) == N
    rdm = R.compute_rdm(x)
    rdm32 = _fp32_rdm(x)
    rows = _rows(dev, N)
    err, err32 = _row_err(rdm, x, rows), _row_err(rdm32, x, rows)
    assert err <= max(ROW_TOL, err32), (point, x.size(1), err, err32)
    assert torch.all(torch.diagonal(rdm) == 0)
    ref64 = rdm_f64(x)
    s_split = _scores(rdm, neural_split, idx)
    s_64 = _scores(ref64, neural_64, idx)
    s_32 = _scores(rdm32, neural_32, idx)
    d64 = float(np.max(np.abs(s_split - s_64)))
    d32 = float(np.max(np.abs(s_split - s_32)))
    record_margin("bench_point_split_gram", point=point, d=x.size(1), rdm_err_split=err, rdm_err_fp32=err32,
                  dspearman_split_vs_f64=d64, dspearman_split_vs_fp32=d32,
                  dspearman_fp32_vs_f64=float(np.max(np.abs(s_32 - s_64))), n_scores=len(s_split))
    assert d64 < SPEARMAN_TOL, (point, d64)
    assert d32 < SPEARMAN_TOL, (point, d32)
    assert float(np.max(np.abs(s_32 - s_64))) < SPEARMAN_TOL


ORACLE_POINTS = ["conv2_post", "conv5_post", "fc1_post"]
# 0-based draws scored by the oracle beyond the first 5: bootstraps #64, #65, #500, #1000.
# With the full set in lane 0 of pass 0, draws 0-62 run in pass 0 (EST 4) and draws 63-999
# in the EST 3 passes -- the k_rankB form behind 840 of the step's 952 B walks.
LATE_DRAWS = [63, 64, 499, 999]


@pytest.mark.parametrize("point", ORACLE_POINTS)
def test_bench_point_vs_cpu_oracle(dev, bench, point):
    """Full-size parity against the CPU oracle itself: the product's
    default path (split-Gram RDMs on the GPU, rank-plan engine, 1000 bootstraps in one call
    as the bench runs them) for the point Spearman, the first 5 bootstraps of
    RandomState(42) and bootstraps #64/#65/#500/#1000 (EST 3 passes) vs the oracle --
    numpy float32 RDMs and scipy.stats.spearmanr, the reference's arithmetic
    (rsa.py:59-129, evals.py:341-373) -- on the bench's own N = 10k features."""
    from visreps_amd._lib import lib

    feats = bench[0]
    x = feats[point]
    gm = R.compute_rdm(x)
    gn = R.compute_rdm(bench[4])
    r0, t0 = int(lib().vr_engine_est_reruns()), int(lib().vr_engine_est_tail_flags())
    point_g, scores_g, _, _ = R.bootstrap_rsa(gm, gn, n_bootstrap=NB, seed=42)
    reruns = int(lib().vr_engine_est_reruns()) - r0
    tail = int(lib().vr_engine_est_tail_flags()) - t0
    del gm, gn
    torch.cuda.empty_cache()
    point_o, scores_o, late_o = _oracle_results(bench)[point].result()
    dp = abs(point_g - point_o)
    db = float(np.max(np.abs(np.asarray(scores_g[:5]) - scores_o)))
    dl = max(abs(float(scores_g[i]) - late_o[i]) for i in LATE_DRAWS)
    record_margin("bench_point_vs_cpu_oracle", point=point, d=x.size(1), point_hip=point_g, point_oracle=point_o,
                  dspearman_point=dp, dspearman_boot5=db, dspearman_late_draws=dl, late_draws=LATE_DRAWS,
                  est_reruns=reruns, est_tail_flags=tail)
    assert tail == 0, "B-side invariant broken on the bench's own RDMs"
    assert dp < SPEARMAN_TOL and db < SPEARMAN_TOL and dl < SPEARMAN_TOL, (point, dp, db, dl)


GRID_POINTS = ["conv1_pre", "conv5_post", "fc1_post"]


def test_bench_grid_walk_full_size(dev, bench, idx):
    """the region-fused grid walk (k_rankB_grid, the bench's dominant kernel)
    at the bench's own size -- N = 10k, the 4 regions' neural RDMs, 1000 RandomState(42)
    bootstraps, model plans conv1_pre / conv5_post / fc1_post:
      * all 4 x 3 x 1001 scores bit-equal to one joined per-region multi call per region;
      * the conv5_post x V1 unit's point, first 5 draws and draws #64/#65/#500/#1000 vs the
        CPU oracle (numpy RDMs + scipy spearmanr, evals.py:341-373);
      * pipeline.all_units_rsa (the bench's route into the grid) equal to per-unit
        bootstrap_rsa for two units, every score and both percentiles."""
    from visreps_amd._lib import ktimer_enable, ktimer_read, lib
    from visreps_amd.pipeline import all_units_rsa

    feats, ys = bench[0], bench[5]
    regions = list(ys)
    rdms_n = {r: R.compute_rdm(ys[r]) for r in regions}
    pns = [R.RankPlan(rdms_n[r]) for r in regions]
    pms = [R.RankPlan(R.compute_rdm(feats[p])) for p in GRID_POINTS]
    sj = R.SharedJoins(pns)
    joins = [sj.join(pm) for pm in pms]  # joins[m][a]
    del sj
    r0, t0 = int(lib().vr_engine_est_reruns()), int(lib().vr_engine_est_tail_flags())
    ktimer_enable(True)
    grid = R.bootstrap_spearman_grid(pns, pms, idx, joins, full_first=True).cpu().numpy()
    launches = ktimer_read("k_rankB_grid")[1]
    ktimer_enable(False)
    assert int(lib().vr_engine_est_reruns()) == r0 and int(lib().vr_engine_est_tail_flags()) == t0
    assert launches == (NB + 1 + 63) // 64 * len(GRID_POINTS) - len(GRID_POINTS), launches  # pass 0: its own slot
    assert grid.shape == (len(regions), len(GRID_POINTS), NB + 1) and np.all(np.isfinite(grid))
    n_equal = 0
    for a, pn in enumerate(pns):
        ref = R.bootstrap_spearman_multi(pn, pms, idx, full_first=True,
                                         joined=[joins[m][a] for m in range(len(pms))]).cpu().numpy()
        assert np.array_equal(grid[a], ref), regions[a]
        n_equal += ref.size
    del joins
    u = grid[regions.index("V1"), GRID_POINTS.index("conv5_post")]
    point_o, boot5_o, late_o = _oracle_results(bench)["conv5_post"].result()
    dp = abs(float(u[0]) - point_o)
    db = float(np.max(np.abs(u[1:6] - boot5_o)))
    dl = max(abs(float(u[1 + i]) - late_o[i]) for i in LATE_DRAWS)
    # the bench's route: all_units_rsa over the 4 regions runs them as one grid call
    ktimer_enable(True)
    res = all_units_rsa(lambda p: R.compute_rdm(feats[p]), GRID_POINTS, rdms_n, N, n_boot=NB, seed=42)
    routed = ktimer_read("k_rankB_grid")[1]
    ktimer_enable(False)
    assert routed == launches, "all_units_rsa did not take the grid walk"
    for p, r in [("conv5_post", "V1"), ("fc1_post", "hV4")]:
        point, scores, lo, hi = R.bootstrap_rsa(R.compute_rdm(feats[p]), rdms_n[r], n_bootstrap=NB, seed=42)
        v = res[(p, r)]
        assert v["score"] == point and v["ci_low"] == lo and v["ci_high"] == hi, (p, r)
        assert np.array_equal(np.asarray(v["bootstrap_scores"]), scores), (p, r)
        assert np.array_equal(grid[regions.index(r), GRID_POINTS.index(p)][1:], scores), (p, r)
    record_margin("bench_grid_full_size", n=N, regions=len(regions), model_plans=len(GRID_POINTS),
                  scores_bit_equal_per_region=n_equal, grid_launches=launches, dspearman_point=dp,
                  dspearman_boot5=db, dspearman_late_draws=dl, late_draws=LATE_DRAWS)
    assert dp < SPEARMAN_TOL and db < SPEARMAN_TOL and dl < SPEARMAN_TOL, (dp, db, dl)


class _engine_form:
    def __init__(self, value):
        self.value = value

    def __enter__(self):
        self.old = os.environ.get("VISREPS_ENGINE_EST")
        os.environ["VISREPS_ENGINE_EST"] = self.value

    def __exit__(self, *a):
        if self.old is None:
            os.environ.pop("VISREPS_ENGINE_EST", None)
        else:
            os.environ["VISREPS_ENGINE_EST"] = self.old


def structured_rdm(dev, n, seed=7):
    """A neural RDM with strong per-stimulus effects (d_ab = u_a + u_b + 0.05 noise, u ~
    Exp(1)^2): bench.structured_est_probe's RDM, where the wave-uniform EST 3 estimate
    drifts furthest from the subsets' true counts."""
    g = torch.Generator(device=dev).manual_seed(seed)
    u = torch.empty(n, device=dev).exponential_(1.0, generator=g) ** 2
    a = u[:, None] + u[None, :] + 0.05 * torch.rand(n, n, device=dev, generator=g)
    a = torch.triu(a, 1)
    return a + a.T


def test_bench_unit_est_equals_exact_form(dev, bench, idx):
    """at N = 10k, all 1001 scores of bench units (conv5_post and conv1_post
    x V1) and of the structured neural RDM against conv5_post are bit-equal between the
    default EST form (whatever it flags and re-runs) and VISREPS_ENGINE_EST=0 (every pass in
    the exact chunk-base form)."""
    from visreps_amd._lib import lib

    feats, neural_split = bench[0], bench[1]
    pn = R.RankPlan(neural_split)
    pms = [R.RankPlan(R.compute_rdm(feats[p])) for p in ("conv5_post", "conv1_post")]
    ps = R.RankPlan(structured_rdm(dev, N))
    out = {}
    for form in ("1", "0"):
        with _engine_form(form):
            r0 = int(lib().vr_engine_est_reruns())
            units = R.bootstrap_spearman_multi(pn, pms, idx, full_first=True).cpu().numpy()
            st = R.bootstrap_spearman(pms[0], ps, idx, full_first=True).cpu().numpy()
            out[form] = (units, st, int(lib().vr_engine_est_reruns()) - r0)
    (u_est, s_est, reruns), (u_ex, s_ex, _) = out["1"], out["0"]
    record_margin("bench_unit_est_vs_exact", n_scores=int(u_est.size + s_est.size), est_reruns=reruns,
                  units_equal=bool(np.array_equal(u_est, u_ex)), structured_equal=bool(np.array_equal(s_est, s_ex)))
    assert u_est.shape == (2, NB + 1) and np.all(np.isfinite(u_est)) and np.all(np.isfinite(s_est))
    assert np.array_equal(u_est, u_ex)
    assert np.array_equal(s_est, s_ex)


_ORACLE_RUNS = {}


def _oracle_results(bench):
    """The three points' oracle runs (numpy RDMs + 10 scipy Spearmans at N = 10k / k = 9000,
    ~80 s each on the host) started together on threads at first use (numpy's sorts and BLAS
    release the GIL), so the three tests cost about one oracle run of wall time."""
    if not _ORACLE_RUNS:
        from concurrent.futures import ThreadPoolExecutor
        on = O.compute_rdm(bench[4].cpu().numpy())
        xs = {p: bench[0][p].cpu().numpy() for p in ORACLE_POINTS}

        def run(p):
            om = O.compute_rdm(xs[p])
            point, boot5 = O.bootstrap_rsa(om, on, n_bootstrap=5, seed=42)[:2]
            return point, boot5, O.bootstrap_scores_at(om, on, LATE_DRAWS, seed=42)

        pool = ThreadPoolExecutor(len(ORACLE_POINTS))
        _ORACLE_RUNS.update({p: pool.submit(run, p) for p in ORACLE_POINTS})
        pool.shutdown(wait=False)
    return _ORACLE_RUNS


# ------------------------------------------------------------------ §8(d) synthetic widths
@pytest.mark.parametrize("d", [290400, 186624, 43264])
def test_synthetic_width_split_gram_parity(dev, idx, d):
    g = torch.Generator(device=dev).manual_seed(20260306)
    z = torch.randn(N, 64, device=dev, generator=g)
    x = z @ (torch.randn(64, d, device=dev, generator=g) / 8)
    x += 2 * torch.randn(N, d, device=dev, generator=g)
    x.relu_()
    y = z @ torch.randn(64, 2000, device=dev, generator=g) + 3 * torch.randn(N, 2000, device=dev, generator=g)
    rdm = R.compute_rdm(x)
    rows = _rows(dev, N, 3)
    err, err32 = _row_err(rdm, x, rows), _row_err(_fp32_rdm(x), x, rows)
    assert err <= max(ROW_TOL, err32), (d, err, err32)
    s_split = _scores(rdm, R.compute_rdm(y), idx)
    s_64 = _scores(rdm_f64(x), rdm_f64(y), idx)
    d64 = float(np.max(np.abs(s_split - s_64)))
    record_margin("synthetic_width_split_gram", d=d, rdm_err_split=err, rdm_err_fp32=err32,
                  dspearman_split_vs_f64=d64)
    assert d64 < SPEARMAN_TOL


# ----------------------------------------------------------------------------- configs[4]
@pytest.fixture(scope="module")
def vit_tokens(dev):
    """ViT-B/16 (random init, torchvision layout) on 50k synthetic images in bf16: the
    tokens of encoder block 6 (197 x 768 = 151,296 features) and the final CLS."""
    from visreps_amd.dataloaders.synthetic import make_images
    from visreps_amd.models.standard_model import ViTBase
    from visreps_amd.models.utils import FeatureExtractor

    n = 50000
    torch.manual_seed(0)
    model = ViTBase("none").to(dev).eval().to(torch.bfloat16)
    ex = FeatureExtractor(model, ["block6"], extract_pre_and_post=False)
    block = torch.empty((n, 197 * 768), dtype=torch.bfloat16, device=dev)
    cls = torch.empty((n, 768), dtype=torch.bfloat16, device=dev)
    with torch.no_grad():
        for b0 in range(0, n, 1000):
            imgs = make_images(range(b0, b0 + 1000), device=dev, dtype=torch.bfloat16)
            ex.features = {}
            tokens = model.forward_features(imgs)  # fires the block6 hook
            block[b0:b0 + 1000] = ex.features["block6"].reshape(1000, -1)
            cls[b0:b0 + 1000] = tokens[:, 0]
    return block, cls


@pytest.mark.parametrize("which", ["block6", "cls"])
def test_cfg5_vit_bf16_rdm(dev, vit_tokens, which):
    x = vit_tokens[0] if which == "block6" else vit_tokens[1]
    assert x.dtype == torch.bfloat16
    rdm = R.compute_rdm(x)  # bf16 kernels: no fp32 copy of the features
    assert rdm.dtype == torch.float32 and rdm.shape == (x.size(0), x.size(0))
    rows = _rows(dev, x.size(0), 9)
    err = _row_err(rdm, x.float(), rows)
    err32 = _row_err(_fp32_rdm(x), x.float(), rows)
    assert err <= max(ROW_TOL, err32), (which, err, err32)
    assert torch.all(torch.diagonal(rdm) == 0)
    cols = _rows(dev, x.size(0), 10)
    assert torch.equal(rdm[rows][:, cols], rdm[cols][:, rows].T)


def _foundation_feats(dev, model, extract_fn, n=50000, batch=500):
    from visreps_amd.dataloaders.synthetic import make_images

    feats = None
    with torch.no_grad():
        for b0 in range(0, n, batch):
            imgs = make_images(range(b0, b0 + batch), device=dev, dtype=torch.bfloat16)
            f = extract_fn(model, imgs)
            if feats is None:
                feats = torch.empty((n, f.size(1)), dtype=torch.bfloat16, device=dev)
            feats[b0:b0 + batch] = f
    return feats


@pytest.mark.parametrize("which", ["clip", "dino", "vitl"])
def test_cfg5_foundation_bf16_rdm(dev, which):
    """configs[4]'s CLIP ViT-L/14 image embedding (encode_image / its norm), the DINOv3
    ViT-L/16 CLS and the supervised ViT-L/16 CLS (vit_representations.py's default model),
    random init, bf16, on 50k synthetic images: bf16 RDM, fp64 rows."""
    from visreps_amd import extract_representations as X
    from visreps_amd.models.foundation import clip_vit_l14, dinov3_vit_l16
    from visreps_amd.models.standard_model import vit_large_patch16_224

    torch.manual_seed(0)
    if which == "clip":
        model, fn = X.clip_image(clip_vit_l14().to(dev).eval().to(torch.bfloat16))
    elif which == "dino":
        model, fn = X.dino_cls(dinov3_vit_l16().to(dev).eval().to(torch.bfloat16))
    else:
        model, fn = X.vit_cls(vit_large_patch16_224().to(dev).eval().to(torch.bfloat16))
    x = _foundation_feats(dev, model, fn)
    del model
    torch.cuda.empty_cache()
    assert x.dtype == torch.bfloat16 and x.shape == (50000, 768 if which == "clip" else 1024)
    if which == "vitl":  # unit rows (the dump's F.normalize), to bf16 rounding
        assert torch.allclose(x[:64].float().norm(dim=1), torch.ones(64, device=dev), atol=1e-2)
    assert torch.isfinite(x).all()
    rdm = R.compute_rdm(x)
    rows = _rows(dev, x.size(0), 11)
    err = _row_err(rdm, x.float(), rows)
    err32 = _row_err(_fp32_rdm(x), x.float(), rows)
    assert err <= max(ROW_TOL, err32), (which, err, err32)
    assert torch.all(torch.diagonal(rdm) == 0)
    cols = _rows(dev, x.size(0), 12)
    assert torch.equal(rdm[rows][:, cols], rdm[cols][:, rows].T)
