"""The bootstrap engine's one-gather-per-pair (EST) pass form against its exact chunk-base
form and the CPU oracle.

EST keeps each pair's absolute doubled A rank modulo 2^16 and recovers it on the B side
from an estimate of the included-pair count (EST 3, the default: one wave-uniform linear
estimate, the pass holding the full set run exact; EST 1: an interpolated per-lane table in
LDS; EST 2: a per-lane linear estimate); a pass whose ranks cannot be recovered is re-run
in the exact form. Both forms are exact integer arithmetic, so scores must agree bit for bit
(VISREPS_ENGINE_EST=1 selects the EST form, =0 the exact form, for every pass;
VISREPS_ENGINE_EST_MODE the estimate).
"""
import os

import numpy as np
import pytest
import torch

from oracle import rsa_oracle as O
from visreps_amd._lib import lib
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices

pytestmark = pytest.mark.gpu


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


def exact_engine():
    """Context: every engine pass in the exact chunk-base form."""
    return _engine_form("0")


@pytest.fixture(autouse=True)
def est_engine():
    """Every test of this module runs the EST form unless it asks for the exact one."""
    with _engine_form("1"):
        yield


def _rdm(dev, n, d, seed, relu=False):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(n, d, device=dev, generator=g)
    return R.compute_rdm(torch.relu(x) if relu else x)


@pytest.mark.parametrize("n,nb", [(40, 70), (700, 200), (3000, 130)])
def test_est_equals_exact_form(dev, n, nb):
    a, b = _rdm(dev, n, 64, 1, relu=True), _rdm(dev, n, 300, 2)
    idx = bootstrap_indices(42, n, int(0.9 * n), nb)
    pa, pb = R.RankPlan(a), R.RankPlan(b)
    r0 = int(lib().vr_engine_est_reruns())
    est = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert int(lib().vr_engine_est_reruns()) == r0, "continuous RDMs must not need the exact re-run"
    with exact_engine():
        ref = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert np.array_equal(est, ref)


def test_est_multi_equals_exact_form(dev):
    n = 1500
    neural = R.RankPlan(_rdm(dev, n, 200, 3))
    models = [R.RankPlan(_rdm(dev, n, 50 * (i + 1), 10 + i, relu=i % 2 == 0)) for i in range(4)]
    idx = bootstrap_indices(42, n, int(0.9 * n), 100)
    est = R.bootstrap_spearman_multi(neural, models, idx, full_first=True).cpu().numpy()
    with exact_engine():
        ref = R.bootstrap_spearman_multi(neural, models, idx, full_first=True).cpu().numpy()
    assert np.array_equal(est, ref)
    for j, pm in enumerate(models):  # and each row equals the per-unit call
        one = R.bootstrap_spearman(pm, neural, idx, full_first=True).cpu().numpy()
        assert np.array_equal(est[j], one)


def test_est_triangle_entry_point_matches_oracle(dev):
    # vr_spearman_triu_f32 runs one lane (lw = 1, FULL = false) in the EST form
    n = 900
    a, b = _rdm(dev, n, 40, 5), _rdm(dev, n, 70, 6, relu=True)
    got = R.compute_rdm_correlation(a, b, correlation="Spearman")
    ref = O.compute_rdm_correlation(a.cpu().numpy(), b.cpu().numpy(), "Spearman")
    assert abs(got - ref) <= 1e-12


def test_est_giant_tie_groups_fall_back_to_exact(dev):
    # Five distinct RDM values over 499,500 pairs: tie groups of ~100k positions, whose
    # shared midrank is ~80k counts from the interpolated estimate at the group ends, so
    # EST flags the passes and they are re-run in the exact form (u32 chunk ranks, 128-bit
    # tie sums). Scores must equal the exact form and the oracle.
    n = 1000
    rs = np.random.RandomState(0)
    vals = rs.randint(0, 5, size=(n, n)).astype(np.float32) / 4.0
    a = np.triu(vals, 1)
    a = a + a.T
    b = np.triu(rs.rand(n, n).astype(np.float32), 1)
    b = b + b.T
    ta, tb = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    idx = bootstrap_indices(42, n, int(0.9 * n), 70)
    pa, pb = R.RankPlan(ta), R.RankPlan(tb)
    r0 = int(lib().vr_engine_est_reruns())
    est = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert int(lib().vr_engine_est_reruns()) > r0, "giant tie groups must trigger the exact re-run"
    with exact_engine():
        ref = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert np.array_equal(est, ref)
    # oracle: point + the first 3 subsets (scipy on the explicit sub-RDMs)
    assert abs(est[0] - O.compute_rdm_correlation(a, b, "Spearman")) <= 1e-12
    for s in range(3):
        i = np.asarray(idx[s])
        ref_s = O.compute_rdm_correlation(a[np.ix_(i, i)], b[np.ix_(i, i)], "Spearman")
        assert abs(est[1 + s] - ref_s) <= 1e-12


@pytest.mark.parametrize("mode", ["1", "2", "3"])
def test_est_modes_equal_exact_form(dev, mode, monkeypatch):
    # every estimate form, a partial last pass (201 subsets: lanes 9..63 hold no subset)
    monkeypatch.setenv("VISREPS_ENGINE_EST_MODE", mode)
    n = 2500
    neural = R.RankPlan(_rdm(dev, n, 120, 21))
    models = [R.RankPlan(_rdm(dev, n, 90, 22, relu=True)), R.RankPlan(_rdm(dev, n, 300, 23))]
    idx = bootstrap_indices(42, n, int(0.9 * n), 200)
    r0 = int(lib().vr_engine_est_reruns())
    est = R.bootstrap_spearman_multi(neural, models, idx, full_first=True).cpu().numpy()
    assert int(lib().vr_engine_est_reruns()) == r0, "continuous RDMs must not need the exact re-run"
    with exact_engine():
        ref = R.bootstrap_spearman_multi(neural, models, idx, full_first=True).cpu().numpy()
    assert np.array_equal(est, ref)


@pytest.mark.parametrize("n,nb", [(2500, 200), (700, 64)])
def test_triangle_order_form_equals_exact_form(dev, n, nb, monkeypatch):
    # EST 5 / 6 (opt-in VISREPS_ENGINE_TRI=1): TB rows at triangle indices, 63 subsets per
    # pass, lane 63 the tag; 201 / 65 draws leave partial last passes
    monkeypatch.setenv("VISREPS_ENGINE_TRI", "1")
    neural = R.RankPlan(_rdm(dev, n, 120, 31))
    models = [R.RankPlan(_rdm(dev, n, 90, 32, relu=True)), R.RankPlan(_rdm(dev, n, 300, 33))]
    idx = bootstrap_indices(42, n, int(0.9 * n), nb)
    r0, t0 = int(lib().vr_engine_est_reruns()), int(lib().vr_engine_est_tail_flags())
    est = R.bootstrap_spearman_multi(neural, models, idx, full_first=True).cpu().numpy()
    assert int(lib().vr_engine_est_reruns()) == r0, "continuous RDMs must not need the exact re-run"
    assert int(lib().vr_engine_est_tail_flags()) == t0
    with exact_engine():
        ref = R.bootstrap_spearman_multi(neural, models, idx, full_first=True).cpu().numpy()
    assert np.array_equal(est, ref)


@pytest.mark.parametrize("n", [5000, 21000])
def test_structured_rdm_leaves_est3_up_front(dev, monkeypatch, n):
    # the heavy per-stimulus effects: the first pass's A counts (k_countA at <= 256
    # boundaries) are already far outside the EST 3 window, so the call leaves EST 3 before
    # spending an EST pass (vr_engine_est_predicted counts it): at n = 5000 (the exact walks'
    # masks in LDS) for the exact form, at 21,000 (masks from L2) for EST 1, whose per-lane tables follow each
    # subset's own counts (vr_engine_est1_fallbacks). The scores equal the exact form, and so do
    # those of VISREPS_ENGINE_EST1_FALLBACK=0; with the check off, the first EST pass is
    # flagged and the call gives up there, same scores.
    g = torch.Generator(device=dev).manual_seed(7)
    u = torch.empty(n, device=dev).exponential_(1.0, generator=g) ** 2
    a = u[:, None] + u[None, :] + 0.05 * torch.rand(n, n, device=dev, generator=g)
    a = torch.triu(a, 1)
    a = a + a.T
    pa, pb = R.RankPlan(a), R.RankPlan(_rdm(dev, n, 90, 41))
    del a
    idx = bootstrap_indices(42, n, int(0.9 * n), 140)
    L = lib()
    p0, f0 = int(L.vr_engine_est_predicted()), int(L.vr_engine_est1_fallbacks())
    est = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert int(L.vr_engine_est_predicted()) - p0 == 1
    assert int(L.vr_engine_est1_fallbacks()) - f0 == (1 if n > 20352 else 0)
    with exact_engine():
        ref = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert np.array_equal(est, ref)
    monkeypatch.setenv("VISREPS_ENGINE_EST1_FALLBACK", "0")
    r0 = int(L.vr_engine_est_reruns())
    ex_up_front = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert int(L.vr_engine_est_reruns()) == r0, "the exact form from the start spends no flagged pass"
    assert np.array_equal(ex_up_front, ref)
    monkeypatch.delenv("VISREPS_ENGINE_EST1_FALLBACK")
    monkeypatch.setenv("VISREPS_ENGINE_EST_PREDICT", "0")
    late = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert int(L.vr_engine_est_reruns()) - r0 >= 1, "without the check the first EST pass is flagged"
    assert np.array_equal(late, ref)


@pytest.mark.parametrize("form", ["1", "0"])
def test_shared_joins_equal_per_unit_joins(dev, form):
    # SharedJoins (one 16-B gather per model pair for up to 4 neural plans) + the joined
    # multi call against the plain multi call, EST and exact forms, 3 and 1 A plans
    n = 1800
    neurals = [R.RankPlan(_rdm(dev, n, 90 + 10 * i, 60 + i)) for i in range(3)]
    models = [R.RankPlan(_rdm(dev, n, 70, 70, relu=True)), R.RankPlan(_rdm(dev, n, 150, 71))]
    idx = bootstrap_indices(42, n, int(0.9 * n), 100)
    with _engine_form(form):
        for group in (neurals, neurals[:1]):
            sj = R.SharedJoins(group)
            joins = [sj.join(pm) for pm in models]  # joins[m][a]
            for a, pn in enumerate(group):
                ref = R.bootstrap_spearman_multi(pn, models, idx, full_first=True).cpu().numpy()
                got = R.bootstrap_spearman_multi(pn, models, idx, full_first=True,
                                                 joined=[joins[m][a] for m in range(len(models))]).cpu().numpy()
                assert np.array_equal(got, ref)


def test_half_tied_rdm_exact_join_is_fast(dev):
    # One tie group over half the 12.5 M pairs (n = 5000): it spans ~1000 of the exact
    # form's group-aligned chunks, so the join's chunk lookup must be a binary search
    # (the old one-chunk-per-step walk made this join take seconds). Exact and
    # EST forms must agree and the call must stay fast.
    import time

    n = 5000
    g = torch.Generator(device=dev).manual_seed(51)
    a = torch.rand(n, n, device=dev, generator=g)
    a = torch.where(torch.rand(n, n, device=dev, generator=g) < 0.5, torch.full_like(a, 0.5), a)
    a = torch.triu(a, 1)
    a = a + a.T
    b = _rdm(dev, n, 100, 52)
    idx = bootstrap_indices(42, n, int(0.9 * n), 127)
    pa, pb = R.RankPlan(a), R.RankPlan(b)
    with exact_engine():
        R.bootstrap_spearman(pa, pb, idx[:2], full_first=True)  # warm
        torch.cuda.synchronize()
        t = time.perf_counter()
        ref = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
        dt = time.perf_counter() - t
    est = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert np.array_equal(est, ref)
    assert dt < 2.0, f"exact-form call with a half-triangle tie group took {dt:.2f}s"
    an = a.cpu().numpy()
    assert abs(ref[0] - O.compute_rdm_correlation(an, b.cpu().numpy(), "Spearman")) <= 1e-12


@pytest.mark.parametrize("inject", [0, 2])
def test_b_side_error_is_flagged_and_rerun(dev, monkeypatch, inject):
    # A B-side recovery error is invisible to the A walk's window checks. Inject one (lanes
    # 1..63 of one TB row off by one after the A walk of EST pass `inject`): the tail's
    # invariants (sum of the gathered A ranks == M'(M'+1), B-side included pairs == M')
    # must flag the pass, the exact re-run must restore every score bit for bit. Pass 0
    # flagged makes the call give up on the estimate (every later pass exact).
    n, nb = 2000, 250
    a, b = _rdm(dev, n, 64, 41, relu=True), _rdm(dev, n, 300, 42)
    idx = bootstrap_indices(42, n, int(0.9 * n), nb)
    pa, pb = R.RankPlan(a), R.RankPlan(b)
    clean = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    r0, t0 = int(lib().vr_engine_est_reruns()), int(lib().vr_engine_est_tail_flags())
    lib().vr_test_engine_inject(inject)  # test-only export (no environment switch in the library)
    try:
        got = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    finally:
        lib().vr_test_engine_inject(-1)
    reruns = int(lib().vr_engine_est_reruns()) - r0
    assert reruns >= 1, "the injected B-side error must flag its pass"
    assert int(lib().vr_engine_est_tail_flags()) - t0 == 1, "flagged by the tail invariants (the A walk cannot see it)"
    assert np.array_equal(got, clean)
    with exact_engine():
        assert np.array_equal(R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy(), clean)


def test_est_strong_stimulus_structure_equals_exact_form(dev):
    # Continuous RDMs with a strong per-stimulus effect (d_ab = u_a + u_b + noise, u heavy-
    # tailed): the included-pair count of a subset drifts far from the uniform estimate along
    # the A order, so the EST passes may be flagged and re-run (or the call gives up on the
    # estimate after its first EST pass). Whatever the path, scores equal the exact form.
    n = 1200
    rs = np.random.RandomState(7)
    u = rs.exponential(1.0, size=n) ** 2
    a = u[:, None] + u[None, :] + 0.05 * rs.rand(n, n)
    a = np.triu(a, 1)
    a = (a + a.T).astype(np.float32)
    b = _rdm(dev, n, 80, 31).cpu().numpy()
    idx = bootstrap_indices(42, n, int(0.9 * n), 150)
    pa, pb = R.RankPlan(torch.from_numpy(a).to(dev)), R.RankPlan(torch.from_numpy(b).to(dev))
    est = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    with exact_engine():
        ref = R.bootstrap_spearman(pa, pb, idx, full_first=True).cpu().numpy()
    assert np.array_equal(est, ref)
    assert abs(est[0] - O.compute_rdm_correlation(a, b, "Spearman")) <= 1e-12


@pytest.mark.parametrize("na", [2, 3, 4])
def test_grid_equals_per_region_calls(dev, na):
    # The region-fused grid call (one B walk per model plan for all regions, k_rankB_grid) is
    # bit-equal to one joined multi call per region, in every pass form it takes: the full-set
    # pass (lane 0 shifted, EST 4) and the EST 3 passes, with ties (ReLU features) and a
    # quantised model RDM whose tie groups take the walk's slow windows
    from visreps_amd._lib import ktimer_enable, ktimer_read

    n = 1800
    neurals = [R.RankPlan(_rdm(dev, n, 90 + 10 * i, 60 + i)) for i in range(na)]
    q = _rdm(dev, n, 40, 77)
    q = (q * 64).floor() / 64
    models = [R.RankPlan(_rdm(dev, n, 70, 70, relu=True)), R.RankPlan(_rdm(dev, n, 150, 71)), R.RankPlan(q)]
    idx = bootstrap_indices(42, n, int(0.9 * n), 130)  # 131 subsets: 3 passes
    sj = R.SharedJoins(neurals)
    joins = [sj.join(pm) for pm in models]  # joins[m][a]
    ktimer_enable(True)
    got = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    grid_launches = ktimer_read("k_rankB_grid")[1]
    ktimer_enable(False)
    assert grid_launches > 0, "the fused walk did not run"
    for a, pn in enumerate(neurals):
        ref = R.bootstrap_spearman_multi(pn, models, idx, full_first=True,
                                         joined=[joins[m][a] for m in range(len(models))]).cpu().numpy()
        assert np.array_equal(got[a], ref)
    with exact_engine():  # the exact form runs the per-region calls
        ex = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    assert np.array_equal(ex, got)
    ktimer_enable(True)
    with exact_engine(), _exact_grid():  # or region-fused (opt-in, k_rankB_gridx)
        ex = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    gridx_launches = ktimer_read("k_rankB_gridx")[1]
    ktimer_enable(False)
    assert gridx_launches == 3 * len(models), "the exact grid walk: one launch per model plan and pass"
    assert np.array_equal(ex, got)


def test_grid_falls_back_on_a_structured_region(dev):
    # A strongly structured neural RDM fails the up-front estimate check: the grid call then
    # runs every region on its own (exact form where needed) and still equals the per-region calls
    n = 1500
    g = torch.Generator(device=dev).manual_seed(91)
    u = torch.randn(n, device=dev, generator=g).abs() ** 3
    s = u[:, None] + u[None, :] + 0.01 * torch.rand(n, n, device=dev, generator=g)
    s = torch.triu(s, 1)
    s = s + s.T
    neurals = [R.RankPlan(s), R.RankPlan(_rdm(dev, n, 80, 92))]
    models = [R.RankPlan(_rdm(dev, n, 60, 93)), R.RankPlan(_rdm(dev, n, 60, 94, relu=True))]
    idx = bootstrap_indices(42, n, int(0.9 * n), 100)
    sj = R.SharedJoins(neurals)
    joins = [sj.join(pm) for pm in models]
    got = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    for a, pn in enumerate(neurals):
        ref = R.bootstrap_spearman_multi(pn, models, idx, full_first=True).cpu().numpy()
        assert np.array_equal(got[a], ref)


def test_grid_l2_masks_equal_per_region_calls(dev, monkeypatch):
    # the grid walk's L2-mask form (what n > 20,352 takes; VISREPS_ENGINE_GRID_LDS=0 forces it
    # here) against the per-region calls, with ties in a quantised model RDM
    from visreps_amd._lib import ktimer_enable, ktimer_read

    monkeypatch.setenv("VISREPS_ENGINE_GRID_LDS", "0")
    n = 1800
    neurals = [R.RankPlan(_rdm(dev, n, 90 + 10 * i, 80 + i)) for i in range(3)]
    q = (_rdm(dev, n, 40, 87) * 64).floor() / 64
    models = [R.RankPlan(_rdm(dev, n, 70, 88, relu=True)), R.RankPlan(q)]
    idx = bootstrap_indices(42, n, int(0.9 * n), 130)
    sj = R.SharedJoins(neurals)
    joins = [sj.join(pm) for pm in models]
    ktimer_enable(True)
    got = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    assert ktimer_read("k_rankB_grid")[1] > 0, "the fused walk did not run"
    ktimer_enable(False)
    for a, pn in enumerate(neurals):
        ref = R.bootstrap_spearman_multi(pn, models, idx, full_first=True,
                                         joined=[joins[m][a] for m in range(len(models))]).cpu().numpy()
        assert np.array_equal(got[a], ref)


@pytest.mark.parametrize("inject", [0, 2])
def test_grid_flagged_region_reruns_alone(dev, inject):
    # a B-side error injected into the first fused region after its A walk of pass
    # `inject` (pass 0 is checked at once, pass 2 at the end): the tail invariants flag it, that
    # region runs again on its own (re-running the flagged pass exact), the other two stay
    # fused, and every score equals the clean per-region calls
    from visreps_amd._lib import ktimer_enable, ktimer_read

    n = 1800
    neurals = [R.RankPlan(_rdm(dev, n, 90 + 10 * i, 100 + i)) for i in range(3)]
    models = [R.RankPlan(_rdm(dev, n, 70, 110, relu=True)), R.RankPlan(_rdm(dev, n, 150, 111))]
    idx = bootstrap_indices(42, n, int(0.9 * n), 130)  # 131 subsets: 3 passes
    sj = R.SharedJoins(neurals)
    joins = [sj.join(pm) for pm in models]
    clean = [R.bootstrap_spearman_multi(pn, models, idx, full_first=True,
                                        joined=[joins[m][a] for m in range(len(models))]).cpu().numpy()
             for a, pn in enumerate(neurals)]
    r0, t0 = int(lib().vr_engine_est_reruns()), int(lib().vr_engine_est_tail_flags())
    lib().vr_test_engine_inject(inject)
    ktimer_enable(True)
    try:
        got = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    finally:
        lib().vr_test_engine_inject(-1)
    grid_launches = ktimer_read("k_rankB_grid")[1]
    ktimer_enable(False)
    assert int(lib().vr_engine_est_reruns()) - r0 >= 1, "the injected error must flag a pass"
    assert int(lib().vr_engine_est_tail_flags()) - t0 >= 1
    assert grid_launches == 2 * len(models), "passes 1-2 stay fused for the other regions"
    for a in range(len(neurals)):
        assert np.array_equal(got[a], clean[a]), a


def test_grid_structured_region_leaves_the_others_fused(dev):
    # one region failing the up-front check runs on its own; the other two
    # still walk each model plan once per pass together
    from visreps_amd._lib import ktimer_enable, ktimer_read

    n = 5000  # test_structured_rdm_leaves_est3_up_front's RDM, which fails the check
    g = torch.Generator(device=dev).manual_seed(7)
    u = torch.empty(n, device=dev).exponential_(1.0, generator=g) ** 2
    s = u[:, None] + u[None, :] + 0.05 * torch.rand(n, n, device=dev, generator=g)
    s = torch.triu(s, 1)
    s = s + s.T
    neurals = [R.RankPlan(_rdm(dev, n, 80, 96)), R.RankPlan(s), R.RankPlan(_rdm(dev, n, 90, 97))]
    del s
    models = [R.RankPlan(_rdm(dev, n, 60, 98)), R.RankPlan(_rdm(dev, n, 60, 99, relu=True))]
    idx = bootstrap_indices(42, n, int(0.9 * n), 100)
    sj = R.SharedJoins(neurals)
    joins = [sj.join(pm) for pm in models]
    p0 = int(lib().vr_engine_est_predicted())
    ktimer_enable(True)
    got = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    grid_launches = ktimer_read("k_rankB_grid")[1]
    ktimer_enable(False)
    assert grid_launches == 1 * len(models), "the two continuous regions stay fused (pass 1)"
    assert int(lib().vr_engine_est_predicted()) - p0 == 1, "the structured region goes exact up front"
    for a, pn in enumerate(neurals):
        ref = R.bootstrap_spearman_multi(pn, models, idx, full_first=True).cpu().numpy()
        assert np.array_equal(got[a], ref)


class _exact_grid:
    """Context: the region-fused exact walk (VISREPS_ENGINE_GRIDX=1, opt-in)."""

    def __enter__(self):
        os.environ["VISREPS_ENGINE_GRIDX"] = "1"

    def __exit__(self, *a):
        os.environ.pop("VISREPS_ENGINE_GRIDX", None)


def _structured_rdm(dev, n, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    u = torch.empty(n, device=dev).exponential_(1.0, generator=g) ** 2
    s = u[:, None] + u[None, :] + 0.05 * torch.rand(n, n, device=dev, generator=g)
    s = torch.triu(s, 1)
    return s + s.T


def test_grid_structured_regions_walk_the_exact_grid(dev):
    # regions whose estimate fails the up-front check go to the exact form; with
    # the exact grid on, two or more of them walk it region-fused (k_rankB_gridx), the
    # continuous ones stay in the EST grid, and every score equals the per-region calls (and
    # the default, the structured regions' own exact calls)
    from visreps_amd._lib import ktimer_enable, ktimer_read

    n = 5000
    neurals = [R.RankPlan(_structured_rdm(dev, n, 7)), R.RankPlan(_rdm(dev, n, 80, 121)),
               R.RankPlan(_structured_rdm(dev, n, 8)), R.RankPlan(_rdm(dev, n, 90, 122))]
    models = [R.RankPlan(_rdm(dev, n, 60, 123)), R.RankPlan(_rdm(dev, n, 60, 124, relu=True))]
    idx = bootstrap_indices(42, n, int(0.9 * n), 100)  # 101 subsets: 2 passes
    sj = R.SharedJoins(neurals)
    joins = [sj.join(pm) for pm in models]
    p0, r0 = int(lib().vr_engine_est_predicted()), int(lib().vr_engine_est_reruns())
    ktimer_enable(True)
    with _exact_grid():
        got = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    est_launches = ktimer_read("k_rankB_grid")[1]
    gridx_launches = ktimer_read("k_rankB_gridx")[1]
    ktimer_enable(False)
    assert int(lib().vr_engine_est_predicted()) - p0 == 2, "both structured regions go exact up front"
    assert est_launches == 1 * len(models), "the two continuous regions stay in the EST grid (pass 1)"
    # (region 0 is off the estimate: the fused walk takes its window parameters from a fused
    # region's workspace, so no pass of the continuous regions is flagged)
    assert int(lib().vr_engine_est_reruns()) - r0 == 0
    assert gridx_launches == 2 * len(models), "the two structured regions walk the exact grid"
    for a, pn in enumerate(neurals):
        ref = R.bootstrap_spearman_multi(pn, models, idx, full_first=True).cpu().numpy()
        assert np.array_equal(got[a], ref), a
    p1, r1 = int(lib().vr_engine_est_predicted()), int(lib().vr_engine_est_reruns())
    off = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    assert int(lib().vr_engine_est_predicted()) - p1 == 2 and int(lib().vr_engine_est_reruns()) - r1 == 0
    assert np.array_equal(off, got)


def test_exact_grid_ties_and_l2_masks(dev, monkeypatch):
    # the exact grid walk with tied A plans (chunks that start after c L, the chunk lookup's
    # step back), tied and quantised B plans, 4 and 2 regions, masks from L2 too
    from visreps_amd._lib import ktimer_enable, ktimer_read

    n = 1800
    neurals = [R.RankPlan((_rdm(dev, n, 40 + 10 * i, 130 + i) * 1024).floor() / 1024) for i in range(3)]
    neurals.append(R.RankPlan(_rdm(dev, n, 70, 134, relu=True)))
    q = (_rdm(dev, n, 40, 135) * 64).floor() / 64
    models = [R.RankPlan(_rdm(dev, n, 70, 136, relu=True)), R.RankPlan(q)]
    idx = bootstrap_indices(42, n, int(0.9 * n), 130)
    sj = R.SharedJoins(neurals)
    joins = [sj.join(pm) for pm in models]
    monkeypatch.setenv("VISREPS_ENGINE_GRIDX", "1")
    with exact_engine():
        refs = [R.bootstrap_spearman_multi(pn, models, idx, full_first=True,
                                           joined=[joins[m][a] for m in range(len(models))]).cpu().numpy()
                for a, pn in enumerate(neurals)]
        for lds in ("1", "0", "global"):  # grid walk masks in LDS / L2; "global": the A walks' too
            monkeypatch.setenv("VISREPS_ENGINE_GRID_LDS", "0" if lds == "global" else lds)
            if lds == "global":
                monkeypatch.setenv("VISREPS_ENGINE_MASKS", "global")
            for na in (4, 2):
                ktimer_enable(True)
                got = R.bootstrap_spearman_grid(neurals[:na], models, idx, [js[:na] for js in joins],
                                                full_first=True).cpu().numpy()
                launches = ktimer_read("k_rankB_gridx")[1]
                ktimer_enable(False)
                assert launches == 3 * len(models), (lds, na)
                for a in range(na):
                    assert np.array_equal(got[a], refs[a]), (lds, na, a)


@pytest.mark.parametrize("n", [12000, 20500])
def test_large_n_engine_forms(dev, n):
    # n above the two-workgroup LDS mask limit (10,176). 12,000 keeps the
    # grid walk's masks in LDS (one workgroup per CU), 20,500 reads them from L2; the A walks
    # and the per-region B walks read L2 masks at both. 127 draws (2 passes). The grid call,
    # the per-region EST calls and the exact form agree bit for bit; the point and draw #100
    # of one unit equal the CPU oracle (scipy spearmanr on the sub-RDMs).
    from visreps_amd._lib import ktimer_enable, ktimer_read

    nb = 127
    neurals = [R.RankPlan(_rdm(dev, n, 64 + 16 * i, 120 + i)) for i in range(2)]
    m_rdm = _rdm(dev, n, 96, 130, relu=True)
    models = [R.RankPlan(m_rdm), R.RankPlan(_rdm(dev, n, 48, 131))]
    idx = bootstrap_indices(42, n, int(0.9 * n), nb)
    sj = R.SharedJoins(neurals)
    joins = [sj.join(pm) for pm in models]
    del sj
    ktimer_enable(True)
    grid = R.bootstrap_spearman_grid(neurals, models, idx, joins, full_first=True).cpu().numpy()
    assert ktimer_read("k_rankB_grid")[1] == len(models), "pass 1 fused"
    ktimer_enable(False)
    del joins
    per = [R.bootstrap_spearman_multi(pn, models, idx, full_first=True).cpu().numpy() for pn in neurals]
    with exact_engine():
        ex = R.bootstrap_spearman(models[0], neurals[0], idx, full_first=True).cpu().numpy()
    for a in range(2):
        assert np.array_equal(grid[a], per[a]), a
    assert np.array_equal(per[0][0], ex)
    if n > 15000:  # (scipy on 2e8 pairs takes minutes of host time: the oracle runs at 12,000)
        return
    # the oracle on the same fp32 RDMs (point and draw #100: subsets of 0.9 n stimuli)
    a_np = m_rdm.cpu().numpy()
    b_np = _rdm(dev, n, 64, 120).cpu().numpy()
    assert abs(float(per[0][0][0]) - O.compute_rdm_correlation(a_np, b_np, "Spearman")) <= 1e-12
    i = np.asarray(idx[99])
    ref = O.compute_rdm_correlation(a_np[np.ix_(i, i)], b_np[np.ix_(i, i)], "Spearman")
    assert abs(float(per[0][0][100]) - ref) <= 1e-12
