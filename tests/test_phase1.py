"""Phase-1 layer selection (reference evals.py:249-287) on the GPU against the oracle.

pipeline.phase1_select projects only the selected stimuli of every point (vr_srp_csr_f32),
which equals projecting every stimulus and selecting afterwards (the projection is row by
row): checked bit for bit here. The selection scores (Spearman of each point's selection
RDM against each region's) are then compared with the oracle on the same projection:
RandomState(42).choice(n, n_select) rows, float64 SRP product, O.compute_rdm, scipy's
Spearman (rsa.py:96-129); best point = first strict maximum (evals.py:273-275).
"""
import numpy as np
import pytest
import torch

from oracle import rsa_oracle as O
from visreps_amd import pipeline as PL
from visreps_amd.analysis import sparse_random_projection as S
from conftest import record_margin

# |dSpearman| between the product and the all-oracle path at these small n (each side builds
# its own RDMs): the north-star bound, with the measured values logged by record_margin
TOL_SMALL_N = 1e-5

pytestmark = pytest.mark.gpu


def test_phase1_select_matches_oracle(dev, tmp_path):
    n, n_select = 700, 300
    dims = [2400, 900, 64]
    xs = O.synthetic_features(n, dims + [40, 70], seed=11, relu=[True, True, False, False, False])
    points = ["p0", "p1", "p2"]
    feats = {p: torch.from_numpy(x).to(dev) for p, x in zip(points, xs[:3])}
    regions = {"V1": xs[3], "V2": xs[4]}
    responses = {r: torch.from_numpy(y).to(dev) for r, y in regions.items()}
    tr = {d: S.get_srp_transformer(D=d, k=min(256, d), density=None, seed=0, cache_dir=str(tmp_path))
          for d in dims}
    projectors = {p: S.SparseProjector(tr[d], dev) for p, d in zip(points, dims)}

    got = PL.phase1_select(feats, projectors, responses, points, n, n_select=n_select, seed=42)

    sel = np.random.RandomState(42).choice(n, n_select, replace=False)
    sel_t = torch.as_tensor(sel, device=dev)
    for p in points:  # the selected rows' projection == every row's projection, then selected
        assert torch.equal(projectors[p](feats[p][sel_t]), projectors[p](feats[p])[sel_t])

    for r, y in regions.items():
        n_rdm = O.compute_rdm(y[sel])
        scores = []
        for p, d in zip(points, dims):
            P = tr[d].components_.astype(np.float64)
            proj = np.asarray((P @ xs[points.index(p)][sel].astype(np.float64).T).T, dtype=np.float32)
            scores.append(O.compute_rdm_correlation(O.compute_rdm(proj), n_rdm, "Spearman"))
        best, scores_got = got[r]
        assert [s["layer"] for s in scores_got] == points
        # different fp32 summation orders (CSR fma chain vs float64) move near-tied RDM
        # entries in the last bits: a few 1e-6 of rho at 44,850 pairs
        d = float(np.max(np.abs(np.array([s["score"] for s in scores_got]) - np.array(scores))))
        record_margin("phase1_select_vs_oracle", region=r, n=n_select, dspearman=d)
        assert d < TOL_SMALL_N
        assert best == points[int(np.argmax(scores))]
