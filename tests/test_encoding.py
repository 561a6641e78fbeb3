"""Encoding score: visreps/analysis/encoding_score.py.

CPU: the oracle's himalaya pieces against scipy / sklearn / closed-form ridge, and the
fold splitter of the product. GPU: the MFMA Gram (vr_gram_f32), the correlation-score
kernel and its bootstrap (vr_corr_score_f32), the dual-form RidgeCV and the whole
compute_encoding_score flow against the oracle's primal-form restatement. The alpha
selection rule is restated from himalaya 0.4.9 (not installed): parity unpinned beyond
this oracle."""
import numpy as np
import pytest
import scipy.stats
from sklearn.model_selection import KFold

from conftest import record_margin
from oracle import encoding_oracle as E


def _data(n, p, v, seed, noise=0.5):
    r = np.random.RandomState(seed)
    X = r.randn(n, p).astype(np.float32)
    W = r.randn(p, v).astype(np.float32) / np.sqrt(p)
    Y = (X @ W + noise * r.randn(n, v)).astype(np.float32)
    return X, Y


# ----------------------------------------------------------------------------- CPU
def test_oracle_correlation_score_matches_scipy_pearson():
    # tests/test_encoding_score.py:1279-1306: per-voxel r equals scipy.stats.pearsonr
    X, Y = _data(60, 10, 3, 0, noise=0.3)
    P = Y + np.random.RandomState(1).randn(*Y.shape)
    ours = E.correlation_score(Y, P)
    ref = [scipy.stats.pearsonr(Y[:, j], P[:, j])[0] for j in range(Y.shape[1])]
    assert np.allclose(ours, ref, atol=1e-10)


def test_oracle_ridge_refit_is_closed_form_ridge():
    X, Y = _data(120, 15, 4, 2)
    Xn = np.random.RandomState(3).randn(7, 15)
    pred, alphas = E.ridge_cv(X, Y, Xn, alphas=np.logspace(-3, 3, 7))
    X64, Y64 = X.astype(np.float64), Y.astype(np.float64)
    for j, a in enumerate(alphas):
        w = np.linalg.solve(X64.T @ X64 + a * np.eye(15), X64.T @ Y64[:, j])
        assert np.allclose(pred[:, j], Xn @ w, atol=1e-8)


def test_oracle_ridge_alpha_selection_tracks_noise():
    # pure-noise targets pick a large alpha, clean targets a small one
    X, Y = _data(200, 20, 2, 4, noise=0.0)
    Y[:, 1] = np.random.RandomState(5).randn(200)
    _, alphas = E.ridge_cv(X, Y, X[:3])
    assert alphas[0] < 1e-2 and alphas[1] > 1e2


@pytest.mark.parametrize("n", [5, 13, 100, 1001])
def test_kfold_splits_match_sklearn(n):
    from visreps_amd.analysis.encoding_score import kfold_splits

    ours = list(kfold_splits(n, 5))
    ref = list(KFold(n_splits=5).split(np.zeros(n)))
    assert len(ours) == len(ref)
    for (a, b), (c, d) in zip(ours, ref):
        assert np.array_equal(a, c) and np.array_equal(b, d)


def test_kfold_splits_too_few_rows():
    from visreps_amd.analysis.encoding_score import kfold_splits

    with pytest.raises(ValueError):
        list(kfold_splits(4, 5))


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("n,d", [(300, 70), (1000, 4096), (2100, 33)])
def test_gram_kernel_matches_fp64(dev, n, d):
    import torch
    from visreps_amd.analysis.encoding_score import gram

    x = np.random.RandomState(n).randn(n, d).astype(np.float32)
    G = gram(torch.from_numpy(x).to(dev)).double().cpu().numpy()
    ref = x.astype(np.float64) @ x.astype(np.float64).T
    assert np.max(np.abs(G - ref)) <= 2e-5 * np.abs(ref).max()
    assert np.array_equal(G, G.T)


@pytest.mark.gpu
@pytest.mark.parametrize("n,p,ld", [(300, 70, 70), (1000, 4096, 4096), (2100, 33, 40), (77, 1000, 1003), (5, 3, 3)])
def test_gram64_kernels_match_fp64(dev, n, p, ld):
    # vr_gram64_f32 (fp64 MFMA tiles): X X^T (kernel form) and X^T X (primal form) of fp32 X
    # vs numpy fp64 products -- exact products, fp64 sums: relative 1e-13; exactly symmetric.
    # Ragged shapes, a row pitch ld > p (unaligned rows) and tiny n.
    import torch
    from visreps_amd.analysis.encoding_score import gram64, gram64_cols

    buf = np.random.RandomState(n + p).randn(n, ld).astype(np.float32)
    x = buf[:, :p]
    xt = torch.from_numpy(buf).to(dev)[:, :p]  # a strided view: row pitch ld
    x64 = x.astype(np.float64)
    for got, ref in ((gram64(xt), x64 @ x64.T), (gram64_cols(xt), x64.T @ x64)):
        g = got.cpu().numpy()
        assert g.dtype == np.float64 and g.shape == ref.shape
        assert np.max(np.abs(g - ref)) <= 1e-13 * max(1.0, np.abs(ref).max())
        assert np.array_equal(g, g.T)


@pytest.mark.gpu
def test_corr_score_point_and_voxels_match_scipy(dev):
    import torch
    from visreps_amd.analysis.encoding_score import corr_score

    _, Y = _data(500, 8, 300, 6)
    P = Y + np.random.RandomState(7).randn(*Y.shape).astype(np.float32)
    s, vox = corr_score(torch.from_numpy(Y).to(dev), torch.from_numpy(P).to(dev), voxels=True)
    Y64, P64 = Y.astype(np.float64), P.astype(np.float64)  # scipy keeps float32 inputs in float32
    ref = np.array([scipy.stats.pearsonr(Y64[:, j], P64[:, j])[0] for j in range(Y.shape[1])])
    assert float(np.max(np.abs(vox[0].cpu().numpy() - ref))) < 1e-10
    assert abs(s - ref.mean()) < 1e-10


@pytest.mark.gpu
def test_corr_score_bootstrap_matches_oracle_loop(dev):
    import torch
    from visreps_amd.analysis.encoding_score import corr_score

    _, Y = _data(230, 8, 700, 8)
    P = Y + np.random.RandomState(9).randn(*Y.shape).astype(np.float32)
    rng = np.random.RandomState(42)
    idx = np.stack([rng.choice(230, 207, replace=False) for _ in range(50)])
    got = corr_score(torch.from_numpy(Y).to(dev), torch.from_numpy(P).to(dev), idx)
    ref = np.array([E.correlation_score(Y[i], P[i]).mean() for i in idx])
    assert np.max(np.abs(got - ref)) < 1e-10


@pytest.mark.gpu
def test_corr_score_constant_column_is_nan(dev):
    import torch
    from visreps_amd.analysis.encoding_score import corr_score

    Y = np.random.RandomState(0).randn(40, 3).astype(np.float32)
    P = Y.copy()
    P[:, 1] = 2.0
    s = corr_score(torch.from_numpy(Y).to(dev), torch.from_numpy(P).to(dev))
    assert np.isnan(s)


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(150, 20), (120, 400)])  # primal n > p and dual p > n
def test_dual_ridge_cv_matches_primal_oracle(dev, n, p):
    import torch
    from visreps_amd.analysis.encoding_score import gram64, ridge_cv_predict

    X, Y = _data(n + 30, p, 5, n + p)
    Y[:, 4] = np.random.RandomState(1).randn(n + 30)  # one pure-noise target
    K = gram64(torch.from_numpy(X).to(dev))
    pred, alphas = ridge_cv_predict(K, np.arange(n), np.arange(n, n + 30),
                                    torch.from_numpy(Y[:n]).to(dev))
    rp, ra = E.ridge_cv(X[:n], Y[:n], X[n:])
    assert np.array_equal(alphas, ra)
    assert np.max(np.abs(pred.cpu().numpy() - rp)) <= 1e-4 * max(1.0, np.abs(rp).max())


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(150, 20), (300, 90)])
def test_primal_ridge_cv_matches_primal_oracle(dev, n, p):
    import torch
    from visreps_amd.analysis.encoding_score import ridge_cv_predict_primal

    X, Y = _data(n + 30, p, 5, n + 2 * p)
    Y[:, 4] = np.random.RandomState(2).randn(n + 30)
    pred, alphas = ridge_cv_predict_primal(torch.from_numpy(X[:n]).to(dev), torch.from_numpy(Y[:n]).to(dev),
                                           torch.from_numpy(X[n:]).to(dev))
    rp, ra = E.ridge_cv(X[:n], Y[:n], X[n:])
    assert np.array_equal(alphas, ra)
    assert np.max(np.abs(pred.cpu().numpy() - rp)) <= 1e-4 * max(1.0, np.abs(rp).max())


def _decaying(n, p, v, cond, seed):
    """X = U diag(s) V^T with s log-spaced over `cond` (condition number), Y = X w + noise."""
    rs = np.random.RandomState(seed)
    r = min(n, p)
    U = np.linalg.qr(rs.randn(n, r))[0]
    Vt = np.linalg.qr(rs.randn(p, r))[0].T
    s = np.logspace(0, -np.log10(cond), r) * 30.0
    X = (U * s) @ Vt
    Y = X @ rs.randn(p, v) + 0.01 * rs.randn(n, v)
    return X.astype(np.float32), Y.astype(np.float32)


def _closed_form(X, Y, X_new, alphas):
    """fp64 ridge per target: X_new (X^T X + a I)^-1 X^T y."""
    X, Y, X_new = (np.asarray(a, np.float64) for a in (X, Y, X_new))
    out = np.empty((X_new.shape[0], Y.shape[1]))
    for t, a in enumerate(alphas):
        w = np.linalg.solve(X.T @ X + a * np.eye(X.shape[1]), X.T @ Y[:, t])
        out[:, t] = X_new @ w
    return out


def test_oracle_ridge_keeps_small_singular_values():
    # himalaya's SVD solver keeps every singular value: on a spectrum decaying over 1e5 the
    # oracle's refit equals the closed-form ridge at its chosen alphas
    X, Y = _decaying(160, 40, 4, 1e5, 3)
    pred, alphas = E.ridge_cv(X[:130], Y[:130], X[130:])
    ref = _closed_form(X[:130], Y[:130], X[130:], alphas)
    assert np.max(np.abs(pred - ref)) <= 1e-8 * np.abs(ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(130, 40), (90, 200)])  # primal and dual
def test_ridge_cv_decaying_spectrum_matches_closed_form(dev, n, p):
    # condition number 1e5: no component above the fp64 floor may be dropped
    import torch
    from visreps_amd.analysis.encoding_score import gram64, ridge_cv_predict, ridge_cv_predict_primal

    X, Y = _decaying(n + 30, p, 4, 1e5, n + p)
    Xt = torch.from_numpy(X).to(dev)
    Yt = torch.from_numpy(Y[:n]).to(dev)
    if p < n:
        pred, alphas = ridge_cv_predict_primal(Xt[:n], Yt, Xt[n:])
    else:
        pred, alphas = ridge_cv_predict(gram64(Xt), np.arange(n), np.arange(n, n + 30), Yt)
    ref = _closed_form(X[:n], Y[:n], X[n:], alphas)
    assert np.max(np.abs(pred.cpu().numpy() - ref)) <= 1e-5 * np.abs(ref).max()
    _, ra = E.ridge_cv(X[:n], Y[:n], X[n:])
    assert np.array_equal(alphas, ra)


@pytest.mark.gpu
def test_compute_encoding_score_matches_oracle(dev):
    import torch
    from visreps_amd.analysis.alignment import AlignmentData
    from visreps_amd.analysis.encoding_score import compute_encoding_score

    r = np.random.RandomState(11)
    n_tr, n_te, v = 260, 90, 40
    Z = r.randn(n_tr + n_te, 6)
    acts = {"conv": r.randn(n_tr + n_te, 4, 3, 3).astype(np.float32),  # 4-D, flattened
            "fc": (Z @ r.randn(6, 30) + 0.5 * r.randn(n_tr + n_te, 30)).astype(np.float32)}
    Y = (Z @ r.randn(6, v) + r.randn(n_tr + n_te, v)).astype(np.float32)
    train = AlignmentData({k: torch.from_numpy(a[:n_tr]).to(dev) for k, a in acts.items()},
                          torch.from_numpy(Y[:n_tr]).to(dev))
    test = AlignmentData({k: torch.from_numpy(a[n_tr:]).to(dev) for k, a in acts.items()},
                         torch.from_numpy(Y[n_tr:]).to(dev))
    before = {k: t.clone() for k, t in train.activations.items()}
    res = compute_encoding_score(train, test, bootstrap=True, n_bootstrap=60, seed=42)[0]
    ref = E.compute_encoding_score({k: a[:n_tr] for k, a in acts.items()}, Y[:n_tr],
                                   {k: a[n_tr:] for k, a in acts.items()}, Y[n_tr:],
                                   bootstrap=True, n_bootstrap=60, seed=42)
    assert res["layer"] == ref["layer"] == "fc"
    assert res["analysis"] == "encoding_score" and res["compare_method"] == "pearson"
    for a, b in zip(res["layer_selection_scores"], ref["layer_selection_scores"]):
        assert a["layer"] == b["layer"] and abs(a["score"] - b["score"]) < 1e-4
    assert abs(res["score"] - ref["score"]) < 1e-4
    assert np.max(np.abs(np.array(res["bootstrap_scores"]) - ref["bootstrap_scores"])) < 1e-4
    assert abs(res["ci_low"] - ref["ci_low"]) < 1e-4 and abs(res["ci_high"] - ref["ci_high"]) < 1e-4
    assert len(res["bootstrap_scores"]) == 60
    for k, t in train.activations.items():  # inputs not mutated
        assert torch.equal(t, before[k])


@pytest.mark.gpu
def test_encoding_refused_for_things_behavior(dev):
    import torch
    from visreps_amd.analysis.alignment import AlignmentData, compute_traintest_alignment
    from visreps_amd.utils import Config

    d = AlignmentData({"fc": torch.zeros(10, 3, device=dev)}, torch.zeros(10, 2, device=dev))
    cfg = Config({"analysis": "encoding_score", "neural_dataset": "things-behavior"})
    with pytest.raises(ValueError):
        compute_traintest_alignment(cfg, d, d)


@pytest.mark.gpu
def test_ridge_cv_full_size_matches_closed_form(dev):
    """BASELINE configs[3]'s ridge at its stated size (reference encoding_score.py:47-62):
    n = 26,000 stimuli (20,800 fit, 5,200 predicted), p = 4,096 features, 48 voxels of
    mixed SNR. The product's primal RidgeCV (fp64 p x p Grams on the device) against an
    independent fp64 closed form on the device: per fold and alpha a Cholesky solve of
    (X_T^T X_T + a I) W = X_T^T Y_T, the fold-mean l2 loss, its first argmax per voxel
    (himalaya's RidgeCV rule, parity unpinned beyond this restatement), then the refit
    predictions X_new (X^T X + a I)^-1 X^T y."""
    import torch
    from visreps_amd.analysis.encoding_score import ALPHAS, kfold_splits, ridge_cv_predict_primal

    n_fit, n_new, p, v = 20800, 5200, 4096, 48
    g = torch.Generator(device=dev).manual_seed(26000)
    Z = torch.randn(n_fit + n_new, 256, device=dev, generator=g, dtype=torch.float64)
    X = (Z @ torch.randn(256, p, device=dev, generator=g, dtype=torch.float64)
         + 0.5 * torch.randn(n_fit + n_new, p, device=dev, generator=g, dtype=torch.float64))
    X = ((X - X.mean(0)) / X.std(0)).float()  # z-normalised as compute_encoding_score does
    B = torch.randn(p, v, device=dev, generator=g, dtype=torch.float64) / 64.0
    snr = torch.logspace(1, -2, v, device=dev, dtype=torch.float64)  # clean ... pure noise
    Y = (X.double() @ B) * snr + torch.randn(n_fit + n_new, v, device=dev, generator=g, dtype=torch.float64)
    Y = Y.float()
    pred, alphas = ridge_cv_predict_primal(X[:n_fit], Y[:n_fit], X[n_fit:])

    a_all = torch.as_tensor(np.asarray(ALPHAS, np.float64), device=dev)
    Xd, Yd = X.double(), Y[:n_fit].double()
    eye = torch.eye(p, device=dev, dtype=torch.float64)

    def solve(rows, a):
        Xt = Xd[rows]
        L = torch.linalg.cholesky(Xt.T @ Xt + a * eye)
        return torch.cholesky_solve(Xt.T @ Yd[rows], L)

    loss = torch.zeros((len(a_all), v), device=dev, dtype=torch.float64)
    for tr, va in kfold_splits(n_fit, 5):
        tr_t, va_t = torch.as_tensor(tr, device=dev), torch.as_tensor(va, device=dev)
        for j, a in enumerate(a_all):
            err = Yd[va_t] - Xd[va_t] @ solve(tr_t, float(a))
            loss[j] -= (err * err).sum(0)
    loss /= 5
    best = torch.argmax(loss, dim=0)
    ref_alphas = a_all[best].cpu().numpy()
    # per voxel: the chosen alpha is the closed form's, unless two alphas' CV losses tie to
    # fp64 rounding (relative 1e-9)
    srt = torch.sort(loss, dim=0, descending=True).values
    tie = ((srt[0] - srt[1]).abs() <= 1e-9 * srt[0].abs()).cpu().numpy()
    assert np.all((alphas == ref_alphas) | tie), (alphas, ref_alphas)
    assert len(set(alphas.tolist())) >= 3  # the SNR sweep exercises several alphas
    all_rows = torch.arange(n_fit, device=dev)
    ref = torch.empty((n_new, v), device=dev, dtype=torch.float64)
    for a in sorted(set(alphas.tolist())):
        cols = torch.as_tensor(np.nonzero(alphas == a)[0], device=dev)
        ref[:, cols] = Xd[n_fit:] @ solve(all_rows, a)[:, cols]
    rel = float((pred.double() - ref).abs().max() / ref.abs().max())
    record_margin("ridge_full_size_vs_closed_form", n_fit=n_fit, n_new=n_new, p=p, voxels=v, rel_err=rel,
                  distinct_alphas=len(set(alphas.tolist())))
    assert rel <= 1e-6, rel
