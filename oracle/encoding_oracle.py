"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference's encoding score (visreps/analysis/encoding_score.py)
and of the himalaya 0.4.9 pieces it calls, used only as the checker by tests/. The
product path (visreps_amd/analysis/encoding_score.py) never imports it.

* ``correlation_score`` — himalaya/scoring.py: mean over rows of zscore(y) * zscore(p)
  with population std, per target (pinned against scipy.stats.pearsonr, as the
  reference's tests/test_encoding_score.py:1251-1376 do).
* ``ridge_cv`` — himalaya ``RidgeCV(alphas, cv=5, fit_intercept=False)``, solver "svd"
  (``solve_ridge_cv_svd``) in its PRIMAL form: per sklearn KFold(5) split the SVD
  X_tr = U diag(s) V^T, predictions X_val V diag(s / (s^2 + alpha)) U^T Y_tr, score
  ``l2_neg_loss`` (negative summed squared error) per target, averaged over folds, best
  alpha per target by first argmax; refit on all rows with per-target alphas. The GPU
  product runs the DUAL (kernel) form, so the two formulations cross-check each other.
  The selection rule itself is restated from himalaya's published algorithm: parity
  unpinned (himalaya is neither vendored nor installed).
* ``compute_encoding_score`` — encoding_score.py:65-260 with numpy.random.RandomState.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
from sklearn.model_selection import KFold

ALPHAS = np.logspace(-10, 10, 20)  # encoding_score.py:108


def correlation_score(y: np.ndarray, p: np.ndarray) -> np.ndarray:
    y = np.asarray(y, np.float64)
    p = np.asarray(p, np.float64)
    zy = (y - y.mean(0)) / y.std(0)
    zp = (p - p.mean(0)) / p.std(0)
    return (zy * zp).mean(0)


def _svd_predict(X_tr, Y_tr, X_new, alphas_per_target):
    U, s, Vt = np.linalg.svd(X_tr, full_matrices=False)
    UTY = U.T @ Y_tr
    XV = X_new @ Vt.T
    # himalaya solve_ridge_cv_svd: every singular value, s / (s^2 + alpha)
    f = s[:, None] / (s[:, None] ** 2 + alphas_per_target[None, :])
    return XV @ (f * UTY)


def ridge_cv(X: np.ndarray, Y: np.ndarray, X_new: np.ndarray, alphas=ALPHAS, cv: int = 5):
    """Predictions for X_new and the per-target alphas (float64 arithmetic)."""
    X = np.asarray(X, np.float64)
    Y = np.asarray(Y, np.float64)
    X_new = np.asarray(X_new, np.float64)
    alphas = np.asarray(alphas, np.float64)
    scores = np.zeros((len(alphas), Y.shape[1]))
    for tr, va in KFold(n_splits=cv).split(X):
        for j, a in enumerate(alphas):
            pred = _svd_predict(X[tr], Y[tr], X[va], np.full(Y.shape[1], a))
            scores[j] += -((Y[va] - pred) ** 2).sum(0)
    scores /= cv
    best = alphas[np.argmax(scores, axis=0)]
    return _svd_predict(X, Y, X_new, best), best


def _znorm_fit(X):
    mean = X.mean(0)
    std = X.std(0, ddof=1) + 1e-8  # torch .std(dim=0): unbiased
    return (X - mean) / std, mean, std


def compute_encoding_score(train_acts: Dict[str, np.ndarray], Y_train: np.ndarray,
                           test_acts: Dict[str, np.ndarray], Y_test: np.ndarray,
                           bootstrap: bool = True, n_bootstrap: int = 1000,
                           seed: int = 42) -> Dict:
    rng = np.random.RandomState(seed)
    n_train, n_test = Y_train.shape[0], Y_test.shape[0]
    split = int(0.8 * n_train)
    perm = rng.permutation(n_train)
    fit_idx, val_idx = perm[:split], perm[split:]
    Y_fit, ym, ys = _znorm_fit(Y_train[fit_idx].astype(np.float64))
    Y_val = (Y_train[val_idx] - ym) / ys
    sel, best_layer, best = [], None, -np.inf
    for layer, a in train_acts.items():
        a = a.reshape(a.shape[0], -1).astype(np.float64)
        X_fit, xm, xs = _znorm_fit(a[fit_idx])
        X_val = (a[val_idx] - xm) / xs
        pred, _ = ridge_cv(X_fit, Y_fit, X_val)
        score = float(correlation_score(Y_val, pred).mean())
        sel.append({"layer": layer, "score": score})
        if score > best:
            best, best_layer = score, layer
    a_tr = train_acts[best_layer].reshape(n_train, -1).astype(np.float64)
    a_te = test_acts[best_layer].reshape(n_test, -1).astype(np.float64)
    X_tr, xm, xs = _znorm_fit(a_tr)
    X_te = (a_te - xm) / xs
    Y_tr, ym, ys = _znorm_fit(Y_train.astype(np.float64))
    Y_te = (Y_test - ym) / ys
    pred, alphas = ridge_cv(X_tr, Y_tr, X_te)
    point = float(correlation_score(Y_te, pred).mean())
    out = {"layer": best_layer, "score": point, "layer_selection_scores": sel,
           "alphas": alphas, "pred": pred, "Y_test": Y_te}
    if bootstrap:
        k = int(n_test * 0.9)
        scores = np.empty(n_bootstrap)
        for i in range(n_bootstrap):
            idx = rng.choice(n_test, size=k, replace=False)
            scores[i] = correlation_score(Y_te[idx], pred[idx]).mean()
        out["bootstrap_scores"] = scores
        out["ci_low"] = float(np.percentile(scores, 2.5))
        out["ci_high"] = float(np.percentile(scores, 97.5))
    return out
