"""Encoding score: cross-validated ridge regression from model features to voxel responses,
scored by mean per-voxel Pearson r (visreps/analysis/encoding_score.py).

Same flow, names and result record as the reference (`compute_encoding_score`,
encoding_score.py:65-260):

1. ``RandomState(seed).permutation(n_train)`` splits train 80/20 into fit/val; Y is
   z-normalised with fit-only statistics. For every layer: X z-normalised with fit
   statistics, RidgeCV on fit, mean Pearson r on val. Best layer = first strict max.
2. Optional PCA reconstruction of the best layer (train-fitted, sklearn as the reference).
3. Refit RidgeCV for the best layer on all train rows (train statistics), predict test.
4. Bootstrap: the same RandomState draws ``choice(n_test, int(0.9 n_test))`` per
   iteration; score = mean per-voxel r on the subsample; CI = numpy percentiles.

The ridge solver restates himalaya 0.4.9's ``RidgeCV(alphas=logspace(-10, 10, 20), cv=5,
fit_intercept=False)`` (solver "svd", himalaya/ridge/_solvers.py ``solve_ridge_cv_svd``;
himalaya is not vendored in the reference and not installed here):
sklearn ``KFold(5)`` (contiguous folds, no shuffle) over the fit rows; per fold and alpha
the validation predictions of the ridge fit on the other folds; score per target =
negative summed squared error (``l2_neg_loss``), averaged over folds; per-target best
alpha = first argmax over alphas (``local_alpha=True``); refit on all fit rows with each
target's alpha. Wide layers (p >= n) run in kernel (dual) form: with K = X X^T = Q diag(lam) Q^T the fit
on rows T predicts rows V as K[V, T] Q diag(1 / (lam + alpha)) Q^T Y[T], which equals the
primal SVD solution X_V V diag(s / (s^2 + alpha)) U^T Y with lam = s^2. Every component
with lam above the fp64 rounding floor of the decomposition (n * eps_64 * lam_max) is kept,
as himalaya's SVD solver keeps every singular value. Narrow layers (p < n) run the primal
form on the p x p Grams X_T^T X_T of each fold (``ridge_cv_predict_primal``). The ridge
Grams are fp64 (the solves are conditioning-sensitive) on the fp64 MFMA tiles of
``vr_gram64_f32`` (``gram64`` = X X^T, ``gram64_cols`` = X^T X: upper triangle only, fp32
products exact in fp64); the eigendecompositions and the small dense products run in fp64 through torch
(rocSOLVER / rocBLAS); the statistic and its bootstrap run in ``vr_corr_score_f32``. The
MFMA Gram kernel (``vr_gram_f32``, ``gram``) stays available for fp32 callers.

Parity: the correlation statistic follows himalaya's ``correlation_score`` (checked
against scipy.stats.pearsonr, as the reference's tests/test_encoding_score.py:1251-1376)
and the ridge solution against a closed-form numpy ridge; the alpha selection rule is
restated from himalaya's published algorithm and is **parity unpinned** (no himalaya
output is available offline). Encoding score is refused for things-behavior
(alignment.py:91-95).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from .._lib import check, lib, stream_of, workspace
from ..utils import rprint
from ._random import LegacyRandomState
from .rsa import percentile

__all__ = ["compute_encoding_score", "gram", "gram64", "gram64_cols", "corr_score", "ridge_cv_predict",
           "ridge_cv_predict_primal", "kfold_splits", "ALPHAS"]

ALPHAS = np.logspace(-10, 10, 20)


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def _device(t: torch.Tensor) -> torch.device:
    if t.is_cuda:
        return t.device
    if not torch.cuda.is_available():
        raise RuntimeError("visreps_amd encoding score needs a HIP (MI355X) device")
    return torch.device("cuda", torch.cuda.current_device())


def gram(x: torch.Tensor) -> torch.Tensor:
    """G = x x^T (fp32, exactly symmetric) on the MFMA Gram kernel (vr_gram_f32)."""
    dev = _device(x)
    x = x.to(dev, torch.float32).contiguous()
    n, d = x.shape
    out = torch.empty((n, n), dtype=torch.float32, device=dev)
    if n == 0:
        return out
    if d == 0:
        return out.zero_()
    L = lib()
    ws = workspace.get(dev, L.vr_rdm_pearson_workspace(n, d), "rdm")
    with torch.cuda.device(dev):
        check(L.vr_gram_f32(_ptr(x), n, d, x.stride(0), _ptr(out), n, _ptr(ws), ws.numel(),
                            stream_of(dev)), "vr_gram_f32")
    return out


def corr_score(y: torch.Tensor, p: torch.Tensor, idx: Optional[np.ndarray] = None,
               voxels: bool = False):
    """Mean over columns of the per-column Pearson r of y and p (himalaya
    correlation_score(...).mean()). idx (draws, k): one score per row subset (float64
    numpy array); idx None: one score over all rows (float). voxels=True also returns the
    per-column r of each draw."""
    dev = _device(y)
    y = y.to(dev, torch.float32).contiguous()
    p = p.to(dev, torch.float32).contiguous()
    if y.shape != p.shape or y.ndim != 2:
        raise ValueError(f"corr_score: shapes {tuple(y.shape)} and {tuple(p.shape)}")
    n, v = y.shape
    if idx is None:
        draws, k, it = 1, n, None
    else:
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        if idx.ndim != 2 or idx.size == 0 or idx.min() < 0 or idx.max() >= n:
            raise ValueError("corr_score: idx must be a non-empty (draws, k) array of rows")
        draws, k = idx.shape
        it = torch.from_numpy(idx).to(dev)
    scores = torch.empty(draws, dtype=torch.float64, device=dev)
    vox = torch.empty((draws, v), dtype=torch.float64, device=dev) if voxels else None
    L = lib()
    ws = workspace.get(dev, L.vr_corr_score_workspace(v, draws), "corr_score")
    with torch.cuda.device(dev):
        check(L.vr_corr_score_f32(_ptr(y), _ptr(p), n, v, v, _ptr(it) if it is not None else None,
                                  k, draws, _ptr(scores), _ptr(vox) if vox is not None else None,
                                  _ptr(ws), ws.numel(), stream_of(dev)), "vr_corr_score_f32")
    s = scores.cpu().numpy()
    out = float(s[0]) if idx is None else s
    return (out, vox) if voxels else out


def kfold_splits(n: int, n_splits: int = 5):
    """sklearn KFold(n_splits) without shuffle: contiguous folds, the first n % n_splits
    one row longer. Yields (train, val) int64 index arrays."""
    if n < n_splits:
        raise ValueError(f"Cannot have number of splits n_splits={n_splits} greater than the "
                         f"number of samples: n_samples={n}.")
    sizes = np.full(n_splits, n // n_splits, dtype=np.int64)
    sizes[: n % n_splits] += 1
    start = 0
    for s in sizes:
        val = np.arange(start, start + s)
        train = np.concatenate([np.arange(0, start), np.arange(start + s, n)])
        yield train, val
        start += s


def _eig(K: torch.Tensor):
    """Eigendecomposition of an fp64 Gram. Every component with lam above the fp64
    rounding floor of the decomposition (n eps_64 lam_max) is kept, as himalaya's SVD
    solver keeps every singular value: below that floor lam is rounding noise whose
    1/(lam + alpha) would only amplify it."""
    lam, Q = torch.linalg.eigh(K)
    tol = lam.abs().max() * K.size(0) * float(np.finfo(np.float64).eps)
    keep = lam > tol
    return lam, Q, keep


def _gram64(x: torch.Tensor, rows: bool) -> torch.Tensor:
    if x.dtype == torch.float64:
        # the kernel reads fp32 (exact products in fp64); a silent cast would drop the low bits
        raise TypeError("gram64 / gram64_cols take fp32 (or narrower) input: cast float64 data "
                        "explicitly, knowing the fp32 rounding")
    dev = _device(x)
    x = x.to(dev, torch.float32)
    if x.ndim != 2 or x.stride(1) != 1:
        x = x.contiguous()
    n, p = x.shape
    m = n if rows else p
    out = torch.empty((m, m), dtype=torch.float64, device=dev)
    if m == 0:
        return out
    if (p if rows else n) == 0:
        return out.zero_()
    L = lib()
    ws = workspace.get(dev, L.vr_gram64_workspace(n, p, int(rows)), "gram64")
    with torch.cuda.device(dev):
        check(L.vr_gram64_f32(_ptr(x), n, p, x.stride(0), int(rows), _ptr(out), m, _ptr(ws), ws.numel(),
                              stream_of(dev)), "vr_gram64_f32")
    return out


def gram64(x: torch.Tensor) -> torch.Tensor:
    """x x^T in fp64 for fp32 x (the kernel form's K; the ridge solves are
    conditioning-sensitive): the fp64 MFMA tiles of vr_gram64_f32, upper triangle only,
    mirrored (the RSA Grams use vr_gram_f32)."""
    return _gram64(x, rows=True)


def gram64_cols(x: torch.Tensor) -> torch.Tensor:
    """x^T x in fp64 for fp32 x (the primal form's p x p Gram), vr_gram64_f32."""
    return _gram64(x, rows=False)


def _dual_predict(K_new: torch.Tensor, lam, Q, keep, Y: torch.Tensor, alphas: torch.Tensor):
    """Predictions for rows of K_new (new x fit) with per-target (v,) or scalar alphas."""
    W = Q.T @ Y  # (r, v)
    denom = lam[:, None] + alphas.reshape(1, -1)
    W = torch.where(keep[:, None], W / denom, torch.zeros_like(W))
    return (K_new @ Q) @ W


def ridge_cv_predict(K: torch.Tensor, fit: np.ndarray, new: np.ndarray, Y_fit: torch.Tensor,
                     alphas=ALPHAS, cv: int = 5):
    """RidgeCV(alphas, cv, fit_intercept=False) fit on rows `fit` of the kernel K (= X X^T
    over all rows), predicting rows `new`. Returns (predictions fp32 (len(new), v), best
    alpha per target)."""
    dev = K.device
    Kd = K.double()
    Yd = Y_fit.to(dev, torch.float64)
    fit_t = torch.as_tensor(np.asarray(fit), device=dev)
    new_t = torch.as_tensor(np.asarray(new), device=dev)
    a = torch.as_tensor(np.asarray(alphas, dtype=np.float64), device=dev)
    n_fit, v = Yd.shape
    scores = torch.zeros((len(a), v), dtype=torch.float64, device=dev)
    for tr, va in kfold_splits(n_fit, cv):
        rows_tr, rows_va = fit_t[tr], fit_t[va]
        lam, Q, keep = _eig(Kd[rows_tr][:, rows_tr])
        KQ = Kd[rows_va][:, rows_tr] @ Q
        QY = Q.T @ Yd[tr]
        for j in range(len(a)):
            W = torch.where(keep[:, None], QY / (lam[:, None] + a[j]), torch.zeros_like(QY))
            err = Yd[va] - KQ @ W
            scores[j] += -(err * err).sum(0)  # l2_neg_loss per target
    scores /= cv
    best = torch.argmax(scores, dim=0)  # first maximum, as argmax
    alpha_t = a[best]
    lam, Q, keep = _eig(Kd[fit_t][:, fit_t])
    pred = _dual_predict(Kd[new_t][:, fit_t], lam, Q, keep, Yd, alpha_t)
    return pred.float(), alpha_t.cpu().numpy()


def ridge_cv_predict_primal(X_fit: torch.Tensor, Y_fit: torch.Tensor, X_new: torch.Tensor,
                            alphas=ALPHAS, cv: int = 5):
    """The same RidgeCV in primal form, for layers narrower than the fit set (p < n): per
    fold the fp64 p x p Gram X_T^T X_T (gram64), its
    eigendecomposition V diag(lam) V^T, and predictions X_V V diag(1/(lam + alpha))
    V^T X_T^T Y_T (= the SVD solution with lam = s^2). Returns (predictions fp32, alphas)."""
    dev = X_fit.device
    Xd = X_fit.to(torch.float32)
    Yd = Y_fit.to(dev, torch.float64)
    a = torch.as_tensor(np.asarray(alphas, dtype=np.float64), device=dev)
    n_fit, v = Yd.shape

    def solve(rows):
        Xt = Xd[rows]
        lam, V, keep = _eig(gram64_cols(Xt))
        VtXtY = V.T @ (Xt.double().T @ Yd[rows])
        return lam, V, keep, VtXtY

    scores = torch.zeros((len(a), v), dtype=torch.float64, device=dev)
    for tr, va in kfold_splits(n_fit, cv):
        lam, V, keep, W0 = solve(torch.as_tensor(tr, device=dev))
        XV = Xd[torch.as_tensor(va, device=dev)].double() @ V
        Yva = Yd[torch.as_tensor(va, device=dev)]
        for j in range(len(a)):
            W = torch.where(keep[:, None], W0 / (lam[:, None] + a[j]), torch.zeros_like(W0))
            err = Yva - XV @ W
            scores[j] += -(err * err).sum(0)
    scores /= cv
    alpha_t = a[torch.argmax(scores, dim=0)]
    lam, V, keep, W0 = solve(torch.arange(n_fit, device=dev))
    W = torch.where(keep[:, None], W0 / (lam[:, None] + alpha_t[None, :]), torch.zeros_like(W0))
    pred = (X_new.to(dev, torch.float64) @ V) @ W
    return pred.float(), alpha_t.cpu().numpy()


def _znorm(X, mean, std):
    """Z-normalise with precomputed statistics (encoding_score.py:28-30)."""
    return (X - mean) / std


def _znorm_fit(X):
    """Z-normalise X with its own column statistics, std + 1e-8 (torch's unbiased std,
    encoding_score.py:33-37). Returns (normalised, mean, std)."""
    mean = X.mean(dim=0)
    std = X.std(dim=0) + 1e-8
    return _znorm(X, mean, std), mean, std


def _flatten_to_cpu(acts) -> Dict[str, torch.Tensor]:
    """Flatten 4-D -> 2-D and return CPU float32 copies; the input dict is not mutated
    (encoding_score.py:39-44). compute_encoding_score keeps activations on the device
    (_flatten); this is the reference's host-side helper, kept for its callers."""
    return {layer: (a.flatten(start_dim=1) if a.ndim > 2 else a).cpu().float()
            for layer, a in acts.items()}


def _flatten(acts, dev) -> Dict[str, torch.Tensor]:
    """Flatten 4-D -> 2-D float32 on the device; new tensors, inputs untouched
    (encoding_score.py:40-45)."""
    return {layer: (a.flatten(start_dim=1) if a.ndim > 2 else a).to(dev, torch.float32)
            for layer, a in acts.items()}


def _fit_and_score(X_fit: torch.Tensor, Y_fit: torch.Tensor, X_new: torch.Tensor,
                   Y_new: torch.Tensor, alphas, backend=None):  # noqa: ARG001
    """RidgeCV on (X_fit, Y_fit), predictions for X_new and their mean Pearson r against
    Y_new (encoding_score.py:47-62). One fp64 Gram of the stacked rows gives both kernel
    blocks. `backend` (the reference's himalaya backend) is accepted and unused: the
    arrays go to X_fit's HIP device. X_new / Y_new may be CPU tensors, as the reference
    allows for X_te."""
    X_fit = torch.as_tensor(X_fit)
    dev = _device(X_fit)
    X_fit = X_fit.to(dev)
    Y_fit = torch.as_tensor(Y_fit).to(dev)
    X_new = torch.as_tensor(X_new).to(dev, X_fit.dtype)
    Y_new = torch.as_tensor(Y_new).to(dev)
    n_fit, p = X_fit.shape
    if p < n_fit:  # narrow layer: p x p Grams per fold (primal)
        pred, _ = ridge_cv_predict_primal(X_fit, Y_fit, X_new, alphas)
        return pred, corr_score(Y_new, pred)
    K = gram64(torch.cat([X_fit, X_new], dim=0))
    fit = np.arange(n_fit)
    new = np.arange(n_fit, K.size(0))
    pred, _ = ridge_cv_predict(K, fit, new, Y_fit, alphas)
    return pred, corr_score(Y_new, pred)


def compute_encoding_score(selection, evaluation, bootstrap: bool = True,
                           n_bootstrap: int = 1000, seed: int = 42, verbose: bool = False,
                           reconstruct_pca_k: Optional[int] = None) -> List[Dict]:
    """Train/test encoding score (encoding_score.py:65-260); see the module docstring."""
    dev = _device(selection.neural)
    compare_method = "pearson"
    rng = LegacyRandomState(seed)
    alphas = ALPHAS

    train_acts = _flatten(selection.activations, dev)
    test_acts = _flatten(evaluation.activations, dev)
    Y_train_raw = selection.neural.to(dev, torch.float32)
    Y_test_raw = evaluation.neural.to(dev, torch.float32)
    n_train, n_test, n_voxels = Y_train_raw.size(0), Y_test_raw.size(0), Y_train_raw.size(1)
    if verbose:
        rprint(f"Train/test encoding: {n_train} train, {n_test} test, {n_voxels} voxels "
               f"(MI355X kernel ridge)", style="info")

    # 1. layer selection on train (80/20 fit/val)
    split = int(0.8 * n_train)
    perm = rng.permutation(n_train)
    fit_idx = torch.as_tensor(perm[:split], device=dev)
    val_idx = torch.as_tensor(perm[split:], device=dev)
    Y_fit, Y_fit_mean, Y_fit_std = _znorm_fit(Y_train_raw[fit_idx])
    Y_val = _znorm(Y_train_raw[val_idx], Y_fit_mean, Y_fit_std)

    selection_scores = []
    best_layer, best_score = None, -float("inf")
    for layer, acts in train_acts.items():
        X_fit, fit_mean, fit_std = _znorm_fit(acts[fit_idx])
        X_val = _znorm(acts[val_idx], fit_mean, fit_std)
        _, score = _fit_and_score(X_fit, Y_fit, X_val, Y_val, alphas)
        selection_scores.append({"layer": layer, "score": score})
        if verbose:
            rprint(f"  [select] {layer:<15} r={score:.4f}  ({acts.size(1)} features)", style="info")
        if score > best_score:
            best_score, best_layer = score, layer
        del X_fit, X_val
    if best_layer is None:  # every score NaN: the reference would fail at the same point
        raise ValueError("no layer produced a finite selection score")

    # 1b. optional PCA reconstruction (train-fitted, as the reference: sklearn on the host)
    if reconstruct_pca_k is not None:
        from sklearn.decomposition import PCA as _PCA

        tr = train_acts[best_layer].cpu().numpy()
        te = test_acts[best_layer].cpu().numpy()
        pca = _PCA(n_components=min(reconstruct_pca_k, tr.shape[1]))
        pca.fit(tr)
        train_acts[best_layer] = torch.from_numpy(
            pca.inverse_transform(pca.transform(tr)).astype(np.float32)).to(dev)
        test_acts[best_layer] = torch.from_numpy(
            pca.inverse_transform(pca.transform(te)).astype(np.float32)).to(dev)

    # 2. refit on full train, evaluate on test
    X_train, train_mean, train_std = _znorm_fit(train_acts[best_layer])
    X_test = _znorm(test_acts[best_layer], train_mean, train_std)
    Y_train, Y_mean, Y_std = _znorm_fit(Y_train_raw)
    Y_test = _znorm(Y_test_raw, Y_mean, Y_std)
    pred_test, point_estimate = _fit_and_score(X_train, Y_train, X_test, Y_test, alphas)
    _, vox = corr_score(Y_test, pred_test, voxels=True)
    median_r = float(vox[0].median())
    if verbose:
        rprint(f"  Test encoding: mean r={point_estimate:.4f}, median r={median_r:.4f} "
               f"({n_voxels} voxels)", style="highlight")

    # 3. bootstrap on the test predictions: the same RandomState continues
    ci_low = ci_high = None
    bootstrap_scores_list = None
    if bootstrap:
        k = int(n_test * 0.9)
        idx = np.stack([rng.choice(n_test, size=k, replace=False) for _ in range(n_bootstrap)])
        scores = corr_score(Y_test, pred_test, idx)
        ci_low, ci_high = percentile(scores, 2.5), percentile(scores, 97.5)
        bootstrap_scores_list = [float(s) for s in scores]

    msg = f"  Encoding  | {best_layer} = {point_estimate:.4f}"
    if bootstrap:
        msg += f"  [95% CI: {ci_low:.4f}, {ci_high:.4f}]"
    rprint(msg, style="highlight")
    result = {
        "layer": best_layer,
        "compare_method": compare_method,
        "score": point_estimate,
        "ci_low": ci_low,
        "ci_high": ci_high,
        "analysis": "encoding_score",
        "layer_selection_scores": selection_scores,
    }
    if bootstrap_scores_list is not None:
        result["bootstrap_scores"] = bootstrap_scores_list
    return [result]
