"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A numpy/scipy restatement of the reference's RSA eval arithmetic, used exclusively as
the checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. The
product path (visreps_amd/) never imports it.

Pinning: the reference package itself may not be run here (the
survey's attempt to run its test suite was refused), so this restatement is pinned by
  * the known-answer and property tests transcribed from
    /root/reference/tests/test_rsa_bootstrap.py (tests/test_oracle.py),
  * scipy.stats.spearmanr / pearsonr / kendalltau (the third-party functions the
    reference calls at rsa.py:43-47,121-122; scipy 1.16.2 pinned in uv.lock, 1.15.3 here,
    same rankdata+corrcoef definition),
  * numpy.random.RandomState (the reference's index stream, evals.py:356,362-364).
Golden fixtures in tests/golden/ are generated from this module by
tests/golden/make_golden.py after those checks pass.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import scipy.stats


def _rank(x: np.ndarray) -> np.ndarray:
    """Ordinal row ranks by double argsort (rsa.py:50-52), stable ties."""
    return np.argsort(np.argsort(x, axis=1, kind="stable"), axis=1, kind="stable").astype(np.float32)


def compute_rdm(X, correlation: str = "Pearson", correction: float = 1e-12) -> np.ndarray:
    """rsa.py:59-93 in float32: centre, std with correction, zero-variance guard,
    cov = x x^T / D, corr = cov / (s_i s_j + c), clamp, diag 1, 1 - corr."""
    corr = correlation.lower()
    if corr not in {"pearson", "spearman"}:
        raise ValueError("correlation must be 'Pearson' or 'Spearman'")
    x = np.array(X, dtype=np.float32, copy=True)
    if corr == "spearman":
        x = _rank(x)
    x -= x.mean(axis=1, keepdims=True, dtype=np.float32).astype(np.float32)
    c32 = np.float32(correction)
    std = np.sqrt(np.mean(x * x, axis=1, dtype=np.float32) + c32).astype(np.float32)
    std[std < correction * 10] = np.float32(1.0)
    cov = (x @ x.T) / np.float32(x.shape[1])
    corr_mat = cov / (std[:, None] * std[None, :] + c32)
    np.clip(corr_mat, -1, 1, out=corr_mat)
    np.fill_diagonal(corr_mat, 1.0)
    return (np.float32(1.0) - corr_mat).astype(np.float32)


def _kendall_tau_a(x: np.ndarray, y: np.ndarray):
    """rsa.py:22-40: tau-a = tau-b * sqrt((n0-tx)(n0-ty)) / n0."""
    n = len(x)
    if n < 2:
        return (float("nan"), float("nan"))
    tau_b = scipy.stats.kendalltau(x, y).statistic
    if np.isnan(tau_b):
        return (float("nan"), float("nan"))
    n0 = n * (n - 1) // 2
    t_x = sum(c * (c - 1) // 2 for c in np.unique(x, return_counts=True)[1])
    t_y = sum(c * (c - 1) // 2 for c in np.unique(y, return_counts=True)[1])
    denom = np.sqrt(np.float64(n0 - t_x) * np.float64(n0 - t_y))
    tau_a = float("nan") if denom == 0 else float(tau_b * denom / n0)
    return (tau_a, float("nan"))


_CORR_FUNCS = {
    "pearson": scipy.stats.pearsonr,
    "spearman": scipy.stats.spearmanr,
    "kendall": _kendall_tau_a,
}


def compute_rdm_correlation(rdm1, rdm2, correlation: str = "Kendall") -> float:
    """rsa.py:96-129: same check order (shape, n<=1, empty, method), NaN on failure."""
    rdm1 = np.asarray(rdm1)
    rdm2 = np.asarray(rdm2)
    if rdm1.shape != rdm2.shape or rdm1.ndim != 2:
        raise ValueError("RDMs must share the same 2-D shape")
    n = rdm1.shape[0]
    if n <= 1:
        return float("nan")
    iu = np.triu_indices(n, 1)
    v1 = rdm1[iu].astype(np.float32)
    v2 = rdm2[iu].astype(np.float32)
    if v1.size == 0:
        return float("nan")
    corr = correlation.lower()
    if corr not in _CORR_FUNCS:
        raise ValueError("correlation must be 'Pearson', 'Spearman', or 'Kendall'")
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            val, _ = _CORR_FUNCS[corr](v1, v2)
        except Exception:
            return float("nan")
    if np.isnan(val):
        return float("nan")
    return float(val)


def midrank_spearman(v1: np.ndarray, v2: np.ndarray) -> float:
    """Spearman as Pearson of average ranks computed with exact integer arithmetic
    (doubled midranks); an independent check of scipy.stats.spearmanr's definition."""
    m = len(v1)
    if m < 2:
        return float("nan")
    r1 = scipy.stats.rankdata(v1, method="average") * 2
    r2 = scipy.stats.rankdata(v2, method="average") * 2
    a = r1.astype(np.int64)
    b = r2.astype(np.int64)
    mu = m * (m + 1) ** 2

    def exact_dot(x, y):  # each product < (2m)^2 fits int64; chunk sums summed as Python ints
        p = x * y
        return sum(int(c) for c in np.add.reduceat(p, np.arange(0, m, 4096)))

    sab, saa, sbb = exact_dot(a, b), exact_dot(a, a), exact_dot(b, b)
    num, va, vb = sab - mu, saa - mu, sbb - mu
    if va <= 0 or vb <= 0:
        return float("nan")
    return max(-1.0, min(1.0, num / math.sqrt(float(va) * float(vb))))


def bootstrap_rsa(model_rdm, neural_rdm, n_bootstrap: int = 1000, seed: int = 42,
                  method: str = "Spearman"):
    """evals.py:341-373: point estimate, fresh RandomState(seed), n_bootstrap draws of
    choice(n, int(0.9n), replace=False), sub-RDM correlation, linear percentiles."""
    model_rdm = np.asarray(model_rdm)
    neural_rdm = np.asarray(neural_rdm)
    point = compute_rdm_correlation(model_rdm, neural_rdm, correlation=method)
    rng = np.random.RandomState(seed)
    n = neural_rdm.shape[0]
    k = int(n * 0.9)
    scores = np.empty(n_bootstrap, dtype=np.float64)
    for i in range(n_bootstrap):
        idx = rng.choice(n, size=k, replace=False)
        scores[i] = compute_rdm_correlation(model_rdm[idx][:, idx], neural_rdm[idx][:, idx],
                                            correlation=method)
    if n_bootstrap == 0:
        return point, scores, None, None
    return (point, scores, float(np.percentile(scores, 2.5)),
            float(np.percentile(scores, 97.5)))


def bootstrap_scores_at(model_rdm, neural_rdm, draws, seed: int = 42, method: str = "Spearman"):
    """Scores of selected bootstrap draws of evals.py:355-369 (0-based draw numbers): the
    RandomState(seed) stream is drawn in full up to the last one, as the reference loop
    does, but only the listed draws' sub-RDMs are scored (a full-size check of late draws
    without the ~2 h of all 1000 Spearmans). Returns {draw: score}."""
    model_rdm = np.asarray(model_rdm)
    neural_rdm = np.asarray(neural_rdm)
    want = set(int(d) for d in draws)
    rng = np.random.RandomState(seed)
    n = neural_rdm.shape[0]
    k = int(n * 0.9)
    out = {}
    for i in range(max(want) + 1):
        idx = rng.choice(n, size=k, replace=False)
        if i in want:
            out[i] = compute_rdm_correlation(model_rdm[idx][:, idx], neural_rdm[idx][:, idx], correlation=method)
    return out


def compute_rsa(cfg: Dict, sel_acts: Dict[str, np.ndarray], sel_neural: np.ndarray,
                eval_acts: Dict[str, np.ndarray], eval_neural: np.ndarray,
                n_select: Optional[int] = None, bootstrap: bool = True,
                n_bootstrap: int = 1000, seed: int = 42, rdm_fn=None) -> List[Dict]:
    """rsa.py:132-281 without the printing: one RandomState(seed) shared by the
    n_select draw and the bootstrap draws; first strict maximum wins the selection.
    rdm_fn replaces compute_rdm (a test hands in the product's RDM kernel to check the
    selection / Spearman / bootstrap logic on bit-identical RDMs)."""
    compute_rdm_ = rdm_fn or compute_rdm
    method = cfg.get("compare_method", "spearman").lower()
    rng = np.random.RandomState(seed)
    n_train = sel_neural.shape[0]
    n_test = eval_neural.shape[0]
    if n_select is not None and n_select < n_train:
        sel_idx = rng.choice(n_train, size=n_select, replace=False)
    else:
        sel_idx = np.arange(n_train)
    neural_rdm_sel = compute_rdm_(sel_neural[sel_idx])
    selection_scores = []
    best_layer, best_score = None, -float("inf")
    for layer, acts in sel_acts.items():
        a = acts[sel_idx]
        flat = a.reshape(a.shape[0], -1)
        score = compute_rdm_correlation(compute_rdm_(flat), neural_rdm_sel,
                                        correlation=method.capitalize())
        selection_scores.append({"layer": layer, "score": score})
        if score > best_score:
            best_score, best_layer = score, layer
    t = eval_acts[best_layer]
    test_model_rdm = compute_rdm_(t.reshape(t.shape[0], -1))
    test_neural_rdm = compute_rdm_(eval_neural)
    point = compute_rdm_correlation(test_model_rdm, test_neural_rdm,
                                    correlation=method.capitalize())
    ci_low = ci_high = None
    scores_list = None
    if bootstrap:
        k = int(n_test * 0.9)
        scores = np.empty(n_bootstrap, dtype=np.float64)
        for i in range(n_bootstrap):
            idx = rng.choice(n_test, size=k, replace=False)
            scores[i] = compute_rdm_correlation(test_model_rdm[idx][:, idx],
                                                test_neural_rdm[idx][:, idx],
                                                correlation=method.capitalize())
        ci_low = float(np.percentile(scores, 2.5))
        ci_high = float(np.percentile(scores, 97.5))
        scores_list = scores.tolist()
    result = {"layer": best_layer, "compare_method": method, "score": point,
              "ci_low": ci_low, "ci_high": ci_high, "analysis": "rsa",
              "layer_selection_scores": selection_scores}
    if scores_list is not None:
        result["bootstrap_scores"] = scores_list
    return [result]


def synthetic_features(n: int, dims, seed: int = 20260306, latent: int = 64,
                       relu=None, noise: float = 2.0) -> List[np.ndarray]:
    """SURVEY.md §8(d) synthetic inputs: Z ~ N(0,1)^{n x latent};
    X_l = relu(Z W_l + noise*E_l) (no relu where relu[l] is False), W_l ~ N(0, 1/latent)."""
    rng = np.random.default_rng(seed)
    z = rng.standard_normal((n, latent), dtype=np.float32)
    out = []
    for i, d in enumerate(dims):
        w = rng.standard_normal((latent, d), dtype=np.float32) / np.float32(math.sqrt(latent))
        x = z @ w + np.float32(noise) * rng.standard_normal((n, d), dtype=np.float32)
        if relu is None or relu[i]:
            np.maximum(x, 0, out=x)
        out.append(x.astype(np.float32))
    return out
