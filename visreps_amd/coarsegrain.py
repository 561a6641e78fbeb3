"""PCA of feature dumps for the coarse-grained PCA labels, on the MI355X (SURVEY.md §8(f)
rank 4: "PCA covariance for coarse labels").

Mirrors scripts/coarsegrain/compute_eigenvectors.py: ``batched_pca(X, n_components,
batch_size)`` returns ``(eigenvectors[:, top], eigenvalues[top], mean, total_variance)``
exactly as the reference's (:23-44), and ``main`` writes the same ``eigenvectors_{model}
.npz`` (eigenvectors, eigenvalues, mean, total_variance; :46-65).

Device path (csrc/cov.hip):
  mean        vr_col_mean_f32: numpy's float32 X.mean(axis=0), bit for bit (rows added in
              row order per column, then / float32(n));
  covariance  vr_pca_cov_f64: sum of ((double)x - mean)^T ((double)x - mean) on the fp64
              MFMA, upper-triangle 64 x 64 tiles mirrored, / (n - 1). The reference adds
              its 10000-row batches with BLAS dgemm; here the rows are summed in fixed
              row slices, so entries agree to fp64 rounding (~1e-15 relative), and
              ``batch_size`` only names the reference's batching;
  eigh        torch.linalg.eigh (rocSOLVER, fp64) of the p x p covariance.
Eigenvector signs are solver-defined (numpy's LAPACK eigh in the reference, rocSOLVER here;
neither makes a sign promise) and are returned raw by default, as the reference does. The
coarse PCA labels depend on the sign of each projection, so labels derived from these
vectors and from reference-produced eigenvectors_*.npz may differ by a per-component flip;
``normalize_signs=True`` flips each vector so its largest-|.| component is positive
(``sign_convention``), a reproducible convention for both sides. Tests compare vectors up to
sign.

Multi-GPU (``batched_pca_sharded``): rows sharded over ranks in order. The float32 column
sum is a chain over ranks (rank r continues rank r-1's running sum: the same sequence of
float32 additions as one device, so the mean is still numpy's); every rank then sums its
rows' centred outer products with denominator 1, an RCCL all-reduce adds the p x p fp64
partials (the one data exchange), and every rank divides by n - 1 and decomposes.
"""
from __future__ import annotations

import argparse
import os
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ._lib import check, lib, stream_of, workspace

__all__ = ["pca_mean_cov", "batched_pca", "batched_pca_sharded", "eig_top", "main"]


def _device_rows(X, device: Optional[torch.device]) -> torch.Tensor:
    if isinstance(X, torch.Tensor):
        dev = device or (X.device if X.is_cuda else torch.device("cuda", torch.cuda.current_device()))
        x = X.to(dev, torch.float32)
    else:
        if not torch.cuda.is_available():
            raise RuntimeError("visreps_amd PCA needs a HIP (MI355X) device")
        dev = device or torch.device("cuda", torch.cuda.current_device())
        x = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(dev)
    if not x.is_cuda:
        raise RuntimeError("visreps_amd PCA needs a HIP (MI355X) device")
    if x.dim() != 2:
        raise ValueError(f"expected a 2-D (n, p) feature matrix, got shape {tuple(x.shape)}")
    if x.stride(1) != 1:
        x = x.contiguous()
    return x


def col_sum(x: torch.Tensor, init: Optional[torch.Tensor] = None) -> torch.Tensor:
    """float32 column sums in row order, continued from init (vr_col_sum_f32)."""
    n, p = x.shape
    out = torch.empty(p, dtype=torch.float32, device=x.device)
    check(lib().vr_col_sum_f32(x.data_ptr(), n, p, x.stride(0),
                               init.data_ptr() if init is not None else None, out.data_ptr(),
                               stream_of(x.device)), "vr_col_sum_f32")
    return out


def mean_from_sum(s: torch.Tensor, n: int) -> torch.Tensor:
    out = torch.empty_like(s)
    check(lib().vr_mean_from_sum_f32(s.data_ptr(), s.numel(), int(n), out.data_ptr(),
                                     stream_of(s.device)), "vr_mean_from_sum_f32")
    return out


def cov_sum(x: torch.Tensor, mean: torch.Tensor, denom: float) -> torch.Tensor:
    """sum over rows of the centred outer products / denom, fp64 (p, p) (vr_pca_cov_f64)."""
    n, p = x.shape
    out = torch.empty((p, p), dtype=torch.float64, device=x.device)
    L = lib()
    ws = workspace.get(x.device, L.vr_pca_cov_workspace(n, p), "pca_cov")
    check(L.vr_pca_cov_f64(x.data_ptr(), n, p, x.stride(0), mean.data_ptr(), float(denom),
                           out.data_ptr(), p, ws.data_ptr(), ws.numel(), stream_of(x.device)),
          "vr_pca_cov_f64")
    return out


def pca_mean_cov(X, device: Optional[torch.device] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(mean float32 (p,), covariance float64 (p, p)) on the device, the reference's
    compute_eigenvectors.py:25-36."""
    x = _device_rows(X, device)
    n, p = x.shape
    mean = torch.empty(p, dtype=torch.float32, device=x.device)
    check(lib().vr_col_mean_f32(x.data_ptr(), n, p, x.stride(0), mean.data_ptr(),
                                stream_of(x.device)), "vr_col_mean_f32")
    return mean, cov_sum(x, mean, n - 1)


def sign_convention(vecs: torch.Tensor) -> torch.Tensor:
    """Flip each column so its largest-magnitude component is positive."""
    i = vecs.abs().argmax(dim=0)
    s = torch.sign(vecs[i, torch.arange(vecs.size(1), device=vecs.device)])
    s[s == 0] = 1
    return vecs * s


def eig_top(cov: torch.Tensor, n_components: int, normalize_signs: bool = False):
    """compute_eigenvectors.py:39-44: eigh, the n_components largest eigenvalues in
    descending order, their vectors (solver signs unless normalize_signs), and the sum of
    all eigenvalues."""
    vals, vecs = torch.linalg.eigh(cov)
    vals_h = vals.cpu().numpy()
    idx = np.argsort(vals_h)[::-1][:n_components]
    top = torch.as_tensor(idx.copy(), device=cov.device)
    comps = vecs[:, top]
    if normalize_signs:
        comps = sign_convention(comps)
    return comps.cpu().numpy(), vals_h[idx], float(vals_h.sum())


def batched_pca(X, n_components: int, batch_size: int = 10000, device: Optional[torch.device] = None,
                normalize_signs: bool = False):
    """Drop-in for compute_eigenvectors.batched_pca (:23-44): (components (p, k) float64,
    eigenvalues (k,) float64, mean (p,) float32, total variance). Component signs are the
    solver's (see the module doc; normalize_signs=True for the largest-|.|-positive
    convention)."""
    if batch_size <= 0:
        raise ValueError("batch_size must be positive")
    mean, cov = pca_mean_cov(X, device)
    comps, vals, total = eig_top(cov, n_components, normalize_signs)
    return comps, vals, mean.cpu().numpy(), np.float64(total)


def batched_pca_sharded(x_local: torch.Tensor, n_components: int, pg=None, normalize_signs: bool = False):
    """batched_pca over row shards (rank r holds rows [sum of earlier shards, +n_r), in
    order). Every rank returns the same (components, eigenvalues, mean, total variance)."""
    x = _device_rows(x_local, None)
    rank, world = dist.get_rank(pg), dist.get_world_size(pg)
    n_r, p = x.shape
    sizes = torch.zeros(world, dtype=torch.int64, device=x.device)
    sizes[rank] = n_r
    dist.all_reduce(sizes, group=pg)
    n = int(sizes.sum())
    glob = (lambda r: dist.get_global_rank(pg, r)) if pg is not None else (lambda r: r)
    # float32 running column sum, chained rank 0 -> 1 -> ... (numpy's addition order)
    run = None
    if rank > 0:
        run = torch.empty(p, dtype=torch.float32, device=x.device)
        dist.recv(run, src=glob(rank - 1), group=pg)
    s = col_sum(x, run)
    if rank + 1 < world:
        dist.send(s, dst=glob(rank + 1), group=pg)
    dist.broadcast(s, src=glob(world - 1), group=pg)
    mean = mean_from_sum(s, n)
    part = cov_sum(x, mean, 1.0)
    dist.all_reduce(part, group=pg)
    # true division (torch divides by a Python scalar as a multiply by its reciprocal)
    cov = part / torch.full_like(part, float(n - 1))
    comps, vals, total = eig_top(cov, n_components, normalize_signs)
    return comps, vals, mean.cpu().numpy(), np.float64(total)


def main(argv=None):
    """compute_eigenvectors.py:46-65 with the paths as arguments."""
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--model_name", default="vit")
    ap.add_argument("--features", default=None)
    ap.add_argument("--output", default=None)
    ap.add_argument("--n_components", type=int, default=20)
    ap.add_argument("--batch_size", type=int, default=10000)
    ap.add_argument("--normalize_signs", action="store_true",
                    help="largest-|.| component positive (reproducible across solvers); default: raw solver signs")
    a = ap.parse_args(argv)
    feats = a.features or f"datasets/obj_cls/imagenet/features_{a.model_name}.npz"
    out = a.output or f"datasets/obj_cls/imagenet/eigenvectors_{a.model_name}.npz"
    print(f"Loading features from {feats}...")
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    data = np.load(feats)  # allow_pickle stays False: features are a plain float32 array
    features = data[f"{a.model_name}_features"]
    print(f"Features shape: {features.shape}")
    comps, vals, mean, total = batched_pca(features, a.n_components, a.batch_size, normalize_signs=a.normalize_signs)
    # the sign convention travels with the vectors: the coarse labels flip with a component's
    # sign, so a label set is reproducible only together with this field (extra key; the
    # reference's four keys are unchanged)
    sign = "largest_abs_positive" if a.normalize_signs else f"raw:rocsolver-syevd torch {torch.__version__}"
    np.savez(out, eigenvectors=comps, eigenvalues=vals, mean=mean, total_variance=total,
             sign_convention=np.array(sign))
    print(f"Eigenvectors saved to {out}")
    print(f"Variance explained by top 6: {(vals[:6].sum() / total) * 100:.2f}%")


if __name__ == "__main__":
    main()
