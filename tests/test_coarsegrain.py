"""PCA covariance for the coarse-grained labels (visreps_amd/coarsegrain.py, SURVEY.md
§8(f4); reference scripts/coarsegrain/compute_eigenvectors.py:23-44).

CPU: the oracle's float32 mean order is numpy's (sequential rows per column); the oracle
covariance equals numpy's own np.cov definition; the sharded orchestration (float32 sum
chain over ranks, fp64 partial all-reduce) on gloo world 2 and 3 with the two device
kernels emulated equals the oracle (mean bit for bit).
GPU: vr_col_mean_f32 is bit-identical to X.mean(axis=0); the fp64 MFMA covariance equals
the oracle's batched covariance to fp64 rounding (relative 1e-12 of the largest entry);
eigenvalues to 1e-10 relative, eigenvectors up to sign to 1e-8; exact symmetry."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import pca_oracle as P


def _feats(n, p, seed=0, scale=1.0):
    rs = np.random.default_rng(seed)
    z = rs.standard_normal((n, 8))
    w = rs.standard_normal((8, p)) * np.linspace(3.0, 0.1, 8)[:, None]
    x = np.maximum(z @ w + 0.5 * rs.standard_normal((n, p)), 0) * scale + 0.25
    return x.astype(np.float32)


# ------------------------------------------------------------------------------ CPU
@pytest.mark.parametrize("shape", [(1, 5), (300, 7), (2000, 4096), (4097, 65)])
def test_oracle_mean_order_is_numpys(shape):
    x = _feats(*shape, seed=1, scale=37.0)
    assert np.array_equal(P.col_sum_sequential(x), x.sum(axis=0))
    assert np.array_equal(P.col_sum_sequential(x) / np.float32(x.shape[0]), x.mean(axis=0))


def test_oracle_cov_is_numpys_definition():
    x = _feats(3000, 96, seed=2)
    comps, vals, mean, total, cov = P.batched_pca(x, 5, batch_size=700)
    ref = np.cov(x.astype(np.float64) - mean.astype(np.float64), rowvar=False)  # same mean
    d = x.astype(np.float64) - mean
    assert np.allclose(cov, (d.T @ d) / (len(x) - 1), rtol=0, atol=1e-12 * np.abs(cov).max())
    assert np.allclose(cov, ref, rtol=0, atol=1e-6 * np.abs(cov).max())  # np.cov re-centres in fp64
    assert np.all(np.diff(vals) <= 0) and abs(total - np.trace(cov)) <= 1e-9 * total
    assert comps.shape == (96, 5)


class _NumpyKernels:
    """vr_col_sum_f32 / vr_mean_from_sum_f32 / vr_pca_cov_f64 restated in numpy."""

    @staticmethod
    def rows(x, device):
        return x

    @staticmethod
    def col_sum(x, init=None):
        s = init.numpy().copy() if init is not None else np.zeros(x.shape[1], np.float32)
        for r in x.numpy():
            s = s + r
        return torch.from_numpy(s)

    @staticmethod
    def mean_from_sum(s, n):
        return torch.from_numpy(s.numpy() / np.float32(n))

    @staticmethod
    def cov_sum(x, mean, denom):
        d = x.numpy().astype(np.float64) - mean.numpy().astype(np.float64)
        return torch.from_numpy((d.T @ d) / denom)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, x, bounds, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from visreps_amd import coarsegrain as C

    C._device_rows = _NumpyKernels.rows
    C.col_sum = _NumpyKernels.col_sum
    C.mean_from_sum = _NumpyKernels.mean_from_sum
    C.cov_sum = _NumpyKernels.cov_sum
    xl = torch.from_numpy(x[bounds[rank]:bounds[rank + 1]].copy())
    comps, vals, mean, total = C.batched_pca_sharded(xl, 4)
    out[rank] = (comps, vals, mean, total)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bounds", [(2, [0, 700, 1500]), (3, [0, 1, 900, 1500])])
def test_sharded_pca_gloo_matches_oracle(world, bounds):
    x = _feats(1500, 40, seed=3, scale=11.0)
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), x, bounds, out), nprocs=world,
                       start_method="spawn")
    comps, vals, mean, total, cov = P.batched_pca(x, 4)
    for r in range(world):
        c, v, m, t = out[r]
        assert np.array_equal(m, mean)  # the chained float32 sum is numpy's
        assert np.allclose(v, vals, rtol=1e-12, atol=0)
        assert abs(t - total) <= 1e-12 * total
        assert np.all(np.abs(np.abs(np.sum(c * comps, axis=0)) - 1) < 1e-9)


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1, 3), (239, 64), (241, 65), (5000, 1000), (20000, 4096)])
def test_col_mean_bit_identical_to_numpy(dev, shape):
    from visreps_amd import coarsegrain as C

    x = _feats(*shape, seed=4, scale=53.0)
    mean, _ = C.pca_mean_cov(torch.from_numpy(x).to(dev))
    assert np.array_equal(mean.cpu().numpy(), x.mean(axis=0))


@pytest.mark.gpu
def test_col_sum_strided_and_chained(dev):
    from visreps_amd import coarsegrain as C

    x = _feats(1000, 200, seed=5, scale=9.0)
    big = torch.zeros((1000, 256), device=dev)
    big[:, :200] = torch.from_numpy(x).to(dev)
    v = big[:, :200]  # leading dimension 256
    assert np.array_equal(C.col_sum(v).cpu().numpy(), x.sum(axis=0))
    s1 = C.col_sum(v[:333])
    s2 = C.col_sum(v[333:], s1)
    assert np.array_equal(s2.cpu().numpy(), x.sum(axis=0))


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(2, 3), (500, 64), (3001, 130), (40000, 1024), (12000, 4096)])
def test_cov_matches_oracle(dev, n, p):
    from visreps_amd import coarsegrain as C

    x = _feats(n, p, seed=6)
    mean, cov = C.pca_mean_cov(torch.from_numpy(x).to(dev))
    got = cov.cpu().numpy()
    _, _, mref, _, ref = P.batched_pca(x, 1)
    assert np.array_equal(mean.cpu().numpy(), mref)
    assert np.array_equal(got, got.T)
    scale = np.abs(ref).max()
    assert np.max(np.abs(got - ref)) <= 1e-12 * scale, np.max(np.abs(got - ref)) / scale


@pytest.mark.gpu
def test_batched_pca_matches_oracle(dev):
    from visreps_amd import coarsegrain as C

    x = _feats(30000, 512, seed=7)
    comps, vals, mean, total = C.batched_pca(x, 20)
    rc, rv, rm, rt, _ = P.batched_pca(x, 20)
    assert comps.shape == rc.shape == (512, 20) and comps.dtype == np.float64
    assert np.array_equal(mean, rm) and mean.dtype == np.float32
    assert np.allclose(vals, rv, rtol=1e-10, atol=0)
    assert abs(total - rt) <= 1e-10 * rt
    # the top 8 eigenvalues are well separated (8 latent factors): vectors agree up to sign
    assert np.all(np.abs(np.abs(np.sum(comps[:, :8] * rc[:, :8], axis=0)) - 1) < 1e-8)
    # opt-in sign convention (the default keeps the solver's signs, as the reference does)
    cn, vn, _, _ = C.batched_pca(x, 20, normalize_signs=True)
    assert np.all(np.abs(cn).max(axis=0) == cn.max(axis=0))
    assert np.array_equal(np.abs(cn), np.abs(comps)) and np.array_equal(vn, vals)


@pytest.mark.gpu
def test_sharded_pca_world1_on_device(dev):
    from visreps_amd import coarsegrain as C

    x = _feats(5000, 256, seed=8)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        comps, vals, mean, total = C.batched_pca_sharded(torch.from_numpy(x).to(dev), 6)
    finally:
        dist.destroy_process_group()
    c1, v1, m1, t1 = C.batched_pca(x, 6)
    assert np.array_equal(mean, m1) and np.array_equal(vals, v1) and np.array_equal(comps, c1)
