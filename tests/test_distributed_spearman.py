"""Distributed full-triangle Spearman (analysis/distributed_spearman.py),
in its count-table form and its sample-sort form. CPU: gloo world 2 and 3, pairs spread over
ranks at random, the device pieces (sort keys, radix sort, midranks, per-key counts, table
midranks, exact dot) emulated in numpy; the collectives, key range, table all-reduce,
splitters, bucket exchange, global offsets and owner routing are the product code; the score
must equal the oracle's midrank Spearman. GPU: world 1 through the HIP pieces equals
spearman_full bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import rsa_oracle as O
from visreps_amd.analysis import distributed_spearman as DS


class NumpyRankKernels(DS.RankKernels):
    @staticmethod
    def keys(values):
        u = values.numpy().view(np.uint32).astype(np.uint64)
        u[u == 0x80000000] = 0
        k = np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint32)
        return torch.from_numpy(k.view(np.int32).copy())

    @staticmethod
    def sort(keys, vals):
        k = keys.numpy().view(np.uint32)
        o = np.argsort(k, kind="stable")
        return torch.from_numpy(keys.numpy()[o].copy()), torch.from_numpy(vals.numpy()[o].copy())

    @staticmethod
    def midranks(keys_sorted, base):
        k = keys_sorted.numpy().view(np.uint32)
        m = len(k)
        if m == 0:
            return torch.zeros(0, dtype=torch.int64), 0
        starts = np.flatnonzero(np.r_[True, k[1:] != k[:-1]])
        ends = np.r_[starts[1:], m]
        gs = np.repeat(starts, ends - starts)
        ge = np.repeat(ends, ends - starts)
        y = 2 * int(base) + gs + ge + 1
        tie = sum(int(e - s) ** 3 - int(e - s) for s, e in zip(starts, ends))
        return torch.from_numpy(y.astype(np.int64)), tie

    @staticmethod
    def counts(keys, kmin, bins):
        k = keys.numpy().view(np.uint32).astype(np.int64) - int(kmin)
        return torch.from_numpy(np.bincount(k, minlength=bins + 1).astype(np.int64))

    @staticmethod
    def table_midranks(keys, kmin, counts):
        c = counts.numpy().astype(np.int64)
        start = np.concatenate([[0], np.cumsum(c)])[:-1]  # exclusive, bins + 1 entries
        k = keys.numpy().view(np.uint32).astype(np.int64) - int(kmin)
        y = start[k] + start[k + 1] + 1
        tie = sum(int(v) ** 3 - int(v) for v in c[c > 1])
        return torch.from_numpy(y.astype(np.int64)), tie

    @staticmethod
    def dot(a, b):
        return int(np.dot(a.numpy().astype(object), b.numpy().astype(object)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tri(n, seed, levels=None, nan=False):
    rs = np.random.RandomState(seed)
    x = rs.randn(n, 12).astype(np.float32)
    r = O.compute_rdm(x)
    if levels:
        r = (np.floor(r * levels) / levels).astype(np.float32)
    if nan:
        r[1, 4] = r[4, 1] = np.nan
    return r[np.triu_indices(n, 1)]


def _worker(rank, world, port, n, seed, levels, nan, out_dir, method="tables", cap=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if cap:  # a key range beyond the table cap: the count-table form falls back to the sample sort
        DS.TABLE_CAP = cap
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = _tri(n, seed, levels), _tri(n, seed + 1, None, nan)
    M = len(a)
    own = np.random.RandomState(seed + 7).randint(0, world, size=M)  # pairs spread at random
    mine = np.flatnonzero(own == rank)
    # B's pairs spread differently from A's
    ownb = np.random.RandomState(seed + 8).randint(0, world, size=M)
    mineb = np.flatnonzero(ownb == rank)
    r = DS.distributed_spearman(torch.from_numpy(a[mine]), torch.from_numpy(mine), torch.from_numpy(b[mineb]),
                                torch.from_numpy(mineb), M, dist.group.WORLD, NumpyRankKernels(), method=method)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(repr(r))
    dist.destroy_process_group()


@pytest.mark.parametrize("method", ["tables", "sort"])
@pytest.mark.parametrize("n,world,levels,nan", [(60, 2, None, False), (150, 3, 6, False), (90, 2, 4, True),
                                                (33, 3, None, False)])
def test_gloo_distributed_spearman_matches_oracle(tmp_path, n, world, levels, nan, method):
    seed = n + world
    mp.spawn(_worker, args=(world, _free_port(), n, seed, levels, nan, str(tmp_path), method), nprocs=world,
             join=True)
    got = [float((tmp_path / f"r{r}.txt").read_text()) for r in range(world)]
    a, b = _tri(n, seed, levels), _tri(n, seed + 1, None, nan)
    if nan:
        assert all(np.isnan(g) for g in got)
        return
    ref = O.midrank_spearman(a, b)
    assert all(g == got[0] for g in got)
    assert abs(got[0] - ref) <= 1e-12


def test_gloo_tables_fall_back_to_sample_sort_beyond_the_cap(tmp_path):
    n, world = 70, 2
    seed = 11
    mp.spawn(_worker, args=(world, _free_port(), n, seed, None, False, str(tmp_path), "tables", 16), nprocs=world,
             join=True)
    got = [float((tmp_path / f"r{r}.txt").read_text()) for r in range(world)]
    ref = O.midrank_spearman(_tri(n, seed), _tri(n, seed + 1))
    assert got[0] == got[1] and abs(got[0] - ref) <= 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["tables", "sort"])
@pytest.mark.parametrize("n,levels", [(500, None), (2000, 7)])
def test_world1_hip_pieces_equal_spearman_full(dev, n, levels, method):
    from visreps_amd.analysis import rsa as R

    a, b = _tri(n, 3, levels), _tri(n, 4)
    M = len(a)
    got = DS.distributed_spearman(torch.from_numpy(a).to(dev), torch.arange(M, device=dev),
                                  torch.from_numpy(b).to(dev), torch.arange(M, device=dev), M, method=method)
    full = np.zeros((n, n), np.float32)
    iu = np.triu_indices(n, 1)
    full[iu] = a
    fa = full + full.T
    full[iu] = b
    fb = np.triu(full, 1) + np.triu(full, 1).T
    ref = R.spearman_full(torch.from_numpy(fa).to(dev), torch.from_numpy(fb).to(dev))
    assert got == ref


@pytest.mark.gpu
@pytest.mark.parametrize("nkeys", [3, 3000])
def test_world1_tables_few_keys(dev, nkeys):
    # a small key range: per-block LDS counts (vr_key_counts_u32 at <= 16384 keys)
    from visreps_amd.analysis import rsa as R

    n = 1500
    g = np.random.default_rng(nkeys)
    tri = lambda k: (0x3F800000 + g.integers(0, k, n * (n - 1) // 2)).astype(np.uint32).view(np.float32)
    a, b = tri(nkeys), tri(nkeys + 5)
    M = len(a)
    got = DS.distributed_spearman(torch.from_numpy(a).to(dev), torch.arange(M, device=dev),
                                  torch.from_numpy(b).to(dev), torch.arange(M, device=dev), M)
    assert abs(got - O.midrank_spearman(a, b)) <= 1e-12
    full = np.zeros((n, n), np.float32)
    iu = np.triu_indices(n, 1)
    full[iu] = a
    fa = full + full.T
    full[iu] = b
    fb = np.triu(full, 1) + np.triu(full, 1).T
    assert got == R.spearman_full(torch.from_numpy(fa).to(dev), torch.from_numpy(fb).to(dev))
