"""Multi-GPU orchestration on CPU with gloo, world_size 2.

The data path is the one bench.py runs over RCCL: stimulus-row shards -> all-gather ->
balanced upper-triangle tile ranges per rank -> zero-filled RDM + sum all-reduce (exactly
one writer per entry), and units round-robin over ranks with an all_gather_object merge.
Here the Gram tile writer and the Spearman unit are the CPU oracle (injected), so the
tests check the orchestration: coverage, exactness and rank-invariance."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import rsa_oracle as O
from visreps_amd import pipeline as P
from visreps_amd.analysis._random import bootstrap_indices
from visreps_amd.dataloaders.synthetic import shard_rows


def _oracle_tiles_into(x, out, t0, t1, times=None):  # noqa: ARG001
    n = x.size(0)
    full = O.compute_rdm(x.numpy())
    for t in range(t0, t1):
        r0, c0, h, w = P.tile_rect(n, t)
        blk = torch.from_numpy(full[r0:r0 + h, c0:c0 + w])
        out[r0:r0 + h, c0:c0 + w] = blk
        if c0 != r0:
            out[c0:c0 + w, r0:r0 + h] = blk.T


@pytest.mark.parametrize("n", [1, 5, 127, 128, 129, 300])
def test_tile_rects_cover_upper_triangle_once(n):
    cover = np.zeros((n, n), np.int32)
    for t in range(int(P.lib().vr_rdm_tile_count(n))):
        r0, c0, h, w = P.tile_rect(n, t)
        assert c0 >= r0 and h > 0 and w > 0
        cover[r0:r0 + h, c0:c0 + w] += 1
    iu = np.triu_indices(n)
    assert np.all(cover[iu] == 1)


@pytest.mark.parametrize("n", [300, 1000, 10000])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_tile_ranges_partition_and_balance(n, world):
    T = int(P.lib().vr_rdm_tile_count(n))
    rng = P.tile_ranges(n, world)
    assert rng[0][0] == 0 and rng[-1][1] == T
    assert all(rng[r][1] == rng[r + 1][0] for r in range(world - 1))
    costs = [sum(P.lib().vr_rdm_tile_cost(n, t) for t in range(a, b)) for a, b in rng]
    biggest = max(P.lib().vr_rdm_tile_cost(n, t) for t in range(T))
    assert max(costs) - min(costs) <= 2 * biggest
    assert sum(costs) == n * (n + 1) // 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, d, n_boot, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pg = dist.group.WORLD
    rng = np.random.default_rng(3)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Y = (X[:, :8] @ rng.standard_normal((8, 40)) + rng.standard_normal((n, 40))).astype(np.float32)
    rows = shard_rows(n, rank, world)
    x_local = torch.from_numpy(X[rows.start:rows.stop])
    y_local = torch.from_numpy(Y[rows.start:rows.stop])
    rdm_x = P.distributed_rdm(x_local, n, pg, tiles_into=_oracle_tiles_into)
    rdm_y = P.distributed_rdm(y_local, n, pg, tiles_into=_oracle_tiles_into)
    # the prefetching source bench.py uses: next point's all-gather in flight (async)
    src = P.PrefetchedRDMs({"x": x_local, "y": y_local}, ["x", "y"], n, pg,
                           tiles_into=_oracle_tiles_into)
    assert torch.equal(src("x"), rdm_x) and torch.equal(src("y"), rdm_y) and not src.pending

    def unit(pm, pn, idx, times):  # noqa: ARG001
        sets = [np.arange(n)] + ([] if idx is None else list(np.asarray(idx)))
        return np.array([O.midrank_spearman(pm[np.ix_(s, s)][np.triu_indices(len(s), 1)],
                                            pn[np.ix_(s, s)][np.triu_indices(len(s), 1)])
                         for s in sets])

    feats = {"a": rdm_x, "b": torch.from_numpy(O.compute_rdm(X[:, ::-1].copy()))}
    res = P.all_units_rsa(lambda p: feats[p], ["a", "b"], {"r0": rdm_y, "r1": rdm_x}, n,
                          n_boot=n_boot, seed=42, pg=pg, plan_fn=lambda r: np.asarray(r),
                          unit_fn=unit)
    np.save(os.path.join(out_dir, f"rdm_x_{rank}.npy"), rdm_x.numpy())
    np.save(os.path.join(out_dir, f"rdm_y_{rank}.npy"), rdm_y.numpy())
    with open(os.path.join(out_dir, f"res_{rank}.txt"), "w") as f:
        for k in sorted(res):
            f.write(f"{k} {res[k]['score']:.17g} {res[k]['ci_low']:.17g} {res[k]['ci_high']:.17g}\n")
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [37, 130])
def test_gloo_world2_matches_single_process(tmp_path, n):
    d, n_boot, world = 24, 6, 2
    mp.spawn(_worker, args=(world, _free_port(), n, d, n_boot, str(tmp_path)), nprocs=world, join=True)
    rng = np.random.default_rng(3)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Y = (X[:, :8] @ rng.standard_normal((8, 40)) + rng.standard_normal((n, 40))).astype(np.float32)
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"rdm_x_{r}.npy"), O.compute_rdm(X))
        assert np.array_equal(np.load(tmp_path / f"rdm_y_{r}.npy"), O.compute_rdm(Y))
    lines = [(tmp_path / f"res_{r}.txt").read_text() for r in range(world)]
    assert lines[0] == lines[1]
    # every unit as the single-process oracle computes it
    idx = bootstrap_indices(42, n, int(0.9 * n), n_boot)
    ry = O.compute_rdm(Y)
    for line in lines[0].splitlines():
        p, r = line.split()[0].strip("(),'"), line.split()[1].strip("(),'")
        a = O.compute_rdm(X) if p == "a" else O.compute_rdm(X[:, ::-1].copy())
        b = ry if r == "r0" else O.compute_rdm(X)
        sets = [np.arange(n)] + list(idx)
        vals = [O.midrank_spearman(a[np.ix_(s, s)][np.triu_indices(len(s), 1)],
                                   b[np.ix_(s, s)][np.triu_indices(len(s), 1)]) for s in sets]
        got = [float(v) for v in line.split()[2:]]
        assert abs(got[0] - vals[0]) < 1e-12
        assert abs(got[1] - np.percentile(vals[1:], 2.5)) < 1e-12
        assert abs(got[2] - np.percentile(vals[1:], 97.5)) < 1e-12
