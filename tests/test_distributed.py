"""Multi-GPU orchestration on CPU with gloo, world_size 2 and 3.

The data path is the one bench.py runs over RCCL: each rank splits its stimulus rows
(row statistics + centred bf16 hi/lo plane records) -> all-gather of the planes and
statistics -> balanced upper-triangle tile ranges per rank -> packed tile ranges
all-gathered and unpacked with their mirrors; units in contiguous ranges over ranks, one
engine call per rank-local region group, all_gather_object merge.

On CPU only the device kernels are replaced: the five RdmKernels entry points
(vr_rdm_split_rows_f32, vr_rdm_pearson_tiles_planes, vr_rdm_tiles_pack / unpack and the
plane geometry queries) by a numpy emulation with the same record layout, and the engine
(RankPlan / bootstrap_spearman_multi) by the oracle's midrank Spearman. Everything else
- gathers, compaction, tile ranges, pack/unpack placement, unit grouping, the engine's
Python wrappers and the merge - is the product code. The distributed RDMs must equal the
emulation's single-process RDM bit for bit, and every unit the single-process oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import rsa_oracle as O
from visreps_amd import pipeline as P
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices
from visreps_amd.dataloaders.synthetic import shard_rows


class CpuKernels(P.RdmKernels):
    """numpy emulation of the distributed RDM kernels, record layout included: per row,
    per 32-feature stage, 32 bf16 hi values then 32 bf16 lo values of the centred row."""

    @staticmethod
    def split_rows(x, correction):  # noqa: ARG004
        rows, d = x.shape
        ns = (d + 31) // 32
        xd = x.double()
        mean = xd.mean(1)
        c = (xd - mean[:, None]).float()
        std = torch.sqrt((c.double() ** 2).mean(1)).float()
        pad = torch.zeros((rows, ns * 32), dtype=torch.float32)
        pad[:, :d] = c
        hi = pad.to(torch.bfloat16)
        lo = (pad - hi.float()).to(torch.bfloat16)
        planes = torch.zeros((rows, ns, 64), dtype=torch.int16)
        planes[:, :, :32] = hi.view(torch.int16).view(rows, ns, 32)
        planes[:, :, 32:] = lo.view(torch.int16).view(rows, ns, 32)
        return planes.view(rows, ns * 64), mean.float(), std

    @staticmethod
    def tiles_from_planes(planes, mean, std, n, d, out, t0, t1, correction, times=None):  # noqa: ARG004
        ns = (d + 31) // 32
        pl = planes[:n].view(n, ns, 64)
        hi = pl[:, :, :32].contiguous().view(torch.bfloat16).float()
        lo = pl[:, :, 32:].contiguous().view(torch.bfloat16).float()
        xc = (hi + lo).reshape(n, ns * 32)[:, :d].double()
        s = std.double()
        for t in range(t0, t1):
            r0, c0, h, w = P.tile_rect(n, t)
            g = xc[r0:r0 + h] @ xc[c0:c0 + w].T / d
            corr = (g / (s[r0:r0 + h, None] * s[None, c0:c0 + w] + correction)).clamp(-1, 1)
            blk = (1 - corr).float()
            if r0 == c0:
                blk.fill_diagonal_(0)
            out[r0:r0 + h, c0:c0 + w] = blk
            out[c0:c0 + w, r0:r0 + h] = blk.T

    @staticmethod
    def pack(out, n, t0, t1, packed):
        for t in range(t0, t1):
            r0, c0, h, w = P.tile_rect(n, t)
            v = packed[t - t0].view(P.TILE, P.TILE)
            v[:h, :w] = out[r0:r0 + h, c0:c0 + w]

    @staticmethod
    def unpack(packed, n, t0, t1, out):
        for t in range(t0, t1):
            r0, c0, h, w = P.tile_rect(n, t)
            blk = packed[t - t0].view(P.TILE, P.TILE)[:h, :w]
            out[r0:r0 + h, c0:c0 + w] = blk
            out[c0:c0 + w, r0:r0 + h] = blk.T


def emulated_rdm(X: np.ndarray) -> np.ndarray:
    """The emulation's single-process RDM of all rows (one rank, every tile)."""
    K = CpuKernels()
    x = torch.from_numpy(X)
    n, d = x.shape
    planes, mean, std = K.split_rows(x, 1e-12)
    full = torch.zeros((K.plane_rows(n), planes.size(1)), dtype=torch.int16)
    full[:n] = planes
    out = torch.empty((n, n), dtype=torch.float32)
    K.tiles_from_planes(full, mean, std, n, d, out, 0, int(P.lib().vr_rdm_tile_count(n)), 1e-12)
    return out.numpy()


class _OraclePlan:
    """RankPlan stand-in: the RDM itself (n = its size)."""

    def __init__(self, rdm):
        self.rdm = np.asarray(torch.as_tensor(rdm).cpu())
        self.n = self.rdm.shape[0]


def _oracle_multi(neural, models, idx, full_first=True):  # noqa: ARG001
    n = neural.n
    sets = [np.arange(n)] + ([] if idx is None else list(np.asarray(idx)))
    out = np.empty((len(models), len(sets)))
    for j, pm in enumerate(models):
        for i, s in enumerate(sets):
            iu = np.triu_indices(len(s), 1)
            out[j, i] = O.midrank_spearman(pm.rdm[np.ix_(s, s)][iu], neural.rdm[np.ix_(s, s)][iu])
    return torch.from_numpy(out)


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


def _data(n, d):
    rng = np.random.default_rng(3)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Y = (X[:, :8] @ rng.standard_normal((8, 40)) + rng.standard_normal((n, 40))).astype(np.float32)
    Z = np.maximum(X[:, ::-1] + 0.3 * rng.standard_normal((n, d)), 0).astype(np.float32)
    return X, Y, Z


def _worker(rank, world, port, n, d, n_boot, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pg = dist.group.WORLD
    R.RankPlan = _OraclePlan  # the engine's kernels (see module doc)
    R.bootstrap_spearman_multi = _oracle_multi
    K = CpuKernels()
    X, Y, Z = _data(n, d)
    rows = shard_rows(n, rank, world)
    loc = {k: torch.from_numpy(v[rows.start:rows.stop]) for k, v in {"x": X, "y": Y, "z": Z}.items()}
    # as bench.py: every point's plane exchange in flight on its own group while the other
    # collectives (neural RDMs, tile ranges, scores) run on pg
    feat_pg = dist.new_group(list(range(world)))
    src = P.PrefetchedRDMs({"x": loc["x"], "z": loc["z"]}, ["x", "z"], n, pg, kernels=K, exchange_pg=feat_pg)
    src.start_all()
    rdm_y = P.distributed_rdm(loc["y"], n, pg, kernels=K)
    res = P.all_units_rsa(src, ["x", "z"], {"r0": rdm_y, "r1": P.distributed_rdm(loc["x"], n, pg, kernels=K)},
                          n, n_boot=n_boot, seed=42, pg=pg)
    assert not src.pending
    again = P.PrefetchedRDMs({"x": loc["x"]}, ["x"], n, pg, kernels=K)("x")
    np.save(os.path.join(out_dir, f"rdm_y_{rank}.npy"), rdm_y.numpy())
    np.save(os.path.join(out_dir, f"rdm_x_{rank}.npy"), again.numpy())
    with open(os.path.join(out_dir, f"res_{rank}.txt"), "w") as f:
        for k in sorted(res):
            f.write(f"{k[0]} {k[1]} {res[k]['score']:.17g} {res[k]['ci_low']:.17g} {res[k]['ci_high']:.17g}\n")
    dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(37, 2), (300, 2), (300, 3)])
def test_gloo_distributed_rdm_and_units_match_single_process(tmp_path, n, world):
    d, n_boot = 40, 6
    mp.spawn(_worker, args=(world, _free_port(), n, d, n_boot, str(tmp_path)), nprocs=world, join=True)
    X, Y, Z = _data(n, d)
    ref = {"x": emulated_rdm(X), "y": emulated_rdm(Y), "z": emulated_rdm(Z)}
    assert np.max(np.abs(ref["x"] - O.compute_rdm(X))) < 1e-5  # the emulation is an RDM
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"rdm_y_{r}.npy"), ref["y"])
        assert np.array_equal(np.load(tmp_path / f"rdm_x_{r}.npy"), ref["x"])
    lines = [(tmp_path / f"res_{r}.txt").read_text() for r in range(world)]
    assert all(l == lines[0] for l in lines)
    idx = bootstrap_indices(42, n, int(0.9 * n), n_boot)
    neural = {"r0": ref["y"], "r1": ref["x"]}
    got_units = set()
    for line in lines[0].splitlines():
        p, r, *vals = line.split()
        got_units.add((p, r))
        a, b = ref[p], neural[r]
        sets = [np.arange(n)] + list(idx)
        sc = [O.midrank_spearman(a[np.ix_(s, s)][np.triu_indices(len(s), 1)],
                                 b[np.ix_(s, s)][np.triu_indices(len(s), 1)]) for s in sets]
        assert abs(float(vals[0]) - sc[0]) < 1e-12
        assert abs(float(vals[1]) - np.percentile(sc[1:], 2.5)) < 1e-12
        assert abs(float(vals[2]) - np.percentile(sc[1:], 97.5)) < 1e-12
    assert got_units == {(p, r) for p in ["x", "z"] for r in ["r0", "r1"]}


def test_compact_and_padded_layout():
    # rows of uneven shards land in rank order, zero tail rows after the last real one
    sizes = [3, 2, 2]
    full = torch.arange(9 * 2, dtype=torch.float32).view(9, 2)
    out = P._compact(full, sizes, 9)
    assert torch.equal(out[:3], full[0:3]) and torch.equal(out[3:5], full[3:5])
    assert torch.equal(out[5:7], full[6:8]) and torch.all(out[7:] == 0)
