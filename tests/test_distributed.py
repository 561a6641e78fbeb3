"""Multi-GPU orchestration on CPU with gloo, world_size 2 and 3.

The data path is the one bench.py runs over RCCL: an RdmSchedule gives every RDM its
owner(s) -- pieces cut at aligned tile boundaries for RDMs heavier than the per-rank mean --
each rank sends its stimulus rows of an RDM to that RDM's owners (all_to_all_single), the
owners compute their pieces from the full rows, and the packed pieces go only to the ranks
whose units read the RDM; units in contiguous ranges over ranks, one engine call per
rank-local region group, all_gather_object merge.

On CPU only the device kernels are replaced: the RdmKernels entry points (tiles from rows,
pack, unpack) by a numpy emulation with the same tile layout, and the engine (RankPlan /
bootstrap_spearman_multi) by the oracle's midrank Spearman. Everything else -- the
schedule, the row and piece exchanges, unpack placement, unit grouping and the merge -- is
the product code. Every RDM a rank holds must equal the emulation's single-process RDM bit
for bit (the tile arithmetic does not depend on the world size), and every unit the
single-process oracle."""
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
    """numpy emulation of the distributed RDM kernels: tiles of the float64 RDM of the
    rows (rsa.py:76-92 arithmetic), rounded to fp32, written with their mirrors."""

    @staticmethod
    def tiles_from_rows(x, out, t0, t1, correction, times=None):  # noqa: ARG004
        n, d = x.shape
        xd = x.double()
        xc = xd - xd.mean(1, keepdim=True)
        s = torch.sqrt((xc * xc).mean(1) + correction)
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
    def plane_elems(d):  # emulated record: per 32-feature stage 32 bf16 hi then 32 bf16 lo
        return (d + 31) // 32 * 64

    @staticmethod
    def split_rows_into(x, correction, planes, mean, std):  # noqa: ARG004
        rows, d = x.shape
        ns = (d + 31) // 32
        xd = x.double()
        m = xd.mean(1)
        c = (xd - m[:, None]).float()
        pad = torch.zeros((rows, ns * 32), dtype=torch.float32)
        pad[:, :d] = c
        hi = pad.to(torch.bfloat16)
        lo = (pad - hi.float()).to(torch.bfloat16)
        pl = planes[:rows].view(rows, ns, 64)
        pl[:, :, :32] = hi.view(torch.int16).view(rows, ns, 32)
        pl[:, :, 32:] = lo.view(torch.int16).view(rows, ns, 32)
        mean.copy_(m.float())
        std.copy_(torch.sqrt((c.double() ** 2).mean(1)).float())

    @staticmethod
    def tiles_from_planes(sr, n, out, t0, t1, correction, times=None):  # noqa: ARG004
        d = sr.d
        ns = (d + 31) // 32
        pl = sr.planes[:n].view(n, ns, 64)
        hi = pl[:, :, :32].contiguous().view(torch.bfloat16).float()
        lo = pl[:, :, 32:].contiguous().view(torch.bfloat16).float()
        xc = (hi + lo).reshape(n, ns * 32)[:, :d].double()
        s = sr.std.double()
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


def emulated_rdm(X: np.ndarray, split: bool = False) -> np.ndarray:
    """The emulation's single-process RDM of all rows (one rank, every tile), from the rows
    or from their split records."""
    K = CpuKernels()
    x = torch.from_numpy(X)
    n = x.size(0)
    out = torch.empty((n, n), dtype=torch.float32)
    if split:
        sr = K.empty_split(n, x.size(1), "cpu")
        K.split_rows_into(x, 1e-12, sr.planes, sr.mean, sr.std)
        K.tiles_from_planes(sr, n, out, 0, int(P.lib().vr_rdm_tile_count(n)), 1e-12)
    else:
        K.tiles_from_rows(x, out, 0, int(P.lib().vr_rdm_tile_count(n)), 1e-12)
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


def _row_boundaries(n, d):  # noqa: ARG001
    """Every 128-tile row start: lets the small test RDMs be cut into pieces (the emulation
    computes any range identically; the HIP kernel's own aligned cuts: test_gpu_distributed)."""
    T = -(-n // P.TILE)
    return [P._tri_start(r, T) for r in range(T)] + [int(P.lib().vr_rdm_tile_count(n))]


def _local_split(K, x):
    sr = K.empty_split(x.size(0), x.size(1), "cpu")
    K.split_rows_into(x, 1e-12, sr.planes, sr.mean, sr.std)
    return sr


def _worker(rank, world, port, n, d, n_boot, out_dir, split, presplit):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pg = dist.group.WORLD
    R.RankPlan = _OraclePlan  # the engine's kernels (see module doc)
    R.bootstrap_spearman_multi = _oracle_multi
    if split:
        P.aligned_boundaries = _row_boundaries
    K = CpuKernels()
    X, Y, Z = _data(n, d)
    rows = shard_rows(n, rank, world)
    loc = {k: torch.from_numpy(v[rows.start:rows.stop]) for k, v in {"x": X, "y": Y, "z": Z}.items()}
    sched = P.make_schedule(n, {"x": d, "z": d}, ["x", "z"], {"r0": Y.shape[1], "r1": d}, world,
                            split_factor=0.3 if split else 1.25)
    if split:
        assert any(len(p) > 1 for p in sched.pieces.values())
    feat_pg = dist.new_group(list(range(world)))
    srcs = {("m", "x"): loc["x"], ("m", "z"): loc["z"], ("n", "r0"): loc["y"], ("n", "r1"): loc["x"]}
    if presplit:  # bench.extract_split: the model points arrive as split rows
        srcs[("m", "x")], srcs[("m", "z")] = _local_split(K, loc["x"]), _local_split(K, loc["z"])
    ex = P.ShardedRDMs(sched, srcs, pg, kernels=K, exchange_pg=feat_pg, window=1)
    ex.start()
    rd = ex.finish()
    assert set(rd) == set(sched.needs(rank)) and not ex.pending
    res = P.all_units_rsa(lambda p: rd[("m", p)], ["x", "z"], {r: rd[("n", r)] for r in ["r0", "r1"] if ("n", r) in rd},
                          n, n_boot=n_boot, seed=42, pg=pg, regions=["r0", "r1"])
    for (kind, name), m in rd.items():
        np.save(os.path.join(out_dir, f"rdm_{kind}{name}_{rank}.npy"), m.numpy())
    np.save(os.path.join(out_dir, f"rdm_all_{rank}.npy"), P.distributed_rdm(loc["z"], n, pg, kernels=K).numpy())
    with open(os.path.join(out_dir, f"res_{rank}.txt"), "w") as f:
        for k in sorted(res):
            f.write(f"{k[0]} {k[1]} {res[k]['score']:.17g} {res[k]['ci_low']:.17g} {res[k]['ci_high']:.17g}\n")
    dist.destroy_process_group()


@pytest.mark.parametrize("n,world,split,presplit", [(37, 2, False, False), (300, 2, False, False),
                                                   (300, 3, False, False), (300, 2, True, False),
                                                   (400, 3, True, False), (300, 3, True, True)])
def test_gloo_distributed_rdm_and_units_match_single_process(tmp_path, n, world, split, presplit):
    d, n_boot = 40, 6
    mp.spawn(_worker, args=(world, _free_port(), n, d, n_boot, str(tmp_path), split, presplit), nprocs=world,
             join=True)
    X, Y, Z = _data(n, d)
    ref = {"mx": emulated_rdm(X, presplit), "mz": emulated_rdm(Z, presplit), "nr0": emulated_rdm(Y),
           "nr1": emulated_rdm(X)}
    assert np.max(np.abs(ref["mx"] - O.compute_rdm(X))) < 1e-5  # the emulation is an RDM
    held = 0
    for r in range(world):
        for key, m in ref.items():
            f = tmp_path / f"rdm_{key}_{r}.npy"
            if f.exists():
                held += 1
                assert np.array_equal(np.load(f), m), (key, r)
        assert np.array_equal(np.load(tmp_path / f"rdm_all_{r}.npy"), emulated_rdm(Z))
    assert held >= 4  # every RDM is held by at least one consumer
    lines = [(tmp_path / f"res_{r}.txt").read_text() for r in range(world)]
    assert all(l == lines[0] for l in lines)
    idx = bootstrap_indices(42, n, int(0.9 * n), n_boot)
    models = {"x": ref["mx"], "z": ref["mz"]}
    if presplit:
        assert not np.array_equal(ref["mx"], ref["nr1"])  # the split path is the one compared
    neural = {"r0": ref["nr0"], "r1": ref["nr1"]}
    got_units = set()
    for line in lines[0].splitlines():
        p, r, *vals = line.split()
        got_units.add((p, r))
        a, b = models[p], neural[r]
        sets = [np.arange(n)] + list(idx)
        sc = [O.midrank_spearman(a[np.ix_(s, s)][np.triu_indices(len(s), 1)],
                                 b[np.ix_(s, s)][np.triu_indices(len(s), 1)]) for s in sets]
        assert abs(float(vals[0]) - sc[0]) < 1e-12
        assert abs(float(vals[1]) - np.percentile(sc[1:], 2.5)) < 1e-12
        assert abs(float(vals[2]) - np.percentile(sc[1:], 97.5)) < 1e-12
    assert got_units == {(p, r) for p in ["x", "z"] for r in ["r0", "r1"]}


BENCH_DIMS = {"conv1_pre": 290400, "conv1_post": 290400, "conv2_pre": 186624, "conv2_post": 186624,
              "conv3_pre": 64896, "conv3_post": 64896, "conv4_pre": 64896, "conv4_post": 64896,
              "conv5_pre": 43264, "conv5_post": 43264, "fc1_pre": 4096, "fc1_post": 4096,
              "fc2_pre": 4096, "fc2_post": 4096}
BENCH_ROIS = {"V1": 2000, "V2": 2000, "V3": 2000, "hV4": 1000}


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_bench_schedule(world):
    """The bench step's schedule (N = 10k, 14 points, 4 ROIs): every RDM is covered by its
    pieces exactly once, pieces of one RDM sit on distinct ranks, every consumer is a rank
    with a unit reading the RDM, units are balanced, and the Gram load per rank stays near
    the mean (the conv1 points are cut at aligned super-tile rows when they exceed it)."""
    n = 10000
    s = P.make_schedule(n, BENCH_DIMS, list(BENCH_DIMS), BENCH_ROIS, world)
    T = int(P.lib().vr_rdm_tile_count(n))
    for name, pcs in s.pieces.items():
        cover = sorted((pc.t0, pc.t1) for pc in pcs)
        assert cover[0][0] == 0 and cover[-1][1] == T
        assert all(cover[i][1] == cover[i + 1][0] for i in range(len(cover) - 1))
        assert len({pc.owner for pc in pcs}) == len(pcs)
    assert len(s.pieces) == 18
    counts = [hi - lo for lo, hi in s.unit_ranges]
    assert sum(counts) == 56 and max(counts) - min(counts) <= 1
    for rk, (lo, hi) in enumerate(s.unit_ranges):
        for p, r in s.units[lo:hi]:
            assert rk in s.consumers[("m", p)] and rk in s.consumers[("n", r)]
    mean = sum(s.load) / world
    assert max(s.load) <= 1.35 * mean + 1e-9, (s.load, mean)
    if world == 1:
        assert all(len(p) == 1 for p in s.pieces.values())
    if world >= 8:
        assert len(s.pieces[("m", "conv1_pre")]) > 1  # the heaviest RDM is split


def test_row_boundaries_for_split_tests_are_a_partition():
    b = _row_boundaries(300, 40)
    assert b[0] == 0 and b[-1] == int(P.lib().vr_rdm_tile_count(300)) and b == sorted(set(b))


def _phase1_worker(rank, world, port, n, n_select, out_dir):
    """pipeline.phase1_select over gloo: points dealt round-robin, projections reduced to
    their owner, region scores all-gathered (kernels emulated as above)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R.RankPlan = _OraclePlan
    R.bootstrap_spearman_multi = _oracle_multi
    X, Y, Z = _data(n, 40)
    rows = shard_rows(n, rank, world)
    feats = {"x": torch.from_numpy(X[rows.start:rows.stop]), "z": torch.from_numpy(Z[rows.start:rows.stop]),
             "w": torch.from_numpy((X[rows.start:rows.stop] * Z[rows.start:rows.stop]).copy())}
    gen = torch.Generator().manual_seed(5)
    mats = {p: torch.randn(40, 24, generator=gen) for p in feats}
    projectors = {p: (lambda x, m=mats[p]: x.double() @ m.double()) for p in feats}
    responses = {"r0": torch.from_numpy(Y[rows.start:rows.stop]), "r1": torch.from_numpy(X[rows.start:rows.stop, :20])}
    sel = P.phase1_select(feats, projectors, responses, list(feats), n, n_select=n_select, seed=42,
                          pg=dist.group.WORLD, kernels=CpuKernels())
    with open(os.path.join(out_dir, f"p1_{world}_{rank}.txt"), "w") as f:
        for r in sorted(sel):
            best, lst = sel[r]
            f.write(r + " " + best + " " + " ".join(f"{e['layer']}:{e['score']:.17g}" for e in lst) + "\n")
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_phase1_points_dealt_over_ranks(tmp_path, world):
    n, n_select = 120, 50
    for w in (1, world):
        mp.spawn(_phase1_worker, args=(w, _free_port(), n, n_select, str(tmp_path)), nprocs=w, join=True)
    ref = (tmp_path / "p1_1_0.txt").read_text()
    for r in range(world):  # every rank, the same selection and scores as one process
        assert (tmp_path / f"p1_{world}_{r}.txt").read_text() == ref
    # and those are the oracle's: SRP of the selection rows, emulated RDMs, midrank Spearman
    X, Y, Z = _data(n, 40)
    sel_idx = np.random.RandomState(42).choice(n, n_select, replace=False)
    gen = torch.Generator().manual_seed(5)
    full = {"x": X, "z": Z, "w": X * Z}
    mats = {p: torch.randn(40, 24, generator=gen) for p in full}
    for line in ref.splitlines():
        r, best, *pairs = line.split()
        y = (Y if r == "r0" else X[:, :20])[sel_idx]
        nr = emulated_rdm(np.ascontiguousarray(y))
        iu = np.triu_indices(n_select, 1)
        want = {}
        for p in full:
            proj = (torch.from_numpy(full[p][sel_idx]).double() @ mats[p].double()).float().numpy()
            want[p] = O.midrank_spearman(emulated_rdm(proj)[iu], nr[iu])
        got = {kv.split(":")[0]: float(kv.split(":")[1]) for kv in pairs}
        assert all(abs(got[p] - want[p]) < 1e-12 for p in full), (got, want)
        assert best == max(full, key=lambda p: (want[p], -list(full).index(p)))


def test_engine_byte_models(monkeypatch):
    # pipeline's algorithmic byte models (bench.py's engine roofline): EST passes move 136 B
    # per pair and unit in the B walk (codes 4 + A position 4 + the 128-B TB row) and 136 B
    # per pair in the A side; the per-unit join 12 B (VISREPS_ENGINE_LO_JOIN=1: + 4 + 4);
    # a joined call (SharedJoins) leaves its joins to shared_join_bytes; the full-set pass's
    # lane-0 shift sums (k_full_corr) read the A positions once more, 4 B per pair and unit
    import visreps_amd.pipeline as P

    monkeypatch.delenv("VISREPS_ENGINE_LO_JOIN", raising=False)
    monkeypatch.delenv("VISREPS_ENGINE_TRI", raising=False)
    assert P.engine_pair_bytes(True) == (136, 136, 12)
    monkeypatch.setenv("VISREPS_ENGINE_LO_JOIN", "1")
    assert P.engine_pair_bytes(True) == (136, 140, 16)
    monkeypatch.delenv("VISREPS_ENGINE_LO_JOIN")
    n, M = 10000, 10000 * 9999 // 2
    per = P.engine_call_bytes(n, 1001, 14)
    assert per == M * (16 * (136 + 14 * 136) + 14 * 12 + 14 * 4)
    assert P.engine_call_bytes(n, 1001, 14, joined=True) == M * (16 * (136 + 14 * 136) + 14 * 4)
    assert P.shared_join_bytes(n, 4, 14) == M * (16 + 16 + 14 * (4 + 16 + 16))
    # the grid call: per pass each region's A side, per model plan one walk (codes once, per
    # region the A position and the TB row), + the full-set pass's shift sums per unit
    assert P.engine_grid_bytes(n, 1001, 4, 14) == M * (16 * (4 * 136 + 14 * (4 + 4 * 132)) + 4 * 4 * 14)


@pytest.mark.parametrize("recv", [[[3, 0, 2], [1, 4, 0], [0, 0, 5]], [[2, 2], [0, 3]]])
def test_list_all_to_all_views_match_all_to_all_single_layout(monkeypatch, recv):
    # the RCCL branch of _all_to_all_rows (list all_to_all into views of `out`) has
    # no multi-rank run on CPU. Emulate `world` ranks in one process: each rank's call records
    # its send parts and receive views; a loopback then does the exchange (recv view j of rank
    # i <- send part i of rank j). Every rank's `out` must equal all_to_all_single's layout:
    # rank j's rows at offset sum(recv_rows[:j]), zero-row blocks included.
    world = len(recv)
    calls = []
    monkeypatch.setattr(P, "_list_all_to_all", lambda out, pg: True)

    def fake_all_to_all(outs, ins, group=None, async_op=False):  # noqa: ARG001
        assert len(outs) == len(ins) == world
        calls.append((outs, ins))
        return P._Done()

    monkeypatch.setattr(P.dist, "all_to_all", fake_all_to_all)
    # recv[i][j] = rows rank i receives from rank j = rows rank j sends to rank i
    sends = [[torch.full((recv[i][j], 3), float(100 * j + 10 * i), dtype=torch.float32)
              + torch.arange(recv[i][j], dtype=torch.float32)[:, None] if recv[i][j] else None
              for i in range(world)] for j in range(world)]
    outs = []
    for r in range(world):
        _, out, _ = P._all_to_all_rows(sends[r], recv[r], (3,), torch.float32, "cpu", None)
        outs.append(out)
    for i in range(world):  # the loopback exchange
        for j in range(world):
            views = calls[i][0]
            part = calls[j][1][i]
            assert views[j].shape == part.shape
            views[j].copy_(part)
    for i in range(world):
        want = torch.cat([sends[j][i] if sends[j][i] is not None else torch.empty((0, 3))
                          for j in range(world)], 0)
        assert torch.equal(outs[i], want)
        assert outs[i].shape[0] == sum(recv[i])
