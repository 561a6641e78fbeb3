"""All-layers x all-ROIs RSA with stimulus sharding over ranks (the bench workload and the
multi-GPU path of the eval driver).

Per step (BASELINE.json configs[1]: CustomCNN points x NSD ROIs, N stimuli, 1000 boots):
  1. extraction   each rank forwards its stimulus shard; the 14 hooked points are
                  flattened into per-point (n_local, D) HBM buffers;
  2. RDMs         per point / ROI: each rank splits its own rows (row statistics +
                  centred bf16 hi/lo planes), RCCL all-gathers the planes (the one
                  feature exchange), computes a cost-balanced range of the 128x128
                  upper-triangle Gram tiles, and the packed tile ranges are all-gathered
                  and unpacked (with their mirrors) into every rank's RDM;
  3. rank plans   each rank sorts the triangles of the RDMs its units use;
  4. units        (point, ROI) units listed ROI-major, one contiguous range per rank; a
                  rank's units sharing a ROI are one engine call (vr_bootstrap_spearman_multi:
                  the neural plan's rank walk runs once per pass for all of them); each unit
                  is the point estimate + n_boot subsets (evals.py:341-373 semantics,
                  RandomState(seed) per unit);
  5. gather       per-unit score vectors are gathered to every rank.
Given the RDMs, scores are exact-integer Spearman values and do not depend on how units
are split over ranks. The RDM entries themselves can differ in the last fp32 bits between
world sizes: the Gram's split-K factor and the wide 256x256 kernel are chosen per launched
tile range (csrc/rdm.hip), so a rank's range may sum a tile in another order than the
one-GPU launch (tests/test_gpu_parity.py::test_rdm_tile_ranges_wide_d_match_within_rounding).
"""
from __future__ import annotations

import functools
import math
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ._lib import check, lib, stream_of, workspace
from .analysis import rsa as R
from .analysis._random import LegacyRandomState, bootstrap_indices, draw_bootstrap_indices
from .dataloaders.synthetic import shard_rows


@dataclass
class StepTimes:
    """HIP-event totals of the hot kernels on this rank (ms)."""

    gram_ms: float = 0.0
    gram_flops: float = 0.0
    engine_ms: float = 0.0
    engine_bytes: float = 0.0      # the engine's own algorithmic bytes (engine_call_bytes)
    engine_ref_bytes: float = 0.0  # reference-equivalent bytes (engine_bytes(), §8(d))
    engine_calls: int = 0          # units
    phase_ms: Dict[str, float] = field(default_factory=dict)  # step phases (bench breakdown)
    _pending: list = field(default_factory=list)

    def phases(self, names: Sequence[str], events: Sequence) -> None:
        """Phase i spans events[i] .. events[i + 1] (HIP events on the compute stream)."""
        self._pending.append(("phases", list(names), list(events), 0.0, 0, 0.0))

    def record(self, kind: str, start, end, work: float, calls: int = 1, ref: float = 0.0):
        self._pending.append((kind, start, end, work, calls, ref))

    def resolve(self):
        for kind, s, e, w, c, ref in self._pending:
            if kind == "phases":
                for i, name in enumerate(s):
                    self.phase_ms[name] = self.phase_ms.get(name, 0.0) + e[i].elapsed_time(e[i + 1])
                continue
            ms = s.elapsed_time(e)
            if kind == "gram":
                self.gram_ms += ms
                self.gram_flops += w
            else:
                self.engine_ms += ms
                self.engine_bytes += w
                self.engine_ref_bytes += ref
                self.engine_calls += c
        self._pending.clear()


def _world(pg) -> Tuple[int, int]:
    if pg is None or not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(pg), dist.get_world_size(pg)


# ---------------------------------------------------------------------------------------
# block-distributed RDM
# ---------------------------------------------------------------------------------------
@functools.lru_cache(maxsize=16)
def _tile_cum_cost(n: int) -> np.ndarray:
    L = lib()
    T = int(L.vr_rdm_tile_count(n))
    costs = np.array([L.vr_rdm_tile_cost(n, t) for t in range(T)], dtype=np.float64)
    return np.concatenate([[0.0], np.cumsum(costs)])


def tile_ranges(n: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous ranges of the upper-triangle tile list with near-equal element counts."""
    cum = _tile_cum_cost(n)
    T = len(cum) - 1
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(np.searchsorted(cum, cum[-1] * r / world)))
    bounds.append(T)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def tile_rect(n: int, tile: int) -> Tuple[int, int, int, int]:
    """(row0, col0, rows, cols) of upper-triangle tile `tile` (vr_rdm_tile_rect)."""
    import ctypes

    v = [ctypes.c_int64() for _ in range(4)]
    check(lib().vr_rdm_tile_rect(n, tile, *[ctypes.byref(x) for x in v]), "vr_rdm_tile_rect")
    return tuple(int(x.value) for x in v)


def _tile_fraction(n: int, t0: int, t1: int) -> float:
    cum = _tile_cum_cost(n)
    return float((cum[t1] - cum[t0]) / cum[-1]) if cum[-1] > 0 else 0.0


def rdm_tiles_into(x: torch.Tensor, out: torch.Tensor, t0: int, t1: int,
                   correction: float = 1e-12, times: Optional[StepTimes] = None) -> None:
    """Write Gram tiles [t0, t1) of x's RDM (and their mirrors) into out."""
    n, d = x.shape
    if t1 <= t0:
        return
    L = lib()
    ws = workspace.get(x.device, L.vr_rdm_tiles_workspace(n, d, t0, t1), "rdm")
    ev = None
    if times is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    check(L.vr_rdm_pearson_tiles_f32(x.data_ptr(), n, d, x.stride(0), out.data_ptr(), n,
                                     float(correction), t0, t1, ws.data_ptr(), ws.numel(),
                                     stream_of(x.device)), "vr_rdm_pearson_tiles_f32")
    if times is not None:
        ev[1].record()
        times.record("gram", ev[0], ev[1], _gram_flops(n, d) * _tile_fraction(n, t0, t1))


def _gram_flops(n: int, d: int) -> float:
    """Algorithmic Gram FLOPs of one RDM: N(N+1)D (unique pairs, 2 FLOP/MAC)."""
    return float(n) * (n + 1) * d


def _gram_exact_fp32() -> bool:
    import os

    return os.environ.get("VISREPS_GRAM") == "fp32"


class RdmKernels:
    """The HIP entry points of the distributed RDM (csrc/rdm.hip). The orchestration below
    calls nothing else on the device, so the gloo tests substitute a CPU emulation of
    exactly these five calls and run the orchestration itself unchanged."""

    @staticmethod
    def plane_rows(n: int) -> int:
        return int(lib().vr_rdm_plane_rows(n))

    @staticmethod
    def plane_elems(d: int) -> int:  # uint16 elements per row of plane records
        return int(lib().vr_rdm_plane_row_bytes(d)) // 2

    @staticmethod
    def split_rows(x: torch.Tensor, correction: float):
        """(planes (rows, plane_elems) int16, mean (rows,), std (rows,)) of local rows."""
        rows, d = x.shape
        planes = torch.empty((rows, RdmKernels.plane_elems(d)), dtype=torch.int16, device=x.device)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        std = torch.empty(rows, dtype=torch.float32, device=x.device)
        if rows:
            check(lib().vr_rdm_split_rows_f32(x.data_ptr(), rows, d, x.stride(0), float(correction),
                                              mean.data_ptr(), std.data_ptr(), planes.data_ptr(),
                                              stream_of(x.device)), "vr_rdm_split_rows_f32")
        return planes, mean, std

    @staticmethod
    def tiles_from_planes(planes, mean, std, n: int, d: int, out: torch.Tensor, t0: int, t1: int,
                          correction: float, times: Optional[StepTimes] = None) -> None:
        if t1 <= t0:
            return
        L = lib()
        ws = workspace.get(out.device, L.vr_rdm_planes_tiles_workspace(n, d, t0, t1), "rdm")
        ev = None
        if times is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        check(L.vr_rdm_pearson_tiles_planes(planes.data_ptr(), mean.data_ptr(), std.data_ptr(), n, d,
                                            out.data_ptr(), n, float(correction), t0, t1, ws.data_ptr(),
                                            ws.numel(), stream_of(out.device)), "vr_rdm_pearson_tiles_planes")
        if times is not None:
            ev[1].record()
            times.record("gram", ev[0], ev[1], _gram_flops(n, d) * _tile_fraction(n, t0, t1))

    @staticmethod
    def pack(out: torch.Tensor, n: int, t0: int, t1: int, packed: torch.Tensor) -> None:
        check(lib().vr_rdm_tiles_pack(out.data_ptr(), n, n, t0, t1, packed.data_ptr(),
                                      stream_of(out.device)), "vr_rdm_tiles_pack")

    @staticmethod
    def unpack(packed: torch.Tensor, n: int, t0: int, t1: int, out: torch.Tensor) -> None:
        check(lib().vr_rdm_tiles_unpack(packed.data_ptr(), n, t0, t1, out.data_ptr(), n,
                                        stream_of(out.device)), "vr_rdm_tiles_unpack")

    @staticmethod
    def tiles_from_rows(x, out, t0, t1, correction, times=None) -> None:
        rdm_tiles_into(x, out, t0, t1, correction, times)


KERNELS = RdmKernels()
TILE = 128  # floats per packed tile edge (csrc/rdm.hip GT)


def _all_gather_padded(t: torch.Tensor, sizes: Sequence[int], pg, async_op: bool = False):
    """All-gather of a rank-local (sizes[rank], ...) tensor, padded to max(sizes) rows;
    returns (work, buffer (world * per, ...), send buffer)."""
    world = len(sizes)
    per = max(sizes)
    send = torch.zeros((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    send[: t.size(0)] = t
    full = torch.empty((world * per,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if dist.get_backend(pg) == "nccl":
        work = dist.all_gather_into_tensor(full, send, group=pg, async_op=async_op)
    else:  # gloo: the CPU tests of the orchestration
        work = dist.all_gather(list(full.chunk(world)), send, group=pg, async_op=async_op)
    return work, full, send


def _compact(full: torch.Tensor, sizes: Sequence[int], rows_out: int) -> torch.Tensor:
    """Rows of every rank's slot of a padded gather, in rank order, into (rows_out, ...)
    with zero rows after the last real one."""
    per = max(sizes)
    out = torch.zeros((rows_out,) + tuple(full.shape[1:]), dtype=full.dtype, device=full.device)
    at = 0
    for r, sz in enumerate(sizes):
        out[at:at + sz] = full[r * per: r * per + sz]
        at += sz
    return out


class _Gathered:
    """The exchanged rows of one point, ready for the rank's tile range."""

    def __init__(self, kind: str, n: int, d: int, **parts):
        self.kind, self.n, self.d, self.parts = kind, n, d, parts


def gather_point_async(x_local: torch.Tensor, n: int, pg, correction: float = 1e-12,
                       kernels: RdmKernels = None):
    """Start one point's feature exchange; returns finish() -> _Gathered.

    Split path (default): the rank splits its OWN rows (row statistics + centred bf16
    hi/lo plane records, vr_rdm_split_rows_f32) and the planes and statistics are
    all-gathered, so no rank recomputes another rank's prepass. Exact-fp32 Gram
    (VISREPS_GRAM=fp32): the fp32 rows themselves. The collective runs on the
    communicator's stream, so work already queued on the compute stream overlaps it."""
    K = kernels or KERNELS
    rank, world = _world(pg)
    x_local = x_local.float().contiguous()
    d = x_local.size(1)
    sizes = [len(shard_rows(n, r, world)) for r in range(world)]
    if _gram_exact_fp32():
        work, full, send = _all_gather_padded(x_local, sizes, pg, async_op=True)

        def finish_rows(_keep=send) -> _Gathered:
            work.wait()
            return _Gathered("rows", n, d, x=_compact(full, sizes, n))

        return finish_rows
    planes, mean, std = K.split_rows(x_local, correction)
    stats = torch.stack([mean, std], dim=1)
    # plane records travel as 8-byte words (RCCL and gloo have no 16-bit integer type; a
    # row is nstage x 128 B, and 8-B elements keep the element count of a 10k x 290,400
    # point (11.6 GB) below 2^31)
    w1, pfull, s1 = _all_gather_padded(planes.view(torch.int64), sizes, pg, async_op=True)
    w2, sfull, s2 = _all_gather_padded(stats, sizes, pg, async_op=True)

    def finish_planes(_keep=(s1, s2)) -> _Gathered:
        w1.wait()
        w2.wait()
        st = _compact(sfull, sizes, n)
        return _Gathered("planes", n, d, planes=_compact(pfull, sizes, K.plane_rows(n)).view(torch.int16),
                         mean=st[:, 0].contiguous(), std=st[:, 1].contiguous())

    return finish_planes


def rdm_from_gathered(g: _Gathered, pg, times: Optional[StepTimes] = None, correction: float = 1e-12,
                      kernels: RdmKernels = None) -> torch.Tensor:
    """Every rank computes its balanced tile range (tile_ranges) into the (n, n) RDM, packs
    it (128 x 128 floats per tile), and the packed ranges are all-gathered and unpacked
    (tile + mirror) into every rank's RDM. Every entry is written by exactly one rank's
    tile, so there is no zero fill and no sum: each rank receives about n^2/2 floats
    instead of the 2 n^2 a ring sum all-reduce of the full matrix moves."""
    K = kernels or KERNELS
    rank, world = _world(pg)
    n = g.n
    dev = g.parts["planes"].device if g.kind == "planes" else g.parts["x"].device
    out = torch.empty((n, n), dtype=torch.float32, device=dev)
    ranges = tile_ranges(n, world) if world > 1 else [(0, int(lib().vr_rdm_tile_count(n)))]
    t0, t1 = ranges[rank]
    if g.kind == "planes":
        K.tiles_from_planes(g.parts["planes"], g.parts["mean"], g.parts["std"], n, g.d, out, t0, t1,
                            correction, times)
    else:
        K.tiles_from_rows(g.parts["x"], out, t0, t1, correction, times)
    if world == 1:
        return out
    counts = [b - a for a, b in ranges]
    packed = torch.empty((t1 - t0, TILE * TILE), dtype=torch.float32, device=dev)
    if t1 > t0:
        K.pack(out, n, t0, t1, packed)
    _, allp, _keep = _all_gather_padded(packed, counts, pg)
    per = max(counts)
    for r, (a, b) in enumerate(ranges):
        if r != rank and b > a:
            K.unpack(allp[r * per: r * per + (b - a)], n, a, b, out)
    return out


def gather_rows(x_local: torch.Tensor, n: int, pg) -> torch.Tensor:
    """RCCL all-gather of every rank's stimulus rows into the full (n, d) matrix."""
    rank, world = _world(pg)
    if world == 1:
        return x_local
    sizes = [len(shard_rows(n, r, world)) for r in range(world)]
    work, full, _keep = _all_gather_padded(x_local, sizes, pg)
    return _compact(full, sizes, n)


class PrefetchedRDMs:
    """RDM source for all_units_rsa over stimulus-sharded features: asking for point
    points[i] first starts the exchange of points[i + 1] (gather_point_async), so the next
    point's plane all-gather overlaps this point's Gram. Every rank asks for the points in
    the same order (all_units_rsa walks `points`), so the collectives are issued in one
    order.

    exchange_pg: a second process group (its own RCCL communicator and stream) for the
    plane all-gathers. With it, start_all() issues every point's exchange at once: they
    stream over xGMI while phase 1, the neural RDMs and the first points' Grams run, and
    the collectives on `pg` (phase-1 rows, packed tile ranges, scores) do not queue
    behind them. All ranks call start_all() at the same point of the step."""

    def __init__(self, feats: Dict[str, torch.Tensor], points: Sequence[str], n: int, pg=None,
                 times: Optional[StepTimes] = None, kernels: RdmKernels = None, exchange_pg=None):
        self.feats, self.points, self.n, self.pg, self.times = feats, list(points), n, pg, times
        self.kernels = kernels or KERNELS
        self.exchange_pg = exchange_pg if exchange_pg is not None else pg
        self.pending: Dict[str, Callable[[], _Gathered]] = {}

    def _start(self, p: str) -> None:
        if p not in self.pending:
            self.pending[p] = gather_point_async(self.feats[p], self.n, self.exchange_pg, kernels=self.kernels)

    def start_all(self) -> None:
        if _world(self.pg)[1] > 1:
            for p in self.points:
                self._start(p)

    def __call__(self, p: str) -> torch.Tensor:
        if _world(self.pg)[1] == 1:  # one GPU: the single-launch RDM (no exchange, no prepass split)
            return distributed_rdm(self.feats[p], self.n, None, self.times)
        self._start(p)
        i = self.points.index(p)
        if i + 1 < len(self.points):
            self._start(self.points[i + 1])
        g = self.pending.pop(p)()
        return rdm_from_gathered(g, self.pg, self.times, kernels=self.kernels)


def distributed_rdm(x_local: torch.Tensor, n: int, pg=None, times: Optional[StepTimes] = None,
                    kernels: RdmKernels = None) -> torch.Tensor:
    """Full (n, n) RDM on every rank from each rank's stimulus rows (gather_point_async +
    rdm_from_gathered). One GPU: the single-launch RDM of the local rows."""
    rank, world = _world(pg)
    if world == 1:
        x = x_local.float().contiguous()
        out = torch.empty((n, n), dtype=torch.float32, device=x.device)
        rdm_tiles_into(x, out, 0, int(lib().vr_rdm_tile_count(n)), times=times)
        return out
    g = gather_point_async(x_local, n, pg, kernels=kernels)()
    return rdm_from_gathered(g, pg, times, kernels=kernels)


# ---------------------------------------------------------------------------------------
# units
# ---------------------------------------------------------------------------------------
def engine_bytes(n: int, n_boot: int) -> float:
    """Reference-equivalent bytes of one unit: 8 * [M(N) + n_boot * M(int(0.9 N))]
    (both fp32 triangles read once per Spearman evaluation). The engine
    never streams these; it is the yardstick of the reference's algorithm."""
    k = int(0.9 * n)
    return 8.0 * (n * (n - 1) // 2 + n_boot * (k * (k - 1) // 2))


# HBM bytes per pair of the engine's own passes (engine.hip). Exact chunk-base form: the A
# walk streams its codes and writes one 128-byte TB row per pair; each B walk streams its
# codes and the two join arrays (posA, chunkA) and gathers one TB row per pair (its 256-byte
# chunk-base rows come from a 2 MB L2-resident table, not HBM). EST form (the default): the
# A side streams its codes twice (count
# pre-pass + rank walk), the B walk reads the window low ends instead of the chunk array (the
# full-set pass 0 runs EST too, lane 0 on its own exact line). k_join reads the B codes and
# one 8-byte pair-map record and writes the A positions, k_join_lo the low ends, per unit.
def engine_pair_bytes(est: Optional[bool] = None) -> Tuple[int, int, int]:
    """(A walk per pass, B walk per pass and unit, join per unit) bytes per pair."""
    if est is None:
        import os
        est = os.environ.get("VISREPS_ENGINE_EST") != "0"
    # A side: codes 4 (EST: count pre-pass + rank walk, 4 each) + 128 B TB row write.
    # B walk: codes 4 + A position 4 + second join array 4 (EST: window low end; exact: A chunk)
    # + 128 B TB row gather (the exact form's 256-B chunk-base rows are L2-resident).
    # Join: B codes 4 + the A map gather (EST: 4-B position map; exact: 8-B pair-map record)
    # + posA write 4 + second array write 4.
    return (4 + 4 + 128, 4 + 4 + 4 + 128, 4 + 4 + 4 + 4) if est else (4 + 128, 4 + 4 + 4 + 128, 4 + 8 + 4 + 4)


def engine_call_bytes(n: int, subsets: int, units: int) -> float:
    """Algorithmic HBM bytes of one engine call: `units` B plans against one A plan over
    `subsets` subsets (64 per pass)."""
    a, b, j = engine_pair_bytes()
    M = n * (n - 1) // 2
    passes = -(-subsets // 64)
    return float(M) * (passes * (a + units * b) + units * j)


def run_unit(plan_m: R.RankPlan, plan_n: R.RankPlan, idx: Optional[np.ndarray],
             times: Optional[StepTimes] = None) -> torch.Tensor:
    ev = None
    if times is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    scores = R.bootstrap_spearman(plan_m, plan_n, idx, full_first=True)
    if times is not None:
        ev[1].record()
        nb = 0 if idx is None else len(idx)
        times.record("engine", ev[0], ev[1], engine_call_bytes(plan_m.n, nb + 1, 1),
                     ref=engine_bytes(plan_m.n, nb))
    return scores


def run_group(plan_n: R.RankPlan, plans_m: Sequence[R.RankPlan], idx: Optional[np.ndarray],
              times: Optional[StepTimes] = None) -> torch.Tensor:
    """Units (m, n) for every model plan m against one neural plan n in one engine call:
    (len(plans_m), 1 + n_boot) scores; the neural plan's rank walk is shared."""
    ev = None
    if times is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    scores = R.bootstrap_spearman_multi(plan_n, plans_m, idx, full_first=True)
    if times is not None:
        ev[1].record()
        nb = 0 if idx is None else len(idx)
        times.record("engine", ev[0], ev[1], engine_call_bytes(plan_n.n, nb + 1, len(plans_m)),
                     calls=len(plans_m), ref=engine_bytes(plan_n.n, nb) * len(plans_m))
    return scores


def unit_split(units: Sequence, world: int) -> List[Tuple[int, int]]:
    """Contiguous, near-equal [lo, hi) ranges of the unit list, one per rank."""
    u = len(units)
    b = [round(r * u / world) for r in range(world + 1)]
    return [(b[r], b[r + 1]) for r in range(world)]


def phase1_select(feats: Dict[str, torch.Tensor], projectors: Dict, responses: Dict[str, torch.Tensor],
                  points: Sequence[str], n: int, *, n_select: int = 1000, seed: int = 42,
                  pg=None, times: Optional[StepTimes] = None) -> Dict[str, Tuple[str, List[Dict]]]:
    """Phase-1 layer selection of the reference eval (evals.py:249-287) on stimulus-sharded
    features. RandomState(seed).choice(n, n_select) picks the selection stimuli (re-created
    per (region, subject); the regions share one subject's stimuli, so one draw serves them
    all); each rank projects its selected rows of every point by the point's SRP matrix (the
    bulk extraction's torch.sparse.mm, models/utils.py:297-344, here vr_srp_csr_f32). The
    projection is row by row, so projecting the selected rows equals projecting every row
    and selecting after, as the reference does: phase 1 reads no other projected row
    (evals.py:254-268) and phase 2 re-extracts. Then selection RDMs of the projected points
    and of each region's responses; Spearman of every point against every region; best =
    first strict maximum.
    Returns {region: (best point, [{"layer", "score"} per point])} on every rank."""
    rank, world = _world(pg)
    rows = shard_rows(n, rank, world)
    k = min(int(n_select), n) if n_select is not None else n
    sel = (LegacyRandomState(seed).choice(n, k, replace=False) if k < n else np.arange(n))
    mine = np.flatnonzero((sel >= rows.start) & (sel < rows.stop))
    dev = next(iter(responses.values())).device
    pos_t = torch.as_tensor(mine, dtype=torch.long, device=dev)
    src_t = torch.as_tensor(sel[mine] - rows.start, dtype=torch.long, device=dev)

    def selected(x_mine: torch.Tensor) -> torch.Tensor:  # this rank's selected rows -> (k, d), every rank
        out = torch.zeros((k, x_mine.size(1)), dtype=torch.float32, device=dev)
        out[pos_t] = x_mine.float()
        if world > 1:  # disjoint rows: the sum is exact
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=pg)
        return out

    def timed_rdm(x: torch.Tensor) -> torch.Tensor:
        out = torch.empty((x.size(0), x.size(0)), dtype=torch.float32, device=dev)
        rdm_tiles_into(x, out, 0, int(lib().vr_rdm_tile_count(x.size(0))), times=times)
        return out

    mplans = []
    for p in points:
        proj = projectors[p](feats[p][src_t])  # SRP of this rank's selected stimuli
        mplans.append(R.RankPlan(timed_rdm(selected(proj))))
        del proj
    out = {}
    for r, y in responses.items():
        pn = R.RankPlan(timed_rdm(selected(y[src_t])))
        sc = R.bootstrap_spearman_multi(pn, mplans, None, full_first=True)[:, 0].cpu().numpy()
        best, best_score, scores = None, -float("inf"), []
        for p, v in zip(points, sc):
            scores.append({"layer": p, "score": float(v)})
            if v > best_score:  # strict: the first maximal point wins (evals.py:273-275)
                best, best_score = p, float(v)
        out[r] = (best, scores)
    return out


def summarize(scores: np.ndarray, bootstrap: bool) -> Dict:
    point = float(scores[0])
    res = {"score": point, "ci_low": None, "ci_high": None}
    if bootstrap:
        boot = scores[1:]
        res["ci_low"] = R.percentile(boot, 2.5)
        res["ci_high"] = R.percentile(boot, 97.5)
        res["bootstrap_scores"] = boot.tolist()
    return res


def all_units_rsa(model_rdm_fn: Callable[[str], torch.Tensor], points: Sequence[str],
                  neural_rdms: Dict[str, torch.Tensor], n: int, *, n_boot: int = 1000,
                  seed: int = 42, pg=None, times: Optional[StepTimes] = None,
                  keep_plans: bool = False, plan_fn=None, unit_fn=None, group_fn=None
                  ) -> Dict[Tuple[str, str], Dict]:
    """Point + bootstrap Spearman RSA for every (point, region) unit; returns the
    per-unit results on every rank.

    Units are listed region-major and cut into one contiguous range per rank, so a
    rank's units come in groups that share a neural RDM; each group is one engine call
    (run_group: the neural plan's rank walk is shared by the group's layers). plan_fn /
    group_fn default to RankPlan / run_group (the HIP engine); a per-unit unit_fn(model
    plan, neural plan, idx, times) may be given instead of group_fn."""
    plan_fn = plan_fn or R.RankPlan
    if group_fn is None:
        if unit_fn is not None:
            def group_fn(pn, pms, idx_, t):
                return [np.asarray(torch.as_tensor(unit_fn(pm, pn, idx_, t)).cpu()) for pm in pms]
        else:
            group_fn = run_group
    rank, world = _world(pg)
    regions = list(neural_rdms)
    units = [(p, r) for r in regions for p in points]
    lo, hi = unit_split(units, world)[rank]
    mine = units[lo:hi]
    k = int(0.9 * n)
    idx = None
    if n_boot > 0:
        # RandomState(seed) is re-created per (region, subject) (evals.py:356), so every unit
        # draws the same (n_boot, k) index sets: drawn once per call (host MT19937), one upload
        dev = next(iter(neural_rdms.values())).device
        idx = torch.from_numpy(draw_bootstrap_indices(seed, n, k, n_boot)).to(dev)
    local: Dict[Tuple[str, str], np.ndarray] = {}
    need = {p for p, _ in mine}
    mplans = {}
    for p in points:
        rdm = model_rdm_fn(p)  # collective: every rank takes part in every point's RDM
        if p in need:
            mplans[p] = plan_fn(rdm)
        del rdm
    by_region: Dict[str, List[str]] = {}
    for p, r in mine:
        by_region.setdefault(r, []).append(p)
    for r, pts in by_region.items():
        pn = plan_fn(neural_rdms[r])
        out = group_fn(pn, [mplans[p] for p in pts], idx, times)
        for j, p in enumerate(pts):
            local[(p, r)] = np.asarray(torch.as_tensor(out[j]).cpu())
        del pn
    del mplans
    if world > 1:
        gathered: List[Dict] = [None] * world
        dist.all_gather_object(gathered, local, group=pg)
        merged = {}
        for g in gathered:
            merged.update(g)
        local = merged
    return {u: summarize(local[u], n_boot > 0) for u in units}
