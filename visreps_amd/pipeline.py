"""All-layers x all-ROIs RSA with stimulus sharding over ranks (the bench workload and the
multi-GPU path of the eval driver).

Per step (BASELINE.json configs[1]: CustomCNN points x NSD ROIs, N stimuli, 1000 boots):
  1. extraction   each rank forwards its stimulus shard; the 14 hooked points are
                  flattened into per-point (n_local, D) HBM buffers;
  2. RDMs         an RdmSchedule (the same on every rank) gives every RDM (14 points, 4
                  ROIs) an owner, or, for an RDM heavier than the per-rank mean, a few
                  owners of pieces cut at the wide kernel's super-tile rows. Each rank
                  sends its rows of an RDM to that RDM's owners only (all_to_all_single
                  over RCCL), each owner computes its pieces with the one-GPU kernel path,
                  and the packed pieces go only to the ranks whose units read the RDM;
  3. rank plans   each rank sorts the triangles of the RDMs its units use;
  4. units        (point, ROI) units listed ROI-major, one contiguous range per rank; a
                  rank's units sharing a ROI are one engine call (vr_bootstrap_spearman_multi:
                  the neural plan's rank walk runs once per pass for all of them); each unit
                  is the point estimate + n_boot subsets (evals.py:341-373 semantics,
                  RandomState(seed) per unit);
  5. gather       per-unit score vectors are gathered to every rank.
Every tile of an RDM is computed by the same kernel, over the same depth order, whatever
rank computes it (pieces are cut only at aligned boundaries, csrc/rdm.hip plan_range), so
the RDMs -- and, the statistic being exact integer arithmetic, the scores -- are bit-identical
at every world size (tests/test_distributed.py, tests/test_gpu_distributed.py).
"""
from __future__ import annotations

import functools
import math
import os
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


@dataclass
class SplitRows:
    """Stimulus rows of one point already split for the Gram (vr_rdm_split_rows_f32): per
    row the float32 mean and std of the reference's compute_rdm (rsa.py:80-87) and the bf16
    hi/lo records of the centred row (planes: (rows_padded, plane_elems) int16, rows past
    `rows` zero). bench.extract writes these straight from the forward hooks, so the Grams
    need no prepass over fp32 copies of the features; the tiles computed from them equal the
    tiles computed from the raw rows bit for bit (tests/test_gpu_distributed.py)."""

    planes: torch.Tensor
    mean: torch.Tensor
    std: torch.Tensor
    rows: int
    d: int

    def size(self, dim: int) -> int:
        return self.rows if dim == 0 else self.d

    @property
    def device(self):
        return self.planes.device


class RdmKernels:
    """The HIP entry points of the distributed RDM (csrc/rdm.hip). The orchestration below
    calls nothing else on the device, so the gloo tests substitute a CPU emulation of
    exactly these calls and run the orchestration itself unchanged."""

    @staticmethod
    def tiles_from_rows(x, out, t0, t1, correction, times=None) -> None:
        """Gram tiles [t0, t1) of x's RDM (+ mirrors) into out (vr_rdm_pearson_tiles_f32)."""
        rdm_tiles_into(x, out, t0, t1, correction, times)

    @staticmethod
    def plane_rows(n: int) -> int:
        return int(lib().vr_rdm_plane_rows(n))

    @staticmethod
    def plane_elems(d: int) -> int:  # int16 elements per row of plane records
        return int(lib().vr_rdm_plane_row_bytes(d)) // 2

    @staticmethod
    def split_rows_into(x: torch.Tensor, correction: float, planes: torch.Tensor, mean: torch.Tensor,
                        std: torch.Tensor) -> None:
        """Row statistics + hi/lo records of x's rows into the given buffers (contiguous,
        row-aligned views of a SplitRows' tensors)."""
        rows, d = x.shape
        if rows:
            check(lib().vr_rdm_split_rows_f32(x.data_ptr(), rows, d, x.stride(0), float(correction),
                                              mean.data_ptr(), std.data_ptr(), planes.data_ptr(),
                                              stream_of(x.device)), "vr_rdm_split_rows_f32")

    @staticmethod
    def split_rows_multi(xs: Sequence[torch.Tensor], correction: float, outs: Sequence[SplitRows], r0: int) -> None:
        """Rows [r0, r0 + rows) of several points' SplitRows from the (rows, d) tensors xs
        (one launch, vr_rdm_split_rows_multi_f32; the same arithmetic as split_rows_into)."""
        import ctypes

        k = len(xs)
        if k == 0 or xs[0].size(0) == 0:
            return
        # the kernel reads fp32 rows with unit inner stride (half/bf16 hook outputs under
        # autocast, or strided views, are widened / compacted here, as tiles_from_rows does)
        xs = [x if (x.dtype == torch.float32 and x.stride(1) == 1) else x.float().contiguous() for x in xs]
        P64, I64 = ctypes.c_void_p * k, ctypes.c_int64 * k
        check(lib().vr_rdm_split_rows_multi_f32(
            k, P64(*[x.data_ptr() for x in xs]), I64(*[x.size(1) for x in xs]), I64(*[x.stride(0) for x in xs]),
            xs[0].size(0), float(correction), P64(*[o.mean[r0:].data_ptr() for o in outs]),
            P64(*[o.std[r0:].data_ptr() for o in outs]), P64(*[o.planes[r0:].data_ptr() for o in outs]),
            stream_of(xs[0].device)), "vr_rdm_split_rows_multi_f32")

    @staticmethod
    def gather_rows_multi(xs: Sequence[torch.Tensor], src, dst, outs: Sequence[torch.Tensor]) -> None:
        """outs[p][dst[i]] = xs[p][src[i]] for every point p (host index lists; one launch,
        vr_gather_rows_multi_f32)."""
        import ctypes

        k, m = len(xs), len(src)
        if k == 0 or m == 0:
            return
        if (any(x.dtype != torch.float32 or x.stride(1) != 1 for x in xs) or any(o.stride(1) != 1 for o in outs)
                or os.environ.get("VISREPS_SEL_GATHER") == "torch"):  # (the latter: A/B timing)
            si = torch.as_tensor(np.asarray(src), dtype=torch.long, device=xs[0].device)
            di = torch.as_tensor(np.asarray(dst), dtype=torch.long, device=xs[0].device)
            for x, o in zip(xs, outs):
                o[di] = x[si].float()
            return
        P64, I64, I32 = ctypes.c_void_p * k, ctypes.c_int64 * k, ctypes.c_int32 * m
        check(lib().vr_gather_rows_multi_f32(
            k, P64(*[x.data_ptr() for x in xs]), I64(*[x.size(1) for x in xs]), I64(*[x.stride(0) for x in xs]),
            m, I32(*[int(v) for v in src]), I32(*[int(v) for v in dst]), P64(*[o.data_ptr() for o in outs]),
            I64(*[o.stride(0) for o in outs]), stream_of(xs[0].device)), "vr_gather_rows_multi_f32")

    @staticmethod
    def tiles_from_planes(sr: SplitRows, n: int, out: torch.Tensor, t0: int, t1: int, correction: float,
                          times: Optional[StepTimes] = None) -> None:
        """Gram tiles [t0, t1) from pre-split rows (vr_rdm_pearson_tiles_planes)."""
        if t1 <= t0:
            return
        L = lib()
        d = sr.d
        ws = workspace.get(out.device, L.vr_rdm_planes_tiles_workspace(n, d, t0, t1), "rdm")
        ev = None
        if times is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        check(L.vr_rdm_pearson_tiles_planes(sr.planes.data_ptr(), sr.mean.data_ptr(), sr.std.data_ptr(), n, d,
                                            out.data_ptr(), n, float(correction), t0, t1, ws.data_ptr(),
                                            ws.numel(), stream_of(out.device)), "vr_rdm_pearson_tiles_planes")
        if times is not None:
            ev[1].record()
            times.record("gram", ev[0], ev[1], _gram_flops(n, d) * _tile_fraction(n, t0, t1))

    def empty_split(self, rows: int, d: int, device) -> SplitRows:
        """Buffers for `rows` split rows: every writer (split_rows*, the owner's row copy)
        fills whole rows incl. the k padding, so only the padding rows past `rows` are zeroed
        (zeroing the whole buffer cost ~8 ms per bench step)."""
        planes = torch.empty((self.plane_rows(rows), self.plane_elems(d)), dtype=torch.int16, device=device)
        planes[rows:].zero_()
        return SplitRows(planes, torch.empty(rows, dtype=torch.float32, device=device),
                         torch.empty(rows, dtype=torch.float32, device=device), rows, d)

    @staticmethod
    def pack(out: torch.Tensor, n: int, t0: int, t1: int, packed: torch.Tensor) -> None:
        check(lib().vr_rdm_tiles_pack(out.data_ptr(), n, n, t0, t1, packed.data_ptr(),
                                      stream_of(out.device)), "vr_rdm_tiles_pack")

    @staticmethod
    def unpack(packed: torch.Tensor, n: int, t0: int, t1: int, out: torch.Tensor) -> None:
        check(lib().vr_rdm_tiles_unpack(packed.data_ptr(), n, t0, t1, out.data_ptr(), n,
                                        stream_of(out.device)), "vr_rdm_tiles_unpack")


KERNELS = RdmKernels()
TILE = 128  # floats per packed tile edge (csrc/rdm.hip GT)


def _tri_start(r: int, t: int) -> int:
    return r * t - r * (r - 1) // 2


def aligned_boundaries(n: int, d: int) -> List[int]:
    """128-tile indices where an RDM may be cut so that every piece's tiles are
    bit-identical to the one-launch RDM (csrc/rdm.hip plan_range): the starts of the wide
    kernel's super-tile rows, tri_start(2r, T) for r <= R, and the end of the triangle (the
    remainder rows below 2R travel with the last piece)."""
    total = int(lib().vr_rdm_tile_count(n))
    R = int(lib().vr_rdm_wide_rows(n, d)) if d > 0 else 0
    T = -(-n // TILE)
    b = [_tri_start(2 * r, T) for r in range(R + 1)] if R > 0 else [0]
    return sorted(set(b + [total]))


@dataclass(frozen=True)
class GramPiece:
    """Tiles [t0, t1) of one RDM, computed by rank `owner`."""

    owner: int
    t0: int
    t1: int


@dataclass
class RdmSchedule:
    """Who computes and who needs every RDM of a step (pure function of the shapes and the
    world size: every rank builds the same one).

    units      (point, region) pairs, region-major; rank r runs units[lo:hi] of unit_ranges[r]
    consumers  name -> ranks whose units read that RDM (name = ("m", point) / ("n", region))
    pieces     name -> Gram pieces (owner, 128-tile range), cut only at aligned boundaries
    load       per-rank Gram cost (n(n+1)d-proportional tile elements x d)"""

    world: int
    n: int
    units: List[Tuple[str, str]]
    unit_ranges: List[Tuple[int, int]]
    consumers: Dict[Tuple[str, str], List[int]]
    pieces: Dict[Tuple[str, str], List[GramPiece]]
    load: List[float]

    def needs(self, rank: int) -> List[Tuple[str, str]]:
        return [k for k, c in self.consumers.items() if rank in c]

    def owners(self, name) -> List[int]:
        return sorted({p.owner for p in self.pieces[name]})


def make_schedule(n: int, dims: Dict[str, int], points: Sequence[str], regions: Dict[str, int],
                  world: int, split_factor: float = 1.25) -> RdmSchedule:
    """Units: region-major, one contiguous range per rank (unit_split), so a rank's units
    share their neural RDM (one A walk per engine call). Grams: one owner per RDM, longest
    first onto the least-loaded rank (a consumer of the RDM when it is within 2 % of the
    least load, which saves one transfer); an RDM costing more than split_factor x the
    per-rank mean is cut at aligned boundaries into that many near-equal pieces on distinct
    ranks. Each owner receives the full rows of its RDMs; consumers receive the packed
    tiles of the pieces they lack."""
    units = [(p, r) for r in regions for p in points]
    ranges = unit_split(units, world)
    consumers: Dict[Tuple[str, str], List[int]] = {}
    for rk, (lo, hi) in enumerate(ranges):
        for p, r in units[lo:hi]:
            consumers.setdefault(("m", p), [])
            consumers.setdefault(("n", r), [])
            if rk not in consumers[("m", p)]:
                consumers[("m", p)].append(rk)
            if rk not in consumers[("n", r)]:
                consumers[("n", r)].append(rk)
    width = {("m", p): int(dims[p]) for p in points}
    width.update({("n", r): int(v) for r, v in regions.items()})
    pieces, load = assign_grams(n, {k: w for k, w in width.items() if k in consumers}, consumers, world,
                                split_factor)
    return RdmSchedule(world, n, units, ranges, consumers, pieces, load)


def assign_grams(n: int, width: Dict, consumers: Dict, world: int, split_factor: float = 1.25):
    """Gram pieces of the RDMs `width` (name -> feature width) over `world` ranks (see
    make_schedule). Returns (pieces {name: [GramPiece]}, per-rank load)."""
    cum = _tile_cum_cost(n)
    cost = {k: float(cum[-1]) * w for k, w in width.items()}
    mean = sum(cost.values()) / world
    load = [0.0] * world
    pieces: Dict = {}
    for k in sorted(cost, key=lambda x: (-cost[x], x)):
        npieces = 1
        if world > 1 and cost[k] > split_factor * mean:
            npieces = min(world, max(2, int(math.ceil(cost[k] / mean - 1e-9))))
        cuts = [0, len(cum) - 1]
        if npieces > 1:
            bnd = aligned_boundaries(n, width[k])
            cuts = [0]
            for j in range(1, npieces):
                target = cum[-1] * j / npieces
                b = min(bnd, key=lambda t: abs(cum[t] - target))
                if cuts[-1] < b < bnd[-1]:
                    cuts.append(b)
            cuts.append(len(cum) - 1)
        used: List[int] = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            c = cost[k] * (cum[b] - cum[a]) / cum[-1]
            free = [rk for rk in range(world) if rk not in used]
            least = min(load[rk] for rk in free)
            near = [rk for rk in free if rk in consumers.get(k, []) and load[rk] <= least + 0.02 * mean]
            rk = near[0] if near else min(free, key=lambda q: (load[q], q))
            used.append(rk)
            load[rk] += c
            pieces.setdefault(k, []).append(GramPiece(rk, int(a), int(b)))
    return pieces, load


def _list_all_to_all(out: torch.Tensor, pg) -> bool:
    """RCCL takes the list form of all-to-all (device tensors, no concatenated copies)."""
    return out.is_cuda and dist.get_backend(pg) == "nccl"


def _all_to_all_rows(send_parts: List[Optional[torch.Tensor]], recv_rows: List[int], row_shape, dtype,
                     device, pg, async_op: bool = False):
    """all_to_all_single of row blocks: send_parts[j] (rows, ...) goes to rank j (None = 0
    rows); returns (work, recv (sum(recv_rows), ...)) with rank i's block at its offset."""
    world = len(recv_rows)
    empty = torch.empty((0,) + tuple(row_shape), dtype=dtype, device=device)
    parts = [pt if pt is not None else empty for pt in send_parts]
    out = torch.empty((sum(recv_rows),) + tuple(row_shape), dtype=dtype, device=device)
    if _list_all_to_all(out, pg):
        # RCCL: the list form (grouped send/recv) sends each part from where it lies and
        # receives into views of `out`: when every rank owns an RDM (distributed_rdm, configs[2])
        # each rank's rows go to all world owners without world concatenated copies of them
        outs = list(out.split([int(r) for r in recv_rows], 0))
        work = dist.all_to_all(outs, [pt.contiguous() for pt in parts], group=pg, async_op=async_op)
        return work, out, parts
    inp = torch.cat(parts, 0) if any(pt.size(0) for pt in parts) else empty
    in_splits = [int(pt.size(0)) for pt in parts]
    if inp.is_cuda:
        # gloo has no all-to-all of device tensors: only the one-GPU rehearsal of the multi-rank
        # path takes this (scripts/gpu_rehearse.sh); RCCL moves device memory directly
        host = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(host, inp.cpu(), output_split_sizes=list(recv_rows), input_split_sizes=in_splits,
                               group=pg)
        out.copy_(host)
        return _Done(), out, inp
    work = dist.all_to_all_single(out, inp, output_split_sizes=list(recv_rows), input_split_sizes=in_splits,
                                  group=pg, async_op=async_op)  # gloo, host tensors (CPU tests)
    return work, out, inp


class _Done:
    def wait(self):
        return True


class ShardedRDMs:
    """The step's RDMs over stimulus-sharded rows (RdmSchedule):

      start()   issues the row exchanges: every rank sends its rows of each RDM to that
                RDM's owner(s) (all_to_all_single on exchange_pg; at most `window` RDMs'
                rows in flight per rank, the rest issued as Grams complete);
      finish()  each owner computes its pieces from the full rows (tiles bit-identical to the
                one-GPU launch), the packed pieces go to the consumers that lack them
                (all_to_all_single), and each consumer unpacks only the RDMs its units read.
    Returns {name: (n, n) RDM} for this rank's names. One rank: every RDM is one launch."""

    def __init__(self, sched: RdmSchedule, rows: Dict[Tuple[str, str], torch.Tensor], pg=None,
                 times: Optional[StepTimes] = None, kernels: RdmKernels = None, exchange_pg=None,
                 window: int = 4, correction: float = 1e-12):
        self.sched, self.rows, self.pg, self.times = sched, rows, pg, times
        self.kernels = kernels or KERNELS
        self.exchange_pg = exchange_pg if exchange_pg is not None else pg
        self.window, self.correction = max(1, int(window)), correction
        self.rank, self.world = _world(pg)
        # exchange order: widest RDM first, so the big owners start first
        self.order = sorted(sched.pieces, key=lambda k: (-int(rows[k].size(1)), k))
        self.pending: Dict[Tuple[str, str], Callable[[], Optional[torch.Tensor]]] = {}
        self._next = 0

    def _issue(self) -> None:
        k = self.order[self._next]
        self._next += 1
        n, world = self.sched.n, self.world
        owners = self.sched.owners(k)
        sizes = [len(shard_rows(n, r, world)) for r in range(world)]
        recv = sizes if self.rank in owners else [0] * world
        src = self.rows[k]
        if isinstance(src, SplitRows):
            # plane records travel as 8-byte words (no 16-bit integer type in RCCL or gloo),
            # the row statistics as (rows, 2) floats; the owner's planes buffer is padded to
            # the super-tile edge with zero rows, as the kernels read it
            K = self.kernels
            pl = src.planes[:src.rows].view(torch.int64)
            stats = torch.stack([src.mean, src.std], dim=1)
            w1, pfull, k1 = _all_to_all_rows([pl if r in owners else None for r in range(world)], recv,
                                             pl.shape[1:], pl.dtype, pl.device, self.exchange_pg, async_op=True)
            w2, sfull, k2 = _all_to_all_rows([stats if r in owners else None for r in range(world)], recv,
                                             stats.shape[1:], stats.dtype, stats.device, self.exchange_pg,
                                             async_op=True)

            def done_split(_keep=(k1, k2)):
                w1.wait()
                w2.wait()
                if self.rank not in owners:
                    return None
                out = K.empty_split(n, src.d, pfull.device)
                out.planes[:n].view(torch.int64).copy_(pfull)
                out.mean.copy_(sfull[:, 0])
                out.std.copy_(sfull[:, 1])
                return out

            self.pending[k] = done_split
            return
        x = src.float().contiguous()
        send = [x if r in owners else None for r in range(world)]
        work, full, keep = _all_to_all_rows(send, recv, x.shape[1:], x.dtype, x.device, self.exchange_pg,
                                            async_op=True)

        def done(_keep=keep):
            work.wait()
            return full if self.rank in owners else None

        self.pending[k] = done

    def _tiles(self, src, out: torch.Tensor, t0: int, t1: int) -> None:
        if isinstance(src, SplitRows):
            self.kernels.tiles_from_planes(src, self.sched.n, out, t0, t1, self.correction, self.times)
        else:
            self.kernels.tiles_from_rows(src.float().contiguous(), out, t0, t1, self.correction, self.times)

    def start(self) -> None:
        if self.world > 1:
            while self._next < len(self.order) and len(self.pending) < self.window:
                self._issue()

    def finish(self, on_ready: Optional[Callable[[Tuple[str, str], torch.Tensor], None]] = None
               ) -> Dict[Tuple[str, str], torch.Tensor]:
        """on_ready(name, rdm), if given, is called for each of this rank's RDMs as soon as its
        kernels are enqueued on the current stream (PlanPrefetch starts its rank plan on a
        second stream there, under the following Grams)."""
        n, K, rank = self.sched.n, self.kernels, self.rank
        mine = set(self.sched.needs(rank))
        if self.world == 1:
            out = {}
            for k in self.order:
                out[k] = o = torch.empty((n, n), dtype=torch.float32, device=self.rows[k].device)
                self._tiles(self.rows[k], o, 0, int(lib().vr_rdm_tile_count(n)))
                if on_ready is not None:
                    on_ready(k, o)
            return out
        self.start()
        dev = next(iter(self.rows.values())).device
        bufs: Dict[Tuple[str, str], torch.Tensor] = {}
        # 1. every owned piece, in exchange order (rows of later RDMs arriving meanwhile)
        for k in self.order:
            while k not in self.pending:
                self._issue()
            full = self.pending.pop(k)()
            if self._next < len(self.order):
                self._issue()  # keep the window full
            mine_pieces = [pc for pc in self.sched.pieces[k] if pc.owner == rank]
            if not mine_pieces:
                continue
            o = bufs.setdefault(k, torch.empty((n, n), dtype=torch.float32, device=dev))
            for pc in mine_pieces:
                self._tiles(full, o, pc.t0, pc.t1)
            del full
        # 2. packed pieces to the consumers that lack them; unpack only what this rank reads
        out = {}
        for k in self.order:
            pcs = self.sched.pieces[k]
            cons = self.sched.consumers[k]
            send: List[Optional[torch.Tensor]] = [None] * self.world
            recv = [0] * self.world
            others = [c for c in cons if c != rank]
            for pc in pcs:
                if pc.owner == rank and others:
                    packed = torch.empty((pc.t1 - pc.t0, TILE * TILE), dtype=torch.float32, device=dev)
                    K.pack(bufs[k], n, pc.t0, pc.t1, packed)
                    for c in others:
                        send[c] = packed if send[c] is None else torch.cat([send[c], packed], 0)
                if rank in cons and pc.owner != rank:
                    recv[pc.owner] += pc.t1 - pc.t0
            # every rank joins every exchanged RDM's collective (same order everywhere); an RDM
            # whose consumers all own every piece of it moves nothing, and every rank sees that
            # from the schedule alone, so all of them skip its collective
            got = None
            if any(c != pc.owner for pc in pcs for c in cons):
                _, got, _ = _all_to_all_rows(send, recv, (TILE * TILE,), torch.float32, dev, self.pg)
            if k in mine:
                o = bufs.pop(k, None)
                if o is None:
                    o = torch.empty((n, n), dtype=torch.float32, device=dev)
                at = 0
                for pc in sorted(pcs, key=lambda q: (q.owner, q.t0)):
                    if pc.owner != rank:
                        K.unpack(got[at: at + pc.t1 - pc.t0], n, pc.t0, pc.t1, o)
                        at += pc.t1 - pc.t0
                out[k] = o
                if on_ready is not None:
                    on_ready(k, o)
            else:
                bufs.pop(k, None)
        return out


class PlanPrefetch:
    """Rank plans built on a second stream as the RDMs come out of the Grams.

    A plan build (triangle keys, radix sort, tie groups, maps: HBM-bound, ~4.5 ms at
    N = 10k) waits only for its RDM's kernels (an event on the producing stream) and then
    runs beside the next RDM's Gram (MFMA-bound) instead of after all of them. `plans()`
    makes the current stream wait for every build and returns {name: RankPlan}.
    Stream hand-offs: each RDM is recorded as used on the plan stream, each plan buffer as
    used on the consuming stream, so the caching allocator reuses neither early."""

    def __init__(self, device, names=None, stream: Optional[torch.cuda.Stream] = None):
        self.device = device
        self.names = None if names is None else set(names)
        self.stream = stream if stream is not None else torch.cuda.Stream(device=device)
        self._plans: Dict[Tuple[str, str], R.RankPlan] = {}

    def __call__(self, name, rdm: torch.Tensor) -> None:
        if self.names is not None and name not in self.names:
            return
        main = torch.cuda.current_stream(self.device)
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ready)
            plan = R.RankPlan(rdm, ws_tag="plan_prefetch")
        rdm.record_stream(self.stream)
        plan.buf.record_stream(main)
        self._plans[name] = plan

    def plans(self) -> Dict[Tuple[str, str], R.RankPlan]:
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        return self._plans


def distributed_rdm(x_local: torch.Tensor, n: int, pg=None, times: Optional[StepTimes] = None,
                    kernels: RdmKernels = None) -> torch.Tensor:
    """Full (n, n) RDM on every rank from each rank's stimulus rows: one RDM scheduled as a
    region every rank consumes (ShardedRDMs). One GPU: the single-launch RDM."""
    rank, world = _world(pg)
    if world == 1:
        x = x_local.float().contiguous()
        out = torch.empty((n, n), dtype=torch.float32, device=x.device)
        (kernels or KERNELS).tiles_from_rows(x, out, 0, int(lib().vr_rdm_tile_count(n)), 1e-12, times)
        return out
    name = ("n", "x")
    cons = {name: list(range(world))}
    pieces, load = assign_grams(n, {name: int(x_local.size(1))}, cons, world)
    sched = RdmSchedule(world, n, [], [(0, 0)] * world, cons, pieces, load)
    return ShardedRDMs(sched, {name: x_local}, pg, times, kernels).finish()[name]


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
# A side streams its codes twice (count pre-pass + rank walk); the B walk streams its codes
# and the A positions and computes the window low ends from them (VISREPS_ENGINE_LO_JOIN=1:
# the join also writes the low ends -- 4 B more per pair there -- which the prefetching EST 3/4
# walk does not read); k_join reads the B codes, gathers the 4-B A position map and writes
# the A positions, per unit.
def engine_tri(n: int, est: Optional[bool] = None) -> bool:
    """Whether the bootstrap calls at n stimuli run the triangle-order EST passes (EST 5/6:
    M <= 2^28, EST 3 estimate, opt-in VISREPS_ENGINE_TRI=1; engine.hip run_engine_multi_impl)."""
    import os

    if est is None:
        est = os.environ.get("VISREPS_ENGINE_EST") != "0"
    return (est and os.environ.get("VISREPS_ENGINE_TRI", "0") != "0"
            and os.environ.get("VISREPS_ENGINE_EST_MODE", "3") == "3" and n * (n - 1) // 2 <= (1 << 28))


def engine_pair_bytes(est: Optional[bool] = None, tri: bool = False) -> Tuple[int, int, int]:
    """(A walk per pass, B walk per pass and unit, join per unit) bytes per pair."""
    import os

    if est is None:
        est = os.environ.get("VISREPS_ENGINE_EST") != "0"
    if est and tri:
        # triangle-order TB: A: codes 4 (count pre-pass) + codes 4 + TB row write 128 (at the
        # pair's triangle index); B: codes 4 + TB row gather 128; no join
        return 4 + 4 + 128, 4 + 128, 0
    if not est:
        # A: codes 4 + TB row write 128; B: codes, posA, chunkA 4 each + TB row 128;
        # join: B codes 4 + 8-B pair-map record + posA and chunkA writes 4 each
        return 4 + 128, 4 + 4 + 4 + 128, 4 + 8 + 4 + 4
    lo = 4 if os.environ.get("VISREPS_ENGINE_LO_JOIN", "0") != "0" else 0
    # A: codes 4 (count pre-pass) + codes 4 + TB row write 128; B: codes 4 + posA 4
    # (+ low end) + TB row gather 128; join: B codes 4 + position-map gather 4 + posA write 4
    # (+ low-end write)
    return 4 + 4 + 128, 4 + 4 + lo + 128, 4 + 4 + 4 + lo


def engine_call_bytes(n: int, subsets: int, units: int, joined: bool = False) -> float:
    """Algorithmic HBM bytes of one engine call: `units` B plans against one A plan over
    `subsets` subsets (64 per pass; 63 in the triangle-order form); joined: the units' joins
    were done beforehand (SharedJoins, counted by shared_join_bytes)."""
    tri = engine_tri(n)
    a, b, j = engine_pair_bytes(tri=tri)
    if joined:
        j = 0
    M = n * (n - 1) // 2
    passes = -(-subsets // (63 if tri else 64))
    # + the full-set pass's lane-0 shift sums (k_full_corr: the A positions again, 4 B per pair
    # and unit; csrc/engine.hip est4_shift)
    return float(M) * (passes * (a + units * b) + units * j + (0 if tri else 4 * units))


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


def engine_grid_bytes(n: int, subsets: int, regions: int, units_per_region: int) -> float:
    """Algorithmic HBM bytes of one grid call (bootstrap_spearman_grid, every unit joined):
    per region its A side as engine_call_bytes; per pass and B plan one walk for all regions,
    the B codes once (4 B per pair) and per region the A position (4) and the TB row (128)."""
    tri = engine_tri(n)
    if tri:  # (the grid form has no triangle-order variant: the per-region calls)
        return regions * engine_call_bytes(n, subsets, units_per_region, joined=True)
    a, b, _ = engine_pair_bytes(tri=False)
    M = n * (n - 1) // 2
    passes = -(-subsets // 64)
    walk = 4 + regions * (b - 4)  # codes once, then per region A position + TB row
    return float(M) * (passes * (regions * a + units_per_region * walk) + 4 * regions * units_per_region)


def run_grid(plans_n: Sequence[R.RankPlan], plans_m: Sequence[R.RankPlan], idx: Optional[np.ndarray],
             joined: Sequence[Sequence[torch.Tensor]], times: Optional[StepTimes] = None) -> torch.Tensor:
    """Units (m, n) for every model plan m against every neural plan n (<= 4 regions) in one
    engine call: (len(plans_n), len(plans_m), 1 + n_boot) scores, each model plan walked once
    per pass for all regions (bootstrap_spearman_grid). joined[m][r] from SharedJoins."""
    ev = None
    if times is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    scores = R.bootstrap_spearman_grid(plans_n, plans_m, idx, joined, full_first=True)
    if times is not None:
        ev[1].record()
        nb = 0 if idx is None else len(idx)
        units = len(plans_n) * len(plans_m)
        times.record("engine", ev[0], ev[1], engine_grid_bytes(plans_n[0].n, nb + 1, len(plans_n), len(plans_m)),
                     calls=units, ref=engine_bytes(plans_n[0].n, nb) * units)
    return scores


def shared_join_bytes(n: int, n_a: int, n_b: int) -> float:
    """Algorithmic bytes of SharedJoins over n_a A plans and n_b B plans: the interleave
    (4 B read per A plan, 16 B written per pair) and per B plan its codes 4 + the 16-B record
    gather + 4 B written per A plan."""
    M = n * (n - 1) // 2
    return float(M) * (4 * n_a + 16 + n_b * (4 + 16 + 4 * n_a))


def run_group(plan_n: R.RankPlan, plans_m: Sequence[R.RankPlan], idx: Optional[np.ndarray],
              times: Optional[StepTimes] = None, joined: Optional[Sequence[torch.Tensor]] = None) -> torch.Tensor:
    """Units (m, n) for every model plan m against one neural plan n in one engine call:
    (len(plans_m), 1 + n_boot) scores; the neural plan's rank walk is shared. joined: the
    units' A positions from SharedJoins."""
    ev = None
    if times is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    if joined is None:
        scores = R.bootstrap_spearman_multi(plan_n, plans_m, idx, full_first=True)
    else:
        scores = R.bootstrap_spearman_multi(plan_n, plans_m, idx, full_first=True, joined=joined)
    if times is not None:
        ev[1].record()
        nb = 0 if idx is None else len(idx)
        times.record("engine", ev[0], ev[1], engine_call_bytes(plan_n.n, nb + 1, len(plans_m), joined is not None),
                     calls=len(plans_m), ref=engine_bytes(plan_n.n, nb) * len(plans_m))
    return scores


def shared_joins(pns: Dict[str, R.RankPlan], by_region: Dict[str, List[str]], mplans: Dict[str, R.RankPlan],
                 times: Optional[StepTimes] = None) -> Dict[Tuple[str, str], torch.Tensor]:
    """A positions of every (point, region) unit, regions in groups of up to 4 sharing one
    16-B gather per model pair (SharedJoins): {(p, r): int32 (M,)}. A group's record table
    exists only while its model joins run."""
    out: Dict[Tuple[str, str], torch.Tensor] = {}
    regions = list(by_region)
    for g0 in range(0, len(regions), 4):
        grp = regions[g0:g0 + 4]
        ev = None
        if times is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        sj = R.SharedJoins([pns[r] for r in grp])
        pts = sorted({p for r in grp for p in by_region[r]}, key=lambda p: list(mplans).index(p))
        for p in pts:
            outs = sj.join(mplans[p])
            for r, t in zip(grp, outs):
                if p in by_region[r]:
                    out[(p, r)] = t
        del sj
        if times is not None:
            ev[1].record()
            times.record("engine", ev[0], ev[1], shared_join_bytes(pns[grp[0]].n, len(grp), len(pts)), calls=0)
    return out


def unit_split(units: Sequence, world: int) -> List[Tuple[int, int]]:
    """Contiguous, near-equal [lo, hi) ranges of the unit list, one per rank."""
    u = len(units)
    b = [round(r * u / world) for r in range(world + 1)]
    return [(b[r], b[r + 1]) for r in range(world)]


def phase1_rows(n: int, n_select: Optional[int], seed: int, rank: int, world: int):
    """The phase-1 selection of evals.py:259-263 seen from one rank: (k, positions in the
    selection list held by this rank, their local row indices in the rank's shard)."""
    rows = shard_rows(n, rank, world)
    k = min(int(n_select), n) if n_select is not None else n
    sel = (LegacyRandomState(seed).choice(n, k, replace=False) if k < n else np.arange(n))
    mine = np.flatnonzero((sel >= rows.start) & (sel < rows.stop))
    return k, mine, sel[mine] - rows.start


def phase1_select(feats: Dict[str, torch.Tensor], projectors: Dict, responses: Dict[str, torch.Tensor],
                  points: Sequence[str], n: int, *, n_select: int = 1000, seed: int = 42,
                  pg=None, times: Optional[StepTimes] = None,
                  selected_rows: Optional[Dict[str, torch.Tensor]] = None,
                  kernels: Optional[RdmKernels] = None) -> Dict[str, Tuple[str, List[Dict]]]:
    """Phase-1 layer selection of the reference eval (evals.py:249-287) on stimulus-sharded
    features. RandomState(seed).choice(n, n_select) picks the selection stimuli (re-created
    per (region, subject); the regions share one subject's stimuli, so one draw serves them
    all); each rank projects its selected rows of every point by the point's SRP matrix (the
    bulk extraction's torch.sparse.mm, models/utils.py:297-344, here vr_srp_csr_f32). The
    projection is row by row, so projecting the selected rows equals projecting every row
    and selecting after, as the reference does: phase 1 reads no other projected row
    (evals.py:254-268) and phase 2 re-extracts.

    Over ranks the points are dealt round-robin: point i's projected rows are summed (the
    ranks' rows are disjoint: exact) onto rank i mod world only, which builds its selection
    RDM and plan and scores it against every region; the regions' selection RDMs (small) are
    built on every rank; the (point, region) scores are all-gathered. Scores do not depend
    on the world size (exact sums, exact-integer Spearman). Best = first strict maximum.
    selected_rows[p] (optional) holds this rank's selected rows of point p in phase1_rows
    order, kept during extraction instead of all of feats[p]. kernels: the RDM entry points
    (RdmKernels; a CPU emulation in the gloo tests). Returns {region: (best point,
    [{"layer", "score"} per point])} on every rank."""
    rank, world = _world(pg)
    K = kernels or KERNELS
    k, mine, src = phase1_rows(n, n_select, seed, rank, world)
    dev = next(iter(responses.values())).device
    pos_t = torch.as_tensor(mine, dtype=torch.long, device=dev)
    src_t = torch.as_tensor(src, dtype=torch.long, device=dev)
    owner = {p: i % world for i, p in enumerate(points)}

    def selected(x_mine: torch.Tensor, dst: Optional[int]) -> torch.Tensor:
        """this rank's selected rows -> (k, d) on rank dst (None: on every rank)"""
        out = torch.zeros((k, x_mine.size(1)), dtype=torch.float32, device=dev)
        out[pos_t] = x_mine.float()
        if world > 1:  # disjoint rows: the sum is exact
            if dst is None or (out.is_cuda and dist.get_backend(pg) != "nccl"):
                # (gloo reduces no device tensors: the one-GPU rehearsal sums on every rank)
                dist.all_reduce(out, op=dist.ReduceOp.SUM, group=pg)
            else:
                g = dst if pg is None or pg == dist.group.WORLD else dist.get_global_rank(pg, dst)
                dist.reduce(out, dst=g, op=dist.ReduceOp.SUM, group=pg)
        return out

    def timed_rdm(x: torch.Tensor) -> torch.Tensor:
        out = torch.empty((x.size(0), x.size(0)), dtype=torch.float32, device=dev)
        K.tiles_from_rows(x, out, 0, int(lib().vr_rdm_tile_count(x.size(0))), 1e-12, times)
        return out

    mplans = {}
    for p in points:
        rows_p = selected_rows[p] if selected_rows is not None else feats[p][src_t]
        proj = projectors[p](rows_p)  # SRP of this rank's selected stimuli
        full = selected(proj, owner[p])
        if owner[p] == rank:
            mplans[p] = R.RankPlan(timed_rdm(full))
        del proj, full
    mine_pts = [p for p in points if p in mplans]
    scores: Dict[Tuple[str, str], float] = {}
    for r, y in responses.items():
        pn = R.RankPlan(timed_rdm(selected(y[src_t], None)))
        if mine_pts:
            sc = torch.as_tensor(R.bootstrap_spearman_multi(pn, [mplans[p] for p in mine_pts], None,
                                                            full_first=True))[:, 0].cpu().numpy()
            for p, v in zip(mine_pts, sc):
                scores[(p, r)] = float(v)
    if world > 1:
        gathered: List[Dict] = [None] * world
        dist.all_gather_object(gathered, scores, group=pg)
        scores = {}
        for g in gathered:
            scores.update(g)
    out = {}
    for r in responses:
        best, best_score, lst = None, -float("inf"), []
        for p in points:
            v = scores[(p, r)]
            lst.append({"layer": p, "score": v})
            if v > best_score:  # strict: the first maximal point wins (evals.py:273-275)
                best, best_score = p, v
        out[r] = (best, lst)
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


def _engine_ws_fits(dev: torch.device, nbytes: int) -> bool:
    """An engine workspace of nbytes fits the device: free memory + torch's cached blocks +
    the pool's current engine buffer (which the new one replaces), with 10 % headroom."""
    if dev.type != "cuda":
        return True
    free = torch.cuda.mem_get_info(dev)[0]
    cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    cur = workspace.current(dev, "engine")
    return nbytes <= 0.9 * (free + cached + cur)


def all_units_rsa(model_rdm_fn: Callable[[str], torch.Tensor], points: Sequence[str],
                  neural_rdms: Dict[str, torch.Tensor], n: int, *, n_boot: int = 1000,
                  seed: int = 42, pg=None, times: Optional[StepTimes] = None,
                  keep_plans: bool = False, plan_fn=None, unit_fn=None, group_fn=None,
                  regions: Optional[Sequence[str]] = None,
                  plans: Optional[Dict[Tuple[str, str], R.RankPlan]] = None,
                  indices: Optional[Callable[[], np.ndarray]] = None) -> Dict[Tuple[str, str], Dict]:
    """Point + bootstrap Spearman RSA for every (point, region) unit; returns the
    per-unit results on every rank.

    Units are listed region-major and cut into one contiguous range per rank (the
    RdmSchedule's unit_ranges), so a rank's units come in groups that share a neural RDM;
    each group is one engine call (run_group: the neural plan's rank walk is shared by the
    group's layers). model_rdm_fn(p) is asked only for the points of this rank's units, and
    neural_rdms needs only this rank's regions (`regions` lists all of them; default: the
    keys of neural_rdms). plan_fn / group_fn default to RankPlan / run_group (the HIP
    engine); a per-unit unit_fn(model plan, neural plan, idx, times) may be given instead.
    plans: prebuilt rank plans by RDM name (("m", point), ("n", region); PlanPrefetch); the
    others are built here."""
    plan_fn = plan_fn or R.RankPlan
    if group_fn is None:
        if unit_fn is not None:
            def group_fn(pn, pms, idx_, t):
                return [np.asarray(torch.as_tensor(unit_fn(pm, pn, idx_, t)).cpu()) for pm in pms]
        else:
            group_fn = run_group
    rank, world = _world(pg)
    regions = list(regions) if regions is not None else list(neural_rdms)
    units = [(p, r) for r in regions for p in points]
    lo, hi = unit_split(units, world)[rank]
    mine = units[lo:hi]
    k = int(0.9 * n)
    idx = None
    if n_boot > 0 and mine:
        # RandomState(seed) is re-created per (region, subject) (evals.py:356), so every unit
        # draws the same (n_boot, k) index sets: drawn once per call (host MT19937), one upload
        # indices(): the same draw started earlier by the caller (bench.py draws on a host
        # thread from the start of the step, so the ~0.2 s of MT19937 overlaps GPU work
        # even when a rank's queue is short, as at 8 GPUs)
        dev = neural_rdms[mine[0][1]].device
        drawn = indices() if indices is not None else draw_bootstrap_indices(seed, n, k, n_boot)
        if drawn.shape != (n_boot, k):
            raise ValueError(f"indices() gave {drawn.shape}, expected {(n_boot, k)}")
        idx = torch.from_numpy(drawn).to(dev)
    local: Dict[Tuple[str, str], np.ndarray] = {}
    need = {p for p, _ in mine}
    mplans = {}
    plans = plans or {}
    for p in points:
        if p in need:
            mplans[p] = plans[("m", p)] if ("m", p) in plans else plan_fn(model_rdm_fn(p))
    by_region: Dict[str, List[str]] = {}
    for p, r in mine:
        by_region.setdefault(r, []).append(p)
    # Shared joins (the default engine, >= 2 regions on this rank, VISREPS_SHARED_JOINS not 0,
    # and the join arrays -- 4 B per pair and unit -- within a quarter of the free memory):
    # every model pair gathers its positions in up to 4 neural plans at once
    joined = None
    if (group_fn is run_group and plan_fn is R.RankPlan and len(by_region) >= 2 and n_boot > 0
            and os.environ.get("VISREPS_SHARED_JOINS", "1") != "0"):
        dev = neural_rdms[mine[0][1]].device
        # the join arrays (4 B per pair and unit, + the 16-B record table) and the neural
        # plans built here, which all stay alive until their region's call is done
        built = sum(1 for r in by_region if ("n", r) not in plans)
        need = 4.0 * (n * (n - 1) // 2) * (len(mine) + 4) + built * float(lib().vr_rank_plan_bytes(n))
        if dev.type == "cuda" and need <= 0.25 * torch.cuda.mem_get_info(dev)[0]:
            pns = {r: (plans[("n", r)] if ("n", r) in plans else plan_fn(neural_rdms[r])) for r in by_region}
            joined = shared_joins(pns, by_region, mplans, times)
    # Regions sharing their point list (all of them on one GPU) run in groups of up to 4 as
    # one grid call each: every model plan walked once per pass for the group's regions. A
    # group whose grid workspace (region 0's full engine workspace + a slim one per further
    # region) does not fit the free device memory runs as per-region calls.
    ran_grid = False
    if joined is not None and os.environ.get("VISREPS_ENGINE_GRID", "1") != "0":
        groups = []
        for r in by_region:
            same = [g for g in groups if by_region[g[0]] == by_region[r] and len(g) < 4]
            if same:
                same[0].append(r)
            else:
                groups.append([r])
        for grp in [g for g in groups if len(g) >= 2]:
            pts = by_region[grp[0]]
            if not _engine_ws_fits(dev, int(lib().vr_bootstrap_grid_joined_workspace(n, len(grp), len(pts)))):
                continue
            ran_grid = True
            pg_n = [plans[("n", r)] if ("n", r) in plans else pns.pop(r) for r in grp]
            out = run_grid(pg_n, [mplans[p] for p in pts], idx,
                           [[joined.pop((p, r)) for r in grp] for p in pts], times)
            for i, r in enumerate(grp):
                for j, p in enumerate(pts):
                    local[(p, r)] = np.asarray(out[i, j].cpu())
                del by_region[r]
            del pg_n, out
    for r, pts in by_region.items():
        pn = plans[("n", r)] if ("n", r) in plans else (pns.pop(r) if joined is not None else plan_fn(neural_rdms[r]))
        if joined is not None:
            out = group_fn(pn, [mplans[p] for p in pts], idx, times, joined=[joined.pop((p, r)) for p in pts])
        else:
            out = group_fn(pn, [mplans[p] for p in pts], idx, times)
        for j, p in enumerate(pts):
            local[(p, r)] = np.asarray(torch.as_tensor(out[j]).cpu())
        del pn  # the last reference to a plan built here: freed before the next region's call
    del mplans
    if ran_grid:  # the pool's grow-only engine buffer goes back to torch's cache
        workspace.release("engine")
    if world > 1:
        gathered: List[Dict] = [None] * world
        dist.all_gather_object(gathered, local, group=pg)
        merged = {}
        for g in gathered:
            merged.update(g)
        local = merged
    return {u: summarize(local[u], n_boot > 0) for u in units}
