"""Full-triangle Spearman of RDMs whose pairs are spread over ranks: a global average rank
by sample sort (the reference's compute_rdm_correlation "Spearman",
rsa.py:111-122, over a triangle no single device holds).

On MI355X one GPU holds configs[2]'s 73k RDM pair and spearman_full's workspace (about
120 GB of 288), so the eval path ranks on one device; this module is the path for RDMs
whose triangle is built distributed and not gathered (the block-distributed Gram's tile
ranges), or larger than one device's memory.

Per RDM, every rank holds an arbitrary subset of the M pairs: (fp32 value, triangle index t).
  1. local   sortable keys, local (key, t) radix sort            vr_f32_sort_keys, vr_sort_pairs_u32
  2. split   32 * world regular samples of every rank's sorted keys, all-gathered; world - 1
             splitters; a key's bucket is a function of the key alone, so a tie group never
             straddles two buckets
  3. a2a     bucket b of every rank -> rank b (all_to_all_single, uneven splits)
  4. rank    local radix sort of the bucket; global offset = pairs in lower buckets; doubled
             midranks 2 offset + gs + ge + 1 and the bucket's tie term      vr_midranks_sorted
  5. a2a     (t, y) -> the rank owning t (ranges [M r // W, M (r+1) // W))
Then sum yA yB over each rank's t range (vr_dot_u64), and the u128 sums and tie terms are
all-reduced as 16-bit limbs (exact in int64 for any world size), and rho follows the
engine's exact formula. Results equal spearman_full / the rank-plan engine bit for bit.

The default count-table form (global_midranks_tables, spearman_full's idea) replaces steps
1-4: the global key range by all-reduce, each rank's per-key counts (vr_key_counts_u32)
summed by one all-reduce, then every rank's doubled midranks and the tie term from the
summed table (vr_key_table_midranks) -- no sort and no key exchange; step 5 routes (t, y)
as before.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .._lib import check, lib, stream_of, workspace

__all__ = ["RankKernels", "distributed_spearman", "global_midranks", "global_midranks_tables"]


def _u32(x: torch.Tensor) -> torch.Tensor:
    """int32 storage of u32 values as int64 numbers (for host-side arithmetic)."""
    return x.to(torch.int64) & 0xFFFFFFFF


class RankKernels:
    """The device pieces (csrc/spearman_full.hip); the gloo tests substitute numpy."""

    @staticmethod
    def keys(values: torch.Tensor) -> torch.Tensor:
        out = torch.empty(values.numel(), dtype=torch.int32, device=values.device)
        if values.numel():
            check(lib().vr_f32_sort_keys(values.data_ptr(), values.numel(), out.data_ptr(),
                                         stream_of(values.device)), "vr_f32_sort_keys")
        return out

    @staticmethod
    def sort(keys: torch.Tensor, vals: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        keys, vals = keys.clone(), vals.clone()
        m = keys.numel()
        if m > 1:
            L = lib()
            ws = workspace.get(keys.device, L.vr_sort_pairs_workspace(m), "dist_sort")
            check(L.vr_sort_pairs_u32(keys.data_ptr(), vals.data_ptr(), m, ws.data_ptr(), ws.numel(),
                                      stream_of(keys.device)), "vr_sort_pairs_u32")
        return keys, vals

    @staticmethod
    def midranks(keys_sorted: torch.Tensor, base: int) -> Tuple[torch.Tensor, int]:
        m = keys_sorted.numel()
        dev = keys_sorted.device
        y = torch.empty(m, dtype=torch.int64, device=dev)
        tie = torch.zeros(2, dtype=torch.int64, device=dev)
        L = lib()
        ws = workspace.get(dev, L.vr_midranks_workspace(m), "dist_midranks")
        check(L.vr_midranks_sorted(keys_sorted.data_ptr(), m, int(base), y.data_ptr(), tie.data_ptr(),
                                   ws.data_ptr(), ws.numel(), stream_of(dev)), "vr_midranks_sorted")
        lo, hi = (int(v) & 0xFFFFFFFFFFFFFFFF for v in tie.cpu().tolist())
        return y, lo | (hi << 64)

    @staticmethod
    def counts(keys: torch.Tensor, kmin: int, bins: int) -> torch.Tensor:
        """Per-key counts of keys in [kmin, kmin + bins) as int64[bins + 1] (last entry 0)."""
        dev = keys.device
        cnt = torch.zeros(bins + 1, dtype=torch.int32, device=dev)
        check(lib().vr_key_counts_u32(keys.data_ptr(), keys.numel(), int(kmin), int(bins), cnt.data_ptr(),
                                      stream_of(dev)), "vr_key_counts_u32")
        return cnt.to(torch.int64) & 0xFFFFFFFF

    @staticmethod
    def table_midranks(keys: torch.Tensor, kmin: int, counts: torch.Tensor) -> Tuple[torch.Tensor, int]:
        """Doubled midranks of keys from the global per-key counts, and the tie term."""
        dev = keys.device
        bins = counts.numel() - 1
        cnt = counts.to(torch.int32).contiguous()  # < 2^32 each: the u32 bit pattern
        y = torch.empty(keys.numel(), dtype=torch.int64, device=dev)
        tie = torch.zeros(2, dtype=torch.int64, device=dev)
        L = lib()
        ws = workspace.get(dev, L.vr_key_table_workspace(bins), "dist_table")
        check(L.vr_key_table_midranks(keys.data_ptr(), keys.numel(), int(kmin), cnt.data_ptr(), bins, y.data_ptr(),
                                      tie.data_ptr(), ws.data_ptr(), ws.numel(), stream_of(dev)),
              "vr_key_table_midranks")
        lo, hi = (int(v) & 0xFFFFFFFFFFFFFFFF for v in tie.cpu().tolist())
        return y, lo | (hi << 64)

    @staticmethod
    def dot(a: torch.Tensor, b: torch.Tensor) -> int:
        out = torch.zeros(2, dtype=torch.int64, device=a.device)
        L = lib()
        ws = workspace.get(a.device, L.vr_dot_u64_workspace(), "dist_dot")
        check(L.vr_dot_u64(a.data_ptr(), b.data_ptr(), a.numel(), out.data_ptr(), ws.data_ptr(),
                           ws.numel(), stream_of(a.device)), "vr_dot_u64")
        lo, hi = (int(v) & 0xFFFFFFFFFFFFFFFF for v in out.cpu().tolist())
        return lo | (hi << 64)


KERNELS = RankKernels()


def _world(pg):
    if pg is None or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(pg), dist.get_world_size(pg)


def _a2a(x: torch.Tensor, send_counts, pg) -> torch.Tensor:
    """all_to_all_single with uneven splits (counts in elements of x's first dimension)."""
    rank, world = _world(pg)
    if world == 1:
        return x
    sc = torch.tensor(send_counts, dtype=torch.int64, device=x.device)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=pg)
    recv = rc.cpu().tolist()
    out = torch.empty((sum(recv),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_to_all_single(out, x.contiguous(), recv, list(send_counts), group=pg)
    return out


def _allreduce_int(v: int, dev, pg) -> int:
    """Exact sum over ranks of a non-negative integer < 2^192 (12 limbs of 16 bits)."""
    rank, world = _world(pg)
    if world == 1:
        return v
    limbs = torch.tensor([(v >> (16 * i)) & 0xFFFF for i in range(12)], dtype=torch.int64, device=dev)
    dist.all_reduce(limbs, group=pg)
    return sum(int(x) << (16 * i) for i, x in enumerate(limbs.cpu().tolist()))


def global_midranks(values: torch.Tensor, tidx: torch.Tensor, M: int, pg=None,
                    kernels: RankKernels = None) -> Tuple[torch.Tensor, int]:
    """Doubled global average ranks of this rank's t range [M r / W, M (r+1) / W) (dense,
    int64) and the RDM's tie term sum (k^3 - k), from pairs (values, tidx) spread over ranks
    in any way (each pair on exactly one rank)."""
    K = kernels or KERNELS
    rank, world = _world(pg)
    dev = values.device
    keys, t = K.sort(K.keys(values.float().contiguous()), tidx.to(torch.int32).contiguous())
    ku = _u32(keys)
    # 2. splitters from regular samples of every rank's sorted keys
    s = 32 * world
    m = ku.numel()
    samp = ku[torch.linspace(0, max(m - 1, 0), s, device=dev).long()] if m else torch.zeros(0, dtype=torch.int64, device=dev)
    cnt = torch.tensor([samp.numel()], dtype=torch.int64, device=dev)
    if world > 1:
        sizes = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(sizes, cnt, group=pg)
        per = max(int(c) for c in sizes)
        buf = torch.full((per,), -1, dtype=torch.int64, device=dev)
        buf[: samp.numel()] = samp
        allb = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(allb, buf, group=pg)
        pool = torch.cat(allb)
        pool = torch.sort(pool[pool >= 0]).values
        spl = pool[torch.linspace(0, pool.numel() - 1, world + 1, device=dev).long()[1:-1]] if pool.numel() else pool
    else:
        spl = torch.zeros(0, dtype=torch.int64, device=dev)
    # 3. bucket b = number of splitters strictly below the key (a function of the key)
    bounds = torch.searchsorted(ku, spl, right=False) if spl.numel() else torch.zeros(0, dtype=torch.int64, device=dev)
    edges = [0] + [int(b) for b in bounds.cpu().tolist()] + [m]
    counts = [edges[i + 1] - edges[i] for i in range(world)]
    rk = _a2a(keys, counts, pg)
    rt = _a2a(t, counts, pg)
    # 4. bucket sort, global offset, doubled midranks
    rk, rt = K.sort(rk, rt)
    mine = torch.tensor([rk.numel()], dtype=torch.int64, device=dev)
    if world > 1:
        sizes = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(sizes, mine, group=pg)
        offset = sum(int(x) for x in sizes[:rank])
    else:
        offset = 0
    y, tie = K.midranks(rk, offset)
    tie = _allreduce_int(tie, dev, pg)
    # 5. (t, y) to the owner of t
    return _to_owners(_u32(rt), y, M, pg), tie


def _to_owners(tt: torch.Tensor, y: torch.Tensor, M: int, pg) -> torch.Tensor:
    """Route (t, y) to the rank owning t ([M r / W, M (r+1) / W)); that rank's dense y."""
    rank, world = _world(pg)
    dev = y.device
    lo = M * rank // world
    hi = M * (rank + 1) // world
    owner = ((tt + 1) * world - 1) // M  # the r with M r // W <= t < M (r + 1) // W
    order = torch.argsort(owner, stable=True)
    oc = torch.bincount(owner, minlength=world).cpu().tolist() if owner.numel() else [0] * world
    gt = _a2a(tt[order], oc, pg)
    gy = _a2a(y[order], oc, pg)
    dense = torch.empty(hi - lo, dtype=torch.int64, device=dev)
    dense[gt - lo] = gy
    return dense


# the count-table form while the key range has at most this many keys (2^27: two 1-GB int64
# tables per RDM in the all-reduce); the sample sort beyond
TABLE_CAP = 1 << 27


def global_midranks_tables(values: torch.Tensor, tidx: torch.Tensor, M: int, pg=None,
                           kernels: RankKernels = None) -> Tuple[torch.Tensor, int]:
    """global_midranks without a sort: the key range [kmin, kmax] by two all-reduces, every
    rank's per-key counts summed by one all-reduce, then each rank's doubled midranks from
    the summed table (start + end + 1 of its key's group) and the (t, y) routing of step 5.
    Falls back to the sample sort when the key range exceeds TABLE_CAP (e.g. values far
    outside a correlation distance's [0, 2]). NaN-free values (the caller checks)."""
    K = kernels or KERNELS
    rank, world = _world(pg)
    dev = values.device
    keys = K.keys(values.float().contiguous())
    ku = _u32(keys)
    ext = torch.tensor([int(ku.min()) if ku.numel() else 1 << 32, -int(ku.max()) if ku.numel() else 0],
                       dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(ext, op=dist.ReduceOp.MIN, group=pg)
    kmin, kmax = int(ext[0]), -int(ext[1])
    if kmax < kmin:  # no pairs anywhere
        return torch.empty(0, dtype=torch.int64, device=dev), 0
    bins = kmax - kmin + 1
    if bins > TABLE_CAP:
        return global_midranks(values, tidx, M, pg, K)
    cnt = K.counts(keys, kmin, bins)
    if world > 1:
        dist.all_reduce(cnt, group=pg)
    y, tie = K.table_midranks(keys, kmin, cnt)
    return _to_owners(_u32(tidx.to(torch.int64)), y, M, pg), tie


def distributed_spearman(a_values: torch.Tensor, a_tidx: torch.Tensor, b_values: torch.Tensor,
                         b_tidx: torch.Tensor, M: int, pg=None, kernels: RankKernels = None,
                         method: str = "tables") -> float:
    """Spearman of two triangles of M pairs, each spread over the ranks as (values, t).
    method "tables": per-key count tables summed over ranks (global_midranks_tables; the
    sample sort when a key range is too wide); "sort": the sample sort (global_midranks)."""
    if method not in ("tables", "sort"):
        raise ValueError(f"method={method!r}: tables or sort")
    K = kernels or KERNELS
    dev = a_values.device
    nan = torch.tensor([int(torch.isnan(a_values).any()) + int(torch.isnan(b_values).any())],
                       dtype=torch.int64, device=dev)
    if _world(pg)[1] > 1:
        dist.all_reduce(nan, group=pg)
    if int(nan.item()) or M < 2:  # scipy: NaN in either triangle or fewer than two pairs
        return float("nan")
    ranks = global_midranks_tables if method == "tables" else global_midranks
    ya, ta = ranks(a_values, a_tidx, M, pg, K)
    yb, tb = ranks(b_values, b_tidx, M, pg, K)
    ab = _allreduce_int(K.dot(ya, yb), dev, pg)
    mu = M * (M + 1) ** 2
    sq = 4 * (M * (M + 1) * (2 * M + 1) // 6)
    va = sq - ta // 3 - mu
    vb = sq - tb // 3 - mu
    if int(nan.item()) or M < 2 or va <= 0 or vb <= 0:
        return float("nan")
    r = _f64(ab - mu) / math.sqrt(_f64(va) * _f64(vb))
    return max(-1.0, min(1.0, r))


def _f64(x: int) -> float:
    """The device's i128 -> double conversion (hi * 2^64 + lo in double arithmetic), so
    the host statistic equals spearman_full's bit for bit."""
    neg = x < 0
    u = -x if neg else x
    d = float(u >> 64) * 18446744073709551616.0 + float(u & 0xFFFFFFFFFFFFFFFF)
    return -d if neg else d
