"""MI355X implementation of visreps.analysis.rsa (reference: visreps/analysis/rsa.py).

Same public names, argument meaning and error behaviour as the reference; the
arithmetic runs in the HIP kernels of libvisreps_hip.so:

  compute_rdm             rsa.py:59-93    fp32 MFMA Gram + fused 1-clamp(corr) epilogue
  compute_rdm_correlation rsa.py:96-129   Spearman: sorted-triangle midrank engine
                                          Kendall: tau-a by bitwise inversion counting
                                          Pearson: fp64 two-pass triangle reduction
  compute_rsa             rsa.py:132-281  layer selection + point + bootstrap on device
  bootstrap_rsa           evals.py:355-373 the inline NSD/TVSD bootstrap, batched

Tensors on a HIP device stay there; CPU tensors are copied to the current device and
results come back on the CPU (the reference's own return device). There is no CPU
fallback: without a HIP device these functions raise.
"""
from __future__ import annotations

import ctypes
import logging
import math
from typing import TYPE_CHECKING, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .._lib import check, lib, stream_of, workspace
from ..utils import rprint
from ._random import LegacyRandomState, bootstrap_indices

if TYPE_CHECKING:  # pragma: no cover
    from .alignment import AlignmentData

logger = logging.getLogger(__name__)

__all__ = [
    "compute_rdm",
    "compute_rdm_correlation",
    "compute_rsa",
    "bootstrap_rsa",
    "RankPlan",
    "bootstrap_spearman",
    "bootstrap_spearman_multi",
    "bootstrap_spearman_grid",
    "bootstrap_kendall",
    "bootstrap_full",
    "spearman_full",
    "percentile",
    "_rank",
    "_concept_average_exact",
    "_kendall_tau_a",
]

_VALID_RDM = {"pearson", "spearman"}
_VALID_CMP = {"pearson", "spearman", "kendall"}


# -----------------------------------------------------------------------------
# device helpers
# -----------------------------------------------------------------------------
def _device_for(*tensors: torch.Tensor) -> torch.device:
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            return t.device
    if not torch.cuda.is_available():
        raise RuntimeError(
            "visreps_amd needs a HIP (MI355X) device: the RSA kernels have no CPU path"
        )
    return torch.device("cuda", torch.cuda.current_device())


def _as_device_f32(x: torch.Tensor, dev: torch.device) -> torch.Tensor:
    if not isinstance(x, torch.Tensor):
        x = torch.as_tensor(np.asarray(x))
    x = x.to(device=dev, dtype=torch.float32)
    if x.ndim == 2 and x.stride(1) != 1:
        x = x.contiguous()
    if x.ndim == 2 and x.size(0) > 0 and x.stride(0) < max(x.size(1), 1):
        x = x.contiguous()
    return x


def _ptr(t: torch.Tensor) -> int:
    return int(t.data_ptr())


def _rank(x: torch.Tensor) -> torch.Tensor:
    """Row-wise ordinal rank via double argsort (rsa.py:50-52); ties are broken by
    position (stable sort), as the reference's CPU argsort does for tie-free data."""
    return torch.argsort(torch.argsort(x, dim=1, stable=True), dim=1, stable=True).float()


# -----------------------------------------------------------------------------
# RDM
# -----------------------------------------------------------------------------
def compute_rdm(
    representations: torch.Tensor, *, correlation: str = "Pearson", correction: float = 1e-12
) -> torch.Tensor:
    """(n, n) float32 RDM = 1 - Pearson correlation of the rows (rsa.py:59-93).

    Diagonal exactly 0; the matrix is exactly symmetric. correlation="Spearman" ranks
    each row first (ordinal ranks, rsa.py:77-78)."""
    corr = correlation.lower()
    if corr not in _VALID_RDM:
        raise ValueError("correlation must be 'Pearson' or 'Spearman'")
    if not isinstance(representations, torch.Tensor):
        representations = torch.as_tensor(np.asarray(representations))
    if representations.ndim != 2:
        raise ValueError("representations must be a 2-D (n_samples, n_features) tensor")
    dev = _device_for(representations)
    if (corr == "pearson" and representations.dtype == torch.bfloat16 and representations.size(0) > 0
            and representations.size(1) > 0):
        # bf16 features (ViT / CLIP, cfg5): the kernels widen them on the fly (rsa.py:76's
        # X.float()); no fp32 copy of the (n, d) features is made
        x = representations.to(dev)
        if x.stride(1) != 1 or x.stride(0) < x.size(1):
            x = x.contiguous()
        n, d = x.shape
        out = torch.empty((n, n), dtype=torch.float32, device=dev)
        L = lib()
        t = int(L.vr_rdm_tile_count(n))
        ws = workspace.get(dev, L.vr_rdm_bf16_workspace(n, d, 0, t), "rdm")
        with torch.cuda.device(dev):
            check(L.vr_rdm_pearson_bf16(_ptr(x), n, d, x.stride(0), _ptr(out), n, float(correction),
                                        _ptr(ws), ws.numel(), stream_of(dev)), "vr_rdm_pearson_bf16")
        return out if representations.is_cuda else out.cpu()
    x = _as_device_f32(representations, dev)
    if corr == "spearman":
        x = _rank(x)
    n, d = x.shape
    out = torch.empty((n, n), dtype=torch.float32, device=dev)
    if n > 0:
        if d == 0:  # mean of nothing: NaN off the diagonal, as the reference's torch path
            out.fill_(float("nan"))
            out.fill_diagonal_(0.0)
        else:
            L = lib()
            nbytes = L.vr_rdm_pearson_workspace(n, d)
            ws = workspace.get(dev, nbytes, "rdm")
            with torch.cuda.device(dev):
                check(
                    L.vr_rdm_pearson_f32(
                        _ptr(x), n, d, x.stride(0), _ptr(out), n, float(correction),
                        _ptr(ws), ws.numel(), stream_of(dev),
                    ),
                    "vr_rdm_pearson_f32",
                )
    return out if representations.is_cuda else out.cpu()


# -----------------------------------------------------------------------------
# Rank plans and the Spearman engine
# -----------------------------------------------------------------------------
class RankPlan:
    """Device-resident sorted upper triangle of one RDM (values, tie groups, chunks).

    Built once per RDM and reused by every Spearman against it: the model RDM of a
    layer serves all ROIs, a neural RDM all layers."""

    def __init__(self, rdm: torch.Tensor, ws_tag: str = "plan_build"):
        # ws_tag: the scratch of builds on another stream (pipeline.PlanPrefetch) is its own
        if rdm.ndim != 2 or rdm.size(0) != rdm.size(1):
            raise ValueError("RankPlan needs a square 2-D RDM")
        self.device = _device_for(rdm)
        r = _as_device_f32(rdm, self.device)
        self.n = int(r.size(0))
        if self.n > 65535:
            raise ValueError("rank plans (the bootstrap engine's 16-bit pair codes) support n <= "
                             "65535 stimuli; the full-triangle Spearman of a larger RDM is "
                             "compute_rdm_correlation / spearman_full")
        L = lib()
        self.buf = torch.empty(L.vr_rank_plan_bytes(self.n), dtype=torch.uint8, device=self.device)
        ws = workspace.get(self.device, L.vr_rank_plan_workspace(self.n), ws_tag)
        with torch.cuda.device(self.device):
            check(
                L.vr_rank_plan_build_f32(
                    _ptr(r), self.n, r.stride(0), _ptr(self.buf), self.buf.numel(),
                    _ptr(ws), ws.numel(), stream_of(self.device),
                ),
                "vr_rank_plan_build_f32",
            )


def bootstrap_spearman(
    plan_a: RankPlan,
    plan_b: RankPlan,
    idx: Optional[np.ndarray | torch.Tensor],
    *,
    full_first: bool = True,
) -> torch.Tensor:
    """Spearman of triu(A[s][:, s]) vs triu(B[s][:, s]) for every subset s (row of idx),
    preceded by the full set when full_first. Returns float64 scores on the device."""
    if plan_a.n != plan_b.n or plan_a.device != plan_b.device:
        raise ValueError("rank plans must describe RDMs of the same size and device")
    dev, n = plan_a.device, plan_a.n
    idx_t = _idx_tensor(idx, dev)
    n_sets, k = (int(idx_t.size(0)), int(idx_t.size(1))) if idx_t.numel() else (0, 0)
    total = n_sets + (1 if full_first else 0)
    scores = torch.empty(total, dtype=torch.float64, device=dev)
    if total == 0:
        return scores
    L = lib()
    ws = workspace.get(dev, L.vr_bootstrap_workspace(n), "engine")
    with torch.cuda.device(dev):
        check(
            L.vr_bootstrap_spearman_plans(
                _ptr(plan_a.buf), _ptr(plan_b.buf), n,
                _ptr(idx_t) if idx_t.numel() else None, k, n_sets, int(full_first),
                _ptr(scores), _ptr(ws), ws.numel(), stream_of(dev),
            ),
            "vr_bootstrap_spearman_plans",
        )
    return scores


def bootstrap_spearman_multi(
    plan_a: RankPlan,
    plans_b: Sequence[RankPlan],
    idx: Optional[np.ndarray | torch.Tensor],
    *,
    full_first: bool = True,
    joined: Optional[Sequence[torch.Tensor]] = None,
) -> torch.Tensor:
    """Spearman of every plan in plans_b against plan_a on the same subsets:
    (len(plans_b), total) float64 scores on the device. Row j equals
    bootstrap_spearman(plans_b[j], plan_a, idx) bit for bit; plan_a's rank walk runs
    once per pass of 64 subsets for all of them (a neural RDM against every layer).
    joined[j]: plans_b[j]'s pairs already joined to plan_a (SharedJoins), so the call skips
    its per-unit joins (vr_bootstrap_spearman_multi_joined)."""
    plans_b = list(plans_b)
    for pb in plans_b:
        if pb.n != plan_a.n or pb.device != plan_a.device:
            raise ValueError("rank plans must describe RDMs of the same size and device")
    dev, n = plan_a.device, plan_a.n
    idx_t = _idx_tensor(idx, dev)
    n_sets, k = (int(idx_t.size(0)), int(idx_t.size(1))) if idx_t.numel() else (0, 0)
    total = n_sets + (1 if full_first else 0)
    nb = len(plans_b)
    scores = torch.empty((nb, total), dtype=torch.float64, device=dev)
    if total == 0 or nb == 0:
        return scores
    L = lib()
    ws = workspace.get(dev, (L.vr_bootstrap_multi_workspace if joined is None
                             else L.vr_bootstrap_multi_joined_workspace)(n, nb), "engine")
    ptrs = (ctypes.c_void_p * nb)(*[_ptr(pb.buf) for pb in plans_b])
    with torch.cuda.device(dev):
        if joined is None:
            check(
                L.vr_bootstrap_spearman_multi(
                    _ptr(plan_a.buf), ctypes.cast(ptrs, ctypes.c_void_p), nb, n,
                    _ptr(idx_t) if idx_t.numel() else None, k, n_sets, int(full_first),
                    _ptr(scores), total, _ptr(ws), ws.numel(), stream_of(dev),
                ),
                "vr_bootstrap_spearman_multi",
            )
        else:
            joined = list(joined)
            M = n * (n - 1) // 2
            if len(joined) != nb or any(t.dtype != torch.int32 or t.numel() != M or t.device != dev
                                        or not t.is_contiguous() for t in joined):
                raise ValueError("joined: one contiguous int32 tensor of M pairs per B plan, on the plans' device")
            jp = (ctypes.c_void_p * nb)(*[_ptr(t) for t in joined])
            check(
                L.vr_bootstrap_spearman_multi_joined(
                    _ptr(plan_a.buf), ctypes.cast(ptrs, ctypes.c_void_p), nb, n,
                    _ptr(idx_t) if idx_t.numel() else None, k, n_sets, int(full_first),
                    _ptr(scores), total, ctypes.cast(jp, ctypes.c_void_p), _ptr(ws), ws.numel(), stream_of(dev),
                ),
                "vr_bootstrap_spearman_multi_joined",
            )
    return scores


def bootstrap_spearman_grid(
    plans_a: Sequence[RankPlan],
    plans_b: Sequence[RankPlan],
    idx: Optional[np.ndarray | torch.Tensor],
    joined: Sequence[Sequence[torch.Tensor]],
    *,
    full_first: bool = True,
) -> torch.Tensor:
    """Spearman of every plan in plans_b against every plan in plans_a (<= 4, the regions a
    model layer is scored against) on the same subsets: (len(plans_a), len(plans_b), total)
    float64 scores on the device, [i, j] equal bit for bit to
    bootstrap_spearman_multi(plans_a[i], plans_b, idx, joined=...)[j]. joined[j][i]: B plan
    j's pairs joined to A plan i (SharedJoins(plans_a).join(plans_b[j])). The EST passes walk
    each B plan once for all A plans (vr_bootstrap_spearman_grid_joined)."""
    plans_a, plans_b = list(plans_a), list(plans_b)
    if not 1 <= len(plans_a) <= 4:
        raise ValueError("bootstrap_spearman_grid takes 1 to 4 A plans")
    pa0 = plans_a[0]
    for p in plans_a + plans_b:
        if p.n != pa0.n or p.device != pa0.device:
            raise ValueError("rank plans must describe RDMs of the same size and device")
    dev, n = pa0.device, pa0.n
    idx_t = _idx_tensor(idx, dev)
    n_sets, k = (int(idx_t.size(0)), int(idx_t.size(1))) if idx_t.numel() else (0, 0)
    total = n_sets + (1 if full_first else 0)
    na, nb = len(plans_a), len(plans_b)
    scores = torch.empty((na, nb, total), dtype=torch.float64, device=dev)
    if total == 0 or nb == 0:
        return scores
    M = n * (n - 1) // 2
    joined = [list(js) for js in joined]
    if len(joined) != nb or any(len(js) != na for js in joined) or any(
            t.dtype != torch.int32 or t.numel() != M or t.device != dev or not t.is_contiguous()
            for js in joined for t in js):
        raise ValueError("joined[j][i]: one contiguous int32 tensor of M pairs per (B plan, A plan), on the plans' device")
    L = lib()
    ws = workspace.get(dev, L.vr_bootstrap_grid_joined_workspace(n, na, nb), "engine")
    pa = (ctypes.c_void_p * na)(*[_ptr(p.buf) for p in plans_a])
    pb = (ctypes.c_void_p * nb)(*[_ptr(p.buf) for p in plans_b])
    jp = (ctypes.c_void_p * (na * nb))(*[_ptr(joined[j][i]) for i in range(na) for j in range(nb)])
    with torch.cuda.device(dev):
        check(
            L.vr_bootstrap_spearman_grid_joined(
                ctypes.cast(pa, ctypes.c_void_p), na, ctypes.cast(pb, ctypes.c_void_p), nb, n,
                _ptr(idx_t) if idx_t.numel() else None, k, n_sets, int(full_first), _ptr(scores), total,
                ctypes.cast(jp, ctypes.c_void_p), _ptr(ws), ws.numel(), stream_of(dev),
            ),
            "vr_bootstrap_spearman_grid_joined",
        )
    return scores


class SharedJoins:
    """The joins of up to 4 A plans (the neural RDMs of a model layer's regions) with any B
    plan, one 16-B gather per B pair instead of one random line per pair and A plan
    (vr_engine_posmap4 once, then vr_engine_join4 per B plan). join(plan_b) -> one int32
    tensor of M positions per A plan, for bootstrap_spearman_multi(..., joined=...)."""

    def __init__(self, plans_a: Sequence[RankPlan]):
        self.plans_a = list(plans_a)
        if not 1 <= len(self.plans_a) <= 4:
            raise ValueError("SharedJoins takes 1 to 4 A plans")
        pa0 = self.plans_a[0]
        for pa in self.plans_a:
            if pa.n != pa0.n or pa.device != pa0.device:
                raise ValueError("rank plans must describe RDMs of the same size and device")
        self.n, self.device = pa0.n, pa0.device
        L = lib()
        self.pm4 = torch.empty(int(L.vr_engine_posmap4_bytes(self.n)), dtype=torch.uint8, device=self.device)
        ptrs = (ctypes.c_void_p * len(self.plans_a))(*[_ptr(pa.buf) for pa in self.plans_a])
        with torch.cuda.device(self.device):
            check(L.vr_engine_posmap4(ctypes.cast(ptrs, ctypes.c_void_p), len(self.plans_a), self.n, _ptr(self.pm4),
                                      stream_of(self.device)), "vr_engine_posmap4")

    def join(self, plan_b: RankPlan) -> List[torch.Tensor]:
        if plan_b.n != self.n or plan_b.device != self.device:
            raise ValueError("rank plans must describe RDMs of the same size and device")
        M = self.n * (self.n - 1) // 2
        outs = [torch.empty(M, dtype=torch.int32, device=self.device) for _ in self.plans_a]
        op = (ctypes.c_void_p * len(outs))(*[_ptr(t) for t in outs])
        with torch.cuda.device(self.device):
            check(lib().vr_engine_join4(_ptr(self.pm4), len(outs), _ptr(plan_b.buf), self.n,
                                        ctypes.cast(op, ctypes.c_void_p), stream_of(self.device)), "vr_engine_join4")
        return outs


def _idx_tensor(idx, dev: torch.device) -> torch.Tensor:
    if idx is None:
        return torch.empty((0, 0), dtype=torch.int32, device=dev)
    if isinstance(idx, np.ndarray) and not idx.flags.writeable:
        idx = idx.copy()
    idx_t = torch.as_tensor(idx).to(device=dev, dtype=torch.int32).contiguous()
    if idx_t.ndim != 2:
        raise ValueError("idx must be (n_sets, k)")
    return idx_t


def bootstrap_kendall(
    plan_a: RankPlan,
    plan_b: RankPlan,
    idx: Optional[np.ndarray | torch.Tensor],
    *,
    full_first: bool = True,
) -> torch.Tensor:
    """Kendall tau-a (rsa.py:22-40) of triu(A[s][:, s]) vs triu(B[s][:, s]) for every subset s
    (row of idx), preceded by the full set when full_first. float64 scores on the device."""
    if plan_a.n != plan_b.n or plan_a.device != plan_b.device:
        raise ValueError("rank plans must describe RDMs of the same size and device")
    dev, n = plan_a.device, plan_a.n
    idx_t = _idx_tensor(idx, dev)
    n_sets, k = (int(idx_t.size(0)), int(idx_t.size(1))) if idx_t.numel() else (0, 0)
    total = n_sets + (1 if full_first else 0)
    scores = torch.empty(total, dtype=torch.float64, device=dev)
    if total == 0:
        return scores
    L = lib()
    ws = workspace.get(dev, L.vr_bootstrap_kendall_workspace(n, n_sets), "kendall")
    with torch.cuda.device(dev):
        check(
            L.vr_bootstrap_kendall_plans(
                _ptr(plan_a.buf), _ptr(plan_b.buf), n,
                _ptr(idx_t) if idx_t.numel() else None, k, n_sets, int(full_first),
                _ptr(scores), _ptr(ws), ws.numel(), stream_of(dev),
            ),
            "vr_bootstrap_kendall_plans",
        )
    return scores


_ENGINES = {"spearman": bootstrap_spearman, "kendall": bootstrap_kendall}
PLAN_MAX_N = 65535  # rank plans (and the bootstrap engines on them) use 16-bit stimulus indices


def bootstrap_full(
    model_rdm: torch.Tensor,
    neural_rdm: torch.Tensor,
    idx: Optional[np.ndarray | torch.Tensor],
    *,
    method: str = "spearman",
    full_first: bool = True,
) -> torch.Tensor:
    """The bootstrap of evals.py:355-373 for RDMs beyond the rank plans (n > 65,535, where the
    engines' 128-B rank rows would need 341 GB at 73k): per draw one plan-free call on the
    sub-RDMs A[idx][:, idx], B[idx][:, idx], read in place (vr_spearman_full_subset_f32 /
    vr_kendall_full_subset_f32: radix sorts, exact integer statistics, so every score equals
    the rank-plan engines' where both run). float64 scores on the device, the full set first
    when full_first. Works at any n with n(n-1)/2 < 2^32."""
    method = method.lower()
    if method not in _ENGINES:
        raise ValueError(f"bootstrap engine for compare_method={method!r}: spearman or kendall")
    dev = _device_for(model_rdm, neural_rdm)
    a, b = _as_device_f32(model_rdm, dev), _as_device_f32(neural_rdm, dev)
    if a.shape != b.shape or a.ndim != 2 or a.size(0) != a.size(1):
        raise ValueError("RDMs must share the same square 2-D shape")
    if a.stride(0) != b.stride(0):
        a, b = a.contiguous(), b.contiguous()
    n = a.size(0)
    idx_t = _idx_tensor(idx, dev)
    n_sets, k = (int(idx_t.size(0)), int(idx_t.size(1))) if idx_t.numel() else (0, 0)
    # a draw's statistic depends on its set of stimuli only (the same pairs, values and ties in
    # any order): read each sub-RDM in ascending stimulus order, whose rows and columns are
    # then nearly contiguous in memory (coalesced) instead of gathered at random
    if idx_t.numel():
        idx_t = torch.sort(idx_t, dim=1).values
    total = n_sets + (1 if full_first else 0)
    scores = torch.empty(total, dtype=torch.float64, device=dev)
    L = lib()
    spear = method == "spearman"
    with torch.cuda.device(dev):
        if spear:
            if full_first:
                _full_spearman_call(L.vr_spearman_full_f32, (_ptr(a), _ptr(b), n, a.stride(0), _ptr(scores)),
                                    dev, n)
            off = 1 if full_first else 0
            for i in range(n_sets):
                _full_spearman_call(L.vr_spearman_full_subset_f32, (_ptr(a), _ptr(b), n, a.stride(0),
                                                                   _ptr(idx_t[i]), k, _ptr(scores[off + i:])), dev, k)
            return scores
        ws = workspace.get(dev, L.vr_kendall_full_workspace(n), "kendall_full")
        st = stream_of(dev)
        if full_first:
            fn = L.vr_kendall_full_f32
            check(fn(_ptr(a), _ptr(b), n, a.stride(0), _ptr(scores), _ptr(ws), ws.numel(), st), fn.__name__)
        sub = L.vr_kendall_full_subset_f32
        off = 1 if full_first else 0
        for i in range(n_sets):
            check(sub(_ptr(a), _ptr(b), n, a.stride(0), _ptr(idx_t[i]), k, _ptr(scores[off + i:]), _ptr(ws),
                      ws.numel(), st), sub.__name__)
    return scores


def percentile(scores: np.ndarray, q: float) -> float:
    """numpy.percentile(scores, q), linear method (evals.py:371-372)."""
    a = np.ascontiguousarray(scores, dtype=np.float64)
    return float(lib().vr_percentile_linear(a.ctypes.data, a.size, float(q)))


# -----------------------------------------------------------------------------
# RDM comparison
# -----------------------------------------------------------------------------
_KENDALL_PAIRWISE_MAX = 1 << 16  # longer vectors: the O(m log m) sort path


def _vec_f64(v, dev: torch.device) -> torch.Tensor:
    if isinstance(v, torch.Tensor):
        return v.detach().reshape(-1).to(device=dev, dtype=torch.float64).contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(v, dtype=np.float64).ravel())).to(dev)


def _kendall_tau_a(x, y) -> tuple:
    """Kendall tau-a of two 1-D arrays, returned as (tau_a, nan) (rsa.py:22-40).

    The reference takes scipy's tau-b and rescales it by sqrt((n0 - t_x)(n0 - t_y)) / n0.
    Here the discordant and tie counts are exact integers -- every pair compared in fp64 up to
    2^16 elements (vr_kendall_tau_a_f64), beyond that the O(m log m) sort-and-inversion form
    (vr_kendall_full_vec_f64, any length < 2^32; both give the same bits) -- then the same fp64
    conversion. NaN for fewer than two elements, any NaN element or a constant input; arrays of
    unequal length raise ValueError, as scipy.stats.kendalltau does. Tensors already on a HIP
    device are used there; host arrays go to the current device."""
    nx = int(x.numel()) if isinstance(x, torch.Tensor) else int(np.size(x))
    ny = int(y.numel()) if isinstance(y, torch.Tensor) else int(np.size(y))
    if nx < 2:  # rsa.py:24-26 checks len(x) before scipy sees y
        return (float("nan"), float("nan"))
    if nx != ny:
        raise ValueError("All inputs to `kendalltau` must be of the same size, found x-size %d and y-size %d"
                         % (nx, ny))
    m = nx
    dev = _device_for(x, y)
    xd, yd = _vec_f64(x, dev), _vec_f64(y, dev)
    out = torch.empty(1, dtype=torch.float64, device=dev)
    L = lib()
    with torch.cuda.device(dev):
        if m <= _KENDALL_PAIRWISE_MAX:
            ws = workspace.get(dev, L.vr_kendall_vec_workspace(m), "kendall_vec")
            check(L.vr_kendall_tau_a_f64(_ptr(xd), _ptr(yd), m, _ptr(out), _ptr(ws), ws.numel(), stream_of(dev)),
                  "vr_kendall_tau_a_f64")
        else:
            ws = workspace.get(dev, L.vr_kendall_full_vec_workspace(m), "kendall_full")
            check(L.vr_kendall_full_vec_f64(_ptr(xd), _ptr(yd), m, _ptr(out), _ptr(ws), ws.numel(),
                                            stream_of(dev)), "vr_kendall_full_vec_f64")
    return (float(out.item()), float("nan"))


def compute_rdm_correlation(
    rdm1: torch.Tensor, rdm2: torch.Tensor, *, correlation: str = "Kendall"
) -> float:
    """Correlation of the strict upper triangles of two RDMs (rsa.py:96-129).

    NaN when undefined (n <= 1, NaN input, constant triangle); ValueError on a shape
    mismatch or an unknown method — checked in the reference's order."""
    if not isinstance(rdm1, torch.Tensor):
        rdm1 = torch.as_tensor(np.asarray(rdm1))
    if not isinstance(rdm2, torch.Tensor):
        rdm2 = torch.as_tensor(np.asarray(rdm2))
    if rdm1.shape != rdm2.shape or rdm1.ndim != 2:
        raise ValueError("RDMs must share the same 2-D shape")
    n = rdm1.size(0)
    if n <= 1:
        logger.warning("RDM dimension <= 1; correlation undefined")
        return float("nan")
    if rdm1.size(1) < n:
        raise ValueError("RDMs must be square")
    corr = correlation.lower()
    if corr not in _VALID_CMP:
        raise ValueError("correlation must be 'Pearson', 'Spearman', or 'Kendall'")
    dev = _device_for(rdm1, rdm2)
    a = _as_device_f32(rdm1, dev)
    b = _as_device_f32(rdm2, dev)
    if a.stride(0) != b.stride(0):
        a, b = a.contiguous(), b.contiguous()
    out = torch.empty(1, dtype=torch.float64, device=dev)
    L = lib()
    with torch.cuda.device(dev):
        if corr == "spearman" and n > 65535:
            return spearman_full(a, b)
        if corr == "spearman":
            ws = workspace.get(dev, L.vr_spearman_triu_workspace(n), "triu")
            check(
                L.vr_spearman_triu_f32(_ptr(a), _ptr(b), n, a.stride(0), _ptr(out),
                                       _ptr(ws), ws.numel(), stream_of(dev)),
                "vr_spearman_triu_f32",
            )
        elif corr == "kendall" and n > 65535:  # beyond the rank plans: the sort-and-inversion path
            ws = workspace.get(dev, L.vr_kendall_full_workspace(n), "kendall_full")
            check(
                L.vr_kendall_full_f32(_ptr(a), _ptr(b), n, a.stride(0), _ptr(out),
                                      _ptr(ws), ws.numel(), stream_of(dev)),
                "vr_kendall_full_f32",
            )
        elif corr == "kendall":
            ws = workspace.get(dev, L.vr_kendall_triu_workspace(n), "kendall_triu")
            check(
                L.vr_kendall_triu_f32(_ptr(a), _ptr(b), n, a.stride(0), _ptr(out),
                                      _ptr(ws), ws.numel(), stream_of(dev)),
                "vr_kendall_triu_f32",
            )
        else:
            ws = workspace.get(dev, L.vr_pearson_triu_workspace(n), "pearson")
            check(
                L.vr_pearson_triu_f32(_ptr(a), _ptr(b), n, a.stride(0), _ptr(out),
                                      _ptr(ws), ws.numel(), stream_of(dev)),
                "vr_pearson_triu_f32",
            )
    val = float(out.item())
    if math.isnan(val):
        logger.warning("NaN returned for %s correlation", correlation)
        return float("nan")
    return val


_VR_EWORKSPACE = -3


def _full_spearman_call(fn, args: tuple, dev: torch.device, n: int) -> None:
    """fn(*args, ws, ws_bytes, stream) on the count-table workspace; a triangle whose key
    range is wider than those tables (values beyond [0, 2]) returns VR_EWORKSPACE, and the
    call runs again on the sort form's workspace."""
    L = lib()
    ws = workspace.get(dev, L.vr_spearman_full_workspace(n), "spearman_full")
    rc = fn(*args, _ptr(ws), ws.numel(), stream_of(dev))
    if rc == _VR_EWORKSPACE:
        ws = workspace.get(dev, L.vr_spearman_full_sort_workspace(n), "spearman_full")
        rc = fn(*args, _ptr(ws), ws.numel(), stream_of(dev))
    check(rc, fn.__name__)


def spearman_full(rdm1: torch.Tensor, rdm2: torch.Tensor) -> float:
    """Spearman of the strict upper triangles without a rank plan (vr_spearman_full_f32):
    average ranks from per-key count tables of each triangle (a radix sort of (value,
    triangle index) when the value range is too wide for them), exact integer sums; any
    n with n(n-1)/2 < 2^32 (n <= 92681). compute_rdm_correlation uses it above the rank
    plan's n <= 65535 (configs[2]'s 73k-stimulus RDM)."""
    dev = _device_for(rdm1, rdm2)
    a = _as_device_f32(rdm1, dev)
    b = _as_device_f32(rdm2, dev)
    if a.shape != b.shape or a.ndim != 2 or a.size(0) != a.size(1):
        raise ValueError("RDMs must share the same square 2-D shape")
    if a.stride(0) != b.stride(0):
        a, b = a.contiguous(), b.contiguous()
    n = a.size(0)
    out = torch.empty(1, dtype=torch.float64, device=dev)
    L = lib()
    with torch.cuda.device(dev):
        _full_spearman_call(L.vr_spearman_full_f32, (_ptr(a), _ptr(b), n, a.stride(0), _ptr(out)), dev, n)
    val = float(out.item())
    if math.isnan(val):
        logger.warning("NaN returned for Spearman correlation")
    return val


# -----------------------------------------------------------------------------
# Bootstrap (evals.py:355-373) and train/test RSA (rsa.py:132-281)
# -----------------------------------------------------------------------------
def bootstrap_rsa(
    model_rdm: torch.Tensor | RankPlan,
    neural_rdm: torch.Tensor | RankPlan,
    *,
    n_bootstrap: int = 1000,
    seed: int = 42,
    idx: Optional[np.ndarray] = None,
    method: str = "spearman",
) -> Tuple[float, np.ndarray, float, float]:
    """Point estimate plus the reference's inline bootstrap: a fresh RandomState(seed),
    n_bootstrap draws of choice(n, int(0.9 n), replace=False), Spearman (or Kendall tau-a)
    of the two sub-RDMs per draw, 2.5/97.5 linear percentiles. Returns
    (point, scores[n_bootstrap], ci_low, ci_high)."""
    engine = _ENGINES.get(method.lower())
    if engine is None:
        raise ValueError(f"bootstrap engine for compare_method={method!r}: spearman or kendall")
    n = model_rdm.n if isinstance(model_rdm, RankPlan) else int(model_rdm.shape[0])
    if idx is None:
        idx = bootstrap_indices(seed, n, int(n * 0.9), int(n_bootstrap)) if n_bootstrap else None
    if n > PLAN_MAX_N and not isinstance(model_rdm, RankPlan):  # beyond the rank plans
        scores = bootstrap_full(model_rdm, neural_rdm, idx, method=method, full_first=True).cpu().numpy()
    else:
        pa = model_rdm if isinstance(model_rdm, RankPlan) else RankPlan(model_rdm)
        pb = neural_rdm if isinstance(neural_rdm, RankPlan) else RankPlan(neural_rdm)
        scores = engine(pa, pb, idx, full_first=True).cpu().numpy()
    point, boot = float(scores[0]), scores[1:].copy()
    if boot.size == 0:
        return point, boot, float("nan"), float("nan")
    return point, boot, percentile(boot, 2.5), percentile(boot, 97.5)


def _flatten(a: torch.Tensor) -> torch.Tensor:
    return a.flatten(start_dim=1) if a.ndim > 2 else a


def _index_rows(a: torch.Tensor, idx: np.ndarray) -> torch.Tensor:
    return a[torch.as_tensor(idx, dtype=torch.long, device=a.device)]


def compute_rsa(
    cfg: Dict,
    selection: "AlignmentData",
    evaluation: "AlignmentData",
    n_select: int | None = None,
    bootstrap: bool = True,
    n_bootstrap: int = 1000,
    seed: int = 42,
    verbose: bool = False,
    re_extract_fn=None,
) -> List[Dict]:
    """Train/test RSA (rsa.py:132-281): best layer on the selection split by Spearman
    of Pearson RDMs (first strict maximum), point estimate on the evaluation split,
    optional 90 % subsample bootstrap. One RandomState(seed) feeds the n_select draw and
    then the bootstrap draws, as in the reference."""
    method = cfg.get("compare_method", "spearman").lower()
    rng = LegacyRandomState(seed)

    n_train = selection.neural.size(0)
    n_test = evaluation.neural.size(0)

    if n_select is not None and n_select < n_train:
        n_sel = n_select
        sel_idx = rng.choice(n_train, size=n_sel, replace=False)
        sel_label = f"subsampling {n_sel}"
    else:
        n_sel = n_train
        sel_idx = np.arange(n_train)
        sel_label = f"using all {n_sel}"

    if verbose:
        rprint(f"Train/test RSA: {n_train} train, {n_test} test, {sel_label} for layer selection",
               style="info")
        rprint(f"Building RDMs with Pearson, comparing with {method.capitalize()}", style="info")

    neural_rdm_sel = compute_rdm(_index_rows(selection.neural, sel_idx))
    engine = _ENGINES.get(method)
    sel_plan = RankPlan(neural_rdm_sel) if engine is not None and 1 < n_sel <= PLAN_MAX_N else None

    selection_scores = []
    best_layer, best_score = None, -float("inf")
    for layer, acts in selection.activations.items():
        flat = _flatten(_index_rows(acts, sel_idx))
        layer_rdm = compute_rdm(flat)
        if sel_plan is not None:
            score = float(engine(RankPlan(layer_rdm), sel_plan, None)[0].item())
            if math.isnan(score):
                logger.warning("NaN returned for %s correlation", method.capitalize())
        else:
            score = compute_rdm_correlation(layer_rdm, neural_rdm_sel,
                                            correlation=method.capitalize())
        selection_scores.append({"layer": layer, "score": score})
        if verbose:
            rprint(f"  [select] {layer:<15} RSA = {score:.4f}", style="info")
        if score > best_score:
            best_score = score
            best_layer = layer

    if verbose:
        rprint(f"  Best layer: {best_layer} (score={best_score:.4f})", style="highlight")

    if re_extract_fn is not None:
        rprint(f"  Re-extracting {best_layer} without SRP for exact test RDMs...", style="info")
        exact_acts, _ = re_extract_fn(best_layer, evaluation.stimulus_ids)
        test_acts_flat = _flatten(exact_acts)
    else:
        test_acts_flat = _flatten(evaluation.activations[best_layer])

    test_neural_rdm = compute_rdm(evaluation.neural)
    test_model_rdm = compute_rdm(test_acts_flat)

    ci_low, ci_high = None, None
    bootstrap_scores_list = None
    if engine is not None and n_test > 1:
        boot_idx = None
        if bootstrap and n_bootstrap > 0:
            k = int(n_test * 0.9)
            boot_idx = np.stack([rng.choice(n_test, size=k, replace=False)
                                 for _ in range(n_bootstrap)]).astype(np.int32)
        if n_test > PLAN_MAX_N:  # beyond the rank plans: one plan-free call per draw
            scores = bootstrap_full(test_model_rdm, test_neural_rdm, boot_idx, method=method).cpu().numpy()
        else:
            plan_m, plan_n = RankPlan(test_model_rdm), RankPlan(test_neural_rdm)
            scores = engine(plan_m, plan_n, boot_idx, full_first=True).cpu().numpy()
        point_estimate = float(scores[0])
        if math.isnan(point_estimate):
            logger.warning("NaN returned for %s correlation", method.capitalize())
        if bootstrap:
            boot = scores[1:].astype(np.float64)
            if boot.size:
                ci_low, ci_high = percentile(boot, 2.5), percentile(boot, 97.5)
            else:  # np.percentile of an empty array raises in the reference
                raise IndexError("cannot compute percentiles of zero bootstrap scores")
            bootstrap_scores_list = boot.tolist()
    else:
        point_estimate = compute_rdm_correlation(test_model_rdm, test_neural_rdm,
                                                 correlation=method.capitalize())
        if bootstrap:
            k = int(n_test * 0.9)
            boot = np.empty(n_bootstrap, dtype=np.float64)
            for i in range(n_bootstrap):
                bi = torch.as_tensor(rng.choice(n_test, size=k, replace=False),
                                     device=test_model_rdm.device)
                boot[i] = compute_rdm_correlation(test_model_rdm[bi][:, bi],
                                                  test_neural_rdm[bi][:, bi],
                                                  correlation=method.capitalize())
            ci_low, ci_high = percentile(boot, 2.5), percentile(boot, 97.5)
            bootstrap_scores_list = boot.tolist()

    if verbose:
        rprint(f"  Test RSA = {point_estimate:.4f}", style="highlight")
    rprint("")
    msg = f"  {method.capitalize():<10}| {best_layer} = {point_estimate:.4f}"
    if bootstrap:
        msg += f"  [95% CI: {ci_low:.4f}, {ci_high:.4f}]"
    rprint(msg, style="highlight")

    result = {
        "layer": best_layer,
        "compare_method": method,
        "score": point_estimate,
        "ci_low": ci_low,
        "ci_high": ci_high,
        "analysis": "rsa",
        "layer_selection_scores": selection_scores,
    }
    if bootstrap_scores_list is not None:
        result["bootstrap_scores"] = bootstrap_scores_list
    return [result]


def _concept_average_exact(raw_acts, raw_ids, data):
    """Concept means of exact per-image activations in data.stimulus_ids order
    (rsa.py:284-305); a concept with no images gets a zero row."""
    id_to_idx = {str(k): i for i, k in enumerate(raw_ids)}
    rows = []
    for concept in data.stimulus_ids:
        img_ids = data.concept_image_ids[concept]
        indices = [id_to_idx[sid] for sid in img_ids if sid in id_to_idx]
        if indices:
            sel = raw_acts[torch.as_tensor(indices, dtype=torch.long, device=raw_acts.device)]
            rows.append(sel.float().mean(0))
        else:
            rows.append(torch.zeros(raw_acts.size(1), device=raw_acts.device))
    return torch.stack(rows).to(raw_acts.dtype)
