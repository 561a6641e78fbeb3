"""ctypes binding of libvisreps_hip.so (the C ABI declared in include/visreps_hip.h).

torch is imported first on purpose: its bundled libamdhip64.so.7 is then the HIP runtime
the library binds to (same SONAME), so device pointers and streams are shared with
torch. There is no CPU fallback anywhere in the product path: if the library is missing
the import of this module raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede loading the HIP library, see module doc)

__all__ = [
    "LIB_PATH",
    "VisrepsHipError",
    "lib",
    "check",
    "stream_of",
    "workspace",
    "EXPORTED_SYMBOLS",
]

# VISREPS_AMD_LIB selects another build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("VISREPS_AMD_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libvisreps_hip.so")


class VisrepsHipError(RuntimeError):
    """A libvisreps_hip call returned a non-zero status."""


_c_i64 = ctypes.c_int64
_c_sz = ctypes.c_size_t
_vp = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/visreps_hip.h
_PROTOTYPES = {
    "vr_version": (ctypes.c_int, []),
    "vr_last_error": (ctypes.c_char_p, []),
    "vr_rdm_pearson_workspace": (_c_sz, [_c_i64, _c_i64]),
    "vr_rdm_pearson_f32": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, ctypes.c_float, _vp, _c_sz, _vp],
    ),
    "vr_rdm_tile_count": (_c_i64, [_c_i64]),
    "vr_rdm_wide_rows": (_c_i64, [_c_i64, _c_i64]),
    "vr_rdm_range_aligned": (ctypes.c_int, [_c_i64, _c_i64, _c_i64, _c_i64]),
    "vr_rdm_tile_cost": (_c_i64, [_c_i64, _c_i64]),
    "vr_rdm_tile_rect": (ctypes.c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp]),
    "vr_rdm_tiles_workspace": (_c_sz, [_c_i64, _c_i64, _c_i64, _c_i64]),
    "vr_rdm_pearson_tiles_f32": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, ctypes.c_float, _c_i64, _c_i64, _vp, _c_sz, _vp],
    ),
    "vr_rdm_bf16_workspace": (_c_sz, [_c_i64, _c_i64, _c_i64, _c_i64]),
    "vr_rdm_pearson_bf16": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, ctypes.c_float, _vp, _c_sz, _vp],
    ),
    "vr_rdm_pearson_tiles_bf16": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, ctypes.c_float, _c_i64, _c_i64, _vp, _c_sz, _vp],
    ),
    "vr_gram_f32": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, _vp, _c_sz, _vp],
    ),
    "vr_corr_score_workspace": (_c_sz, [_c_i64, _c_i64]),
    "vr_corr_score_f32": (
        ctypes.c_int,
        [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _c_sz, _vp],
    ),
    "vr_row_stats_f32": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, ctypes.c_float, _vp],
    ),
    "vr_rank_plan_bytes": (_c_sz, [_c_i64]),
    "vr_rank_plan_workspace": (_c_sz, [_c_i64]),
    "vr_rank_plan_build_f32": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _vp, _c_sz, _vp, _c_sz, _vp],
    ),
    "vr_spearman_triu_workspace": (_c_sz, [_c_i64]),
    "vr_spearman_triu_f32": (
        ctypes.c_int,
        [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_sz, _vp],
    ),
    "vr_pearson_triu_workspace": (_c_sz, [_c_i64]),
    "vr_pearson_triu_f32": (
        ctypes.c_int,
        [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_sz, _vp],
    ),
    "vr_bootstrap_workspace": (_c_sz, [_c_i64]),
    "vr_bootstrap_spearman_plans": (
        ctypes.c_int,
        [_vp, _vp, _c_i64, _vp, _c_i64, _c_i64, ctypes.c_int, _vp, _vp, _c_sz, _vp],
    ),
    "vr_bootstrap_multi_workspace": (_c_sz, [_c_i64, _c_i64]),
    "vr_bootstrap_multi_joined_workspace": (_c_sz, [_c_i64, _c_i64]),
    "vr_bootstrap_spearman_multi": (
        ctypes.c_int,
        [_vp, _vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64, ctypes.c_int, _vp, _c_i64, _vp, _c_sz, _vp],
    ),
    "vr_bootstrap_spearman_multi_joined": (
        ctypes.c_int,
        [_vp, _vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64, ctypes.c_int, _vp, _c_i64, _vp, _vp, _c_sz, _vp],
    ),
    "vr_bootstrap_grid_joined_workspace": (_c_sz, [_c_i64, _c_i64, _c_i64]),
    "vr_bootstrap_spearman_grid_joined": (
        ctypes.c_int,
        [_vp, _c_i64, _vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64, ctypes.c_int, _vp, _c_i64, _vp, _vp, _c_sz, _vp],
    ),
    "vr_engine_posmap4_bytes": (_c_sz, [_c_i64]),
    "vr_engine_posmap4": (ctypes.c_int, [_vp, _c_i64, _c_i64, _vp, _vp]),
    "vr_engine_join4": (ctypes.c_int, [_vp, _c_i64, _vp, _c_i64, _vp, _vp]),
    "vr_engine_est_reruns": (_c_i64, []),
    "vr_engine_est_tail_flags": (_c_i64, []),
    "vr_test_engine_inject": (ctypes.c_int, [_c_i64]),
    "vr_engine_est_predicted": (_c_i64, []),
    "vr_engine_est1_fallbacks": (_c_i64, []),
    "vr_ktimer_enable": (ctypes.c_int, [ctypes.c_int]),
    "vr_trace_mark": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _vp]),
    "vr_ktimer_read": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]),
    "vr_bootstrap_spearman_workspace": (_c_sz, [_c_i64]),
    "vr_bootstrap_spearman_f32": (
        ctypes.c_int,
        [_vp, _vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64, ctypes.c_int, _vp, _vp, _c_sz, _vp],
    ),
    "vr_kendall_triu_workspace": (_c_sz, [_c_i64]),
    "vr_kendall_triu_f32": (
        ctypes.c_int,
        [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_sz, _vp],
    ),
    "vr_kendall_vec_workspace": (_c_sz, [_c_i64]),
    "vr_kendall_tau_a_f64": (ctypes.c_int, [_vp, _vp, _c_i64, _vp, _vp, _c_sz, _vp]),
    "vr_kendall_full_vec_workspace": (_c_sz, [_c_i64]),
    "vr_kendall_full_vec_f64": (ctypes.c_int, [_vp, _vp, _c_i64, _vp, _vp, _c_sz, _vp]),
    "vr_kendall_full_workspace": (_c_sz, [_c_i64]),
    "vr_kendall_full_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_sz, _vp]),
    "vr_bootstrap_kendall_workspace": (_c_sz, [_c_i64, _c_i64]),
    "vr_bootstrap_kendall_plans": (
        ctypes.c_int,
        [_vp, _vp, _c_i64, _vp, _c_i64, _c_i64, ctypes.c_int, _vp, _vp, _c_sz, _vp],
    ),
    "vr_srp_workspace": (_c_sz, [_c_i64, _c_i64]),
    "vr_srp_csr_f32": (
        ctypes.c_int,
        [_vp, _vp, _vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64, _vp, _c_i64, _vp, _c_sz, _vp],
    ),
    "vr_col_sum_f32": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp]),
    "vr_col_mean_f32": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp]),
    "vr_mean_from_sum_f32": (ctypes.c_int, [_vp, _c_i64, _c_i64, _vp, _vp]),
    "vr_pca_cov_workspace": (_c_sz, [_c_i64, _c_i64]),
    "vr_pca_cov_f64": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _vp, ctypes.c_double, _vp, _c_i64, _vp, _c_sz, _vp],
    ),
    "vr_gram64_workspace": (_c_sz, [_c_i64, _c_i64, ctypes.c_int]),
    "vr_gram64_f32": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, ctypes.c_int, _vp, _c_i64, _vp, _c_sz, _vp]),
    "vr_spearman_full_workspace": (_c_sz, [_c_i64]),
    "vr_spearman_full_sort_workspace": (_c_sz, [_c_i64]),
    "vr_spearman_full_last_form": (ctypes.c_int, []),
    "vr_key_counts_u32": (ctypes.c_int, [_vp, _c_i64, ctypes.c_uint32, _c_i64, _vp, _vp]),
    "vr_key_table_workspace": (_c_sz, [_c_i64]),
    "vr_key_table_midranks": (ctypes.c_int, [_vp, _c_i64, ctypes.c_uint32, _vp, _c_i64, _vp, _vp, _vp, _c_sz, _vp]),
    "vr_spearman_full_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_sz, _vp]),
    "vr_spearman_full_subset_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _vp, _c_i64, _vp, _vp, _c_sz, _vp]),
    "vr_kendall_full_subset_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _vp, _c_i64, _vp, _vp, _c_sz, _vp]),
    "vr_f32_sort_keys": (ctypes.c_int, [_vp, _c_i64, _vp, _vp]),
    "vr_sort_pairs_workspace": (_c_sz, [_c_i64]),
    "vr_sort_pairs_u32": (ctypes.c_int, [_vp, _vp, _c_i64, _vp, _c_sz, _vp]),
    "vr_midranks_workspace": (_c_sz, [_c_i64]),
    "vr_midranks_sorted": (ctypes.c_int, [_vp, _c_i64, ctypes.c_uint64, _vp, _vp, _vp, _c_sz, _vp]),
    "vr_dot_u64_workspace": (_c_sz, []),
    "vr_dot_u64": (ctypes.c_int, [_vp, _vp, _c_i64, _vp, _vp, _c_sz, _vp]),
    "vr_rdm_plane_rows": (_c_i64, [_c_i64]),
    "vr_rdm_plane_row_bytes": (_c_sz, [_c_i64]),
    "vr_rdm_split_rows_f32": (
        ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, ctypes.c_float, _vp, _vp, _vp, _vp]),
    "vr_rdm_split_rows_multi_f32": (
        ctypes.c_int, [ctypes.c_int, _vp, _vp, _vp, _c_i64, ctypes.c_float, _vp, _vp, _vp, _vp]),
    "vr_gather_rows_multi_f32": (
        ctypes.c_int, [ctypes.c_int, _vp, _vp, _vp, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    "vr_rdm_planes_tiles_workspace": (_c_sz, [_c_i64, _c_i64, _c_i64, _c_i64]),
    "vr_rdm_pearson_tiles_planes": (
        ctypes.c_int,
        [_vp, _vp, _vp, _c_i64, _c_i64, _vp, _c_i64, ctypes.c_float, _c_i64, _c_i64, _vp, _c_sz, _vp],
    ),
    "vr_rccl_available": (ctypes.c_int, []),
    "vr_rccl_unique_id": (ctypes.c_int, [_vp]),
    "vr_rccl_comm_init": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _vp, ctypes.c_int]),
    "vr_rccl_comm_destroy": (ctypes.c_int, [_vp]),
    "vr_rdm_sharded_range": (ctypes.c_int, [_c_i64, _c_i64, ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "vr_rdm_sharded_workspace": (_c_sz, [_c_i64, _c_i64, ctypes.c_int]),
    "vr_rdm_pearson_sharded": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _c_i64, _vp, _c_i64, ctypes.c_float, _vp, ctypes.c_int, ctypes.c_int, _vp,
         _c_sz, _vp],
    ),
    "vr_comm_rccl": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int]),
    "vr_rdm_pearson_sharded_comm": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _c_i64, _vp, _c_i64, ctypes.c_float, _vp, _vp, _c_sz, _vp],
    ),
    "vr_rdm_tiles_pack": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _c_i64, _vp, _vp]),
    "vr_rdm_tiles_unpack": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, _vp]),
    "vr_transform_workspace": (_c_sz, [_c_i64, _c_i64, _c_i64, _c_i64, _c_i64, ctypes.c_int]),
    "vr_transform_u8": (
        ctypes.c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, ctypes.c_int, _vp, _vp, _vp, _vp, _c_sz, _vp],
    ),
    "vr_rng_state_bytes": (_c_sz, []),
    "vr_rng_seed": (ctypes.c_int, [_vp, ctypes.c_uint32]),
    "vr_rng_permutation": (ctypes.c_int, [_vp, _c_i64, _vp]),
    "vr_rng_choice": (ctypes.c_int, [_vp, _c_i64, _c_i64, _vp]),
    "vr_rng_random_u32": (ctypes.c_int, [_vp, _c_i64, _vp]),
    "vr_legacy_choice": (ctypes.c_int, [ctypes.c_uint32, _c_i64, _c_i64, _c_i64, _vp]),
    "vr_percentile_linear": (ctypes.c_double, [_vp, _c_i64, ctypes.c_double]),
}

EXPORTED_SYMBOLS = tuple(_PROTOTYPES)

# typedef int (*vr_allgather_fn)(const void* send, void* recv, size_t bytes, void* user, void* stream)
VR_ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, _vp, _c_sz, _vp, _vp)


class VrComm(ctypes.Structure):
    """struct vr_comm (include/visreps_hip.h): the collective table of the sharded entry points."""
    _fields_ = [("world", ctypes.c_int), ("rank", ctypes.c_int), ("all_gather", VR_ALLGATHER_FN), ("user", _vp)]

_lib = None
_lock = threading.Lock()


def lib() -> ctypes.CDLL:
    """The loaded library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} not found: build the MI355X kernels first "
                    "(python -c 'import __graft_entry__ as g; g.build()' or "
                    "make -C visreps_amd/csrc). There is no CPU fallback."
                )
            handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in _PROTOTYPES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def check(rc: int, fn: str) -> None:
    if rc != 0:
        msg = lib().vr_last_error().decode(errors="replace")
        raise VisrepsHipError(f"{fn} failed (status {rc}): {msg}")


def stream_of(device: torch.device) -> int:
    """hipStream_t of torch's current stream on `device`, as an integer."""
    return int(torch.cuda.current_stream(device).cuda_stream)


class _WorkspacePool:
    """Per-(device, tag) grow-only scratch buffers handed to the library.

    The library never allocates; every call gets its scratch from here. Buffers are
    reused across calls on the same stream (torch's caching allocator keeps stream
    order), so a tag must not be shared by two calls that are live at once.
    """

    def __init__(self):
        self._bufs: dict[tuple, torch.Tensor] = {}

    def get(self, device: torch.device, nbytes: int, tag: str = "ws") -> torch.Tensor:
        key = (str(device), tag)
        buf = self._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            self._bufs.pop(key, None)
            buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            self._bufs[key] = buf
        return buf

    def current(self, device: torch.device, tag: str = "ws") -> int:
        """Bytes of the (device, tag) buffer held now (0 if none)."""
        buf = self._bufs.get((str(device), tag))
        return 0 if buf is None else int(buf.numel())

    def release(self, tag: str | None = None) -> None:
        if tag is None:
            self._bufs.clear()
        else:
            for k in [k for k in self._bufs if k[1] == tag]:
                del self._bufs[k]


workspace = _WorkspacePool()


KTIMER_KERNELS = {"k_rankB_est": 0, "k_rankB_exact": 1, "k_rankA": 2, "k_join": 3,
                  "k_gram_wide": 4, "k_gram_tile": 5, "k_countA": 6, "k_rankB_full": 7,
                  "k_kwalk": 8, "k_cov": 9, "k_join4": 10,
                  "k_full_corr": 11, "k_rankB_grid": 12, "k_rankB_gridx": 13}


def ktimer_enable(on: bool = True) -> None:
    """Start (clearing the totals) or stop the library's per-launch HIP-event timing of the
    hot kernels (vr_ktimer_enable)."""
    check(lib().vr_ktimer_enable(1 if on else 0), "vr_ktimer_enable")


def ktimer_read(kernel: str) -> tuple[float, int, float]:
    """(total ms, launches, units) of one hot kernel since ktimer_enable; units are pairs
    walked (engine kernels) or tile FLOPs (Gram kernels)."""
    ms, n, u = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
    check(lib().vr_ktimer_read(KTIMER_KERNELS[kernel], ctypes.byref(ms), ctypes.byref(n), ctypes.byref(u)),
          "vr_ktimer_read")
    return ms.value, n.value, u.value


def build_id() -> str:
    """sha256[:16] of the loaded library file: ties a committed profile to the build it
    measured (bench.py emits PMC-derived figures only for the same build)."""
    import hashlib

    with open(LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]
