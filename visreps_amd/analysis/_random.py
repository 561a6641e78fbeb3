"""Legacy numpy RandomState index streams from the native MT19937 (bit-exact).

Only the calls the RSA path makes are provided: ``RandomState(seed)``,
``.choice(n, size, replace=False)`` and ``.permutation(n)``
(visreps/evals.py:260-261,356,362-364; visreps/analysis/rsa.py:169,176,248-250;
evals.py:111-113). Results are int64 numpy arrays, like numpy's.
"""
from __future__ import annotations

import ctypes
import functools

import numpy as np

from .._lib import check, lib

__all__ = ["LegacyRandomState", "bootstrap_indices", "draw_bootstrap_indices"]


class LegacyRandomState:
    """Drop-in for ``np.random.RandomState(seed)`` restricted to the RSA path's calls."""

    def __init__(self, seed: int):
        seed = int(seed)
        if seed < 0 or seed > 0xFFFFFFFF:
            raise ValueError("Seed must be between 0 and 2**32 - 1")
        self._state = ctypes.create_string_buffer(lib().vr_rng_state_bytes())
        check(lib().vr_rng_seed(self._state, ctypes.c_uint32(seed)), "vr_rng_seed")

    def permutation(self, n: int) -> np.ndarray:
        n = int(n)
        out = np.empty(n, dtype=np.int32)
        check(lib().vr_rng_permutation(self._state, n, out.ctypes.data), "vr_rng_permutation")
        return out.astype(np.int64)

    def choice(self, a: int, size: int | None = None, replace: bool = True, p=None) -> np.ndarray:
        if replace or p is not None:
            raise NotImplementedError("only choice(n, size, replace=False) is on the RSA path")
        n = int(a)
        if size is None:
            raise NotImplementedError("size is required")
        k = int(size)
        if k > n:
            raise ValueError("Cannot take a larger sample than population when 'replace=False'")
        if k < 0:
            raise ValueError("negative dimensions are not allowed")
        out = np.empty(k, dtype=np.int32)
        check(lib().vr_rng_choice(self._state, n, k, out.ctypes.data), "vr_rng_choice")
        return out.astype(np.int64)

    def random_u32(self, count: int) -> np.ndarray:
        out = np.empty(int(count), dtype=np.uint32)
        check(lib().vr_rng_random_u32(self._state, int(count), out.ctypes.data), "vr_rng_random_u32")
        return out


def draw_bootstrap_indices(seed: int, n: int, k: int, n_draws: int) -> np.ndarray:
    """``[RandomState(seed).choice(n, k, replace=False) for _ in range(n_draws)]`` as an
    int32 (n_draws, k) array, drawn now (host MT19937, no cache)."""
    out = np.empty((int(n_draws), int(k)), dtype=np.int32)
    check(lib().vr_legacy_choice(int(seed), int(n), int(k), int(n_draws), out.ctypes.data), "vr_legacy_choice")
    return out


@functools.lru_cache(maxsize=8)
def _cached_bootstrap_indices(seed: int, n: int, k: int, n_draws: int) -> np.ndarray:
    out = draw_bootstrap_indices(seed, n, k, n_draws)
    out.setflags(write=False)
    return out


def bootstrap_indices(seed: int, n: int, k: int, n_draws: int) -> np.ndarray:
    """``[RandomState(seed).choice(n, k, replace=False) for _ in range(n_draws)]`` as an
    int32 (n_draws, k) array. Cached: the reference resets RandomState(42) for every
    (region, subject) pair (evals.py:356), so every unit with the same n shares it."""
    return _cached_bootstrap_indices(int(seed), int(n), int(k), int(n_draws))
