// Shared helpers for libvisreps_hip.so: error reporting, workspace carving, launch
// geometry. gfx950 (CDNA4) only: wave64, 256 CUs in 8 XCDs.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdint>

#include "../../include/visreps_hip.h"

namespace vr {

void set_error(const char* fmt, ...);
void clear_error();

// Carves aligned sub-buffers out of one caller workspace. With base == nullptr it only
// measures, so the *_workspace() queries and the launches share one layout function.
struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base(static_cast<char*>(b)) {}
  template <class T>
  T* take(size_t count, size_t align = 256) {
    off = (off + align - 1) / align * align;
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += count * sizeof(T);
    return p;
  }
  size_t bytes() const { return (off + 255) / 256 * 256; }
};

// Compute units of the current device (cached per device id).
int num_cus();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Strict upper-triangle linear index (row-major, torch.triu_indices(n, n, 1) order)
// of the pair (a, b), a < b.
__host__ __device__ inline uint64_t tri_index(uint64_t a, uint64_t b, uint64_t n) {
  return a * n - a * (a + 1) / 2 + (b - a - 1);
}

inline int64_t pairs_of(int64_t n) { return n > 1 ? n * (n - 1) / 2 : 0; }

// Bijective XCD-aware block remap (cdna_hip_programming.md §5, T1): blocks b and b+8
// share an XCD, so consecutive logical tiles are dealt to one XCD's L2.
__device__ inline uint32_t xcd_remap(uint32_t orig, uint32_t nwg) {
  const uint32_t nx = 8;
  if (nwg < nx) return orig;
  uint32_t q = nwg / nx, r = nwg % nx, xcd = orig % nx;
  uint32_t base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / nx;
}

}  // namespace vr

#define VR_CHECK_HIP(expr)                                                       \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess) {                                                      \
      vr::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),        \
                    __FILE__, __LINE__);                                         \
      return VR_EHIP;                                                            \
    }                                                                            \
  } while (0)

#define VR_CHECK_LAUNCH() VR_CHECK_HIP(hipGetLastError())

#define VR_REQUIRE(cond, ...)     \
  do {                            \
    if (!(cond)) {                \
      vr::set_error(__VA_ARGS__); \
      return VR_EINVAL;           \
    }                             \
  } while (0)

#define VR_TRY(expr)          \
  do {                        \
    int rc_ = (expr);         \
    if (rc_ != VR_OK) return rc_; \
  } while (0)

// One-time setup (hipFuncSetAttribute of a kernel instantiation) run exactly once per
// process even when host threads enter together: a function-local static is initialised
// once under the C++11 guarantee, so the library stays thread-safe across distinct streams
// (SURVEY §8(b)). Every later call returns the first call's status.
#define VR_ONCE(...)                                                         \
  do {                                                                       \
    static const int once_rc_ = [&]() -> int { __VA_ARGS__; return VR_OK; }();\
    if (once_rc_ != VR_OK) return once_rc_;                                  \
  } while (0)
