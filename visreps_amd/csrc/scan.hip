// Device-wide exclusive scan of uint32: reduce-then-scan in three launches.
// Used for radix-sort digit offsets and for tie-group numbering of sorted triangles.
#include "internal.h"

namespace vr {

__global__ __launch_bounds__(SCAN_BS) void k_scan_reduce(const uint32_t* __restrict__ in,
                                                         int64_t n,
                                                         uint32_t* __restrict__ partial) {
  __shared__ uint32_t lds[SCAN_BS / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < SCAN_IPT; ++j) {
    int64_t i = base + (int64_t)j * SCAN_BS + threadIdx.x;  // striped: coalesced
    if (i < n) s += in[i];
  }
  uint32_t total;
  block_exclusive_scan<SCAN_BS>(s, lds, total);
  if (threadIdx.x == 0) partial[blockIdx.x] = total;
}

// One block scans the per-tile totals (any count; each thread owns a contiguous run).
__global__ __launch_bounds__(1024) void k_scan_partials(uint32_t* __restrict__ partial,
                                                       int64_t nb,
                                                       uint32_t* __restrict__ total_out) {
  __shared__ uint32_t lds[1024 / 64 + 1];
  const int64_t per = (nb + 1023) / 1024;
  const int64_t b0 = (int64_t)threadIdx.x * per;
  uint32_t s = 0;
  for (int64_t i = b0; i < b0 + per && i < nb; ++i) s += partial[i];
  uint32_t total;
  uint32_t run = block_exclusive_scan<1024>(s, lds, total);
  for (int64_t i = b0; i < b0 + per && i < nb; ++i) {
    uint32_t t = partial[i];
    partial[i] = run;
    run += t;
  }
  if (threadIdx.x == 0 && total_out) *total_out = total;
}

__global__ __launch_bounds__(SCAN_BS) void k_scan_down(const uint32_t* in, uint32_t* out,
                                                       int64_t n,
                                                       const uint32_t* __restrict__ partial) {
  __shared__ uint32_t lds[SCAN_BS / 64 + 1];
  __shared__ uint32_t tile[SCAN_TILE + SCAN_TILE / 32];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  // striped load into LDS, then each thread scans its 16 consecutive elements
#pragma unroll
  for (int j = 0; j < SCAN_IPT; ++j) {
    int64_t i = base + (int64_t)j * SCAN_BS + threadIdx.x;
    tile[lds_pad(j * SCAN_BS + threadIdx.x)] = (i < n) ? in[i] : 0u;
  }
  __syncthreads();
  uint32_t v[SCAN_IPT];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < SCAN_IPT; ++j) {
    v[j] = tile[lds_pad(threadIdx.x * SCAN_IPT + j)];
    s += v[j];
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan<SCAN_BS>(s, lds, total) + partial[blockIdx.x];
#pragma unroll
  for (int j = 0; j < SCAN_IPT; ++j) {
    tile[lds_pad(threadIdx.x * SCAN_IPT + j)] = run;
    run += v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SCAN_IPT; ++j) {
    int64_t i = base + (int64_t)j * SCAN_BS + threadIdx.x;
    if (i < n) out[i] = tile[lds_pad(j * SCAN_BS + threadIdx.x)];
  }
}

size_t scan_ws_elems(int64_t n) { return (size_t)((n + SCAN_TILE - 1) / SCAN_TILE) + 64; }

int scan_exclusive_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev,
                       uint32_t* ws, hipStream_t st) {
  if (n <= 0) {
    if (total_dev) VR_CHECK_HIP(hipMemsetAsync(total_dev, 0, sizeof(uint32_t), st));
    return VR_OK;
  }
  const int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  k_scan_reduce<<<(unsigned)nb, SCAN_BS, 0, st>>>(in, n, ws);
  VR_CHECK_LAUNCH();
  k_scan_partials<<<1, 1024, 0, st>>>(ws, nb, total_dev);
  VR_CHECK_LAUNCH();
  k_scan_down<<<(unsigned)nb, SCAN_BS, 0, st>>>(in, out, n, ws);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // namespace vr

// Trace markers: empty kernels whose dispatches bracket a region in a rocprofv3 kernel
// trace (bench.py marks its timed steps; scripts/check_timed_kernels.py reads them).
__global__ void k_trace_mark_begin(int) {}
__global__ void k_trace_mark_end(int) {}

extern "C" int vr_trace_mark(int begin, int tag, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (begin)
    k_trace_mark_begin<<<1, 64, 0, st>>>(tag);
  else
    k_trace_mark_end<<<1, 64, 0, st>>>(tag);
  VR_CHECK_LAUNCH();
  return VR_OK;
}
