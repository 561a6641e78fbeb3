// Internal (non-ABI) declarations shared between the .hip translation units.
#pragma once

#include "common.h"

namespace vr {

// ---- device-wide exclusive scan of uint32 (scan.hip) -------------------------------
constexpr int SCAN_BS = 256;
constexpr int SCAN_IPT = 16;
constexpr int SCAN_TILE = SCAN_BS * SCAN_IPT;
size_t scan_ws_elems(int64_t n);  // uint32 elements of scratch
// out[i] = sum(in[0:i]); *total_dev (if non-null) = sum(in). in may alias out.
int scan_exclusive_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev,
                       uint32_t* ws, hipStream_t st);

// ---- LSD radix sort of (uint32 key, uint32 value) pairs (sort.hip) -----------------
constexpr int RS_BS = 256;
#ifndef VR_RS_IPT
#define VR_RS_IPT 16
#endif
constexpr int RS_IPT = VR_RS_IPT;
constexpr int RS_TILE = RS_BS * RS_IPT;
// One LSD pass (8-bit digit at `shift`) of (ki, vi) into (ko, vo): the building block of
// radix_sort_kv, also the engine's partition of (B position, A position) pairs.
int radix_pass_kv(const uint32_t* ki, const uint32_t* vi, uint32_t* ko, uint32_t* vo, int64_t n,
                  int shift, uint32_t* ws, hipStream_t st);
size_t radix_ws_elems(int64_t n);  // uint32 elements of scratch (histograms + scan)
// The pass's offsets alone: ws[tile * 256 + d] = output position of tile `tile`'s first key
// of digit d (tiles of RS_TILE keys), for kernels that scatter their own records.
int radix_offsets(const uint32_t* ki, int64_t n, int shift, uint32_t* ws, hipStream_t st);
// One pass on keys alone (no values).
int radix_pass_k(const uint32_t* ki, uint32_t* ko, int64_t n, int shift, uint32_t* ws, hipStream_t st);
// Sorts ascending by key, stable. keys/vals hold the result; *_alt are ping-pong
// buffers of the same length.
int radix_sort_kv(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                  int64_t n, uint32_t* ws, hipStream_t st);

// ---- block-level helpers -----------------------------------------------------------
// Exclusive scan across a block of BS threads (BS multiple of 64, <= 1024).
// lds must hold BS/64 + 1 uint32. Returns this thread's exclusive prefix; total = sum.
template <int BS>
__device__ inline uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < BS / 64; ++w) {
      uint32_t t = lds[w];
      lds[w] = s;
      s += t;
    }
    lds[BS / 64] = s;
  }
  __syncthreads();
  uint32_t r = x - v + lds[wid];
  total = lds[BS / 64];
  __syncthreads();
  return r;
}

// Padded LDS index for tiles read both striped (lane-contiguous) and blocked (16
// consecutive per thread): one pad dword per 32 keeps both patterns conflict-free.
// Block -> work item for a 1-D grid of nb items such that the blocks one XCD receives
// (blockIdx % 8 equal, as the dispatcher deals them) take consecutive items: neighbouring
// items' partial-line writes then meet in one L2.
__device__ inline int64_t xcd_item(int64_t nb) {
  const int64_t b = blockIdx.x, x = b & 7, k = b >> 3, per = nb >> 3, rem = nb & 7;
  return x * per + (x < rem ? x : rem) + k;
}

__device__ inline int lds_pad(int p) { return p + (p >> 5); }

// Sortable transform of an fp32 value: ascending uint32 order == ascending float order,
// -0.0 canonicalised to +0.0 so the two tie (scipy.stats.rankdata semantics).
__device__ inline uint32_t f32_sort_key(float f) {
  uint32_t u = __float_as_uint(f);
  if (u == 0x80000000u) u = 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

}  // namespace vr

// ---- kernel-level HIP-event timing of the hot kernels (ktimer.cpp) -----------------
// Off by default (vr_ktimer_enable). A KtScope records an event on the launch stream
// before and after the one launch it brackets; vr_ktimer_read resolves them.
namespace vr {
enum KtKernel : int {
  KT_RANKB_EST = 0,   // k_rankB, EST forms over bootstrap subsets (EST 3; the probe forms 1/2)
  KT_RANKB_EXACT = 1, // k_rankB, exact chunk-base form (VISREPS_ENGINE_EST=0, flagged reruns)
  KT_RANKA = 2,       // k_rankA (both forms)
  KT_JOIN = 3,        // k_join / k_join_lo
  KT_GRAM_WIDE = 4,   // k_gram3p / k_gram3w (256^2 super-tiles)
  KT_GRAM_TILE = 5,   // k_gram3 / k_gram (128^2 tiles)
  KT_COUNTA = 6,      // k_countA
  KT_RANKB_FULL = 7,  // k_rankB on the pass holding the full stimulus set (EST 4 A side: EST 3 B walks)
  KT_KWALK = 8,       // k_kwalk: one Kendall stream walk (inversion level or tie stream) of one pass
  KT_COV = 9,         // k_cov: fp64 MFMA covariance / Gram tiles (PCA covariance, ridge kernel matrix)
  KT_JOIN4 = 10,      // k_join4: shared join of one B plan to up to 4 A plans (units = algorithmic bytes)
  KT_FULL_CORR = 11,  // k_full_corr: lane 0's shift sums of an EST 4 pass, per unit (4 B / pair streamed)
  KT_RANKB_GRID = 12,  // k_rankB_grid: one B plan x up to 4 regions, EST 3 (units: pairs x regions)
  KT_RANKB_GRIDX = 13, // k_rankB_gridx: the same in the exact chunk-base form (units: pairs x regions)
  KT_N = 14
};
bool ktimer_on();
struct KtScope {
  KtScope(int kernel, double units, hipStream_t st);  // units: pairs (engine) or FLOPs (Gram)
  ~KtScope();
  int kernel;
  double units;
  hipStream_t st;
  hipEvent_t e0 = nullptr;
};
}  // namespace vr
