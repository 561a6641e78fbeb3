// 64-position window machinery shared by the rank engines (engine.hip: Spearman,
// kendall.hip: Kendall tau-a).
//
// A pass evaluates up to 64 stimulus subsets at once: lane s of a wave is subset s and
// masks[x] bit s says whether stimulus x is in subset s. A stream of pair codes
// ((a << 16) | b, in some sorted order) is walked in windows of 64 positions: lane j
// loads the code of position w0 + j, ANDs the masks of its two stimuli, and a 64x64 bit
// transpose across the wave hands lane s the inclusion bits of all 64 positions for its
// subset. Per-window counts are then popcounts.
#pragma once

#include "plan.h"

namespace vr {

typedef unsigned __int128 u128;
typedef __int128 i128;

constexpr int LANES = 64;

__device__ inline uint32_t wave_uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ inline uint32_t readlane_u32(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// Uniform-address load through the constant address space: selected as SMEM (s_load).
template <typename T>
__device__ inline T sload(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}

__device__ inline uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}

#ifndef VR_FAST_XOR
#define VR_FAST_XOR 1  // lane exchanges of the transpose: 1: DPP (xor 1, 2), ds_swizzle (4, 8, 16), permlane32_swap (32);
                       // 2: DPP for 4, 8 and permlane16_swap for 16 (more VALU: measured slower); 0: ds_bpermute
#endif

// v from lane (lane ^ W). W = 1, 2: DPP quad_perm on the VALU (no LDS-pipe round trip);
// W = 4, 8, 16: ds_swizzle bit-mask mode (xor within 32 lanes, no address register);
// W = 32: v_permlane32_swap (gfx950) of v with itself: afterwards the first result holds
// [v(0..31), v(0..31)] and the second [v(32..63), v(32..63)] across the wave.
template <int W>
__device__ inline uint32_t xor_lane(uint32_t v, int lane) {
  if constexpr (!VR_FAST_XOR) {
    return (uint32_t)__shfl_xor((int)v, W);
  } else if constexpr (W == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return lane < 32 ? r[1] : r[0];
  } else if constexpr (W == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (W == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (W == 4 && VR_FAST_XOR >= 2) {
    // i ^ 4 = half-row mirror (7 - i in 8) of the quad mirror (3 - i in 4)
    const int m = __builtin_amdgcn_mov_dpp((int)v, 0x1B, 0xF, 0xF, false);  // quad_perm [3,2,1,0]
    return (uint32_t)__builtin_amdgcn_mov_dpp(m, 0x141, 0xF, 0xF, false);    // row_half_mirror
  } else if constexpr (W == 8 && VR_FAST_XOR >= 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  } else if constexpr (W == 16 && VR_FAST_XOR >= 2) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? r[0] : r[1];
  } else {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (W << 10) | 0x1F);  // and 0x1f, xor W
  }
}

template <int W>
__device__ inline uint64_t xor_lane64(uint64_t v, int lane) {
  const uint32_t lo = xor_lane<W>((uint32_t)v, lane);
  const uint32_t hi = xor_lane<W>((uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

template <int ST>
__device__ inline uint64_t transpose_stage(uint64_t x, int lane) {
  constexpr uint64_t K[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                             0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
  constexpr int w = 32 >> ST;
  const uint64_t p = xor_lane64<w>(x, lane);
  const uint64_t hi = (x & ~K[ST]) | ((p & ~K[ST]) >> w);  // lanes with bit w set
  const uint64_t lo = (x & K[ST]) | ((p & K[ST]) << w);
  // per-lane select on a lane-id bit: a v_cndmask pair on an SGPR-pair lane mask (no
  // 64-bit all-ones/zeros VGPR constants, which the walks' 64-VGPR budget had to spill)
  return ((lane >> (5 - ST)) & 1) ? hi : lo;
}

// Transpose forms (template argument XM of transpose64 / window_bits):
//   1: the 64-bit stages above;
//   2: half-word stages (one exchange, one per-lane rotate, one bit select per 32-bit half;
//      the w = 32 stage one permlane32_swap), per-lane stage constants rebuilt per call;
//   3: the same with the constants loop-invariant (the compiler keeps them in ~9 VGPRs).
// Defaults per walk (A side: count and rank walks; B side: the rank walks at their VGPR
// budget, where 2 measured no faster than 1; Kendall: the stream walks).
#ifndef VR_XPOSE_A
#define VR_XPOSE_A 3
#endif
#ifndef VR_XPOSE_B
#define VR_XPOSE_B 1
#endif
#ifndef VR_XPOSE_K
#define VR_XPOSE_K 3
#endif

// Stage ST >= 1 (w = 32 >> ST <= 16) on one 32-bit half: the stage's bit moves stay inside
// each half. A lane with lane bit w clear keeps its K bits and takes the partner's K bits
// shifted up by w; a lane with it set keeps its ~K bits and takes the partner's ~K bits
// shifted down by w. Rotating the partner's word right by sa = (set ? w : 32 - w) puts both
// in place (the wrapped bits land on the kept positions of K = ...0000 1111 patterns), and
// one bit select with Ml = K ^ F (F = all ones on set lanes) merges.
template <int ST>
__device__ inline void transpose_stage_h(uint32_t& lo, uint32_t& hi, int lane) {
  constexpr uint32_t K[6] = {0u, 0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
  constexpr int w = 32 >> ST;
  const uint32_t F = (uint32_t)__builtin_amdgcn_sbfe(lane, 5 - ST, 1);  // 0 or all ones
  const uint32_t Ml = K[ST] ^ F;
  const uint32_t sa = (F & (uint32_t)w) | (~F & (uint32_t)(32 - w));
  const uint32_t pl = xor_lane<w>(lo, lane), ph = xor_lane<w>(hi, lane);
  const uint32_t tl = __builtin_amdgcn_alignbit(pl, pl, sa), th = __builtin_amdgcn_alignbit(ph, ph, sa);
  lo = ((lo ^ tl) & Ml) ^ tl;  // one 3-input bit op per half
  hi = ((hi ^ th) & Ml) ^ th;
}

// 64x64 bit-matrix transpose across the wave: on entry bit s of lane j is element (j, s);
// on exit bit j of lane s is. Recursive block swap, 6 stages of one 64-bit exchange.
template <int XM>
__device__ inline uint64_t transpose64(uint64_t x, int lane) {
  static_assert(XM >= 1 && XM <= 3, "transpose form");
  if constexpr (XM == 1) {
    x = transpose_stage<0>(x, lane);
    x = transpose_stage<1>(x, lane);
    x = transpose_stage<2>(x, lane);
    x = transpose_stage<3>(x, lane);
    x = transpose_stage<4>(x, lane);
    return transpose_stage<5>(x, lane);
  }
  if constexpr (XM == 2) asm volatile("" : "+v"(lane));  // opaque per call: not loop-invariant
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  {  // w = 32: lanes 0-31 take lanes 32-63's low words as their high words and vice versa
    const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
    lo = r[0];
    hi = r[1];
  }
  transpose_stage_h<1>(lo, hi, lane);
  transpose_stage_h<2>(lo, hi, lane);
  transpose_stage_h<3>(lo, hi, lane);
  transpose_stage_h<4>(lo, hi, lane);
  transpose_stage_h<5>(lo, hi, lane);
  return ((uint64_t)hi << 32) | lo;
}

// the round-1 form (every exchange a ds_bpermute): kept for reference timing
__device__ inline uint64_t transpose64_bperm(uint64_t x, int lane) {
  constexpr uint64_t K[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                             0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
  for (int st = 0; st < 6; ++st) {
    const int w = 32 >> st;
    const uint64_t p = shfl_xor64(x, w);
    const uint64_t hi = (x & ~K[st]) | ((p & ~K[st]) >> w);  // lanes with bit w set
    const uint64_t lo = (x & K[st]) | ((p & K[st]) << w);
    const uint64_t sel = 0ull - (uint64_t)((lane >> (5 - st)) & 1);  // branch-free select
    x = (hi & sel) | (lo & ~sel);
  }
  return x;
}

__host__ __device__ inline uint64_t lowmask(uint32_t b) { return b >= 64 ? ~0ull : ((1ull << b) - 1ull); }

__device__ inline uint32_t popc64(uint64_t x) { return (uint32_t)__popcll(x); }

// Inclusion bits of the window for this lane's subset (bit j <-> position w0 + j), from
// the window's codes (lane j holds pair w0 + j).
template <int XM>
__device__ inline uint64_t window_bits(const uint64_t* m, uint32_t code, uint32_t w0, uint32_t P0,
                                       uint32_t P1, int lane, bool active) {
  const uint32_t pos = w0 + (uint32_t)lane;
  uint64_t x = 0;
  if (pos >= P0 && pos < P1) x = m[code >> 16] & m[code & 0xffffu];
  x = transpose64<XM>(x, lane);
  return active ? x : 0ull;
}

// The block's copy of the masks: LDS when they fit, else the global table itself.
template <bool LDS>
__device__ inline const uint64_t* stage_masks(const uint64_t* __restrict__ gmask, int64_t n,
                                              uint64_t* smem) {
  if (!LDS) return gmask;
  for (int64_t x = threadIdx.x; x < n; x += blockDim.x) smem[x] = gmask[x];
  __syncthreads();
  return smem;
}

// Inclusion masks of one pass: bit w of masks[x] <- stimulus x in subset (set0 + w),
// subset 0 being "all stimuli" when full_first; lanes >= nl stay empty. masks is zeroed
// first. idx rows hold k stimulus indices each (engine.hip).
int build_pass_masks(const int32_t* idx, int64_t k, int64_t set0, int nl, int full_first,
                     uint64_t* masks, int64_t n, hipStream_t st);

}  // namespace vr
