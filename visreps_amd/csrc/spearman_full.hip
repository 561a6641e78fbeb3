// Full-triangle Spearman without the rank plan's pair codes: the path of
// compute_rdm_correlation(.., "Spearman") (visreps/analysis/rsa.py:96-129: scipy spearmanr
// of the two strict upper triangles, average ranks for ties) for RDMs beyond the engine's
// 16-bit stimulus indices, up to M = n(n-1)/2 < 2^32 pairs (n <= 92681): the configs[2]
// 73k-stimulus RDM.
//
// Three forms, all exact integer statistics (bit-equal to each other and to the rank-plan
// engine). A triangle's fp32 sort keys lie in [kmin, kmax]; with cnt[v] the number of pairs of
// key kmin + v and cum its exclusive prefix sum, a pair's doubled midrank is
// cum[v] + cum[v + 1] + 1 and its tie group has cnt[v] members -- no sort is needed.
// Correlation-distance RDMs (values in [0, 2]) span at most 2^30 + 1 keys; typical ones
// (values in [0.25, 2)) about 2^24.6.
//   k_tab_range + k_tab_mm   key range and NaNs of both triangles (to the host), every form
// bucketed count tables (default; both ranges <= 2^26 keys): see k_cb_* below -- block
//   histograms of coarse key buckets, records written bucket by bucket, per-key counts in
//   LDS, one random 8-B table read per pair in the dot
// plain count tables (only when VISREPS_FULL_FORM=table names them):
//            k_tab_count    global-atomic counts of both triangles' keys
//            k_tab_ties + scan, k_tab_dot (two random table reads per pair)
// sort form (key ranges beyond 2^26 keys or the workspace, or VISREPS_FULL_FORM=sort):
//   per RDM  k_full_keys    (sortable fp32 key, triangle index t) of every pair
//            radix_sort_kv  by key (sort.hip; u32 offsets, M < 2^32)
//            k_tile_bounds  first / last tie-group start of every 4096-position tile
//            k_tile_carry   the group start before / after each tile (prefix max, suffix min)
//   A        k_y_side<0>    doubled midrank y = gs + ge + 1 from wave scans of the group
//                           starts, scattered to yA[t]; tie terms
//   B        k_y_side<1>    sum yB * yA[t] (u128); tie terms
// then k_full_final: rho from the exact integer sums (fp64 at the end only). With M pairs and
// doubled midranks, rho = (sum yA yB - M (M+1)^2) / sqrt(va vb),
// v = 4 M(M+1)(2M+1)/6 - T/3 - M (M+1)^2.
// k_group_flags_full / k_group_starts_full / midrank2 are the local pieces of the
// distributed global rank (analysis/distributed_spearman.py: sample sort over ranks).
#include "window.h"

#include <atomic>
#include <string>

namespace vr {

// grid (column blocks, row slots): rows a = blockIdx.y, + gridDim.y, ... (a 1-D grid of
// n * n / 256 blocks would exceed the 2^32 work-items a launch dimension can address)
__global__ void k_full_keys(const float* __restrict__ rdm, int64_t n, int64_t ld,
                            uint32_t* __restrict__ keys, uint32_t* __restrict__ tidx,
                            uint32_t* __restrict__ nan_flag) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t a = blockIdx.y; a < n; a += gridDim.y) {
    if (b <= a || b >= n) continue;
    const float v = rdm[a * ld + b];
    if (v != v) atomicOr(nan_flag, 1u);
    const uint64_t t = tri_index((uint64_t)a, (uint64_t)b, (uint64_t)n);
    keys[t] = f32_sort_key(v);
    tidx[t] = (uint32_t)t;
  }
}

// the sub-RDM A[idx][:, idx]'s strict upper triangle (evals.py:362-364's `A[idx][:, idx]`, never
// materialised): pair (a, b), a < b of the k subset rows, value rdm[idx[a] * ld + idx[b]], at
// its triangle index in the k x k sub-RDM
__global__ void k_full_keys_sub(const float* __restrict__ rdm, const int32_t* __restrict__ idx, int64_t k,
                                int64_t ld, uint32_t* __restrict__ keys, uint32_t* __restrict__ tidx,
                                uint32_t* __restrict__ nan_flag) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= k) return;
  const int64_t cb = idx[b];
  for (int64_t a = blockIdx.y; a < b; a += gridDim.y) {
    const float v = rdm[(int64_t)idx[a] * ld + cb];
    if (v != v) atomicOr(nan_flag, 1u);
    const uint64_t t = tri_index((uint64_t)a, (uint64_t)b, (uint64_t)k);
    keys[t] = f32_sort_key(v);
    tidx[t] = (uint32_t)t;
  }
}

__global__ void k_group_flags_full(const uint32_t* __restrict__ keys, int64_t M,
                                   uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  flags[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ void k_group_starts_full(const uint32_t* __restrict__ flags,
                                    const uint32_t* __restrict__ gidx, int64_t M,
                                    uint32_t* __restrict__ gstart) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  if (flags[i]) gstart[gidx[i]] = (uint32_t)i;
  if (i == M - 1) gstart[gidx[i] + flags[i]] = (uint32_t)M;
}

// doubled midrank of sorted position i, its group's size (k) and whether it opens the group
__device__ inline uint64_t midrank2(const uint32_t* flags, const uint32_t* gidx,
                                    const uint32_t* gstart, int64_t i, uint64_t& k) {
  const uint32_t g = gidx[i] + flags[i] - 1u;
  const uint64_t gs = gstart[g], ge = gstart[g + 1];
  k = ge - gs;
  return gs + ge + 1u;
}

constexpr int FULL_BS = 256;

// block sum of a u128 (as two u64 words) into part[blockIdx.x]
__device__ inline void block_sum_u128(u128 v, uint64_t* part, int slot, int nslots) {
  __shared__ uint64_t lo[FULL_BS], hi[FULL_BS];
  lo[threadIdx.x] = (uint64_t)v;
  hi[threadIdx.x] = (uint64_t)(v >> 64);
  __syncthreads();
  if (threadIdx.x == 0) {
    u128 s = 0;
    for (int j = 0; j < FULL_BS; ++j) s += ((u128)hi[j] << 64) | lo[j];
    part[((size_t)blockIdx.x * nslots + slot) * 2] = (uint64_t)s;
    part[((size_t)blockIdx.x * nslots + slot) * 2 + 1] = (uint64_t)(s >> 64);
  }
  __syncthreads();
}

// block sum of a u128 into dst[0..1] (lo, hi)
__device__ inline void block_sum_u128_to(u128 v, uint64_t* dst) {
  __shared__ uint64_t lo[FULL_BS], hi[FULL_BS];
  lo[threadIdx.x] = (uint64_t)v;
  hi[threadIdx.x] = (uint64_t)(v >> 64);
  __syncthreads();
  if (threadIdx.x == 0) {
    u128 s = 0;
    for (int j = 0; j < FULL_BS; ++j) s += ((u128)hi[j] << 64) | lo[j];
    dst[0] = (uint64_t)s;
    dst[1] = (uint64_t)(s >> 64);
  }
}

constexpr uint32_t NONE32 = 0xFFFFFFFFu;

__device__ inline uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = max(x, (uint32_t)__shfl_xor(x, o, 64));
  return x;
}
__device__ inline uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = min(x, (uint32_t)__shfl_xor(x, o, 64));
  return x;
}

// first[T] = smallest group start among tile T's sorted positions (NONE32: none),
// lastp1[T] = largest group start + 1 (0: none). A group starts where the key changes.
__global__ __launch_bounds__(RS_BS) void k_tile_bounds(const uint32_t* __restrict__ keys, int64_t M,
                                                       uint32_t* __restrict__ first,
                                                       uint32_t* __restrict__ lastp1) {
  __shared__ uint32_t smn[RS_BS / 64], smx[RS_BS / 64];
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  uint32_t mn = NONE32, mx = 0;
#pragma unroll 4
  for (int j = 0; j < RS_IPT; ++j) {
    const int64_t i = base + j * RS_BS + threadIdx.x;
    if (i < M && (i == 0 || keys[i] != keys[i - 1])) {
      mn = min(mn, (uint32_t)i);
      mx = max(mx, (uint32_t)(i + 1));
    }
  }
  mn = wave_min_u32(mn);
  mx = wave_max_u32(mx);
  if ((threadIdx.x & 63) == 0) {
    smn[threadIdx.x >> 6] = mn;
    smx[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 1; q < RS_BS / 64; ++q) {
      mn = min(mn, smn[q]);
      mx = max(mx, smx[q]);
    }
    first[blockIdx.x] = mn;
    lastp1[blockIdx.x] = mx;
  }
}

// One block: lastp1[T] := max over tiles before T (the last group start before the tile, + 1);
// first[T] := min over tiles after T, or M (the first group start after the tile).
__global__ __launch_bounds__(1024) void k_tile_carry(uint32_t* __restrict__ first,
                                                     uint32_t* __restrict__ lastp1, int64_t nt,
                                                     uint32_t M) {
  __shared__ uint32_t smx[1024], smn[1024];
  const int t = threadIdx.x;
  const int64_t per = (nt + 1023) / 1024, t0 = t * per, t1 = t0 + per < nt ? t0 + per : nt;
  uint32_t mx = 0, mn = NONE32;
  for (int64_t T = t0; T < t1; ++T) {
    mx = max(mx, lastp1[T]);
    mn = min(mn, first[T]);
  }
  smx[t] = mx;
  smn[t] = mn;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive prefix max, inclusive suffix min
    const uint32_t a = t >= o ? smx[t - o] : 0u;
    const uint32_t b = t + o < 1024 ? smn[t + o] : NONE32;
    __syncthreads();
    smx[t] = max(smx[t], a);
    smn[t] = min(smn[t], b);
    __syncthreads();
  }
  uint32_t run = t > 0 ? smx[t - 1] : 0u;
  for (int64_t T = t0; T < t1; ++T) {
    const uint32_t x = lastp1[T];
    lastp1[T] = run;
    run = max(run, x);
  }
  run = min(t < 1023 ? smn[t + 1] : NONE32, M);
  for (int64_t T = t1 - 1; T >= t0; --T) {
    const uint32_t x = first[T];
    first[T] = run;
    run = min(run, x);
  }
}

// One tile of sorted positions (grid = tiles, xcd_item order): doubled midrank
// y = gs + ge + 1 of every position, with gs the group start at or before it (an inclusive
// max-scan of start + 1 over the wave's 16 rounds of 64) and ge the next start after it (an
// exclusive suffix-min); waves and tiles before / after fill what the wave itself does not
// close (k_tile_carry). A side (DOT false): yA[t] = y. B side: sum y * yA[t]. Both: the tie
// term sum (k^3 - k) at every group start. Partials per tile (lo, hi words).
template <bool DOT>
__global__ __launch_bounds__(RS_BS) void k_y_side(
    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ tidx, int64_t M, int64_t nt,
    const uint32_t* __restrict__ cgs, const uint32_t* __restrict__ cge, uint64_t* __restrict__ yA,
    uint64_t* __restrict__ tiepart, uint64_t* __restrict__ dotpart) {
  constexpr int NW = RS_BS / 64, WT = RS_TILE / NW;
  __shared__ uint32_t wlast[NW], wfirst[NW];
  __shared__ uint64_t red[2][2][NW];

  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int64_t tile = xcd_item(nt);
  const int64_t base = tile * RS_TILE;
  const int64_t left = M - base;
  const int nvalid = left < RS_TILE ? (int)left : RS_TILE;
  uint32_t tk[RS_IPT], gs[RS_IPT], ge[RS_IPT];
  uint32_t fl = 0, carry = 0;
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    const int p = w * WT + j * 64 + lane;
    const int64_t i = base + p;
    const bool valid = p < nvalid;
    bool f = true;
    tk[j] = 0;
    if (valid) {
      tk[j] = tidx[i];
      f = i == 0 || keys[i] != keys[i - 1];
    }
    fl |= (uint32_t)f << j;
    uint32_t x = (f && valid) ? (uint32_t)(i + 1) : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x = max(x, y);
    }
    x = max(x, carry);
    carry = __shfl(x, 63, 64);
    gs[j] = x;
  }
  uint32_t back = NONE32;
#pragma unroll
  for (int j = RS_IPT - 1; j >= 0; --j) {
    const int p = w * WT + j * 64 + lane;
    uint32_t x = ((fl >> j) & 1u) ? (p < nvalid ? (uint32_t)(base + p) : (uint32_t)M) : NONE32;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_down(x, o, 64);
      if (lane + o < 64) x = min(x, y);
    }
    x = min(x, back);
    const uint32_t nx = __shfl_down(x, 1, 64);
    ge[j] = lane < 63 ? nx : back;
    back = __shfl(x, 0, 64);
  }
  if (lane == 0) {
    wlast[w] = carry;
    wfirst[w] = back;
  }
  __syncthreads();
  uint32_t gs_in = cgs[tile], ge_in = cge[tile];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    if (q < w) gs_in = max(gs_in, wlast[q]);
    if (q > w) ge_in = min(ge_in, wfirst[q]);
  }
  u128 tie = 0, ab = 0;
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    if (w * WT + j * 64 + lane >= nvalid) continue;
    const uint32_t s = (gs[j] ? gs[j] : gs_in) - 1u;
    const uint32_t e = ge[j] != NONE32 ? ge[j] : ge_in;
    const uint64_t y = (uint64_t)s + e + 1u;
    if (DOT)
      ab += (u128)y * yA[tk[j]];
    else
      yA[tk[j]] = y;
    if ((fl >> j) & 1u) {
      const uint64_t k = (uint64_t)(e - s);
      tie += (u128)(k * k) * k - k;
    }
  }
  // block sums of tie (and ab)
#pragma unroll
  for (int v = 0; v < (DOT ? 2 : 1); ++v) {
    const u128 x = v ? ab : tie;
    uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const uint64_t l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
      const uint64_t s = lo + l2;
      hi += h2 + (s < lo ? 1u : 0u);
      lo = s;
    }
    if (lane == 0) {
      red[v][0][w] = lo;
      red[v][1][w] = hi;
    }
  }
  __syncthreads();
  if (t < (DOT ? 2 : 1)) {
    u128 sum = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) sum += ((u128)red[t][1][q] << 64) | red[t][0][q];
    uint64_t* part = t ? dotpart : tiepart;
    part[2 * tile] = (uint64_t)sum;
    part[2 * tile + 1] = (uint64_t)(sum >> 64);
  }
}

// one block: out[0..1] = sum of the n u128 partials in part
__global__ __launch_bounds__(FULL_BS) void k_reduce_u128(const uint64_t* __restrict__ part, int64_t n,
                                                         uint64_t* __restrict__ out) {
  u128 s = 0;
  for (int64_t b = threadIdx.x; b < n; b += FULL_BS) s += ((u128)part[2 * b + 1] << 64) | part[2 * b];
  block_sum_u128(s, out, 0, 1);
}

// ---------------------------------------------------------------------------------
// Count-table form (no sort). A triangle's values are fp32 keys in [kmin, kmax]; with
// cnt[v] = number of pairs of key kmin + v and cum its exclusive prefix sum, the doubled
// midrank of a pair of key kmin + v is cum[v] + cum[v + 1] + 1 (group start + group end + 1)
// and its tie group has cnt[v] members. Correlation-distance RDMs (values in [0, 2]) span at
// most 2^30 + 1 keys, so both tables fit a few GB at any n; a pass over the two triangles
// counts (global atomics into tables that the L2 / MALL hold for the usual value spread), a
// scan turns counts into starts, and a second pass sums yA * yB. No per-pair arrays.
// ---------------------------------------------------------------------------------
// (a, b) visit of the strict upper triangle (SUB: of the sub-RDM at rows / columns idx)
template <bool SUB>
__device__ inline float tri_value(const float* rdm, const int32_t* idx, int64_t ld, int64_t a, int64_t b) {
  return SUB ? rdm[(int64_t)idx[a] * ld + idx[b]] : rdm[a * ld + b];
}

// per block [min A, max A, min B, max B] of the keys (k_tab_mm folds them); nan[0 / 1]: a NaN in A / B
template <bool SUB>
__global__ __launch_bounds__(256) void k_tab_range(const float* __restrict__ A, const float* __restrict__ B,
                                                   const int32_t* __restrict__ idx, int64_t n, int64_t ld,
                                                   uint32_t* __restrict__ mmpart, uint32_t* __restrict__ nan) {
  __shared__ uint32_t red[4][4];
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t mnA = NONE32, mxA = 0, mnB = NONE32, mxB = 0, bad = 0;
  if (b < n) {
    for (int64_t a = blockIdx.y; a < b; a += gridDim.y) {
      const float va = tri_value<SUB>(A, idx, ld, a, b), vb = tri_value<SUB>(B, idx, ld, a, b);
      bad |= (va != va ? 1u : 0u) | (vb != vb ? 2u : 0u);
      const uint32_t ka = f32_sort_key(va), kb = f32_sort_key(vb);
      mnA = min(mnA, ka);
      mxA = max(mxA, ka);
      mnB = min(mnB, kb);
      mxB = max(mxB, kb);
    }
  }
  mnA = wave_min_u32(mnA);
  mxA = wave_max_u32(mxA);
  mnB = wave_min_u32(mnB);
  mxB = wave_max_u32(mxB);
  bad = wave_max_u32(bad & 1u) | (wave_max_u32(bad & 2u));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = mnA;
    red[w][1] = mxA;
    red[w][2] = mnB;
    red[w][3] = mxB;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int c = threadIdx.x;
    uint32_t v = red[0][c];
#pragma unroll
    for (int q = 1; q < 4; ++q) v = (c & 1) ? max(v, red[q][c]) : min(v, red[q][c]);
    mmpart[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + c] = v;
  }
  if (threadIdx.x == 0 && bad) {
    if (bad & 1u) atomicOr(&nan[0], 1u);
    if (bad & 2u) atomicOr(&nan[1], 1u);
  }
}

__global__ __launch_bounds__(1024) void k_tab_mm(const uint32_t* __restrict__ mmpart, int64_t nblk,
                                                  uint32_t* __restrict__ mm) {
  __shared__ uint32_t red[16][4];
  uint32_t v[4] = {NONE32, 0u, NONE32, 0u};
  for (int64_t b = threadIdx.x; b < nblk; b += 1024) {
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = (c & 1) ? max(v[c], mmpart[4 * b + c]) : min(v[c], mmpart[4 * b + c]);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = (c & 1) ? wave_max_u32(v[c]) : wave_min_u32(v[c]);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int c = 0; c < 4; ++c) red[w][c] = v[c];
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int c = threadIdx.x;
    uint32_t x = red[0][c];
    for (int q = 1; q < 16; ++q) x = (c & 1) ? max(x, red[q][c]) : min(x, red[q][c]);
    mm[c] = x;
  }
}

template <bool SUB>
__global__ __launch_bounds__(256) void k_tab_count(const float* __restrict__ A, const float* __restrict__ B,
                                                   const int32_t* __restrict__ idx, int64_t n, int64_t ld,
                                                   const uint32_t* __restrict__ mm, uint32_t* __restrict__ cA,
                                                   uint32_t* __restrict__ cB) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const uint32_t a0 = mm[0], b0 = mm[2];
  for (int64_t a = blockIdx.y; a < b; a += gridDim.y) {
    atomicAdd(&cA[f32_sort_key(tri_value<SUB>(A, idx, ld, a, b)) - a0], 1u);
    atomicAdd(&cB[f32_sort_key(tri_value<SUB>(B, idx, ld, a, b)) - b0], 1u);
  }
}

// tie term sum (c^3 - c) of a count table (before its scan)
__global__ __launch_bounds__(FULL_BS) void k_tab_ties(const uint32_t* __restrict__ cnt, int64_t bins,
                                                      uint64_t* __restrict__ part) {
  u128 s = 0;
  for (int64_t v = (int64_t)blockIdx.x * FULL_BS + threadIdx.x; v < bins; v += (int64_t)gridDim.x * FULL_BS) {
    const uint64_t c = cnt[v];
    if (c > 1) s += (u128)(c * c) * c - c;
  }
  block_sum_u128(s, part, 0, 1);
}

template <bool SUB>
__global__ __launch_bounds__(256) void k_tab_dot(const float* __restrict__ A, const float* __restrict__ B,
                                                 const int32_t* __restrict__ idx, int64_t n, int64_t ld,
                                                 const uint32_t* __restrict__ mm, const uint32_t* __restrict__ sA,
                                                 const uint32_t* __restrict__ sB, uint64_t* __restrict__ part) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t a0 = mm[0], b0 = mm[2];
  u128 ab = 0;
  if (b < n) {
    for (int64_t a = blockIdx.y; a < b; a += gridDim.y) {
      const uint32_t ka = f32_sort_key(tri_value<SUB>(A, idx, ld, a, b)) - a0;
      const uint32_t kb = f32_sort_key(tri_value<SUB>(B, idx, ld, a, b)) - b0;
      const uint64_t ya = (uint64_t)sA[ka] + sA[ka + 1] + 1u, yb = (uint64_t)sB[kb] + sB[kb + 1] + 1u;
      ab += (u128)ya * yb;
    }
  }
  block_sum_u128_to(ab, part + 2 * ((int64_t)blockIdx.y * gridDim.x + blockIdx.x));
}

// ---------------------------------------------------------------------------------
// Bucketed count-table form (the default when both key ranges are at most 2^26 keys): the
// key offsets k - kmin split into at most 4096 coarse buckets of W = 2^sh <= 16384 keys.
//   k_cb_keys   both triangles' key offsets in triangle order (kA[t], kB[t])
//   radix       B's offsets ordered by bucket (keys only), then A's (kA, kB) pairs by A's
//               bucket: one or two 8-bit LSD passes each (sort.hip: coalesced digit runs)
//   k_cb_bstart bucket starts of each ordered array
//   k_cb_fine   counts per key: runs of one bucket counted in LDS (W counters) and added to
//               the table once per block; short runs count in global memory
//   k_cb_dot    sum yA * yB over A's ordered pairs: A's table reads stay inside one bucket's
//               window (cached), B's are one random 8-B read per pair
// ---------------------------------------------------------------------------------
constexpr int CB_MAXB = 4096;  // coarse buckets per RDM (cb_geom: 12 bits)
static_assert(CB_MAXB == 1 << 12, "cb_geom splits the key range into 2^12 buckets at most");
constexpr int CB_MAXSH = 14;   // keys per bucket <= 2^14 (64 KB of LDS counters)

// grid (column blocks, row slots) as k_full_keys
template <bool SUB>
__global__ void k_cb_keys(const float* __restrict__ A, const float* __restrict__ B, const int32_t* __restrict__ idx,
                          int64_t n, int64_t ld, const uint32_t* __restrict__ mm, uint32_t* __restrict__ kA,
                          uint32_t* __restrict__ kB) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const uint32_t a0 = mm[0], b0 = mm[2];
  for (int64_t a = blockIdx.y; a < b; a += gridDim.y) {
    const uint64_t t = tri_index((uint64_t)a, (uint64_t)b, (uint64_t)n);
    kA[t] = f32_sort_key(tri_value<SUB>(A, idx, ld, a, b)) - a0;
    kB[t] = f32_sort_key(tri_value<SUB>(B, idx, ld, a, b)) - b0;
  }
}

// bstart[g] = first position of bucket g in keys ordered by bucket (empty buckets: the next
// bucket's start), bstart[nb] = M
__global__ void k_cb_bstart(const uint32_t* __restrict__ keys, int64_t M, int sh, int nb,
                            uint32_t* __restrict__ bstart) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const int g = (int)(keys[i] >> sh);
  const int gp = i > 0 ? (int)(keys[i - 1] >> sh) : -1;
  for (int x = gp + 1; x <= g; ++x) bstart[x] = (uint32_t)i;
  if (i == M - 1)
    for (int x = g + 1; x <= nb; ++x) bstart[x] = (uint32_t)M;
}

// one key per bucket (sh = 0): the counts are the bucket sizes
__global__ void k_cb_sizes(const uint32_t* __restrict__ bstart, int nb, uint32_t* __restrict__ cnt) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < nb) cnt[g] = bstart[g + 1] - bstart[g];
}

constexpr int CB_FINE_BS = 1024;
constexpr int64_t CB_SEG = (int64_t)1 << 21;  // records per k_cb_fine block
constexpr int64_t CB_LDS_RUN = 2048;          // shorter runs count in global memory

// counts of one side's key offsets (recA's low words: STRIDE 2; recB: 1), grouped by bucket
template <int STRIDE>
__global__ __launch_bounds__(CB_FINE_BS) void k_cb_fine(const uint32_t* __restrict__ off, int64_t M,
                                                        const uint32_t* __restrict__ bstart, int nb, int sh,
                                                        uint32_t* __restrict__ cnt) {
  __shared__ uint32_t lc[1 << CB_MAXSH];
  const int64_t s0 = (int64_t)blockIdx.x * CB_SEG, s1 = s0 + CB_SEG < M ? s0 + CB_SEG : M;
  const int W = 1 << sh;
  int lo = 0, hi = nb;  // first bucket whose end lies beyond s0
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)bstart[mid + 1] <= s0) lo = mid + 1; else hi = mid;
  }
  for (int bk = lo; bk < nb && (int64_t)bstart[bk] < s1; ++bk) {
    const int64_t r0 = max(s0, (int64_t)bstart[bk]), r1 = min(s1, (int64_t)bstart[bk + 1]);
    if (r1 <= r0) continue;
    if (r1 - r0 < CB_LDS_RUN || W == 1) {
      for (int64_t p = r0 + threadIdx.x; p < r1; p += CB_FINE_BS) atomicAdd(&cnt[off[p * STRIDE]], 1u);
      continue;
    }
    for (int f = threadIdx.x; f < W; f += CB_FINE_BS) lc[f] = 0;
    __syncthreads();
    for (int64_t p = r0 + threadIdx.x; p < r1; p += CB_FINE_BS) atomicAdd(&lc[off[p * STRIDE] & (W - 1)], 1u);
    __syncthreads();
    uint32_t* dst = cnt + ((int64_t)bk << sh);
    for (int f = threadIdx.x; f < W; f += CB_FINE_BS) {
      const uint32_t c = lc[f];
      if (c) atomicAdd(&dst[f], c);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(FULL_BS) void k_cb_dot(const uint32_t* __restrict__ kA, const uint32_t* __restrict__ kB,
                                                    int64_t M, const uint32_t* __restrict__ sA,
                                                    const uint32_t* __restrict__ sB, uint64_t* __restrict__ part) {
  u128 ab = 0;
  for (int64_t p = (int64_t)blockIdx.x * FULL_BS + threadIdx.x; p < M; p += (int64_t)gridDim.x * FULL_BS) {
    const uint32_t ka = kA[p], kb = kB[p];
    const uint64_t ya = (uint64_t)sA[ka] + sA[ka + 1] + 1u, yb = (uint64_t)sB[kb] + sB[kb + 1] + 1u;
    ab += (u128)ya * yb;
  }
  block_sum_u128(ab, part, 0, 1);
}

__device__ inline double i128_to_f64_full(i128 x) {
  const bool neg = x < 0;
  const u128 u = neg ? (u128)(-x) : (u128)x;
  const double d = (double)(uint64_t)(u >> 64) * 18446744073709551616.0 + (double)(uint64_t)u;
  return neg ? -d : d;
}

// sums: [tie A, tie B, sum yA yB] as u128 (lo, hi)
__global__ void k_full_final(const uint64_t* __restrict__ sums, int64_t M,
                             const uint32_t* __restrict__ nan_flag, double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const u128 tA = ((u128)sums[1] << 64) | sums[0];
  const u128 tB = ((u128)sums[3] << 64) | sums[2];
  const u128 ab = ((u128)sums[5] << 64) | sums[4];
  const u128 Mp = (u128)M;
  const u128 mu = Mp * (Mp + 1) * (Mp + 1);
  const u128 sq = 4 * (Mp * (Mp + 1) * (2 * Mp + 1) / 6);
  const i128 num = (i128)ab - (i128)mu;
  const i128 va = (i128)(sq - tA / 3) - (i128)mu;
  const i128 vb = (i128)(sq - tB / 3) - (i128)mu;
  double r;
  if (nan_flag[0] || nan_flag[1] || M < 2 || va <= 0 || vb <= 0) {
    r = __builtin_nan("");
  } else {
    r = i128_to_f64_full(num) / sqrt(i128_to_f64_full(va) * i128_to_f64_full(vb));
    r = r > 1.0 ? 1.0 : (r < -1.0 ? -1.0 : r);
  }
  *out = r;
}

static int full_grid() { return num_cus() * 8; }

struct FullWs {
  uint32_t *keys, *tidx, *keys_alt, *tidx_alt, *first, *lastp1, *radix;
  uint64_t *yA, *tiepart, *dotpart;
  int64_t nt;
};

// the sort form's arrays, after the common header (TabHead)
static FullWs full_layout(Carver& c, int64_t n) {
  const int64_t M = pairs_of(n);
  FullWs w;
  w.nt = (M + RS_TILE - 1) / RS_TILE;
  w.keys = c.take<uint32_t>((size_t)M);
  w.tidx = c.take<uint32_t>((size_t)M);
  w.keys_alt = c.take<uint32_t>((size_t)M);
  w.tidx_alt = c.take<uint32_t>((size_t)M);
  w.first = c.take<uint32_t>((size_t)w.nt);
  w.lastp1 = c.take<uint32_t>((size_t)w.nt);
  w.radix = c.take<uint32_t>(radix_ws_elems(M));
  w.yA = c.take<uint64_t>((size_t)M);
  w.tiepart = c.take<uint64_t>((size_t)w.nt * 2);
  w.dotpart = c.take<uint64_t>((size_t)w.nt * 2);
  return w;
}

// triangle passes: (column blocks of 256, row slots)
static dim3 tri_grid(int64_t n) {
  return dim3((unsigned)((n + 255) / 256), (unsigned)std::max<int64_t>(1, std::min<int64_t>(n, 1024)));
}

// header of both forms: key range, NaN flags, per-block partials, the three u128 sums
struct TabHead {
  uint32_t *mm, *nan, *mmpart;
  uint64_t *part, *sums;
  int64_t nblk;
};

static TabHead head_layout(Carver& c, int64_t n) {
  TabHead h;
  const dim3 g = tri_grid(n);
  h.nblk = (int64_t)g.x * g.y;
  h.mm = c.take<uint32_t>(8);  // [min A, max A, min B, max B, NaN in A, NaN in B]: one copy to the host
  h.nan = h.mm + 4;
  h.mmpart = c.take<uint32_t>((size_t)h.nblk * 4);
  h.part = c.take<uint64_t>((size_t)std::max<int64_t>(h.nblk, full_grid()) * 2);
  h.sums = c.take<uint64_t>(6);
  return h;
}

// count tables of binsA / binsB keys (+ 1 each: the scan's end entry)
static size_t tab_bytes(int64_t n, uint64_t binsA, uint64_t binsB) {
  Carver c(nullptr);
  head_layout(c, n);
  c.take<uint32_t>(scan_ws_elems((int64_t)std::max(binsA, binsB) + 1));
  c.take<uint32_t>((size_t)binsA + 1);
  c.take<uint32_t>((size_t)binsB + 1);
  return c.bytes();
}

static size_t sort_bytes(int64_t n) {
  Carver c(nullptr);
  head_layout(c, n);
  full_layout(c, n);
  return c.bytes();
}

// a correlation-distance RDM's values lie in [0, 2]: keys 0x80000000 .. 0xC0000000
constexpr uint64_t TAB_CAP = ((uint64_t)1 << 30) + 1;

// form of the last call (0 bucketed tables, 1 tables, 2 sort): vr_spearman_full_last_form
static std::atomic<int> g_full_form{-1};

// bucketed form: coarse buckets of W = 2^sh keys (at most CB_MAXB of them)
struct CbGeom {
  int sh, nb;
  uint64_t tab;  // table entries nb << sh (>= the key range)
};
static CbGeom cb_geom(uint64_t R) {
  int bits = 0;
  while (bits < 40 && ((R - 1) >> bits) != 0) ++bits;
  const int sh = bits > 12 ? bits - 12 : 0;
  const int nb = (int)(((R - 1) >> sh) + 1);
  return CbGeom{sh, nb, (uint64_t)nb << sh};
}
constexpr uint64_t CB_CAP = (uint64_t)1 << (12 + CB_MAXSH);  // 2^26 keys

struct CbWs {
  uint32_t *sw, *cA, *cB, *bsA, *bsB, *radix;
  uint32_t* k[5];  // key arrays (triangle order, then the radix passes' outputs)
};

static CbWs cb_layout(Carver& c, int64_t n, const CbGeom& ga, const CbGeom& gb) {
  const int64_t M = pairs_of(n);
  CbWs w;
  w.sw = c.take<uint32_t>(scan_ws_elems((int64_t)std::max(ga.tab, gb.tab) + 1));
  w.cA = c.take<uint32_t>((size_t)ga.tab + 1);
  w.cB = c.take<uint32_t>((size_t)gb.tab + 1);
  w.bsA = c.take<uint32_t>((size_t)ga.nb + 1);
  w.bsB = c.take<uint32_t>((size_t)gb.nb + 1);
  w.radix = c.take<uint32_t>(radix_ws_elems(M));
  for (int i = 0; i < 5; ++i) w.k[i] = c.take<uint32_t>((size_t)M);
  return w;
}

static size_t cb_bytes(int64_t n, uint64_t RA, uint64_t RB) {
  Carver c(nullptr);
  head_layout(c, n);
  cb_layout(c, n, cb_geom(RA), cb_geom(RB));
  return c.bytes();
}

// sort form, one RDM: keys sorted, tile group bounds and carries
static int full_sorted(const float* rdm, int64_t n, int64_t ld, const FullWs& w, uint32_t* nan,
                       hipStream_t st, const int32_t* idx) {
  const int64_t M = pairs_of(n);
  const dim3 grid((unsigned)((n + 255) / 256), (unsigned)std::min<int64_t>(n, 16384));
  if (idx)
    k_full_keys_sub<<<grid, 256, 0, st>>>(rdm, idx, n, ld, w.keys, w.tidx, nan);
  else
    k_full_keys<<<grid, 256, 0, st>>>(rdm, n, ld, w.keys, w.tidx, nan);
  VR_CHECK_LAUNCH();
  VR_TRY(radix_sort_kv(w.keys, w.tidx, w.keys_alt, w.tidx_alt, M, w.radix, st));
  k_tile_bounds<<<(unsigned)w.nt, RS_BS, 0, st>>>(w.keys, M, w.first, w.lastp1);
  VR_CHECK_LAUNCH();
  k_tile_carry<<<1, 1024, 0, st>>>(w.first, w.lastp1, w.nt, (uint32_t)M);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

static int full_sort_form(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                          const TabHead& h, const FullWs& w, hipStream_t st) {
  const int64_t M = pairs_of(n);
  VR_TRY(full_sorted(A, n, ld, w, h.nan, st, idx));
  k_y_side<false><<<(unsigned)w.nt, RS_BS, 0, st>>>(w.keys, w.tidx, M, w.nt, w.lastp1, w.first, w.yA,
                                                    w.tiepart, nullptr);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(w.tiepart, w.nt, h.sums);
  VR_CHECK_LAUNCH();
  VR_TRY(full_sorted(B, n, ld, w, h.nan + 1, st, idx));
  k_y_side<true><<<(unsigned)w.nt, RS_BS, 0, st>>>(w.keys, w.tidx, M, w.nt, w.lastp1, w.first, w.yA,
                                                   w.tiepart, w.dotpart);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(w.tiepart, w.nt, h.sums + 2);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(w.dotpart, w.nt, h.sums + 4);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

template <bool SUB>
static int full_tab_form(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                         const TabHead& h, uint64_t binsA, uint64_t binsB, Carver& c, hipStream_t st) {
  uint32_t* sw = c.take<uint32_t>(scan_ws_elems((int64_t)std::max(binsA, binsB) + 1));
  uint32_t* cA = c.take<uint32_t>((size_t)binsA + 1);
  uint32_t* cB = c.take<uint32_t>((size_t)binsB + 1);
  VR_CHECK_HIP(hipMemsetAsync(cA, 0, (binsA + 1) * sizeof(uint32_t), st));
  VR_CHECK_HIP(hipMemsetAsync(cB, 0, (binsB + 1) * sizeof(uint32_t), st));
  const dim3 g = tri_grid(n);
  k_tab_count<SUB><<<g, 256, 0, st>>>(A, B, idx, n, ld, h.mm, cA, cB);
  VR_CHECK_LAUNCH();
  const int fg = full_grid();
  k_tab_ties<<<fg, FULL_BS, 0, st>>>(cA, (int64_t)binsA, h.part);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(h.part, fg, h.sums);
  VR_CHECK_LAUNCH();
  k_tab_ties<<<fg, FULL_BS, 0, st>>>(cB, (int64_t)binsB, h.part);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(h.part, fg, h.sums + 2);
  VR_CHECK_LAUNCH();
  VR_TRY(scan_exclusive_u32(cA, cA, (int64_t)binsA + 1, nullptr, sw, st));
  VR_TRY(scan_exclusive_u32(cB, cB, (int64_t)binsB + 1, nullptr, sw, st));
  k_tab_dot<SUB><<<g, 256, 0, st>>>(A, B, idx, n, ld, h.mm, cA, cB, h.part);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(h.part, h.nblk, h.sums + 4);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // namespace vr

using namespace vr;

template <bool SUB>
static int full_cb_form(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                        const TabHead& h, uint64_t RA, uint64_t RB, Carver& c, hipStream_t st) {
  const int64_t M = pairs_of(n);
  const CbGeom ga = cb_geom(RA), gb = cb_geom(RB);
  const CbWs w = cb_layout(c, n, ga, gb);
  VR_CHECK_HIP(hipMemsetAsync(w.cA, 0, (ga.tab + 1) * sizeof(uint32_t), st));
  VR_CHECK_HIP(hipMemsetAsync(w.cB, 0, (gb.tab + 1) * sizeof(uint32_t), st));
  uint32_t *ka = w.k[0], *kb = w.k[1];
  const dim3 kg((unsigned)((n + 255) / 256), (unsigned)std::min<int64_t>(n, 16384));
  k_cb_keys<SUB><<<kg, 256, 0, st>>>(A, B, idx, n, ld, h.mm, ka, kb);
  VR_CHECK_LAUNCH();
  // B's offsets by bucket (8-bit digits of the bucket, low first), then A's pairs
  uint32_t* bo = w.k[2];
  VR_TRY(radix_pass_k(kb, bo, M, gb.sh, w.radix, st));
  uint32_t* spare = w.k[4];
  if (gb.nb > 256) {
    VR_TRY(radix_pass_k(bo, w.k[4], M, gb.sh + 8, w.radix, st));
    spare = bo;
    bo = w.k[4];
  }
  uint32_t *oa = w.k[3], *ob = spare;
  VR_TRY(radix_pass_kv(ka, kb, oa, ob, M, ga.sh, w.radix, st));
  if (ga.nb > 256) {
    VR_TRY(radix_pass_kv(oa, ob, ka, kb, M, ga.sh + 8, w.radix, st));
    oa = ka;
    ob = kb;
  }
  const unsigned gm = (unsigned)((M + 255) / 256);
  k_cb_bstart<<<gm, 256, 0, st>>>(oa, M, ga.sh, ga.nb, w.bsA);
  VR_CHECK_LAUNCH();
  k_cb_bstart<<<gm, 256, 0, st>>>(bo, M, gb.sh, gb.nb, w.bsB);
  VR_CHECK_LAUNCH();
  const unsigned fb = (unsigned)((M + CB_SEG - 1) / CB_SEG);
  if (ga.sh == 0)
    k_cb_sizes<<<(unsigned)((ga.nb + 255) / 256), 256, 0, st>>>(w.bsA, ga.nb, w.cA);
  else
    k_cb_fine<1><<<fb, CB_FINE_BS, 0, st>>>(oa, M, w.bsA, ga.nb, ga.sh, w.cA);
  VR_CHECK_LAUNCH();
  if (gb.sh == 0)
    k_cb_sizes<<<(unsigned)((gb.nb + 255) / 256), 256, 0, st>>>(w.bsB, gb.nb, w.cB);
  else
    k_cb_fine<1><<<fb, CB_FINE_BS, 0, st>>>(bo, M, w.bsB, gb.nb, gb.sh, w.cB);
  VR_CHECK_LAUNCH();
  const int fg = full_grid();
  k_tab_ties<<<fg, FULL_BS, 0, st>>>(w.cA, (int64_t)ga.tab, h.part);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(h.part, fg, h.sums);
  VR_CHECK_LAUNCH();
  k_tab_ties<<<fg, FULL_BS, 0, st>>>(w.cB, (int64_t)gb.tab, h.part);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(h.part, fg, h.sums + 2);
  VR_CHECK_LAUNCH();
  VR_TRY(scan_exclusive_u32(w.cA, w.cA, (int64_t)ga.tab + 1, nullptr, w.sw, st));
  VR_TRY(scan_exclusive_u32(w.cB, w.cB, (int64_t)gb.tab + 1, nullptr, w.sw, st));
  k_cb_dot<<<fg, FULL_BS, 0, st>>>(oa, ob, M, w.cA, w.cB, h.part);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(h.part, fg, h.sums + 4);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

static int spearman_full_impl(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                              double* out, void* ws, size_t ws_bytes, hipStream_t st);

extern "C" {

size_t vr_spearman_full_workspace(int64_t n) {
  if (n < 2) return 256;
  return std::min(sort_bytes(n), cb_bytes(n, CB_CAP, CB_CAP));
}

int vr_spearman_full_last_form(void) { return g_full_form.load(); }

size_t vr_spearman_full_sort_workspace(int64_t n) {
  if (n < 2) return 256;
  return std::max(sort_bytes(n), std::max(tab_bytes(n, TAB_CAP, TAB_CAP), cb_bytes(n, CB_CAP, CB_CAP)));
}

int vr_spearman_full_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out, void* ws,
                         size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && ld >= n && out, "vr_spearman_full_f32: bad shape n=%lld ld=%lld", (long long)n,
             (long long)ld);
  return spearman_full_impl(A, B, n, ld, nullptr, out, ws, ws_bytes, as_stream(stream));
}

int vr_spearman_full_subset_f32(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                                int64_t k, double* out, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && ld >= n && k >= 0 && k <= n && out, "vr_spearman_full_subset_f32: bad shape n=%lld "
             "ld=%lld k=%lld", (long long)n, (long long)ld, (long long)k);
  VR_REQUIRE(idx != nullptr || k == 0, "vr_spearman_full_subset_f32: null idx");
  return spearman_full_impl(A, B, k, ld, idx, out, ws, ws_bytes, as_stream(stream));
}

}  // extern "C"

static int spearman_full_impl(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                              double* out, void* ws, size_t ws_bytes, hipStream_t st) {
  VR_REQUIRE(pairs_of(n) < ((int64_t)1 << 32), "vr_spearman_full_f32: n=%lld has 2^32 or more pairs",
             (long long)n);
  const int64_t M = pairs_of(n);
  const double nan = __builtin_nan("");
  if (M < 2) {  // scipy: NaN for fewer than two pairs
    VR_CHECK_HIP(hipMemcpyAsync(out, &nan, sizeof(double), hipMemcpyHostToDevice, st));
    VR_CHECK_HIP(hipStreamSynchronize(st));
    return VR_OK;
  }
  VR_REQUIRE(A && B && ws, "vr_spearman_full_f32: null pointer");
  Carver c(ws);
  const TabHead h = head_layout(c, n);
  if (ws_bytes < c.bytes()) {
    set_error("vr_spearman_full_f32: workspace %zu < %zu", ws_bytes, c.bytes());
    return VR_EWORKSPACE;
  }
  // key range and NaNs of both triangles (one read of each), to the host
  VR_CHECK_HIP(hipMemsetAsync(h.nan, 0, 2 * sizeof(uint32_t), st));
  const dim3 g = tri_grid(n);
  if (idx)
    k_tab_range<true><<<g, 256, 0, st>>>(A, B, idx, n, ld, h.mmpart, h.nan);
  else
    k_tab_range<false><<<g, 256, 0, st>>>(A, B, idx, n, ld, h.mmpart, h.nan);
  VR_CHECK_LAUNCH();
  k_tab_mm<<<1, 1024, 0, st>>>(h.mmpart, h.nblk, h.mm);
  VR_CHECK_LAUNCH();
  uint32_t hv[6];
  VR_CHECK_HIP(hipMemcpyAsync(hv, h.mm, 6 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VR_CHECK_HIP(hipStreamSynchronize(st));
  if (hv[4] || hv[5]) {  // scipy: NaN in either triangle -> NaN
    VR_CHECK_HIP(hipMemcpyAsync(out, &nan, sizeof(double), hipMemcpyHostToDevice, st));
    VR_CHECK_HIP(hipStreamSynchronize(st));
    return VR_OK;
  }
  const uint64_t binsA = (uint64_t)hv[1] - hv[0] + 1, binsB = (uint64_t)hv[3] - hv[2] + 1;
  // forms in order of preference: bucketed count tables, then the sort (any key range, any
  // tie structure); the plain count tables only when VISREPS_FULL_FORM=table names them (their
  // global atomics serialise on the few hot keys of quantized RDMs whose range is wide); a form
  // named in VISREPS_FULL_FORM (bucket / table / sort) runs when it applies and fits
  const size_t need_tab = tab_bytes(n, binsA, binsB), need_sort = sort_bytes(n);
  const bool cb_fits = binsA <= CB_CAP && binsB <= CB_CAP && cb_bytes(n, binsA, binsB) <= ws_bytes;
  const char* fe = getenv("VISREPS_FULL_FORM");
  const std::string forced = fe ? fe : "";
  int form = cb_fits ? 0 : (need_sort <= ws_bytes ? 2 : -1);
  if (forced == "table" && need_tab <= ws_bytes) form = 1;
  if (forced == "sort" && need_sort <= ws_bytes) form = 2;
  g_full_form = form;
  if (form == 0) {
    if (idx)
      VR_TRY(full_cb_form<true>(A, B, n, ld, idx, h, binsA, binsB, c, st));
    else
      VR_TRY(full_cb_form<false>(A, B, n, ld, idx, h, binsA, binsB, c, st));
  } else if (form == 1) {
    if (idx)
      VR_TRY(full_tab_form<true>(A, B, n, ld, idx, h, binsA, binsB, c, st));
    else
      VR_TRY(full_tab_form<false>(A, B, n, ld, idx, h, binsA, binsB, c, st));
  } else if (form == 2) {
    const FullWs w = full_layout(c, n);
    VR_TRY(full_sort_form(A, B, n, ld, idx, h, w, st));
  } else {
    set_error("vr_spearman_full_f32: key range %llu / %llu needs the sort form's workspace %zu "
              "(vr_spearman_full_sort_workspace), given %zu", (unsigned long long)binsA,
              (unsigned long long)binsB, need_sort, ws_bytes);
    return VR_EWORKSPACE;
  }
  k_full_final<<<1, 64, 0, st>>>(h.sums, M, h.nan, out);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

extern "C" {

// ---------------------------------------------------------------------------------
// Local pieces of the distributed global rank (analysis/distributed_spearman.py)
// ---------------------------------------------------------------------------------
size_t vr_sort_pairs_workspace(int64_t m) {
  if (m <= 1) return 256;
  Carver c(nullptr);
  c.take<uint32_t>((size_t)m);
  c.take<uint32_t>((size_t)m);
  c.take<uint32_t>(radix_ws_elems(m));
  return c.bytes();
}

int vr_sort_pairs_u32(uint32_t* keys, uint32_t* vals, int64_t m, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(m >= 0 && m < ((int64_t)1 << 32), "vr_sort_pairs_u32: m=%lld", (long long)m);
  if (m <= 1) return VR_OK;
  VR_REQUIRE(keys && vals && ws && ws_bytes >= vr_sort_pairs_workspace(m), "vr_sort_pairs_u32: workspace");
  Carver c(ws);
  uint32_t* ka = c.take<uint32_t>((size_t)m);
  uint32_t* va = c.take<uint32_t>((size_t)m);
  uint32_t* rw = c.take<uint32_t>(radix_ws_elems(m));
  return radix_sort_kv(keys, vals, ka, va, m, rw, as_stream(stream));
}

__global__ void k_sort_keys(const float* __restrict__ v, int64_t m, uint32_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) keys[i] = f32_sort_key(v[i]);
}

int vr_f32_sort_keys(const float* v, int64_t m, uint32_t* keys, void* stream) {
  VR_REQUIRE(m >= 0 && m < ((int64_t)1 << 32), "vr_f32_sort_keys: m=%lld", (long long)m);
  if (m == 0) return VR_OK;
  VR_REQUIRE(v && keys, "vr_f32_sort_keys: null pointer");
  k_sort_keys<<<(unsigned)((m + 255) / 256), 256, 0, as_stream(stream)>>>(v, m, keys);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

__global__ __launch_bounds__(FULL_BS) void k_midranks_run(const uint32_t* __restrict__ flags,
                                                           const uint32_t* __restrict__ gidx,
                                                           const uint32_t* __restrict__ gstart, int64_t m,
                                                           uint64_t base2, uint64_t* __restrict__ y,
                                                           uint64_t* __restrict__ part) {
  u128 tie = 0;
  for (int64_t i = (int64_t)blockIdx.x * FULL_BS + threadIdx.x; i < m; i += (int64_t)gridDim.x * FULL_BS) {
    uint64_t k;
    y[i] = base2 + midrank2(flags, gidx, gstart, i, k);
    if (flags[i]) tie += (u128)(k * k) * k - k;
  }
  block_sum_u128(tie, part, 0, 1);
}

__global__ __launch_bounds__(FULL_BS) void k_dot_u64(const uint64_t* __restrict__ a,
                                                      const uint64_t* __restrict__ b, int64_t m,
                                                      uint64_t* __restrict__ part) {
  u128 s = 0;
  for (int64_t i = (int64_t)blockIdx.x * FULL_BS + threadIdx.x; i < m; i += (int64_t)gridDim.x * FULL_BS)
    s += (u128)a[i] * b[i];
  block_sum_u128(s, part, 0, 1);
}

__global__ void k_sum_parts(const uint64_t* __restrict__ part, int nblk, uint64_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  u128 s = 0;
  for (int b = 0; b < nblk; ++b) s += ((u128)part[2 * b + 1] << 64) | part[2 * b];
  out[0] = (uint64_t)s;
  out[1] = (uint64_t)(s >> 64);
}

size_t vr_midranks_workspace(int64_t m) {
  Carver c(nullptr);
  c.take<uint32_t>((size_t)std::max<int64_t>(m, 1));
  c.take<uint32_t>((size_t)std::max<int64_t>(m, 1));
  c.take<uint32_t>((size_t)m + 1);
  c.take<uint32_t>(scan_ws_elems(m));
  c.take<uint64_t>((size_t)full_grid() * 2);
  return c.bytes();
}

int vr_midranks_sorted(const uint32_t* keys, int64_t m, uint64_t base, uint64_t* y, uint64_t* tie,
                       void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(m >= 0 && m < ((int64_t)1 << 32), "vr_midranks_sorted: m=%lld", (long long)m);
  VR_REQUIRE(tie && ws && ws_bytes >= vr_midranks_workspace(m), "vr_midranks_sorted: workspace");
  hipStream_t st = as_stream(stream);
  if (m == 0) {
    VR_CHECK_HIP(hipMemsetAsync(tie, 0, 2 * sizeof(uint64_t), st));
    return VR_OK;
  }
  VR_REQUIRE(keys && y, "vr_midranks_sorted: null pointer");
  Carver c(ws);
  uint32_t* flags = c.take<uint32_t>((size_t)m);
  uint32_t* gidx = c.take<uint32_t>((size_t)m);
  uint32_t* gstart = c.take<uint32_t>((size_t)m + 1);
  uint32_t* sw = c.take<uint32_t>(scan_ws_elems(m));
  uint64_t* part = c.take<uint64_t>((size_t)full_grid() * 2);
  const unsigned gb = (unsigned)((m + 255) / 256);
  k_group_flags_full<<<gb, 256, 0, st>>>(keys, m, flags);
  VR_CHECK_LAUNCH();
  VR_TRY(scan_exclusive_u32(flags, gidx, m, nullptr, sw, st));
  k_group_starts_full<<<gb, 256, 0, st>>>(flags, gidx, m, gstart);
  VR_CHECK_LAUNCH();
  k_midranks_run<<<full_grid(), FULL_BS, 0, st>>>(flags, gidx, gstart, m, 2 * base, y, part);
  VR_CHECK_LAUNCH();
  k_sum_parts<<<1, 64, 0, st>>>(part, full_grid(), tie);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// ---- count-table form of the distributed global rank: per-key counts of a rank's keys,
// all-reduced by the caller, then starts, tie terms and the doubled midranks of its keys
__global__ void k_key_counts(const uint32_t* __restrict__ keys, int64_t m, uint32_t kmin,
                             uint32_t* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) atomicAdd(&cnt[keys[i] - kmin], 1u);
}

// tables of <= 16384 keys: per-block counts in LDS (a few hot keys would serialise global
// atomics), added to the table once per block
constexpr int KC_LDS_BINS = 16384;
__global__ __launch_bounds__(1024) void k_key_counts_lds(const uint32_t* __restrict__ keys, int64_t m, uint32_t kmin,
                                                         int bins, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[KC_LDS_BINS];
  for (int i = threadIdx.x; i < bins; i += 1024) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < m; i += (int64_t)gridDim.x * 1024)
    atomicAdd(&h[keys[i] - kmin], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < bins; i += 1024)
    if (h[i]) atomicAdd(&cnt[i], h[i]);
}

__global__ void k_key_midranks(const uint32_t* __restrict__ keys, int64_t m, uint32_t kmin,
                               const uint32_t* __restrict__ start, uint64_t* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) {
    const uint32_t k = keys[i] - kmin;
    y[i] = (uint64_t)start[k] + start[k + 1] + 1u;
  }
}

int vr_key_counts_u32(const uint32_t* keys, int64_t m, uint32_t kmin, int64_t bins, uint32_t* cnt, void* stream) {
  VR_REQUIRE(m >= 0 && bins >= 1 && bins < ((int64_t)1 << 32), "vr_key_counts_u32: m=%lld bins=%lld",
             (long long)m, (long long)bins);
  if (m == 0) return VR_OK;
  VR_REQUIRE(keys && cnt, "vr_key_counts_u32: null pointer");
  if (bins <= KC_LDS_BINS)
    k_key_counts_lds<<<(unsigned)std::min<int64_t>((m + 1023) / 1024, full_grid()), 1024, 0, as_stream(stream)>>>(
        keys, m, kmin, (int)bins, cnt);
  else
    k_key_counts<<<(unsigned)((m + 255) / 256), 256, 0, as_stream(stream)>>>(keys, m, kmin, cnt);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

size_t vr_key_table_workspace(int64_t bins) {
  Carver c(nullptr);
  c.take<uint32_t>(scan_ws_elems(std::max<int64_t>(bins, 1) + 1));
  c.take<uint64_t>((size_t)full_grid() * 2);
  return c.bytes();
}

int vr_key_table_midranks(const uint32_t* keys, int64_t m, uint32_t kmin, uint32_t* cnt, int64_t bins, uint64_t* y,
                          uint64_t* tie, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(m >= 0 && bins >= 1 && bins < ((int64_t)1 << 32) && cnt && tie,
             "vr_key_table_midranks: m=%lld bins=%lld", (long long)m, (long long)bins);
  VR_REQUIRE(ws && ws_bytes >= vr_key_table_workspace(bins), "vr_key_table_midranks: workspace");
  hipStream_t st = as_stream(stream);
  Carver c(ws);
  uint32_t* sw = c.take<uint32_t>(scan_ws_elems(bins + 1));
  uint64_t* part = c.take<uint64_t>((size_t)full_grid() * 2);
  k_tab_ties<<<full_grid(), FULL_BS, 0, st>>>(cnt, bins, part);
  VR_CHECK_LAUNCH();
  k_reduce_u128<<<1, FULL_BS, 0, st>>>(part, full_grid(), tie);
  VR_CHECK_LAUNCH();
  VR_TRY(scan_exclusive_u32(cnt, cnt, bins + 1, nullptr, sw, st));
  if (m > 0) {
    VR_REQUIRE(keys && y, "vr_key_table_midranks: null pointer");
    k_key_midranks<<<(unsigned)((m + 255) / 256), 256, 0, st>>>(keys, m, kmin, cnt, y);
    VR_CHECK_LAUNCH();
  }
  return VR_OK;
}

size_t vr_dot_u64_workspace(void) { return (size_t)full_grid() * 2 * sizeof(uint64_t) + 256; }

int vr_dot_u64(const uint64_t* a, const uint64_t* b, int64_t m, uint64_t* out, void* ws, size_t ws_bytes,
               void* stream) {
  VR_REQUIRE(m >= 0 && out && ws && ws_bytes >= vr_dot_u64_workspace(), "vr_dot_u64: bad arguments");
  hipStream_t st = as_stream(stream);
  uint64_t* part = static_cast<uint64_t*>(ws);
  k_dot_u64<<<full_grid(), FULL_BS, 0, st>>>(a, b, m, part);
  VR_CHECK_LAUNCH();
  k_sum_parts<<<1, 64, 0, st>>>(part, full_grid(), out);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // extern "C"
