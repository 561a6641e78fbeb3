// LSD radix sort of (uint32 key, uint32 value) pairs, 8-bit digits, 4 passes.
// Per pass: tile histograms (tile-major) -> exclusive scan in (digit, tile) order -> stable
// scatter, where each 4096-element tile is first ordered by digit in LDS, then written
// out digit-run by digit-run (coalesced). The in-tile order comes from wave ballots
// (k_rs_scatter: each wave ranks its 1024 keys in rounds of 64 by the peer masks of
// eight ballots, then per-wave digit totals place them); VR_RS_SPLIT8 builds the older
// form, eight stable 1-bit splits over the tile.
// Used once per RDM to order its strict upper triangle by value (the rank plan).
#include "internal.h"

namespace vr {

#ifndef VR_RS_XCD
#define VR_RS_XCD 1
#endif
// Tile of this block. With VR_RS_XCD the blocks one XCD receives take consecutive tiles
// (xcd_item), so the digit runs that neighbouring tiles write side by side meet in the
// same L2 instead of in eight.
__device__ inline int64_t rs_tile(int64_t nb) {
#if VR_RS_XCD
  return xcd_item(nb);
#else
  (void)nb;
  return blockIdx.x;
#endif
}

__global__ __launch_bounds__(RS_BS) void k_rs_hist(const uint32_t* __restrict__ keys,
                                                   int64_t n, int shift,
                                                   uint32_t* __restrict__ hist, int64_t nb) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t tile = rs_tile(nb);
  const int64_t base = tile * RS_TILE;
  if (base + RS_TILE <= n && (reinterpret_cast<uintptr_t>(keys) & 15) == 0) {
    const uint4* k4 = reinterpret_cast<const uint4*>(keys + base);
    uint4 q[RS_IPT / 4];
#pragma unroll
    for (int j = 0; j < RS_IPT / 4; ++j) q[j] = k4[j * RS_BS + threadIdx.x];
#pragma unroll
    for (int j = 0; j < RS_IPT / 4; ++j) {
      atomicAdd(&h[(q[j].x >> shift) & 255u], 1u);
      atomicAdd(&h[(q[j].y >> shift) & 255u], 1u);
      atomicAdd(&h[(q[j].z >> shift) & 255u], 1u);
      atomicAdd(&h[(q[j].w >> shift) & 255u], 1u);
    }
  } else {
#pragma unroll
    for (int j = 0; j < RS_IPT; ++j) {
      int64_t i = base + (int64_t)j * RS_BS + threadIdx.x;
      if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
    }
  }
  __syncthreads();
  hist[tile * 256 + threadIdx.x] = h[threadIdx.x];  // tile-major: one 1-KB row
}

// Exclusive scan of the tile histograms in (digit, tile) order while they stay tile-major
// ([tile][digit], so the big passes read and write coalesced 1-KB rows): per-chunk column
// sums (k_rs_colsum), each digit's column of chunk sums scanned by its own block
// (k_rs_colscan, which leaves the digit total), then every chunk adds the digit bases
// (a block scan of the 256 totals) and writes its in-chunk column prefixes (k_rs_colapply).
struct RsChunks {
  int64_t ch;  // tiles per chunk
  int64_t c;   // chunks (<= 1024)
};
static RsChunks rs_chunks(int64_t nb) {
  int64_t ch = (nb + 1023) / 1024;
  if (ch < 16) ch = 16;
  return RsChunks{ch, (nb + ch - 1) / ch};
}

__global__ __launch_bounds__(256) void k_rs_colsum(const uint32_t* __restrict__ h, int64_t nb,
                                                   int64_t ch, uint32_t* __restrict__ cs) {
  const int d = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * ch;
  const int64_t t1 = t0 + ch < nb ? t0 + ch : nb;
  uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t t = t0;
  for (; t + 8 <= t1; t += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += h[(t + u) * 256 + d];
  }
  for (; t < t1; ++t) acc[0] += h[t * 256 + d];
  cs[(int64_t)blockIdx.x * 256 + d] =
      acc[0] + acc[1] + acc[2] + acc[3] + acc[4] + acc[5] + acc[6] + acc[7];
}

// grid = 256 digits; block of 256 threads, each owning a run of up to 4 chunks
__global__ __launch_bounds__(256) void k_rs_colscan(uint32_t* __restrict__ cs, int64_t c,
                                                    uint32_t* __restrict__ total) {
  __shared__ uint32_t scan_lds[256 / 64 + 1];
  const int d = blockIdx.x, i = threadIdx.x;
  uint32_t x[4], sum = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t q = (int64_t)i * 4 + u;
    x[u] = q < c ? cs[q * 256 + d] : 0u;
    sum += x[u];
  }
  uint32_t tot;
  uint32_t acc = block_exclusive_scan<256>(sum, scan_lds, tot);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t q = (int64_t)i * 4 + u;
    if (q < c) cs[q * 256 + d] = acc;
    acc += x[u];
  }
  if (i == 0) total[d] = tot;
}

__global__ __launch_bounds__(256) void k_rs_colapply(uint32_t* __restrict__ h, int64_t nb,
                                                     int64_t ch, const uint32_t* __restrict__ cs,
                                                     const uint32_t* __restrict__ total) {
  __shared__ uint32_t scan_lds[256 / 64 + 1];
  const int d = threadIdx.x;
  uint32_t tot;
  const uint32_t base = block_exclusive_scan<256>(total[d], scan_lds, tot);
  const int64_t t0 = (int64_t)blockIdx.x * ch;
  const int64_t t1 = t0 + ch < nb ? t0 + ch : nb;
  uint32_t acc = base + cs[(int64_t)blockIdx.x * 256 + d];
  int64_t t = t0;
  for (; t + 8 <= t1; t += 8) {
    uint32_t x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = h[(t + u) * 256 + d];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      h[(t + u) * 256 + d] = acc;
      acc += x[u];
    }
  }
  for (; t < t1; ++t) {
    const uint32_t x = h[t * 256 + d];
    h[t * 256 + d] = acc;
    acc += x;
  }
}

#ifndef VR_RS_SPLIT8
#define VR_RS_SPLIT8 0
#endif

#if !VR_RS_SPLIT8
// Each wave ranks its own 1024 consecutive keys in 16 rounds of 64 with no block barrier:
// a key's rank among the same-digit keys of its round from the peer mask of eight
// ballots, plus the wave's running count of that digit (wave-private LDS counters). The
// block then needs two barriers: the per-wave digit totals give every key its slot in the
// digit-ordered tile (digit start + same-digit keys of the waves before + wave rank).
// KV false: keys only (vin / vout unused).
template <bool KV = true>
__global__ __launch_bounds__(RS_BS) void k_rs_scatter(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, int64_t n, int shift,
    const uint32_t* __restrict__ offs, int64_t nb) {
  static_assert(RS_BS == 256, "one thread per digit");
  constexpr int NW = RS_BS / 64, WT = RS_TILE / NW;  // waves, keys per wave
  __shared__ uint32_t sk[RS_TILE];
  __shared__ uint32_t sv[RS_TILE];
  __shared__ uint32_t wcnt[NW][256];  // wave w's running (then total) count of digit d
  __shared__ uint32_t start[256];
  __shared__ uint32_t scan_lds[RS_BS / 64 + 1];

  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int64_t tile = rs_tile(nb);
  const int64_t base = tile * RS_TILE;
  const int64_t left = n - base;
  const int nvalid = left < RS_TILE ? (int)left : RS_TILE;
#pragma unroll
  for (int q = 0; q < NW; ++q) wcnt[q][t] = 0;
  __syncthreads();
  uint32_t kk[RS_IPT], vv[RS_IPT], rk[RS_IPT];
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    const int p = w * WT + j * 64 + lane;
    kk[j] = 0xFFFFFFFFu;
    vv[j] = 0;
    if (p < nvalid) {
      kk[j] = kin[base + p];
      if constexpr (KV) vv[j] = vin[base + p];
    }
  }
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    const bool valid = w * WT + j * 64 + lane < nvalid;
    const uint32_t d = (kk[j] >> shift) & 255u;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    // all lanes read before the leaders write (one wave: LDS ops complete in order)
    const uint32_t before = wcnt[w][d];
    rk[j] = before + r;
    if (valid && r == 0) wcnt[w][d] = before + (uint32_t)__popcll(m);
  }
  __syncthreads();
  {
    uint32_t c = 0, tot;
#pragma unroll
    for (int q = 0; q < NW; ++q) c += wcnt[q][t];
    const uint32_t s0 = block_exclusive_scan<RS_BS>(c, scan_lds, tot);  // ends with a barrier
    start[t] = s0;
    uint32_t acc = s0;  // wcnt[q][t] becomes the slot of digit t's first key of wave q
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const uint32_t x = wcnt[q][t];
      wcnt[q][t] = acc;
      acc += x;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    if (w * WT + j * 64 + lane < nvalid) {
      const uint32_t pos = wcnt[w][(kk[j] >> shift) & 255u] + rk[j];
      sk[pos] = kk[j];
      if constexpr (KV) sv[pos] = vv[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    const int s = j * RS_BS + t;
    if (s < nvalid) {
      const uint32_t k = sk[s];
      const uint32_t d = (k >> shift) & 255u;
      const int64_t g = (int64_t)offs[tile * 256 + d] + (uint32_t)s - start[d];
      kout[g] = k;
      if constexpr (KV) vout[g] = sv[s];
    }
  }
}
#else
template <bool KV = true>
__global__ __launch_bounds__(RS_BS) void k_rs_scatter(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, int64_t n, int shift,
    const uint32_t* __restrict__ offs, int64_t nb) {
  constexpr int PADDED = RS_TILE + RS_TILE / 32;
  __shared__ uint32_t sk[PADDED];
  __shared__ uint32_t sv[PADDED];
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t start[256];
  __shared__ uint32_t scan_lds[RS_BS / 64 + 1];

  const int t = threadIdx.x;
  const int64_t tile = rs_tile(nb);
  const int64_t base = tile * RS_TILE;
  cnt[t] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    int p = j * RS_BS + t;
    int64_t i = base + p;
    uint32_t k = 0xFFFFFFFFu, v = 0;
    if (i < n) {
      k = kin[i];
      if constexpr (KV) v = vin[i];
      atomicAdd(&cnt[(k >> shift) & 255u], 1u);
    }
    sk[lds_pad(p)] = k;
    sv[lds_pad(p)] = v;
  }
  __syncthreads();

  // Stable local ordering by the 8 digit bits: 8 one-bit splits on the blocked layout
  // (thread t owns positions 16t .. 16t+15). Padding keys (0xFFFFFFFF) stay last.
  for (int bit = 0; bit < 8; ++bit) {
    uint32_t kk[RS_IPT], vv[RS_IPT];
    uint32_t zeros = 0;
#pragma unroll
    for (int j = 0; j < RS_IPT; ++j) {
      kk[j] = sk[lds_pad(t * RS_IPT + j)];
      vv[j] = sv[lds_pad(t * RS_IPT + j)];
      zeros += ((kk[j] >> (shift + bit)) & 1u) ^ 1u;
    }
    uint32_t Z;
    uint32_t Zt = block_exclusive_scan<RS_BS>(zeros, scan_lds, Z);  // ends with a barrier
    uint32_t zb = 0;
#pragma unroll
    for (int j = 0; j < RS_IPT; ++j) {
      uint32_t b = (kk[j] >> (shift + bit)) & 1u;
      uint32_t idx = (uint32_t)(t * RS_IPT + j);
      uint32_t pos = b ? (Z + idx - (Zt + zb)) : (Zt + zb);
      zb += b ^ 1u;
      sk[lds_pad((int)pos)] = kk[j];
      sv[lds_pad((int)pos)] = vv[j];
    }
    __syncthreads();
  }

  // digit start offsets inside the tile (valid elements only)
  {
    uint32_t c = cnt[t], tot;
    uint32_t s = block_exclusive_scan<RS_BS>(c, scan_lds, tot);
    start[t] = s;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    int s = j * RS_BS + t;
    uint32_t k = sk[lds_pad(s)];
    uint32_t d = (k >> shift) & 255u;
    uint32_t r = (uint32_t)s - start[d];
    if (r < cnt[d]) {
      int64_t g = (int64_t)offs[tile * 256 + d] + r;
      kout[g] = k;
      if constexpr (KV) vout[g] = sv[lds_pad(s)];
    }
  }
}
#endif

size_t radix_ws_elems(int64_t n) {
  const int64_t nb = (n + RS_TILE - 1) / RS_TILE;
  return (size_t)(256 * nb + 64) + (size_t)256 * rs_chunks(nb).c + 256;
}

int radix_offsets(const uint32_t* ki, int64_t n, int shift, uint32_t* ws, hipStream_t st) {
  if (n <= 0) return VR_OK;
  const int64_t nb = (n + RS_TILE - 1) / RS_TILE;
  const RsChunks C = rs_chunks(nb);
  uint32_t* hist = ws;
  uint32_t* cs = ws + 256 * nb + 64;
  k_rs_hist<<<(unsigned)nb, RS_BS, 0, st>>>(ki, n, shift, hist, nb);
  VR_CHECK_LAUNCH();
  k_rs_colsum<<<(unsigned)C.c, 256, 0, st>>>(hist, nb, C.ch, cs);
  VR_CHECK_LAUNCH();
  k_rs_colscan<<<256, 256, 0, st>>>(cs, C.c, cs + 256 * C.c);
  VR_CHECK_LAUNCH();
  k_rs_colapply<<<(unsigned)C.c, 256, 0, st>>>(hist, nb, C.ch, cs, cs + 256 * C.c);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

int radix_pass_kv(const uint32_t* ki, const uint32_t* vi, uint32_t* ko, uint32_t* vo, int64_t n,
                  int shift, uint32_t* ws, hipStream_t st) {
  if (n <= 0) return VR_OK;
  const int64_t nb = (n + RS_TILE - 1) / RS_TILE;
  VR_TRY(radix_offsets(ki, n, shift, ws, st));
  k_rs_scatter<true><<<(unsigned)nb, RS_BS, 0, st>>>(ki, vi, ko, vo, n, shift, ws, nb);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

int radix_pass_k(const uint32_t* ki, uint32_t* ko, int64_t n, int shift, uint32_t* ws, hipStream_t st) {
  if (n <= 0) return VR_OK;
  const int64_t nb = (n + RS_TILE - 1) / RS_TILE;
  VR_TRY(radix_offsets(ki, n, shift, ws, st));
  k_rs_scatter<false><<<(unsigned)nb, RS_BS, 0, st>>>(ki, nullptr, ko, nullptr, n, shift, ws, nb);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

int radix_sort_kv(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                  int64_t n, uint32_t* ws, hipStream_t st) {
  if (n <= 1) return VR_OK;
  uint32_t *ki = keys, *vi = vals, *ko = keys_alt, *vo = vals_alt;
  for (int pass = 0; pass < 4; ++pass) {
    VR_TRY(radix_pass_kv(ki, vi, ko, vo, n, pass * 8, ws, st));
    uint32_t* tk = ki; ki = ko; ko = tk;
    uint32_t* tv = vi; vi = vo; vo = tv;
  }
  // four passes: the sorted data is back in (keys, vals)
  return VR_OK;
}

}  // namespace vr
