// LSD radix sort of (uint32 key, uint32 value) pairs, 8-bit digits, 4 passes.
// Per pass: tile histograms (digit-major) -> device-wide exclusive scan -> stable
// scatter, where each 4096-element tile is first ordered by digit in LDS with eight
// stable 1-bit splits, then written out digit-run by digit-run (coalesced).
// Used once per RDM to order its strict upper triangle by value (the rank plan).
#include "internal.h"

namespace vr {

__global__ __launch_bounds__(RS_BS) void k_rs_hist(const uint32_t* __restrict__ keys,
                                                   int64_t n, int shift,
                                                   uint32_t* __restrict__ hist, int64_t nb) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    int64_t i = base + (int64_t)j * RS_BS + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

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
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  cnt[t] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RS_IPT; ++j) {
    int p = j * RS_BS + t;
    int64_t i = base + p;
    uint32_t k = 0xFFFFFFFFu, v = 0;
    if (i < n) {
      k = kin[i];
      v = vin[i];
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
      int64_t g = (int64_t)offs[(int64_t)d * nb + blockIdx.x] + r;
      kout[g] = k;
      vout[g] = sv[lds_pad(s)];
    }
  }
}

size_t radix_ws_elems(int64_t n) {
  const int64_t nb = (n + RS_TILE - 1) / RS_TILE;
  const int64_t h = 256 * nb;
  return (size_t)(h + 64) + scan_ws_elems(h);
}

int radix_sort_kv(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                  int64_t n, uint32_t* ws, hipStream_t st) {
  if (n <= 1) return VR_OK;
  const int64_t nb = (n + RS_TILE - 1) / RS_TILE;
  const int64_t h = 256 * nb;
  uint32_t* hist = ws;
  uint32_t* scan_ws = ws + h + 64;
  uint32_t *ki = keys, *vi = vals, *ko = keys_alt, *vo = vals_alt;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = pass * 8;
    k_rs_hist<<<(unsigned)nb, RS_BS, 0, st>>>(ki, n, shift, hist, nb);
    VR_CHECK_LAUNCH();
    VR_TRY(scan_exclusive_u32(hist, hist, h, nullptr, scan_ws, st));
    k_rs_scatter<<<(unsigned)nb, RS_BS, 0, st>>>(ki, vi, ko, vo, n, shift, hist, nb);
    VR_CHECK_LAUNCH();
    uint32_t* tk = ki; ki = ko; ko = tk;
    uint32_t* tv = vi; vi = vo; vo = tv;
  }
  // four passes: the sorted data is back in (keys, vals)
  return VR_OK;
}

}  // namespace vr
