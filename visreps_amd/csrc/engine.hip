// Bootstrapped Spearman RSA engine and the triangle-Spearman entry points.
//
// Replaces, per (model RDM A, neural RDM B) unit, the reference loop
//   point = spearmanr(triu(A), triu(B))                                 evals.py:347-349
//   for i in range(1000): idx = rng.choice(n, int(.9n), replace=False)
//       scores[i] = spearmanr(triu(A[idx][:,idx]), triu(B[idx][:,idx]))    evals.py:361-369
// with scipy's average-rank (midrank) ties (rsa.py:43-47,121-122).
//
// For a stimulus subset S a pair (a,b) is included iff a, b in S; its midrank among the
// included pairs is (c_s + c_e + 1)/2 with c_s / c_e the included counts before / through
// its tie group in sorted order. Everything is kept as doubled ranks y = 2 c_s + k + 1
// (integers), and rho = (sum yA yB - M'(M'+1)^2) / sqrt((sum yA^2 - mu)(sum yB^2 - mu)),
// mu = M'(M'+1)^2, M' = included pairs: exact integer sums -> fp64 at the end, so scores
// do not depend on chunking, lane grouping, launch order or GPU count.
//
// One pass evaluates 64 subsets: lane w of every wave is subset w, masks[x] bit w says
// whether stimulus x is in subset w (LDS). Waves own contiguous segments of chunks.
//  k_rankA   walk A order; per tie group y'_A (segment-relative); scatter the chunk-
//            relative rank yA~ = y'_A - 2 lp_c to the pair's B position:
//            TB[posB][w] (u16 when chunk spans fit, else u32); segment sums n, n y', n y'^2
//  k_scan_seg + k_add_base   chunk bases baseA[c][w] (segment prefix + local prefix)
//  k_rankB   walk B order streaming TB rows; yA = 2 baseA[chunkA(pair)][w] + yA~; per B
//            tie group S = sum of included yA, then y'_B S, n y'_B, n y'_B^2 (segment-rel.)
//  k_final   combine segments with their bases -> rho per lane
#include <type_traits>
#include <vector>

#include "plan.h"

namespace vr {

typedef unsigned __int128 u128;
typedef __int128 i128;

constexpr int ENG_THREADS = 1024;  // 16 waves per workgroup
constexpr int WAVES_PER_WG = ENG_THREADS / 64;
constexpr int LANES = 64;
constexpr int U = 16;  // pairs per block: one vector load brings 16 pair codes

struct EngineCfg {
  int grid;      // persistent workgroups
  int nwaves;    // grid * WAVES_PER_WG = number of chunk segments
  size_t lds;    // dynamic LDS for the masks (0: masks read from global)
  bool use_lds;
};

static EngineCfg engine_cfg(int64_t n) {
  EngineCfg c;
  const size_t need = (size_t)n * sizeof(uint64_t);
  const size_t cap = 160 * 1024 - 1024;
  c.use_lds = need <= cap;
  const int per_cu = c.use_lds ? std::max<int>(1, std::min<int>(2, (int)(cap / std::max<size_t>(need, 1)))) : 2;
  c.grid = num_cus() * per_cu;
  c.nwaves = c.grid * WAVES_PER_WG;
  c.lds = c.use_lds ? need : 0;
  return c;
}

struct EngineWs {
  uint64_t* masks;      // [n]
  uint32_t* posB_byA;   // [M]  A position -> B position (per unit)
  uint32_t* chunkA_byB; // [M]  B position -> A chunk (per unit)
  void* TB;             // [M * lw] u16 or u32 chunk-relative yA~
  uint32_t* lpA;        // [nch * 64] local prefix at chunk start within its segment
  uint32_t* baseA;      // [nch * 64]
  uint32_t* segA_tot;   // [nw * 64]
  uint64_t* segA_part;  // [nw * 64 * 3]  sum n y', sum n y'^2 (u128)
  uint32_t* segA_pre;   // [nw * 64]
  uint32_t* segB_tot;   // [nw * 64]
  uint64_t* segB_part;  // [nw * 64 * 6]  acc (u128), St, NY, NY2 (u128)
  uint32_t* totA;       // [64]
};

static EngineWs engine_layout(void* base, int64_t n, int lw, int nwaves, size_t* bytes) {
  const int64_t M = pairs_of(n);
  const size_t nch = plan_nchunks(M);
  Carver c(base);
  EngineWs e;
  e.masks = c.take<uint64_t>((size_t)n);
  e.posB_byA = c.take<uint32_t>((size_t)M);
  e.chunkA_byB = c.take<uint32_t>((size_t)M);
  e.TB = c.take<uint32_t>((size_t)M * (size_t)lw);  // sized for u32
  e.lpA = c.take<uint32_t>(nch * LANES);
  e.baseA = c.take<uint32_t>(nch * LANES);
  e.segA_tot = c.take<uint32_t>((size_t)nwaves * LANES);
  e.segA_part = c.take<uint64_t>((size_t)nwaves * LANES * 3);
  e.segA_pre = c.take<uint32_t>((size_t)nwaves * LANES);
  e.segB_tot = c.take<uint32_t>((size_t)nwaves * LANES);
  e.segB_part = c.take<uint64_t>((size_t)nwaves * LANES * 6);
  e.totA = c.take<uint32_t>(LANES);
  if (bytes) *bytes = c.bytes();
  return e;
}

// ---------------------------------------------------------------------------------
// per-unit join and per-pass masks
// ---------------------------------------------------------------------------------
__global__ void k_join(const uint32_t* __restrict__ codesA, const uint32_t* __restrict__ codesB,
                       int64_t M, int64_t n, const uint32_t* __restrict__ posOfPairB,
                       const uint32_t* __restrict__ chunkOfPairA,
                       uint32_t* __restrict__ posB_byA, uint32_t* __restrict__ chunkA_byB) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t ca = codesA[i], cb = codesB[i];
  posB_byA[i] = posOfPairB[tri_index(ca >> 16, ca & 0xffffu, (uint64_t)n)];
  chunkA_byB[i] = chunkOfPairA[tri_index(cb >> 16, cb & 0xffffu, (uint64_t)n)];
}

// bit w of masks[x] <- x in subset (set0 + w); subset 0 is "all stimuli" when full_first.
__global__ void k_masks_sets(const int32_t* __restrict__ idx, int64_t k, int64_t set0,
                             int nl, int full_first, uint64_t* __restrict__ masks) {
  const int w = blockIdx.y;
  if (w >= nl) return;
  const int64_t s = set0 + w;
  if (full_first && s == 0) return;  // handled by k_masks_full
  const int64_t row = s - (full_first ? 1 : 0);
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t x = idx[row * k + j];
    atomicOr(reinterpret_cast<unsigned long long*>(&masks[x]), 1ull << w);
  }
}

__global__ void k_masks_full(uint64_t* __restrict__ masks, int64_t n) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x < n) masks[x] |= 1ull;  // lane 0 of the first pass
}

// ---------------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------------
template <bool LDS>
__device__ inline const uint64_t* stage_masks(const uint64_t* __restrict__ gmask, int64_t n,
                                              uint64_t* smem) {
  if (!LDS) return gmask;
  for (int64_t x = threadIdx.x; x < n; x += blockDim.x) smem[x] = gmask[x];
  __syncthreads();
  return smem;
}

__device__ inline uint32_t wave_uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ inline uint32_t readlane_u32(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ inline uint64_t readlane_u64(uint64_t v, uint32_t l) {
  return ((uint64_t)readlane_u32((uint32_t)(v >> 32), l) << 32) | readlane_u32((uint32_t)v, l);
}

// Group-start bits of positions [p, p+16) (bit t <-> position p+t), wave-uniform.
__device__ inline uint32_t flags16(const uint32_t* __restrict__ gflag, uint32_t p) {
  const uint32_t w = p >> 5, sh = p & 31;
  const uint64_t two = ((uint64_t)gflag[w + 1] << 32) | gflag[w];
  return (uint32_t)(two >> sh) & 0xffffu;
}

// Lane (l & 15) looks up both stimulus masks of pair p + (l & 15); the AND is then
// broadcast per pair with readlane.
__device__ inline uint64_t block_masks(const uint64_t* m, const uint32_t* __restrict__ codes,
                                       uint32_t p, uint32_t cnt, int lane) {
  const uint32_t sub = lane & (U - 1);
  uint64_t both = 0;
  if (sub < cnt) {
    const uint32_t code = codes[p + sub];
    both = m[code >> 16] & m[code & 0xffffu];
  }
  return both;
}

__device__ inline uint32_t incl(uint64_t both_block, int t, int lane) {
  return (uint32_t)(readlane_u64(both_block, t) >> lane) & 1u;
}

// Uniform-address load through the constant address space: always selected as SMEM
// (s_load, lgkmcnt) so it never queues behind the wave's outstanding vector stores.
template <typename T>
__device__ inline T sload(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}

struct Segment {
  uint32_t c0, c1;
};
__device__ inline Segment my_segment(uint32_t nchunks, uint32_t nwaves, uint32_t wave) {
  const uint32_t per = (nchunks + nwaves - 1) / nwaves;
  const uint32_t c0 = min(nchunks, wave * per);
  return {c0, min(nchunks, c0 + per)};
}

// ---------------------------------------------------------------------------------
// A pass
// ---------------------------------------------------------------------------------
// Every load in this loop is scalar (codes, posB, flags: s_load) or LDS (masks), so
// the only vector-memory instructions are the TB stores: nothing ever waits on vmcnt
// (CDNA4 counts loads and stores in one in-order vmcnt; a vector load consumed after
// outstanding stores would wait for all of them).
template <bool LDS, bool FULL, typename TBT>
__global__ __launch_bounds__(ENG_THREADS) void k_rankA(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gstart,
    const uint32_t* __restrict__ chunk_g, const uint32_t* __restrict__ gflag, uint32_t nchunks,
    const uint64_t* __restrict__ gmask, int64_t n, const uint32_t* __restrict__ posB_byA,
    TBT* __restrict__ TB, int lw, uint32_t* __restrict__ lpA, uint32_t* __restrict__ seg_tot,
    uint64_t* __restrict__ seg_part) {
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const int lane = threadIdx.x & 63;
  const bool active = FULL || lane < lw;
  const uint32_t stride = FULL ? (uint32_t)LANES : (uint32_t)lw;
  const uint32_t wave = wave_uniform(blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6));
  const Segment sg = my_segment(nchunks, gridDim.x * WAVES_PER_WG, wave);
  TBT* tb_lane = TB + lane;

  // chunk sums of k y~, k y~^2: 64-bit while chunk spans fit 16-bit ranks, else 128-bit
  using Acc = std::conditional_t<sizeof(TBT) == 2, uint64_t, u128>;
  uint32_t csl = 0;  // included count since the segment start
  u128 seg_k = 0, seg_ky = 0, seg_ky2 = 0;  // sums over the segment of k, k y', k y'^2
  for (uint32_t c = sg.c0; c < sg.c1; ++c) {
    lpA[(size_t)c * LANES + lane] = csl;
    const uint32_t p0 = sload(gstart + sload(chunk_g + c)), p1 = sload(gstart + sload(chunk_g + c + 1));
    uint32_t cl = 0, k = 0, gs = p0;     // chunk-relative count, open group's count/start
    Acc ky = 0, ky2 = 0;
    auto close_group = [&](uint32_t ge) {
      const uint32_t y = 2u * cl + k + 1u;  // chunk-relative doubled midrank
      if (active) {
        const TBT v = (TBT)y;
        for (uint32_t q = gs; q < ge; ++q) tb_lane[(size_t)sload(posB_byA + q) * stride] = v;
      }
      const uint64_t t = (uint64_t)k * y;
      ky += t;
      ky2 += (Acc)t * y;
      cl += k;
      k = 0;
      gs = ge;
    };
    uint32_t p = p0;
    for (; p < p1; p += 32) {
      const uint32_t nb = min(32u, p1 - p);
      const uint32_t f = (uint32_t)((((uint64_t)sload(gflag + (p >> 5) + 1) << 32) |
                                      sload(gflag + (p >> 5))) >> (p & 31));
#pragma unroll 8
      for (uint32_t t = 0; t < nb; ++t) {
        if (((f >> t) & 1u) && p + t != gs) close_group(p + t);
        const uint32_t code = sload(codes + p + t);
        const uint64_t both = m[code >> 16] & m[code & 0xffffu];
        k += (uint32_t)(both >> lane) & 1u;
      }
    }
    close_group(p1);  // chunks end on a group boundary
    // fold the chunk into the segment sums with its base lp = csl:  y' = y~ + 2 lp
    const u128 lp = csl, K = cl;
    seg_k += K;
    seg_ky += (u128)ky + 2 * lp * K;
    seg_ky2 += (u128)ky2 + 4 * lp * (u128)ky + 4 * lp * lp * K;
    csl += cl;
  }
  seg_tot[(size_t)wave * LANES + lane] = csl;
  uint64_t* o = seg_part + ((size_t)wave * LANES + lane) * 3;
  o[0] = (uint64_t)seg_ky;  // sum k y' fits 64 bits for any segment of < 2^31 pairs
  o[1] = (uint64_t)seg_ky2;
  o[2] = (uint64_t)(seg_ky2 >> 64);
  (void)seg_k;
}

// Exclusive scan of per-segment totals (per lane), one block of 16 waves.
__global__ __launch_bounds__(1024) void k_scan_seg(const uint32_t* __restrict__ tot,
                                                  uint32_t nseg, uint32_t* __restrict__ pre,
                                                  uint32_t* __restrict__ total) {
  __shared__ uint32_t part[16][LANES];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const uint32_t per = (nseg + 15) / 16;
  const uint32_t s0 = min(nseg, v * per), s1 = min(nseg, s0 + per);
  uint32_t s = 0;
  for (uint32_t i = s0; i < s1; ++i) s += tot[(size_t)i * LANES + lane];
  part[v][lane] = s;
  __syncthreads();
  uint32_t run = 0;
  for (int u = 0; u < v; ++u) run += part[u][lane];
  for (uint32_t i = s0; i < s1; ++i) {
    const uint32_t t = tot[(size_t)i * LANES + lane];
    pre[(size_t)i * LANES + lane] = run;
    run += t;
  }
  if (v == 15 && total) total[lane] = run;
}

__global__ void k_add_base(const uint32_t* __restrict__ lpA, const uint32_t* __restrict__ segpre,
                           uint32_t nchunks, uint32_t nwaves, uint32_t* __restrict__ baseA) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)nchunks * LANES) return;
  const uint32_t c = (uint32_t)(i / LANES), lane = (uint32_t)(i % LANES);
  const uint32_t per = (nchunks + nwaves - 1) / nwaves;
  baseA[i] = segpre[(size_t)(c / per) * LANES + lane] + lpA[i];
}

// ---------------------------------------------------------------------------------
// B pass
// ---------------------------------------------------------------------------------
// Loads only (no stores in the loop): 16 TB rows + 16 baseA rows + one lane-parallel
// code / chunk load per 16 pairs. Per-group sums are u64 and chunk-local; each chunk is
// folded into the u128 segment sums once.
template <bool LDS, bool FULL, typename TBT, bool WIDEB>
__global__ __launch_bounds__(ENG_THREADS) void k_rankB(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gstart,
    const uint32_t* __restrict__ chunk_g, const uint32_t* __restrict__ gflag, uint32_t nchunks,
    const uint64_t* __restrict__ gmask, int64_t n, const TBT* __restrict__ TB, int lw,
    const uint32_t* __restrict__ chunkA_byB, const uint32_t* __restrict__ baseA,
    uint32_t* __restrict__ seg_tot, uint64_t* __restrict__ seg_part) {
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const int lane = threadIdx.x & 63;
  const uint32_t sub = lane & (U - 1);
  const bool active = FULL || lane < lw;
  const uint32_t stride = FULL ? (uint32_t)LANES : (uint32_t)lw;
  const uint32_t wave = wave_uniform(blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6));
  const Segment sg = my_segment(nchunks, gridDim.x * WAVES_PER_WG, wave);
  const TBT* tb_lane = TB + lane;
  const uint32_t* base_lane = baseA + lane;

  // chunk sums: 64-bit unless B's chunks can span > 32k positions or ranks exceed 2^32/2^16
  using Acc = std::conditional_t<WIDEB, u128, uint64_t>;
  uint32_t csl = 0;
  u128 acc = 0, St = 0, ny = 0, ny2 = 0;  // segment sums (B side relative to segment start)
  for (uint32_t c = sg.c0; c < sg.c1; ++c) {
    const uint32_t p0 = gstart[chunk_g[c]], p1 = gstart[chunk_g[c + 1]];
    uint32_t cl = 0, k = 0;
    uint64_t S = 0;
    Acc cacc = 0, cSt = 0, cny = 0, cny2 = 0;
    auto close_group = [&]() {
      const uint32_t y = 2u * cl + k + 1u;  // chunk-relative doubled B midrank
      cacc += (Acc)S * y;
      cSt += S;
      const uint64_t t = (uint64_t)k * y;
      cny += t;
      cny2 += (Acc)t * y;
      cl += k;
      k = 0;
      S = 0;
    };
    auto block = [&](uint32_t p, uint32_t nb, auto full_tag) {
      constexpr bool FB = decltype(full_tag)::value;
      const uint32_t f = flags16(gflag, p);
      const uint32_t ca = (FB || sub < nb) ? chunkA_byB[p + sub] : 0u;
      const TBT* row = tb_lane + (size_t)p * stride;
      uint32_t ya[U];
#pragma unroll
      for (int t = 0; t < U; ++t) {
        if (active && (FB || (uint32_t)t < nb)) {
          const uint32_t cat = readlane_u32(ca, t);
          ya[t] = 2u * base_lane[(size_t)cat * LANES] + (uint32_t)row[(size_t)t * stride];
        } else {
          ya[t] = 0u;
        }
      }
      const uint64_t both = block_masks(m, codes, p, nb, lane);
#pragma unroll
      for (int t = 0; t < U; ++t) {
        if (FB || (uint32_t)t < nb) {
          if ((f >> t) & 1u) close_group();  // empty groups contribute nothing
          const uint32_t inc = incl(both, t, lane);
          S += inc ? (uint64_t)ya[t] : 0ull;
          k += inc;
        }
      }
    };
    uint32_t p = p0;
    for (; p + U <= p1; p += U) block(p, (uint32_t)U, std::true_type{});
    if (p < p1) block(p, p1 - p, std::false_type{});
    close_group();
    // fold: y'_B = y~ + 2 lp with lp = csl (segment-relative)
    const u128 lp = csl, K = cl;
    acc += (u128)cacc + 2 * lp * (u128)cSt;
    St += cSt;
    ny += (u128)cny + 2 * lp * K;
    ny2 += (u128)cny2 + 4 * lp * (u128)cny + 4 * lp * lp * K;
    csl += cl;
  }
  seg_tot[(size_t)wave * LANES + lane] = csl;
  uint64_t* o = seg_part + ((size_t)wave * LANES + lane) * 6;
  o[0] = (uint64_t)acc;
  o[1] = (uint64_t)(acc >> 64);
  o[2] = (uint64_t)St;
  o[3] = (uint64_t)ny;
  o[4] = (uint64_t)ny2;
  o[5] = (uint64_t)(ny2 >> 64);
}

// ---------------------------------------------------------------------------------
// final combination
// ---------------------------------------------------------------------------------
__device__ inline double i128_to_f64(i128 x) {
  const bool neg = x < 0;
  u128 u = neg ? (u128)(-x) : (u128)x;
  double d = (double)(uint64_t)(u >> 64) * 18446744073709551616.0 + (double)(uint64_t)u;
  return neg ? -d : d;
}

__global__ __launch_bounds__(1024) void k_final(
    const uint32_t* __restrict__ segA_tot, const uint64_t* __restrict__ segA_part,
    const uint32_t* __restrict__ segA_pre, const uint32_t* __restrict__ segB_tot,
    const uint64_t* __restrict__ segB_part, uint32_t nseg, const PlanHeader* __restrict__ hA,
    const PlanHeader* __restrict__ hB, int nl, double* __restrict__ scores) {
  __shared__ uint32_t cnt[16][LANES];
  __shared__ u128 red[3][16][LANES];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const uint32_t per = (nseg + 15) / 16;
  const uint32_t s0 = min(nseg, v * per), s1 = min(nseg, s0 + per);
  uint32_t c = 0;
  for (uint32_t s = s0; s < s1; ++s) c += segB_tot[(size_t)s * LANES + lane];
  cnt[v][lane] = c;
  __syncthreads();
  u128 bB = 0;
  for (int u = 0; u < v; ++u) bB += cnt[u][lane];
  u128 a2 = 0, ab = 0, b2 = 0;
  for (uint32_t s = s0; s < s1; ++s) {
    const size_t i = (size_t)s * LANES + lane;
    // A side: sum over groups of k (2 bA + y')^2
    const u128 kA = segA_tot[i], bA = segA_pre[i];
    const uint64_t* pa = segA_part + i * 3;
    const u128 nyA = pa[0], ny2A = ((u128)pa[2] << 64) | pa[1];
    a2 += 4 * bA * bA * kA + 4 * bA * nyA + ny2A;
    // B side
    const u128 kB = segB_tot[i];
    const uint64_t* pb = segB_part + i * 6;
    const u128 acc = ((u128)pb[1] << 64) | pb[0];
    const u128 St = pb[2], nyB = pb[3], ny2B = ((u128)pb[5] << 64) | pb[4];
    ab += acc + 2 * bB * St;
    b2 += 4 * bB * bB * kB + 4 * bB * nyB + ny2B;
    bB += kB;
  }
  red[0][v][lane] = a2;
  red[1][v][lane] = ab;
  red[2][v][lane] = b2;
  __syncthreads();
  if (v != 0) return;
  uint32_t Mp32 = 0;
  for (int u = 0; u < 16; ++u) Mp32 += cnt[u][lane];
  for (int u = 1; u < 16; ++u) {
    a2 += red[0][u][lane];
    ab += red[1][u][lane];
    b2 += red[2][u][lane];
  }
  if (lane >= nl) return;
  const u128 Mp = Mp32;
  const u128 mu = Mp * (Mp + 1) * (Mp + 1);
  const i128 num = (i128)ab - (i128)mu;
  const i128 va = (i128)a2 - (i128)mu;
  const i128 vb = (i128)b2 - (i128)mu;
  double r;
  if (hA->has_nan || hB->has_nan || Mp < 2 || va <= 0 || vb <= 0) {
    r = __builtin_nan("");
  } else {
    r = i128_to_f64(num) / sqrt(i128_to_f64(va) * i128_to_f64(vb));
    r = r > 1.0 ? 1.0 : (r < -1.0 ? -1.0 : r);
  }
  scores[lane] = r;
}

__global__ void k_fill_nan(double* out, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = __builtin_nan("");
}

// ---------------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------------
template <bool LDS, bool FULL, typename TBT, bool WIDEB>
static int set_lds_attr() {
  static bool done = false;
  if (LDS && !done) {
    const int mx = 160 * 1024;
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_rankA<LDS, FULL, TBT>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_rankB<LDS, FULL, TBT, WIDEB>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    done = true;
  }
  return VR_OK;
}

template <bool LDS, bool FULL, typename TBT, bool WIDEB>
static int run_pass(const PlanView& A, const PlanView& B, int64_t n, const EngineWs& E, int lw,
                    int nl, double* scores_out, const EngineCfg& cfg, hipStream_t st) {
  const int64_t M = pairs_of(n);
  const uint32_t nch = plan_nchunks(M);
  VR_TRY((set_lds_attr<LDS, FULL, TBT, WIDEB>()));
  TBT* TB = static_cast<TBT*>(E.TB);
  k_rankA<LDS, FULL, TBT><<<cfg.grid, ENG_THREADS, cfg.lds, st>>>(
      A.codes, A.gstart, A.chunk_g, A.gflag, nch, E.masks, n, E.posB_byA, TB, lw, E.lpA,
      E.segA_tot, E.segA_part);
  VR_CHECK_LAUNCH();
  k_scan_seg<<<1, 1024, 0, st>>>(E.segA_tot, (uint32_t)cfg.nwaves, E.segA_pre, E.totA);
  VR_CHECK_LAUNCH();
  const size_t nb = ((size_t)nch * LANES + 255) / 256;
  k_add_base<<<(unsigned)nb, 256, 0, st>>>(E.lpA, E.segA_pre, nch, (uint32_t)cfg.nwaves, E.baseA);
  VR_CHECK_LAUNCH();
  k_rankB<LDS, FULL, TBT, WIDEB><<<cfg.grid, ENG_THREADS, cfg.lds, st>>>(
      B.codes, B.gstart, B.chunk_g, B.gflag, nch, E.masks, n, TB, lw, E.chunkA_byB, E.baseA,
      E.segB_tot, E.segB_part);
  VR_CHECK_LAUNCH();
  k_final<<<1, 1024, 0, st>>>(E.segA_tot, E.segA_part, E.segA_pre, E.segB_tot, E.segB_part,
                              (uint32_t)cfg.nwaves, A.hdr, B.hdr, nl, scores_out);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

template <bool LDS, bool FULL>
static int run_pass_tb(bool narrow, bool wideb, const PlanView& A, const PlanView& B, int64_t n,
                       const EngineWs& E, int lw, int nl, double* out, const EngineCfg& cfg,
                       hipStream_t st) {
  if (narrow)
    return wideb ? run_pass<LDS, FULL, uint16_t, true>(A, B, n, E, lw, nl, out, cfg, st)
                 : run_pass<LDS, FULL, uint16_t, false>(A, B, n, E, lw, nl, out, cfg, st);
  return wideb ? run_pass<LDS, FULL, uint32_t, true>(A, B, n, E, lw, nl, out, cfg, st)
               : run_pass<LDS, FULL, uint32_t, false>(A, B, n, E, lw, nl, out, cfg, st);
}

// Scores for `total` subsets (full set first if full_first), 64 per pass.
static int run_engine(const PlanView& A, const PlanView& B, int64_t n, const int32_t* idx,
                      int64_t k, int64_t n_sets, int full_first, double* scores,
                      const EngineWs& E, int lw, const EngineCfg& cfg, hipStream_t st) {
  const int64_t M = pairs_of(n);
  const int64_t total = n_sets + (full_first ? 1 : 0);
  if (total == 0) return VR_OK;
  if (M == 0) {  // no pairs: every score is NaN (scipy on empty input)
    k_fill_nan<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(scores, total);
    VR_CHECK_LAUNCH();
    return VR_OK;
  }
  // u16 chunk-relative ranks need every chunk span (< L + largest tie group) <= 32767;
  // B's 64-bit chunk sums need the same of B and absolute ranks (2M+1) below 2^33
  PlanHeader h[2];
  VR_CHECK_HIP(hipMemcpyAsync(&h[0], A.hdr, sizeof(PlanHeader), hipMemcpyDeviceToHost, st));
  VR_CHECK_HIP(hipMemcpyAsync(&h[1], B.hdr, sizeof(PlanHeader), hipMemcpyDeviceToHost, st));
  VR_CHECK_HIP(hipStreamSynchronize(st));
  const bool narrow = (uint64_t)PLAN_L + h[0].max_group <= 32767u;
  const bool wideb = (uint64_t)PLAN_L + h[1].max_group > 32767u || M > (int64_t)1 << 30;
  k_join<<<(unsigned)((M + 255) / 256), 256, 0, st>>>(A.codes, B.codes, M, n, B.pos_of_pair,
                                                     A.chunk_of_pair, E.posB_byA, E.chunkA_byB);
  VR_CHECK_LAUNCH();
  for (int64_t set0 = 0; set0 < total; set0 += lw) {
    const int nl = (int)std::min<int64_t>(lw, total - set0);
    VR_CHECK_HIP(hipMemsetAsync(E.masks, 0, (size_t)n * sizeof(uint64_t), st));
    if (full_first && set0 == 0) {
      k_masks_full<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(E.masks, n);
      VR_CHECK_LAUNCH();
    }
    const int64_t nrows = nl - ((full_first && set0 == 0) ? 1 : 0);
    if (nrows > 0 && k > 0) {
      dim3 grid((unsigned)std::min<int64_t>((k + 255) / 256, 64), (unsigned)nl);
      k_masks_sets<<<grid, 256, 0, st>>>(idx, k, set0, nl, full_first, E.masks);
      VR_CHECK_LAUNCH();
    }
    double* out = scores + set0;
    if (cfg.use_lds) {
      if (lw == LANES)
        VR_TRY((run_pass_tb<true, true>(narrow, wideb, A, B, n, E, lw, nl, out, cfg, st)));
      else
        VR_TRY((run_pass_tb<true, false>(narrow, wideb, A, B, n, E, lw, nl, out, cfg, st)));
    } else {
      if (lw == LANES)
        VR_TRY((run_pass_tb<false, true>(narrow, wideb, A, B, n, E, lw, nl, out, cfg, st)));
      else
        VR_TRY((run_pass_tb<false, false>(narrow, wideb, A, B, n, E, lw, nl, out, cfg, st)));
    }
  }
  return VR_OK;
}

static size_t oneshot_bytes(int64_t n, int lw, int nwaves, void* base, PlanView* A, PlanView* B,
                            PlanBuildWs* W, EngineWs* E) {
  Carver c(base);
  const size_t pb = plan_bytes(n);
  char* pa = c.take<char>(pb);
  char* pbb = c.take<char>(pb);
  size_t wb = 0, eb = 0;
  plan_build_layout(nullptr, n, &wb);
  engine_layout(nullptr, n, lw, nwaves, &eb);
  char* wsb = c.take<char>(std::max(wb, eb));  // plan-build scratch is dead once plans exist
  if (base) {
    *A = plan_layout(pa, n);
    *B = plan_layout(pbb, n);
    *W = plan_build_layout(wsb, n, nullptr);
    *E = engine_layout(wsb, n, lw, nwaves, nullptr);
  }
  return c.bytes();
}

}  // namespace vr

using namespace vr;

extern "C" {

size_t vr_bootstrap_workspace(int64_t n) {
  size_t b = 0;
  n = n < 0 ? 0 : n;
  engine_layout(nullptr, n, LANES, engine_cfg(n).nwaves, &b);
  return b;
}

int vr_bootstrap_spearman_plans(const void* planA, const void* planB, int64_t n,
                                const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                                double* scores, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535, "vr_bootstrap_spearman_plans: n=%lld out of range", (long long)n);
  VR_REQUIRE(planA && planB && scores, "vr_bootstrap_spearman_plans: null pointer");
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "vr_bootstrap_spearman_plans: bad k=%lld sets=%lld",
             (long long)k, (long long)n_sets);
  VR_REQUIRE(idx != nullptr || n_sets == 0 || k == 0, "vr_bootstrap_spearman_plans: null idx");
  const EngineCfg cfg = engine_cfg(n);
  size_t need = 0;
  EngineWs E = engine_layout(ws, n, LANES, cfg.nwaves, &need);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_bootstrap_spearman_plans: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView A = plan_layout(const_cast<void*>(planA), n);
  PlanView B = plan_layout(const_cast<void*>(planB), n);
  return run_engine(A, B, n, idx, k, n_sets, full_first, scores, E, LANES, cfg, as_stream(stream));
}

size_t vr_bootstrap_spearman_workspace(int64_t n) {
  n = n < 0 ? 0 : n;
  return oneshot_bytes(n, LANES, engine_cfg(n).nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int vr_bootstrap_spearman_f32(const float* A, const float* B, int64_t n, int64_t ld,
                              const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                              double* scores, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535 && ld >= n, "vr_bootstrap_spearman_f32: bad shape");
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "vr_bootstrap_spearman_f32: bad k");
  VR_REQUIRE(scores != nullptr, "vr_bootstrap_spearman_f32: null scores");
  const EngineCfg cfg = engine_cfg(n);
  const size_t need = oneshot_bytes(n, LANES, cfg.nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_bootstrap_spearman_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView PA, PB;
  PlanBuildWs W;
  EngineWs E;
  oneshot_bytes(n, LANES, cfg.nwaves, ws, &PA, &PB, &W, &E);
  hipStream_t st = as_stream(stream);
  VR_TRY(build_plan(A, n, ld, PA, W, st));
  VR_TRY(build_plan(B, n, ld, PB, W, st));
  return run_engine(PA, PB, n, idx, k, n_sets, full_first, scores, E, LANES, cfg, st);
}

size_t vr_spearman_triu_workspace(int64_t n) {
  n = n < 0 ? 0 : n;
  return oneshot_bytes(n, 1, engine_cfg(n).nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int vr_spearman_triu_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out,
                         void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535 && ld >= n, "vr_spearman_triu_f32: bad shape n=%lld ld=%lld",
             (long long)n, (long long)ld);
  VR_REQUIRE(out != nullptr, "vr_spearman_triu_f32: null out");
  const EngineCfg cfg = engine_cfg(n);
  const size_t need = oneshot_bytes(n, 1, cfg.nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_spearman_triu_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView PA, PB;
  PlanBuildWs W;
  EngineWs E;
  oneshot_bytes(n, 1, cfg.nwaves, ws, &PA, &PB, &W, &E);
  hipStream_t st = as_stream(stream);
  VR_TRY(build_plan(A, n, ld, PA, W, st));
  VR_TRY(build_plan(B, n, ld, PB, W, st));
  return run_engine(PA, PB, n, nullptr, 0, 0, 1, out, E, 1, cfg, st);
}

}  // extern "C"
