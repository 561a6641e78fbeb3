// Upper-triangle midrank Spearman and the bootstrapped Spearman RSA engine.
//
// Replaces, per (model RDM, neural RDM) unit, the reference loop
//   point = spearmanr(triu(A), triu(B))                               evals.py:347-349
//   for i in range(1000): idx = rng.choice(n, int(.9n), replace=False)
//       scores[i] = spearmanr(triu(A[idx][:,idx]), triu(B[idx][:,idx]))  evals.py:361-369
// with scipy's average-rank (midrank) ties (rsa.py:43-47,121-122).
//
// Rank plan (once per RDM): the M = n(n-1)/2 strict-upper-triangle values are radix
// sorted; equal fp32 values form tie groups; positions are cut into chunks of ~L pairs
// aligned to group starts. For any subset S of stimuli, a pair (a,b) is included iff
// a, b in S, and its midrank among included pairs is  (c_s + c_e + 1)/2  where c_s,
// c_e are the included counts before / through its tie group in sorted order. We keep
// everything in doubled ranks (integers): y = 2*rank = 2*c_s + n_g + 1.
//
// Engine (64 subsets per pass, lane w of every wave = subset w):
//  masks[x] bit w = (stimulus x in subset w)                      (LDS, 8 B/stimulus)
//  countA : per A-chunk included counts               -> scanA: chunk bases
//  rankA  : walk A order per chunk, per group y_A = 2c_s+n+1, scatter y_A to the
//           pair's B position: TB[posB(pair)][w]                 (256 B rows, coalesced)
//  rankB  : walk B order per chunk, stream TB rows; per B group with local base
//           accumulate S = sum y_A, y_B,loc * S, n*y_B,loc, n*y_B,loc^2 (exact ints)
//  final  : combine with B chunk bases; rho = (sum yA yB - M'(M'+1)^2) /
//           sqrt((sum yA^2 - M'(M'+1)^2)(sum yB^2 - M'(M'+1)^2))   (int128 -> fp64)
// Every sum is an exact integer, so scores are independent of chunking, lane
// grouping, launch order and GPU count.
#include <type_traits>

#include "internal.h"

namespace vr {

typedef unsigned __int128 u128;
typedef __int128 i128;

constexpr uint32_t PLAN_L = 4096;  // target pairs per chunk
constexpr int ENG_THREADS = 512;   // 8 waves per workgroup
constexpr int LANES = 64;

struct PlanHeader {
  int64_t n;
  int64_t M;
  uint32_t G;        // tie groups (device-written)
  uint32_t nchunks;
  uint32_t L;
  uint32_t has_nan;  // device-written
  uint32_t pad[56];
};
static_assert(sizeof(PlanHeader) == 256, "header size");

struct PlanView {
  PlanHeader* hdr;
  uint32_t* codes;       // [M]    (a << 16) | b, sorted by value
  uint32_t* gstart;      // [M+1]  first G+1 valid: position of each group start, gstart[G]=M
  uint32_t* pos_of_pair; // [M]    triangle index -> sorted position
  uint32_t* chunk_g;     // [nchunks+1] first group of each chunk
  uint32_t* gflag;       // [(M+31)/32 + 2] bit i = position i starts a tie group
};

static inline uint32_t plan_nchunks(int64_t M) { return (uint32_t)((M + PLAN_L - 1) / PLAN_L); }

static PlanView plan_layout(void* base, int64_t n) {
  const int64_t M = pairs_of(n);
  Carver c(base);
  PlanView v;
  v.hdr = c.take<PlanHeader>(1);
  v.codes = c.take<uint32_t>((size_t)M);
  v.gstart = c.take<uint32_t>((size_t)M + 1);
  v.pos_of_pair = c.take<uint32_t>((size_t)M);
  v.chunk_g = c.take<uint32_t>((size_t)plan_nchunks(M) + 1);
  v.gflag = c.take<uint32_t>((size_t)(M + 31) / 32 + 2);
  return v;
}
static size_t plan_bytes(int64_t n) {
  Carver c(nullptr);
  const int64_t M = pairs_of(n);
  c.take<PlanHeader>(1);
  c.take<uint32_t>((size_t)M);
  c.take<uint32_t>((size_t)M + 1);
  c.take<uint32_t>((size_t)M);
  c.take<uint32_t>((size_t)plan_nchunks(M) + 1);
  c.take<uint32_t>((size_t)(M + 31) / 32 + 2);
  return c.bytes();
}

struct PlanBuildWs {
  uint32_t *keys, *keys_alt, *vals_alt, *flags, *gidx, *radix, *scan;
};
static PlanBuildWs plan_build_layout(void* base, int64_t n, size_t* bytes) {
  const int64_t M = pairs_of(n);
  Carver c(base);
  PlanBuildWs w;
  w.keys = c.take<uint32_t>((size_t)M);
  w.keys_alt = c.take<uint32_t>((size_t)M);
  w.vals_alt = c.take<uint32_t>((size_t)M);
  w.flags = c.take<uint32_t>((size_t)M);
  w.gidx = c.take<uint32_t>((size_t)M);
  w.radix = c.take<uint32_t>(radix_ws_elems(M));
  w.scan = c.take<uint32_t>(scan_ws_elems(M));
  if (bytes) *bytes = c.bytes();
  return w;
}

// ---------------------------------------------------------------------------------
// Plan construction
// ---------------------------------------------------------------------------------
__global__ void k_triu_keys(const float* __restrict__ rdm, int64_t n, int64_t ld,
                            uint32_t* __restrict__ keys, uint32_t* __restrict__ codes,
                            PlanHeader* hdr, int64_t col_blocks) {
  const int64_t a = blockIdx.x / col_blocks;
  const int64_t b = (blockIdx.x % col_blocks) * blockDim.x + threadIdx.x;
  if (b <= a || b >= n) return;
  const float v = rdm[a * ld + b];
  if (v != v) atomicOr(&hdr->has_nan, 1u);
  const uint64_t t = tri_index((uint64_t)a, (uint64_t)b, (uint64_t)n);
  keys[t] = f32_sort_key(v);
  codes[t] = ((uint32_t)a << 16) | (uint32_t)b;
}

__global__ void k_group_flags(const uint32_t* __restrict__ keys, int64_t M,
                              uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  flags[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ void k_group_starts(const uint32_t* __restrict__ flags,
                               const uint32_t* __restrict__ gidx, int64_t M,
                               uint32_t* __restrict__ gstart) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  if (flags[i]) gstart[gidx[i]] = (uint32_t)i;
  if (i == M - 1) gstart[gidx[i] + flags[i]] = (uint32_t)M;
}

__global__ void k_pos_of_pair(const uint32_t* __restrict__ codes, int64_t M, int64_t n,
                              uint32_t* __restrict__ pos_of_pair) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t c = codes[i];
  pos_of_pair[tri_index(c >> 16, c & 0xffffu, (uint64_t)n)] = (uint32_t)i;
}

// chunk_g[c] = first group whose start position is >= c*L (group-aligned chunks).
__global__ void k_chunk_groups(const uint32_t* __restrict__ gstart,
                               const PlanHeader* __restrict__ hdr, uint32_t nchunks,
                               uint32_t L, uint32_t* __restrict__ chunk_g, int64_t M) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t G = hdr->G;
  if (g > G) return;
  const int64_t cg = (g == G) ? (int64_t)nchunks : (int64_t)(gstart[g] / L);
  const int64_t cp = (g == 0) ? -1 : (int64_t)(gstart[g - 1] / L);
  for (int64_t c = cp + 1; c <= cg; ++c) chunk_g[c] = (uint32_t)g;
  (void)M;
}

__global__ void k_init_header(PlanHeader* hdr, int64_t n, int64_t M, uint32_t nchunks,
                              uint32_t L) {
  if (threadIdx.x == 0) {
    hdr->n = n;
    hdr->M = M;
    hdr->G = 0;
    hdr->nchunks = nchunks;
    hdr->L = L;
    hdr->has_nan = 0;
  }
}

__global__ void k_pack_flags(const uint32_t* __restrict__ flags, int64_t M,
                             uint32_t* __restrict__ gflag, int64_t words) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= words) return;
  uint32_t v = 0;
  for (int b = 0; b < 32; ++b) {
    const int64_t i = w * 32 + b;
    if (i < M && flags[i]) v |= 1u << b;
  }
  gflag[w] = v;
}

static int build_plan(const float* rdm, int64_t n, int64_t ld, const PlanView& P,
                      const PlanBuildWs& W, hipStream_t st) {
  const int64_t M = pairs_of(n);
  const uint32_t nchunks = plan_nchunks(M);
  k_init_header<<<1, 64, 0, st>>>(P.hdr, n, M, nchunks, PLAN_L);
  VR_CHECK_LAUNCH();
  if (M == 0) {
    VR_CHECK_HIP(hipMemsetAsync(P.gstart, 0, sizeof(uint32_t), st));
    VR_CHECK_HIP(hipMemsetAsync(P.chunk_g, 0, sizeof(uint32_t), st));
    return VR_OK;
  }
  const int64_t col_blocks = (n + 255) / 256;
  k_triu_keys<<<(unsigned)(n * col_blocks), 256, 0, st>>>(rdm, n, ld, W.keys, P.codes, P.hdr,
                                                          col_blocks);
  VR_CHECK_LAUNCH();
  VR_TRY(radix_sort_kv(W.keys, P.codes, W.keys_alt, W.vals_alt, M, W.radix, st));
  const unsigned gb = (unsigned)((M + 255) / 256);
  k_group_flags<<<gb, 256, 0, st>>>(W.keys, M, W.flags);
  VR_CHECK_LAUNCH();
  VR_TRY(scan_exclusive_u32(W.flags, W.gidx, M, &P.hdr->G, W.scan, st));
  k_group_starts<<<gb, 256, 0, st>>>(W.flags, W.gidx, M, P.gstart);
  VR_CHECK_LAUNCH();
  k_pos_of_pair<<<gb, 256, 0, st>>>(P.codes, M, n, P.pos_of_pair);
  VR_CHECK_LAUNCH();
  k_chunk_groups<<<(unsigned)((M + 1 + 255) / 256), 256, 0, st>>>(P.gstart, P.hdr, nchunks,
                                                                  PLAN_L, P.chunk_g, M);
  VR_CHECK_LAUNCH();
  const int64_t words = (M + 31) / 32 + 2;
  k_pack_flags<<<(unsigned)((words + 255) / 256), 256, 0, st>>>(W.flags, M, P.gflag, words);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// ---------------------------------------------------------------------------------
// Engine
// ---------------------------------------------------------------------------------
struct EngineWs {
  uint64_t* masks;     // [n]
  uint32_t* cntA;      // [nchA*64]
  uint32_t* baseA;     // [nchA*64]
  uint32_t* totA;      // [64]
  uint64_t* partA;     // [nchA*64*2]    sum n*y^2 (u128)
  uint32_t* posB_byA;  // [M]
  uint32_t* TB;        // [M*lw]
  uint64_t* partB;     // [nchB*64*6]
  uint32_t* cntB;      // [nchB*64]
  uint32_t* baseB;     // [nchB*64]
  uint32_t* totB;      // [64]
};

static EngineWs engine_layout(void* base, int64_t n, int lw, size_t* bytes) {
  const int64_t M = pairs_of(n);
  const uint32_t nch = plan_nchunks(M);
  Carver c(base);
  EngineWs e;
  e.masks = c.take<uint64_t>((size_t)n);
  e.cntA = c.take<uint32_t>((size_t)nch * LANES);
  e.baseA = c.take<uint32_t>((size_t)nch * LANES);
  e.totA = c.take<uint32_t>(LANES);
  e.partA = c.take<uint64_t>((size_t)nch * LANES * 2);
  e.posB_byA = c.take<uint32_t>((size_t)M);
  e.TB = c.take<uint32_t>((size_t)M * (size_t)lw);
  e.partB = c.take<uint64_t>((size_t)nch * LANES * 6);
  e.cntB = c.take<uint32_t>((size_t)nch * LANES);
  e.baseB = c.take<uint32_t>((size_t)nch * LANES);
  e.totB = c.take<uint32_t>(LANES);
  if (bytes) *bytes = c.bytes();
  return e;
}

__global__ void k_join(const uint32_t* __restrict__ codesA, int64_t M, int64_t n,
                       const uint32_t* __restrict__ posOfPairB, uint32_t* __restrict__ posB_byA) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t c = codesA[i];
  posB_byA[i] = posOfPairB[tri_index(c >> 16, c & 0xffffu, (uint64_t)n)];
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

template <bool LDS>
__device__ inline const uint64_t* stage_masks(const uint64_t* __restrict__ gmask, int64_t n,
                                              uint64_t* smem) {
  if (!LDS) return gmask;
  for (int64_t x = threadIdx.x; x < n; x += blockDim.x) smem[x] = gmask[x];
  __syncthreads();
  return smem;
}

__device__ inline uint32_t wave_uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ inline uint32_t incl_bit(const uint64_t* m, uint32_t code, int lane) {
  const uint64_t both = m[code >> 16] & m[code & 0xffffu];
  return (uint32_t)(both >> lane) & 1u;
}

constexpr int U = 16;  // pairs per block: one vector load brings 16 pair codes

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

// Per block of U positions, lane (l & 15) looks up the inclusion masks of pair
// (p + (l & 15)); the AND of both stimulus masks is then broadcast per pair.
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

template <bool LDS>
__global__ __launch_bounds__(ENG_THREADS) void k_boot_count(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gstart,
    const uint32_t* __restrict__ chunk_g, uint32_t nchunks,
    const uint64_t* __restrict__ gmask, int64_t n, uint32_t* __restrict__ cnt) {
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const int lane = threadIdx.x & 63;
  const uint32_t wave = wave_uniform(blockIdx.x * (ENG_THREADS / 64) + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * (ENG_THREADS / 64);
  for (uint32_t c = wave; c < nchunks; c += nwaves) {
    const uint32_t p0 = gstart[chunk_g[c]], p1 = gstart[chunk_g[c + 1]];
    uint32_t k = 0;
    uint32_t p = p0;
    for (; p + U <= p1; p += U) {
      const uint64_t both = block_masks(m, codes, p, U, lane);
#pragma unroll
      for (int t = 0; t < U; ++t) k += (uint32_t)(readlane_u64(both, t) >> lane) & 1u;
    }
    if (p < p1) {
      const uint32_t nb = p1 - p;
      const uint64_t both = block_masks(m, codes, p, nb, lane);
#pragma unroll
      for (int t = 0; t < U; ++t)
        if ((uint32_t)t < nb) k += (uint32_t)(readlane_u64(both, t) >> lane) & 1u;
    }
    cnt[(size_t)c * LANES + lane] = k;
  }
}

// Exclusive scan over chunks, independently per lane. One block, 16 waves.
__global__ __launch_bounds__(1024) void k_scan_chunks(const uint32_t* __restrict__ cnt,
                                                     uint32_t nchunks,
                                                     uint32_t* __restrict__ base,
                                                     uint32_t* __restrict__ total) {
  __shared__ uint32_t tot[16][LANES];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const uint32_t per = (nchunks + 15) / 16;
  const uint32_t c0 = v * per, c1 = min(nchunks, c0 + per);
  uint32_t s = 0;
  for (uint32_t c = c0; c < c1; ++c) s += cnt[(size_t)c * LANES + lane];
  tot[v][lane] = s;
  __syncthreads();
  uint32_t run = 0;
  for (int u = 0; u < v; ++u) run += tot[u][lane];
  for (uint32_t c = c0; c < c1; ++c) {
    const uint32_t t = cnt[(size_t)c * LANES + lane];
    base[(size_t)c * LANES + lane] = run;
    run += t;
  }
  if (v == 15) total[lane] = run;
}

// Lane w walks the chunk in sorted-A order; when a tie group closes its doubled
// midrank y = 2 c_s + k + 1 is scattered to the B positions of its members.
template <bool LDS, bool FULL>
__global__ __launch_bounds__(ENG_THREADS) void k_boot_rankA(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gstart,
    const uint32_t* __restrict__ chunk_g, const uint32_t* __restrict__ gflag,
    uint32_t nchunks, const uint64_t* __restrict__ gmask, int64_t n,
    const uint32_t* __restrict__ baseA, const uint32_t* __restrict__ posB_byA,
    uint32_t* __restrict__ TB, int lw, uint64_t* __restrict__ partA) {
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const int lane = threadIdx.x & 63;
  const uint32_t sub = lane & (U - 1);
  const bool active = FULL || lane < lw;
  const uint32_t stride = FULL ? (uint32_t)LANES : (uint32_t)lw;
  const uint32_t wave = wave_uniform(blockIdx.x * (ENG_THREADS / 64) + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * (ENG_THREADS / 64);
  for (uint32_t c = wave; c < nchunks; c += nwaves) {
    const uint32_t p0 = gstart[chunk_g[c]], p1 = gstart[chunk_g[c + 1]];
    if (p0 == p1) {
      partA[((size_t)c * LANES + lane) * 2 + 0] = 0;
      partA[((size_t)c * LANES + lane) * 2 + 1] = 0;
      continue;
    }
    uint32_t cs = baseA[(size_t)c * LANES + lane];
    uint32_t k = 0, gs = p0;
    u128 sq = 0;
    uint32_t pb = 0;  // posB of pair (p + sub) of the current block
    uint32_t p = p0;
    // closes the group [gs, ge); members at >= p are in the current block (readlane)
    auto close_group = [&](uint32_t ge) {
      const uint32_t y = 2u * cs + k + 1u;
      if (active) {
        for (uint32_t q = gs; q < ge; ++q) {
          const uint32_t dst = (q >= p) ? readlane_u32(pb, q - p) : posB_byA[q];
          TB[(size_t)dst * stride + lane] = y;
        }
      }
      sq += (u128)((uint64_t)k * y) * y;
      cs += k;
      k = 0;
      gs = ge;
    };
    auto block = [&](uint32_t nb, auto full_tag) {
      constexpr bool FB = decltype(full_tag)::value;
      const uint32_t f = flags16(gflag, p);
      const uint64_t both = block_masks(m, codes, p, nb, lane);
      pb = (FB || sub < nb) ? posB_byA[p + sub] : 0u;
#pragma unroll
      for (int t = 0; t < U; ++t) {
        if (FB || (uint32_t)t < nb) {
          if (((f >> t) & 1u) && p + t != gs) close_group(p + t);
          k += (uint32_t)(readlane_u64(both, t) >> lane) & 1u;
        }
      }
    };
    for (; p + U <= p1; p += U) block((uint32_t)U, std::true_type{});
    if (p < p1) block(p1 - p, std::false_type{});
    if (p >= p1) p = p1 - 1 - ((p1 - 1 - p0) % U);  // readlane base of the last block
    close_group(p1);  // chunks end on a group boundary
    partA[((size_t)c * LANES + lane) * 2 + 0] = (uint64_t)sq;
    partA[((size_t)c * LANES + lane) * 2 + 1] = (uint64_t)(sq >> 64);
  }
}

// Lane w walks the chunk in sorted-B order, streaming the y_A row of every pair; per B
// tie group it accumulates S = sum of included y_A, then y_B(local) * S etc.
template <bool LDS, bool FULL>
__global__ __launch_bounds__(ENG_THREADS) void k_boot_rankB(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gstart,
    const uint32_t* __restrict__ chunk_g, const uint32_t* __restrict__ gflag,
    uint32_t nchunks, const uint64_t* __restrict__ gmask, int64_t n,
    const uint32_t* __restrict__ TB, int lw, uint64_t* __restrict__ partB,
    uint32_t* __restrict__ cntB) {
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const int lane = threadIdx.x & 63;
  const bool active = FULL || lane < lw;
  const uint32_t stride = FULL ? (uint32_t)LANES : (uint32_t)lw;
  const uint32_t wave = wave_uniform(blockIdx.x * (ENG_THREADS / 64) + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * (ENG_THREADS / 64);
  for (uint32_t c = wave; c < nchunks; c += nwaves) {
    const uint32_t p0 = gstart[chunk_g[c]], p1 = gstart[chunk_g[c + 1]];
    uint32_t csl = 0, k = 0;
    u128 acc = 0, ny2 = 0;
    uint64_t St = 0, ny = 0, S = 0;
    auto close_group = [&]() {
      const uint32_t y = 2u * csl + k + 1u;
      acc += (u128)S * y;
      St += S;
      const uint64_t ky = (uint64_t)k * y;
      ny += ky;
      ny2 += (u128)ky * y;
      csl += k;
      k = 0;
      S = 0;
    };
    auto block = [&](uint32_t p, uint32_t nb, auto full_tag) {
      constexpr bool FB = decltype(full_tag)::value;
      const uint32_t f = flags16(gflag, p);
      uint32_t ya[U];
#pragma unroll
      for (int t = 0; t < U; ++t)
        ya[t] = (active && (FB || (uint32_t)t < nb)) ? TB[(size_t)(p + t) * stride + lane] : 0u;
      const uint64_t both = block_masks(m, codes, p, nb, lane);
#pragma unroll
      for (int t = 0; t < U; ++t) {
        if (FB || (uint32_t)t < nb) {
          if ((f >> t) & 1u) close_group();  // empty groups contribute nothing
          const uint32_t inc = (uint32_t)(readlane_u64(both, t) >> lane) & 1u;
          S += inc ? (uint64_t)ya[t] : 0ull;
          k += inc;
        }
      }
    };
    uint32_t p = p0;
    for (; p + U <= p1; p += U) block(p, (uint32_t)U, std::true_type{});
    if (p < p1) block(p, p1 - p, std::false_type{});
    close_group();
    uint64_t* o = partB + ((size_t)c * LANES + lane) * 6;
    o[0] = (uint64_t)acc;
    o[1] = (uint64_t)(acc >> 64);
    o[2] = St;
    o[3] = ny;
    o[4] = (uint64_t)ny2;
    o[5] = (uint64_t)(ny2 >> 64);
    cntB[(size_t)c * LANES + lane] = csl;
  }
}

__device__ inline double i128_to_f64(i128 x) {
  const bool neg = x < 0;
  u128 u = neg ? (u128)(-x) : (u128)x;
  double d = (double)(uint64_t)(u >> 64) * 18446744073709551616.0 + (double)(uint64_t)u;
  return neg ? -d : d;
}

__global__ __launch_bounds__(1024) void k_boot_final(
    const uint64_t* __restrict__ partA, uint32_t nchA, const uint64_t* __restrict__ partB,
    const uint32_t* __restrict__ cntB, const uint32_t* __restrict__ baseB, uint32_t nchB,
    const uint32_t* __restrict__ totB, const PlanHeader* __restrict__ hA,
    const PlanHeader* __restrict__ hB, int nl, double* __restrict__ scores) {
  __shared__ u128 red[3][16][LANES];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  u128 a2 = 0, ab = 0, b2 = 0;
  for (uint32_t c = v; c < nchA; c += 16) {
    const uint64_t* p = partA + ((size_t)c * LANES + lane) * 2;
    a2 += ((u128)p[1] << 64) | p[0];
  }
  for (uint32_t c = v; c < nchB; c += 16) {
    const uint64_t* p = partB + ((size_t)c * LANES + lane) * 6;
    const u128 acc = ((u128)p[1] << 64) | p[0];
    const u128 St = p[2], ny = p[3];
    const u128 ny2 = ((u128)p[5] << 64) | p[4];
    const u128 bB = baseB[(size_t)c * LANES + lane];
    const u128 k = cntB[(size_t)c * LANES + lane];
    ab += acc + 2 * bB * St;
    b2 += 4 * bB * bB * k + 4 * bB * ny + ny2;
  }
  red[0][v][lane] = a2;
  red[1][v][lane] = ab;
  red[2][v][lane] = b2;
  __syncthreads();
  if (v != 0) return;
  for (int u = 1; u < 16; ++u) {
    a2 += red[0][u][lane];
    ab += red[1][u][lane];
    b2 += red[2][u][lane];
  }
  if (lane >= nl) return;
  const u128 Mp = totB[lane];
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

struct EngineCfg {
  int grid;
  size_t lds;
  bool use_lds;
};

static EngineCfg engine_cfg(int64_t n) {
  EngineCfg c;
  const size_t need = (size_t)n * sizeof(uint64_t);
  const size_t lds_cap = 160 * 1024;
  c.use_lds = need <= lds_cap - 1024;
  const int per_cu = c.use_lds ? std::max<int>(1, std::min<int>(2, (int)((lds_cap - 1024) / std::max<size_t>(need, 1)))) : 2;
  c.grid = num_cus() * per_cu;
  c.lds = c.use_lds ? need : 0;
  return c;
}

template <bool LDS>
static int set_lds_attr(size_t bytes) {
  static bool done = false;
  if (LDS && !done && bytes > 0) {
    const int mx = 160 * 1024;
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_boot_count<true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_boot_rankA<true, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_boot_rankA<true, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_boot_rankB<true, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_boot_rankB<true, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    done = true;
  }
  return VR_OK;
}

template <bool LDS>
static int run_pass(const PlanView& A, const PlanView& B, int64_t n, const EngineWs& E,
                    int lw, int nl, double* scores_out, const EngineCfg& cfg, hipStream_t st) {
  const int64_t M = pairs_of(n);
  const uint32_t nch = plan_nchunks(M);
  VR_TRY(set_lds_attr<LDS>(cfg.lds));
  k_boot_count<LDS><<<cfg.grid, ENG_THREADS, cfg.lds, st>>>(A.codes, A.gstart, A.chunk_g, nch,
                                                            E.masks, n, E.cntA);
  VR_CHECK_LAUNCH();
  k_scan_chunks<<<1, 1024, 0, st>>>(E.cntA, nch, E.baseA, E.totA);
  VR_CHECK_LAUNCH();
  if (lw == LANES) {
    k_boot_rankA<LDS, true><<<cfg.grid, ENG_THREADS, cfg.lds, st>>>(
        A.codes, A.gstart, A.chunk_g, A.gflag, nch, E.masks, n, E.baseA, E.posB_byA, E.TB, lw,
        E.partA);
    VR_CHECK_LAUNCH();
    k_boot_rankB<LDS, true><<<cfg.grid, ENG_THREADS, cfg.lds, st>>>(
        B.codes, B.gstart, B.chunk_g, B.gflag, nch, E.masks, n, E.TB, lw, E.partB, E.cntB);
    VR_CHECK_LAUNCH();
  } else {
    k_boot_rankA<LDS, false><<<cfg.grid, ENG_THREADS, cfg.lds, st>>>(
        A.codes, A.gstart, A.chunk_g, A.gflag, nch, E.masks, n, E.baseA, E.posB_byA, E.TB, lw,
        E.partA);
    VR_CHECK_LAUNCH();
    k_boot_rankB<LDS, false><<<cfg.grid, ENG_THREADS, cfg.lds, st>>>(
        B.codes, B.gstart, B.chunk_g, B.gflag, nch, E.masks, n, E.TB, lw, E.partB, E.cntB);
    VR_CHECK_LAUNCH();
  }
  k_scan_chunks<<<1, 1024, 0, st>>>(E.cntB, nch, E.baseB, E.totB);
  VR_CHECK_LAUNCH();
  k_boot_final<<<1, 1024, 0, st>>>(E.partA, nch, E.partB, E.cntB, E.baseB, nch, E.totB,
                                   A.hdr, B.hdr, nl, scores_out);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// Scores for `total` subsets (full set first if full_first), 64 per pass.
static int run_engine(const PlanView& A, const PlanView& B, int64_t n, const int32_t* idx,
                      int64_t k, int64_t n_sets, int full_first, double* scores,
                      const EngineWs& E, int lw, hipStream_t st) {
  const int64_t M = pairs_of(n);
  const int64_t total = n_sets + (full_first ? 1 : 0);
  if (total == 0) return VR_OK;
  if (M > 0) {
    k_join<<<(unsigned)((M + 255) / 256), 256, 0, st>>>(A.codes, M, n, B.pos_of_pair,
                                                       E.posB_byA);
    VR_CHECK_LAUNCH();
  }
  const EngineCfg cfg = engine_cfg(n);
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
    if (M == 0) {
      // no pairs: every score is NaN (scipy on empty input)
      std::vector<double> nan((size_t)nl, std::nan(""));
      VR_CHECK_HIP(hipMemcpyAsync(scores + set0, nan.data(), nan.size() * sizeof(double),
                                  hipMemcpyHostToDevice, st));
      VR_CHECK_HIP(hipStreamSynchronize(st));
      continue;
    }
    if (cfg.use_lds)
      VR_TRY(run_pass<true>(A, B, n, E, lw, nl, scores + set0, cfg, st));
    else
      VR_TRY(run_pass<false>(A, B, n, E, lw, nl, scores + set0, cfg, st));
  }
  return VR_OK;
}

// ---------------------------------------------------------------------------------
// Pearson of the two triangles (fp64, two pass, deterministic fixed-order reductions)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pearson_rows(const float* __restrict__ A,
                                                      const float* __restrict__ B, int64_t n,
                                                      int64_t ld, const double* __restrict__ mu,
                                                      double* __restrict__ part) {
  __shared__ double red[5][4];
  const int64_t a = blockIdx.x;
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0;
  const double ma = mu ? mu[0] : 0.0, mb = mu ? mu[1] : 0.0;
  for (int64_t b = a + 1 + threadIdx.x; b < n; b += 256) {
    const double x = (double)A[a * ld + b], y = (double)B[a * ld + b];
    if (!mu) {
      s0 += x;
      s1 += y;
    } else {
      const double dx = x - ma, dy = y - mb;
      s2 += dx * dy;
      s3 += dx * dx;
      s4 += dy * dy;
    }
  }
  double v[5] = {s0, s1, s2, s3, s4};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    double t = v[q];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o, 64);
    if (lane == 0) red[q][w] = t;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    const int q = threadIdx.x;
    part[a * 5 + q] = red[q][0] + red[q][1] + red[q][2] + red[q][3];
  }
}

__global__ __launch_bounds__(256) void k_pearson_reduce(const double* __restrict__ part,
                                                        int64_t n, double* __restrict__ mu,
                                                        double* __restrict__ out, int stage,
                                                        double M) {
  __shared__ double red[5][4];
  double v[5] = {0, 0, 0, 0, 0};
  for (int64_t a = threadIdx.x; a < n; a += 256)
    for (int q = 0; q < 5; ++q) v[q] += part[a * 5 + q];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    double t = v[q];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o, 64);
    if (lane == 0) red[q][w] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s[5];
    for (int q = 0; q < 5; ++q) s[q] = red[q][0] + red[q][1] + red[q][2] + red[q][3];
    if (stage == 0) {
      mu[0] = s[0] / M;
      mu[1] = s[1] / M;
    } else {
      double r;
      if (M < 2 || !(s[3] > 0) || !(s[4] > 0)) {
        r = (s[3] != s[3] || s[4] != s[4] || s[2] != s[2]) ? __builtin_nan("") : __builtin_nan("");
      } else {
        r = s[2] / sqrt(s[3] * s[4]);
        r = r > 1.0 ? 1.0 : (r < -1.0 ? -1.0 : r);
      }
      out[0] = r;
    }
  }
}

}  // namespace vr

using namespace vr;

extern "C" {

size_t vr_rank_plan_bytes(int64_t n) { return plan_bytes(n < 0 ? 0 : n); }

size_t vr_rank_plan_workspace(int64_t n) {
  size_t b = 0;
  plan_build_layout(nullptr, n < 0 ? 0 : n, &b);
  return b;
}

int vr_rank_plan_build_f32(const float* rdm, int64_t n, int64_t ld, void* plan,
                           size_t plan_bytes_, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535 && ld >= n, "vr_rank_plan_build_f32: bad shape n=%lld ld=%lld",
             (long long)n, (long long)ld);
  VR_REQUIRE(plan != nullptr && plan_bytes_ >= plan_bytes(n),
             "vr_rank_plan_build_f32: plan buffer %zu < %zu", plan_bytes_, plan_bytes(n));
  VR_REQUIRE(rdm != nullptr || n <= 1, "vr_rank_plan_build_f32: null rdm");
  size_t need = 0;
  PlanBuildWs W = plan_build_layout(ws, n, &need);
  if (ws_bytes < need || (ws == nullptr && need > 0)) {
    set_error("vr_rank_plan_build_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  return build_plan(rdm, n, ld, plan_layout(plan, n), W, as_stream(stream));
}

size_t vr_bootstrap_workspace(int64_t n) {
  size_t b = 0;
  engine_layout(nullptr, n < 0 ? 0 : n, LANES, &b);
  return b;
}

int vr_bootstrap_spearman_plans(const void* planA, const void* planB, int64_t n,
                                const int32_t* idx, int64_t k, int64_t n_sets,
                                int full_first, double* scores, void* ws, size_t ws_bytes,
                                void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535, "vr_bootstrap_spearman_plans: n=%lld out of range", (long long)n);
  VR_REQUIRE(planA && planB && scores, "vr_bootstrap_spearman_plans: null pointer");
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "vr_bootstrap_spearman_plans: bad k=%lld sets=%lld",
             (long long)k, (long long)n_sets);
  VR_REQUIRE(idx != nullptr || n_sets == 0 || k == 0, "vr_bootstrap_spearman_plans: null idx");
  size_t need = 0;
  EngineWs E = engine_layout(ws, n, LANES, &need);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_bootstrap_spearman_plans: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView A = plan_layout(const_cast<void*>(planA), n);
  PlanView B = plan_layout(const_cast<void*>(planB), n);
  return run_engine(A, B, n, idx, k, n_sets, full_first, scores, E, LANES, as_stream(stream));
}

static size_t oneshot_bytes(int64_t n, int lw, void* base, PlanView* A, PlanView* B,
                            PlanBuildWs* W, EngineWs* E) {
  Carver c(base);
  const size_t pb = plan_bytes(n);
  char* pa = c.take<char>(pb);
  char* pbb = c.take<char>(pb);
  size_t wb = 0, eb = 0;
  plan_build_layout(nullptr, n, &wb);
  engine_layout(nullptr, n, lw, &eb);
  char* wsb = c.take<char>(std::max(wb, eb));  // plan-build scratch is dead once plans exist
  if (base) {
    *A = plan_layout(pa, n);
    *B = plan_layout(pbb, n);
    *W = plan_build_layout(wsb, n, nullptr);
    *E = engine_layout(wsb, n, lw, nullptr);
  }
  return c.bytes();
}

size_t vr_bootstrap_spearman_workspace(int64_t n) {
  return oneshot_bytes(n < 0 ? 0 : n, LANES, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int vr_bootstrap_spearman_f32(const float* A, const float* B, int64_t n, int64_t ld,
                              const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                              double* scores, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535 && ld >= n, "vr_bootstrap_spearman_f32: bad shape");
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "vr_bootstrap_spearman_f32: bad k");
  const size_t need = oneshot_bytes(n, LANES, nullptr, nullptr, nullptr, nullptr, nullptr);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_bootstrap_spearman_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView PA, PB;
  PlanBuildWs W;
  EngineWs E;
  oneshot_bytes(n, LANES, ws, &PA, &PB, &W, &E);
  hipStream_t st = as_stream(stream);
  VR_TRY(build_plan(A, n, ld, PA, W, st));
  VR_TRY(build_plan(B, n, ld, PB, W, st));
  return run_engine(PA, PB, n, idx, k, n_sets, full_first, scores, E, LANES, st);
}

size_t vr_spearman_triu_workspace(int64_t n) {
  return oneshot_bytes(n < 0 ? 0 : n, 1, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int vr_spearman_triu_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out,
                         void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535 && ld >= n, "vr_spearman_triu_f32: bad shape n=%lld ld=%lld",
             (long long)n, (long long)ld);
  VR_REQUIRE(out != nullptr, "vr_spearman_triu_f32: null out");
  const size_t need = oneshot_bytes(n, 1, nullptr, nullptr, nullptr, nullptr, nullptr);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_spearman_triu_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView PA, PB;
  PlanBuildWs W;
  EngineWs E;
  oneshot_bytes(n, 1, ws, &PA, &PB, &W, &E);
  hipStream_t st = as_stream(stream);
  VR_TRY(build_plan(A, n, ld, PA, W, st));
  VR_TRY(build_plan(B, n, ld, PB, W, st));
  return run_engine(PA, PB, n, nullptr, 0, 0, 1, out, E, 1, st);
}

size_t vr_pearson_triu_workspace(int64_t n) {
  Carver c(nullptr);
  c.take<double>((size_t)std::max<int64_t>(n, 1) * 5);
  c.take<double>(2);
  return c.bytes();
}

int vr_pearson_triu_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out,
                        void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && ld >= n && out != nullptr, "vr_pearson_triu_f32: bad arguments");
  const size_t need = vr_pearson_triu_workspace(n);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_pearson_triu_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int64_t M = pairs_of(n);
  if (M < 2) {
    const double nan = std::nan("");
    VR_CHECK_HIP(hipMemcpyAsync(out, &nan, sizeof(double), hipMemcpyHostToDevice, st));
    VR_CHECK_HIP(hipStreamSynchronize(st));
    return VR_OK;
  }
  Carver c(ws);
  double* part = c.take<double>((size_t)n * 5);
  double* mu = c.take<double>(2);
  k_pearson_rows<<<(unsigned)n, 256, 0, st>>>(A, B, n, ld, nullptr, part);
  VR_CHECK_LAUNCH();
  k_pearson_reduce<<<1, 256, 0, st>>>(part, n, mu, out, 0, (double)M);
  VR_CHECK_LAUNCH();
  k_pearson_rows<<<(unsigned)n, 256, 0, st>>>(A, B, n, ld, mu, part);
  VR_CHECK_LAUNCH();
  k_pearson_reduce<<<1, 256, 0, st>>>(part, n, mu, out, 1, (double)M);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // extern "C"
