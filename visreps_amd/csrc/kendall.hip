// Kendall tau-a comparison of two RDMs and its bootstrap, the MI355X replacement of
//   compute_rdm_correlation(A, B, correlation="Kendall")  -> _kendall_tau_a(triu(A), triu(B))
// visreps/analysis/rsa.py:22-40,96-129 (scipy.stats.kendalltau tau-b, converted to tau-a)
// and of the bootstrap loop evals.py:355-373 / rsa.py:233-261 with compare_method=kendall.
//
// scipy's tau-b (scipy/stats/_stats_py.py kendalltau) from exact integers, per subset:
//   tot = M'(M'-1)/2 over the M' included pairs (elements of the triangle vectors),
//   xtie / ytie / ntie = sum over tie groups of x / of y / of (x, y) jointly of C(k, 2),
//   dis = discordant pairs = inversions of y's dense rank in (x, y)-lexicographic order,
//   tau_b = (tot - xtie - ytie + ntie - 2 dis) / sqrt(tot - xtie) / sqrt(tot - ytie),
// then the reference's conversion tau_a = tau_b sqrt((tot - xtie)(tot - ytie)) / tot,
// each in the same fp64 operation order, so the value matches scipy + rsa.py exactly.
//
// Inversions are counted bit by bit of the y rank (an MSD binary radix split): at level b
// the stream is the (x, y)-lexicographic order stably sorted by y >> (b+1); an inverted
// pair has its highest differing y bit at exactly one level, where it is a (1 before 0)
// pair inside one bucket of equal y >> (b+1). Each level is one stream of pair codes plus
// two bit planes (bit b of y, bucket starts), built once per (A, B) unit by a stable split
// of the previous level (k_level_split) and walked once per pass of 64 subsets with the
// engine's window machinery (window.h) and the bit-parallel counters of kcount.h. Tie sums
// are the same segmented count over the multi-element tie groups of the x-lex order (x and
// joint ties) and of B's order (y ties). All counts are exact integers, so scores do not
// depend on launch geometry or pass grouping.
//
// Memory: one level is resident at a time (streams are walked level by level, every pass
// against it); per unit ~14 x M x 4 B of scratch.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "kcount.h"
#include "window.h"

namespace vr {

constexpr int KW_THREADS = 1024;
constexpr int KW_WAVES = KW_THREADS / 64;
constexpr int KFIX_GROUPS = KW_THREADS / 64;
// the per-wave partials a walk composes into its block summary; they live in the walk's
// dynamic LDS, over the masks once the walk is done (kw_parts), so at n = 10k two 16-wave
// blocks fit a CU (80 KB of masks each) instead of one
constexpr size_t KW_STATIC_LDS = (size_t)KW_WAVES * 64 * (8 + 8 + 4 + 4 + 4);

enum KField { KF_DIS = 0, KF_XTIE, KF_NTIE, KF_YTIE, KF_INCL, KF_N };

struct KCfg {
  int grid;
  int nwaves;
  size_t lds;
  bool use_lds;
};

#ifndef VR_KW_MINB
#define VR_KW_MINB 2  // walk blocks per CU the walks are compiled for (launch bounds)
#endif
static KCfg kendall_cfg(int64_t n) {
  KCfg c;
  const size_t need = (size_t)n * sizeof(uint64_t);
  const size_t cap = 160 * 1024 - 1024;
  const char* e = getenv("VISREPS_KENDALL_MASKS");  // "global": masks from L2 (A/B timing)
  c.use_lds = need <= cap && !(e && strcmp(e, "global") == 0);
  const size_t per_block = std::max(c.use_lds ? need : (size_t)0, KW_STATIC_LDS);
  const int per_cu = std::max<int>(1, std::min<int>(VR_KW_MINB, (int)(cap / per_block)));
  c.grid = num_cus() * per_cu;
  c.nwaves = c.grid * KW_WAVES;
  c.lds = per_block;  // masks (LDS) and, after the walk, the partials
  return c;
}

__host__ __device__ inline int64_t kwindows(int64_t M) { return (M + 63) / 64; }
// two u32 words per window; the plane kernels run whole 256-thread blocks (4 windows)
static inline int64_t kflag_words(int64_t M) { return 2 * ((kwindows(M) + 3) / 4 * 4) + 2; }

struct KendallWs {
  uint64_t* masks;   // [npass][n]
  uint32_t* gidxA;   // [M] dense tie-group index of each A position
  uint32_t* gidxB;   // [M] ... of each B position
  uint32_t* wcnt;    // [(M+31)/32 + 1]
  uint32_t* keys;    // [M]
  uint32_t* vals;    // [M]
  uint32_t* keys_alt;
  uint32_t* vals_alt;
  uint32_t* radix;
  uint32_t* scan;
  uint32_t* ecode[2];  // level streams: pair code and y (dense B rank), ping-pong
  uint32_t* ey[2];
  uint32_t* lv_start[2];  // [FW] bucket starts of a level (double-buffered: level b walked while
  uint32_t* lv_bits[2];   //      level b-1 is prepared); bit b of y
  uint32_t* xa_start;  // [FW] x-lex order: starts / members of multi-element A groups
  uint32_t* xa_mem;
  uint32_t* xj_start;  //               ... of multi-element joint (A, B) groups
  uint32_t* xj_mem;
  uint32_t* yb_start;  // B order: starts / members of multi-element B groups
  uint32_t* yb_mem;
  uint64_t* w_acc;     // [pass][grid][64] per-block summaries (KSum s, g, a, b) and included counts
  uint64_t* w_g;
  uint64_t* w_a;
  uint32_t* w_b;
  uint32_t* w_incl;
  uint64_t* w2_acc;    // the same for the B tie stream, walked on the side stream beside the
  uint64_t* w2_g;      // x-lex preparation and tie walks
  uint64_t* w2_a;
  uint32_t* w2_b;
  uint32_t* w2_incl;
  uint64_t* w3[3];     // two more sets for the fused top-level walk's tie streams: acc, g, a
  uint32_t* w3bi[2];   // b, incl
  uint64_t* w4[3];
  uint32_t* w4bi[2];
  uint64_t* tot;       // [KF_N][cap]
};

static KendallWs kendall_layout(void* base, int64_t n, int64_t cap_sets, int nwaves, size_t* bytes) {
  const int64_t M = pairs_of(n);
  const int64_t FW = kflag_words(M);
  const int64_t npass = (cap_sets + LANES - 1) / LANES;
  Carver c(base);
  KendallWs w;
  w.masks = c.take<uint64_t>((size_t)std::max<int64_t>(npass, 1) * (size_t)n);
  w.gidxA = c.take<uint32_t>((size_t)M);
  w.gidxB = c.take<uint32_t>((size_t)M);
  w.wcnt = c.take<uint32_t>((size_t)(M + 31) / 32 + 1);
  w.keys = c.take<uint32_t>((size_t)M);
  w.vals = c.take<uint32_t>((size_t)M);
  w.keys_alt = c.take<uint32_t>((size_t)M);
  w.vals_alt = c.take<uint32_t>((size_t)M);
  w.radix = c.take<uint32_t>(radix_ws_elems(M));
  w.scan = c.take<uint32_t>(scan_ws_elems(M));
  for (int i = 0; i < 2; ++i) {
    w.ecode[i] = c.take<uint32_t>((size_t)M);
    w.ey[i] = c.take<uint32_t>((size_t)M);
  }
  uint32_t** fl[] = {&w.lv_start[0], &w.lv_bits[0], &w.lv_start[1], &w.lv_bits[1], &w.xa_start, &w.xa_mem, &w.xj_start, &w.xj_mem,
                     &w.yb_start, &w.yb_mem};
  for (uint32_t** f : fl) *f = c.take<uint32_t>((size_t)FW);
  // block summaries of every pass of one stream: [pass][block][lane] (grid = nwaves / 16)
  const size_t wsum = (size_t)std::max<int64_t>(nwaves, std::max<int64_t>(npass, 1) * (nwaves / KW_WAVES)) * LANES;
  w.w_acc = c.take<uint64_t>(wsum);
  w.w_g = c.take<uint64_t>(wsum);
  w.w_a = c.take<uint64_t>(wsum);
  w.w_b = c.take<uint32_t>(wsum);
  w.w_incl = c.take<uint32_t>(wsum);
  w.w2_acc = c.take<uint64_t>(wsum);
  w.w2_g = c.take<uint64_t>(wsum);
  w.w2_a = c.take<uint64_t>(wsum);
  w.w2_b = c.take<uint32_t>(wsum);
  w.w2_incl = c.take<uint32_t>(wsum);
  for (int i = 0; i < 3; ++i) w.w3[i] = c.take<uint64_t>(wsum), w.w4[i] = c.take<uint64_t>(wsum);
  for (int i = 0; i < 2; ++i) w.w3bi[i] = c.take<uint32_t>(wsum), w.w4bi[i] = c.take<uint32_t>(wsum);
  w.tot = c.take<uint64_t>((size_t)KF_N * (size_t)std::max<int64_t>(cap_sets, 1));
  if (bytes) *bytes = c.bytes();
  return w;
}

// ---------------------------------------------------------------------------------
// per-unit precompute
// ---------------------------------------------------------------------------------
__global__ void k_word_popc(const uint32_t* __restrict__ gflag, int64_t words,
                            uint32_t* __restrict__ out) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < words) out[w] = (uint32_t)__popc(gflag[w]);
}

// gidx[p] = dense index of the tie group holding sorted position p
__global__ void k_group_index(const uint32_t* __restrict__ gflag, const uint32_t* __restrict__ wpre,
                              int64_t M, uint32_t* __restrict__ gidx) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= M) return;
  const uint32_t w = gflag[p >> 5];
  gidx[p] = wpre[p >> 5] + (uint32_t)__popc(w & (0xFFFFFFFFu >> (31 - (p & 31)))) - 1u;
}

// B position i -> (key = A group of its pair, value = i); sorting stably by key from B
// order gives the (x, y)-lexicographic order of scipy's kendalltau
__global__ void k_kendall_keys(const uint32_t* __restrict__ codesB, int64_t M, int64_t n,
                               const uint32_t* __restrict__ posMapA,
                               const uint32_t* __restrict__ gidxA, uint32_t* __restrict__ keys,
                               uint32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t cb = codesB[i];
  keys[i] = gidxA[posMapA[tri_index(cb >> 16, cb & 0xffffu, (uint64_t)n)]];
  vals[i] = (uint32_t)i;
}

__global__ void k_kendall_elems(const uint32_t* __restrict__ vals, const uint32_t* __restrict__ codesB,
                                const uint32_t* __restrict__ gidxB, int64_t M,
                                uint32_t* __restrict__ ecode, uint32_t* __restrict__ ey) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= M) return;
  const uint32_t i = vals[p];
  ecode[p] = codesB[i];
  ey[p] = gidxB[i];
}

// 64 positions per wave -> two u32 words of each bit plane
__device__ inline void put_plane(uint32_t* plane, int64_t p, bool bit) {
  const uint64_t b = __ballot(bit);
  if ((threadIdx.x & 63) == 0) {
    plane[(p >> 6) * 2] = (uint32_t)b;
    plane[(p >> 6) * 2 + 1] = (uint32_t)(b >> 32);
  }
}

// x-lex order tie planes: starts and members of multi-element A groups and of
// multi-element joint (A, B) groups
__global__ void k_xlex_flags(const uint32_t* __restrict__ gA, const uint32_t* __restrict__ ey,
                             int64_t M, uint32_t* __restrict__ xa_start, uint32_t* __restrict__ xa_mem,
                             uint32_t* __restrict__ xj_start, uint32_t* __restrict__ xj_mem) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool v = p < M;
  bool nsA = false, memA = false, nsJ = false, memJ = false;
  if (v) {
    const uint32_t a = gA[p], y = ey[p];
    const bool sA = p == 0 || gA[p - 1] != a;
    const bool sJ = sA || ey[p - 1] != y;
    const bool last = p + 1 >= M;
    const bool sA1 = last || gA[p + 1] != a;
    const bool sJ1 = sA1 || ey[p + 1] != y;
    nsA = sA && !sA1;
    memA = !(sA && sA1);
    nsJ = sJ && !sJ1;
    memJ = !(sJ && sJ1);
  }
  put_plane(xa_start, p, nsA);
  put_plane(xa_mem, p, memA);
  put_plane(xj_start, p, nsJ);
  put_plane(xj_mem, p, memJ);
}

// B order tie planes from the plan's group-start bitmask
__global__ void k_border_flags(const uint32_t* __restrict__ gflag, int64_t M,
                               uint32_t* __restrict__ yb_start, uint32_t* __restrict__ yb_mem) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool v = p < M;
  bool ns = false, mem = false;
  if (v) {
    const bool s = (gflag[p >> 5] >> (p & 31)) & 1u;
    const int64_t q = p + 1;
    const bool s1 = q >= M || ((gflag[q >> 5] >> (q & 31)) & 1u);
    ns = s && !s1;
    mem = !(s && s1);
  }
  put_plane(yb_start, p, ns);
  put_plane(yb_mem, p, mem);
}

// level b planes of the current stream (sorted by y >> (b+1)): bit b of y, bucket starts
__global__ void k_level_flags(const uint32_t* __restrict__ ey, int64_t M, int b,
                              uint32_t* __restrict__ lv_start, uint32_t* __restrict__ lv_bits) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool v = p < M;
  bool st = false, bit = false;
  if (v) {
    const uint32_t y = ey[p];
    bit = (y >> b) & 1u;
    st = p == 0 || (ey[p - 1] >> (b + 1)) != (y >> (b + 1));
  }
  put_plane(lv_start, p, st);
  put_plane(lv_bits, p, bit);
}

// stable split of every bucket by bit b: the stream for level b-1 (sorted by y >> b).
// gstartB[g] = number of elements with y < g, so the bucket of y >> (b+1) starts at
// gstartB[(y >> (b+1)) << (b+1)] and its one-half at gstartB[(y >> b) << b]. Zeros before a
// position come from the level's bit plane: q - (ones in whole words before q, wpre = the
// exclusive scan of the plane's word popcounts) - (ones below q in its word).
__device__ inline uint32_t zeros_before(const uint32_t* __restrict__ bits, const uint32_t* __restrict__ wpre,
                                        uint32_t q) {
  return q - wpre[q >> 5] - (uint32_t)__popc(bits[q >> 5] & ((1u << (q & 31u)) - 1u));
}
__global__ void k_level_split(const uint32_t* __restrict__ ecode, const uint32_t* __restrict__ ey,
                              const uint32_t* __restrict__ bits, const uint32_t* __restrict__ wpre,
                              const uint32_t* __restrict__ gstartB, int64_t M, int b,
                              uint32_t* __restrict__ ecode_out, uint32_t* __restrict__ ey_out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= M) return;
  const uint32_t y = ey[p];
  const uint32_t bs = gstartB[(y >> (b + 1)) << (b + 1)];
  const uint32_t zb = zeros_before(bits, wpre, bs), zp = zeros_before(bits, wpre, (uint32_t)p);
  uint32_t np;
  if ((y >> b) & 1u)
    np = gstartB[(y >> b) << b] + ((uint32_t)p - bs) - (zp - zb);
  else
    np = bs + (zp - zb);
  ecode_out[np] = ecode[p];
  ey_out[np] = y;
}

// ---------------------------------------------------------------------------------
// per-pass stream walk
// ---------------------------------------------------------------------------------
// TIE: o = z = included members (aux plane) of multi-element groups, S = their starts;
// else (inversions): o / z = included positions with bit b of y set / clear (aux plane),
// S = bucket starts.
// A range summary as an affine map of the carry C into it (the ones of the segment open at
// its start): contribution s + g C, carry out a + b C (b in {0, 1}). A wave range is
// (acc, zlead, c, !seen); ranges compose left to right.
struct KSum {
  uint64_t s, g, a;
  uint32_t b;
};
__device__ inline KSum ksum_identity() { return {0ull, 0ull, 0ull, 1u}; }
// S then R: R's carry in is S's carry out a_S + b_S C
__device__ inline void ksum_push(KSum& S, uint64_t s, uint64_t g, uint64_t a, uint32_t b) {
  S.s += s + g * S.a;
  S.g += S.b ? g : 0ull;
  S.a = a + (b ? S.a : 0ull);
  S.b = S.b & b;
}

// where a walk writes its block summaries (per pass: [block][lane])
struct KOut {
  uint64_t *acc, *g, *a;
  uint32_t *b, *incl;
};
// the partials' arrays in the dynamic LDS (over the masks: kw_block_summary's first barrier
// orders them after every wave's last mask read)
struct KParts {
  uint64_t *acc, *zl;
  uint32_t *c, *inc, *seen;
};
__device__ inline KParts kw_parts(uint64_t* smem) {
  KParts p;
  p.acc = smem;
  p.zl = smem + KW_WAVES * LANES;
  uint32_t* u = reinterpret_cast<uint32_t*>(smem + 2 * KW_WAVES * LANES);
  p.c = u;
  p.inc = u + KW_WAVES * LANES;
  p.seen = u + 2 * KW_WAVES * LANES;
  return p;
}

__device__ inline void kw_block_summary(const KSeg& a, bool seen, uint32_t incl, const KOut& o, uint64_t* s_acc,
                                        uint64_t* s_zl, uint32_t* s_c, uint32_t* s_inc, uint32_t* s_seen) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();  // the arrays' previous use is done
  s_acc[wv * LANES + lane] = a.acc;
  s_zl[wv * LANES + lane] = a.zlead;
  s_c[wv * LANES + lane] = a.c;
  s_seen[wv * LANES + lane] = seen ? 1u : 0u;
  s_inc[wv * LANES + lane] = incl;
  __syncthreads();
  if (wv == 0) {
    KSum S = ksum_identity();
    uint32_t inc = 0;
    for (int w = 0; w < KW_WAVES; ++w) {
      ksum_push(S, s_acc[w * LANES + lane], s_zl[w * LANES + lane], s_c[w * LANES + lane],
                s_seen[w * LANES + lane] == 0u);
      inc += s_inc[w * LANES + lane];
    }
    const size_t off = (size_t)blockIdx.x * LANES + lane;
    o.acc[off] = S.s;
    o.g[off] = S.g;
    o.a[off] = S.a;
    o.b[off] = S.b;
    o.incl[off] = inc;
  }
}

template <bool LDS, bool TIE>
__global__ __launch_bounds__(KW_THREADS, VR_KW_MINB) void k_kwalk(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ sflag,
    const uint32_t* __restrict__ aux, int64_t M, const uint64_t* __restrict__ gmask, int64_t n,
    int nl, uint32_t nwaves, uint64_t* __restrict__ w_acc, uint64_t* __restrict__ w_g,
    uint64_t* __restrict__ w_a, uint32_t* __restrict__ w_b, uint32_t* __restrict__ w_incl) {
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const int lane = threadIdx.x & 63;
  const bool active = lane < nl;
  const uint32_t wave = wave_uniform(blockIdx.x * KW_WAVES + (threadIdx.x >> 6));
  const uint64_t nwin = (uint64_t)kwindows(M);
  const uint32_t wb = (uint32_t)(nwin * wave / nwaves), we = (uint32_t)(nwin * (wave + 1) / nwaves);
  KSeg a{0ull, 0u, 0u};
  bool seen = false;
  uint32_t incl = 0;
#ifndef VR_KW_PAIR
#define VR_KW_PAIR 1  // 1: two windows per trip (mask lookups, transposes and pair counts of both
                      // first, straight-line, so their dependency chains interleave)
#endif
  auto code_at = [&](uint32_t win) -> uint32_t {
    const uint32_t q = win * 64u + (uint32_t)lane;
    return q < (uint64_t)M ? codes[q] : 0u;
  };
  auto bits_of = [&](uint32_t cd, uint32_t win) -> uint64_t {
    const uint32_t pos = win * 64u + (uint32_t)lane;
    const uint64_t mb = pos < (uint64_t)M ? (m[cd >> 16] & m[cd & 0xffffu]) : 0ull;
    const uint64_t x = transpose64<VR_XPOSE_K>(mb, lane);
    return active ? x : 0ull;
  };
  auto plane = [&](const uint32_t* f, uint32_t win) -> uint64_t {
    return ((uint64_t)sload(f + 2 * win + 1) << 32) | sload(f + 2 * win);
  };
  if (VR_KW_PAIR) {
    uint32_t c0 = 0, c1 = 0;
    if (wb < we) c0 = code_at(wb);
    if (wb + 1 < we) c1 = code_at(wb + 1);
    for (uint32_t win = wb; win < we; win += 2) {
      const bool two = win + 1 < we;  // wave-uniform
      const uint32_t d0 = c0, d1 = c1;
      if (win + 2 < we) c0 = code_at(win + 2);  // the next pair's codes, one trip ahead
      if (win + 3 < we) c1 = code_at(win + 3);
      const uint64_t x0 = bits_of(d0, win);
      const uint64_t x1 = two ? bits_of(d1, win + 1) : 0ull;
      const uint64_t S0 = plane(sflag, win), X0 = plane(aux, win);
      const uint64_t S1 = plane(sflag, win + 1), X1 = plane(aux, win + 1);  // in the padded planes
      const uint64_t o0 = x0 & X0, z0 = TIE ? o0 : (x0 & ~X0);
      const uint64_t o1 = x1 & X1, z1 = TIE ? o1 : (x1 & ~X1);
      const uint64_t i0 = kseg_inner<TIE>(o0, z0), i1 = kseg_inner<TIE>(o1, z1);
      incl += popc64(x0) + popc64(x1);
      kseg_window_inner<TIE>(o0, z0, S0, i0, a, seen);
      if (two) kseg_window_inner<TIE>(o1, z1, S1, i1, a, seen);
    }
  } else {
    uint32_t cd = 0;
    if (wb < we) cd = code_at(wb);
    for (uint32_t win = wb; win < we; ++win) {
      const uint32_t d = cd;
      if (win + 1 < we) cd = code_at(win + 1);  // next window's code, one ahead
      const uint64_t x = bits_of(d, win);
      const uint64_t S = plane(sflag, win), X = plane(aux, win);
      incl += popc64(x);
      if (TIE) {
        const uint64_t o = x & X;
        kseg_window<true>(o, o, S, a, seen);
      } else {
        kseg_window<false>(x & X, x & ~X, S, a, seen);
      }
    }
  }
  // The block's 16 wave ranges are consecutive: compose them here (affine carry maps, see
  // k_kfix) and write one summary per block, so the fix-up reads grid x 64 entries instead
  // of nwaves x 64 (16x less: the single-block fix-up was bound by reading them).
  const KParts pt = kw_parts(smask);
  kw_block_summary(a, seen, incl, KOut{w_acc, w_g, w_a, w_b, w_incl}, pt.acc, pt.zl, pt.c, pt.inc, pt.seen);
}

// The top inversion level fused with the two x-lex tie streams (A ties, joint ties): the same
// pair codes (the x-lex order), so one walk shares the code loads, mask lookups and
// transposes; three segment states, three block summaries (one k_kfix each).
template <bool LDS>
__global__ __launch_bounds__(KW_THREADS, VR_KW_MINB) void k_kwalk_top3(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ s0, const uint32_t* __restrict__ x0p,
    const uint32_t* __restrict__ s1, const uint32_t* __restrict__ x1p, const uint32_t* __restrict__ s2,
    const uint32_t* __restrict__ x2p, int64_t M, const uint64_t* __restrict__ gmask, int64_t n, int nl,
    uint32_t nwaves, KOut o0, KOut o1, KOut o2) {
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const int lane = threadIdx.x & 63;
  const bool active = lane < nl;
  const uint32_t wave = wave_uniform(blockIdx.x * KW_WAVES + (threadIdx.x >> 6));
  const uint64_t nwin = (uint64_t)kwindows(M);
  const uint32_t wb = (uint32_t)(nwin * wave / nwaves), we = (uint32_t)(nwin * (wave + 1) / nwaves);
  KSeg a0{0ull, 0u, 0u}, a1{0ull, 0u, 0u}, a2{0ull, 0u, 0u};
  bool seen0 = false, seen1 = false, seen2 = false;
  uint32_t incl = 0;
  auto code_at = [&](uint32_t win) -> uint32_t {
    const uint32_t q = win * 64u + (uint32_t)lane;
    return q < (uint64_t)M ? codes[q] : 0u;
  };
  auto bits_of = [&](uint32_t cd, uint32_t win) -> uint64_t {
    const uint32_t pos = win * 64u + (uint32_t)lane;
    const uint64_t mb = pos < (uint64_t)M ? (m[cd >> 16] & m[cd & 0xffffu]) : 0ull;
    const uint64_t x = transpose64<VR_XPOSE_K>(mb, lane);
    return active ? x : 0ull;
  };
  auto plane = [&](const uint32_t* f, uint32_t win) -> uint64_t {
    return ((uint64_t)sload(f + 2 * win + 1) << 32) | sload(f + 2 * win);
  };
  uint32_t cd = 0;
  if (wb < we) cd = code_at(wb);
  for (uint32_t win = wb; win < we; ++win) {
    const uint32_t d = cd;
    if (win + 1 < we) cd = code_at(win + 1);  // next window's code, one ahead
    const uint64_t x = bits_of(d, win);
    incl += popc64(x);
    {  // the level: ones = bit set, zeros = bit clear
      const uint64_t X = plane(x0p, win);
      kseg_window<false>(x & X, x & ~X, plane(s0, win), a0, seen0);
    }
    {  // the tie streams: included members of multi-element groups
      const uint64_t t1 = x & plane(x1p, win);
      kseg_window<true>(t1, t1, plane(s1, win), a1, seen1);
      const uint64_t t2 = x & plane(x2p, win);
      kseg_window<true>(t2, t2, plane(s2, win), a2, seen2);
    }
  }
  const KParts pt = kw_parts(smask);
  kw_block_summary(a0, seen0, incl, o0, pt.acc, pt.zl, pt.c, pt.inc, pt.seen);
  kw_block_summary(a1, seen1, incl, o1, pt.acc, pt.zl, pt.c, pt.inc, pt.seen);
  kw_block_summary(a2, seen2, incl, o2, pt.acc, pt.zl, pt.c, pt.inc, pt.seen);
}

// Stream total per lane: the block summaries (k_kwalk) composed in block order with carry 0
// into the first, added into tot[field][set0 + lane]; optionally the included-pair count into
// tot[KF_INCL]. One block per pass (set0 = 64 x pass), all passes of a stream in one launch;
// 16 groups compose contiguous block ranges, group 0 composes the groups.
__global__ __launch_bounds__(KW_THREADS) void k_kfix(
    const uint64_t* __restrict__ w_acc, const uint64_t* __restrict__ w_g,
    const uint64_t* __restrict__ w_a, const uint32_t* __restrict__ w_b,
    const uint32_t* __restrict__ w_incl, uint32_t nblk, int64_t total, int field, int add_incl,
    uint64_t* __restrict__ tot, int64_t cap) {
  const int64_t set0 = (int64_t)blockIdx.x * LANES;
  const int nl = (int)(total - set0 < LANES ? total - set0 : LANES);
  const size_t pbase = (size_t)blockIdx.x * nblk * LANES;
  w_acc += pbase, w_g += pbase, w_a += pbase, w_b += pbase, w_incl += pbase;
  __shared__ uint64_t s_s[KFIX_GROUPS][LANES], s_g[KFIX_GROUPS][LANES], s_a[KFIX_GROUPS][LANES],
      s_inc[KFIX_GROUPS][LANES];
  __shared__ uint32_t s_b[KFIX_GROUPS][LANES];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const uint32_t per = (nblk + KFIX_GROUPS - 1) / KFIX_GROUPS;
  const uint32_t b0 = grp * per, b1 = min(nblk, b0 + per);
  KSum S = ksum_identity();
  uint64_t inc = 0;
  for (uint32_t b = b0; b < b1; ++b) {
    const size_t o = (size_t)b * LANES + lane;
    ksum_push(S, w_acc[o], w_g[o], w_a[o], w_b[o]);
    inc += w_incl[o];
  }
  s_s[grp][lane] = S.s;
  s_g[grp][lane] = S.g;
  s_a[grp][lane] = S.a;
  s_b[grp][lane] = S.b;
  s_inc[grp][lane] = inc;
  __syncthreads();
  if (grp != 0) return;
  KSum T = ksum_identity();
  uint64_t incl = 0;
  for (int g = 0; g < KFIX_GROUPS; ++g) {
    ksum_push(T, s_s[g][lane], s_g[g][lane], s_a[g][lane], s_b[g][lane]);
    incl += s_inc[g][lane];
  }
  if (lane < nl) {
    tot[(size_t)field * cap + set0 + lane] += T.s;  // carry 0 into the stream
    if (add_incl) tot[(size_t)KF_INCL * cap + set0 + lane] = incl;
  }
}

// tau-a per subset from the exact counts, in scipy's / rsa.py's fp64 operation order
__global__ void k_kfinal(const uint64_t* __restrict__ tot, int64_t cap, int64_t total_sets,
                         double* __restrict__ scores) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= total_sets) return;
  const uint64_t Mp = tot[(size_t)KF_INCL * cap + s];
  const uint64_t dis = tot[(size_t)KF_DIS * cap + s];
  const uint64_t xt = tot[(size_t)KF_XTIE * cap + s];
  const uint64_t nt = tot[(size_t)KF_NTIE * cap + s];
  const uint64_t yt = tot[(size_t)KF_YTIE * cap + s];
  double r = __builtin_nan("");
  if (Mp >= 2) {
    const uint64_t t = Mp * (Mp - 1) / 2;
    if (xt != t && yt != t) {
      const int64_t cmd = (int64_t)(t - xt - yt + nt) - 2 * (int64_t)dis;
      double taub = (double)cmd / sqrt((double)(t - xt)) / sqrt((double)(t - yt));
      taub = fmin(1.0, fmax(-1.0, taub));
      const double denom = sqrt((double)(t - xt) * (double)(t - yt));
      r = denom == 0.0 ? __builtin_nan("") : taub * denom / (double)t;
    }
  }
  scores[s] = r;
}

__global__ void k_kfill_nan(double* out, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = __builtin_nan("");
}

// ---------------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------------
static unsigned blocks_for(int64_t count, int bs) { return (unsigned)((count + bs - 1) / bs); }

template <bool LDS>
static int set_kwalk_attr() {
  if (!LDS) return VR_OK;
  VR_ONCE({
    const int mx = 160 * 1024 - 1024;
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_kwalk<LDS, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_kwalk<LDS, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    VR_CHECK_HIP(hipFuncSetAttribute((const void*)k_kwalk_top3<LDS>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, mx));
  });
  return VR_OK;
}

// one stream against every pass, totals into tot[field]
static int walk_stream(bool tie, const uint32_t* codes, const uint32_t* sflag, const uint32_t* aux,
                       int64_t M, const KendallWs& W, int64_t n, int64_t total, int field,
                       bool add_incl, int64_t cap, const KCfg& cfg, hipStream_t st) {
  if (cfg.use_lds) VR_TRY(set_kwalk_attr<true>());
  auto walk = [&](const uint64_t* mk, int nl, size_t o) {
    const size_t lds = cfg.lds;  // the masks (LDS form) and the block-summary partials
    auto* k = cfg.use_lds ? (tie ? k_kwalk<true, true> : k_kwalk<true, false>)
                          : (tie ? k_kwalk<false, true> : k_kwalk<false, false>);
    k<<<cfg.grid, KW_THREADS, lds, st>>>(codes, sflag, aux, M, mk, n, nl, (uint32_t)cfg.nwaves, W.w_acc + o,
                                         W.w_g + o, W.w_a + o, W.w_b + o, W.w_incl + o);
  };
  int64_t npass = 0;
  for (int64_t set0 = 0; set0 < total; set0 += LANES, ++npass) {
    const int nl = (int)std::min<int64_t>(LANES, total - set0);
    KtScope kt(KT_KWALK, (double)M, st);  // the walk only, not the fix-up
    walk(W.masks + (size_t)npass * (size_t)n, nl, (size_t)npass * (size_t)cfg.grid * LANES);
    VR_CHECK_LAUNCH();
  }
  k_kfix<<<(unsigned)npass, KW_THREADS, 0, st>>>(W.w_acc, W.w_g, W.w_a, W.w_b, W.w_incl, (uint32_t)cfg.grid,
                                                 total, field, add_incl ? 1 : 0, W.tot, cap);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// the fused top level + x-lex tie streams against every pass: totals into tot[KF_DIS] (with the
// included-pair count), tot[fa] (A ties) and tot[KF_NTIE]
static int walk_top3(const uint32_t* codes, const uint32_t* lvs, const uint32_t* lvb, const KendallWs& W,
                     int64_t M, int64_t n, int64_t total, int fa, int64_t cap, const KCfg& cfg, hipStream_t st) {
  if (cfg.use_lds) VR_TRY(set_kwalk_attr<true>());
  const KOut o0{W.w_acc, W.w_g, W.w_a, W.w_b, W.w_incl};
  const KOut o1{W.w3[0], W.w3[1], W.w3[2], W.w3bi[0], W.w3bi[1]};
  const KOut o2{W.w4[0], W.w4[1], W.w4[2], W.w4bi[0], W.w4bi[1]};
  auto shift = [&](KOut o, size_t d) { return KOut{o.acc + d, o.g + d, o.a + d, o.b + d, o.incl + d}; };
  int64_t npass = 0;
  for (int64_t set0 = 0; set0 < total; set0 += LANES, ++npass) {
    const int nl = (int)std::min<int64_t>(LANES, total - set0);
    const size_t d = (size_t)npass * (size_t)cfg.grid * LANES;
    // bytes: the pair code + six bit planes, in the 4.25-B-per-walk units of k_kwalk
    KtScope kt(KT_KWALK, (double)M * (4.75 / 4.25), st);
    const uint64_t* mk = W.masks + (size_t)npass * (size_t)n;
    if (cfg.use_lds)
      k_kwalk_top3<true><<<cfg.grid, KW_THREADS, cfg.lds, st>>>(codes, lvs, lvb, W.xa_start, W.xa_mem, W.xj_start,
                                                               W.xj_mem, M, mk, n, nl, (uint32_t)cfg.nwaves,
                                                               shift(o0, d), shift(o1, d), shift(o2, d));
    else
      k_kwalk_top3<false><<<cfg.grid, KW_THREADS, cfg.lds, st>>>(codes, lvs, lvb, W.xa_start, W.xa_mem, W.xj_start,
                                                          W.xj_mem, M, mk, n, nl, (uint32_t)cfg.nwaves,
                                                          shift(o0, d), shift(o1, d), shift(o2, d));
    VR_CHECK_LAUNCH();
  }
  const KOut outs[3] = {o0, o1, o2};
  const int fields[3] = {KF_DIS, fa, KF_NTIE};
  for (int i = 0; i < 3; ++i) {
    k_kfix<<<(unsigned)npass, KW_THREADS, 0, st>>>(outs[i].acc, outs[i].g, outs[i].a, outs[i].b, outs[i].incl,
                                                   (uint32_t)cfg.grid, total, fields[i], i == 0 ? 1 : 0, W.tot, cap);
    VR_CHECK_LAUNCH();
  }
  return VR_OK;
}

static int group_index(const PlanView& P, int64_t M, const KendallWs& W, uint32_t* gidx,
                       hipStream_t st) {
  const int64_t words = (M + 31) / 32;
  k_word_popc<<<blocks_for(words, 256), 256, 0, st>>>(P.gflag, words, W.wcnt);
  VR_CHECK_LAUNCH();
  VR_TRY(scan_exclusive_u32(W.wcnt, W.wcnt, words, nullptr, W.scan, st));
  k_group_index<<<blocks_for(M, 256), 256, 0, st>>>(P.gflag, W.wcnt, M, gidx);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// The level preparation's side stream and its events, one set per device, created once. The
// mutex serialises the enqueue of one call's levels (the events are reused across calls).
struct KSide {
  hipStream_t sp = nullptr;
  hipEvent_t masks = nullptr, in = nullptr, prep[2] = {nullptr, nullptr}, walked[2] = {nullptr, nullptr};
  hipEvent_t done = nullptr;
  std::mutex mu;
};

// The caller's stream waits for everything enqueued on the side stream, on every way out of
// run_kendall -- an error return included -- so no side-stream kernel can still be writing
// the caller's workspace when the next call on it starts.
struct KSideJoin {
  hipStream_t sp, st;
  hipEvent_t ev;
  bool armed = true;
  int join() {
    if (!armed) return VR_OK;
    armed = false;
    VR_CHECK_HIP(hipEventRecord(ev, sp));
    VR_CHECK_HIP(hipStreamWaitEvent(st, ev, 0));
    return VR_OK;
  }
  ~KSideJoin() { (void)join(); }
};
static int kendall_side(KSide*& out) {
  static KSide sides[64];
  static std::mutex init_mu;
  int dev = 0;
  VR_CHECK_HIP(hipGetDevice(&dev));
  VR_REQUIRE(dev >= 0 && dev < 64, "kendall: device %d out of range", dev);
  KSide& k = sides[dev];
  std::lock_guard<std::mutex> g(init_mu);
  if (!k.sp) {
    VR_CHECK_HIP(hipStreamCreateWithFlags(&k.sp, hipStreamNonBlocking));
    hipEvent_t* evs[] = {&k.masks, &k.in, &k.prep[0], &k.prep[1], &k.walked[0], &k.walked[1], &k.done};
    for (hipEvent_t* e : evs) VR_CHECK_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  out = &k;
  return VR_OK;
}

static int run_kendall(const PlanView& A, const PlanView& B, int64_t n, const int32_t* idx, int64_t k,
                       int64_t n_sets, int full_first, double* scores, const KendallWs& W,
                       int64_t cap, const KCfg& cfg, hipStream_t st) {
  const int64_t M = pairs_of(n);
  const int64_t total = n_sets + (full_first ? 1 : 0);
  if (total == 0) return VR_OK;
  PlanHeader h[2];
  if (M > 0) {
    VR_CHECK_HIP(hipMemcpyAsync(&h[0], A.hdr, sizeof(PlanHeader), hipMemcpyDeviceToHost, st));
    VR_CHECK_HIP(hipMemcpyAsync(&h[1], B.hdr, sizeof(PlanHeader), hipMemcpyDeviceToHost, st));
    VR_CHECK_HIP(hipStreamSynchronize(st));
  }
  // no pairs, a NaN anywhere, or a constant triangle: NaN for every subset (scipy:
  // empty input / nan_policy='propagate' / xtie == tot)
  if (M == 0 || h[0].has_nan || h[1].has_nan || h[0].G <= 1 || h[1].G <= 1) {
    k_kfill_nan<<<blocks_for(total, 256), 256, 0, st>>>(scores, total);
    VR_CHECK_LAUNCH();
    return VR_OK;
  }
  // Discordance and the joint ties are symmetric in the two plans: the one with fewer distinct
  // values plays y (its dense-rank bits are the levels walked), and each plan's tie total
  // still lands in its own field (x = A's, y = B's), so k_kfinal's fp64 order is unchanged.
  auto levels = [](uint32_t G) {
    int L = 0;
    while (L < 32 && ((G - 1u) >> L) != 0u) ++L;
    return L;
  };
  const bool swap = levels(h[0].G) < levels(h[1].G);
  const PlanView& PA = swap ? B : A;
  const PlanView& PB = swap ? A : B;
  const PlanHeader hx = swap ? h[1] : h[0], hy = swap ? h[0] : h[1];
  const int fx = swap ? KF_YTIE : KF_XTIE, fy = swap ? KF_XTIE : KF_YTIE;
  const unsigned gbM = blocks_for(M, 256);
  const unsigned gbW = blocks_for(kwindows(M) * 64, 256);  // whole windows: ballots
  KSide* side = nullptr;
  VR_TRY(kendall_side(side));
  std::unique_lock<std::mutex> side_lock(side->mu);
  hipStream_t sp = side->sp;
  KSideJoin side_join{sp, st, side->done};  // (destroyed before side_lock: still under the lock)
  // masks of every pass, totals zeroed
  for (int64_t set0 = 0, p = 0; set0 < total; set0 += LANES, ++p) {
    const int nl = (int)std::min<int64_t>(LANES, total - set0);
    VR_TRY(build_pass_masks(idx, k, set0, nl, full_first, W.masks + (size_t)p * (size_t)n, n, st));
  }
  VR_CHECK_HIP(hipMemsetAsync(W.tot, 0, sizeof(uint64_t) * (size_t)KF_N * (size_t)cap, st));
  VR_CHECK_HIP(hipEventRecord(side->masks, st));
  // B tie stream (B order: needs only the B plan) on the side stream, its own block summaries,
  // beside the x-lex order's construction below
  VR_CHECK_HIP(hipStreamWaitEvent(sp, side->masks, 0));
  if (hy.max_group > 1) {
    KendallWs Wy = W;
    Wy.w_acc = W.w2_acc, Wy.w_g = W.w2_g, Wy.w_a = W.w2_a, Wy.w_b = W.w2_b, Wy.w_incl = W.w2_incl;
    k_border_flags<<<gbW, 256, 0, sp>>>(PB.gflag, M, W.yb_start, W.yb_mem);
    VR_CHECK_LAUNCH();
    VR_TRY(walk_stream(true, PB.codes, W.yb_start, W.yb_mem, M, Wy, n, total, fy, false, cap, cfg, sp));
  }
  // dense group ranks of both orders
  VR_TRY(group_index(PA, M, W, W.gidxA, st));
  VR_TRY(group_index(PB, M, W, W.gidxB, st));
  // (x, y)-lexicographic order: stable sort of B order by A group
  k_kendall_keys<<<gbM, 256, 0, st>>>(PB.codes, M, n, PA.pos_map, W.gidxA, W.keys, W.vals);
  VR_CHECK_LAUNCH();
  VR_TRY(radix_sort_kv(W.keys, W.vals, W.keys_alt, W.vals_alt, M, W.radix, st));
  k_kendall_elems<<<gbM, 256, 0, st>>>(W.vals, PB.codes, W.gidxB, M, W.ecode[0], W.ey[0]);
  VR_CHECK_LAUNCH();
  VR_CHECK_HIP(hipEventRecord(side->in, st));  // the level-0 stream exists: preparation may start
  // x-lex tie streams (only when A has multi-element groups)
  // (fused into the top level's walk below unless VISREPS_KENDALL_TOP3=0)
  static const bool top3 = !(getenv("VISREPS_KENDALL_TOP3") && atoi(getenv("VISREPS_KENDALL_TOP3")) == 0);
  const bool xties = hx.max_group > 1;
  if (xties) {
    k_xlex_flags<<<gbW, 256, 0, st>>>(W.keys, W.ey[0], M, W.xa_start, W.xa_mem, W.xj_start, W.xj_mem);
    VR_CHECK_LAUNCH();
    if (!top3) {
      VR_TRY(walk_stream(true, W.ecode[0], W.xa_start, W.xa_mem, M, W, n, total, fx, false, cap, cfg, st));
      VR_TRY(walk_stream(true, W.ecode[0], W.xj_start, W.xj_mem, M, W, n, total, KF_NTIE, false, cap, cfg, st));
    }
  }
  // inversion levels, most significant y bit first
  const uint32_t G = hy.G;
  int Lb = 0;
  while (Lb < 32 && ((G - 1u) >> Lb) != 0u) ++Lb;
  // Level b walks stream c = (Lb - 1 - b) & 1 (ecode/ey[c], planes lv_*[c]) on the caller's
  // stream while the side stream prepares level b - 1 into the other buffers (plane word
  // scan, stable split, next planes): VALU-bound walks and memory-bound preparation share the
  // CUs (a walk block holds one 16-wave workgroup per CU). The preparation of b - 1 waits for
  // the walks of b + 1, the last readers of the buffers it writes.
  const int64_t words = (M + 31) / 32;
  VR_CHECK_HIP(hipStreamWaitEvent(sp, side->in, 0));
  k_level_flags<<<gbW, 256, 0, sp>>>(W.ey[0], M, Lb - 1, W.lv_start[0], W.lv_bits[0]);
  VR_CHECK_LAUNCH();
  VR_CHECK_HIP(hipEventRecord(side->prep[0], sp));
  for (int b = Lb - 1; b >= 0; --b) {
    const int c = (Lb - 1 - b) & 1;
    if (b > 0) {
      if (b < Lb - 1) VR_CHECK_HIP(hipStreamWaitEvent(sp, side->walked[c ^ 1], 0));
      k_word_popc<<<blocks_for(words, 256), 256, 0, sp>>>(W.lv_bits[c], words, W.wcnt);
      VR_CHECK_LAUNCH();
      VR_TRY(scan_exclusive_u32(W.wcnt, W.wcnt, words, nullptr, W.scan, sp));
      k_level_split<<<gbM, 256, 0, sp>>>(W.ecode[c], W.ey[c], W.lv_bits[c], W.wcnt, PB.gstart, M, b,
                                         W.ecode[c ^ 1], W.ey[c ^ 1]);
      VR_CHECK_LAUNCH();
      k_level_flags<<<gbW, 256, 0, sp>>>(W.ey[c ^ 1], M, b - 1, W.lv_start[c ^ 1], W.lv_bits[c ^ 1]);
      VR_CHECK_LAUNCH();
      VR_CHECK_HIP(hipEventRecord(side->prep[c ^ 1], sp));
    }
    VR_CHECK_HIP(hipStreamWaitEvent(st, side->prep[c], 0));
    if (b == Lb - 1 && xties && top3)  // level 0's stream is the x-lex order the tie streams walk
      VR_TRY(walk_top3(W.ecode[c], W.lv_start[c], W.lv_bits[c], W, M, n, total, fx, cap, cfg, st));
    else
      VR_TRY(walk_stream(false, W.ecode[c], W.lv_start[c], W.lv_bits[c], M, W, n, total, KF_DIS, b == Lb - 1,
                         cap, cfg, st));
    VR_CHECK_HIP(hipEventRecord(side->walked[c], st));
  }
  VR_TRY(side_join.join());
  side_lock.unlock();
  k_kfinal<<<blocks_for(total, 256), 256, 0, st>>>(W.tot, cap, total, scores);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// ---------------------------------------------------------------------------------
// Kendall tau-a of two plain vectors (rsa.py:22-40 `_kendall_tau_a(x, y)` itself, which the
// reference's tests call on short arrays and on RDM triangles): every unordered pair (i, j)
// compared directly in fp64, exact integer counts. A block holds KV_ROWS rows i in
// registers and streams a KV_COLS-wide strip of j > i through LDS; counts go through a
// wave reduction into one u64 atomic per field and block (integer adds: order-free).
// ---------------------------------------------------------------------------------
constexpr int KV_ROWS = 256;
constexpr int KV_COLS = 4096;

__device__ inline uint64_t wave_sum_u64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(KV_ROWS) void k_kendall_vec_pairs(const double* __restrict__ x,
                                                               const double* __restrict__ y, int64_t m,
                                                               uint64_t* __restrict__ tot) {
  __shared__ double sx[KV_ROWS], sy[KV_ROWS];
  const int64_t i = (int64_t)blockIdx.x * KV_ROWS + threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * KV_ROWS;  // the block's first row
  const int64_t c0 = (int64_t)blockIdx.y * KV_COLS;
  const int64_t c1 = c0 + KV_COLS < m ? c0 + KV_COLS : m;
  if (c1 <= r0 + 1) return;  // the strip holds no j > i for any row of the block
  const double xi = i < m ? x[i] : 0.0, yi = i < m ? y[i] : 0.0;
  uint64_t dis = 0, xt = 0, yt = 0, nt = 0;
  for (int64_t t0 = c0 > r0 ? c0 : r0; t0 < c1; t0 += KV_ROWS) {
    __syncthreads();
    const int64_t j = t0 + threadIdx.x;
    sx[threadIdx.x] = j < c1 ? x[j] : 0.0;
    sy[threadIdx.x] = j < c1 ? y[j] : 0.0;
    __syncthreads();
    const int cnt = (int)((c1 - t0) < KV_ROWS ? (c1 - t0) : KV_ROWS);
    uint32_t d = 0, a = 0, b = 0, ab = 0;
    if (i < m) {
      // only j > i: the tile's entries from i + 1 - t0 on
      for (int q = i + 1 - t0 > 0 ? (int)(i + 1 - t0) : 0; q < cnt; ++q) {
        const double xj = sx[q], yj = sy[q];
        const bool tx = xi == xj, ty = yi == yj;
        const bool gx = xi > xj, gy = yi > yj;
        d += (!tx && !ty && gx != gy) ? 1u : 0u;
        a += tx ? 1u : 0u;
        b += ty ? 1u : 0u;
        ab += (tx && ty) ? 1u : 0u;
      }
    }
    dis += d;
    xt += a;
    yt += b;
    nt += ab;
  }
  dis = wave_sum_u64(dis);
  xt = wave_sum_u64(xt);
  yt = wave_sum_u64(yt);
  nt = wave_sum_u64(nt);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd((unsigned long long*)&tot[KF_DIS], (unsigned long long)dis);
    atomicAdd((unsigned long long*)&tot[KF_XTIE], (unsigned long long)xt);
    atomicAdd((unsigned long long*)&tot[KF_YTIE], (unsigned long long)yt);
    atomicAdd((unsigned long long*)&tot[KF_NTIE], (unsigned long long)nt);
  }
}

__global__ void k_kendall_vec_init(const double* __restrict__ x, const double* __restrict__ y, int64_t m,
                                   uint64_t* __restrict__ tot, uint32_t* __restrict__ nan_flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < KF_N) tot[i] = i == KF_INCL ? (uint64_t)m : 0ull;
  if (i < m && (x[i] != x[i] || y[i] != y[i])) atomicOr(nan_flag, 1u);  // nan_policy='propagate'
}

__global__ void k_kendall_vec_final(const uint64_t* __restrict__ tot, const uint32_t* __restrict__ nan_flag,
                                    double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  if (*nan_flag) {
    out[0] = __builtin_nan("");
    return;
  }
  // k_kfinal's fp64 order for one set (cap 1)
  const uint64_t t = tot[KF_INCL] * (tot[KF_INCL] - 1) / 2;
  const uint64_t dis = tot[KF_DIS], xt = tot[KF_XTIE], yt = tot[KF_YTIE], nt = tot[KF_NTIE];
  double r = __builtin_nan("");
  if (xt != t && yt != t) {
    const int64_t cmd = (int64_t)(t - xt - yt + nt) - 2 * (int64_t)dis;
    double taub = (double)cmd / sqrt((double)(t - xt)) / sqrt((double)(t - yt));
    taub = fmin(1.0, fmax(-1.0, taub));
    const double denom = sqrt((double)(t - xt) * (double)(t - yt));
    r = denom == 0.0 ? __builtin_nan("") : taub * denom / (double)t;
  }
  out[0] = r;
}

static size_t k_oneshot_bytes(int64_t n, int64_t cap, int nwaves, void* base, PlanView* A, PlanView* B,
                              PlanBuildWs* PW, KendallWs* W) {
  Carver c(base);
  const size_t pb = plan_bytes(n);
  char* pa = c.take<char>(pb);
  char* pbb = c.take<char>(pb);
  size_t wb = 0, kb = 0;
  plan_build_layout(nullptr, n, &wb);
  kendall_layout(nullptr, n, cap, nwaves, &kb);
  char* wsb = c.take<char>(std::max(wb, kb));  // plan-build scratch is dead once plans exist
  if (base) {
    *A = plan_layout(pa, n);
    *B = plan_layout(pbb, n);
    *PW = plan_build_layout(wsb, n, nullptr);
    *W = kendall_layout(wsb, n, cap, nwaves, nullptr);
  }
  return c.bytes();
}

}  // namespace vr

using namespace vr;

extern "C" {

size_t vr_bootstrap_kendall_workspace(int64_t n, int64_t n_sets) {
  size_t b = 0;
  n = n < 0 ? 0 : n;
  n_sets = n_sets < 0 ? 0 : n_sets;
  kendall_layout(nullptr, n, n_sets + 1, kendall_cfg(n).nwaves, &b);
  return b;
}

int vr_bootstrap_kendall_plans(const void* planA, const void* planB, int64_t n, const int32_t* idx,
                               int64_t k, int64_t n_sets, int full_first, double* scores, void* ws,
                               size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535, "vr_bootstrap_kendall_plans: n=%lld out of range", (long long)n);
  VR_REQUIRE(planA && planB && scores, "vr_bootstrap_kendall_plans: null pointer");
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "vr_bootstrap_kendall_plans: bad k=%lld sets=%lld",
             (long long)k, (long long)n_sets);
  VR_REQUIRE(idx != nullptr || n_sets == 0 || k == 0, "vr_bootstrap_kendall_plans: null idx");
  const KCfg cfg = kendall_cfg(n);
  const int64_t cap = n_sets + 1;
  size_t need = 0;
  KendallWs W = kendall_layout(ws, n, cap, cfg.nwaves, &need);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_bootstrap_kendall_plans: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView A = plan_layout(const_cast<void*>(planA), n);
  PlanView B = plan_layout(const_cast<void*>(planB), n);
  return run_kendall(A, B, n, idx, k, n_sets, full_first, scores, W, cap, cfg, as_stream(stream));
}

size_t vr_kendall_triu_workspace(int64_t n) {
  n = n < 0 ? 0 : n;
  return k_oneshot_bytes(n, 1, kendall_cfg(n).nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int vr_kendall_triu_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out, void* ws,
                        size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535 && ld >= n, "vr_kendall_triu_f32: bad shape n=%lld ld=%lld",
             (long long)n, (long long)ld);
  VR_REQUIRE(out != nullptr, "vr_kendall_triu_f32: null out");
  const KCfg cfg = kendall_cfg(n);
  const size_t need = k_oneshot_bytes(n, 1, cfg.nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_kendall_triu_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView PA, PB;
  PlanBuildWs PW;
  KendallWs W;
  k_oneshot_bytes(n, 1, cfg.nwaves, ws, &PA, &PB, &PW, &W);
  hipStream_t st = as_stream(stream);
  VR_TRY(build_plan(A, n, ld, PA, PW, st));
  VR_TRY(build_plan(B, n, ld, PB, PW, st));
  return run_kendall(PA, PB, n, nullptr, 0, 0, 1, out, W, 1, cfg, st);
}

size_t vr_kendall_vec_workspace(int64_t m) {
  (void)m;
  return 256;  // KF_N u64 totals + the NaN flag
}

int vr_kendall_tau_a_f64(const double* x, const double* y, int64_t m, double* out, void* ws, size_t ws_bytes,
                         void* stream) {
  VR_REQUIRE(m >= 0 && m <= ((int64_t)1 << 22), "vr_kendall_tau_a_f64: m=%lld out of range (<= 2^22)",
             (long long)m);
  VR_REQUIRE(out != nullptr && (m == 0 || (x != nullptr && y != nullptr)), "vr_kendall_tau_a_f64: null pointer");
  if (ws == nullptr || ws_bytes < vr_kendall_vec_workspace(m)) {
    set_error("vr_kendall_tau_a_f64: workspace %zu < %zu", ws_bytes, vr_kendall_vec_workspace(m));
    return VR_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (m < 2) {  // rsa.py:25-26: fewer than two elements -> NaN
    k_kfill_nan<<<1, 64, 0, st>>>(out, 1);
    VR_CHECK_LAUNCH();
    return VR_OK;
  }
  uint64_t* tot = static_cast<uint64_t*>(ws);
  uint32_t* nan_flag = reinterpret_cast<uint32_t*>(tot + KF_N);
  VR_CHECK_HIP(hipMemsetAsync(nan_flag, 0, sizeof(uint32_t), st));
  k_kendall_vec_init<<<blocks_for(std::max<int64_t>(m, KF_N), 256), 256, 0, st>>>(x, y, m, tot, nan_flag);
  VR_CHECK_LAUNCH();
  const dim3 grid((unsigned)((m + KV_ROWS - 1) / KV_ROWS), (unsigned)((m + KV_COLS - 1) / KV_COLS));
  k_kendall_vec_pairs<<<grid, KV_ROWS, 0, st>>>(x, y, m, tot);
  VR_CHECK_LAUNCH();
  k_kendall_vec_final<<<1, 64, 0, st>>>(tot, nan_flag, out);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // extern "C"
