// RDM = 1 - Pearson correlation of the rows of X (n x d), the MI355X replacement of
// compute_rdm(.., correlation="Pearson") in visreps/analysis/rsa.py:59-93:
//   x = X.float(); x -= x.mean(1); std = sqrt(mean(x^2, 1) + c); std[std < 10c] = 1
//   cov = x @ x.T / D; corr = cov / (std_i std_j + c); clamp(-1, 1); diag = 1; 1 - corr
//
// Kernels
//  k_row_stats   one block per row, two passes (mean, then centred sum of squares),
//                fp64 accumulation of fp32 terms -> fp32 mean / std.     [HBM-bound]
//  k_gram        symmetric Gram of the centred rows on the fp32 matrix cores
//                (v_mfma_f32_32x32x2_f32, exact fp32 fma chains). Only tiles with
//                bi <= bj are computed; centring is fused into the register staging
//                of each 128x32 panel; the epilogue writes the tile and its mirror.
//                Split-K over d when the tile count cannot fill 256 CUs, with fp32
//                partial tiles reduced in fixed order by k_gram_reduce.  [MFMA-bound]
#include <cstdlib>
#include <cstring>

#include "internal.h"

namespace vr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------------------------
// Row statistics
// ------------------------------------------------------------------------------------
constexpr int RSTAT_BS = 256;

__device__ inline double block_sum_f64(double v, double* lds) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  double s = 0;
  if (threadIdx.x == 0) {
    for (int w = 0; w < RSTAT_BS / 64; ++w) s += lds[w];
    lds[RSTAT_BS / 64] = s;
  }
  __syncthreads();
  s = lds[RSTAT_BS / 64];
  __syncthreads();
  return s;
}

// Input elements as fp32: float as is, bf16 (stored as its 16-bit pattern) exactly widened,
// which is the reference's X.float() (rsa.py:76) without materialising an fp32 copy.
__device__ inline float in_f32(float v) { return v; }
__device__ inline float in_f32(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ inline f32x4 in_f32x4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ inline f32x4 in_f32x4(const uint16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}

template <typename T>
__global__ __launch_bounds__(RSTAT_BS) void k_row_stats(const T* __restrict__ X, int64_t d,
                                                        int64_t ldx, float* __restrict__ mean,
                                                        float* __restrict__ stdv,
                                                        float correction, int vec) {
  __shared__ double lds[RSTAT_BS / 64 + 1];
  const T* row = X + (int64_t)blockIdx.x * ldx;
  double s = 0;
  if (vec) {
    const int64_t d4 = d / 4;
    for (int64_t i = threadIdx.x; i < d4; i += RSTAT_BS) {
      f32x4 v = in_f32x4(row + 4 * i);
      s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
    }
    for (int64_t i = d4 * 4 + threadIdx.x; i < d; i += RSTAT_BS) s += (double)in_f32(row[i]);
  } else {
    for (int64_t i = threadIdx.x; i < d; i += RSTAT_BS) s += (double)in_f32(row[i]);
  }
  s = block_sum_f64(s, lds);
  const float m = (float)(s / (double)d);
  double q = 0;
  if (vec) {
    const int64_t d4 = d / 4;
    for (int64_t i = threadIdx.x; i < d4; i += RSTAT_BS) {
      f32x4 v = in_f32x4(row + 4 * i);
      float a = v.x - m, b = v.y - m, c = v.z - m, e = v.w - m;
      q += (double)(a * a) + (double)(b * b) + (double)(c * c) + (double)(e * e);
    }
    for (int64_t i = d4 * 4 + threadIdx.x; i < d; i += RSTAT_BS) {
      float a = in_f32(row[i]) - m;
      q += (double)(a * a);
    }
  } else {
    for (int64_t i = threadIdx.x; i < d; i += RSTAT_BS) {
      float a = in_f32(row[i]) - m;
      q += (double)(a * a);
    }
  }
  q = block_sum_f64(q, lds);
  if (threadIdx.x == 0) {
    float var = (float)(q / (double)d);
    float sd = sqrtf(var + correction);
    if (sd < correction * 10.0f) sd = 1.0f;  // rsa.py:84-87 zero-variance guard
    mean[blockIdx.x] = m;
    stdv[blockIdx.x] = sd;
  }
}

// ------------------------------------------------------------------------------------
// Symmetric Gram on fp32 MFMA
// ------------------------------------------------------------------------------------
constexpr int GT = 128;            // tile edge (rows of the i and j panels)
constexpr int GK = 32;             // k per LDS stage
constexpr int GLD = GK + 4;        // padded LDS row: conflict-free ds_read_b128
constexpr int G_THREADS = 256;     // 4 waves as 2x2, each wave 64x64 = 2x2 MFMA tiles
constexpr int G_STAGE = GT * GLD;  // floats per panel per stage

struct GramParams {
  const float* X;
  const float* mean;
  const float* stdv;
  float* rdm;
  float* partial;   // split-K fp32 partial tiles (null when splits == 1)
  int64_t n, d, ldx, ldr;
  int64_t kslice;   // k extent of one split (multiple of GK)
  int T;            // tiles per dimension
  int ntiles;       // T*(T+1)/2
  int splits;
  int tile0;        // first upper-triangle tile of this launch (block-distributed Gram)
  int tile_count;   // tiles in this launch
  float correction;
  int vec;          // 16-B aligned rows: float4 staging
  const uint16_t* planes;  // split Gram: bf16 hi/lo stage records (null: fp32 kernel)
  int64_t nstage;          // 32-k stages per plane row
  int blk0;                // first launch position of this generation (see gram_generation)
  int raw;                 // 1: plain Gram X X^T (no centring, no correlation epilogue)
  int flush;               // k stages between accumulator flushes (0: none), see gram_flush
  float* fbuf;             // flush buffer: one tile of fp32 per block of a launch
  int one;                 // bf16 input, one product: records hold raw x (64 k per stage), centring in the epilogue
  int64_t dk;              // k extent in 32-k units the split-K geometry covers (d; 32 nstage when one)
};

// Accumulation error. Every MFMA rounds its output to fp32, so an accumulator that runs over
// the whole depth sums D/16 (x3 for the split kernel) increments into one growing fp32 value;
// on post-ReLU rows (centred zeros: coherent positive products) that chain left RDM entries
// ~1e-4 off at D = 43k-290k and Spearman scores up to 3e-5 off (profiles/r2_gram_accuracy.log).
// Flushing: every `flush` k stages each lane adds its accumulators into the block's fp32 tile
// in fbuf (stores them on the first flush) and restarts them at zero; the epilogue adds the
// tile back. The inner chains are `flush` stages long and the outer sum has D / (32 flush)
// terms: a two-level sum, like the k-blocked accumulation of a CPU sgemm.
// The lane's base pointer passes through an empty asm so it is formed here, at the flush,
// and not hoisted out of the k loop with its 2 x M_ x N_ x 16 derived addresses.
template <int LD, int M_, int N_>
__device__ inline float* flush_base(float* buf, int r0, int c0) {
  const int lane = threadIdx.x & 63;
  uint32_t off = (uint32_t)((r0 + 4 * (lane >> 5)) * LD + c0 + (lane & 31));
  asm volatile("" : "+v"(off));
  return buf + off;
}

template <int LD, int M_, int N_>
__device__ inline void gram_flush(f32x16 (&acc)[M_][N_], float* buf, int r0, int c0, bool first) {
  float* b = flush_base<LD, M_, N_>(buf, r0, c0);
#pragma unroll
  for (int m = 0; m < M_; ++m)
#pragma unroll
    for (int nn = 0; nn < N_; ++nn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float* p = b + (m * 32 + (r & 3) + 8 * (r >> 2)) * LD + nn * 32;
        *p = first ? acc[m][nn][r] : *p + acc[m][nn][r];
        acc[m][nn][r] = 0.f;
      }
}

template <int LD, int M_, int N_>
__device__ inline void gram_unflush(f32x16 (&acc)[M_][N_], float* buf, int r0, int c0) {
  const float* b = flush_base<LD, M_, N_>(buf, r0, c0);
#pragma unroll
  for (int m = 0; m < M_; ++m)
#pragma unroll
    for (int nn = 0; nn < N_; ++nn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][nn][r] += b[(m * 32 + (r & 3) + 8 * (r >> 2)) * LD + nn * 32];
}

__device__ inline void tile_coords(int p, int T, int& bi, int& bj) {
  // row-major enumeration of the upper triangle: row bi holds T - bi tiles
  float tf = (float)T;
  int r = (int)((2.f * tf + 1.f - sqrtf((2.f * tf + 1.f) * (2.f * tf + 1.f) - 8.f * (float)p)) * 0.5f);
  if (r < 0) r = 0;
  if (r > T - 1) r = T - 1;
  auto off = [&](int b) { return b * T - b * (b - 1) / 2; };
  while (r > 0 && off(r) > p) --r;
  while (r + 1 < T && off(r + 1) <= p) ++r;
  bi = r;
  bj = r + (p - off(r));
}

// Launch order of the tiles [t0, t0 + count) of the row-major upper-triangle numbering:
// bands of GBAND tile rows (counted from the range's first row), each band walked column
// by column. After xcd_remap one XCD runs consecutive positions, so the ~64 blocks it
// holds at once share ~GBAND row panels and ~GBAND column panels in its L2 instead of
// one row panel and ~64 column panels. Position p -> tile (bi, bj); a bijection on the
// range, so any contiguous tile range (block-distributed Gram) keeps its exact tile set.
constexpr int GBAND = 8;

__device__ inline int64_t tri_row_start(int r, int T) {
  return (int64_t)r * T - (int64_t)r * (r - 1) / 2;
}

__device__ inline void band_tile(int p, int t0, int count, int T, int& bi, int& bj) {
  int ra, ca, rz, cz, r, c;
  tile_coords(t0, T, ra, ca);
  tile_coords(t0 + count - 1, T, rz, cz);
  tile_coords(t0 + p, T, r, c);
  const int i0 = ra + (r - ra) / GBAND * GBAND;
  const int i1 = min(rz, i0 + GBAND - 1);
  const int64_t gs = (i0 == ra) ? (int64_t)t0 : tri_row_start(i0, T);
  const int q = (int)((int64_t)t0 + p - gs);
  // columns [lo(i), hi(i)) of band row i inside the range
  auto lo = [&](int i) { return i == ra ? ca : i; };
  auto hi = [&](int i) { return i == rz ? cz + 1 : T; };
  auto before = [&](int col) {  // band tiles in columns < col
    int s = 0;
    for (int i = i0; i <= i1; ++i) s += max(0, min(col, hi(i)) - lo(i));
    return s;
  };
  int a = 0, b = T;  // before(a) <= q < before(b)
  while (b - a > 1) {
    const int m = (a + b) >> 1;
    if (before(m) <= q) a = m; else b = m;
  }
  int k = q - before(a);  // the k-th band row holding column a
  bi = r;
  bj = c;
  for (int i = i0; i <= i1; ++i) {
    if (lo(i) <= a && a < hi(i)) {
      if (k == 0) {
        bi = i;
        bj = a;
        return;
      }
      --k;
    }
  }
}

// Loads this thread's 4 float4 of a 128 x 32 panel (rows row0.., k in [k, k+32)).
// Interior stages (whole panel inside [0,n) x [k0,k1), 16-B rows) take the unguarded
// path: four independent loads whose data is first touched after the stage's MFMAs, so
// their latency hides under them. Edge stages zero-fill outside the matrix; centring is
// applied at the LDS store (store_panel), where out-of-range elements stay exactly 0.
__device__ inline void load_panel_fast(const GramParams& P, int64_t row0, int64_t k, f32x4 out[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int f = threadIdx.x + G_THREADS * s;
    const int r = f >> 3, c4 = f & 7;
    out[s] = *reinterpret_cast<const f32x4*>(P.X + (row0 + r) * P.ldx + k + c4 * 4);
  }
}

__device__ inline void load_panel_edge(const GramParams& P, int64_t row0, int64_t k, int64_t k1,
                                       f32x4 out[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int f = threadIdx.x + G_THREADS * s;
    const int r = f >> 3, c4 = f & 7;
    const int64_t row = row0 + r;
    const int64_t kk = k + c4 * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < P.n) {
      const float* src = P.X + row * P.ldx + kk;
      if (kk + 0 < k1) v.x = src[0];
      if (kk + 1 < k1) v.y = src[1];
      if (kk + 2 < k1) v.z = src[2];
      if (kk + 3 < k1) v.w = src[3];
    }
    out[s] = v;
  }
}

// Both panels of a stage behind one uniform branch (a diagonal tile's B rows are its A
// rows: the duplicate loads hit cache and are not staged).
__device__ inline void load_stage(const GramParams& P, bool fast, int64_t row0, int64_t col0,
                                  int64_t k, int64_t k1, f32x4 a[4], f32x4 b[4]) {
  if (fast) {
    load_panel_fast(P, row0, k, a);
    load_panel_fast(P, col0, k, b);
  } else {
    load_panel_edge(P, row0, k, k1, a);
    load_panel_edge(P, col0, k, k1, b);
  }
}

// Centre and stage a panel: element (r, k) <- x - mean_r inside the matrix, 0 outside.
__device__ inline void store_panel(const GramParams& P, float* lds, int64_t row0, int64_t k,
                                   int64_t k1, const float mrow[4], const f32x4 v[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int f = threadIdx.x + G_THREADS * s;
    const int r = f >> 3, c4 = f & 7;
    const int64_t kk = k + c4 * 4;
    const bool rin = row0 + r < P.n;
    f32x4 w;
    w.x = (rin && kk + 0 < k1) ? v[s].x - mrow[s] : 0.f;
    w.y = (rin && kk + 1 < k1) ? v[s].y - mrow[s] : 0.f;
    w.z = (rin && kk + 2 < k1) ? v[s].z - mrow[s] : 0.f;
    w.w = (rin && kk + 3 < k1) ? v[s].w - mrow[s] : 0.f;
    *reinterpret_cast<f32x4*>(lds + r * GLD + c4 * 4) = w;
  }
}

// Epilogue for one element: rdm = 1 - clamp(G/d / (s_i s_j + c)), exactly the
// reference's fp32 operation order; NaN propagates like torch.clamp.
// ONE (one product, bf16 input): g = sum x_i x_j of the raw values; the centring is the
// rank-1 correction cov = g/d - mean_i mean_j, in fp64, rounded once (then the reference's order)
template <bool ONE>
__device__ inline float rdm_value_t(float g, int64_t i, int64_t j, const GramParams& P,
                                    float si, float sj) {
  if (P.raw) return g;  // vr_gram_f32
  float cov;
  if constexpr (ONE)
    cov = (float)((double)g / (double)P.d -
                  (double)(i < P.n ? P.mean[i] : 0.f) * (double)(j < P.n ? P.mean[j] : 0.f));
  else
    cov = g / (float)P.d;
  float c = cov / (si * sj + P.correction);
  c = (c < -1.f) ? -1.f : ((c > 1.f) ? 1.f : c);
  if (i == j) c = 1.f;
  return 1.f - c;
}
__device__ inline float rdm_value(float g, int64_t i, int64_t j, const GramParams& P, float si, float sj) {
  return P.one ? rdm_value_t<true>(g, i, j, P, si, sj) : rdm_value_t<false>(g, i, j, P, si, sj);
}

// Tile epilogue (one 2x2 grid of 32x32 accumulators per wave). C/D map of the 32x32 MFMAs
// (fp32 and bf16 alike): col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5). A diagonal
// tile writes each i < j entry from its (i, j) accumulator to both (i, j) and (j, i), so
// the RDM is exactly symmetric whatever the product order of the two accumulators.
__device__ inline void gram_store(const GramParams& P, f32x16 (&acc)[2][2], int64_t row0,
                                  int64_t col0, bool diag, int split, int ltile) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  if (P.splits == 1) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn) {
        const int64_t j = col0 + wc * 64 + nn * 32 + l32;
        const float sj = (j < P.n) ? P.stdv[j] : 1.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int64_t ib = row0 + wr * 64 + m * 32 + 8 * g + 4 * h;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t i = ib + e;
            const float si = (i < P.n) ? P.stdv[i] : 1.f;
            v[e] = rdm_value(acc[m][nn][4 * g + e], i, j, P, si, sj);
          }
          if (diag) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int64_t i = ib + e;
              if (i <= j && j < P.n) {
                P.rdm[i * P.ldr + j] = v[e];
                if (i < j) P.rdm[j * P.ldr + i] = v[e];
              }
            }
            continue;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t i = ib + e;
            if (i < P.n && j < P.n) P.rdm[i * P.ldr + j] = v[e];
          }
          if (j < P.n) {  // mirror: rows ib..ib+3 are 4 consecutive columns of row j
            float* dst = P.rdm + j * P.ldr + ib;
            if (P.vec && ib + 3 < P.n && ((P.ldr & 3) == 0)) {
              f32x4 w = {v[0], v[1], v[2], v[3]};
              *reinterpret_cast<f32x4*>(dst) = w;
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (ib + e < P.n) dst[e] = v[e];
            }
          }
        }
      }
  } else {
    float* out = P.partial + ((int64_t)split * P.tile_count + ltile) * (GT * GT);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn) {
        const int lj = wc * 64 + nn * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int li = wr * 64 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          out[li * GT + lj] = acc[m][nn][r];
        }
      }
  }
}

__global__ __launch_bounds__(G_THREADS, 2) void k_gram(GramParams P) {
  __shared__ __attribute__((aligned(16))) float lds[2 * 2 * G_STAGE];  // [buf][A/B]
  const int nwg = gridDim.x;
  const int id = P.blk0 + (int)xcd_remap(blockIdx.x, (uint32_t)nwg);
  const int ltile = id / P.splits, split = id % P.splits;
  int bi, bj;
  band_tile(ltile, P.tile0, P.tile_count, P.T, bi, bj);
  const bool diag = (bi == bj);
  const int64_t row0 = (int64_t)bi * GT, col0 = (int64_t)bj * GT;
  const int64_t k0 = (int64_t)split * P.kslice;
  const int64_t k1 = min(P.d, k0 + P.kslice);
  const int nk = (int)((k1 - k0 + GK - 1) / GK);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;

  float mA[4], mB[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int r = (threadIdx.x + G_THREADS * s) >> 3;
    mA[s] = (row0 + r < P.n) ? P.mean[row0 + r] : 0.f;
    mB[s] = (col0 + r < P.n) ? P.mean[col0 + r] : 0.f;
  }

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  // a stage is "fast" when both panels lie inside the matrix (rows and k) with 16-B rows
  const bool rows_in = P.vec && row0 + GT <= P.n && col0 + GT <= P.n;
  auto fast_at = [&](int64_t k) { return rows_in && k + GK <= k1; };
  f32x4 ga[4], gb[4];
  if (nk > 0) {
    load_stage(P, fast_at(k0), row0, col0, k0, k1, ga, gb);
    store_panel(P, lds, row0, k0, k1, mA, ga);
    if (!diag) store_panel(P, lds + G_STAGE, col0, k0, k1, mB, gb);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const float* As = lds + cur * 2 * G_STAGE;
    const float* Bs = diag ? As : As + G_STAGE;
    const bool more = kt + 1 < nk;
    const int64_t kn = k0 + (int64_t)(kt + 1) * GK;
    if (more) load_stage(P, fast_at(kn), row0, col0, kn, k1, ga, gb);  // lands under the MFMAs
    // lane half h owns k in [16h, 16h+16) of this stage (a consistent k permutation of
    // the MFMA's 2-deep k; the Gram sums over k so any fixed permutation is exact)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 av[2], bv[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int ar = wr * 64 + m * 32 + l32;
        av[m] = *reinterpret_cast<const f32x4*>(As + ar * GLD + h * 16 + q * 4);
        const int br = wc * 64 + m * 32 + l32;
        bv[m] = *reinterpret_cast<const f32x4*>(Bs + br * GLD + h * 16 + q * 4);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nn = 0; nn < 2; ++nn)
            acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m][e], bv[nn][e], acc[m][nn], 0, 0, 0);
    }
    if (more) {
      float* nxt = lds + (cur ^ 1) * 2 * G_STAGE;
      store_panel(P, nxt, row0, kn, k1, mA, ga);
      if (!diag) store_panel(P, nxt + G_STAGE, col0, kn, k1, mB, gb);
    }
    if (P.flush && more && (kt + 1) % P.flush == 0) {
      gram_flush<GT>(acc, P.fbuf + (size_t)blockIdx.x * GT * GT, wr * 64, wc * 64, kt + 1 == P.flush);
    }
    __syncthreads();
  }
  if (P.flush && nk > P.flush) gram_unflush<GT>(acc, P.fbuf + (size_t)blockIdx.x * GT * GT, wr * 64, wc * 64);

  gram_store(P, acc, row0, col0, diag, split, ltile);
}

// ------------------------------------------------------------------------------------
// Split Gram: the centred rows as two bf16 planes, x - mean = hi + lo with
// |x - mean - hi - lo| <= 2^-18 |x - mean|, and three bf16 MFMA products per k-step
// (hi.hi + hi.lo + lo.hi, fp32 accumulate). The dropped lo.lo term and the lo rounding
// are uncorrelated across k, so a Gram entry's error against the exact centred Gram is
// ~2^-17 sqrt(sum_k x_ik^2 x_jk^2): below the fp32 summation error of the reference's own
// sgemm for these shapes. CDNA4's bf16 matrix rate is 16x its fp32 rate.
// ------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int SROW = 72;              // LDS row: 32 hi + 32 lo bf16 + 8 pad (144 B, conflict-free b128)
constexpr int S_STAGE = GT * SROW;    // bf16 per panel per stage

// Planes: per row and 32-k stage one 128-byte record [hi k0..31 | lo k0..31]; rows padded
// to the tile edge and k to the stage with exact zeros (so the Gram kernel has no edges).
// Fused prepass of the split kernel: the row statistics of k_row_stats (same per-thread
// fp64 sums in the same order, so mean and std are bit-identical to it) and, in the
// centred second pass, the bf16 hi/lo stage records (x - mean = hi + lo, hi = bf16(v), lo = bf16(v - hi)). One
// read of X fewer than separate statistics and split passes (12 instead of 16 B per element). Rows in
// [n, gridDim.x) and k in [d, 32 nstage) get exact-zero records.
__device__ inline void split_pair(float v, uint16_t& h, uint16_t& l) {
  const __bf16 hb = (__bf16)v;
  h = __builtin_bit_cast(uint16_t, hb);
  l = __builtin_bit_cast(uint16_t, (__bf16)(v - (float)hb));
}

__device__ inline void split_store4(uint16_t* prow, int64_t i, f32x4 v) {
  uint16_t h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) split_pair(v[e], h[e], l[e]);
  uint16_t* dst = prow + (i >> 3) * 64 + (i & 7) * 4;  // stage i / 8, 4-k group i % 8
  *reinterpret_cast<uint2*>(dst) = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
  *reinterpret_cast<uint2*>(dst + 32) = make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
}

__device__ inline void split_store1(uint16_t* prow, int64_t k, float v) {
  uint16_t h, l;
  split_pair(v, h, l);
  prow[(k >> 5) * 64 + (k & 31)] = h;
  prow[(k >> 5) * 64 + 32 + (k & 31)] = l;
}

// One row of k_stats_split (one block per row): fp64 row sum -> fp32 mean, then the centred
// values -> fp64 sum of squares (std, with the reference's zero-variance guard) and their
// bf16 hi/lo records, in the same pass.
template <typename T>
__device__ inline void stats_split_row(const T* __restrict__ X, int64_t n, int64_t d, int64_t ldx, int64_t nstage,
                                       float correction, int vec, float* __restrict__ mean,
                                       float* __restrict__ stdv, uint16_t* __restrict__ planes, int64_t r,
                                       double* lds) {
  const int64_t kp = nstage * GK;
  uint16_t* prow = planes + r * nstage * 64;
  if (r >= n) {  // padding row
    for (int64_t i = threadIdx.x; i < kp / 4; i += RSTAT_BS) split_store4(prow, i, f32x4{0.f, 0.f, 0.f, 0.f});
    return;
  }
  const T* row = X + r * ldx;
  double s = 0;
  const int64_t d4 = vec ? d / 4 : 0;
  if (vec) {
    for (int64_t i = threadIdx.x; i < d4; i += RSTAT_BS) {
      f32x4 v = in_f32x4(row + 4 * i);
      s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
    }
    for (int64_t i = d4 * 4 + threadIdx.x; i < d; i += RSTAT_BS) s += (double)in_f32(row[i]);
  } else {
    for (int64_t i = threadIdx.x; i < d; i += RSTAT_BS) s += (double)in_f32(row[i]);
  }
  s = block_sum_f64(s, lds);
  const float m = (float)(s / (double)d);
  double q = 0;
  if (vec) {
    for (int64_t i = threadIdx.x; i < d4; i += RSTAT_BS) {
      f32x4 v = in_f32x4(row + 4 * i);
      f32x4 c = {v.x - m, v.y - m, v.z - m, v.w - m};
      q += (double)(c.x * c.x) + (double)(c.y * c.y) + (double)(c.z * c.z) + (double)(c.w * c.w);
      split_store4(prow, i, c);
    }
    for (int64_t i = d4 * 4 + threadIdx.x; i < d; i += RSTAT_BS) {
      float a = in_f32(row[i]) - m;
      q += (double)(a * a);
    }
    for (int64_t k = d4 * 4 + threadIdx.x; k < kp; k += RSTAT_BS)  // tail and k padding
      split_store1(prow, k, k < d ? in_f32(row[k]) - m : 0.f);
  } else {
    for (int64_t k = threadIdx.x; k < kp; k += RSTAT_BS) {
      float a = 0.f;
      if (k < d) {
        a = in_f32(row[k]) - m;
        q += (double)(a * a);
      }
      split_store1(prow, k, a);
    }
  }
  q = block_sum_f64(q, lds);
  if (threadIdx.x == 0) {
    float var = (float)(q / (double)d);
    float sd = sqrtf(var + correction);
    if (sd < correction * 10.0f) sd = 1.0f;  // rsa.py:84-87 zero-variance guard
    mean[r] = m;
    stdv[r] = sd;
  }
}

template <typename T>
__global__ __launch_bounds__(RSTAT_BS) void k_stats_split(const T* __restrict__ X, int64_t n, int64_t d,
                                                          int64_t ldx, int64_t nstage, float correction, int vec,
                                                          float* __restrict__ mean, float* __restrict__ stdv,
                                                          uint16_t* __restrict__ planes) {
  __shared__ double lds[RSTAT_BS / 64 + 1];
  stats_split_row<T>(X, n, d, ldx, nstage, correction, vec, mean, stdv, planes, blockIdx.x, lds);
}

// The same rows of several points in one launch (blockIdx.y = point): a bench extraction
// batch's hooked outputs split together, so the launch holds rows x points blocks.
constexpr int SPLIT_MULTI_MAX = 32;
struct SplitMulti {
  const float* X[SPLIT_MULTI_MAX];
  float* mean[SPLIT_MULTI_MAX];
  float* stdv[SPLIT_MULTI_MAX];
  uint16_t* planes[SPLIT_MULTI_MAX];
  int64_t d[SPLIT_MULTI_MAX];
  int64_t ldx[SPLIT_MULTI_MAX];
  int vec[SPLIT_MULTI_MAX];
};

__global__ __launch_bounds__(RSTAT_BS) void k_stats_split_multi(SplitMulti S, int64_t rows, float correction) {
  __shared__ double lds[RSTAT_BS / 64 + 1];
  const int p = blockIdx.y;
  stats_split_row<float>(S.X[p], rows, S.d[p], S.ldx[p], (S.d[p] + GK - 1) / GK, correction, S.vec[p], S.mean[p],
                         S.stdv[p], S.planes[p], blockIdx.x, lds);
}

// One-product prepass (bf16 input, vr_rdm_pearson_bf16): the row statistics as
// stats_split_row computes them (fp64 sum -> fp32 mean; fp64 sum of squares of the
// fp32-centred values -> std with the zero-variance guard) and raw stage records: record st
// of a row holds its bf16 values k 64 st .. 64 st + 63 (exact zeros past d; rows >= n zero).
// bf16 x bf16 products are exact in fp32, so one MFMA product per k gives sum x_i x_j; the
// centring is the epilogue's rank-1 correction (rdm_value). That subtraction cancels digits
// when a row's mean is large against its spread: *flag is set when mean^2 > 4 var for some
// row, and the call then takes the split (centred hi/lo) records instead.
__global__ __launch_bounds__(RSTAT_BS) void k_stats_one(const uint16_t* __restrict__ X, int64_t n, int64_t d,
                                                        int64_t ldx, int64_t nstage1, float correction,
                                                        float* __restrict__ mean, float* __restrict__ stdv,
                                                        uint16_t* __restrict__ planes, uint32_t* __restrict__ flag) {
  __shared__ double lds[RSTAT_BS / 64 + 1];
  const int64_t r = blockIdx.x, kp = nstage1 * 64;
  uint16_t* prow = planes + r * kp;
  if (r >= n) {
    for (int64_t k = threadIdx.x; k < kp; k += RSTAT_BS) prow[k] = 0;
    return;
  }
  const uint16_t* row = X + r * ldx;
  double s = 0;
  for (int64_t k = threadIdx.x; k < kp; k += RSTAT_BS) {
    const uint16_t v = k < d ? row[k] : (uint16_t)0;
    prow[k] = v;
    if (k < d) s += (double)in_f32(v);
  }
  s = block_sum_f64(s, lds);
  const float m = (float)(s / (double)d);
  double q = 0;
  for (int64_t k = threadIdx.x; k < d; k += RSTAT_BS) {
    const float a = in_f32(row[k]) - m;
    q += (double)(a * a);
  }
  q = block_sum_f64(q, lds);
  if (threadIdx.x == 0) {
    const float var = (float)(q / (double)d);
    float sd = sqrtf(var + correction);
    if (sd < correction * 10.0f) sd = 1.0f;  // rsa.py:84-87 zero-variance guard
    mean[r] = m;
    stdv[r] = sd;
    if ((double)m * (double)m > 4.0 * (double)var) *flag = 1u;  // benign race: every writer stores 1
  }
}

template <typename T>
static int stats_split(const T* X, int64_t n, int64_t rows, int64_t d, int64_t ldx, float correction,
                       float* mean, float* stdv, uint16_t* planes, hipStream_t st) {
  const int vec = ((reinterpret_cast<uintptr_t>(X) & (sizeof(T) == 4 ? 15 : 7)) == 0) && ((ldx & 3) == 0);
  k_stats_split<T><<<(unsigned)rows, RSTAT_BS, 0, st>>>(X, n, d, ldx, (d + GK - 1) / GK, correction, vec, mean,
                                                          stdv, planes);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// this thread's 4 x 16 B of a panel's stage record block (128 rows x 128 B)
__device__ inline void load_rec(const GramParams& P, int64_t row0, int64_t st, u32x4 out[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int f = threadIdx.x + G_THREADS * s;
    const int r = f >> 3, c = f & 7;
    out[s] = *reinterpret_cast<const u32x4*>(P.planes + ((row0 + r) * P.nstage + st) * 64 + c * 8);
  }
}

__device__ inline void store_rec(uint16_t* lds, const u32x4 v[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int f = threadIdx.x + G_THREADS * s;
    const int r = f >> 3, c = f & 7;
    *reinterpret_cast<u32x4*>(lds + r * SROW + c * 8) = v[s];
  }
}

template <bool ONE>
__global__ __launch_bounds__(G_THREADS, 2) void k_gram3(GramParams P) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * S_STAGE];  // [buf][A/B]
  const int nwg = gridDim.x;
  const int id = P.blk0 + (int)xcd_remap(blockIdx.x, (uint32_t)nwg);
  const int ltile = id / P.splits, split = id % P.splits;
  int bi, bj;
  band_tile(ltile, P.tile0, P.tile_count, P.T, bi, bj);
  const bool diag = (bi == bj);
  const int64_t row0 = (int64_t)bi * GT, col0 = (int64_t)bj * GT;
  const int64_t k0 = (int64_t)split * P.kslice;
  const int64_t k1 = min(P.dk, k0 + P.kslice);
  const int64_t st0 = k0 / GK;
  const int ns = (int)((k1 - k0 + GK - 1) / GK);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  u32x4 ga[4], gb[4];
  if (ns > 0) {
    load_rec(P, row0, st0, ga);
    if (!diag) load_rec(P, col0, st0, gb);
    store_rec(lds, ga);
    if (!diag) store_rec(lds + S_STAGE, gb);
  }
  __syncthreads();

  for (int kt = 0; kt < ns; ++kt) {
    const int cur = kt & 1;
    const uint16_t* As = lds + cur * 2 * S_STAGE;
    const uint16_t* Bs = diag ? As : As + S_STAGE;
    const bool more = kt + 1 < ns;
    if (more) {  // lands under the MFMAs
      load_rec(P, row0, st0 + kt + 1, ga);
      if (!diag) load_rec(P, col0, st0 + kt + 1, gb);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {  // k-steps of 16: lane holds k = 16t + 8h + j
      bf16x8 aH[2], aL[2], bH[2], bL[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const uint16_t* ar = As + (wr * 64 + m * 32 + l32) * SROW + t * 16 + h * 8;
        const uint16_t* br = Bs + (wc * 64 + m * 32 + l32) * SROW + t * 16 + h * 8;
        aH[m] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(ar));
        aL[m] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(ar + 32));
        bH[m] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(br));
        bL[m] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(br + 32));
      }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
          acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH[m], bH[nn], acc[m][nn], 0, 0, 0);
      if constexpr (ONE) {  // the record's second half is k 32..63 of the raw row: one product more
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nn = 0; nn < 2; ++nn)
            acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL[m], bL[nn], acc[m][nn], 0, 0, 0);
      } else {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nn = 0; nn < 2; ++nn)
            acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH[m], bL[nn], acc[m][nn], 0, 0, 0);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nn = 0; nn < 2; ++nn)
            acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL[m], bH[nn], acc[m][nn], 0, 0, 0);
      }
    }
    if (more) {
      uint16_t* nxt = lds + (cur ^ 1) * 2 * S_STAGE;
      store_rec(nxt, ga);
      if (!diag) store_rec(nxt + S_STAGE, gb);
    }
    if (P.flush && more && (kt + 1) % P.flush == 0) {
      gram_flush<GT>(acc, P.fbuf + (size_t)blockIdx.x * GT * GT, wr * 64, wc * 64, kt + 1 == P.flush);
    }
    __syncthreads();
  }
  if (P.flush && ns > P.flush) gram_unflush<GT>(acc, P.fbuf + (size_t)blockIdx.x * GT * GT, wr * 64, wc * 64);
  gram_store(P, acc, row0, col0, diag, split, ltile);
}

// ------------------------------------------------------------------------------------
// Wide split Gram: 256 x 256 super-tiles (2 x 2 of the 128-tiles), 8 waves as 2 x 4, each
// wave 128 x 64 = 4 x 2 accumulators. Against k_gram3 it halves the global->LDS traffic
// and the LDS writes per FLOP and cuts LDS fragment reads per MFMA from 2/3 to 1/2
// (12 ds_read_b128 per 24 MFMAs per 16-k step). 147 KB of LDS: one block (8 waves) per CU.
// Super-tile rows [0, R) of the upper triangle; a diagonal super-tile computes its lower
// 128-tile too and writes only i <= j entries (mirrored), as the 128 kernel does.
// ------------------------------------------------------------------------------------
constexpr int WT = 256;               // super-tile edge
constexpr int W_THREADS = 512;        // 8 waves
constexpr int W_STAGE = WT * SROW;    // bf16 per panel per stage

__device__ inline void load_rec_w(const GramParams& P, int64_t row0, int64_t st, u32x4 out[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int f = threadIdx.x + W_THREADS * s;
    const int r = f >> 3, c = f & 7;
    out[s] = *reinterpret_cast<const u32x4*>(P.planes + ((row0 + r) * P.nstage + st) * 64 + c * 8);
  }
}

__device__ inline void store_rec_w(uint16_t* lds, const u32x4 v[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int f = threadIdx.x + W_THREADS * s;
    const int r = f >> 3, c = f & 7;
    *reinterpret_cast<u32x4*>(lds + r * SROW + c * 8) = v[s];
  }
}

// Epilogue of one wave's 128 x 64 block (4 x 2 accumulators of 32 x 32).
__device__ inline void gram_store_w(const GramParams& P, f32x16 (&acc)[4][2], int64_t row0,
                                    int64_t col0, bool diag) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3, h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn) {
      const int64_t j = col0 + wc * 64 + nn * 32 + l32;
      const float sj = (j < P.n) ? P.stdv[j] : 1.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t ib = row0 + wr * 128 + m * 32 + 8 * g + 4 * h;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t i = ib + e;
          const float si = (i < P.n) ? P.stdv[i] : 1.f;
          v[e] = rdm_value(acc[m][nn][4 * g + e], i, j, P, si, sj);
        }
        if (diag) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t i = ib + e;
            if (i <= j && j < P.n) {
              P.rdm[i * P.ldr + j] = v[e];
              if (i < j) P.rdm[j * P.ldr + i] = v[e];
            }
          }
          continue;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t i = ib + e;
          if (i < P.n && j < P.n) P.rdm[i * P.ldr + j] = v[e];
        }
        if (j < P.n) {
          float* dst = P.rdm + j * P.ldr + ib;
          if (P.vec && ib + 3 < P.n && ((P.ldr & 3) == 0)) {
            f32x4 w = {v[0], v[1], v[2], v[3]};
            *reinterpret_cast<f32x4*>(dst) = w;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (ib + e < P.n) dst[e] = v[e];
          }
        }
      }
    }
}

// Super-tile position p (row-major over super rows [0, R) of a T2 x T2 triangle).
__device__ inline void super_tile(int p, int T2, int& bi, int& bj) { tile_coords(p, T2, bi, bj); }

__global__ __launch_bounds__(W_THREADS, 1) void k_gram3w(GramParams P) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * W_STAGE];  // [buf][A/B]
  const int id = P.blk0 + (int)xcd_remap(blockIdx.x, (uint32_t)gridDim.x);
  int bi, bj;
  band_tile(id, P.tile0, P.tile_count, P.T, bi, bj);  // P.T = super-tiles per dimension here
  const bool diag = (bi == bj);
  const int64_t row0 = (int64_t)bi * WT, col0 = (int64_t)bj * WT;
  const int ns = (int)P.nstage;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3, h = lane >> 5, l32 = lane & 31;

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  u32x4 ga[4], gb[4];
  load_rec_w(P, row0, 0, ga);
  if (!diag) load_rec_w(P, col0, 0, gb);
  store_rec_w(lds, ga);
  if (!diag) store_rec_w(lds + W_STAGE, gb);
  __syncthreads();
  for (int kt = 0; kt < ns; ++kt) {
    const int cur = kt & 1;
    const uint16_t* As = lds + cur * 2 * W_STAGE;
    const uint16_t* Bs = diag ? As : As + W_STAGE;
    const bool more = kt + 1 < ns;
    if (more) {
      load_rec_w(P, row0, kt + 1, ga);
      if (!diag) load_rec_w(P, col0, kt + 1, gb);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16x8 aH[4], aL[4], bH[2], bL[2];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const uint16_t* ar = As + (wr * 128 + m * 32 + l32) * SROW + t * 16 + h * 8;
        aH[m] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(ar));
        aL[m] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(ar + 32));
      }
#pragma unroll
      for (int nn = 0; nn < 2; ++nn) {
        const uint16_t* br = Bs + (wc * 64 + nn * 32 + l32) * SROW + t * 16 + h * 8;
        bH[nn] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(br));
        bL[nn] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(br + 32));
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
          acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH[m], bH[nn], acc[m][nn], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
          acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aH[m], bL[nn], acc[m][nn], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
          acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aL[m], bH[nn], acc[m][nn], 0, 0, 0);
    }
    if (more) {
      uint16_t* nxt = lds + (cur ^ 1) * 2 * W_STAGE;
      store_rec_w(nxt, ga);
      if (!diag) store_rec_w(nxt + W_STAGE, gb);
    }
    if (P.flush && more && (kt + 1) % P.flush == 0) {
      gram_flush<WT>(acc, P.fbuf + (size_t)blockIdx.x * WT * WT, wr * 128, wc * 64, kt + 1 == P.flush);
    }
    __syncthreads();
  }
  if (P.flush && ns > P.flush) gram_unflush<WT>(acc, P.fbuf + (size_t)blockIdx.x * WT * WT, wr * 128, wc * 64);
  gram_store_w(P, acc, row0, col0, diag);
}

// ------------------------------------------------------------------------------------
// Pipelined wide split Gram (default for full RDMs): k_gram3w's 256 x 256 super-tiles and
// 8-wave 2 x 4 decomposition, with the panels moved global -> LDS by global_load_lds
// (16 B per lane, no register staging) in 16-k sub-stages: a sub-stage is, per row, the
// 64 bytes [hi k0..15 | lo k0..15] of a 32-k record (two 32-B pieces), 16 KB per panel.
// Four sub-stage slots (A + B = 32 KB each, 128 KB of LDS): while sub-stage q is consumed
// (24 MFMAs per wave), q+1 and q+2 are in flight and q+3 is issued into the slot q-1 used.
// Each wave waits only for its own loads of q (counted vmcnt: the loads of q+1 and q+2
// stay in flight) and then a raw s_barrier, after which every wave's part of q has landed;
// the slot rewritten by q+3 was last read in iteration q-1, before that barrier. The LDS
// image is lane-linear per wave-instruction (16 rows x 64 B); 16-B chunk j of row r sits
// at chunk j ^ ((r >> 2) & 3), applied on the global source address, so a fragment read
// (32 rows, one chunk) touches 16 distinct 16-B bank slots per 16 lanes.
// ------------------------------------------------------------------------------------
#ifndef VR_GRAM_PRIO
#define VR_GRAM_PRIO 0  // 1: raise the wave priority over its MFMA block (A/B)
#endif
constexpr int P_PANEL = WT * 64;       // bytes of one panel sub-stage
constexpr int P_SLOT = 2 * P_PANEL;    // A + B
#ifndef VR_GRAM_SLOTS
#define VR_GRAM_SLOTS 4  // sub-stage slots in LDS (5: 160 KB, one more sub-stage in flight; A/B)
#endif
constexpr int P_SLOTS = VR_GRAM_SLOTS;
constexpr int P_AHEAD = P_SLOTS - 1;  // iteration q issues sub-stage q + P_AHEAD

// this wave's two 1-KB pieces (16 rows each) of a panel sub-stage: rows [16 (2 w + i), +16)
__device__ inline void p_issue(const GramParams& P, char* panel, int64_t row0, int q) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t st = q >> 1;
  const int t = q & 1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rbase = (wid * 2 + i) * 16;
    const int r = rbase + (lane >> 2);
    const int j = (lane & 3) ^ ((r >> 2) & 3);  // the logical chunk this lane's slot holds
    const int off = ((j & 2) << 5) + 32 * t + ((j & 1) << 4);
    const char* src = reinterpret_cast<const char*>(P.planes) + ((row0 + r) * P.nstage + st) * 128 + off;
    __builtin_amdgcn_global_load_lds(src, panel + rbase * 64, 16, 0, 0);
  }
}

// one 1-KB piece (i = 0, 1) of p_issue
__device__ inline void p_issue1(const GramParams& P, char* panel, int64_t row0, int q, int i) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t st = q >> 1;
  const int t = q & 1;
  const int rbase = (wid * 2 + i) * 16;
  const int r = rbase + (lane >> 2);
  const int j = (lane & 3) ^ ((r >> 2) & 3);
  const int off = ((j & 2) << 5) + 32 * t + ((j & 1) << 4);
  const char* src = reinterpret_cast<const char*>(P.planes) + ((row0 + r) * P.nstage + st) * 128 + off;
  __builtin_amdgcn_global_load_lds(src, panel + rbase * 64, 16, 0, 0);
}

__device__ inline bf16x8 p_frag(const char* panel, int row, int j) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(panel + row * 64 + ((j ^ ((row >> 2) & 3)) << 4)));
}

template <int N>
__device__ inline void p_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct PFrag {
  bf16x8 aH[4], aL[4], bH[2], bL[2];
};

__device__ inline void p_read(const char* As, const char* Bs, PFrag& f) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3, h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int r = wr * 128 + m * 32 + l32;
    f.aH[m] = p_frag(As, r, h);
    f.aL[m] = p_frag(As, r, 2 + h);
  }
#pragma unroll
  for (int nn = 0; nn < 2; ++nn) {
    const int r = wc * 64 + nn * 32 + l32;
    f.bH[nn] = p_frag(Bs, r, h);
    f.bL[nn] = p_frag(Bs, r, 2 + h);
  }
}

#ifndef VR_GRAM_ILV
#define VR_GRAM_ILV 0  // 1: the next sub-stage's LDS-DMA pieces issued between the MFMAs (A/B)
#endif

// p_mfma with callback g(k) after the 6k-th MFMA (k = 1..3): the same MFMA order
template <typename G>
__device__ inline void p_mfma_ilv(const PFrag& f, f32x16 (&acc)[4][2], G&& g) {
  int c = 0;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn) {
      acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.aH[m], f.bH[nn], acc[m][nn], 0, 0, 0);
      if (++c % 6 == 0) g(c / 6);
    }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn) {
      acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.aH[m], f.bL[nn], acc[m][nn], 0, 0, 0);
      if (++c % 6 == 0) g(c / 6);
    }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn) {
      acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.aL[m], f.bH[nn], acc[m][nn], 0, 0, 0);
      if (++c % 6 == 0) g(c / 6);
    }
}

__device__ inline void p_mfma(const PFrag& f, f32x16 (&acc)[4][2]) {
#if VR_GRAM_PRIO
  __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
      acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.aH[m], f.bH[nn], acc[m][nn], 0, 0, 0);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
      acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.aH[m], f.bL[nn], acc[m][nn], 0, 0, 0);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
      acc[m][nn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.aL[m], f.bH[nn], acc[m][nn], 0, 0, 0);
#if VR_GRAM_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
}

// Iteration q: sub-stage q's fragments are already in registers (cur); wait for this wave's
// loads of q+1 (q+2 stays in flight), barrier, issue q+3 into the slot sub-stage q-1 used,
// start the LDS reads of q+1 into nxt, then the 24 MFMAs of q, which do not wait for them.
template <bool DIAG>
__device__ inline void gram3p_step(const GramParams& P, char* lds, int64_t row0, int64_t col0, int q, int Q,
                                   const PFrag& cur, PFrag& nxt, f32x16 (&acc)[4][2]) {
  constexpr int PER = DIAG ? 2 : 4;  // glds per wave per sub-stage
  if (q + 1 < Q) {
    // this wave's loads of q+1 done; those of q+2 .. q+P_AHEAD-1 (issued) may stay in flight
    const int left = Q - 2 - q;
    if (P_AHEAD >= 4 && left >= 2)
      p_wait<(P_AHEAD >= 4 ? 2 : 1) * PER>();
    else if (left >= 1)
      p_wait<PER>();
    else
      p_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (!VR_GRAM_ILV && q + P_AHEAD < Q) {
      char* slot = lds + ((q + P_AHEAD) % P_SLOTS) * P_SLOT;
      p_issue(P, slot, row0, q + P_AHEAD);
      if (!DIAG) p_issue(P, slot + P_PANEL, col0, q + P_AHEAD);
    }
    const char* As = lds + ((q + 1) % P_SLOTS) * P_SLOT;
    p_read(As, DIAG ? As : As + P_PANEL, nxt);
  }
  if constexpr (VR_GRAM_ILV) {
    // the slot of q+3 was last read in iteration q-1, before this iteration's barrier; the
    // pieces are in flight before the next iteration's counted wait either way
    static_assert(!VR_GRAM_ILV || P_AHEAD == 3, "interleaved issue: 4 slots");
    const bool more = q + 3 < Q;
    char* slot = lds + ((q + 3) % P_SLOTS) * P_SLOT;
    p_mfma_ilv(cur, acc, [&](int k) {
      if (!more) return;
      if (DIAG) {
        if (k <= 2) p_issue1(P, slot, row0, q + 3, k - 1);
      } else {
        if (k == 1) p_issue1(P, slot, row0, q + 3, 0);
        if (k == 2) {
          p_issue1(P, slot, row0, q + 3, 1);
          p_issue1(P, slot + P_PANEL, col0, q + 3, 0);
        }
        if (k == 3) p_issue1(P, slot + P_PANEL, col0, q + 3, 1);
      }
    });
  } else {
    p_mfma(cur, acc);
  }
  // every P.flush stages (the same two-level sum as k_gram3w); its global loads and stores
  // drain this wave's loads in flight (the compiler waits vmcnt(0)): correct, and rare
  if (P.flush && (q & 1) && q + 1 < Q && ((q >> 1) + 1) % P.flush == 0) {
    const int wid = threadIdx.x >> 6;
    gram_flush<WT>(acc, P.fbuf + (size_t)blockIdx.x * WT * WT, (wid >> 2) * 128, (wid & 3) * 64,
                   (q >> 1) + 1 == P.flush);
  }
}

template <bool DIAG>
__device__ inline void gram3p_loop(const GramParams& P, char* lds, int64_t row0, int64_t col0, int ns,
                                   f32x16 (&acc)[4][2]) {
  const int Q = 2 * ns;  // even
  constexpr int PER = DIAG ? 2 : 4;
  for (int q = 0; q < P_AHEAD && q < Q; ++q) {
    char* slot = lds + q * P_SLOT;
    p_issue(P, slot, row0, q);
    if (!DIAG) p_issue(P, slot + P_PANEL, col0, q);
  }
  // sub-stage 0 landed: the loads of 1 .. P_AHEAD-1 may stay in flight
  if (P_AHEAD >= 4 && Q > 3)
    p_wait<(P_AHEAD >= 4 ? 3 : 2) * PER>();
  else if (Q > 2)
    p_wait<2 * PER>();
  else if (Q > 1)
    p_wait<PER>();
  else
    p_wait<0>();
  __builtin_amdgcn_s_barrier();
  PFrag f0, f1;
  p_read(lds, DIAG ? lds : lds + P_PANEL, f0);
  for (int q = 0; q < Q; q += 2) {  // two sub-stages per trip: the fragment sets swap roles
    gram3p_step<DIAG>(P, lds, row0, col0, q, Q, f0, f1, acc);
    gram3p_step<DIAG>(P, lds, row0, col0, q + 1, Q, f1, f0, acc);
  }
}

// Split-K partial of one wave's 128 x 64 block: fp32 [split][super-tile][256 x 256]
__device__ inline void gram_partial_w(const GramParams& P, f32x16 (&acc)[4][2], int split, int ltile) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3, h = lane >> 5, l32 = lane & 31;
  float* out = P.partial + ((int64_t)split * P.tile_count + ltile) * (WT * WT);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn) {
      const int lj = wc * 64 + nn * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int li = wr * 128 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[li * WT + lj] = acc[m][nn][r];
      }
    }
}

// Launch position id -> (super-tile, k split): split-major, so the blocks an XCD holds at
// once are neighbouring tiles of one k range (shared panels in its L2). Split s covers
// stages [s kslice / GK, min(nstage, (s + 1) kslice / GK)); one split: the whole depth.
__global__ __launch_bounds__(W_THREADS, 1) void k_gram3p(GramParams P) {
  __shared__ __attribute__((aligned(16))) char lds[P_SLOTS * P_SLOT];
  const int id = P.blk0 + (int)xcd_remap(blockIdx.x, (uint32_t)gridDim.x);
  const int split = id / P.tile_count, ltile = id % P.tile_count;
  int bi, bj;
  band_tile(ltile, P.tile0, P.tile_count, P.T, bi, bj);  // P.T = super-tiles per dimension here
  const bool diag = (bi == bj);
  const int64_t row0 = (int64_t)bi * WT, col0 = (int64_t)bj * WT;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  (void)lane;
  const int64_t sper = P.kslice / GK;  // stages per split
  const int64_t st0 = (int64_t)split * sper;
  const int ns = (int)(P.nstage - st0 < sper ? P.nstage - st0 : sper);
  GramParams S = P;
  S.planes = P.planes + st0 * 64;  // records of stage st0 onwards (the row stride stays nstage)
  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  if (diag)
    gram3p_loop<true>(S, lds, row0, col0, ns, acc);
  else
    gram3p_loop<false>(S, lds, row0, col0, ns, acc);
  if (P.flush && ns > P.flush)
    gram_unflush<WT>(acc, P.fbuf + (size_t)blockIdx.x * WT * WT, wr * 128, wc * 64);
  if (P.splits == 1)
    gram_store_w(P, acc, row0, col0, diag);
  else
    gram_partial_w(P, acc, split, ltile);
}

// Sums the split partials of one super-tile in split order and applies the epilogue
// (k_gram_reduce for 256-tiles): block (t, strip) handles rows [32 strip, +32) of
// super-tile t; a diagonal super-tile takes (i, j) and (j, i) from one partial entry.
__global__ __launch_bounds__(256) void k_gram_reduce_w(GramParams P) {
  __shared__ float tr[32][33];
  const int ltile = blockIdx.x;
  int bi, bj;
  band_tile(ltile, P.tile0, P.tile_count, P.T, bi, bj);
  const bool diag = (bi == bj);
  const int64_t row0 = (int64_t)bi * WT, col0 = (int64_t)bj * WT;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const int si0 = blockIdx.y * 32;
  for (int sj0 = 0; sj0 < WT; sj0 += 32) {
    for (int yy = ty; yy < 32; yy += 8) {
      const int li = si0 + yy, lj = sj0 + tx;
      const int pi = (diag && li > lj) ? lj : li, pj = (diag && li > lj) ? li : lj;
      float g = 0.f;
      for (int s = 0; s < P.splits; ++s)
        g += P.partial[((int64_t)s * P.tile_count + ltile) * (WT * WT) + pi * WT + pj];
      const int64_t i = row0 + li, j = col0 + lj;
      const float sI = (i < P.n) ? P.stdv[i] : 1.f, sJ = (j < P.n) ? P.stdv[j] : 1.f;
      const float v = rdm_value(g, i, j, P, sI, sJ);
      if (i < P.n && j < P.n) P.rdm[i * P.ldr + j] = v;
      tr[yy][tx] = v;
    }
    __syncthreads();
    if (!diag) {
      for (int yy = ty; yy < 32; yy += 8) {
        const int64_t j = col0 + sj0 + yy, i = row0 + si0 + tx;
        if (i < P.n && j < P.n) P.rdm[j * P.ldr + i] = tr[tx][yy];
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------
// Phased wide split Gram on v_mfma_f32_16x16x32_bf16 (k_gram3e, VISREPS_GRAM_KERNEL=e).
// The same 256 x 256 super-tiles, 8 waves as 2 x 4 and 128 x 64 wave tiles as k_gram3p,
// the same three products per k, but whole 32-k stage records in LDS (one 128-B record
// per row) and the 16 x 16 MFMA shape, which the chip clocks higher than 32 x 32 under
// load (MI355X_MICROARCH.md, DVFS give-back item 7).
// A stage is four 16-KB half-tiles (A rows 0-127 / 128-255, B the same), two stages
// double-buffered (128 KB). A wave's 128 x 64 block is four quadrants (64-row half a0/a1
// of its rows x 32-column half b0/b1): one phase per quadrant, 24 MFMAs each, in the
// order (a0,b0) (a0,b1) (a1,b1) (a1,b0). Each phase first issues the LDS reads of the
// fragments the NEXT phase needs (registers AX/AY for the A halves, BP/BQ for the B
// halves: 96 VGPRs), then its MFMAs, which use fragments read one phase earlier:
//   P0(t): MFMA a0 b0; read b1(t)        P1(t): MFMA a0 b1; read a1(t)
//   P2(t): MFMA a1 b1; read a0(t+1)      P3(t): MFMA a1 b0; read b0(t+1)
// One half-tile is staged per phase by LDS-DMA (two 1-KB pieces per wave):
//   P0(t): A-bot(t+1)   P1(t): B-right(t+1)   P2(t): B-left(t+2)   P3(t): A-top(t+2)
// so a buffer is restaged >= 2 phases after its last read (the reads of phase p are
// consumed by phase p+1's MFMAs, which every wave has passed at phase p+2's barrier), and
// each wave waits (counted vmcnt) before the barrier of the phase that first reads a
// stage: P2(t) for the A halves of t+1 (B-right(t+1) may stay in flight), P3(t) for the B
// halves (B-left(t+2) may). Diagonal super-tiles stage and read the A halves only.
// LDS image of a half-tile: row r's 16-B chunk c at r * 128 + (c ^ ((r >> 1) & 7)) * 16;
// a fragment read (16 rows of a 16-row block, one chunk per 16 lanes) then touches 16
// distinct 16-B bank slots in each ds_read_b128 lane group.
// ------------------------------------------------------------------------------------
constexpr int E_HALF = 128 * 128;    // bytes of a half-tile stage (128 rows x 128 B)
constexpr int E_STAGE = 4 * E_HALF;  // A-top, A-bot, B-left, B-right

// this wave's two 1-KB pieces (rows [16 wid, +16)) of half-tile h (0/1: A rows 0-127 /
// 128-255 of the super-tile, 2/3: B) of stage st into the stage buffer sb. The lane part
// of the source address (row rr of the half-tile, logical chunk c) is the same for every
// half-tile and stage: a 32-bit offset computed once (e_issue_off); the rest is uniform.
__device__ inline uint32_t e_issue_off(const GramParams& P, int k) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rr = wid * 16 + k * 8 + (lane >> 3);
  const int c = (lane & 7) ^ ((rr >> 1) & 7);  // the logical chunk this lane's slot holds
  return (uint32_t)rr * (uint32_t)P.nstage * 128u + (uint32_t)c * 16u;
}
__device__ inline void e_issue(const GramParams& P, char* sb, int h, int64_t row0, int64_t col0, int64_t st,
                               const uint32_t (&io)[2]) {
  const int wid = threadIdx.x >> 6;
  const int64_t rbase = (h < 2 ? row0 : col0) + (h & 1) * 128;
  const char* base = reinterpret_cast<const char*>(P.planes) + (rbase * P.nstage + st) * 128;
  char* half = sb + h * E_HALF;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    uint32_t off = io[k];
    asm volatile("" : "+v"(off));  // formed here: no 64-bit address per half-tile hoisted out of the loop
    __builtin_amdgcn_global_load_lds(base + off, half + (wid * 16 + k * 8) * 128, 16, 0, 0);
  }
}

struct EFragA {
  bf16x8 hi[4], lo[4];  // 4 row blocks of 16
};
struct EFragB {
  bf16x8 hi[2], lo[2];  // 2 column blocks of 16
};

// rows r0 + 16 m + (lane & 15) of a half-tile (r0 a multiple of 16); lane group
// g = lane >> 4 holds k 8g..8g+7. The swizzle term of a row depends only on lane & 15, so
// every read is this lane's constant offset (hi or lo chunk) plus a uniform immediate.
struct ELane {
  uint32_t hi, lo;  // byte offsets of this lane's hi / lo chunk in its row of a 16-row block
};
__device__ inline ELane e_lane() {
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15, swz = (l16 >> 1) & 7;
  return ELane{(uint32_t)(l16 * 128 + ((g ^ swz) << 4)), (uint32_t)(l16 * 128 + (((4 + g) ^ swz) << 4))};
}
__device__ inline void e_read_a(const char* half, int r0, const ELane& o, EFragA& f) {
  uint32_t ohi = o.hi, olo = o.lo;  // opaque per call: the read addresses are formed here
  asm volatile("" : "+v"(ohi), "+v"(olo));
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const char* row = half + (r0 + m * 16) * 128;
    f.hi[m] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(row + ohi));
    f.lo[m] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(row + olo));
  }
}
__device__ inline void e_read_b(const char* half, int r0, const ELane& o, EFragB& f) {
  uint32_t ohi = o.hi, olo = o.lo;  // opaque per call: the read addresses are formed here
  asm volatile("" : "+v"(ohi), "+v"(olo));
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const char* row = half + (r0 + n * 16) * 128;
    f.hi[n] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(row + ohi));
    f.lo[n] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(row + olo));
  }
}

#ifndef VR_E_PRIO
#define VR_E_PRIO 0  // 1: s_setprio(1) over each phase's MFMAs (A/B)
#endif
// quadrant (MA, NB) of the wave's block: 4 x 2 tiles of 16 x 16, hh, hl, lh products
// ONE (bf16 input, raw records of 64 k): hi = k 0..31, lo = k 32..63 of the stage, 2 products
template <int MA, int NB, bool ONE>
__device__ inline void e_mfma(const EFragA& a, const EFragB& b, f32x4 (&acc)[8][4]) {
#if VR_E_PRIO
  __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
      acc[MA * 4 + m][NB * 2 + n] =
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi[m], b.hi[n], acc[MA * 4 + m][NB * 2 + n], 0, 0, 0);
  if constexpr (ONE) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        acc[MA * 4 + m][NB * 2 + n] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo[m], b.lo[n], acc[MA * 4 + m][NB * 2 + n], 0, 0, 0);
#if VR_E_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    return;
  }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
      acc[MA * 4 + m][NB * 2 + n] =
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi[m], b.lo[n], acc[MA * 4 + m][NB * 2 + n], 0, 0, 0);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
      acc[MA * 4 + m][NB * 2 + n] =
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo[m], b.hi[n], acc[MA * 4 + m][NB * 2 + n], 0, 0, 0);
#if VR_E_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
}

// 16 x 16 C/D map: col = lane & 15, row = 4 (lane >> 4) + e. Flush buffer: the block's
// 256 x 256 fp32 tile (k_gram3p's two-level sum, same interval).
__device__ inline float* e_flush_base(float* buf) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t off = (uint32_t)(((wid >> 2) * 128 + 4 * (lane >> 4)) * WT + (wid & 3) * 64 + (lane & 15));
  asm volatile("" : "+v"(off));
  return buf + off;
}
__device__ inline void e_flush(f32x4 (&acc)[8][4], float* buf, bool first) {
  float* b = e_flush_base(buf);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float* p = b + (i * 16 + e) * WT + j * 16;
        *p = first ? acc[i][j][e] : *p + acc[i][j][e];
        acc[i][j][e] = 0.f;
      }
}
__device__ inline void e_unflush(f32x4 (&acc)[8][4], const float* buf) {
  const float* b = e_flush_base(const_cast<float*>(buf));
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[i][j][e] += b[(i * 16 + e) * WT + j * 16];
}

// Epilogue of the wave's 128 x 64 block (8 x 4 tiles of 16 x 16), as gram_store_w: a
// diagonal super-tile writes each i < j entry from its (i, j) accumulator to both places.
template <bool ONE>
__device__ inline void e_store(const GramParams& P, f32x4 (&acc)[8][4], int64_t row0, int64_t col0, bool diag) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3, g = lane >> 4, l16 = lane & 15;
#pragma unroll
  for (int j4 = 0; j4 < 4; ++j4) {
    const int64_t j = col0 + wc * 64 + j4 * 16 + l16;
    const float sj = (j < P.n) ? P.stdv[j] : 1.f;
#pragma unroll
    for (int i8 = 0; i8 < 8; ++i8) {
      const int64_t ib = row0 + wr * 128 + i8 * 16 + 4 * g;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t i = ib + e;
        const float si = (i < P.n) ? P.stdv[i] : 1.f;
        v[e] = rdm_value_t<ONE>(acc[i8][j4][e], i, j, P, si, sj);
      }
      if (diag) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t i = ib + e;
          if (i <= j && j < P.n) {
            P.rdm[i * P.ldr + j] = v[e];
            if (i < j) P.rdm[j * P.ldr + i] = v[e];
          }
        }
        continue;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t i = ib + e;
        if (i < P.n && j < P.n) P.rdm[i * P.ldr + j] = v[e];
      }
      if (j < P.n) {
        float* dst = P.rdm + j * P.ldr + ib;
        if (P.vec && ib + 3 < P.n && ((P.ldr & 3) == 0)) {
          f32x4 w = {v[0], v[1], v[2], v[3]};
          *reinterpret_cast<f32x4*>(dst) = w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (ib + e < P.n) dst[e] = v[e];
        }
      }
    }
  }
}

// One stage t of the phase loop. ODD selects the B register roles: in even stages b0
// arrives in BP and b1 in BQ, in odd stages the other way round (see above).
// s_barrier plus a compiler fence: no LDS read or LDS-DMA issue moves across it
__device__ inline void e_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <bool DIAG, bool ODD, bool ONE>
__device__ inline void e_stage(const GramParams& P, char* lds, int64_t row0, int64_t col0, int t, int ns,
                               const ELane& o, const uint32_t (&io)[2], EFragA& AX, EFragA& AY,
                               EFragB& BP, EFragB& BQ, f32x4 (&acc)[8][4]) {
  const int wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  EFragB& B0 = ODD ? BQ : BP;  // b0 of this stage
  EFragB& B1 = ODD ? BP : BQ;  // b1 of this stage, then b0 of the next
  char* cur = lds + (t & 1) * E_STAGE;
  char* nxt = lds + ((t + 1) & 1) * E_STAGE;
  const int ha = wr, hb = DIAG ? (wc >> 1) : 2 + (wc >> 1);  // this wave's A / B half-tiles
  const int rb = (wc & 1) * 64;                               // its 64 columns inside hb
  const bool more1 = t + 1 < ns, more2 = t + 2 < ns;
  // P0: MFMA a0 b0; read b1(t); stage A-bot(t+1)
  e_barrier();
  if (more1) e_issue(P, nxt, 1, row0, col0, t + 1, io);
  e_read_b(cur + hb * E_HALF, rb + 32, o, B1);
  e_mfma<0, 0, ONE>(AX, B0, acc);
  // P1: MFMA a0 b1; read a1(t); stage B-right(t+1)
  e_barrier();
  if (!DIAG && more1) e_issue(P, nxt, 3, row0, col0, t + 1, io);
  e_read_a(cur + ha * E_HALF, 64, o, AY);
  e_mfma<0, 1, ONE>(AX, B1, acc);
  // P2: MFMA a1 b1; read a0(t+1) (wait for the A halves of t+1); stage B-left(t+2)
  if (more1) {
    if (DIAG)
      p_wait<0>();
    else
      p_wait<2>();
  }
  e_barrier();
  if (!DIAG && more2) e_issue(P, cur, 2, row0, col0, t + 2, io);
  if (more1) e_read_a(nxt + ha * E_HALF, 0, o, AX);
  e_mfma<1, 1, ONE>(AY, B1, acc);
  // P3: MFMA a1 b0; read b0(t+1) into B1's registers (wait for the B halves of t+1);
  // stage A-top(t+2)
  if (!DIAG && more1) {
    if (more2)
      p_wait<2>();
    else
      p_wait<0>();
  }
  e_barrier();
  if (more2) e_issue(P, cur, 0, row0, col0, t + 2, io);
  if (more1) e_read_b(nxt + hb * E_HALF, rb, o, B1);
  e_mfma<1, 0, ONE>(AY, B0, acc);
  if (P.flush && more1 && (t + 1) % P.flush == 0) e_flush(acc, P.fbuf + (size_t)blockIdx.x * WT * WT, t + 1 == P.flush);
}

template <bool DIAG, bool ONE>
__device__ inline void e_loop(const GramParams& P, char* lds, int64_t row0, int64_t col0, int ns,
                              f32x4 (&acc)[8][4]) {
  const int wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int ha = wr, hb = DIAG ? (wc >> 1) : 2 + (wc >> 1), rb = (wc & 1) * 64;
  const uint32_t io[2] = {e_issue_off(P, 0), e_issue_off(P, 1)};
  // prologue: stage 0 whole, and stage 1's first two half-tiles (B-left, A-top), in the
  // order the loop issues them
  e_issue(P, lds, 0, row0, col0, 0, io);
  e_issue(P, lds, 1, row0, col0, 0, io);
  if (!DIAG) {
    e_issue(P, lds, 2, row0, col0, 0, io);
    e_issue(P, lds, 3, row0, col0, 0, io);
  }
  if (ns > 1) {
    if (!DIAG) e_issue(P, lds + E_STAGE, 2, row0, col0, 1, io);
    e_issue(P, lds + E_STAGE, 0, row0, col0, 1, io);
    if (DIAG)
      p_wait<2>();
    else
      p_wait<4>();
  } else {
    p_wait<0>();
  }
  e_barrier();
  const ELane o = e_lane();
  EFragA AX, AY;
  EFragB BP, BQ;
  e_read_a(lds + ha * E_HALF, 0, o, AX);
  e_read_b(lds + hb * E_HALF, rb, o, BP);
  for (int t = 0; t < ns; t += 2) {
    e_stage<DIAG, false, ONE>(P, lds, row0, col0, t, ns, o, io, AX, AY, BP, BQ, acc);
    if (t + 1 < ns) e_stage<DIAG, true, ONE>(P, lds, row0, col0, t + 1, ns, o, io, AX, AY, BP, BQ, acc);
  }
}

// Split-K partial of the wave's block: fp32 [split][super-tile][256 x 256] (k_gram_reduce_w)
__device__ inline void e_partial(const GramParams& P, f32x4 (&acc)[8][4], int split, int ltile) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3, g = lane >> 4, l16 = lane & 15;
  float* out = P.partial + ((int64_t)split * P.tile_count + ltile) * (WT * WT);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) out[(wr * 128 + i * 16 + 4 * g + e) * WT + wc * 64 + j * 16 + l16] = acc[i][j][e];
}

// Launch position id -> (super-tile, k split) as k_gram3p: split-major; one split = the
// whole depth (P.kslice = nstage * GK).
template <bool ONE>
__global__ __launch_bounds__(W_THREADS, 1) void k_gram3e(GramParams P) {
  __shared__ __attribute__((aligned(16))) char lds[2 * E_STAGE];
  const int id = P.blk0 + (int)xcd_remap(blockIdx.x, (uint32_t)gridDim.x);
  const int split = id / P.tile_count, ltile = id % P.tile_count;
  int bi, bj;
  band_tile(ltile, P.tile0, P.tile_count, P.T, bi, bj);  // P.T = super-tiles per dimension
  const bool diag = (bi == bj);
  const int64_t row0 = (int64_t)bi * WT, col0 = (int64_t)bj * WT;
  const int64_t sper = P.kslice / GK;  // stages per split
  const int64_t st0 = (int64_t)split * sper;
  const int ns = (int)(P.nstage - st0 < sper ? P.nstage - st0 : sper);
  GramParams S = P;
  S.planes = P.planes + st0 * 64;  // records of stage st0 onwards (the row stride stays nstage)
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (diag)
    e_loop<true, ONE>(S, lds, row0, col0, ns, acc);
  else
    e_loop<false, ONE>(S, lds, row0, col0, ns, acc);
  if (P.flush && ns > P.flush) e_unflush(acc, P.fbuf + (size_t)blockIdx.x * WT * WT);
  if (P.splits == 1)
    e_store<ONE>(P, acc, row0, col0, diag);
  else
    e_partial(P, acc, split, ltile);
}

// The full-depth wide launches run k_gram3e (measured +3.5-8.5 % over k_gram3p on whole
// RDMs at N = 10k, profiles/r3_gram_ab.log); VISREPS_GRAM_KERNEL=p selects k_gram3p (A/B).
static bool env_flag(const char* name, bool dflt) {
  const char* e = getenv(name);
  return e && *e ? strcmp(e, "0") != 0 : dflt;
}

static bool gram_phased() {
  const char* e = getenv("VISREPS_GRAM_KERNEL");
  return !(e && strcmp(e, "p") == 0);
}

// VISREPS_GRAM_PIPE=0: the register-staged k_gram3w (A/B timing)
static bool gram_pipe() {
  const char* e = getenv("VISREPS_GRAM_PIPE");
  return !(e && strcmp(e, "0") == 0);
}

// Sums the split partials of one tile in split order and applies the epilogue; the
// mirror half goes through an LDS transpose so both writes are row-coalesced.
__global__ __launch_bounds__(256) void k_gram_reduce(GramParams P) {
  __shared__ float tr[32][33];
  const int ltile = blockIdx.x;
  int bi, bj;
  band_tile(ltile, P.tile0, P.tile_count, P.T, bi, bj);
  const bool diag = (bi == bj);
  const int64_t row0 = (int64_t)bi * GT, col0 = (int64_t)bj * GT;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int sb = 0; sb < (GT / 32) * (GT / 32); ++sb) {
    const int si0 = (sb / (GT / 32)) * 32, sj0 = (sb % (GT / 32)) * 32;
    for (int yy = ty; yy < 32; yy += 8) {
      const int li = si0 + yy, lj = sj0 + tx;
      float g = 0.f;
      // a diagonal tile takes (i, j) and (j, i) from one accumulator: exact symmetry
      const int pi = (diag && li > lj) ? lj : li, pj = (diag && li > lj) ? li : lj;
      for (int s = 0; s < P.splits; ++s)
        g += P.partial[((int64_t)s * P.tile_count + ltile) * (GT * GT) + pi * GT + pj];
      const int64_t i = row0 + li, j = col0 + lj;
      const float sI = (i < P.n) ? P.stdv[i] : 1.f, sJ = (j < P.n) ? P.stdv[j] : 1.f;
      const float v = rdm_value(g, i, j, P, sI, sJ);
      if (i < P.n && j < P.n) P.rdm[i * P.ldr + j] = v;
      tr[yy][tx] = v;
    }
    __syncthreads();
    if (!diag) {
      for (int yy = ty; yy < 32; yy += 8) {
        // mirror row j = col0 + sj0 + yy, columns i = row0 + si0 + tx
        const int64_t j = col0 + sj0 + yy, i = row0 + si0 + tx;
        if (i < P.n && j < P.n) P.rdm[j * P.ldr + i] = tr[tx][yy];
      }
    }
    __syncthreads();
  }
}

static int64_t gram_tiles(int64_t n) {
  const int64_t T = (n + GT - 1) / GT;
  return T * (T + 1) / 2;
}

// Split-K factor for `count` tiles of depth d: enough blocks for two per CU.
// fit = true (the tail of a generation launch, gram_tail): at most one resident set.
static void gram_geometry(int64_t n, int64_t d, int64_t count, int& T, int& ntiles,
                          int& splits, int64_t& kslice, bool fit = false) {
  T = (int)((n + GT - 1) / GT);
  ntiles = T * (T + 1) / 2;
  const int64_t kt = (d + GK - 1) / GK;  // k stages
  const int target = 2 * num_cus();     // two resident blocks per CU
  int s = 1;
  if (count < target) {
    s = fit ? (int)std::max<int64_t>(1, target / count) : (int)((target + count - 1) / count);
    const int64_t maxs = std::max<int64_t>(1, kt / 4);  // >= 4 stages per split
    if (s > maxs) s = (int)maxs;
  }
  const int64_t per = (kt + s - 1) / s;
  kslice = per * GK;
  splits = (int)((d + kslice - 1) / kslice);
  if (splits < 1) splits = 1;
}

// Gram arithmetic per call: VISREPS_GRAM=fp32 / =split force the exact-fp32 or the bf16
// split kernel; otherwise the split kernel runs where the Gram costs time (n^2 d >= 1e10
// MACs, ~0.2 ms on the fp32 kernel) and the fp32 kernel below that, where its smaller
// rounding error keeps tie-sensitive statistics of small RDMs closest to the reference.
// Read per call, so the workspace query and the launch of one call agree.
static bool gram_split(int64_t n, int64_t d) {
  const char* e = getenv("VISREPS_GRAM");
  if (e && strcmp(e, "fp32") == 0) return false;
  if (e && strcmp(e, "split") == 0) return true;
  return (double)n * (double)n * (double)d >= 1e10;
}

// Blocks per Gram launch. Every tile streams the same k range, so blocks that start
// together stay within a few stages of each other, and the ~64 a generation puts on one
// XCD (band order: an ~8 x 8 square of tiles, 16 distinct panels) then share each stage
// record in its L2. One launch over all tiles let finished blocks be replaced one at a
// time: the resident blocks drifted a whole tile apart in k and the L2 hit rate was 26 %
// (TCC_HIT / (HIT + MISS), N = 10k, D = 43264), so the kernel drew ~6 TB/s from HBM.
// A generation is one resident set (2 blocks per CU); VISREPS_GRAM_GEN=0 launches
// everything at once (A/B timing), another value sets the generation size.
static int gram_generation(int nblk) {
  int gen = 2 * num_cus();
  if (const char* e = getenv("VISREPS_GRAM_GEN")) {
    const int v = atoi(e);
    gen = v > 0 ? v : nblk;
  }
  return std::max(1, gen);
}

// Tiles of a launch's last, partial generation that run as their own split-K launch.
// With whole-k tiles the last generation of N = 10k (3160 tiles over 512 slots) keeps
// 88 blocks busy for one full tile time while 424 slots idle; split over k the same
// tiles fill the chip. Only a small tail (<= half a generation) of a multi-generation
// launch is split; its fp32 partials are summed in fixed order by k_gram_reduce.
static int64_t gram_tail(int64_t count) {
  const int gen = 2 * num_cus();
  if (getenv("VISREPS_GRAM_GEN") || count <= gen) return 0;
  const int64_t tail = count % gen;
  return (tail > 0 && tail <= gen / 2) ? tail : 0;
}

// Split-K partial floats of one tile range as run_split launches it (main + tail).
static size_t range_partial(int64_t n, int64_t d, int64_t count, bool fit_one = false) {
  if (count <= 0) return 0;
  int T, ntiles, splits;
  int64_t kslice;
  if (fit_one && count < 2 * num_cus()) {
    gram_geometry(n, d, count, T, ntiles, splits, kslice, true);
    return splits > 1 ? (size_t)splits * count * GT * GT : 0;
  }
  const int64_t tail = gram_tail(count);
  gram_geometry(n, d, count - tail, T, ntiles, splits, kslice);
  size_t part = splits > 1 ? (size_t)splits * (count - tail) : 0;
  if (tail > 0) {
    gram_geometry(n, d, tail, T, ntiles, splits, kslice, true);
    if (splits > 1) part = std::max(part, (size_t)splits * tail);
  }
  return part * GT * GT;
}

static int64_t tri_start(int64_t r, int64_t T) { return r * T - r * (r - 1) / 2; }

// Super-tile rows [0, R) of the wide split kernel in a full-RDM launch (0: not used).
// R is the largest whose super-tile count fits whole generations of one block per CU;
// the 128-tile rows [2R, T) below them run on k_gram3 (generations + tail split).
// VISREPS_GRAM_WIDE=0 turns the wide kernel off (A/B timing).
static int gram_wide_rows(int64_t n, int64_t d, bool split3) {
  if (!split3) return 0;
  if (const char* e = getenv("VISREPS_GRAM_WIDE"))
    if (strcmp(e, "0") == 0) return 0;
  const int64_t T2 = (n + WT - 1) / WT, gen = num_cus();
  const int64_t full = (T2 * (T2 + 1) / 2) / gen * gen;
  if (full < gen) return 0;
  int64_t R = 0;
  while (R + 1 <= T2 && tri_start(R + 1, T2) <= full) ++R;
  (void)d;
  return (int)R;
}

// How a launch over 128-tiles [t0, t1) runs. Every tile of an RDM is computed the same way
// whatever range it is launched in -- the full-RDM decomposition (super-tile rows [0, R) on
// the wide kernel, whole depth per tile; the remainder rows [2R, T) as one run_split) --
// so a range whose ends are super-tile row starts (tri_start(2r, T), r <= R) or the end of
// the triangle gives tiles bit-identical to the full launch: the multi-GPU path splits an
// RDM only at those boundaries (vr_rdm_range_aligned). Other ranges (legacy callers) run
// as one run_split of their own (split-K geometry of the range: last-bit differences).
struct RangePlan {
  bool wide = false;
  int64_t s0 = 0, s1 = 0;          // super-tiles [s0, s1) of the wide kernel, whole depth
  int64_t r0 = 0, r_count = 0;     // super-tile rows [R, T2) (the triangle's end): wide, split-K
  int r_splits = 1;
  int64_t rem0 = 0, rem_count = 0;  // 128-tiles of the run_split part (unaligned ranges)
  bool rem_fit = false;             // run_split's fit_one
};

// k splits of the wide kernel's remainder launch: enough blocks for one per CU, at least
// 8 stages per split
static int wide_rem_splits(int64_t count, int64_t nstage) {
  const int64_t gen = num_cus();
  if (count <= 0 || count >= gen) return 1;
  int64_t s = gen / count;
  s = std::min<int64_t>(s, std::max<int64_t>(1, nstage / 8));
  const int64_t per = (nstage + s - 1) / s;
  return (int)((nstage + per - 1) / per);
}

static RangePlan plan_range(int64_t n, int64_t d, int64_t t0, int64_t t1, bool split3) {
  RangePlan rp;
  const int64_t total = gram_tiles(n), T = (n + GT - 1) / GT, T2 = (n + WT - 1) / WT;
  const int R = gram_wide_rows(n, d, split3);
  rp.rem0 = t0;
  rp.rem_count = t1 - t0;
  if (R == 0 || t1 <= t0) return rp;
  int64_t r0 = -1, r1 = -1;
  for (int64_t r = 0; r <= R; ++r) {
    if (tri_start(2 * r, T) == t0) r0 = r;
    if (tri_start(2 * r, T) == t1) r1 = r;
  }
  if (r0 < 0 || (t1 != total && r1 < 0)) return rp;  // not aligned: legacy run_split
  const int64_t trem = tri_start(2 * (int64_t)R, T);
  rp.wide = true;
  rp.s0 = tri_start(r0, T2);
  rp.s1 = t1 == total ? tri_start(R, T2) : tri_start(r1, T2);
  rp.rem_count = 0;
  // The rows below R run on the wide kernel split over k (one generation, partials summed
  // in split order by k_gram_reduce_w); VISREPS_GRAM_WIDE_REM=0 runs them as 128-tiles
  // (run_split). With k_gram3e: +1.4 % on whole RDMs at D = 290,400, equal at 43,264
  // (profiles/r3_gram_ab.log) -- the wide kernel's per-CU rate, less +16 % work (the
  // diagonal super-tiles' lower quadrants), 220 of 256 CUs busy and the partial round trip.
  static const bool wide_rem = !(getenv("VISREPS_GRAM_WIDE_REM") && strcmp(getenv("VISREPS_GRAM_WIDE_REM"), "0") == 0);
  if (t1 == total && !wide_rem) {
    rp.rem0 = trem;
    rp.rem_count = total - trem;
    rp.rem_fit = true;
  } else if (t1 == total) {
    rp.r0 = tri_start(R, T2);
    rp.r_count = T2 * (T2 + 1) / 2 - rp.r0;
    rp.r_splits = wide_rem_splits(rp.r_count, (d + GK - 1) / GK);
  }
  return rp;
}

// Scratch of one RDM launch over `count` tiles: row stats, split-K partial tiles, and the
// bf16 plane records of the split kernel (rows padded to the 256-row super-tile edge).
// Accumulator flush interval in k stages (VISREPS_GRAM_FLUSH, 0 = off; default 256 stages =
// 8192 k) and the flush buffer: one fp32 tile per block of the largest launch (a generation:
// 2 x CUs 128-tiles or 1 x CUs 256-super-tiles).
static int gram_flush_stages() {
  int f = 256;  // k = 8192 per flush: profiles/r2_gram_flush.log (128: -7 % TF/s, errors within 2x)
  if (const char* e = getenv("VISREPS_GRAM_FLUSH")) f = atoi(e);
  return f > 0 ? f : 0;
}
static size_t gram_fbuf_floats() {
  return std::max<size_t>((size_t)2 * num_cus() * GT * GT, (size_t)num_cus() * WT * WT);
}

static size_t gram_ws(int64_t n, int64_t d, int64_t t0, int64_t t1, bool split3, void* base, float** mean,
                      float** stdv, float** partial, uint16_t** planes, float** fbuf = nullptr,
                      bool own_planes = true, uint32_t** flag = nullptr) {
  const RangePlan rp = plan_range(n, d, t0, t1, split3);
  size_t part = range_partial(n, d, rp.rem_count, rp.rem_fit);
  if (rp.r_splits > 1) part = std::max(part, (size_t)rp.r_count * rp.r_splits * WT * WT);
  Carver c(base);
  float* m = c.take<float>((size_t)n);
  float* s = c.take<float>((size_t)n);
  float* p = part ? c.take<float>(part) : nullptr;
  const int64_t prow = (n + WT - 1) / WT * WT;
  uint16_t* pl = split3 && own_planes ? c.take<uint16_t>((size_t)prow * (size_t)((d + GK - 1) / GK) * 64)
                                      : nullptr;
  const bool flush = gram_flush_stages() > 0 && (d + GK - 1) / GK > gram_flush_stages();
  float* fb = flush ? c.take<float>(gram_fbuf_floats()) : nullptr;
  uint32_t* fl = c.take<uint32_t>(64);
  if (flag) *flag = fl;
  if (fbuf) *fbuf = fb;
  if (mean) *mean = m;
  if (stdv) *stdv = s;
  if (partial) *partial = p;
  if (planes) *planes = pl;
  return c.bytes();
}

}  // namespace vr

using namespace vr;

extern "C" {

size_t vr_rdm_pearson_workspace(int64_t n, int64_t d) {
  if (n <= 0 || d <= 0) return 256;
  return gram_ws(n, d, 0, gram_tiles(n), gram_split(n, d), nullptr, nullptr, nullptr, nullptr, nullptr);
}

size_t vr_rdm_tiles_workspace(int64_t n, int64_t d, int64_t tile_begin, int64_t tile_end) {
  if (n <= 0 || d <= 0 || tile_end <= tile_begin) return 256;
  return gram_ws(n, d, tile_begin, tile_end, gram_split(n, d), nullptr, nullptr, nullptr, nullptr,
                 nullptr);
}

int64_t vr_rdm_tile_count(int64_t n) { return n > 0 ? gram_tiles(n) : 0; }

int64_t vr_rdm_wide_rows(int64_t n, int64_t d) {
  return n > 0 && d > 0 ? gram_wide_rows(n, d, gram_split(n, d)) : 0;
}

int vr_rdm_range_aligned(int64_t n, int64_t d, int64_t tile_begin, int64_t tile_end) {
  if (n <= 0 || d <= 0 || tile_begin < 0 || tile_end > gram_tiles(n) || tile_end < tile_begin) return 0;
  if (tile_begin == tile_end) return 1;
  if (tile_begin == 0 && tile_end == gram_tiles(n)) return 1;
  return plan_range(n, d, tile_begin, tile_end, gram_split(n, d)).wide ? 1 : 0;
}

int64_t vr_rdm_tile_cost(int64_t n, int64_t tile) {
  // elements of the tile on or above the diagonal (the work the balancer spreads)
  int T = (int)((n + GT - 1) / GT), bi, bj;
  int p = (int)tile, r = 0;
  while (r + 1 < T && (int64_t)(r + 1) * T - (int64_t)(r + 1) * r / 2 <= p) ++r;
  bi = r;
  bj = r + (p - (r * T - r * (r - 1) / 2));
  const int64_t h = std::min<int64_t>(GT, n - (int64_t)bi * GT), w = std::min<int64_t>(GT, n - (int64_t)bj * GT);
  return bi == bj ? h * (h + 1) / 2 : h * w;
}

int vr_rdm_tile_rect(int64_t n, int64_t tile, int64_t* row0, int64_t* col0, int64_t* rows,
                     int64_t* cols) {
  VR_REQUIRE(n > 0 && tile >= 0 && tile < gram_tiles(n), "vr_rdm_tile_rect: tile %lld of %lld",
             (long long)tile, (long long)(n > 0 ? gram_tiles(n) : 0));
  VR_REQUIRE(row0 && col0 && rows && cols, "vr_rdm_tile_rect: null output");
  const int T = (int)((n + GT - 1) / GT);
  int p = (int)tile, r = 0;
  while (r + 1 < T && (int64_t)(r + 1) * T - (int64_t)(r + 1) * r / 2 <= p) ++r;
  const int bi = r, bj = r + (p - (r * T - r * (r - 1) / 2));
  *row0 = (int64_t)bi * GT;
  *col0 = (int64_t)bj * GT;
  *rows = std::min<int64_t>(GT, n - *row0);
  *cols = std::min<int64_t>(GT, n - *col0);
  return VR_OK;
}

int vr_row_stats_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* mean,
                     float* stdv, float correction, void* stream) {
  VR_REQUIRE(n >= 0 && d > 0 && ldx >= d, "vr_row_stats_f32: bad shape n=%lld d=%lld ldx=%lld",
             (long long)n, (long long)d, (long long)ldx);
  if (n == 0) return VR_OK;
  VR_REQUIRE(X && mean && stdv, "vr_row_stats_f32: null pointer");
  VR_REQUIRE(n <= INT32_MAX, "vr_row_stats_f32: n too large");
  const int vec = ((reinterpret_cast<uintptr_t>(X) & 15) == 0) && ((ldx & 3) == 0);
  k_row_stats<float><<<(unsigned)n, RSTAT_BS, 0, as_stream(stream)>>>(X, d, ldx, mean, stdv,
                                                                       correction, vec);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// bf16 rows (16-bit patterns): the same statistics of the exactly widened values
static int row_stats_bf16(const uint16_t* X, int64_t n, int64_t d, int64_t ldx, float* mean,
                          float* stdv, float correction, hipStream_t st) {
  const int vec = ((reinterpret_cast<uintptr_t>(X) & 7) == 0) && ((ldx & 3) == 0);
  k_row_stats<uint16_t><<<(unsigned)n, RSTAT_BS, 0, st>>>(X, d, ldx, mean, stdv, correction, vec);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// bf16 input always takes the split kernel: only the row statistics and the split prepass
// read X, so no fp32 copy of the features is ever made (the exact-fp32 kernel stages X).
// Precomputed split rows (the multi-GPU path: each rank splits its own stimulus rows and
// the planes + row statistics are all-gathered): the launch skips its prepass.
struct PreSplit {
  const uint16_t* planes = nullptr;  // [vr_rdm_plane_rows(n)][nstage][64], rows >= n zero
  const float* mean = nullptr;       // [n]
  const float* stdv = nullptr;       // [n]
};

static int rdm_launch(const void* Xv, int64_t n, int64_t d, int64_t ldx, float* rdm, int64_t ldr,
                      float correction, int64_t tile_begin, int64_t tile_end, void* ws,
                      size_t ws_bytes, void* stream, size_t need, bool raw = false, bool bf16 = false,
                      const PreSplit& pre = PreSplit{}) {
  const float* X = static_cast<const float*>(Xv);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_rdm_pearson: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  GramParams P{};
  const bool split3 = bf16 || pre.planes || gram_split(n, d);
  float *mean, *stdv;
  uint16_t* planes;
  uint32_t* one_flag;
  gram_ws(n, d, tile_begin, tile_end, split3, ws, &mean, &stdv, &P.partial, &planes, &P.fbuf,
          pre.planes == nullptr, &one_flag);
  const int flush_stages = P.fbuf ? gram_flush_stages() : 0;
  P.raw = raw ? 1 : 0;
  P.dk = d;
  bool one = false;  // bf16 input, one product per k (the default for bf16; VISREPS_GRAM_ONE=0: split)
  if (bf16 && !pre.planes && !raw && gram_phased() && env_flag("VISREPS_GRAM_ONE", true)) {
    const int64_t rows = (n + WT - 1) / WT * WT, nst1 = (d + 2 * GK - 1) / (2 * GK);
    VR_CHECK_HIP(hipMemsetAsync(one_flag, 0, sizeof(uint32_t), st));
    k_stats_one<<<(unsigned)rows, RSTAT_BS, 0, st>>>(static_cast<const uint16_t*>(Xv), n, d, ldx, nst1, correction,
                                                     mean, stdv, planes, one_flag);
    VR_CHECK_LAUNCH();
    uint32_t bad = 0;
    VR_CHECK_HIP(hipMemcpyAsync(&bad, one_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    VR_CHECK_HIP(hipStreamSynchronize(st));
    one = bad == 0;
    if (one) {
      P.one = 1;
      P.planes = planes;
      P.nstage = nst1;
      P.dk = nst1 * GK;  // the split-K geometry in 32-k units of the 64-k stages
    }
  }
  if (pre.planes) {
    mean = const_cast<float*>(pre.mean);
    stdv = const_cast<float*>(pre.stdv);
    P.planes = pre.planes;
    P.nstage = (d + GK - 1) / GK;
  } else if (one) {  // statistics and raw records already written
  } else if (raw) {  // zero means: the panels stage X itself
    VR_CHECK_HIP(hipMemsetAsync(mean, 0, (size_t)n * sizeof(float), st));
    VR_CHECK_HIP(hipMemsetAsync(stdv, 0, (size_t)n * sizeof(float), st));
  } else if (split3) {  // row statistics + hi/lo records in one pass over X
    const int64_t rows = (n + WT - 1) / WT * WT;
    if (bf16)
      VR_TRY(stats_split(static_cast<const uint16_t*>(Xv), n, rows, d, ldx, correction, mean, stdv, planes, st));
    else
      VR_TRY(stats_split(X, n, rows, d, ldx, correction, mean, stdv, planes, st));
    P.planes = planes;
    P.nstage = (d + GK - 1) / GK;
  } else if (bf16) {
    VR_TRY(row_stats_bf16(static_cast<const uint16_t*>(Xv), n, d, ldx, mean, stdv, correction, st));
  } else {
    VR_TRY(vr_row_stats_f32(X, n, d, ldx, mean, stdv, correction, stream));
  }
  P.X = X;
  P.mean = mean;
  P.stdv = stdv;
  P.rdm = rdm;
  P.n = n;
  P.d = d;
  P.ldx = ldx;
  P.ldr = ldr;
  P.correction = correction;
  P.vec = (pre.planes || (((reinterpret_cast<uintptr_t>(Xv) & 15) == 0) && ((ldx & 3) == 0))) &&
          ((reinterpret_cast<uintptr_t>(rdm) & 15) == 0);
  // tile range [t0, t0 + count): its own split-K geometry, generations, reduction
  auto run_range = [&](int64_t t0, int64_t count, bool fit) -> int {
    if (count <= 0) return VR_OK;
    gram_geometry(n, P.dk, count, P.T, P.ntiles, P.splits, P.kslice, fit);
    P.tile0 = (int)t0;
    P.tile_count = (int)count;
    const int nblk = P.tile_count * P.splits;
    const int gen = gram_generation(nblk);
    // a flush needs one buffer tile per block of the launch
    P.flush = (size_t)std::min(gen, nblk) * GT * GT <= gram_fbuf_floats() ? flush_stages : 0;
    for (int b0 = 0; b0 < nblk; b0 += gen) {
      P.blk0 = b0;
      const unsigned nb = (unsigned)std::min(gen, nblk - b0);
      KtScope kt(KT_GRAM_TILE, 2.0 * (double)nb / P.splits * GT * GT * (double)d, st);  // tile FLOPs
      if (split3 && P.one)
        k_gram3<true><<<nb, G_THREADS, 0, st>>>(P);
      else if (split3)
        k_gram3<false><<<nb, G_THREADS, 0, st>>>(P);
      else
        k_gram<<<nb, G_THREADS, 0, st>>>(P);
      VR_CHECK_LAUNCH();
    }
    if (P.splits > 1) {
      k_gram_reduce<<<(unsigned)P.tile_count, 256, 0, st>>>(P);
      VR_CHECK_LAUNCH();
    }
    return VR_OK;
  };
  // fit_one: a range smaller than one generation splits over k into at most one
  // generation (floor) instead of spilling a few blocks into a second one (ceil)
  auto run_split = [&](int64_t t0, int64_t count, bool fit_one) -> int {
    if (fit_one && count < 2 * num_cus()) return run_range(t0, count, true);
    const int64_t tail = gram_tail(count);
    VR_TRY(run_range(t0, count - tail, false));
    return run_range(t0 + count - tail, tail, true);
  };
  const RangePlan rp = plan_range(n, d, tile_begin, tile_end, split3);
  if (!rp.wide) return run_split(tile_begin, tile_end - tile_begin, false);
  // wide super-tiles [s0, s1) (rows of the full RDM's wide part), then the 128-tile rows
  // below them when the range holds them
  GramParams W = P;
  W.T = (int)((n + WT - 1) / WT);
  W.tile0 = (int)rp.s0;
  W.tile_count = (int)(rp.s1 - rp.s0);
  W.splits = 1;
  W.kslice = P.nstage * GK;
  const int gen = num_cus();
  const bool pipe = gram_pipe(), phased = gram_phased();
  W.flush = (size_t)gen * WT * WT <= gram_fbuf_floats() ? flush_stages : 0;
  for (int b0 = 0; b0 < W.tile_count; b0 += gen) {
    W.blk0 = b0;
    KtScope kt(KT_GRAM_WIDE, 2.0 * (double)std::min(gen, W.tile_count - b0) * WT * WT * (double)d, st);
    if (phased && W.one)
      k_gram3e<true><<<(unsigned)std::min(gen, W.tile_count - b0), W_THREADS, 0, st>>>(W);
    else if (phased)
      k_gram3e<false><<<(unsigned)std::min(gen, W.tile_count - b0), W_THREADS, 0, st>>>(W);
    else if (pipe)
      k_gram3p<<<(unsigned)std::min(gen, W.tile_count - b0), W_THREADS, 0, st>>>(W);
    else
      k_gram3w<<<(unsigned)std::min(gen, W.tile_count - b0), W_THREADS, 0, st>>>(W);
    VR_CHECK_LAUNCH();
  }
  if (rp.r_count > 0) {  // rows [R, T2): split over k, partials summed in split order
    GramParams Rm = W;
    Rm.tile0 = (int)rp.r0;
    Rm.tile_count = (int)rp.r_count;
    Rm.splits = rp.r_splits;
    Rm.kslice = (P.nstage + rp.r_splits - 1) / rp.r_splits * GK;
    const int nblk = Rm.tile_count * Rm.splits;
    for (int b0 = 0; b0 < nblk; b0 += gen) {
      Rm.blk0 = b0;
      const int nb = std::min(gen, nblk - b0);
      KtScope kt(KT_GRAM_WIDE, 2.0 * (double)nb / Rm.splits * WT * WT * (double)d, st);
      if (phased && Rm.one)
        k_gram3e<true><<<(unsigned)nb, W_THREADS, 0, st>>>(Rm);
      else if (phased)
        k_gram3e<false><<<(unsigned)nb, W_THREADS, 0, st>>>(Rm);
      else
        k_gram3p<<<(unsigned)nb, W_THREADS, 0, st>>>(Rm);
      VR_CHECK_LAUNCH();
    }
    if (Rm.splits > 1) {
      k_gram_reduce_w<<<dim3((unsigned)Rm.tile_count, WT / 32), 256, 0, st>>>(Rm);
      VR_CHECK_LAUNCH();
    }
  }
  return run_split(rp.rem0, rp.rem_count, true);
}

int vr_rdm_pearson_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* rdm,
                       int64_t ldr, float correction, void* ws, size_t ws_bytes,
                       void* stream) {
  VR_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldr >= n,
             "vr_rdm_pearson_f32: bad shape n=%lld d=%lld ldx=%lld ldr=%lld", (long long)n,
             (long long)d, (long long)ldx, (long long)ldr);
  if (n == 0) return VR_OK;
  VR_REQUIRE(X && rdm, "vr_rdm_pearson_f32: null pointer");
  VR_REQUIRE(n <= (1 << 20), "vr_rdm_pearson_f32: n=%lld too large", (long long)n);
  return rdm_launch(X, n, d, ldx, rdm, ldr, correction, 0, gram_tiles(n), ws, ws_bytes, stream,
                    vr_rdm_pearson_workspace(n, d));
}

int vr_rdm_pearson_tiles_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* rdm,
                             int64_t ldr, float correction, int64_t tile_begin,
                             int64_t tile_end, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldr >= n,
             "vr_rdm_pearson_tiles_f32: bad shape n=%lld d=%lld", (long long)n, (long long)d);
  VR_REQUIRE(n <= (1 << 20), "vr_rdm_pearson_tiles_f32: n too large");
  VR_REQUIRE(tile_begin >= 0 && tile_end >= tile_begin && tile_end <= gram_tiles(n),
             "vr_rdm_pearson_tiles_f32: tile range [%lld, %lld) outside [0, %lld)",
             (long long)tile_begin, (long long)tile_end, (long long)gram_tiles(n));
  if (n == 0 || tile_end == tile_begin) return VR_OK;
  VR_REQUIRE(X && rdm, "vr_rdm_pearson_tiles_f32: null pointer");
  return rdm_launch(X, n, d, ldx, rdm, ldr, correction, tile_begin, tile_end, ws, ws_bytes,
                    stream, vr_rdm_tiles_workspace(n, d, tile_begin, tile_end));
}

size_t vr_rdm_bf16_workspace(int64_t n, int64_t d, int64_t tile_begin, int64_t tile_end) {
  if (n <= 0 || d <= 0 || tile_end <= tile_begin) return 256;
  return gram_ws(n, d, tile_begin, tile_end, true, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int vr_rdm_pearson_tiles_bf16(const uint16_t* X, int64_t n, int64_t d, int64_t ldx, float* rdm,
                              int64_t ldr, float correction, int64_t tile_begin, int64_t tile_end,
                              void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldr >= n,
             "vr_rdm_pearson_tiles_bf16: bad shape n=%lld d=%lld", (long long)n, (long long)d);
  VR_REQUIRE(n <= (1 << 20), "vr_rdm_pearson_tiles_bf16: n too large");
  VR_REQUIRE(tile_begin >= 0 && tile_end >= tile_begin && tile_end <= gram_tiles(n),
             "vr_rdm_pearson_tiles_bf16: tile range [%lld, %lld) outside [0, %lld)",
             (long long)tile_begin, (long long)tile_end, (long long)gram_tiles(n));
  if (n == 0 || tile_end == tile_begin) return VR_OK;
  VR_REQUIRE(X && rdm, "vr_rdm_pearson_tiles_bf16: null pointer");
  return rdm_launch(X, n, d, ldx, rdm, ldr, correction, tile_begin, tile_end, ws, ws_bytes, stream,
                    vr_rdm_bf16_workspace(n, d, tile_begin, tile_end), false, true);
}

int vr_rdm_pearson_bf16(const uint16_t* X, int64_t n, int64_t d, int64_t ldx, float* rdm, int64_t ldr,
                        float correction, void* ws, size_t ws_bytes, void* stream) {
  return vr_rdm_pearson_tiles_bf16(X, n, d, ldx, rdm, ldr, correction, 0, n > 0 ? gram_tiles(n) : 0, ws,
                                   ws_bytes, stream);
}

int vr_gram_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* G, int64_t ldg,
                void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldg >= n,
             "vr_gram_f32: bad shape n=%lld d=%lld ldx=%lld ldg=%lld", (long long)n, (long long)d,
             (long long)ldx, (long long)ldg);
  if (n == 0) return VR_OK;
  VR_REQUIRE(X && G, "vr_gram_f32: null pointer");
  VR_REQUIRE(n <= (1 << 20), "vr_gram_f32: n=%lld too large", (long long)n);
  return rdm_launch(X, n, d, ldx, G, ldg, 0.f, 0, gram_tiles(n), ws, ws_bytes, stream,
                    vr_rdm_pearson_workspace(n, d), true);
}


// ---------------------------------------------------------------------------------
// Multi-GPU pieces: split rows locally, Gram tiles from gathered planes, tile exchange
// ---------------------------------------------------------------------------------
int64_t vr_rdm_plane_rows(int64_t n) { return n > 0 ? (n + WT - 1) / WT * WT : 0; }

size_t vr_rdm_plane_row_bytes(int64_t d) {
  return d > 0 ? (size_t)((d + GK - 1) / GK) * 64 * sizeof(uint16_t) : 0;
}

int vr_rdm_split_rows_multi_f32(int npts, const float* const* X, const int64_t* d, const int64_t* ldx, int64_t rows,
                                float correction, float* const* mean, float* const* stdv, uint16_t* const* planes,
                                void* stream) {
  VR_REQUIRE(npts >= 0 && npts <= SPLIT_MULTI_MAX && rows >= 0, "vr_rdm_split_rows_multi_f32: npts=%d rows=%lld",
             npts, (long long)rows);
  if (npts == 0 || rows == 0) return VR_OK;
  VR_REQUIRE(X && d && ldx && mean && stdv && planes, "vr_rdm_split_rows_multi_f32: null pointer");
  SplitMulti S{};
  for (int p = 0; p < npts; ++p) {
    VR_REQUIRE(X[p] && mean[p] && stdv[p] && planes[p] && d[p] > 0 && ldx[p] >= d[p],
               "vr_rdm_split_rows_multi_f32: point %d: bad pointer or shape", p);
    S.X[p] = X[p];
    S.mean[p] = mean[p];
    S.stdv[p] = stdv[p];
    S.planes[p] = planes[p];
    S.d[p] = d[p];
    S.ldx[p] = ldx[p];
    S.vec[p] = ((reinterpret_cast<uintptr_t>(X[p]) & 15) == 0) && ((ldx[p] & 3) == 0);
  }
  k_stats_split_multi<<<dim3((unsigned)rows, (unsigned)npts), RSTAT_BS, 0, as_stream(stream)>>>(S, rows, correction);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // extern "C"

namespace vr {
// Rows src[i] of every point's batch output X[p] -> rows dst[i] of out[p] (fp32), one
// block per (row, point): the phase-1 selection rows kept during extraction, one launch per
// batch instead of an index_put per point.
constexpr int GATHER_MULTI_ROWS = 64;
struct GatherMulti {
  const float* X[SPLIT_MULTI_MAX];
  float* out[SPLIT_MULTI_MAX];
  int64_t d[SPLIT_MULTI_MAX];
  int64_t ldx[SPLIT_MULTI_MAX];
  int64_t ldo[SPLIT_MULTI_MAX];
  int32_t src[GATHER_MULTI_ROWS];
  int32_t dst[GATHER_MULTI_ROWS];
};
constexpr int GATHER_CHUNK = 8192;  // floats per block
__global__ __launch_bounds__(256) void k_gather_rows_multi(GatherMulti G) {
  const int i = blockIdx.y, p = blockIdx.z;
  const int64_t k0 = (int64_t)blockIdx.x * GATHER_CHUNK;
  if (k0 >= G.d[p]) return;
  const int64_t k1 = std::min<int64_t>(G.d[p], k0 + GATHER_CHUNK);
  const float* x = G.X[p] + (int64_t)G.src[i] * G.ldx[p];
  float* o = G.out[p] + (int64_t)G.dst[i] * G.ldo[p];
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(o)) & 15) == 0 && (k1 - k0) % 4 == 0 &&
                   k0 % 4 == 0;
  if (vec) {
    for (int64_t k = k0 + 4 * (int64_t)threadIdx.x; k < k1; k += 4 * (int64_t)blockDim.x)
      *reinterpret_cast<f32x4*>(o + k) = *reinterpret_cast<const f32x4*>(x + k);
  } else {
    for (int64_t k = k0 + threadIdx.x; k < k1; k += blockDim.x) o[k] = x[k];
  }
}
}  // namespace vr

extern "C" {

int vr_gather_rows_multi_f32(int npts, const float* const* X, const int64_t* d, const int64_t* ldx, int nrows,
                             const int32_t* src, const int32_t* dst, float* const* out, const int64_t* ldo,
                             void* stream) {
  VR_REQUIRE(npts >= 0 && npts <= SPLIT_MULTI_MAX && nrows >= 0, "vr_gather_rows_multi_f32: npts=%d nrows=%d",
             npts, nrows);
  if (npts == 0 || nrows == 0) return VR_OK;
  VR_REQUIRE(X && d && ldx && src && dst && out && ldo, "vr_gather_rows_multi_f32: null pointer");
  for (int r0 = 0; r0 < nrows; r0 += GATHER_MULTI_ROWS) {
    const int m = std::min(GATHER_MULTI_ROWS, nrows - r0);
    GatherMulti G{};
    for (int p = 0; p < npts; ++p) {
      VR_REQUIRE(X[p] && out[p] && d[p] > 0 && ldx[p] >= d[p] && ldo[p] >= d[p],
                 "vr_gather_rows_multi_f32: point %d: bad pointer or shape", p);
      G.X[p] = X[p];
      G.out[p] = out[p];
      G.d[p] = d[p];
      G.ldx[p] = ldx[p];
      G.ldo[p] = ldo[p];
    }
    for (int i = 0; i < m; ++i) {
      VR_REQUIRE(src[r0 + i] >= 0 && dst[r0 + i] >= 0, "vr_gather_rows_multi_f32: negative row");
      G.src[i] = src[r0 + i];
      G.dst[i] = dst[r0 + i];
    }
    int64_t dmax = 0;
    for (int p = 0; p < npts; ++p) dmax = std::max<int64_t>(dmax, d[p]);
    const unsigned chunks = (unsigned)((dmax + GATHER_CHUNK - 1) / GATHER_CHUNK);
    k_gather_rows_multi<<<dim3(chunks, (unsigned)m, (unsigned)npts), 256, 0, as_stream(stream)>>>(G);
    VR_CHECK_LAUNCH();
  }
  return VR_OK;
}

int vr_rdm_split_rows_f32(const float* X, int64_t rows, int64_t d, int64_t ldx, float correction,
                          float* mean, float* stdv, uint16_t* planes, void* stream) {
  VR_REQUIRE(rows >= 0 && d > 0 && ldx >= d, "vr_rdm_split_rows_f32: bad shape rows=%lld d=%lld",
             (long long)rows, (long long)d);
  if (rows == 0) return VR_OK;
  VR_REQUIRE(X && mean && stdv && planes, "vr_rdm_split_rows_f32: null pointer");
  return stats_split(X, rows, rows, d, ldx, correction, mean, stdv, planes, as_stream(stream));
}

size_t vr_rdm_planes_tiles_workspace(int64_t n, int64_t d, int64_t tile_begin, int64_t tile_end) {
  if (n <= 0 || d <= 0 || tile_end <= tile_begin) return 256;
  return gram_ws(n, d, tile_begin, tile_end, true, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                 false);
}

int vr_rdm_pearson_tiles_planes(const uint16_t* planes, const float* mean, const float* stdv,
                                int64_t n, int64_t d, float* rdm, int64_t ldr, float correction,
                                int64_t tile_begin, int64_t tile_end, void* ws, size_t ws_bytes,
                                void* stream) {
  VR_REQUIRE(n >= 0 && d > 0 && ldr >= n, "vr_rdm_pearson_tiles_planes: bad shape n=%lld d=%lld",
             (long long)n, (long long)d);
  VR_REQUIRE(n <= (1 << 20), "vr_rdm_pearson_tiles_planes: n too large");
  if (n == 0 || tile_end <= tile_begin) return VR_OK;
  VR_REQUIRE(tile_begin >= 0 && tile_end <= gram_tiles(n), "vr_rdm_pearson_tiles_planes: tiles [%lld, %lld)",
             (long long)tile_begin, (long long)tile_end);
  VR_REQUIRE(planes && mean && stdv && rdm, "vr_rdm_pearson_tiles_planes: null pointer");
  PreSplit pre;
  pre.planes = planes;
  pre.mean = mean;
  pre.stdv = stdv;
  return rdm_launch(planes, n, d, (d + 3) / 4 * 4, rdm, ldr, correction, tile_begin, tile_end, ws,
                    ws_bytes, stream, vr_rdm_planes_tiles_workspace(n, d, tile_begin, tile_end),
                    false, false, pre);
}

}  // extern "C"

namespace vr {
// tile index -> (block row, block col) of the upper-triangle tile list (GT tiles)
__device__ inline void tile_rc(int64_t T, int64_t p, int64_t& bi, int64_t& bj) {
  // r = largest row with tri_start(r, T) <= p
  double disc = (2.0 * T + 1) * (2.0 * T + 1) - 8.0 * (double)p;
  int64_t r = (int64_t)(((2.0 * T + 1) - sqrt(disc)) / 2.0);
  if (r < 0) r = 0;
  while (r > 0 && r * T - r * (r - 1) / 2 > p) --r;
  while ((r + 1) * T - (r + 1) * r / 2 <= p) ++r;
  bi = r;
  bj = r + (p - (r * T - r * (r - 1) / 2));
}

// packed[(t - t0) * GT * GT + i * GT + j] <-> rdm[(row0 + i) * ldr + col0 + j]
template <bool PACK>
__global__ __launch_bounds__(256) void k_tiles_move(float* __restrict__ rdm, int64_t ldr, int64_t n,
                                                    int64_t t0, float* __restrict__ packed) {
  const int64_t T = (n + GT - 1) / GT;
  int64_t bi, bj;
  tile_rc(T, t0 + blockIdx.x, bi, bj);
  const int64_t r0 = bi * GT, c0 = bj * GT;
  const int64_t h = n - r0 < GT ? n - r0 : GT, w = n - c0 < GT ? n - c0 : GT;
  float* pk = packed + (size_t)blockIdx.x * GT * GT;
  for (int e = threadIdx.x; e < GT * GT; e += blockDim.x) {
    const int i = e / GT, j = e % GT;
    if (i >= h || j >= w) continue;
    float* dst = rdm + (size_t)(r0 + i) * ldr + c0 + j;
    if (PACK) {
      pk[e] = *dst;
    } else {
      *dst = pk[e];
      rdm[(size_t)(c0 + j) * ldr + r0 + i] = pk[e];  // mirror (diagonal tiles: itself)
    }
  }
}
}  // namespace vr

extern "C" {

int vr_rdm_tiles_pack(const float* rdm, int64_t ldr, int64_t n, int64_t tile_begin, int64_t tile_end,
                      float* packed, void* stream) {
  VR_REQUIRE(n > 0 && ldr >= n && tile_begin >= 0 && tile_end <= gram_tiles(n),
             "vr_rdm_tiles_pack: bad range n=%lld [%lld, %lld)", (long long)n, (long long)tile_begin,
             (long long)tile_end);
  if (tile_end <= tile_begin) return VR_OK;
  VR_REQUIRE(rdm && packed, "vr_rdm_tiles_pack: null pointer");
  k_tiles_move<true><<<(unsigned)(tile_end - tile_begin), 256, 0, as_stream(stream)>>>(
      const_cast<float*>(rdm), ldr, n, tile_begin, packed);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

int vr_rdm_tiles_unpack(const float* packed, int64_t n, int64_t tile_begin, int64_t tile_end, float* rdm,
                        int64_t ldr, void* stream) {
  VR_REQUIRE(n > 0 && ldr >= n && tile_begin >= 0 && tile_end <= gram_tiles(n),
             "vr_rdm_tiles_unpack: bad range n=%lld [%lld, %lld)", (long long)n, (long long)tile_begin,
             (long long)tile_end);
  if (tile_end <= tile_begin) return VR_OK;
  VR_REQUIRE(rdm && packed, "vr_rdm_tiles_unpack: null pointer");
  k_tiles_move<false><<<(unsigned)(tile_end - tile_begin), 256, 0, as_stream(stream)>>>(
      rdm, ldr, n, tile_begin, const_cast<float*>(packed));
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // extern "C"
