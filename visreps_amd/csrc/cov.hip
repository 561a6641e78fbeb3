// PCA covariance of extracted features: replaces batched_pca's
// mean and covariance, scripts/coarsegrain/compute_eigenvectors.py:23-36,
//   mean = X.mean(axis=0)                                 numpy, X float32 C-order (n, p)
//   cov  = sum over batches of (X[b].astype(f64) - mean)^T (X[b].astype(f64) - mean)
//   cov /= n - 1                                          (p, p) float64
//
// k_col_sum   numpy's float32 mean along axis 0 of a C-order array adds whole rows in row
//             order (the inner loop runs over columns), so every column is a sequential
//             float32 sum. One workgroup per 64 columns keeps that order exactly: 15
//             waves stream rows into an LDS ring, wave 0 adds them in order. Bit-identical
//             to numpy; `init` continues a sum (the multi-GPU chain over row shards).
// k_cov       upper-triangle 64 x 64 tiles of the centred Gram in fp64 on the fp64 MFMA
//             (v_mfma_f64_16x16x4_f64): 16-row stages of both column panels are centred
//             in fp64 ((double)x - (double)mean, exact, as astype(float64) - mean) while
//             they are staged into LDS, double-buffered; 4 waves as 2 x 2, each 32 x 32.
//             The rows are split into S slices so small p still fills the chip; a slice
//             writes its fp64 partial tile and k_cov_reduce adds the slices in fixed order,
//             divides by the denominator and writes each entry and its mirror (the result
//             is exactly symmetric, like the reference's batch.T @ batch).
// Roofline: fp64 MFMA, algorithmic FLOPs = n p (p + 1) (the unique entries i <= j).
#include "internal.h"

namespace vr {

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float cf32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------
// column sums in numpy's order
// ------------------------------------------------------------------------------------
constexpr int MS_THREADS = 1024;        // 16 waves: wave 0 adds, waves 1..15 load
constexpr int MS_COLS = 64;             // columns per workgroup (one per lane of wave 0)
constexpr int MS_HALF = 240;            // rows per ring half (15 loader waves x 16 rows)

__global__ __launch_bounds__(MS_THREADS) void k_col_sum(const float* __restrict__ X, int64_t n, int64_t p,
                                                        int64_t ldx, const float* __restrict__ init,
                                                        float* __restrict__ sum) {
  __shared__ float ring[2][MS_HALF][MS_COLS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * MS_COLS + lane;
  const bool cin = col < p;
  const int64_t nh = (n + MS_HALF - 1) / MS_HALF;
  // loader wave w (1..15) fills rows [16 (w - 1), 16 w) of a half
  auto fill = [&](int64_t h, int buf) {
    const int64_t r0 = h * MS_HALF + 16 * (wid - 1);
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = (cin && r0 + i < n) ? X[(r0 + i) * ldx + col] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) ring[buf][16 * (wid - 1) + i][lane] = v[i];
  };
  float s = (init != nullptr && cin) ? init[col] : 0.f;
  if (wid > 0 && nh > 0) fill(0, 0);
  __syncthreads();
  for (int64_t h = 0; h < nh; ++h) {
    const int buf = (int)(h & 1);
    if (wid > 0) {
      if (h + 1 < nh) fill(h + 1, buf ^ 1);
    } else {
      const int rows = (int)min<int64_t>(MS_HALF, n - h * MS_HALF);
      for (int i = 0; i < rows; ++i) s = s + ring[buf][i][lane];  // row order, float32
    }
    __syncthreads();
  }
  if (wid == 0 && cin) sum[col] = s;
}

// mean = sum / n in float32 (numpy's true_divide of the float32 sum by the count)
__global__ void k_col_div(const float* __restrict__ sum, int64_t p, float cnt, float* __restrict__ mean) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < p) mean[i] = sum[i] / cnt;
}

// ------------------------------------------------------------------------------------
// fp64 covariance tiles
// ------------------------------------------------------------------------------------
constexpr int CT = 64;          // tile edge (columns of X)
constexpr int CK = 16;          // rows per stage
constexpr int CLD = CT + 16;    // LDS row pitch (doubles): 4 k-rows of a fragment read hit 2 bank sets
constexpr int C_THREADS = 256;
constexpr int C_STAGE = CK * CLD;  // doubles per panel per stage

struct CovParams {
  const float* X;
  int64_t n, p, ldx;
  const float* mean;  // null: uncentred (the ridge Grams)
  double* partial;  // [S][ntile][CT * CT]
  int T;            // tile rows
  int ntile;        // T (T + 1) / 2
  int S;            // row slices
  int64_t kslice;   // rows per slice (multiple of CK)
  bool vec;         // 16-B aligned rows: float4 panel loads
};

// TRANS (the kernel-form ridge Gram X X^T of a row-major (p, n) X): the contraction runs
// along X's rows, so panel entry (k, c) is X[c * ldx + k]. Each thread loads 4 consecutive
// k of one column c (one float4 when aligned) and scatters them down the LDS column.
__device__ inline cf32x4 cov_load_t(const CovParams& P, int64_t col0, int64_t k, int64_t k1) {
  const int c = threadIdx.x >> 2, kq = (threadIdx.x & 3) * 4;
  cf32x4 v = {0.f, 0.f, 0.f, 0.f};
  const int64_t col = col0 + c, r = k + kq;
  if (col >= P.p || r >= k1) return v;
  const float* src = P.X + col * P.ldx + r;
  if (P.vec && r + 4 <= k1) {
    v = *reinterpret_cast<const cf32x4*>(src);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (r + e < k1) ? src[e] : 0.f;
  }
  return v;
}

__device__ inline void cov_store_t(double* lds, const cf32x4 v) {
  const int c = threadIdx.x >> 2, kq = (threadIdx.x & 3) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) lds[(kq + e) * CLD + c] = (double)v[e];  // out-of-range entries are 0
}

// tile t of the upper triangle (row-major: (0,0), (0,1), .., (0,T-1), (1,1), ..)
__device__ inline void cov_tile(int t, int T, int& bi, int& bj) {
  int r = 0, start = 0;
  while (start + (T - r) <= t) {
    start += T - r;
    ++r;
  }
  bi = r;
  bj = r + (t - start);
}

// this thread's 4 columns of a 16-row panel stage: row kr = tid >> 4, columns 4 (tid & 15)
__device__ inline cf32x4 cov_load(const CovParams& P, int64_t col0, int64_t k, int64_t k1) {
  const int kr = threadIdx.x >> 4, c = (threadIdx.x & 15) * 4;
  const int64_t r = k + kr;
  cf32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (r >= k1) return v;
  const float* src = P.X + r * P.ldx + col0 + c;
  if (P.vec && col0 + c + 4 <= P.p) {
    v = *reinterpret_cast<const cf32x4*>(src);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (col0 + c + e < P.p) ? src[e] : 0.f;
  }
  return v;
}

__device__ inline void cov_store(double* lds, const cf32x4 v, const double m[4], int64_t k, int64_t k1) {
  const int kr = threadIdx.x >> 4, c = (threadIdx.x & 15) * 4;
  const bool in = k + kr < k1;
  double* dst = lds + kr * CLD + c;
#pragma unroll
  for (int e = 0; e < 4; ++e) dst[e] = in ? (double)v[e] - m[e] : 0.0;  // padded rows add exact zeros
}

template <bool TRANS>
__global__ __launch_bounds__(C_THREADS, 2) void k_cov(CovParams P) {
  __shared__ __attribute__((aligned(16))) double lds[2][2][C_STAGE];  // [buf][A/B]
  const int id = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int tile = id / P.S, slice = id % P.S;
  int bi, bj;
  cov_tile(tile, P.T, bi, bj);
  const bool diag = bi == bj;
  const int64_t ci = (int64_t)bi * CT, cj = (int64_t)bj * CT;
  const int64_t k0 = (int64_t)slice * P.kslice;
  const int64_t k1 = min(P.n, k0 + P.kslice);
  const int nk = k1 > k0 ? (int)((k1 - k0 + CK - 1) / CK) : 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  double mA[4], mB[4];
  {
    const int c = (threadIdx.x & 15) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      mA[e] = (P.mean && ci + c + e < P.p) ? (double)P.mean[ci + c + e] : 0.0;
      mB[e] = (P.mean && cj + c + e < P.p) ? (double)P.mean[cj + c + e] : 0.0;
    }
  }
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};

  auto load = [&](int64_t col0, int64_t k) { return TRANS ? cov_load_t(P, col0, k, k1) : cov_load(P, col0, k, k1); };
  auto store = [&](double* dst, const cf32x4 v, const double* m, int64_t k) {
    if constexpr (TRANS)
      cov_store_t(dst, v);
    else
      cov_store(dst, v, m, k, k1);
  };
  cf32x4 ga = {0.f, 0.f, 0.f, 0.f}, gb = ga;
  if (nk > 0) {
    ga = load(ci, k0);
    if (!diag) gb = load(cj, k0);
    store(lds[0][0], ga, mA, k0);
    if (!diag) store(lds[0][1], gb, mB, k0);
  }
  __syncthreads();
  // fragment of the 16x16x4 f64 MFMA: lane l supplies A[m = l & 15][k = l >> 4] and
  // B[k = l >> 4][n = l & 15]; here A = X^T (panel of columns ci), B = X (columns cj)
  const int fk = lane >> 4, fm = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const double* As = lds[cur][0];
    const double* Bs = diag ? As : lds[cur][1];
    const bool more = kt + 1 < nk;
    const int64_t kn = k0 + (int64_t)(kt + 1) * CK;
    if (more) {
      ga = load(ci, kn);
      if (!diag) gb = load(cj, kn);
    }
#pragma unroll
    for (int ks = 0; ks < CK / 4; ++ks) {
      const int kr = ks * 4 + fk;
      double a[2], b[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        a[m] = As[kr * CLD + wr * 32 + m * 16 + fm];
        b[m] = Bs[kr * CLD + wc * 32 + m * 16 + fm];
      }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
          acc[m][nn] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[nn], acc[m][nn], 0, 0, 0);
    }
    if (more) {
      store(lds[cur ^ 1][0], ga, mA, kn);
      if (!diag) store(lds[cur ^ 1][1], gb, mB, kn);
    }
    __syncthreads();
  }
  // C/D of the f64 MFMA: col = lane & 15, row = (lane >> 4) + 4 r
  double* out = P.partial + ((int64_t)slice * P.ntile + tile) * (CT * CT);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int li = wr * 32 + m * 16 + fk + 4 * r;
        const int lj = wc * 32 + nn * 16 + fm;
        out[li * CT + lj] = acc[m][nn][r];
      }
}

// sum of the slices in slice order, / denom, into cov (entry and mirror)
__global__ __launch_bounds__(256) void k_cov_reduce(const double* __restrict__ partial, int S, int ntile,
                                                    int T, int64_t p, double denom, double* __restrict__ cov,
                                                    int64_t ldc) {
  const int tile = blockIdx.x;
  int bi, bj;
  cov_tile(tile, T, bi, bj);
  const int64_t ci = (int64_t)bi * CT, cj = (int64_t)bj * CT;
  for (int e = threadIdx.x; e < CT * CT; e += blockDim.x) {
    const int li = e / CT, lj = e % CT;
    const int64_t i = ci + li, j = cj + lj;
    if (i >= p || j >= p || (bi == bj && li > lj)) continue;
    double s = 0.0;
    for (int q = 0; q < S; ++q) s += partial[((int64_t)q * ntile + tile) * (CT * CT) + e];
    s /= denom;
    cov[i * ldc + j] = s;
    if (i != j) cov[j * ldc + i] = s;
  }
}

static void cov_geometry(int64_t n, int64_t p, int& T, int& ntile, int& S, int64_t& kslice) {
  T = (int)((p + CT - 1) / CT);
  ntile = T * (T + 1) / 2;
  // enough workgroups for ~4 per CU, each slice at least 64 stages of rows
  const int64_t want = std::max<int64_t>(1, (4LL * num_cus() + ntile - 1) / ntile);
  const int64_t maxs = std::max<int64_t>(1, n / (64 * CK));
  S = (int)std::min<int64_t>(want, maxs);
  kslice = ((n + S - 1) / S + CK - 1) / CK * CK;
  if (kslice == 0) kslice = CK;
  S = (int)std::max<int64_t>(1, (n + kslice - 1) / kslice);
}

}  // namespace vr

using namespace vr;

extern "C" {

int vr_col_sum_f32(const float* X, int64_t n, int64_t p, int64_t ldx, const float* init, float* sum,
                   void* stream) {
  clear_error();
  VR_REQUIRE(n >= 0 && p >= 0 && ldx >= p, "vr_col_sum_f32: bad shape n=%lld p=%lld ldx=%lld",
             (long long)n, (long long)p, (long long)ldx);
  if (p == 0) return VR_OK;
  VR_REQUIRE(sum != nullptr && (n == 0 || X != nullptr), "vr_col_sum_f32: null pointer");
  const unsigned grid = (unsigned)((p + MS_COLS - 1) / MS_COLS);
  k_col_sum<<<grid, MS_THREADS, 0, as_stream(stream)>>>(X, n, p, ldx, init, sum);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

int vr_col_mean_f32(const float* X, int64_t n, int64_t p, int64_t ldx, float* mean, void* stream) {
  VR_TRY(vr_col_sum_f32(X, n, p, ldx, nullptr, mean, stream));
  if (p == 0) return VR_OK;
  k_col_div<<<(unsigned)((p + 255) / 256), 256, 0, as_stream(stream)>>>(mean, p, (float)n, mean);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

int vr_mean_from_sum_f32(const float* sum, int64_t p, int64_t n, float* mean, void* stream) {
  clear_error();
  VR_REQUIRE(p >= 0 && n >= 0, "vr_mean_from_sum_f32: bad shape");
  if (p == 0) return VR_OK;
  k_col_div<<<(unsigned)((p + 255) / 256), 256, 0, as_stream(stream)>>>(sum, p, (float)n, mean);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

size_t vr_pca_cov_workspace(int64_t n, int64_t p) {
  if (n <= 0 || p <= 0) return 256;
  int T, ntile, S;
  int64_t kslice;
  cov_geometry(n, p, T, ntile, S, kslice);
  Carver c(nullptr);
  c.take<double>((size_t)S * ntile * CT * CT);
  return c.bytes();
}

// (n = contraction length, p = output order) -> k_cov + k_cov_reduce
static int cov_launch(bool trans, const float* X, int64_t n, int64_t p, int64_t ldx, const float* mean,
                      double denom, double* cov, int64_t ldc, void* ws, hipStream_t st) {
  CovParams P;
  P.X = X;
  P.n = n;
  P.p = p;
  P.ldx = ldx;
  P.mean = mean;
  cov_geometry(std::max<int64_t>(n, 1), p, P.T, P.ntile, P.S, P.kslice);
  Carver c(ws);
  P.partial = c.take<double>((size_t)P.S * P.ntile * CT * CT);
  P.vec = (ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  {
    KtScope kt(KT_COV, (double)n * (double)p * (double)(p + 1), st);  // algorithmic FLOPs
    if (trans)
      k_cov<true><<<(unsigned)(P.ntile * P.S), C_THREADS, 0, st>>>(P);
    else
      k_cov<false><<<(unsigned)(P.ntile * P.S), C_THREADS, 0, st>>>(P);
    VR_CHECK_LAUNCH();
  }
  k_cov_reduce<<<(unsigned)P.ntile, 256, 0, st>>>(P.partial, P.S, P.ntile, P.T, p, denom, cov, ldc);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

int vr_pca_cov_f64(const float* X, int64_t n, int64_t p, int64_t ldx, const float* mean, double denom,
                   double* cov, int64_t ldc, void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VR_REQUIRE(n >= 0 && p >= 1 && ldx >= p && ldc >= p, "vr_pca_cov_f64: bad shape n=%lld p=%lld",
             (long long)n, (long long)p);
  VR_REQUIRE(mean != nullptr && cov != nullptr && (n == 0 || X != nullptr), "vr_pca_cov_f64: null pointer");
  VR_REQUIRE(ws_bytes >= vr_pca_cov_workspace(n, p), "vr_pca_cov_f64: workspace too small");
  return cov_launch(false, X, n, p, ldx, mean, denom, cov, ldc, ws, as_stream(stream));
}

size_t vr_gram64_workspace(int64_t n, int64_t p, int rows) {
  return rows ? vr_pca_cov_workspace(p, n) : vr_pca_cov_workspace(n, p);
}

int vr_gram64_f32(const float* X, int64_t n, int64_t p, int64_t ldx, int rows, double* G, int64_t ldg,
                  void* ws, size_t ws_bytes, void* stream) {
  clear_error();
  VR_REQUIRE(n >= 1 && p >= 0 && ldx >= p, "vr_gram64_f32: bad shape n=%lld p=%lld ldx=%lld", (long long)n,
             (long long)p, (long long)ldx);
  VR_REQUIRE(ldg >= (rows ? n : p), "vr_gram64_f32: ldg %lld too small", (long long)ldg);
  VR_REQUIRE(G != nullptr && (p == 0 || X != nullptr), "vr_gram64_f32: null pointer");
  VR_REQUIRE(ws_bytes >= vr_gram64_workspace(n, p, rows), "vr_gram64_f32: workspace too small");
  if (rows) {  // X X^T (n x n): contraction over the p columns, X read transposed
    VR_REQUIRE(p >= 1, "vr_gram64_f32: rows Gram of zero-width X");
    return cov_launch(true, X, p, n, ldx, nullptr, 1.0, G, ldg, ws, as_stream(stream));
  }
  VR_REQUIRE(p >= 1, "vr_gram64_f32: columns Gram of zero-width X");
  return cov_launch(false, X, n, p, ldx, nullptr, 1.0, G, ldg, ws, as_stream(stream));
}

}  // extern "C"
