// Encoding-score statistics on the GPU: mean per-voxel Pearson r between measured and
// predicted responses, for the point estimate and for every bootstrap subsample.
//
// Replaces, in visreps/analysis/encoding_score.py:
//   voxel_scores = correlation_score(Y_test, pred_test)                     :206-208
//   for i in range(n_bootstrap):                                             :219-224
//       boot_idx = rng.choice(n_test, size=int(0.9 n_test), replace=False)
//       scores[i] = correlation_score(Y_test[boot_idx], pred_test[boot_idx]).mean()
// himalaya 0.4.9 correlation_score(y, p) = mean over rows of zscore(y) * zscore(p)
// (population std), i.e. Pearson r per column; a zero-variance column gives NaN.
//
//  k_corr_cols   grid (draws, column blocks): one thread per voxel column, the draw's row
//                indices staged in LDS; five fp64 sums over the rows (coalesced row reads
//                across the block's columns; Y and P stay L2/MALL resident across draws);
//                per block the sum of its columns' r                       [HBM/L2-bound]
//  k_corr_fold   per draw, the block partials summed in fixed order / v -> score (fp64)
#include "internal.h"

namespace vr {

constexpr int CS_THREADS = 256;
constexpr int CS_IDX = 4096;  // row indices staged per LDS round

__global__ __launch_bounds__(CS_THREADS) void k_corr_cols(
    const float* __restrict__ Y, const float* __restrict__ P, int64_t n, int64_t v, int64_t ld,
    const int32_t* __restrict__ idx, int64_t k, double* __restrict__ voxel_r,
    double* __restrict__ part) {
  __shared__ int32_t rows[CS_IDX];
  __shared__ double red[CS_THREADS / 64];
  const int64_t b = blockIdx.x;
  const int64_t c = (int64_t)blockIdx.y * CS_THREADS + threadIdx.x;
  const bool on = c < v;
  const int32_t* my = idx ? idx + b * k : nullptr;
  double sy = 0, sp = 0, syy = 0, spp = 0, syp = 0;
  for (int64_t r0 = 0; r0 < k; r0 += CS_IDX) {
    const int m = (int)min<int64_t>(CS_IDX, k - r0);
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += CS_THREADS) rows[i] = my ? my[r0 + i] : (int32_t)(r0 + i);
    __syncthreads();
    if (on) {
      for (int i = 0; i < m; ++i) {
        const int64_t o = (int64_t)rows[i] * ld + c;
        const double y = (double)Y[o], p = (double)P[o];
        sy += y;
        sp += p;
        syy += y * y;
        spp += p * p;
        syp += y * p;
      }
    }
  }
  double r = 0.0;
  if (on) {
    const double kk = (double)k;
    const double my_ = sy / kk, mp = sp / kk;
    const double vy = syy / kk - my_ * my_, vp = spp / kk - mp * mp;
    const double cov = syp / kk - my_ * mp;
    r = cov / sqrt((vy > 0 ? vy : 0.0) * (vp > 0 ? vp : 0.0));  // 0/0 -> NaN like zscore
    if (voxel_r) voxel_r[b * v + c] = r;
  }
  for (int o = 32; o > 0; o >>= 1) r += __shfl_down(r, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = r;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int w = 0; w < CS_THREADS / 64; ++w) s += red[w];
    part[b * gridDim.y + blockIdx.y] = s;
  }
}

__global__ void k_corr_fold(const double* __restrict__ part, int nblk, int64_t draws, int64_t v,
                            double* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= draws) return;
  double s = 0;
  for (int i = 0; i < nblk; ++i) s += part[b * nblk + i];
  out[b] = s / (double)v;
}

}  // namespace vr

using namespace vr;

extern "C" {

size_t vr_corr_score_workspace(int64_t v, int64_t draws) {
  const int64_t nblk = (v + CS_THREADS - 1) / CS_THREADS;
  return (size_t)std::max<int64_t>(1, draws * nblk) * sizeof(double);
}

int vr_corr_score_f32(const float* Y, const float* P, int64_t n, int64_t v, int64_t ld,
                      const int32_t* idx, int64_t k, int64_t draws, double* scores,
                      double* voxel_r, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n > 0 && v > 0 && ld >= v, "vr_corr_score_f32: bad shape n=%lld v=%lld ld=%lld",
             (long long)n, (long long)v, (long long)ld);
  VR_REQUIRE(draws >= 1 && k >= 1 && k <= n, "vr_corr_score_f32: draws=%lld k=%lld n=%lld",
             (long long)draws, (long long)k, (long long)n);
  VR_REQUIRE(idx != nullptr || (draws == 1 && k == n),
             "vr_corr_score_f32: idx may be null only for one draw over all rows");
  VR_REQUIRE(Y && P && scores, "vr_corr_score_f32: null pointer");
  VR_REQUIRE(draws <= 65535 * 1024, "vr_corr_score_f32: too many draws");
  const int64_t nblk = (v + CS_THREADS - 1) / CS_THREADS;
  VR_REQUIRE(nblk <= 65535, "vr_corr_score_f32: v too large");
  if (ws == nullptr || ws_bytes < vr_corr_score_workspace(v, draws)) {
    set_error("vr_corr_score_f32: workspace %zu < %zu", ws_bytes, vr_corr_score_workspace(v, draws));
    return VR_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  double* part = static_cast<double*>(ws);
  k_corr_cols<<<dim3((unsigned)draws, (unsigned)nblk), CS_THREADS, 0, st>>>(Y, P, n, v, ld, idx, k,
                                                                          voxel_r, part);
  VR_CHECK_LAUNCH();
  k_corr_fold<<<(unsigned)((draws + 255) / 256), 256, 0, st>>>(part, (int)nblk, draws, v, scores);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // extern "C"
