// Pearson of two RDMs' strict upper triangles in fp64, replacing
// compute_rdm_correlation(.., correlation="Pearson") -> scipy.stats.pearsonr
// (visreps/analysis/rsa.py:43-47,121-122). Two passes (means, then centred sums) with
// fixed-order reductions, so the result is deterministic.
#include "internal.h"

namespace vr {

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
      if (M < 2 || !(s[3] > 0) || !(s[4] > 0)) {  // constant or NaN input: undefined
        r = __builtin_nan("");
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
