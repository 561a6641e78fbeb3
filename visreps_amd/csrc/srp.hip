// Phase-1 sparse random projection: out (B x k) = X (B x D) * P^T with P a CSR (k x D)
// matrix (sklearn SparseRandomProjection.components_, density 1/sqrt(D) so each row
// holds ~sqrt(D) nonzeros).
//
// Replaces  torch.sparse.mm(proj_matrix, flat.t()).t()    visreps/models/utils.py:334-336
// with the matrix built as in                   visreps/models/utils.py:297-322
//                                               visreps/analysis/sparse_random_projection.py:83-150
//
// Two kernels:
//  k_srp_transpose  X (B x D, ld) -> XT (D x Bp), Bp = B rounded up to 64: one 64-float row
//                   per input feature, so a nonzero's batch column is one coalesced row
//  k_srp_spmm       a workgroup owns 64 output features x 64 batch rows; each wave walks
//                   16 CSR rows (index/value loads are wave-uniform s_loads), lane = batch
//                   row, SRP_U row loads in flight, fp32 fma in CSR order; the tile is transposed through LDS so the
//                   (B x k) output is written in 256-byte rows.
#include "internal.h"

namespace vr {

constexpr int SRP_T = 64;
#ifndef VR_SRP_U
#define VR_SRP_U 16
#endif
constexpr int SRP_U = VR_SRP_U;  // nonzeros per batch of row loads

__global__ __launch_bounds__(256) void k_srp_transpose(const float* __restrict__ X, int64_t B,
                                                       int64_t D, int64_t ldx, int64_t Bp,
                                                       float* __restrict__ XT) {
  __shared__ float tile[SRP_T][SRP_T + 1];
  const int64_t d0 = (int64_t)blockIdx.x * SRP_T, b0 = (int64_t)blockIdx.y * SRP_T;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 4 rows per sweep
  for (int r = ty; r < SRP_T; r += 4) {
    const int64_t b = b0 + r, d = d0 + tx;
    tile[r][tx] = (b < B && d < D) ? X[b * ldx + d] : 0.0f;
  }
  __syncthreads();
  for (int r = ty; r < SRP_T; r += 4) {
    const int64_t d = d0 + r, b = b0 + tx;
    if (d < D && b < Bp) XT[d * Bp + b] = tile[tx][r];
  }
}

template <typename T>
__device__ inline T srp_sload(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}

__global__ __launch_bounds__(256) void k_srp_spmm(const int32_t* __restrict__ indptr,
                                                  const int32_t* __restrict__ indices,
                                                  const float* __restrict__ vals, int64_t k,
                                                  const float* __restrict__ XT, int64_t B,
                                                  int64_t Bp, float* __restrict__ out,
                                                  int64_t ldo) {
  __shared__ float tile[SRP_T][SRP_T + 1];  // [feature][batch]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t r0 = (int64_t)blockIdx.x * SRP_T, b0 = (int64_t)blockIdx.y * SRP_T;
  const float* xt = XT + b0 + lane;
  for (int i = wave; i < SRP_T; i += 4) {
    const int64_t r = r0 + i;
    float acc = 0.0f;
    if (r < k) {
      const int32_t j0 = srp_sload(indptr + r), j1 = srp_sload(indptr + r + 1);
      int32_t j = j0;
      for (; j + SRP_U <= j1; j += SRP_U) {  // SRP_U independent row loads in flight, then the
        float x[SRP_U];                      // fmas in CSR order
#pragma unroll
        for (int u = 0; u < SRP_U; ++u) x[u] = xt[(int64_t)srp_sload(indices + j + u) * Bp];
#pragma unroll
        for (int u = 0; u < SRP_U; ++u) acc = __builtin_fmaf(srp_sload(vals + j + u), x[u], acc);
      }
      for (; j < j1; ++j) acc = __builtin_fmaf(srp_sload(vals + j), xt[(int64_t)srp_sload(indices + j) * Bp], acc);
    }
    tile[i][lane] = acc;
  }
  __syncthreads();
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int bb = ty; bb < SRP_T; bb += 4) {
    const int64_t b = b0 + bb, r = r0 + tx;
    if (b < B && r < k) out[b * ldo + r] = tile[tx][bb];
  }
}

static inline int64_t srp_bp(int64_t B) { return (B + SRP_T - 1) / SRP_T * SRP_T; }

}  // namespace vr

using namespace vr;

extern "C" {

size_t vr_srp_workspace(int64_t B, int64_t D) {
  if (B <= 0 || D <= 0) return 0;
  return (size_t)srp_bp(B) * (size_t)D * sizeof(float);
}

int vr_srp_csr_f32(const int32_t* indptr, const int32_t* indices, const float* values, int64_t k,
                   int64_t D, const float* X, int64_t B, int64_t ldx, float* out, int64_t ldo,
                   void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(k >= 0 && D >= 0 && B >= 0, "vr_srp_csr_f32: negative size");
  VR_REQUIRE(ldx >= D && ldo >= k, "vr_srp_csr_f32: ldx=%lld < D=%lld or ldo=%lld < k=%lld",
             (long long)ldx, (long long)D, (long long)ldo, (long long)k);
  if (B == 0 || k == 0) return VR_OK;
  VR_REQUIRE(indptr && X && out, "vr_srp_csr_f32: null pointer");
  VR_REQUIRE((int64_t)(unsigned)((k + SRP_T - 1) / SRP_T) == (k + SRP_T - 1) / SRP_T &&
                 (B + SRP_T - 1) / SRP_T <= 65535 && (D + SRP_T - 1) / SRP_T <= 0x7fffffff,
             "vr_srp_csr_f32: grid too large");
  const size_t need = vr_srp_workspace(B, D);
  if (ws == nullptr || ws_bytes < need) {
    set_error("vr_srp_csr_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* XT = static_cast<float*>(ws);
  const int64_t Bp = srp_bp(B);
  if (D > 0) {
    dim3 gt((unsigned)((D + SRP_T - 1) / SRP_T), (unsigned)(Bp / SRP_T));
    k_srp_transpose<<<gt, 256, 0, st>>>(X, B, D, ldx, Bp, XT);
    VR_CHECK_LAUNCH();
  }
  dim3 gs((unsigned)((k + SRP_T - 1) / SRP_T), (unsigned)(Bp / SRP_T));
  k_srp_spmm<<<gs, 256, 0, st>>>(indptr, indices, values, k, XT, B, Bp, out, ldo);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // extern "C"
