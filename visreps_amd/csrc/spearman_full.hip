// Full-triangle Spearman without the rank plan's pair codes: the path of
// compute_rdm_correlation(.., "Spearman") (visreps/analysis/rsa.py:96-129: scipy spearmanr
// of the two strict upper triangles, average ranks for ties) for RDMs beyond the engine's
// 16-bit stimulus indices, up to M = n(n-1)/2 < 2^32 pairs (n <= 92681): the configs[2]
// 73k-stimulus RDM.
//
//   per RDM  k_full_keys    (sortable fp32 key, triangle index t) of every pair
//            radix_sort_kv  by key (sort.hip; u32 offsets, M < 2^32)
//            k_group_flags + scan + k_group_starts (plan.hip): tie groups
//   A        k_full_ranks   doubled midrank y = gs + ge + 1 scattered to t (u64)
//   B        k_full_dot     sum_i yB(i) * yA[t_i] (u128), tie terms sum (k^3 - k)
//            k_full_final   rho from the exact integer sums (fp64 at the end only)
// The statistic is the engine's: with M pairs and doubled midranks,
//   rho = (sum yA yB - M (M+1)^2) / sqrt(va vb),  v = 4 M(M+1)(2M+1)/6 - T/3 - M (M+1)^2.
// The same kernels are the local pieces of the distributed global rank
// (analysis/distributed_spearman.py: sample sort over ranks).
#include "window.h"

namespace vr {

// grid (column blocks, row slots): rows a = blockIdx.y, + gridDim.y, ... (a 1-D grid of
// n * n / 256 blocks would exceed the 2^32 work-items a launch dimension can address)
__global__ void k_full_keys(const float* __restrict__ rdm, int64_t n, int64_t ld,
                            uint32_t* __restrict__ keys, uint32_t* __restrict__ tidx,
                            uint32_t* __restrict__ nan_flag) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t a = blockIdx.y; a < n; a += gridDim.y) {
    if (b <= a || b >= n) continue;
    const float v = rdm[a * ld + b];
    if (v != v) atomicOr(nan_flag, 1u);
    const uint64_t t = tri_index((uint64_t)a, (uint64_t)b, (uint64_t)n);
    keys[t] = f32_sort_key(v);
    tidx[t] = (uint32_t)t;
  }
}

// the sub-RDM A[idx][:, idx]'s strict upper triangle (evals.py:362-364's `A[idx][:, idx]`, never
// materialised): pair (a, b), a < b of the k subset rows, value rdm[idx[a] * ld + idx[b]], at
// its triangle index in the k x k sub-RDM
__global__ void k_full_keys_sub(const float* __restrict__ rdm, const int32_t* __restrict__ idx, int64_t k,
                                int64_t ld, uint32_t* __restrict__ keys, uint32_t* __restrict__ tidx,
                                uint32_t* __restrict__ nan_flag) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= k) return;
  const int64_t cb = idx[b];
  for (int64_t a = blockIdx.y; a < b; a += gridDim.y) {
    const float v = rdm[(int64_t)idx[a] * ld + cb];
    if (v != v) atomicOr(nan_flag, 1u);
    const uint64_t t = tri_index((uint64_t)a, (uint64_t)b, (uint64_t)k);
    keys[t] = f32_sort_key(v);
    tidx[t] = (uint32_t)t;
  }
}

__global__ void k_group_flags_full(const uint32_t* __restrict__ keys, int64_t M,
                                   uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  flags[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ void k_group_starts_full(const uint32_t* __restrict__ flags,
                                    const uint32_t* __restrict__ gidx, int64_t M,
                                    uint32_t* __restrict__ gstart) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  if (flags[i]) gstart[gidx[i]] = (uint32_t)i;
  if (i == M - 1) gstart[gidx[i] + flags[i]] = (uint32_t)M;
}

// doubled midrank of sorted position i, its group's size (k) and whether it opens the group
__device__ inline uint64_t midrank2(const uint32_t* flags, const uint32_t* gidx,
                                    const uint32_t* gstart, int64_t i, uint64_t& k) {
  const uint32_t g = gidx[i] + flags[i] - 1u;
  const uint64_t gs = gstart[g], ge = gstart[g + 1];
  k = ge - gs;
  return gs + ge + 1u;
}

constexpr int FULL_BS = 256;

// block sum of a u128 (as two u64 words) into part[blockIdx.x]
__device__ inline void block_sum_u128(u128 v, uint64_t* part, int slot, int nslots) {
  __shared__ uint64_t lo[FULL_BS], hi[FULL_BS];
  lo[threadIdx.x] = (uint64_t)v;
  hi[threadIdx.x] = (uint64_t)(v >> 64);
  __syncthreads();
  if (threadIdx.x == 0) {
    u128 s = 0;
    for (int j = 0; j < FULL_BS; ++j) s += ((u128)hi[j] << 64) | lo[j];
    part[((size_t)blockIdx.x * nslots + slot) * 2] = (uint64_t)s;
    part[((size_t)blockIdx.x * nslots + slot) * 2 + 1] = (uint64_t)(s >> 64);
  }
  __syncthreads();
}

// A side: yA[t] = doubled midrank; tie term of every group (counted at its start position)
__global__ __launch_bounds__(FULL_BS) void k_full_ranks(
    const uint32_t* __restrict__ tidx, const uint32_t* __restrict__ flags,
    const uint32_t* __restrict__ gidx, const uint32_t* __restrict__ gstart, int64_t M,
    uint64_t* __restrict__ yA, uint64_t* __restrict__ part) {
  u128 tie = 0;
  for (int64_t i = (int64_t)blockIdx.x * FULL_BS + threadIdx.x; i < M; i += (int64_t)gridDim.x * FULL_BS) {
    uint64_t k;
    yA[tidx[i]] = midrank2(flags, gidx, gstart, i, k);
    if (flags[i]) tie += (u128)(k * k) * k - k;
  }
  block_sum_u128(tie, part, 0, 1);
}

// B side: sum over sorted B positions of yB * yA[t]; B's tie term
__global__ __launch_bounds__(FULL_BS) void k_full_dot(
    const uint32_t* __restrict__ tidx, const uint32_t* __restrict__ flags,
    const uint32_t* __restrict__ gidx, const uint32_t* __restrict__ gstart, int64_t M,
    const uint64_t* __restrict__ yA, uint64_t* __restrict__ part) {
  u128 ab = 0, tie = 0;
  for (int64_t i = (int64_t)blockIdx.x * FULL_BS + threadIdx.x; i < M; i += (int64_t)gridDim.x * FULL_BS) {
    uint64_t k;
    const uint64_t yb = midrank2(flags, gidx, gstart, i, k);
    ab += (u128)yb * yA[tidx[i]];
    if (flags[i]) tie += (u128)(k * k) * k - k;
  }
  block_sum_u128(ab, part, 0, 2);
  block_sum_u128(tie, part, 1, 2);
}

__device__ inline double i128_to_f64_full(i128 x) {
  const bool neg = x < 0;
  const u128 u = neg ? (u128)(-x) : (u128)x;
  const double d = (double)(uint64_t)(u >> 64) * 18446744073709551616.0 + (double)(uint64_t)u;
  return neg ? -d : d;
}

__global__ void k_full_final(const uint64_t* __restrict__ partA, const uint64_t* __restrict__ partB,
                             int nblk, int64_t M, const uint32_t* __restrict__ nan_flag,
                             double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  u128 tA = 0, ab = 0, tB = 0;
  for (int b = 0; b < nblk; ++b) {
    tA += ((u128)partA[2 * b + 1] << 64) | partA[2 * b];
    ab += ((u128)partB[4 * b + 1] << 64) | partB[4 * b];
    tB += ((u128)partB[4 * b + 3] << 64) | partB[4 * b + 2];
  }
  const u128 Mp = (u128)M;
  const u128 mu = Mp * (Mp + 1) * (Mp + 1);
  const u128 sq = 4 * (Mp * (Mp + 1) * (2 * Mp + 1) / 6);
  const i128 num = (i128)ab - (i128)mu;
  const i128 va = (i128)(sq - tA / 3) - (i128)mu;
  const i128 vb = (i128)(sq - tB / 3) - (i128)mu;
  double r;
  if (nan_flag[0] || nan_flag[1] || M < 2 || va <= 0 || vb <= 0) {
    r = __builtin_nan("");
  } else {
    r = i128_to_f64_full(num) / sqrt(i128_to_f64_full(va) * i128_to_f64_full(vb));
    r = r > 1.0 ? 1.0 : (r < -1.0 ? -1.0 : r);
  }
  *out = r;
}

struct FullWs {
  uint32_t *keys, *tidx, *keys_alt, *tidx_alt, *gstart, *radix, *scan, *nan;
  uint64_t *yA, *partA, *partB;
};

static int full_grid() { return num_cus() * 8; }

static FullWs full_layout(void* base, int64_t n, size_t* bytes) {
  const int64_t M = pairs_of(n);
  Carver c(base);
  FullWs w;
  w.keys = c.take<uint32_t>((size_t)M);
  w.tidx = c.take<uint32_t>((size_t)M);
  w.keys_alt = c.take<uint32_t>((size_t)M);  // after the sort: group flags
  w.tidx_alt = c.take<uint32_t>((size_t)M);  // after the sort: group index
  w.gstart = c.take<uint32_t>((size_t)M + 1);
  w.radix = c.take<uint32_t>(radix_ws_elems(M));
  w.scan = c.take<uint32_t>(scan_ws_elems(M));
  w.nan = c.take<uint32_t>(2);
  w.yA = c.take<uint64_t>((size_t)M);
  w.partA = c.take<uint64_t>((size_t)full_grid() * 2);
  w.partB = c.take<uint64_t>((size_t)full_grid() * 4);
  if (bytes) *bytes = c.bytes();
  return w;
}

// sort one RDM's triangle by value (idx: the sub-RDM of those n rows and columns); flags /
// gidx / gstart of its tie groups
static int full_sorted_groups(const float* rdm, int64_t n, int64_t ld, const FullWs& w, uint32_t* nan,
                              hipStream_t st, const int32_t* idx = nullptr) {
  const int64_t M = pairs_of(n);
  const dim3 grid((unsigned)((n + 255) / 256), (unsigned)std::min<int64_t>(n, 16384));
  if (idx)
    k_full_keys_sub<<<grid, 256, 0, st>>>(rdm, idx, n, ld, w.keys, w.tidx, nan);
  else
    k_full_keys<<<grid, 256, 0, st>>>(rdm, n, ld, w.keys, w.tidx, nan);
  VR_CHECK_LAUNCH();
  VR_TRY(radix_sort_kv(w.keys, w.tidx, w.keys_alt, w.tidx_alt, M, w.radix, st));
  const unsigned gb = (unsigned)((M + 255) / 256);
  k_group_flags_full<<<gb, 256, 0, st>>>(w.keys, M, w.keys_alt);
  VR_CHECK_LAUNCH();
  VR_TRY(scan_exclusive_u32(w.keys_alt, w.tidx_alt, M, nullptr, w.scan, st));
  k_group_starts_full<<<gb, 256, 0, st>>>(w.keys_alt, w.tidx_alt, M, w.gstart);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // namespace vr

using namespace vr;

static int spearman_full_impl(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                              double* out, void* ws, size_t ws_bytes, hipStream_t st);

extern "C" {

size_t vr_spearman_full_workspace(int64_t n) {
  if (n < 2) return 256;
  size_t b = 0;
  full_layout(nullptr, n, &b);
  return b;
}

int vr_spearman_full_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out, void* ws,
                         size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && ld >= n && out, "vr_spearman_full_f32: bad shape n=%lld ld=%lld", (long long)n,
             (long long)ld);
  return spearman_full_impl(A, B, n, ld, nullptr, out, ws, ws_bytes, as_stream(stream));
}

int vr_spearman_full_subset_f32(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                                int64_t k, double* out, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && ld >= n && k >= 0 && k <= n && out, "vr_spearman_full_subset_f32: bad shape n=%lld "
             "ld=%lld k=%lld", (long long)n, (long long)ld, (long long)k);
  VR_REQUIRE(idx != nullptr || k == 0, "vr_spearman_full_subset_f32: null idx");
  return spearman_full_impl(A, B, k, ld, idx, out, ws, ws_bytes, as_stream(stream));
}

}  // extern "C"

static int spearman_full_impl(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                              double* out, void* ws, size_t ws_bytes, hipStream_t st) {
  VR_REQUIRE(pairs_of(n) < ((int64_t)1 << 32), "vr_spearman_full_f32: n=%lld has 2^32 or more pairs",
             (long long)n);
  const int64_t M = pairs_of(n);
  if (M < 2) {  // scipy: NaN for fewer than two pairs
    const double nan = __builtin_nan("");
    VR_CHECK_HIP(hipMemcpyAsync(out, &nan, sizeof(double), hipMemcpyHostToDevice, st));
    VR_CHECK_HIP(hipStreamSynchronize(st));
    return VR_OK;
  }
  VR_REQUIRE(A && B && ws, "vr_spearman_full_f32: null pointer");
  size_t need = 0;
  const FullWs w = full_layout(ws, n, &need);
  if (ws_bytes < need) {
    set_error("vr_spearman_full_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  VR_CHECK_HIP(hipMemsetAsync(w.nan, 0, 2 * sizeof(uint32_t), st));
  const int grid = full_grid();
  VR_TRY(full_sorted_groups(A, n, ld, w, w.nan, st, idx));
  k_full_ranks<<<grid, FULL_BS, 0, st>>>(w.tidx, w.keys_alt, w.tidx_alt, w.gstart, M, w.yA, w.partA);
  VR_CHECK_LAUNCH();
  VR_TRY(full_sorted_groups(B, n, ld, w, w.nan + 1, st, idx));
  k_full_dot<<<grid, FULL_BS, 0, st>>>(w.tidx, w.keys_alt, w.tidx_alt, w.gstart, M, w.yA, w.partB);
  VR_CHECK_LAUNCH();
  k_full_final<<<1, 64, 0, st>>>(w.partA, w.partB, grid, M, w.nan, out);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

extern "C" {

// ---------------------------------------------------------------------------------
// Local pieces of the distributed global rank (analysis/distributed_spearman.py)
// ---------------------------------------------------------------------------------
size_t vr_sort_pairs_workspace(int64_t m) {
  if (m <= 1) return 256;
  Carver c(nullptr);
  c.take<uint32_t>((size_t)m);
  c.take<uint32_t>((size_t)m);
  c.take<uint32_t>(radix_ws_elems(m));
  return c.bytes();
}

int vr_sort_pairs_u32(uint32_t* keys, uint32_t* vals, int64_t m, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(m >= 0 && m < ((int64_t)1 << 32), "vr_sort_pairs_u32: m=%lld", (long long)m);
  if (m <= 1) return VR_OK;
  VR_REQUIRE(keys && vals && ws && ws_bytes >= vr_sort_pairs_workspace(m), "vr_sort_pairs_u32: workspace");
  Carver c(ws);
  uint32_t* ka = c.take<uint32_t>((size_t)m);
  uint32_t* va = c.take<uint32_t>((size_t)m);
  uint32_t* rw = c.take<uint32_t>(radix_ws_elems(m));
  return radix_sort_kv(keys, vals, ka, va, m, rw, as_stream(stream));
}

__global__ void k_sort_keys(const float* __restrict__ v, int64_t m, uint32_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) keys[i] = f32_sort_key(v[i]);
}

int vr_f32_sort_keys(const float* v, int64_t m, uint32_t* keys, void* stream) {
  VR_REQUIRE(m >= 0 && m < ((int64_t)1 << 32), "vr_f32_sort_keys: m=%lld", (long long)m);
  if (m == 0) return VR_OK;
  VR_REQUIRE(v && keys, "vr_f32_sort_keys: null pointer");
  k_sort_keys<<<(unsigned)((m + 255) / 256), 256, 0, as_stream(stream)>>>(v, m, keys);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

__global__ __launch_bounds__(FULL_BS) void k_midranks_run(const uint32_t* __restrict__ flags,
                                                           const uint32_t* __restrict__ gidx,
                                                           const uint32_t* __restrict__ gstart, int64_t m,
                                                           uint64_t base2, uint64_t* __restrict__ y,
                                                           uint64_t* __restrict__ part) {
  u128 tie = 0;
  for (int64_t i = (int64_t)blockIdx.x * FULL_BS + threadIdx.x; i < m; i += (int64_t)gridDim.x * FULL_BS) {
    uint64_t k;
    y[i] = base2 + midrank2(flags, gidx, gstart, i, k);
    if (flags[i]) tie += (u128)(k * k) * k - k;
  }
  block_sum_u128(tie, part, 0, 1);
}

__global__ __launch_bounds__(FULL_BS) void k_dot_u64(const uint64_t* __restrict__ a,
                                                      const uint64_t* __restrict__ b, int64_t m,
                                                      uint64_t* __restrict__ part) {
  u128 s = 0;
  for (int64_t i = (int64_t)blockIdx.x * FULL_BS + threadIdx.x; i < m; i += (int64_t)gridDim.x * FULL_BS)
    s += (u128)a[i] * b[i];
  block_sum_u128(s, part, 0, 1);
}

__global__ void k_sum_parts(const uint64_t* __restrict__ part, int nblk, uint64_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  u128 s = 0;
  for (int b = 0; b < nblk; ++b) s += ((u128)part[2 * b + 1] << 64) | part[2 * b];
  out[0] = (uint64_t)s;
  out[1] = (uint64_t)(s >> 64);
}

size_t vr_midranks_workspace(int64_t m) {
  Carver c(nullptr);
  c.take<uint32_t>((size_t)std::max<int64_t>(m, 1));
  c.take<uint32_t>((size_t)std::max<int64_t>(m, 1));
  c.take<uint32_t>((size_t)m + 1);
  c.take<uint32_t>(scan_ws_elems(m));
  c.take<uint64_t>((size_t)full_grid() * 2);
  return c.bytes();
}

int vr_midranks_sorted(const uint32_t* keys, int64_t m, uint64_t base, uint64_t* y, uint64_t* tie,
                       void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(m >= 0 && m < ((int64_t)1 << 32), "vr_midranks_sorted: m=%lld", (long long)m);
  VR_REQUIRE(tie && ws && ws_bytes >= vr_midranks_workspace(m), "vr_midranks_sorted: workspace");
  hipStream_t st = as_stream(stream);
  if (m == 0) {
    VR_CHECK_HIP(hipMemsetAsync(tie, 0, 2 * sizeof(uint64_t), st));
    return VR_OK;
  }
  VR_REQUIRE(keys && y, "vr_midranks_sorted: null pointer");
  Carver c(ws);
  uint32_t* flags = c.take<uint32_t>((size_t)m);
  uint32_t* gidx = c.take<uint32_t>((size_t)m);
  uint32_t* gstart = c.take<uint32_t>((size_t)m + 1);
  uint32_t* sw = c.take<uint32_t>(scan_ws_elems(m));
  uint64_t* part = c.take<uint64_t>((size_t)full_grid() * 2);
  const unsigned gb = (unsigned)((m + 255) / 256);
  k_group_flags_full<<<gb, 256, 0, st>>>(keys, m, flags);
  VR_CHECK_LAUNCH();
  VR_TRY(scan_exclusive_u32(flags, gidx, m, nullptr, sw, st));
  k_group_starts_full<<<gb, 256, 0, st>>>(flags, gidx, m, gstart);
  VR_CHECK_LAUNCH();
  k_midranks_run<<<full_grid(), FULL_BS, 0, st>>>(flags, gidx, gstart, m, 2 * base, y, part);
  VR_CHECK_LAUNCH();
  k_sum_parts<<<1, 64, 0, st>>>(part, full_grid(), tie);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

size_t vr_dot_u64_workspace(void) { return (size_t)full_grid() * 2 * sizeof(uint64_t) + 256; }

int vr_dot_u64(const uint64_t* a, const uint64_t* b, int64_t m, uint64_t* out, void* ws, size_t ws_bytes,
               void* stream) {
  VR_REQUIRE(m >= 0 && out && ws && ws_bytes >= vr_dot_u64_workspace(), "vr_dot_u64: bad arguments");
  hipStream_t st = as_stream(stream);
  uint64_t* part = static_cast<uint64_t*>(ws);
  k_dot_u64<<<full_grid(), FULL_BS, 0, st>>>(a, b, m, part);
  VR_CHECK_LAUNCH();
  k_sum_parts<<<1, 64, 0, st>>>(part, full_grid(), out);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // extern "C"
