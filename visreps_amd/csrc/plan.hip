// Rank plan construction: the once-per-RDM precompute of every Spearman on that RDM
// (replaces the per-call scipy.stats.rankdata(.., 'average') inside spearmanr,
// visreps/analysis/rsa.py:43-47,121-122).
//
//  k_triu_keys     strict upper triangle (torch.triu_indices order, rsa.py:111) ->
//                  (sortable fp32 key, pair code (a<<16)|b); NaN flag
//  radix_sort_kv   LSD radix sort by value (sort.hip)
//  k_group_flags   tie-group starts (equal keys; -0.0 == +0.0 by the key transform)
//  scan            group numbering -> G
//  k_group_starts  group start positions, largest group
//  k_pos_map       pair index -> sorted position
//  k_chunk_groups  group-aligned chunks of ~plan_chunk_len(M) positions
//  k_pack_flags    group-start bitmask read by the engine
#include "plan.h"

namespace vr {

__global__ void k_init_header(PlanHeader* hdr, int64_t n, int64_t M, uint32_t nchunks,
                              uint32_t L) {
  if (threadIdx.x == 0) {
    hdr->n = n;
    hdr->M = M;
    hdr->G = 0;
    hdr->nchunks = nchunks;
    hdr->L = L;
    hdr->has_nan = 0;
    hdr->max_group = M > 0 ? 1u : 0u;
  }
}

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

__global__ void k_group_sizes(const uint32_t* __restrict__ gstart, PlanHeader* hdr) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)hdr->G) return;
  const uint32_t sz = gstart[g + 1] - gstart[g];
  if (sz > 1) atomicMax(&hdr->max_group, sz);
}

__global__ void k_pos_map(const uint32_t* __restrict__ codes, int64_t M, int64_t n,
                          uint32_t* __restrict__ pos_map) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t c = codes[i];
  pos_map[tri_index(c >> 16, c & 0xffffu, (uint64_t)n)] = (uint32_t)i;
}

// chunk_g[c] = first group whose start position is >= c*L (group-aligned chunks).
__global__ void k_chunk_groups(const uint32_t* __restrict__ gstart,
                               const PlanHeader* __restrict__ hdr, uint32_t nchunks,
                               uint32_t L, uint32_t* __restrict__ chunk_g) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t G = hdr->G;
  if (g > G) return;
  const int64_t cg = (g == G) ? (int64_t)nchunks : (int64_t)(gstart[g] / L);
  const int64_t cp = (g == 0) ? -1 : (int64_t)(gstart[g - 1] / L);
  for (int64_t c = cp + 1; c <= cg; ++c) chunk_g[c] = (uint32_t)g;
}

// One flag per lane (coalesced reads), a wave ballot packs 64 of them into two words.
__global__ void k_pack_flags(const uint32_t* __restrict__ flags, int64_t M,
                             uint32_t* __restrict__ gflag, int64_t words) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool bit = i < M && flags[i] != 0u;
  const uint64_t b = __ballot(bit);
  const int lane = threadIdx.x & 63;
  const int64_t w = (i - lane) / 32 + (lane >> 5);  // word of this lane's half-wave
  if ((lane & 31) == 0 && w < words) gflag[w] = (uint32_t)(lane ? (b >> 32) : b);
}

int build_plan(const float* rdm, int64_t n, int64_t ld, const PlanView& P, const PlanBuildWs& W,
               hipStream_t st) {
  const int64_t M = pairs_of(n);
  const uint32_t nchunks = plan_nchunks(M);
  const uint32_t L = plan_chunk_len(M);
  k_init_header<<<1, 64, 0, st>>>(P.hdr, n, M, nchunks, L);
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
  k_group_sizes<<<gb, 256, 0, st>>>(P.gstart, P.hdr);
  VR_CHECK_LAUNCH();
  k_pos_map<<<gb, 256, 0, st>>>(P.codes, M, n, P.pos_map);
  VR_CHECK_LAUNCH();
  k_chunk_groups<<<(unsigned)((M + 1 + 255) / 256), 256, 0, st>>>(P.gstart, P.hdr, nchunks, L,
                                                                  P.chunk_g);
  VR_CHECK_LAUNCH();
  const int64_t words = (M + 31) / 32 + 2;
  k_pack_flags<<<(unsigned)((words * 32 + 255) / 256), 256, 0, st>>>(W.flags, M, P.gflag, words);
  VR_CHECK_LAUNCH();
  return VR_OK;
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

}  // extern "C"
