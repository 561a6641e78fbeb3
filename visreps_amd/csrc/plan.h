// Rank plan layout shared by plan.hip (construction) and engine.hip (use).
//
// A rank plan is the one-time per-RDM precompute behind every Spearman on that RDM:
// the M = n(n-1)/2 strict-upper-triangle values radix-sorted, tie groups (equal fp32
// values) marked, positions cut into chunks of ~PLAN_L pairs aligned to group starts.
#pragma once

#include "internal.h"

namespace vr {

#ifndef VR_PLAN_L
#define VR_PLAN_L 6144
#endif
// Target pairs per chunk: the per-wave work grain of the engine and the size of its
// chunk-base table (nchunks x 256 B). 6144 gives one chunk per wave at N=10k on 256 CUs
// (8192 waves) and a 2 MB table that stays in L2: 42.4 -> 36.3 ms per unit vs 2048.
constexpr uint32_t PLAN_L = VR_PLAN_L;

struct PlanHeader {
  int64_t n;
  int64_t M;
  uint32_t G;          // tie groups (device-written)
  uint32_t nchunks;
  uint32_t L;
  uint32_t has_nan;    // device-written: any NaN in the triangle
  uint32_t max_group;  // device-written: largest tie group
  uint32_t pad[55];
};
static_assert(sizeof(PlanHeader) == 256, "header size");

struct PlanView {
  PlanHeader* hdr;
  uint32_t* codes;          // [M]    (a << 16) | b, sorted by value
  uint32_t* gstart;         // [M+1]  first G+1 valid: group start positions, gstart[G] = M
  uint32_t* pos_map;        // [M]    triangle index -> sorted position (4 B: the joins'
                            //        gather table, 200 MB at N = 10k, which the 256-MB MALL
                            //        can hold across the joins that share this plan; the exact
                            //        form's A chunk follows from the position, k_join)
  uint32_t* chunk_g;        // [nchunks+1] first group of each chunk
  uint32_t* gflag;          // [(M+31)/32 + 2] bit i = position i starts a tie group
};

// Chunk length of a triangle of M pairs: PLAN_L, or for small triangles the length that gives
// ~8192 chunks (one per engine wave at 2 x 16 waves on 256 CUs; 64-pair windows, so >= 64):
// phase 1's 1000-stimulus plans (M ~ 5e5) otherwise have 82 chunks, 1 % of the waves busy.
inline uint32_t plan_chunk_len(int64_t M) {
  const int64_t per = (M + 8191) / 8192;
  const int64_t L = (per + 63) / 64 * 64;
  return (uint32_t)(L < 64 ? 64 : (L > (int64_t)PLAN_L ? (int64_t)PLAN_L : L));
}
inline uint32_t plan_nchunks(int64_t M) {
  const uint32_t L = plan_chunk_len(M);
  return (uint32_t)((M + L - 1) / L);
}

inline PlanView plan_layout(void* base, int64_t n, size_t* bytes = nullptr) {
  const int64_t M = pairs_of(n);
  Carver c(base);
  PlanView v;
  v.hdr = c.take<PlanHeader>(1);
  v.codes = c.take<uint32_t>((size_t)M);
  v.gstart = c.take<uint32_t>((size_t)M + 1);
  v.pos_map = c.take<uint32_t>((size_t)M);
  v.chunk_g = c.take<uint32_t>((size_t)plan_nchunks(M) + 1);
  v.gflag = c.take<uint32_t>((size_t)(M + 31) / 32 + 2);
  if (bytes) *bytes = c.bytes();
  return v;
}

inline size_t plan_bytes(int64_t n) {
  size_t b = 0;
  plan_layout(nullptr, n, &b);
  return b;
}

struct PlanBuildWs {
  uint32_t *keys, *keys_alt, *vals_alt, *flags, *gidx, *radix, *scan;
};

inline PlanBuildWs plan_build_layout(void* base, int64_t n, size_t* bytes) {
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

int build_plan(const float* rdm, int64_t n, int64_t ld, const PlanView& P, const PlanBuildWs& W,
               hipStream_t st);

}  // namespace vr
