// Multi-GPU RDM behind the C ABI (SURVEY §8(b) vr_rdm_pearson_sharded, §8(e)): rank r of an
// RCCL communicator holds a contiguous block of stimulus rows; every rank ends with the full
// n x n RDM -- compute_rdm (visreps/analysis/rsa.py:59-93) of the concatenated rows -- without
// any PyTorch on the caller's side. The Python pipeline (visreps_amd/pipeline.py ShardedRDMs)
// schedules many RDMs over owner ranks; this entry point is the one-RDM form a C caller binds:
//
//   1. the block sizes are all-gathered (one int64 per rank), so row offsets are known;
//   2. each rank splits its rows (row statistics + bf16 hi/lo plane records,
//      vr_rdm_split_rows_f32) into a block padded to the largest block, and the blocks are
//      all-gathered (ncclAllGather over xGMI) and laid out as the full plane buffer;
//   3. each rank computes one tile range of the upper triangle, cut only at the wide kernel's
//      aligned boundaries (so every tile is bit-identical to the one-GPU launch, see
//      vr_rdm_range_aligned) with near-equal Gram cost per rank;
//   4. the ranges are packed, all-gathered and unpacked (tile + mirror) on every rank.
//
// RCCL is bound at run time (dlopen of librccl.so.1: torch's copy when torch is loaded, the
// system's otherwise) so the library has no link-time RCCL dependency; the communicator must
// come from the same RCCL (vr_rccl_comm_init, or the caller's own when they share it).
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"
#include "../../include/visreps_hip.h"

extern "C" {
int64_t vr_rdm_tile_count(int64_t n);
int64_t vr_rdm_wide_rows(int64_t n, int64_t d);
int64_t vr_rdm_tile_cost(int64_t n, int64_t tile);
int64_t vr_rdm_plane_rows(int64_t n);
size_t vr_rdm_plane_row_bytes(int64_t d);
int vr_rdm_split_rows_f32(const float* X, int64_t rows, int64_t d, int64_t ldx, float correction, float* mean,
                          float* stdv, uint16_t* planes, void* stream);
size_t vr_rdm_planes_tiles_workspace(int64_t n, int64_t d, int64_t tile_begin, int64_t tile_end);
int vr_rdm_pearson_tiles_planes(const uint16_t* planes, const float* mean, const float* stdv, int64_t n, int64_t d,
                                float* rdm, int64_t ldr, float correction, int64_t tile_begin, int64_t tile_end,
                                void* ws, size_t ws_bytes, void* stream);
int vr_rdm_tiles_pack(const float* rdm, int64_t ldr, int64_t n, int64_t tile_begin, int64_t tile_end, float* packed,
                      void* stream);
int vr_rdm_tiles_unpack(const float* packed, int64_t n, int64_t tile_begin, int64_t tile_end, float* rdm,
                        int64_t ldr, void* stream);
}

namespace vr {
namespace {

// the RCCL entry points used here (rccl.h: ncclResult_t is an int enum, ncclInt8 = 0)
struct Rccl {
  int (*get_unique_id)(void*) = nullptr;
  int (*comm_init_rank)(void**, int, const char*, int) = nullptr;  // ncclUniqueId passed by value: see call
  int (*comm_destroy)(void*) = nullptr;
  int (*all_gather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  const char* (*error_string)(int) = nullptr;
  bool ok = false;
};
constexpr int NCCL_INT8 = 0;
constexpr int UNIQUE_ID_BYTES = 128;
struct UniqueId {
  char internal[UNIQUE_ID_BYTES];
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // already loaded (torch's copy)
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    r.get_unique_id = reinterpret_cast<int (*)(void*)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<int (*)(void**, int, const char*, int)>(dlsym(h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<int (*)(void*)>(dlsym(h, "ncclCommDestroy"));
    r.all_gather =
        reinterpret_cast<int (*)(const void*, void*, size_t, int, void*, hipStream_t)>(dlsym(h, "ncclAllGather"));
    r.error_string = reinterpret_cast<const char* (*)(int)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.error_string;
  });
  return r;
}

#define VR_RCCL(expr)                                                                             \
  do {                                                                                            \
    const int rc_ = (expr);                                                                       \
    if (rc_ != 0) {                                                                               \
      set_error("%s failed: %s (%s:%d)", #expr, rccl().error_string(rc_), __FILE__, __LINE__);    \
      return VR_EHIP;                                                                             \
    }                                                                                             \
  } while (0)

int64_t tri_start(int64_t r, int64_t T) { return r * T - r * (r - 1) / 2; }

// Tile range of every rank: cut only at aligned boundaries (the wide kernel's super-tile row
// starts tri_start(2r, T), r <= R, and the end of the triangle), each cut the boundary closest
// to an equal share of the Gram cost (pipeline.assign_grams' rule for a piece count = world).
std::vector<int64_t> rank_cuts(int64_t n, int64_t d, int world) {
  const int64_t total = vr_rdm_tile_count(n);
  std::vector<int64_t> cuts(world + 1, total);
  cuts[0] = 0;
  if (world == 1 || total == 0) return cuts;
  std::vector<double> cum(total + 1, 0.0);
  for (int64_t t = 0; t < total; ++t) cum[t + 1] = cum[t] + (double)vr_rdm_tile_cost(n, t);
  const int64_t R = d > 0 ? vr_rdm_wide_rows(n, d) : 0;
  const int64_t T = (n + 127) / 128;
  std::vector<int64_t> bnd;
  if (R > 0)
    for (int64_t r = 0; r <= R; ++r) bnd.push_back(tri_start(2 * r, T));
  else
    bnd.push_back(0);
  bnd.push_back(total);
  std::sort(bnd.begin(), bnd.end());
  bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
  for (int r = 1; r < world; ++r) {
    const double target = cum[total] * r / world;
    int64_t best = bnd.front();
    for (int64_t b : bnd)
      if (std::abs(cum[b] - target) < std::abs(cum[best] - target)) best = b;
    cuts[r] = std::max(best, cuts[r - 1]);  // monotone; an empty range is allowed
  }
  return cuts;
}

struct ShardLayout {
  size_t row_bytes;     // plane bytes per row
  int64_t maxc;         // rows per rank block (padded)
  int64_t prow;         // plane rows of the full buffer
  int64_t maxt;         // tiles per rank block (padded)
  size_t tiles_ws;      // the largest rank range's tile workspace
  std::vector<int64_t> cuts;
};

ShardLayout shard_layout(int64_t n, int64_t d, int world) {
  ShardLayout L;
  L.row_bytes = vr_rdm_plane_row_bytes(d);
  L.maxc = (n + world - 1) / world;
  L.prow = vr_rdm_plane_rows(n);
  L.cuts = rank_cuts(n, d, world);
  L.maxt = 0;
  L.tiles_ws = 256;
  for (int r = 0; r < world; ++r) {
    L.maxt = std::max<int64_t>(L.maxt, L.cuts[r + 1] - L.cuts[r]);
    L.tiles_ws = std::max(L.tiles_ws, vr_rdm_planes_tiles_workspace(n, d, L.cuts[r], L.cuts[r + 1]));
  }
  return L;
}

struct ShardWs {
  int64_t* counts;   // [world] block sizes (device)
  char* send;        // [maxc rows] local plane block | [maxc][2] stats
  char* recv;        // [world][maxc rows] ... | [world][maxc][2]
  uint16_t* planes;  // [prow rows] full planes
  float* mean;       // [n]
  float* stdv;       // [n]
  float* psend;      // [maxt][128 * 128]
  float* precv;      // [world][maxt][128 * 128]
  void* tws;         // tile workspace
  size_t block_bytes;
};

ShardWs shard_ws(void* base, const ShardLayout& L, int64_t n, int world, size_t* bytes) {
  Carver c(base);
  ShardWs w;
  w.block_bytes = (size_t)L.maxc * (L.row_bytes + 2 * sizeof(float));
  w.counts = c.take<int64_t>((size_t)world);
  w.send = c.take<char>(w.block_bytes);
  w.recv = c.take<char>(w.block_bytes * (size_t)world);
  w.planes = c.take<uint16_t>((size_t)L.prow * L.row_bytes / sizeof(uint16_t));
  w.mean = c.take<float>((size_t)n);
  w.stdv = c.take<float>((size_t)n);
  w.psend = c.take<float>((size_t)std::max<int64_t>(L.maxt, 1) * 128 * 128);
  w.precv = c.take<float>((size_t)std::max<int64_t>(L.maxt, 1) * 128 * 128 * (size_t)world);
  w.tws = c.take<char>(L.tiles_ws);
  if (bytes) *bytes = c.bytes();
  return w;
}

// interleave [mean, std] pairs of the local rows into the block's stats region
__global__ void k_pack_stats(const float* __restrict__ mean, const float* __restrict__ stdv, int64_t rows,
                             float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < rows) {
    out[2 * i] = mean[i];
    out[2 * i + 1] = stdv[i];
  }
}
__global__ void k_unpack_stats(const float* __restrict__ in, int64_t rows, float* __restrict__ mean,
                               float* __restrict__ stdv) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < rows) {
    mean[i] = in[2 * i];
    stdv[i] = in[2 * i + 1];
  }
}

// vr_comm's all_gather over RCCL: user = the ncclComm_t
int rccl_all_gather(const void* send, void* recv, size_t bytes, void* user, void* stream) {
  const int rc = rccl().all_gather(send, recv, bytes, NCCL_INT8, user, as_stream(stream));
  if (rc != 0) set_error("ncclAllGather failed: %s", rccl().error_string(rc));
  return rc;
}

#define VR_ALLGATHER(C, send, recv, bytes, stream)                                                  \
  do {                                                                                              \
    clear_error();                                                                                  \
    const int rc_ = (C)->all_gather((send), (recv), (bytes), (C)->user, (stream));                  \
    if (rc_ != 0) {                                                                                 \
      if (vr_last_error()[0] == 0) set_error("vr_comm all_gather failed (rc %d, %s:%d)", rc_, __FILE__, __LINE__); \
      return VR_EHIP;                                                                               \
    }                                                                                               \
  } while (0)

}  // namespace
}  // namespace vr

using namespace vr;

extern "C" {

int vr_rccl_available(void) { return rccl().ok ? 1 : 0; }

int vr_rccl_unique_id(void* out) {
  VR_REQUIRE(out != nullptr, "vr_rccl_unique_id: null out");
  VR_REQUIRE(rccl().ok, "vr_rccl_unique_id: librccl.so.1 not found");
  VR_RCCL(rccl().get_unique_id(out));
  return VR_OK;
}

int vr_rccl_comm_init(void** comm, int world, const void* unique_id, int rank) {
  VR_REQUIRE(comm && unique_id && world >= 1 && rank >= 0 && rank < world, "vr_rccl_comm_init: bad arguments");
  VR_REQUIRE(rccl().ok, "vr_rccl_comm_init: librccl.so.1 not found");
  // ncclCommInitRank(ncclComm_t*, int nranks, ncclUniqueId commId, int rank): the 128-byte id
  // is passed by value
  UniqueId id;
  std::memcpy(id.internal, unique_id, UNIQUE_ID_BYTES);
  auto fn = reinterpret_cast<int (*)(void**, int, UniqueId, int)>(rccl().comm_init_rank);
  VR_RCCL(fn(comm, world, id, rank));
  return VR_OK;
}

int vr_rccl_comm_destroy(void* comm) {
  if (comm == nullptr) return VR_OK;
  VR_REQUIRE(rccl().ok, "vr_rccl_comm_destroy: librccl.so.1 not found");
  VR_RCCL(rccl().comm_destroy(comm));
  return VR_OK;
}

int vr_rdm_sharded_range(int64_t n, int64_t d, int world, int rank, int64_t* tile_begin, int64_t* tile_end) {
  VR_REQUIRE(n >= 0 && d >= 0 && world >= 1 && rank >= 0 && rank < world && tile_begin && tile_end,
             "vr_rdm_sharded_range: bad arguments");
  const std::vector<int64_t> cuts = rank_cuts(n, d, world);
  *tile_begin = cuts[rank];
  *tile_end = cuts[rank + 1];
  return VR_OK;
}

size_t vr_rdm_sharded_workspace(int64_t n, int64_t d, int world) {
  if (n <= 0 || d <= 0 || world < 1) return 256;
  size_t b = 0;
  shard_ws(nullptr, shard_layout(n, d, world), n, world, &b);
  return b;
}

int vr_comm_rccl(vr_comm* out, void* nccl_comm, int world, int rank) {
  VR_REQUIRE(out && nccl_comm && world >= 1 && rank >= 0 && rank < world, "vr_comm_rccl: bad arguments");
  VR_REQUIRE(rccl().ok, "vr_comm_rccl: librccl.so.1 not found");
  out->world = world;
  out->rank = rank;
  out->all_gather = rccl_all_gather;
  out->user = nccl_comm;
  return VR_OK;
}

int vr_rdm_pearson_sharded(const float* X_local, int64_t rows_local, int64_t n, int64_t d, int64_t ldx,
                           float* rdm, int64_t ldr, float correction, void* comm, int rank, int world, void* ws,
                           size_t ws_bytes, void* stream) {
  clear_error();
  VR_REQUIRE(comm != nullptr, "vr_rdm_pearson_sharded: null comm");
  vr_comm c;
  VR_TRY(vr_comm_rccl(&c, comm, world, rank));
  return vr_rdm_pearson_sharded_comm(X_local, rows_local, n, d, ldx, rdm, ldr, correction, &c, ws, ws_bytes, stream);
}

int vr_rdm_pearson_sharded_comm(const float* X_local, int64_t rows_local, int64_t n, int64_t d, int64_t ldx,
                                float* rdm, int64_t ldr, float correction, const vr_comm* C, void* ws,
                                size_t ws_bytes, void* stream) {
  clear_error();
  VR_REQUIRE(C != nullptr && C->all_gather != nullptr, "vr_rdm_pearson_sharded: null comm table");
  const int world = C->world, rank = C->rank;
  VR_REQUIRE(n >= 1 && d >= 1 && ldx >= d && ldr >= n && world >= 1 && rank >= 0 && rank < world,
             "vr_rdm_pearson_sharded: bad shape n=%lld d=%lld world=%d rank=%d", (long long)n, (long long)d, world,
             rank);
  VR_REQUIRE(rows_local >= 0 && rows_local <= (n + world - 1) / world,
             "vr_rdm_pearson_sharded: %lld local rows (blocks hold at most ceil(n / world) = %lld)",
             (long long)rows_local, (long long)((n + world - 1) / world));
  VR_REQUIRE(rdm && ws && (rows_local == 0 || X_local), "vr_rdm_pearson_sharded: null pointer");
  const ShardLayout L = shard_layout(n, d, world);
  size_t need = 0;
  const ShardWs W = shard_ws(ws, L, n, world, &need);
  if (ws_bytes < need) {
    set_error("vr_rdm_pearson_sharded: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  // 1. block sizes -> row offsets (host)
  VR_CHECK_HIP(hipMemcpyAsync(W.counts + rank, &rows_local, sizeof(int64_t), hipMemcpyHostToDevice, st));
  VR_ALLGATHER(C, W.counts + rank, W.counts, sizeof(int64_t), stream);
  std::vector<int64_t> counts((size_t)world);
  VR_CHECK_HIP(hipMemcpyAsync(counts.data(), W.counts, counts.size() * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  VR_CHECK_HIP(hipStreamSynchronize(st));
  int64_t sum = 0;
  for (int64_t c : counts) {
    VR_REQUIRE(c >= 0 && c <= L.maxc, "vr_rdm_pearson_sharded: a rank holds %lld rows", (long long)c);
    sum += c;
  }
  VR_REQUIRE(sum == n, "vr_rdm_pearson_sharded: blocks hold %lld rows, n = %lld", (long long)sum, (long long)n);
  // 2. split the local rows into the send block, all-gather the blocks, lay out the planes
  uint16_t* lplanes = reinterpret_cast<uint16_t*>(W.send);
  float* lstats = reinterpret_cast<float*>(W.send + (size_t)L.maxc * L.row_bytes);
  if (rows_local > 0) {
    // the row statistics go to this rank's slice of mean / stdv first (scratch), then into the block
    VR_TRY(vr_rdm_split_rows_f32(X_local, rows_local, d, ldx, correction, W.mean, W.stdv, lplanes, stream));
    k_pack_stats<<<(unsigned)((rows_local + 255) / 256), 256, 0, st>>>(W.mean, W.stdv, rows_local, lstats);
    VR_CHECK_LAUNCH();
  }
  VR_ALLGATHER(C, W.send, W.recv, W.block_bytes, stream);
  int64_t off = 0;
  for (int r = 0; r < world; ++r) {
    const char* blk = W.recv + (size_t)r * W.block_bytes;
    if (counts[(size_t)r] > 0) {
      VR_CHECK_HIP(hipMemcpyAsync(reinterpret_cast<char*>(W.planes) + (size_t)off * L.row_bytes, blk,
                                  (size_t)counts[(size_t)r] * L.row_bytes, hipMemcpyDeviceToDevice, st));
      k_unpack_stats<<<(unsigned)((counts[(size_t)r] + 255) / 256), 256, 0, st>>>(
          reinterpret_cast<const float*>(blk + (size_t)L.maxc * L.row_bytes), counts[(size_t)r], W.mean + off,
          W.stdv + off);
      VR_CHECK_LAUNCH();
    }
    off += counts[(size_t)r];
  }
  if (L.prow > n)  // the kernels read whole super-tile rows: padding rows are exact zeros
    VR_CHECK_HIP(hipMemsetAsync(reinterpret_cast<char*>(W.planes) + (size_t)n * L.row_bytes, 0,
                                (size_t)(L.prow - n) * L.row_bytes, st));
  // 3. this rank's aligned tile range
  const int64_t t0 = L.cuts[(size_t)rank], t1 = L.cuts[(size_t)rank + 1];
  VR_TRY(vr_rdm_pearson_tiles_planes(W.planes, W.mean, W.stdv, n, d, rdm, ldr, correction, t0, t1, W.tws, L.tiles_ws,
                                     stream));
  // 4. exchange the packed ranges, unpack the others' (tile + mirror)
  if (world > 1) {
    const size_t tile_floats = 128 * 128;
    if (t1 > t0) VR_TRY(vr_rdm_tiles_pack(rdm, ldr, n, t0, t1, W.psend, stream));
    VR_ALLGATHER(C, W.psend, W.precv, (size_t)std::max<int64_t>(L.maxt, 1) * tile_floats * sizeof(float), stream);
    for (int r = 0; r < world; ++r) {
      const int64_t a = L.cuts[(size_t)r], b = L.cuts[(size_t)r + 1];
      if (r == rank || b <= a) continue;
      VR_TRY(vr_rdm_tiles_unpack(W.precv + (size_t)r * std::max<int64_t>(L.maxt, 1) * tile_floats, n, a, b, rdm, ldr,
                                 stream));
    }
  }
  return VR_OK;
}

}  // extern "C"
