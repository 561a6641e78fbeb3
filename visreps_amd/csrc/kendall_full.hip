// Kendall tau-a without rank plans or subsets: long vectors (rsa.py:22-40 `_kendall_tau_a(x, y)`
// on any number of elements) and the strict upper triangles of RDMs beyond the rank plans'
// 16-bit stimulus indices (compute_rdm_correlation(.., "Kendall") at n > 65,535, up to
// M = n(n-1)/2 < 2^32 elements: configs[2]'s 73k-stimulus RDM).
//
// scipy.stats.kendalltau's tau-b (scipy/stats/_stats_py.py) from exact integers, then the
// reference's tau-a conversion, in k_kfinal's fp64 operation order (kendall.hip):
//   1  sort (y key, index) by y               radix_sort_kv (sort.hip)
//      dense y rank r of every sorted position, y tie pairs (sum over groups of C(k, 2))
//      (the x keys ride along as the sort's payload)
//   2  stable sort of those dense y ranks by their x keys: the (x, y)-lexicographic order
//      with the sequence of y ranks r; x tie pairs and joint (x, y) tie pairs
//   3  discordant pairs = inversions of that r sequence, counted bit by bit of r from the top
//      (an MSD binary radix split: at level b the sequence is stably ordered by r >> (b+1);
//      a pair i < j with r_i > r_j has its highest differing bit at exactly one level, where
//      it is a (1, 0) pair of bit b inside one bucket of equal r >> (b+1)). Per level three
//      streaming passes over 4096-element tiles: ones of bit b per tile and bucket starts;
//      the tiles' prefix; the ones before every bucket start; then per element the ones
//      before it in its bucket (added to the count when its own bit is 0) and its place in
//      the next level (zeros of the bucket first, then ones, each in order).
// For f64 vectors the keys are 64-bit: each is first mapped to its dense rank (two stable
// 32-bit sorts), then the same u32 pipeline runs. All counts are exact integers.
#include "internal.h"
#include "window.h"

namespace vr {

constexpr int KF_BS = 256;
constexpr int KF_IPT = 16;
constexpr int KF_TILE = KF_BS * KF_IPT;
constexpr int KF_GRID = 2048;  // grid-stride kernels (tie sums)
enum { KFP_XT = 0, KFP_YT, KFP_NT, KFP_N };

__host__ __device__ inline int64_t kf_tiles(int64_t m) { return (m + KF_TILE - 1) / KF_TILE; }

struct KfWs {
  uint32_t *kx, *ky;               // [m] the two vectors' u32 keys (sortable f32 bits or dense ranks)
  uint32_t *a, *b, *c, *d;         // [m] sort buffers, then the level streams and bucket tables
  uint32_t *flags, *gidx, *gstart; // [m], [m], [m + 1] tie groups of a sorted sequence
  uint32_t *radix, *scan, *tile;   // sort / scan scratch; [tiles + 64] level tile counts
  uint32_t *tot;                   // [4] scan totals (groups, ones)
  uint32_t *nan;                   // [1]
  uint64_t *tpart;                 // [KFP_N][KF_GRID] tie-pair block sums
  uint64_t *dpart;                 // [tiles] discordant pairs per tile (summed over levels)
};

static KfWs kf_layout(void* base, int64_t m, size_t* bytes) {
  Carver c(base);
  KfWs w;
  const size_t M = (size_t)std::max<int64_t>(m, 1);
  w.kx = c.take<uint32_t>(M);
  w.ky = c.take<uint32_t>(M);
  w.a = c.take<uint32_t>(M);
  w.b = c.take<uint32_t>(M);
  w.c = c.take<uint32_t>(M);
  w.d = c.take<uint32_t>(M);
  w.flags = c.take<uint32_t>(M);
  w.gidx = c.take<uint32_t>(M);
  w.gstart = c.take<uint32_t>(M + 1);
  w.radix = c.take<uint32_t>(radix_ws_elems((int64_t)M));
  w.scan = c.take<uint32_t>(scan_ws_elems((int64_t)M));
  w.tile = c.take<uint32_t>((size_t)kf_tiles((int64_t)M) + 64);
  w.tot = c.take<uint32_t>(4);
  w.nan = c.take<uint32_t>(1);
  w.tpart = c.take<uint64_t>((size_t)KFP_N * KF_GRID);
  w.dpart = c.take<uint64_t>((size_t)kf_tiles((int64_t)M));
  if (bytes) *bytes = c.bytes();
  return w;
}

// --------------------------------------------------------------------------- keys
// both RDMs' strict upper triangles in triu order; grid (column blocks, row slots)
__global__ void k_kf_tri_keys(const float* __restrict__ A, const float* __restrict__ B, int64_t n, int64_t ld,
                              uint32_t* __restrict__ kx, uint32_t* __restrict__ ky, uint32_t* __restrict__ nan) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t a = blockIdx.y; a < n; a += gridDim.y) {
    if (b <= a || b >= n) continue;
    const float x = A[a * ld + b], y = B[a * ld + b];
    if (x != x || y != y) *nan = 1u;  // benign race: every writer stores 1
    const uint64_t t = tri_index((uint64_t)a, (uint64_t)b, (uint64_t)n);
    kx[t] = f32_sort_key(x);
    ky[t] = f32_sort_key(y);
  }
}

// the same for the sub-RDMs A[idx][:, idx], B[idx][:, idx] (a bootstrap draw, never materialised)
__global__ void k_kf_tri_keys_sub(const float* __restrict__ A, const float* __restrict__ B,
                                  const int32_t* __restrict__ idx, int64_t k, int64_t ld, uint32_t* __restrict__ kx,
                                  uint32_t* __restrict__ ky, uint32_t* __restrict__ nan) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= k) return;
  const int64_t cb = idx[b];
  for (int64_t a = blockIdx.y; a < b; a += gridDim.y) {
    const int64_t o = (int64_t)idx[a] * ld + cb;
    const float x = A[o], y = B[o];
    if (x != x || y != y) *nan = 1u;
    const uint64_t t = tri_index((uint64_t)a, (uint64_t)b, (uint64_t)k);
    kx[t] = f32_sort_key(x);
    ky[t] = f32_sort_key(y);
  }
}

// f64 -> ascending-order u64 split in (hi, lo); -0.0 as +0.0 (they tie in scipy)
__global__ void k_kf_keys64(const double* __restrict__ v, int64_t m, uint32_t* __restrict__ hi,
                            uint32_t* __restrict__ lo, uint32_t* __restrict__ nan) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const double x = v[i];
  if (x != x) *nan = 1u;
  uint64_t u = (uint64_t)__double_as_longlong(x);
  if (u == 0x8000000000000000ull) u = 0ull;
  u = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
  hi[i] = (uint32_t)(u >> 32);
  lo[i] = (uint32_t)u;
}

__global__ void k_kf_iota(uint32_t* __restrict__ v, int64_t m) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) v[i] = (uint32_t)i;
}

// dst[i] = src[idx[i]]
__global__ void k_kf_gather(const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx, int64_t m,
                            uint32_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) dst[i] = src[idx[i]];
}

// group starts of a sorted sequence of keys (k2 non-null: of (k1, k2) pairs)
__global__ void k_kf_flags(const uint32_t* __restrict__ k1, const uint32_t* __restrict__ k2, int64_t m,
                           uint32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  bool s = i == 0 || k1[i] != k1[i - 1];
  if (k2 != nullptr) s = s || (i > 0 && k2[i] != k2[i - 1]);
  flags[i] = s ? 1u : 0u;
}

// gstart[g] = first position of group g (gidx: exclusive scan of flags)
__global__ void k_kf_starts(const uint32_t* __restrict__ flags, const uint32_t* __restrict__ gidx, int64_t m,
                            uint32_t* __restrict__ gstart) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m && flags[i]) gstart[gidx[i]] = (uint32_t)i;
}

// dense rank (group index) of sorted position i
__device__ inline uint32_t kf_rank(const uint32_t* flags, const uint32_t* gidx, int64_t i) {
  return gidx[i] + flags[i] - 1u;
}

// sum over groups of C(k, 2) = sum over positions of (position - its group's start): block sums
__global__ __launch_bounds__(KF_BS) void k_kf_tie_pairs(const uint32_t* __restrict__ flags,
                                                        const uint32_t* __restrict__ gidx,
                                                        const uint32_t* __restrict__ gstart, int64_t m,
                                                        uint64_t* __restrict__ part) {
  __shared__ uint64_t red[KF_BS / 64];
  uint64_t s = 0;
  for (int64_t i = (int64_t)blockIdx.x * KF_BS + threadIdx.x; i < m; i += (int64_t)gridDim.x * KF_BS)
    s += (uint64_t)i - gstart[kf_rank(flags, gidx, i)];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// dense y rank of every y-sorted position: the sort payload of step 2
__global__ void k_kf_yrank(const uint32_t* __restrict__ flags, const uint32_t* __restrict__ gidx, int64_t m,
                           uint32_t* __restrict__ r) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) r[i] = kf_rank(flags, gidx, i);
}

// dense ranks back to element order: rank[order[i]] = rank of sorted position i
__global__ void k_kf_scatter_rank(const uint32_t* __restrict__ order, const uint32_t* __restrict__ flags,
                                  const uint32_t* __restrict__ gidx, int64_t m, uint32_t* __restrict__ rank) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) rank[order[i]] = kf_rank(flags, gidx, i);
}

// --------------------------------------------------------------------------- levels
__device__ inline uint32_t kf_bucket(uint32_t r, int b) { return b >= 31 ? 0u : r >> (b + 1); }

// ones of bit b per tile; bucket starts (bstart[g] = first position of bucket g)
__global__ __launch_bounds__(KF_BS) void k_kf_lvl_count(const uint32_t* __restrict__ cur, int64_t m, int b,
                                                        uint32_t* __restrict__ tile, uint32_t* __restrict__ bstart) {
  __shared__ uint32_t red[KF_BS / 64];
  const int64_t base = (int64_t)blockIdx.x * KF_TILE;
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < KF_IPT; ++j) {
    const int64_t i = base + (int64_t)j * KF_BS + threadIdx.x;
    if (i < m) {
      const uint32_t v = cur[i];
      s += (v >> b) & 1u;
      const uint32_t g = kf_bucket(v, b);
      if (i == 0 || kf_bucket(cur[i - 1], b) != g) bstart[g] = (uint32_t)i;
    }
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tile[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

#ifndef VR_KF_LV_BS
#define VR_KF_LV_BS 512
#endif
// the level kernels' blocks: LV_BS threads x LV_IPT consecutive elements = one KF_TILE
constexpr int LV_BS = VR_KF_LV_BS;
constexpr int LV_IPT = KF_TILE / LV_BS;
static_assert(LV_BS * LV_IPT == KF_TILE, "level tile");

// The tile in LDS: loaded striped (each load instruction one coalesced 256-element row), read
// back blocked (LV_IPT consecutive elements per thread) through the padded index, which keeps
// both patterns free of bank conflicts.
constexpr int KF_PAD = KF_TILE + KF_TILE / 32;
__device__ inline void kf_stage(const uint32_t* __restrict__ cur, int64_t m, uint32_t* sv, uint32_t (&v)[LV_IPT],
                                int64_t& i0) {
  const int64_t base = (int64_t)blockIdx.x * KF_TILE;
#pragma unroll
  for (int j = 0; j < LV_IPT; ++j) {
    const int q = j * LV_BS + (int)threadIdx.x;
    sv[lds_pad(q)] = base + q < m ? cur[base + q] : 0u;
  }
  __syncthreads();
  i0 = base + (int64_t)threadIdx.x * LV_IPT;
#pragma unroll
  for (int j = 0; j < LV_IPT; ++j) v[j] = sv[lds_pad((int)threadIdx.x * LV_IPT + j)];
}

// this thread's LV_IPT consecutive elements of the tile (staged) and the ones of bit b before
// each (tile prefix + block scan); tot <- the tile's ones
__device__ inline void kf_tile_scan(const uint32_t* __restrict__ cur, int64_t m, int b, uint32_t tile_pre,
                                    uint32_t (&v)[LV_IPT], uint32_t (&p)[LV_IPT], int64_t& i0, uint32_t* lds,
                                    uint32_t* sv, uint32_t& tot) {
  kf_stage(cur, m, sv, v, i0);
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < LV_IPT; ++j) {
    p[j] = s;
    s += i0 + j < m ? (v[j] >> b) & 1u : 0u;
  }
  const uint32_t run = block_exclusive_scan<LV_BS>(s, lds, tot) + tile_pre;
#pragma unroll
  for (int j = 0; j < LV_IPT; ++j) p[j] += run;
}

// ones before every bucket start: bP[g]
__global__ __launch_bounds__(LV_BS) void k_kf_lvl_bucket(const uint32_t* __restrict__ cur, int64_t m, int b,
                                                         const uint32_t* __restrict__ tile,
                                                         uint32_t* __restrict__ bP) {
  __shared__ uint32_t lds[LV_BS / 64 + 1];
  __shared__ uint32_t sv[KF_PAD];
  uint32_t v[LV_IPT], p[LV_IPT], tot;
  int64_t i0;
  kf_tile_scan(cur, m, b, tile[blockIdx.x], v, p, i0, lds, sv, tot);
  // the element before this thread's first: the previous thread's last (LDS) or the tile's
  // predecessor (global)
  const uint32_t prev = threadIdx.x > 0 ? sv[lds_pad((int)threadIdx.x * LV_IPT - 1)] : (i0 > 0 ? cur[i0 - 1] : 0u);
#pragma unroll
  for (int j = 0; j < LV_IPT; ++j) {
    const int64_t i = i0 + j;
    if (i >= m) break;
    const uint32_t g = kf_bucket(v[j], b);
    const uint32_t gp = j > 0 ? kf_bucket(v[j - 1], b) : (i > 0 ? kf_bucket(prev, b) : ~0u);
    if (i == 0 || gp != g) bP[g] = p[j];
  }
}

// inversions of this level (ones before each zero inside its bucket) into dpart[tile]; the
// next level's stream (per bucket: zeros, then ones, each in order) unless last. The tile's
// elements are first put in their output order inside the tile (per bucket segment of the
// tile: its zeros, then its ones) with their destinations, then written out striped: each
// store instruction covers runs of consecutive destinations.
__global__ __launch_bounds__(LV_BS) void k_kf_lvl_split(const uint32_t* __restrict__ cur, int64_t m, int b,
                                                        const uint32_t* __restrict__ tile,
                                                        const uint32_t* __restrict__ bstart,
                                                        const uint32_t* __restrict__ bP, uint32_t nbk,
                                                        const uint32_t* __restrict__ ones_total,
                                                        uint32_t* __restrict__ next, uint64_t* __restrict__ dpart) {
  __shared__ uint32_t lds[LV_BS / 64 + 1];
  __shared__ uint64_t red[LV_BS / 64];
  __shared__ uint32_t sv[KF_PAD], sb[KF_PAD], sp[KF_TILE + 2];
  uint32_t* sd = sb;  // the destinations, once the bucket table is read
  uint32_t v[LV_IPT], p[LV_IPT], tot;
  int64_t i0;
  const uint32_t tpre = tile[blockIdx.x];
  kf_tile_scan(cur, m, b, tpre, v, p, i0, lds, sv, tot);
  const uint32_t P_all = *ones_total;
  const int64_t tb = (int64_t)blockIdx.x * KF_TILE;
  const int64_t te = tb + KF_TILE < m ? tb + KF_TILE : m;
  // the tile's buckets are one contiguous range [gf, gl] (the stream is ordered by bucket):
  // their starts and ones-before, and the next bucket's, staged into LDS with striped loads
  const uint32_t gf = kf_bucket(sv[lds_pad(0)], b), gl = kf_bucket(sv[lds_pad((int)(te - tb) - 1)], b);
  const int nt = (int)(gl - gf) + 2;
  for (int x = (int)threadIdx.x; x < nt; x += LV_BS) {
    const uint32_t g = gf + (uint32_t)x;
    sb[x] = g < nbk ? bstart[g] : (uint32_t)m;
    sp[x] = g < nbk ? bP[g] : P_all;
  }
  __syncthreads();
  uint64_t dis = 0;
  uint32_t q[LV_IPT], dst[LV_IPT];
#pragma unroll
  for (int j = 0; j < LV_IPT; ++j) {
    const int64_t i = i0 + j;
    if (i >= m) break;
    const uint32_t g = kf_bucket(v[j], b);
    const uint32_t s = sb[g - gf], Ps = sp[g - gf];
    const uint32_t before = p[j] - Ps;  // ones of bit b before i in its bucket
    const bool one = (v[j] >> b) & 1u;
    if (!one) dis += before;
    if (next != nullptr) {
      const uint32_t e = sb[g + 1 - gf];
      const uint32_t Pe = sp[g + 1 - gf];
      dst[j] = !one ? (uint32_t)i - before                           // bucket start + zeros before
                    : s + ((e - s) - (Pe - Ps)) + before;           // after the bucket's zeros
      // the bucket's segment [seg0, seg1) of this tile, its ones, and i's place in it
      const int64_t seg0 = (int64_t)s > tb ? (int64_t)s : tb, seg1 = (int64_t)e < te ? (int64_t)e : te;
      const uint32_t P0 = (int64_t)s >= tb ? Ps : tpre;
      const uint32_t P1 = (int64_t)e < te ? Pe : tpre + tot;
      const uint32_t ob = p[j] - P0;  // ones before i in the segment
      const uint32_t zs = (uint32_t)(seg1 - seg0) - (P1 - P0);
      q[j] = (uint32_t)(seg0 - tb) + (one ? zs + ob : (uint32_t)(i - seg0) - ob);
    }
  }
  if (next != nullptr) {
    __syncthreads();  // every thread has read its staged elements
#pragma unroll
    for (int j = 0; j < LV_IPT; ++j) {
      if (i0 + j >= m) break;
      sv[lds_pad((int)q[j])] = v[j];
      sd[lds_pad((int)q[j])] = dst[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < LV_IPT; ++j) {
      const int r = j * LV_BS + (int)threadIdx.x;
      if (tb + r < m) next[sd[lds_pad(r)]] = sv[lds_pad(r)];
    }
  }
  for (int o = 32; o > 0; o >>= 1) dis += __shfl_xor(dis, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = dis;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
#pragma unroll
    for (int w = 0; w < LV_BS / 64; ++w) t += red[w];
    dpart[blockIdx.x] += t;
  }
}

// tau-a from the exact counts: k_kfinal's fp64 order (kendall.hip) for one set of m elements
__global__ void k_kf_final(const uint64_t* __restrict__ tpart, const uint64_t* __restrict__ dpart, int64_t ntiles,
                           int64_t m, const uint32_t* __restrict__ nan, double* __restrict__ out) {
  __shared__ uint64_t red[4][KF_BS / 64];
  uint64_t s[4] = {0, 0, 0, 0};
  for (int64_t i = threadIdx.x; i < ntiles; i += KF_BS) s[0] += dpart[i];
  for (int i = threadIdx.x; i < KF_GRID; i += KF_BS) {
    s[1] += tpart[KFP_XT * KF_GRID + i];
    s[2] += tpart[KFP_YT * KF_GRID + i];
    s[3] += tpart[KFP_NT * KF_GRID + i];
  }
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    for (int o = 32; o > 0; o >>= 1) s[f] += __shfl_xor(s[f], o, 64);
    if ((threadIdx.x & 63) == 0) red[f][threadIdx.x >> 6] = s[f];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint64_t v[4];
  for (int f = 0; f < 4; ++f) v[f] = red[f][0] + red[f][1] + red[f][2] + red[f][3];
  const uint64_t dis = v[0], xt = v[1], yt = v[2], nt = v[3];
  double r = __builtin_nan("");
  const uint64_t t = (uint64_t)m * (uint64_t)(m - 1) / 2;
  if (!*nan && m >= 2 && xt != t && yt != t) {
    const int64_t cmd = (int64_t)(t - xt - yt + nt) - 2 * (int64_t)dis;
    double taub = (double)cmd / sqrt((double)(t - xt)) / sqrt((double)(t - yt));
    taub = fmin(1.0, fmax(-1.0, taub));
    const double denom = sqrt((double)(t - xt) * (double)(t - yt));
    r = denom == 0.0 ? __builtin_nan("") : taub * denom / (double)t;
  }
  *out = r;
}

// --------------------------------------------------------------------------- host
static unsigned kf_blocks(int64_t m, int bs = 256) { return (unsigned)((m + bs - 1) / bs); }

// tie groups of the sorted sequence (k1[, k2]) into flags / gidx / gstart, group count into
// *groups; sum of C(k, 2) into tpart[slot]
static int kf_groups(const uint32_t* k1, const uint32_t* k2, int64_t m, const KfWs& w, uint32_t* groups, int slot,
                     hipStream_t st) {
  k_kf_flags<<<kf_blocks(m), 256, 0, st>>>(k1, k2, m, w.flags);
  VR_CHECK_LAUNCH();
  VR_TRY(scan_exclusive_u32(w.flags, w.gidx, m, groups, w.scan, st));
  k_kf_starts<<<kf_blocks(m), 256, 0, st>>>(w.flags, w.gidx, m, w.gstart);
  VR_CHECK_LAUNCH();
  if (slot >= 0) {
    k_kf_tie_pairs<<<KF_GRID, KF_BS, 0, st>>>(w.flags, w.gidx, w.gstart, m, w.tpart + (size_t)slot * KF_GRID);
    VR_CHECK_LAUNCH();
  }
  return VR_OK;
}

// the u32 pipeline on w.kx / w.ky (m >= 2, both overwritten): tau-a into out
static int kf_run(int64_t m, const KfWs& w, double* out, hipStream_t st) {
  const int64_t nt = kf_tiles(m);
  VR_CHECK_HIP(hipMemsetAsync(w.dpart, 0, (size_t)nt * sizeof(uint64_t), st));
  // 1  y order with the x keys as the payload (no element order, no gather), dense y ranks,
  //    y ties
  //    (in place: kx / ky are not read again)
  VR_TRY(radix_sort_kv(w.ky, w.kx, w.c, w.d, m, w.radix, st));  // ky: sorted y keys, kx: x keys in y order
  VR_TRY(kf_groups(w.ky, nullptr, m, w, w.tot, KFP_YT, st));     // tot[0]: distinct y values G
  // 2  (x, y)-lexicographic order: the dense y ranks, stably sorted by the x keys
  k_kf_yrank<<<kf_blocks(m), 256, 0, st>>>(w.flags, w.gidx, m, w.d);
  VR_CHECK_LAUNCH();
  VR_TRY(radix_sort_kv(w.kx, w.d, w.a, w.c, m, w.radix, st));  // kx: sorted x keys, d: y ranks
  VR_TRY(kf_groups(w.kx, nullptr, m, w, w.tot + 1, KFP_XT, st));
  VR_TRY(kf_groups(w.kx, w.d, m, w, w.tot + 1, KFP_NT, st));
  // 3  inversions of the y ranks d, most significant level first (levels: bits of G - 1)
  uint32_t G = 0;
  VR_CHECK_HIP(hipMemcpyAsync(&G, w.tot, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VR_CHECK_HIP(hipStreamSynchronize(st));
  int L = 0;
  while (L < 32 && G > 0 && ((G - 1u) >> L) != 0u) ++L;
  uint32_t *cur = w.d, *next = w.a;
  uint32_t* bstart = w.b;  // bucket tables: at most G / 2 + 1 buckets
  uint32_t* bP = w.gstart;
  for (int b = L - 1; b >= 0; --b) {
    const uint32_t nbk = b >= 31 ? 1u : ((G - 1u) >> (b + 1)) + 1u;
    k_kf_lvl_count<<<(unsigned)nt, KF_BS, 0, st>>>(cur, m, b, w.tile, bstart);
    VR_CHECK_LAUNCH();
    VR_TRY(scan_exclusive_u32(w.tile, w.tile, nt, w.tot + 2, w.scan, st));
    k_kf_lvl_bucket<<<(unsigned)nt, LV_BS, 0, st>>>(cur, m, b, w.tile, bP);
    VR_CHECK_LAUNCH();
    k_kf_lvl_split<<<(unsigned)nt, LV_BS, 0, st>>>(cur, m, b, w.tile, bstart, bP, nbk, w.tot + 2,
                                                   b > 0 ? next : nullptr, w.dpart);
    VR_CHECK_LAUNCH();
    std::swap(cur, next);
  }
  k_kf_final<<<1, KF_BS, 0, st>>>(w.tpart, w.dpart, nt, m, w.nan, out);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// dense ranks of an f64 vector into rank[m] (hi/lo scratch: w.c, w.d)
static int kf_dense_rank64(const double* v, int64_t m, const KfWs& w, uint32_t* rank, hipStream_t st) {
  k_kf_keys64<<<kf_blocks(m), 256, 0, st>>>(v, m, w.c, w.d, w.nan);  // c: hi, d: lo
  VR_CHECK_LAUNCH();
  VR_CHECK_HIP(hipMemcpyAsync(w.a, w.d, (size_t)m * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
  k_kf_iota<<<kf_blocks(m), 256, 0, st>>>(w.b, m);
  VR_CHECK_LAUNCH();
  uint32_t* alt_k = w.flags;  // free until the groups below
  uint32_t* alt_v = w.gidx;
  VR_TRY(radix_sort_kv(w.a, w.b, alt_k, alt_v, m, w.radix, st));  // by lo: b = order
  k_kf_gather<<<kf_blocks(m), 256, 0, st>>>(w.c, w.b, m, w.a);     // hi in that order
  VR_CHECK_LAUNCH();
  VR_TRY(radix_sort_kv(w.a, w.b, alt_k, alt_v, m, w.radix, st));  // stable by hi: (hi, lo) order
  k_kf_gather<<<kf_blocks(m), 256, 0, st>>>(w.d, w.b, m, w.c);     // lo in that order
  VR_CHECK_LAUNCH();
  VR_TRY(kf_groups(w.a, w.c, m, w, w.tot + 3, -1, st));
  k_kf_scatter_rank<<<kf_blocks(m), 256, 0, st>>>(w.b, w.flags, w.gidx, m, rank);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

static int kf_nan_out(double* out, hipStream_t st) {
  const double nan = __builtin_nan("");
  VR_CHECK_HIP(hipMemcpyAsync(out, &nan, sizeof(double), hipMemcpyHostToDevice, st));
  VR_CHECK_HIP(hipStreamSynchronize(st));
  return VR_OK;
}

}  // namespace vr

using namespace vr;

static int kendall_full_impl(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx, double* out,
                             void* ws, size_t ws_bytes, hipStream_t st);

extern "C" {

size_t vr_kendall_full_vec_workspace(int64_t m) {
  size_t b = 0;
  kf_layout(nullptr, m < 0 ? 0 : m, &b);
  return b;
}

int vr_kendall_full_vec_f64(const double* x, const double* y, int64_t m, double* out, void* ws, size_t ws_bytes,
                            void* stream) {
  VR_REQUIRE(m >= 0 && m < ((int64_t)1 << 32), "vr_kendall_full_vec_f64: m=%lld out of range (< 2^32)",
             (long long)m);
  VR_REQUIRE(out != nullptr && (m == 0 || (x && y)), "vr_kendall_full_vec_f64: null pointer");
  hipStream_t st = as_stream(stream);
  if (m < 2) return kf_nan_out(out, st);  // rsa.py:25-26
  size_t need = 0;
  const KfWs w = kf_layout(ws, m, &need);
  if (ws == nullptr || ws_bytes < need) {
    set_error("vr_kendall_full_vec_f64: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  VR_CHECK_HIP(hipMemsetAsync(w.nan, 0, sizeof(uint32_t), st));
  VR_TRY(kf_dense_rank64(x, m, w, w.kx, st));
  VR_TRY(kf_dense_rank64(y, m, w, w.ky, st));
  return kf_run(m, w, out, st);
}

size_t vr_kendall_full_workspace(int64_t n) {
  size_t b = 0;
  kf_layout(nullptr, pairs_of(n < 0 ? 0 : n), &b);
  return b;
}

int vr_kendall_full_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out, void* ws,
                        size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && ld >= n && out, "vr_kendall_full_f32: bad shape n=%lld ld=%lld", (long long)n, (long long)ld);
  return kendall_full_impl(A, B, n, ld, nullptr, out, ws, ws_bytes, as_stream(stream));
}

int vr_kendall_full_subset_f32(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx, int64_t k,
                               double* out, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && ld >= n && k >= 0 && k <= n && out, "vr_kendall_full_subset_f32: bad shape n=%lld ld=%lld "
             "k=%lld", (long long)n, (long long)ld, (long long)k);
  VR_REQUIRE(idx != nullptr || k == 0, "vr_kendall_full_subset_f32: null idx");
  return kendall_full_impl(A, B, k, ld, idx, out, ws, ws_bytes, as_stream(stream));
}

}  // extern "C"

static int kendall_full_impl(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx, double* out,
                             void* ws, size_t ws_bytes, hipStream_t st) {
  VR_REQUIRE(pairs_of(n) < ((int64_t)1 << 32), "vr_kendall_full_f32: n=%lld has 2^32 or more pairs", (long long)n);
  const int64_t M = pairs_of(n);
  if (M < 2) return kf_nan_out(out, st);
  VR_REQUIRE(A && B, "vr_kendall_full_f32: null pointer");
  size_t need = 0;
  const KfWs w = kf_layout(ws, M, &need);
  if (ws == nullptr || ws_bytes < need) {
    set_error("vr_kendall_full_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  VR_CHECK_HIP(hipMemsetAsync(w.nan, 0, sizeof(uint32_t), st));
  const dim3 grid((unsigned)((n + 255) / 256), (unsigned)std::min<int64_t>(n, 16384));
  if (idx)
    k_kf_tri_keys_sub<<<grid, 256, 0, st>>>(A, B, idx, n, ld, w.kx, w.ky, w.nan);
  else
    k_kf_tri_keys<<<grid, 256, 0, st>>>(A, B, n, ld, w.kx, w.ky, w.nan);
  VR_CHECK_LAUNCH();
  return kf_run(M, w, out, st);
}
