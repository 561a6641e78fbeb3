// Bootstrapped Spearman RSA engine and the triangle-Spearman entry points.
//
// Replaces, per (model RDM A, neural RDM B) unit, the reference loop
//   point = spearmanr(triu(A), triu(B))                                 evals.py:347-349
//   for i in range(1000): idx = rng.choice(n, int(.9n), replace=False)
//       scores[i] = spearmanr(triu(A[idx][:,idx]), triu(B[idx][:,idx]))    evals.py:361-369
// with scipy's average-rank (midrank) ties (rsa.py:43-47,121-122).
//
// For a stimulus subset S a pair (a,b) is included iff a, b in S; its midrank among the
// included pairs is (c_s + c_e + 1)/2 with c_s / c_e the included counts before / through
// its tie group in sorted order. Everything is kept as doubled ranks y = 2 c_s + k + 1
// (integers), and rho = (sum yA yB - M'(M'+1)^2) / sqrt((sum yA^2 - mu)(sum yB^2 - mu)),
// mu = M'(M'+1)^2, M' = included pairs: exact integer sums -> fp64 at the end, so scores
// do not depend on chunking, lane grouping, launch order or GPU count.
//
// One pass evaluates 64 subsets: lane s of every wave is subset s, masks[x] bit s says
// whether stimulus x is in subset s (LDS). Waves own contiguous segments of chunks and
// walk them in 64-position windows: lane j looks up pair w0+j (one coalesced code load,
// two LDS mask reads), and a 64x64 bit transpose across the wave hands lane s the
// inclusion bits of all 64 pairs for subset s. Counts before any position are then
// popcounts, so a tie group [gs, ge) closes in O(1): y = c(gs) + c(ge) + 1.
//  k_rankA   A order, one 128-byte TB row per pair written in A order. EST form (default):
//            the absolute doubled rank mod 2^16 (k_countA first gives each segment its
//            base), every value checked against the B side's count estimate; exact form:
//            the chunk-relative rank (u16 when chunk spans fit, else u32), lpA[chunk] =
//            chunk start count, then a per-lane scan -> baseA[chunk].
//  k_rankB   B order: yA gathered per pair from its TB row (EST: recovered from its 16 bits
//            and the window low end; exact: + 2 baseA[chunkA], a second gather); per B group
//            S = sum of included yA; segment sums S y'_B, S, tie terms (segment-relative)
//  k_tail_part + k_tail_top   all units of a pass at once: blockwise prefix products combine
//            the segments -> rho per lane
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "window.h"

namespace vr {

#ifndef VR_ENG_THREADS
#define VR_ENG_THREADS 1024
#endif
constexpr int ENG_THREADS = VR_ENG_THREADS;  // waves per workgroup share one LDS mask table
constexpr int WAVES_PER_WG = ENG_THREADS / 64;
constexpr int SCAN_SEGS = 256;     // segments per block in the segment scans / final fold

// ---------------------------------------------------------------------------------
// Count-estimate table (EST mode, the default pass form).
// The A side stores each pair's ABSOLUTE doubled rank y_A modulo 2^16 (one u16 per subset,
// a 128-byte row per pair). The B side recovers y_A exactly from those 16 bits and the low
// end lo of a 2^16-wide window known to hold it: y_A = lo + (u16)(t - lo). lo interpolates
// the doubled included count between coarse boundaries q_c = c 2^b in 4096 steps per
// interval: lo = L_c + D_c * step (one v_mad_u32_u24 per pair and lane; {L_c, D_c} per
// interval and lane, <= EST_NC rows of 64 lanes staged in LDS), so the only per-pair
// global access of the B walk is the TB row. Measured on N=10k RDMs the interpolation error is a few hundred counts
// (profiles/r2_est_deviation.log) against the 2^14 the 16 bits allow; the A walk checks
// every stored value against the same estimate and flags the pass, and flagged passes
// are re-run in the exact chunk-base form (baseA rows), so scores never depend on it.
// ---------------------------------------------------------------------------------
constexpr int EST_NC = 256;
constexpr int EST_STEP_BITS = 12;  // interpolation steps per interval: 2^12
#ifndef VR_EST_CHECK
#define VR_EST_CHECK 1  // 0: timing probe only (no A-side recoverability checks: unsafe)
#endif
// Timing probes (wrong scores; never in the default build; profiles/r3_engine_probes.log):
// VR_PROBE_WB replaces k_rankB's window mask lookups and transposes by a constant pattern,
// VR_PROBE_ACC 1-3 strip its singleton accumulation (no 64-bit multiply / no St / one
// 32-bit add), VR_PROBE_STW gives k_rankA one 4-byte store per two singleton rows.
#ifndef VR_PROBE_STW
#define VR_PROBE_STW 0  // k_rankA timing probe: half as many (4-byte) singleton stores
#endif
#ifndef VR_PROBE_WB
#define VR_PROBE_WB 0
#endif
#ifndef VR_PROBE_WBA
#define VR_PROBE_WBA 0  // the same for k_rankA
#endif
#ifndef VR_PROBE_ACC
#define VR_PROBE_ACC 0
#endif
static std::atomic<int64_t> g_est_reruns{0};      // passes re-run in the exact form (vr_engine_est_reruns)
static std::atomic<int64_t> g_est_predicted{0};   // calls sent to the exact form before any EST pass (vr_engine_est_predicted)
static std::atomic<int64_t> g_est_tail_flags{0};  // of those, flagged by the tail invariants alone (vr_engine_est_tail_flags)
static std::atomic<int64_t> g_est1_fallbacks{0};  // calls run in EST 1 after EST 3's up-front check failed

// log2 of the coarse interval: the smallest b >= 12 (windows of 64 never straddle a
// boundary; the 4096 steps are whole positions) with ceil(M / 2^b) <= 96, or, for larger
// triangles, <= EST_NC (a step of 2^(b-12) positions moves lo by <= 2^(b-11): b <= 23
// keeps that at a few thousand of the 2^15 of slack).
// maxrows < EST_NC: the table must fit beside the masks in LDS (fewer, longer intervals).
static int est_bits(int64_t M, uint32_t maxrows = EST_NC, uint32_t target = 96) {
  int b = 12;
  while (((M + ((int64_t)1 << b) - 1) >> b) > (int64_t)target && b < 23) ++b;
  while (((M + ((int64_t)1 << b) - 1) >> b) > (int64_t)maxrows && b < 31) ++b;
  return b;
}
static uint32_t est_intervals(int64_t M, int b) { return (uint32_t)((M + ((int64_t)1 << b) - 1) >> b); }

// EST form by default (VISREPS_ENGINE_EST=0: every pass exact). Measured on the bench RDMs
// (profiles/r2_engine_est3.log): k_rankB 1.56 ms per pass in EST 3 against 1.96 ms in the
// exact form. The table form (EST 1) and the masks-from-L2 variants measured 1.86-2.04 ms
// (profiles/r2_engine_ab.log): their per-pair table reads cost what the base gather saved.
static bool engine_est() {
  const char* e = getenv("VISREPS_ENGINE_EST");
  return !(e && strcmp(e, "0") == 0);
}

// Launch shape. The walks are bound by the latency of their random TB gathers, so they run
// two 16-wave workgroups per CU (32 waves): the exact-form kernels and the EST count
// pre-pass keep the masks in LDS while two copies fit (N <= 10176), the EST rank walks
// read them from L2 (80 KB at N = 10k) and hold only the interval table in LDS.
struct EngineCfg {
  int grid;      // workgroups
  int nwaves;    // grid * WAVES_PER_WG = number of chunk segments (A and B each)
  bool use_lds;  // exact kernels, k_countA: masks in LDS
  size_t lds;    // their dynamic LDS (the masks, or 0)
  // EST passes (every kernel of one EST pass uses these; est_nwaves <= nwaves)
  bool est_lds;   // EST rank walks: masks in LDS beside the table (else masks from L2)
  int est_grid, est_nwaves;
  int est_mode;       // 1: interval table in LDS, 2: one linear interval in registers
  int est_b;          // log2 of the table interval
  uint32_t est_rows;  // table rows (intervals)
  uint32_t est_nseg;   // EST B-walk segments (work queue; est_segments)
  uint32_t est_nsegA;  // EST A-side segments: est_nseg x est_ratioA (k_countA, k_rankA)
  uint32_t est_ratioA;
  bool prejoined = false;  // the units' A positions arrive joined (vr_bootstrap_spearman_multi_joined)
  size_t tab;         // EST rank walks' dynamic LDS: [masks] + table
};

static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}

#ifndef VR_SEGS_PER_WAVE
#define VR_SEGS_PER_WAVE 4  // most EST A-side segments per resident wave (workspace bound)
#endif
// EST B walks take segments of >= 256 positions from a work queue, one per resident wave;
// the A side cuts each of them into est_ratioA (VISREPS_ENGINE_SEGS_A, default and most
// VR_SEGS_PER_WAVE) for its own queue (k_rankA; k_countA takes them round-robin).
static uint32_t est_segments(int64_t M, int est_nwaves) {
  const int64_t by_len = (M + 255) / 256;
  return (uint32_t)std::max<int64_t>(1, std::min<int64_t>(by_len, (int64_t)est_nwaves));
}

// mode: the EST estimate (0: VISREPS_ENGINE_EST_MODE, default 3; 1: the per-lane table, the
// fallback of a call whose EST 3 estimate fails its up-front check)
static EngineCfg engine_cfg(int64_t n, int mode = 0) {
  EngineCfg c;
  const int64_t M = pairs_of(n);
  const size_t need = (size_t)n * sizeof(uint64_t);
  const size_t cap = 160 * 1024 - 1024;
  const char* e = getenv("VISREPS_ENGINE_MASKS");  // "global": masks from L2 (A/B timing)
  c.use_lds = need <= cap && !(e && strcmp(e, "global") == 0);
  c.lds = c.use_lds ? need : 0;
  const int per_cu = std::max<int>(1, std::min<int>(2048 / ENG_THREADS, (int)(cap / std::max<size_t>(c.lds, 1))));
  c.grid = num_cus() * per_cu;
  c.nwaves = c.grid * WAVES_PER_WG;
  // EST: masks and table both in LDS when the table gets >= 1 row beside the masks at
  // VISREPS_ENGINE_EST_WG workgroups per CU (default 2, the exact form's occupancy);
  // otherwise masks from L2 and the table alone in LDS.
  const size_t row = (size_t)LANES * sizeof(uint2);
  const int est_wg = std::max(1, std::min(per_cu, env_int("VISREPS_ENGINE_EST_WG", per_cu)));
  const size_t per_wg = cap / est_wg;
  c.est_lds = c.use_lds && env_int("VISREPS_ENGINE_EST_LDS", 1) != 0 && per_wg >= need + row;
  // VISREPS_ENGINE_EST_LIN=1: one linear interval (EST 2), no table in LDS
  c.est_mode = mode > 0 ? mode : std::max(1, std::min(3, env_int("VISREPS_ENGINE_EST_MODE", 3)));
  if (c.est_mode >= 2) c.est_lds = c.use_lds && env_int("VISREPS_ENGINE_EST_LDS", 1) != 0 && per_wg >= need;
  uint32_t rows_fit =
      c.est_lds ? (uint32_t)std::min<size_t>(EST_NC, (per_wg - need) / row) : (uint32_t)EST_NC;
  if (c.est_mode >= 2) rows_fit = 1;
  // EST 1 with masks from L2: the table alone in LDS, up to 144 intervals (72 KB: two
  // workgroups per CU still fit) -- finer knots for the large structured triangles it serves
  const uint32_t target = (c.est_mode == 1 && !c.est_lds) ? 144u : 96u;
  c.est_b = est_bits(M, rows_fit, target);
  c.est_rows = M > 0 ? est_intervals(M, c.est_b) : 0;
  c.est_grid = c.est_lds ? num_cus() * est_wg : c.grid;
  c.est_nwaves = c.est_grid * WAVES_PER_WG;
  c.est_nseg = est_segments(M, c.est_nwaves);
  c.est_ratioA = (uint32_t)std::max(1, std::min(VR_SEGS_PER_WAVE, env_int("VISREPS_ENGINE_SEGS_A", VR_SEGS_PER_WAVE)));
  // A segments of >= 1024 positions: small triangles (phase 1's M ~ 5e5) keep one per B
  // segment, where thousands of one-window segments would queue on a single counter
  while (c.est_ratioA > 1 && (uint64_t)c.est_nseg * c.est_ratioA * 1024u > (uint64_t)M) --c.est_ratioA;
  c.est_nsegA = c.est_nseg * c.est_ratioA;
  c.tab = (c.est_lds ? need : 0) + (c.est_mode == 1 ? (size_t)c.est_rows * row : 0);
  return c;
}

static inline uint32_t scan_blocks(uint32_t nseg) { return (nseg + SCAN_SEGS - 1) / SCAN_SEGS; }

// Segment partials are structure-of-arrays [field][seg][lane] so every access is a row.
enum { PA_TIEL = 0, PA_TIEH, PA_N };
enum { PB_ACCL = 0, PB_ACCH, PB_ST, PB_TIEL, PB_TIEH, PB_N };

struct EngineWs {
  uint64_t* masks;      // [n]
  uint32_t* posA_byB;   // [M]  B position -> A position (per unit)
  uint32_t* chunkA_byB; // [M]  B position -> A chunk (per unit)
  void* TB;             // [M * lw] u16 or u32 chunk-relative yA~, A order
  uint32_t* lpA;        // [nch * 64] count at chunk start, relative to its segment
  uint32_t* baseA;      // [nch * 64] absolute count at chunk start
  uint32_t* segA_tot;   // [nw * 64]
  uint64_t* segA_part;  // [PA_N][nw][64]  tie term sum (k^3 - k)
  uint32_t* segA_pre;   // [nw * 64]
  size_t useg;          // nw * 64: unit stride of the B segment partials
  uint32_t* segB_tot;   // [units][nw * 64]
  uint64_t* segB_part;  // [units][PB_N][nw][64]  sum S y'_B, sum S, tie term
  uint32_t* bsum;       // [scan_blocks * 64] scan scratch
  uint64_t* fpart;      // [min(units, 64)][scan_blocks][FP_N][64] tail partials
  uint32_t* totA;       // [64] included pairs per subset
  uint32_t* c0rel;      // [EST_NC][64]     EST: that count relative to its segment
  uint32_t* c0seg;      // [EST_NC]         EST: the segment holding each boundary
  uint2* ftab;          // [EST_NC][64]     EST: {L_c, D_c} per interval (window low end, step)
  uint32_t* viol;       // [EST_MAX_PASSES] EST: pass flagged for the exact re-run;
                        // [EST_MAX_PASSES]: an exact-form pass broke the tail invariants
  uint32_t* segposA;    // [nsegmax + 1] EST segment starts of the A plan (k_seg_table)
  uint32_t* segposB;    // [units][nw + 1] ... of each B plan
  size_t segstride;     // nw + 1
  uint32_t* queue;      // [QSLOTS] EST work-queue counters of one pass's launches
  uint64_t* corr;       // [units][CORR_F][CORR_BLK] EST 4: lane 0's shift sums (k_full_corr blocks)
};
constexpr int CORR_F = 5;       // sum d, then sum d yB as four 32-bit limb sums
constexpr int CORR_BLK = 2048;  // k_full_corr's fixed grid
constexpr size_t CORR_N = (size_t)CORR_F * CORR_BLK;  // per unit
constexpr int QSLOTS = 256;
enum { QS_RANKA = 0, QS_RANKB = 1 };  // queue slots of an EST pass's launches

constexpr int EST_MAX_PASSES = 512;  // passes between two checks of the EST flags

// slim: a grid call's region 1.. workspace (run_engine_grid): EST passes only, so the TB is
// u16 and there are no join arrays (the units arrive joined; flagged or exact-form work of
// any region runs on region 0's full workspace)
static EngineWs engine_layout(void* base, int64_t n, int lw, int nwaves, size_t* bytes, int64_t units = 1,
                              bool slim = false) {
  const int64_t M = pairs_of(n);
  const size_t nch = plan_nchunks(M);
  // A-side segment partials: up to VR_SEGS_PER_WAVE per wave (EST); B-side: one per wave
  const size_t nsegmax = (size_t)nwaves * VR_SEGS_PER_WAVE;
  const size_t nsb = scan_blocks((uint32_t)nsegmax);
  Carver c(base);
  EngineWs e;
  e.c0rel = c.take<uint32_t>((size_t)EST_NC * LANES);
  e.c0seg = c.take<uint32_t>((size_t)EST_NC);
  e.ftab = c.take<uint2>((size_t)EST_NC * LANES);
  e.viol = c.take<uint32_t>((size_t)EST_MAX_PASSES + 1);  // + the exact form's invariant flag
  e.masks = c.take<uint64_t>((size_t)n);
  e.posA_byB = slim ? nullptr : c.take<uint32_t>((size_t)M);
  e.chunkA_byB = slim ? nullptr : c.take<uint32_t>((size_t)M);
  if (slim)
    e.TB = c.take<uint16_t>((size_t)M * (size_t)lw);
  else
    e.TB = c.take<uint32_t>((size_t)M * (size_t)lw);  // sized for u32 (exact form, wide chunk ranks)
  e.lpA = c.take<uint32_t>(nch * LANES);
  e.baseA = c.take<uint32_t>(nch * LANES);
  e.segA_tot = c.take<uint32_t>(nsegmax * LANES);
  e.segA_part = c.take<uint64_t>(nsegmax * LANES * PA_N);
  e.segA_pre = c.take<uint32_t>(nsegmax * LANES);
  units = std::max<int64_t>(units, 1);
  e.segstride = (size_t)nwaves + 1;
  e.segposA = c.take<uint32_t>(nsegmax + 1);
  e.segposB = c.take<uint32_t>(e.segstride * (size_t)units);
  e.queue = c.take<uint32_t>(QSLOTS);
  e.useg = (size_t)nwaves * LANES;
  e.segB_tot = c.take<uint32_t>(e.useg * (size_t)units);
  e.segB_part = c.take<uint64_t>(e.useg * PB_N * (size_t)units);
  e.bsum = c.take<uint32_t>(nsb * LANES);
  e.fpart = c.take<uint64_t>((size_t)std::min<int64_t>(units, 64) * nsb * 8 * LANES);
  e.totA = c.take<uint32_t>(LANES);
  e.corr = c.take<uint64_t>(CORR_N * (size_t)units);
  if (bytes) *bytes = c.bytes();
  return e;
}

// ---------------------------------------------------------------------------------
// per-unit join and per-pass masks
// ---------------------------------------------------------------------------------
// The second array: the A chunk (exact form, JOIN_CHUNK) or the EST 3 window low end of the
// A position, L + (2 posA R >> 32) (JOIN_LO): the B walk then reads it instead of computing it.
enum { JOIN_NONE = 0, JOIN_CHUNK = 1, JOIN_LO = 2 };
// Every join gathers the 4-B A positions (posMapA), a table the MALL can keep across the
// joins of one A plan. JOIN_CHUNK also needs the A chunk of the position: chunks are
// group-aligned, chunk c starting at the first group start >= c L, so the chunk of a
// position is the last c <= pos / L whose start is <= pos. Chunk starts are non-decreasing
// in c, so that is a binary search (log2 of the chunks a tie group spans, not one step per
// chunk: a tie group over half the pairs spans thousands of chunks).
__global__ void k_join(const uint32_t* __restrict__ codesB, int64_t M, int64_t n,
                       const uint32_t* __restrict__ gstartA, const uint32_t* __restrict__ chunk_gA,
                       uint32_t L, uint32_t nchA, const uint32_t* __restrict__ posMapA,
                       uint32_t* __restrict__ posA_byB, uint32_t* __restrict__ second, int mode,
                       uint32_t Lu, uint32_t Ru) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t cb = __builtin_nontemporal_load(codesB + i);
  const uint64_t t = tri_index(cb >> 16, cb & 0xffffu, (uint64_t)n);
  const uint32_t pa = posMapA[t];
  if (mode == JOIN_CHUNK) {
    uint32_t hi = min(pa / L, nchA - 1u);
    uint32_t c = hi;
    if (gstartA[chunk_gA[hi]] > pa) {  // the last c in [0, hi) with start <= pa (chunk 0 starts at 0)
      uint32_t lo = 0;                 // invariant: start(lo) <= pa < start(hi)
      while (hi - lo > 1) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (gstartA[chunk_gA[mid]] <= pa)
          lo = mid;
        else
          hi = mid;
      }
      c = lo;
    }
    posA_byB[i] = pa;
    second[i] = c;
    return;
  }
  __builtin_nontemporal_store(pa, posA_byB + i);
  if (mode == JOIN_LO) __builtin_nontemporal_store(Lu + __umulhi(pa << 1, Ru), second + i);
}

// JOIN_LO from the A positions already joined (no second pair-map gather)
__global__ void k_join_lo(const uint32_t* __restrict__ posA_byB, int64_t M, uint32_t* __restrict__ second,
                          uint32_t Lu, uint32_t Ru) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < M) second[i] = Lu + __umulhi(posA_byB[i] << 1, Ru);
}

// Shared joins: the position maps of up to 4 A plans interleaved into 16-B records, so one
// random 16-B gather per B pair gives its A position in every one of them (k_join4) where
// separate joins each pay a random line per pair for 4 B.
struct Maps4 {
  const uint32_t* p[4];
};
struct Outs4 {
  uint32_t* p[4];
};
__global__ void k_posmap4(Maps4 m, int na, int64_t M, uint4* __restrict__ pm4) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= M) return;
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  for (int i = 0; i < na; ++i) v[i] = __builtin_nontemporal_load(m.p[i] + q);
  pm4[q] = make_uint4(v[0], v[1], v[2], v[3]);
}
__global__ void k_join4(const uint32_t* __restrict__ codesB, int64_t M, int64_t n, const uint4* __restrict__ pm4,
                        int na, Outs4 out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t cb = __builtin_nontemporal_load(codesB + i);
  const uint4 r = pm4[tri_index(cb >> 16, cb & 0xffffu, (uint64_t)n)];
  const uint32_t v[4] = {r.x, r.y, r.z, r.w};
  for (int a = 0; a < na; ++a) __builtin_nontemporal_store(v[a], out.p[a] + i);
}

// bit w of masks[x] <- x in subset (set0 + w); subset 0 is "all stimuli" when full_first.
__global__ void k_masks_sets(const int32_t* __restrict__ idx, int64_t k, int64_t set0,
                             int nl, int full_first, uint64_t* __restrict__ masks) {
  const int w = blockIdx.y;
  if (w >= nl) return;
  const int64_t s = set0 + w;
  if (full_first && s == 0) return;  // handled by k_masks_full
  const int64_t row = s - (full_first ? 1 : 0);
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t x = idx[row * k + j];
    atomicOr(reinterpret_cast<unsigned long long*>(&masks[x]), 1ull << w);
  }
}

__global__ void k_masks_full(uint64_t* __restrict__ masks, int64_t n) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x < n) masks[x] |= 1ull;  // lane 0 of the first pass
}

__device__ inline uint64_t restrict_flags(uint64_t F, uint32_t w0, uint32_t P0, uint32_t P1) {
  if (P0 >= w0) F &= ~lowmask(P0 - w0 + 1);
  if (P1 - w0 < 64) F = (F & lowmask(P1 - w0)) | (1ull << (P1 - w0));
  return F;
}

// sum over tie groups of k^3 - k = k (k^2 - 1). When the plan's largest tie group is below
// 2^16 (BIGT false, the normal case) one 32x32+64 multiply-add per group, and the sum stays
// below 2^63 for any segment; otherwise 128-bit.
template <bool BIGT>
__device__ inline void tie_add(uint64_t& t64, u128& tbig, uint32_t k) {
  if (!BIGT) {
    t64 += (uint64_t)k * (k * k - 1u);
  } else {
    tbig += (u128)((uint64_t)k * k) * k - k;
  }
}

#ifndef VR_TB_STORE_NT
#define VR_TB_STORE_NT 1  // TB rows written with nontemporal stores (0: default policy, A/B)
#endif
template <typename T>
__device__ inline void tb_store(T v, T* p) {
  if constexpr (VR_TB_STORE_NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// rows [r0, r0 + cnt) of TB get v in this lane's column: row addresses are wave-uniform
// (SGPR base + lane offset), four rows per step
template <bool FULL, typename TBT>
__device__ inline void store_rows(TBT* __restrict__ TB, uint32_t stride, uint32_t r0, uint32_t cnt,
                                  int lane, TBT v) {
  TBT* row = TB + (size_t)r0 * stride + lane;
  uint32_t i = 0;
  for (; i + 4 <= cnt; i += 4, row += 4 * (size_t)stride) {
    tb_store(v, row);
    tb_store(v, row + stride);
    tb_store(v, row + 2 * stride);
    tb_store(v, row + 3 * stride);
  }
  for (; i < cnt; ++i, row += stride) tb_store(v, row);
}

struct Segment {
  uint32_t c0, c1;
};
// Wave w owns chunks [floor(w C / W), floor((w+1) C / W)): every wave gets floor or ceil
// of C / W chunks. seg_of_chunk is the inverse.
__host__ __device__ inline Segment my_segment(uint32_t nchunks, uint32_t nwaves, uint32_t wave) {
  return {(uint32_t)((uint64_t)wave * nchunks / nwaves),
          (uint32_t)((uint64_t)(wave + 1) * nchunks / nwaves)};
}
__host__ __device__ inline uint32_t seg_of_chunk(uint32_t c, uint32_t nchunks, uint32_t nwaves) {
  return (uint32_t)(((uint64_t)(c + 1) * nwaves - 1) / nchunks);
}

// The EST kernels' work queue: lane 0 takes the next segment index of this launch's
// counter (a vector atomic), the wave reads it from lane 0.
__device__ inline uint32_t next_segment(uint32_t* q) {
  uint32_t s = 0;
  if ((threadIdx.x & 63) == 0) s = atomicAdd(q, 1u);
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)s);
}

// EST segment starts of a plan: segpos[s] = the first tie-group start >= s M / nseg
// (segpos[nseg] = M), a binary search over the G + 1 group starts. Segments may be empty
// (a tie group longer than M / nseg).
__global__ void k_seg_table(const uint32_t* __restrict__ gstart, const PlanHeader* __restrict__ hdr, int64_t M,
                            uint32_t nseg, uint32_t* __restrict__ segpos) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s > nseg) return;
  const uint64_t nominal = (uint64_t)s * (uint64_t)M / nseg;
  uint32_t lo = 0, hi = hdr->G;  // gstart[hi] = M >= nominal
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if ((uint64_t)gstart[mid] >= nominal)
      hi = mid;
    else
      lo = mid + 1;
  }
  segpos[s] = s == nseg ? (uint32_t)M : gstart[lo];
}

__device__ inline uint32_t chunk_start(const uint32_t* __restrict__ gstart,
                                       const uint32_t* __restrict__ chunk_g, uint32_t c) {
  return sload(gstart + sload(chunk_g + c));
}

int build_pass_masks(const int32_t* idx, int64_t k, int64_t set0, int nl, int full_first,
                     uint64_t* masks, int64_t n, hipStream_t st) {
  VR_CHECK_HIP(hipMemsetAsync(masks, 0, (size_t)n * sizeof(uint64_t), st));
  if (full_first && set0 == 0) {
    k_masks_full<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(masks, n);
    VR_CHECK_LAUNCH();
  }
  const int64_t nrows = nl - ((full_first && set0 == 0) ? 1 : 0);
  if (nrows > 0 && k > 0) {
    dim3 grid((unsigned)std::min<int64_t>((k + 255) / 256, 64), (unsigned)nl);
    k_masks_sets<<<grid, 256, 0, st>>>(idx, k, set0, nl, full_first, masks);
    VR_CHECK_LAUNCH();
  }
  return VR_OK;
}

// EST: the copy of the interval table in LDS (the rank walks read the masks from L2)
__device__ inline const uint2* stage_table(const uint2* __restrict__ gtab, uint32_t rows, uint2* smem) {
  for (uint32_t i = threadIdx.x; i < rows * LANES; i += blockDim.x) smem[i] = gtab[i];
  __syncthreads();
  return smem;
}

// EST: low end of the 2^16-wide window holding the doubled rank of A position pos for this
// lane's subset: L_c + D_c * step, step = the position's 1/4096th of interval c. Monotone
// non-decreasing in pos, over interval boundaries too (L_c + D_c 4095 <= L_{c+1}).
__device__ inline uint32_t est_lo(const uint2* tab, uint32_t pos, int lane, int bits) {
  const uint2 e = tab[(pos >> bits) * LANES + lane];
  const uint32_t step = (pos & ((1u << bits) - 1u)) >> (bits - EST_STEP_BITS);
  return e.x + __umul24(e.y, step);  // v_mad_u32_u24 (D_c <= 2^(b-11) < 2^24)
}

// EST: the doubled rank whose low 16 bits are v, in the window [lo, lo + 2^16)
__device__ inline uint32_t est_recover(uint32_t v, uint32_t lo) { return lo + (uint32_t)(uint16_t)(v - lo); }

// EST: true if y is outside the window [lo, lo + 2^16)
__device__ inline bool est_bad(uint32_t y, uint32_t lo) { return y - lo > 65535u; }

// The window low end of either EST form. EST 1: the interpolated interval table (LDS).
// EST 2 (one interval over the whole triangle): lo = trunc(fma(R, pos, L)) in f32 from two
// per-lane registers, R = 2 M'/M and L = 1 - 2^15 (k_c0_lin): no table read per pair.
// Both are deterministic and monotone non-decreasing in pos (the A side checks only the
// ends of a group), and the A and B walks evaluate the same function.
// EST 3 (every active lane a subset of the same size, so one included-pair total M' for
// the wave): lo = L + (2 pos R >> 32), R = floor(2^32 M'/M), L = 1 - 2^15: wave-uniform,
// scalar arithmetic (s_mul_hi_u32), no per-lane work besides the 16-bit recovery.
struct EstLo {
  const uint2* tab;
  int bits;
  float L, R;
  uint32_t Lu, Ru;
  uint32_t sh;  // EST 6: the coarse A position is pos >> sh
  uint32_t g;   // EST 5: lane 63 holds the EST 3 low end + 2^15, >> g
};

// 32-bit triangle index of pair code (a << 16) | b (M < 2^32: a n < 2^32, a (a + 1) < 2^32)
__device__ inline uint32_t tri32(uint32_t code, uint32_t n) {
  const uint32_t a = code >> 16, b = code & 0xffffu;
  return a * n - ((a * (a + 1u)) >> 1) + b - a - 1u;
}

// EST 5 / 6 (the triangle-order TB, VISREPS_ENGINE_TRI): the TB row of a pair sits at its
// triangle index and lane 63 holds a 16-bit tag of its A position pos from which both walks
// evaluate the same window low end (monotone non-decreasing in pos, like EST 3):
//  EST 5  tag = (EST 3 low end + 2^15) >> g, low end = (tag << g) - 2^15: the EST 3 window
//         rounded down to a multiple of 2^g (g = 11 at N = 10k: <= 2047 of the 2^15 slack),
//         one shift and one subtract on the B side;
//  EST 6  (the pass holding the full set in lane 0) tag = pos >> sh, the EST 4 low ends at the
//         middle of the coarse interval.
__device__ inline uint32_t est5_u(const EstLo& e, uint32_t pos) { return 1u + __umulhi(pos << 1, e.Ru); }
__device__ inline uint32_t est5_lo_tag(const EstLo& e, uint32_t tag) { return (tag << e.g) - 32768u; }
template <int EST>
__device__ inline uint32_t tri_tag(const EstLo& e, uint32_t pos) {
  return EST == 5 ? est5_u(e, pos) >> e.g : pos >> e.sh;
}
__device__ inline uint32_t est_lo_pc(const EstLo& e, uint32_t pc, int lane, bool full_lane0) {
  const uint32_t mid = (pc << e.sh) + ((1u << e.sh) >> 1);
  const uint32_t lo = e.Lu + __umulhi(mid << 1, e.Ru);  // wave-uniform (scalar) arithmetic
  if (!full_lane0) return lo;
  // lane 0 (the full set): + the uniform difference of its low end, masked to lane 0 --
  // two VALU ops on scalar operands, no per-lane branch
  const uint32_t d0 = 2u * mid + (1u - 32768u) - lo;
  return lo + (d0 & (0u - (uint32_t)(lane == 0)));
}
// EST 4: EST 3 with lane 0 holding the full set (pass 0 of a full_first call): its count
// before A position pos is pos itself, so its low end is 2 pos + 1 - 2^15 (est_lo_t<4>, the
// A side's checks). Lane 0 stores its doubled rank y shifted down by the gap between that low
// end and the EST 3 one every other lane uses, d(pos) = 2 pos - (2 pos Ru >> 32) (y - d lies
// in the EST 3 window exactly when y lies in lane 0's own), so the B walk recovers all 64
// lanes with one wave-uniform window: the EST 3 kernel, no per-pair lane-0 select. Lane 0's
// B-side sums then miss sum_p d(posA(p)) in sum yA and sum_p d(posA(p)) yB(p) in sum yA yB,
// which k_full_corr adds up per unit and k_tail_top puts back (exact integers either way).
// d is non-decreasing in pos, and y - d >= 1 is checked per group (k_rankA), so the shifted
// value is a positive u32 like every other lane's rank.
__device__ inline uint32_t est4_shift(uint32_t Ru, uint32_t pos) {
  const uint32_t p2 = pos << 1;
  return p2 - __umulhi(p2, Ru);
}
template <int EST>
__device__ inline uint32_t est_lo_t(const EstLo& e, uint32_t pos, int lane) {
  if constexpr (EST == 5)
    return est5_lo_tag(e, est5_u(e, pos) >> e.g);
  else if constexpr (EST == 6)
    return est_lo_pc(e, pos >> e.sh, lane, true);
  else if constexpr (EST == 4)
    return lane == 0 ? 2u * pos + (1u - 32768u) : e.Lu + __umulhi(pos << 1, e.Ru);
  else if constexpr (EST == 3)
    return e.Lu + __umulhi(pos << 1, e.Ru);
  else if constexpr (EST == 2)
    return (uint32_t)(int32_t)__builtin_fmaf(e.R, (float)pos, e.L);
  else
    return est_lo(e.tab, pos, lane, e.bits);
}
template <int EST>
__device__ inline EstLo est_setup(const uint2* __restrict__ gtab, uint32_t rows, int bits, uint2* smem) {
  EstLo e{nullptr, bits, 0.f, 0.f, 0u, 0u, 0u, 0u};
  if constexpr (EST >= 3) {
    e.Lu = wave_uniform(sload(&gtab->x));
    e.Ru = wave_uniform(sload(&gtab->y));
    if constexpr (EST >= 5) {
      e.sh = wave_uniform(sload(&gtab[1].x));
      e.g = wave_uniform(sload(&gtab[1].y));
    }
  } else if constexpr (EST == 2) {
    const uint2 v = gtab[threadIdx.x & 63];
    e.L = __uint_as_float(v.x);
    e.R = __uint_as_float(v.y);
  } else if constexpr (EST == 1) {
    e.tab = stage_table(gtab, rows, smem);
  }
  return e;
}

// ---------------------------------------------------------------------------------
// EST pre-pass: included pairs per A segment (for the absolute ranks of k_rankA<EST>)
// and the segment-relative count at every coarse boundary inside the segment
// ---------------------------------------------------------------------------------
template <bool LDS, bool FULL>
__global__ __launch_bounds__(ENG_THREADS, 8) void k_countA(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gstart,
    const uint32_t* __restrict__ chunk_g, uint32_t nchunks, const uint64_t* __restrict__ gmask,
    int64_t n, int lw, int bits, uint32_t* __restrict__ c0rel, uint32_t* __restrict__ c0seg,
    uint32_t* __restrict__ seg_tot, uint32_t nseg, const uint32_t* __restrict__ segpos) {
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const int lane = threadIdx.x & 63;
  const bool active = FULL || lane < lw;
  (void)gstart;
  (void)chunk_g;
  (void)nchunks;
  // segments [segpos[s], segpos[s + 1]) round-robin (a count walk is too short per segment
  // for a shared work-queue counter: 32 k atomics on one address cost more than it saves)
  const uint32_t wave = wave_uniform(blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6));
  for (uint32_t sidx = wave; sidx < nseg; sidx += gridDim.x * WAVES_PER_WG) {
    const uint32_t P0 = segpos[sidx], P1 = segpos[sidx + 1];
    uint32_t cw = 0;
    if (P0 < P1) {
      const uint32_t bmask = (1u << bits) - 1u;
      uint32_t w0 = P0 & ~63u;
      uint32_t cd = (w0 + lane >= P0 && w0 + lane < P1) ? codes[w0 + lane] : 0u;
      for (; w0 < P1; w0 += 64) {
        const uint64_t x = window_bits<VR_XPOSE_A>(m, cd, w0, P0, P1, lane, active);
        if (w0 + 64 < P1) {
          const uint32_t q = w0 + 64 + lane;
          cd = q < P1 ? codes[q] : 0u;
        }
        if ((w0 & bmask) == 0 && w0 >= P0) {  // boundary q = w0: count before it
          c0rel[(size_t)(w0 >> bits) * LANES + lane] = cw;
          if (lane == 0) c0seg[w0 >> bits] = sidx;
        }
        cw += popc64(x);
      }
    }
    seg_tot[(size_t)sidx * LANES + lane] = cw;
  }
}

// Interval c of the EST table from the included counts at its two boundaries: c0 = segment
// base + relative count (k_countA); the end of the last, possibly partial, interval is
// extrapolated to a full 2^b span so the step keeps its meaning. L_c is 2^15 below the
// doubled rank 2 c0 + 1 at the boundary (modulo 2^32); D_c = floor(2 (c0' - c0) / 4096).
__device__ inline uint32_t c0_at(uint32_t c, int lane, const uint32_t* c0rel, const uint32_t* c0seg,
                                 const uint32_t* segpre) {
  return segpre[(size_t)c0seg[c] * LANES + lane] + c0rel[(size_t)c * LANES + lane];
}

__global__ void k_c0(const uint32_t* __restrict__ c0rel, const uint32_t* __restrict__ c0seg,
                     const uint32_t* __restrict__ segpre, const uint32_t* __restrict__ total,
                     uint32_t nc, int bits, int64_t M, uint2* __restrict__ ftab) {
  const uint32_t c = blockIdx.x;
  const int lane = threadIdx.x;
  const uint32_t a = c0_at(c, lane, c0rel, c0seg, segpre);
  uint64_t d;  // included pairs over the (extrapolated) interval
  if (c + 1 < nc) {
    d = c0_at(c + 1, lane, c0rel, c0seg, segpre) - a;
  } else {
    const uint64_t span = (uint64_t)M - ((uint64_t)c << bits);
    d = ((uint64_t)(total[lane] - a) << bits) / span;
  }
  ftab[(size_t)c * LANES + lane] = make_uint2(2u * a + 1u - 32768u, (uint32_t)((2 * d) >> EST_STEP_BITS));
}

// EST 3 / 5: the wave-uniform estimate {L, R} (est3_params) into ftab row 0, EST 5's coarse
// position shift into row 1
__global__ void k_c0_u(uint32_t Lu, uint32_t Ru, uint32_t sh, uint32_t g, uint2* __restrict__ ftab) {
  ftab[0] = make_uint2(Lu, Ru);
  ftab[1] = make_uint2(sh, g);
}

// EST 3 estimate of a call whose subsets all hold k stimuli: M' = k (k - 1) / 2 included
// pairs per lane, R = floor(2^32 M'/M) (host and device use these same two words; a lane
// whose count differs, e.g. an index row with repeats, is caught by the A-side check).
static inline uint2 est3_params(int64_t k, int64_t M) {
  const unsigned __int128 mp = (unsigned __int128)(uint64_t)(k * (k - 1) / 2);
  unsigned __int128 r = M > 0 ? (mp << 32) / (unsigned __int128)(uint64_t)M : 0;
  if (r > 0xffffffffu) r = 0xffffffffu;
  return make_uint2(1u - 32768u, (uint32_t)r);
}

// EST 2: the one-interval estimate {L, R} per lane (f32 bit patterns in ftab row 0)
__global__ void k_c0_lin(const uint32_t* __restrict__ total, int64_t M, uint2* __restrict__ ftab) {
  const int lane = threadIdx.x;
  const float R = (float)(2.0 * (double)total[lane] / (double)M);
  ftab[lane] = make_uint2(__float_as_uint(1.0f - 32768.0f), __float_as_uint(R));
}

// EST 3 up-front check (est_predict): lane `lane`'s included count a at coarse boundary
// q = c 2^bits against the wave-uniform estimate. The first included pair at or after q has
// doubled rank >= 2a + 1 while the window it must fall in is centred on
// 1 + (2 q R >> 32); a boundary already 2^15 + 2^13 off (the 2^13: slack for the next
// included pair's distance and tie groups) means a stored rank of that lane falls outside
// its window there, so the pass would be flagged. Lanes >= nl hold no subset; lane 0 of a
// full-first pass (the full set, EST 4) is exact by construction.
__global__ void k_est_predict(const uint32_t* __restrict__ c0rel, const uint32_t* __restrict__ c0seg,
                              const uint32_t* __restrict__ segpre, int bits, uint32_t Ru, int nl, int skip0,
                              uint32_t* __restrict__ flag) {
  const uint32_t c = blockIdx.x;
  const int lane = threadIdx.x;
  if (lane >= nl || (skip0 && lane == 0)) return;
  const uint64_t q = (uint64_t)c << bits;
  const int64_t a = (int64_t)c0_at(c, lane, c0rel, c0seg, segpre);
  const int64_t dv = 2 * a - (int64_t)((2 * q * (uint64_t)Ru) >> 32);
  const int64_t lim = (1 << 15) + (1 << 13);
  if (dv > lim || dv < -lim) *flag = 1u;  // benign race: every writer stores 1
}

// ---------------------------------------------------------------------------------
// A pass
// ---------------------------------------------------------------------------------
// EST: the k_rankA outputs besides TB
struct EstA {
  const uint32_t* segpre;  // [nseg][64] included pairs before each A segment (k_countA scan)
  const uint2* ftab;       // interval table (k_c0), tabrows rows
  uint32_t tabrows;
  int bits;
  uint32_t* viol;          // this pass's flag: some stored rank is not recoverable
  int nl;                  // lanes holding a subset (the others have no included pair)
};

// rows [r0, r0 + cnt) of TB get y mod 2^16 (EST); bad |= some row's y is not recoverable.
// lo is monotone in the position, so the group's two end rows bound the rest.
template <int EST>
__device__ inline void store_rows_est(uint16_t* __restrict__ TB, uint32_t stride, uint32_t r0,
                                      uint32_t cnt, int lane, uint32_t y, const EstLo& el, bool& bad) {
  if (cnt == 0) return;
  // a group inside one 64-position window is covered by that window's check (k_rankA)
  if (VR_EST_CHECK && (r0 >> 6) != ((r0 + cnt - 1u) >> 6))
    bad |= est_bad(y, est_lo_t<EST>(el, r0, lane)) || est_bad(y, est_lo_t<EST>(el, r0 + cnt - 1u, lane));
  uint16_t* row = TB + (size_t)r0 * stride + lane;
  if constexpr (EST == 4) {  // lane 0 (the full set): y - d(r) per row, positive (est4_shift)
    const uint32_t l0 = 0u - (uint32_t)(lane == 0);
    if (VR_EST_CHECK) bad |= lane == 0 && (int32_t)(y - est4_shift(el.Ru, r0 + cnt - 1u)) < 1;
    for (uint32_t i = 0; i < cnt; ++i, row += stride) tb_store((uint16_t)(y - (est4_shift(el.Ru, r0 + i) & l0)), row);
    return;
  }
  uint32_t i = 0;
  for (; i + 4 <= cnt; i += 4, row += 4 * (size_t)stride) {
    tb_store((uint16_t)y, row);
    tb_store((uint16_t)y, row + stride);
    tb_store((uint16_t)y, row + 2 * stride);
    tb_store((uint16_t)y, row + 3 * stride);
  }
  for (; i < cnt; ++i, row += stride) tb_store((uint16_t)y, row);
}

// EST 5 / 6: the same rows at their triangle indices (row_t(r) for A position r), lane 63 of
// each row holding the row's coarse A position r >> sh instead of a rank
template <int EST, typename RowT>
__device__ inline void store_rows_tri(uint16_t* __restrict__ TB, uint32_t r0, uint32_t cnt, int lane,
                                      uint32_t y, const EstLo& el, bool& bad, RowT&& row_t) {
  if (cnt == 0) return;
  if (VR_EST_CHECK && (r0 >> 6) != ((r0 + cnt - 1u) >> 6))
    bad |= est_bad(y, est_lo_t<EST>(el, r0, lane)) || est_bad(y, est_lo_t<EST>(el, r0 + cnt - 1u, lane));
  for (uint32_t i = 0; i < cnt; ++i) {
    const uint32_t r = r0 + i;
    const uint16_t v = lane == LANES - 1 ? (uint16_t)tri_tag<EST>(el, r) : (uint16_t)y;
    tb_store(v, TB + (size_t)row_t(r) * LANES + lane);
  }
}

// A side. Exact form (EST false): chunk-relative doubled ranks y - 2 lp (u16 or u32) and
// the chunk-start counts lpA for baseA. EST form: absolute doubled ranks modulo 2^16,
// each checked against the count estimate the B side will use.
template <bool LDS, bool FULL, typename TBT, bool BIGT, int EST>
__global__ __launch_bounds__(ENG_THREADS, 8) void k_rankA(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gstart,
    const uint32_t* __restrict__ chunk_g, const uint32_t* __restrict__ gflag, uint32_t nchunks,
    const uint64_t* __restrict__ gmask, int64_t n, TBT* __restrict__ TB, int lw,
    uint32_t* __restrict__ lpA, uint32_t* __restrict__ seg_tot, uint64_t* __restrict__ seg_part,
    uint32_t nseg, EstA est, const uint32_t* __restrict__ segpos, uint32_t* __restrict__ queue) {
  static_assert(!EST || sizeof(TBT) == 2, "EST ranks are u16");
  constexpr bool TRI = EST >= 5;  // triangle-order TB rows (EST 5 / 6)
  static_assert(!TRI || FULL, "triangle-order passes use whole 64-lane rows");
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  EstLo el{nullptr, 0, 0.f, 0.f, 0u, 0u, 0u, 0u};
  if constexpr (EST != 0)
    el = est_setup<EST>(est.ftab, est.tabrows, est.bits, reinterpret_cast<uint2*>(smask + (LDS ? n : 0)));
  // TRI: triangle index and lane-63 tag of each position of window wt (lane j: position
  // wt + j), computed once per window in the vector unit; rows of a tie group that began in
  // an earlier window get theirs from their code (scalar loads)
  uint32_t tl = 0, tg = 0, wt = 0;
  auto row_t = [&](uint32_t r) -> uint32_t {
    return r - wt < 64u ? readlane_u32(tl, r - wt) : tri32(sload(codes + r), (uint32_t)n);
  };
  (void)row_t;
  const int lane = threadIdx.x & 63;
  const bool active = FULL || lane < lw;
  const uint32_t stride = FULL ? (uint32_t)LANES : (uint32_t)lw;
  const uint32_t wave = wave_uniform(blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6));
  bool bad = false;  // EST: a stored rank is not recoverable from its 16 bits
  // One segment [P0, P1) = chunks [c0, c1) (exact form) or a work-queue segment (EST:
  // segpos, no chunk bookkeeping), partial sums at index sidx (k_rankB's walk_segment)
  auto walk_segment = [&](uint32_t sidx, uint32_t c0, uint32_t c1, uint32_t P0, uint32_t P1) {
    uint64_t tie = 0;  // sum over groups of k^3 - k (k < 2^16)
    u128 tie_big = 0;  //   (k >= 2^16)
    uint32_t cw = 0;   // included count before the window (segment-relative)
    if (P0 < P1) {
      // EST: 2 x (included pairs before this segment); exact form: 0
      const uint32_t y0 = EST ? 2u * est.segpre[(size_t)sidx * LANES + lane] : 0u;
      uint32_t cn = c0;  // next chunk whose start is not yet recorded
      uint32_t pn = P0;
      uint32_t lp = 0;      // count at the current chunk's start (exact form)
      while (cn < c1 && pn == P0) {
        if (!EST) lpA[(size_t)cn * LANES + lane] = 0;
        ++cn;
        pn = cn < c1 ? chunk_start(gstart, chunk_g, cn) : P1;
      }
      uint32_t gs = P0, cgs = 0;  // open group start and the count before it
      // close the open group [gs, xe) given ce = included count before xe
      auto close = [&](uint32_t xe, uint32_t ce) {
        tie_add<BIGT>(tie, tie_big, ce - cgs);
        if (active) {
          if constexpr (TRI)
            store_rows_tri<EST>(reinterpret_cast<uint16_t*>(TB), gs, xe - gs, lane, y0 + cgs + ce + 1u, el, bad,
                                row_t);
          else if constexpr (EST)
            store_rows_est<EST>(reinterpret_cast<uint16_t*>(TB), stride, gs, xe - gs, lane, y0 + cgs + ce + 1u,
                                el, bad);
          else
            store_rows<FULL, TBT>(TB, stride, gs, xe - gs, lane, (TBT)(cgs + ce + 1u - 2u * lp));
        }
        gs = xe;
        cgs = ce;
        while (cn < c1 && pn == xe) {  // chunk boundaries are group starts
          if (!EST) lpA[(size_t)cn * LANES + lane] = ce;
          lp = ce;
          ++cn;
          pn = cn < c1 ? chunk_start(gstart, chunk_g, cn) : P1;
        }
      };
      uint32_t w0 = P0 & ~63u;
      // next window's codes (vector, lane j = pair w0 + j) and flags (scalar), one ahead
      uint32_t cd = (w0 + lane >= P0 && w0 + lane < P1) ? codes[w0 + lane] : 0u;
      uint32_t f0 = sload(gflag + (w0 >> 5)), f1 = sload(gflag + (w0 >> 5) + 1);
      for (; w0 < P1; w0 += 64) {
        if constexpr (TRI) {
          tl = (w0 + lane >= P0 && w0 + lane < P1) ? tri32(cd, (uint32_t)n) : 0u;
          tg = tri_tag<EST>(el, w0 + (uint32_t)lane);
          wt = w0;
        }
  #if VR_PROBE_WBA  // timing probe only (wrong scores): k_rankA without mask lookups / transposes
        const uint64_t x = active ? (0xF7DFBEFDFBF7EFDFull ^ ((uint64_t)(cd & 7u) << 3)) : 0ull;
  #else
        const uint64_t x = window_bits<VR_XPOSE_A>(m, cd, w0, P0, P1, lane, active);
  #endif
        uint64_t F = restrict_flags(((uint64_t)f1 << 32) | f0, w0, P0, P1);
        asm volatile("" ::"v"(x) : "memory");
        if constexpr (EST) {
          // Every group that starts and ends in this window has y = y0 + cgs + ce + 1 in
          // [Y0, Y0 + 128] (Y0 = y0 + 2 cw + 1: cw <= cgs <= ce <= cw + 64), and lo is monotone,
          // in [lo(w0), lo(w0 + 63)]: these two checks make all of them recoverable. Longer
          // groups are checked where they close.
          if (VR_EST_CHECK) {
            const uint32_t Y0 = y0 + 2u * cw + 1u;
            bad |= est_bad(Y0, est_lo_t<EST>(el, w0 + 63u, lane)) || est_bad(Y0 + 128u, est_lo_t<EST>(el, w0, lane));
          }
        }
        if (w0 + 64 < P1) {
          const uint32_t q = w0 + 64 + lane;
          cd = q < P1 ? codes[q] : 0u;
          f0 = sload(gflag + ((w0 + 64) >> 5));
          f1 = sload(gflag + ((w0 + 64) >> 5) + 1);
        }
        if (F == ~0ull) {  // every position starts a group: close the carried one, then
          close(w0, cw);   // 63 singletons need only a running count
          if (cn >= c1 || pn > w0 + 63u) {
            uint32_t t = EST ? y0 + 2u * cw + 1u : 2u * (cw - lp) + 1u;
            TBT* row = TB + (size_t)w0 * stride + lane;
            if constexpr (TRI) {
  #pragma unroll
              for (int j = 0; j < 63; ++j) {
                const uint32_t bit = (uint32_t)(x >> j) & 1u;
                const uint32_t v = t + bit;
                const uint32_t pc = readlane_u32(tg, j);
                tb_store((TBT)(lane == LANES - 1 ? pc : v), TB + (size_t)readlane_u32(tl, j) * LANES + lane);
                t = v + bit;
              }
            } else {
  #if VR_PROBE_STW  // timing probe only (wrong TB layout): one 4-byte store per two rows
            uint32_t* row2 = reinterpret_cast<uint32_t*>(TB + (size_t)w0 * stride) + lane;
  #pragma unroll
            for (int j = 0; j < 62; j += 2) {
              const uint32_t b0 = (uint32_t)(x >> j) & 1u, b1 = (uint32_t)(x >> (j + 1)) & 1u;
              const uint32_t v0 = t + b0, v1 = v0 + b0 + b1;
              if (active) __builtin_nontemporal_store(v0 | (v1 << 16), row2 + (size_t)j * stride / 2);
              t = v1 + b1;
            }
            if (active) tb_store((TBT)t, row + (size_t)62 * stride);
  #else
  #pragma unroll
            for (int j = 0; j < 63; ++j) {
              const uint32_t bit = (uint32_t)(x >> j) & 1u;
              const uint32_t v = t + bit;
              if constexpr (EST == 4) {  // lane 0: shifted (est4_shift; singletons: y - d >= 2)
                const uint32_t sub = est4_shift(el.Ru, w0 + (uint32_t)j) & (0u - (uint32_t)(lane == 0));
                if (active) tb_store((TBT)(v - sub), row + (size_t)j * stride);
              } else {
                if (active) tb_store((TBT)v, row + (size_t)j * stride);
              }
              t = v + bit;
            }
  #endif
            }
            gs = w0 + 63u;
            cgs = cw + popc64(x & lowmask(63));
            F = 0;
          } else {
            F &= ~1ull;
          }
        }
        while (F) {
          const uint32_t b = (uint32_t)__builtin_ctzll(F);
          F &= F - 1;
          close(w0 + b, cw + popc64(x & lowmask(b)));
        }
        cw += popc64(x);
      }
      if ((P1 & 63u) == 0) close(P1, cw);  // a 64-aligned segment end is in no window
    }
    const size_t o = (size_t)sidx * LANES + lane, fs = (size_t)nseg * LANES;
    const u128 t = tie_big + tie;
    seg_tot[o] = cw;
    seg_part[PA_TIEL * fs + o] = (uint64_t)t;
    seg_part[PA_TIEH * fs + o] = (uint64_t)(t >> 64);
  };
  if constexpr (EST != 0) {
    for (;;) {
      const uint32_t sidx = next_segment(queue);
      if (sidx >= nseg) break;
      walk_segment(sidx, 0u, 0u, segpos[sidx], segpos[sidx + 1]);
    }
    if (__ballot(bad && lane < est.nl) != 0 && lane == 0) *est.viol = 1u;  // benign race: every writer stores 1
  } else {
    const Segment sg = my_segment(nchunks, nseg, wave);
    const bool any = sg.c0 < sg.c1;
    walk_segment(wave, sg.c0, sg.c1, any ? chunk_start(gstart, chunk_g, sg.c0) : 0u,
                 any ? chunk_start(gstart, chunk_g, sg.c1) : 0u);
  }
}

// ---------------------------------------------------------------------------------
// per-lane exclusive scan over segments: tot[nseg][64] -> pre[nseg][64], total[64]
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_lscan_reduce(const uint32_t* __restrict__ tot,
                                                      uint32_t nseg, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t part[16][LANES];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const uint32_t s0 = blockIdx.x * SCAN_SEGS + v * (SCAN_SEGS / 16);
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_SEGS / 16; ++i)
    if (s0 + i < nseg) s += tot[(size_t)(s0 + i) * LANES + lane];
  part[v][lane] = s;
  __syncthreads();
  if (v == 0) {
    uint32_t r = 0;
    for (int u = 0; u < 16; ++u) r += part[u][lane];
    bsum[(size_t)blockIdx.x * LANES + lane] = r;
  }
}

__global__ void k_lscan_top(uint32_t* __restrict__ bsum, uint32_t nblk, uint32_t* __restrict__ total) {
  const int lane = threadIdx.x;
  uint32_t run = 0;
  for (uint32_t b = 0; b < nblk; ++b) {
    const uint32_t t = bsum[(size_t)b * LANES + lane];
    bsum[(size_t)b * LANES + lane] = run;
    run += t;
  }
  if (total) total[lane] = run;
}

__global__ __launch_bounds__(1024) void k_lscan_down(const uint32_t* __restrict__ tot,
                                                    uint32_t nseg, const uint32_t* __restrict__ bsum,
                                                    uint32_t* __restrict__ pre) {
  __shared__ uint32_t part[16][LANES];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  constexpr int PER = SCAN_SEGS / 16;
  const uint32_t s0 = blockIdx.x * SCAN_SEGS + v * PER;
  uint32_t t[PER];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    t[i] = s0 + i < nseg ? tot[(size_t)(s0 + i) * LANES + lane] : 0u;
    s += t[i];
  }
  part[v][lane] = s;
  __syncthreads();
  uint32_t run = bsum[(size_t)blockIdx.x * LANES + lane];
  for (int u = 0; u < v; ++u) run += part[u][lane];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    if (s0 + i < nseg) pre[(size_t)(s0 + i) * LANES + lane] = run;
    run += t[i];
  }
}

static int lane_scan(const uint32_t* tot, uint32_t nseg, uint32_t* bsum, uint32_t* pre,
                     uint32_t* total, hipStream_t st) {
  const uint32_t nb = scan_blocks(nseg);
  k_lscan_reduce<<<nb, 1024, 0, st>>>(tot, nseg, bsum);
  VR_CHECK_LAUNCH();
  k_lscan_top<<<1, LANES, 0, st>>>(bsum, nb, total);
  VR_CHECK_LAUNCH();
  k_lscan_down<<<nb, 1024, 0, st>>>(tot, nseg, bsum, pre);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

__global__ void k_add_base(const uint32_t* __restrict__ lpA, const uint32_t* __restrict__ segpre,
                           uint32_t nchunks, uint32_t nwaves, uint32_t* __restrict__ baseA) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)nchunks * LANES) return;
  const uint32_t c = (uint32_t)(i / LANES), lane = (uint32_t)(i % LANES);
  baseA[i] = segpre[(size_t)seg_of_chunk(c, nchunks, nwaves) * LANES + lane] + lpA[i];
}

// ---------------------------------------------------------------------------------
// B pass
// ---------------------------------------------------------------------------------
// Loads only. Per window three coalesced rows (codes, posA, chunkA) fetched one window
// ahead; per pair its TB row (HBM, random) and A-chunk base row (L2-resident), issued 16
// pairs at a time.
#ifndef VR_RANKB_MINW
#define VR_RANKB_MINW 8  // waves per SIMD the B pass is compiled for (8: 64 VGPRs)
#endif
#ifndef VR_RANKB_EST_MINW
#define VR_RANKB_EST_MINW 8  // EST B walk: 8 waves per SIMD (two 1024-thread workgroups per CU)
#endif
#ifndef VR_XW_SLO
#define VR_XW_SLO 0  // EST 3 prefetching walk: 1 = low ends in SALU from the address readlane (A/B; spills SGPRs)
#endif
#ifndef VR_RANKB_PIPE
#define VR_RANKB_PIPE 0  // 1: gather batch h+1 in flight while batch h is consumed
#endif
constexpr int BB = 8;  // pairs per gather batch
#ifndef VR_TB_CACHE
#define VR_TB_CACHE " nt"  // TB rows are read once: streaming loads keep L2 for the baseA rows
#endif
#ifndef VR_PROBE_NO_BASEA
#define VR_PROBE_NO_BASEA 0
#endif

// BB pairs' yA = 2 baseA[chunkA] + TB[posA] for this lane. The loads are issued in the
// saddr form (wave-uniform 64-bit row address in SGPRs + 32-bit lane byte offset), which
// the compiler does not select on its own here; their completion is an explicit
// s_waitcnt tied to every result. This kernel issues no vector stores and all of the
// compiler's own vector loads are older than these, so its waits stay conservative.
template <typename TBT>
__device__ inline void gather_issue(const TBT* __restrict__ TB, const uint32_t* __restrict__ baseA,
                                    uint32_t stride, uint32_t pa, uint32_t ca, uint32_t j0,
                                    uint32_t lane_bt, uint32_t lane_b4, uint32_t t[BB], uint32_t b[BB]) {
#pragma unroll
  for (int q = 0; q < BB; ++q) {
    const char* trow = reinterpret_cast<const char*>(TB) +
                       (size_t)readlane_u32(pa, j0 + q) * (stride * sizeof(TBT));
    const char* brow = reinterpret_cast<const char*>(baseA) + (size_t)readlane_u32(ca, j0 + q) * (LANES * 4);
    if constexpr (sizeof(TBT) == 2)
      asm volatile("global_load_ushort %0, %1, %2" VR_TB_CACHE : "=v"(t[q]) : "v"(lane_bt), "s"(trow) : "memory");
    else
      asm volatile("global_load_dword %0, %1, %2" : "=v"(t[q]) : "v"(lane_bt), "s"(trow) : "memory");
#if VR_PROBE_NO_BASEA  // timing probe only: wrong scores
    b[q] = 0u;
#else
    asm volatile("global_load_dword %0, %1, %2" : "=v"(b[q]) : "v"(lane_b4), "s"(brow) : "memory");
#endif
  }
}

// wait until at most PENDING of this wave's loads are outstanding; ties t, b
template <int PENDING>
__device__ inline void gather_wait(uint32_t t[BB], uint32_t b[BB]) {
  static_assert(BB == 8, "the wait below names 16 registers");
  static_assert(PENDING == 0 || PENDING == 2 * BB, "vmcnt immediate");
  if constexpr (PENDING == 0)
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]),
                   "+v"(t[7]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]),
                   "+v"(b[6]), "+v"(b[7])
                 :
                 : "memory");
  else
    asm volatile("s_waitcnt vmcnt(16)"
                 : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]),
                   "+v"(t[7]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]),
                   "+v"(b[6]), "+v"(b[7])
                 :
                 : "memory");
}

#ifndef VR_EST_BB
#define VR_EST_BB 8  // EST: pairs per gather batch (8, 16 or 32 loads in flight per wave)
#endif
#ifndef VR_EST_ASM
#define VR_EST_ASM 1  // 0: plain loads (the compiler places the waits)
#endif
constexpr int EBB = VR_EST_BB;
static_assert(EBB == 4 || EBB == 8 || EBB == 16 || EBB == 32, "EST batch");

// EST: EBB pairs' TB entries only (absolute doubled ranks modulo 2^16), same load form
__device__ inline void gather_issue_t(const uint16_t* __restrict__ TB, uint32_t stride, uint32_t pa,
                                      uint32_t j0, uint32_t lane_bt, uint32_t t[EBB]) {
#pragma unroll
  for (int q = 0; q < EBB; ++q) {
    const char* trow = reinterpret_cast<const char*>(TB) + (size_t)readlane_u32(pa, j0 + q) * (stride * 2);
#if VR_XP & 16  // timing probe only (wrong scores): no TB row gathers, the row address stands in
    asm volatile("v_xor_b32 %0, %1, %2" : "=v"(t[q]) : "v"(lane_bt), "s"((uint32_t)(uintptr_t)trow) : "memory");
#else
    asm volatile("global_load_ushort %0, %1, %2" VR_TB_CACHE : "=v"(t[q]) : "v"(lane_bt), "s"(trow) : "memory");
#endif
  }
}

// EST 3 prefetching walk: the same loads, and each pair's window low end L + (2 posA R >> 32)
// computed in SALU from the row index the address already needed in an SGPR (one
// v_readlane per pair instead of two: the walk is bound by its vector-instruction issue,
// DESIGN.md §3.3)
__device__ inline void gather_issue_tl(const uint16_t* __restrict__ TB, uint32_t stride, uint32_t pa,
                                       uint32_t j0, uint32_t lane_bt, uint32_t t[EBB], uint32_t lo[EBB],
                                       uint32_t Lu, uint32_t Ru) {
#pragma unroll
  for (int q = 0; q < EBB; ++q) {
    const uint32_t r = readlane_u32(pa, j0 + q);
    const char* trow = reinterpret_cast<const char*>(TB) + (size_t)r * (stride * 2);
    lo[q] = Lu + __umulhi(r << 1, Ru);
#if VR_XP & 16  // timing probe only (wrong scores): no TB row gathers, the row address stands in
    asm volatile("v_xor_b32 %0, %1, %2" : "=v"(t[q]) : "v"(lane_bt), "s"((uint32_t)(uintptr_t)trow) : "memory");
#else
    asm volatile("global_load_ushort %0, %1, %2" VR_TB_CACHE : "=v"(t[q]) : "v"(lane_bt), "s"(trow) : "memory");
#endif
  }
}

// wait for all of this wave's loads; ties the EBB results (16 per asm statement: the first
// waits, the others only tell the compiler the registers are defined from here on)
__device__ inline void wait_tie16(uint32_t* t, bool wait) {
  if (wait)
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]),
                   "+v"(t[7]), "+v"(t[8]), "+v"(t[9]), "+v"(t[10]), "+v"(t[11]), "+v"(t[12]), "+v"(t[13]),
                   "+v"(t[14]), "+v"(t[15])
                 :
                 : "memory");
  else
    asm volatile(""
                 : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]),
                   "+v"(t[7]), "+v"(t[8]), "+v"(t[9]), "+v"(t[10]), "+v"(t[11]), "+v"(t[12]), "+v"(t[13]),
                   "+v"(t[14]), "+v"(t[15])
                 :
                 : "memory");
}

__device__ inline void gather_wait_t(uint32_t t[EBB]) {
  if constexpr (EBB == 4) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]) : : "memory");
  } else if constexpr (EBB == 8) {
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]),
                   "+v"(t[7])
                 :
                 : "memory");
  } else {
#pragma unroll
    for (int g = 0; g < EBB / 16; ++g) wait_tie16(t + 16 * g, g == 0);
  }
}

#ifndef VR_EST_ASM
#define VR_EST_ASM 1  // 0: plain loads (the compiler places the waits)
#endif
#ifndef VR_EST_D16
#define VR_EST_D16 0  // 1: two pairs' u16 entries per VGPR (short_d16 / short_d16_hi loads)
#endif

// EST, d16: wait for all of this wave's loads; ties the EBB / 2 packed registers
__device__ inline void gather_wait_t16(uint32_t p[EBB / 2]) {
  if constexpr (EBB == 8) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]) : : "memory");
  } else if constexpr (EBB == 16) {
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]), "+v"(p[6]),
                   "+v"(p[7])
                 :
                 : "memory");
  } else {
    wait_tie16(p, true);
  }
}

// EST, d16: pairs j0 + 2i and j0 + 2i + 1 land in the low / high half of t[i], so a batch
// of EBB pairs in flight holds EBB / 2 VGPRs
__device__ inline void gather_issue_t16(const uint16_t* __restrict__ TB, uint32_t stride, uint32_t pa,
                                        uint32_t j0, uint32_t lane_bt, uint32_t t[EBB / 2]) {
#pragma unroll
  for (int q = 0; q < EBB / 2; ++q) {
    const char* r0 = reinterpret_cast<const char*>(TB) + (size_t)readlane_u32(pa, j0 + 2 * q) * (stride * 2);
    const char* r1 = reinterpret_cast<const char*>(TB) + (size_t)readlane_u32(pa, j0 + 2 * q + 1) * (stride * 2);
    asm volatile("global_load_short_d16 %0, %1, %2" VR_TB_CACHE : "=v"(t[q]) : "v"(lane_bt), "s"(r0) : "memory");
    asm volatile("global_load_short_d16_hi %0, %1, %2" VR_TB_CACHE : "+v"(t[q]) : "v"(lane_bt), "s"(r1) : "memory");
  }
}

// EST: yA of the window's 64 pairs (TB row entry + the window low end), EBB pairs per
// batch, handed to fn(h, ya[EBB]). Default (EPS > 1, pipe_batch): batch H+1's loads are
// issued before batch H is waited for and consumed, so compiler-generated code (fn, the
// low ends) runs while asm loads are in flight. The compiler cannot see those loads, so
// this is correct only if that code never touches (reads, copies or spills) their
// destination VGPRs before the asm `s_waitcnt` that retires them. Nothing in the source
// can promise that: tests/test_isa_guard.py checks it on every build's code object
// (control-flow dataflow over every k_rankB instantiation, and zero scratch for the
// default forms). EPS = 1 waits for each batch right after issuing it.
#ifndef VR_EST_PIPE
#define VR_EST_PIPE 2  // EST: gather batches in flight per wave (software pipeline depth; 1 = none)
#endif
constexpr int EPS = VR_EST_PIPE;

// B side: the window low end of pair j of the window (lane j of pa / la holds pair j). EST 3
// and 4 read the join's precomputed value (EST 4's lane 0: 2 posA + 1 - 2^15).
template <int EST>
__device__ inline uint32_t est_lo_b(const EstLo& el, uint32_t pa, uint32_t la, int j, int lane, uint32_t tv) {
  if constexpr (EST == 5) {  // the tag in lane 63 of the gathered row (tv: this pair's loaded entry)
    return est5_lo_tag(el, readlane_u32(tv, LANES - 1));
  } else if constexpr (EST == 6) {
    return est_lo_pc(el, readlane_u32(tv, LANES - 1), lane, true);
  } else if constexpr (EST == 4) {
    const uint32_t l = readlane_u32(la, j);
    const uint32_t l0 = 2u * readlane_u32(pa, j) + (1u - 32768u);
    return lane == 0 ? l0 : l;
  } else if constexpr (EST == 3) {
    return readlane_u32(la, j);
  } else {
    return est_lo_t<EST>(el, readlane_u32(pa, j), lane);
  }
}

// wait until at most N of this wave's loads are outstanding; ties the EBB registers t
template <int N>
__device__ inline void gather_wait_n(uint32_t* t) {
  if constexpr (EBB == 4) {
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]) : "n"(N) : "memory");
  } else {
    static_assert(EBB == 8, "pipelined EST batches are 4 or 8 pairs");
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7])
                 : "n"(N)
                 : "memory");
  }
}

// Software-pipelined batch H of a window: batches H+1 .. H+EPS-1 are issued before it is
// consumed, so EPS batches (EPS * EBB loads) are in flight per wave while it computes.
template <int EST, int H, typename Fn>
__device__ inline void pipe_batch(const uint16_t* __restrict__ TB, uint32_t stride, const EstLo& el,
                                  uint32_t pa, uint32_t la, uint32_t lane_bt, int lane, uint32_t (&t)[EPS][EBB],
                                  Fn&& fn) {
  constexpr int NBT = 64 / EBB;
  if constexpr (H + EPS - 1 < NBT) gather_issue_t(TB, stride, pa, (H + EPS - 1) * EBB, lane_bt, t[(H + EPS - 1) % EPS]);
  constexpr int ahead = (NBT - 1 - H) < (EPS - 1) ? (NBT - 1 - H) : (EPS - 1);  // batches issued after H
  gather_wait_n<ahead * EBB>(t[H % EPS]);
  uint32_t y[EBB];
#pragma unroll
  for (int q = 0; q < EBB; ++q)
    y[q] = est_recover(t[H % EPS][q], est_lo_b<EST>(el, pa, la, H * EBB + q, lane, t[H % EPS][q]));
  fn(H, y);
  if constexpr (H + 1 < NBT) pipe_batch<EST, H + 1>(TB, stride, el, pa, la, lane_bt, lane, t, fn);
}

template <int EST, typename Fn>
__device__ inline void gather_window_est(const uint16_t* __restrict__ TB, uint32_t stride, const EstLo& el,
                                         uint32_t pa, uint32_t la, uint32_t lane_bt, int lane, Fn&& fn) {
  if constexpr (EPS > 1 && !VR_EST_D16) {
    // the walk is bound by the gathers' round trip: keep EPS batches in flight
    uint32_t t[EPS][EBB];
#pragma unroll
    for (int g = 0; g < EPS - 1; ++g) gather_issue_t(TB, stride, pa, g * EBB, lane_bt, t[g]);
    pipe_batch<EST, 0>(TB, stride, el, pa, la, lane_bt, lane, t, fn);
    return;
  }
#pragma unroll
  for (int h = 0; h < 64 / EBB; ++h) {
    uint32_t t[EBB];
    if constexpr (VR_EST_D16 && EBB >= 8) {
      uint32_t p[EBB / 2];
      gather_issue_t16(TB, stride, pa, h * EBB, lane_bt, p);
      gather_wait_t16(p);
#pragma unroll
      for (int q = 0; q < EBB / 2; ++q) {
        t[2 * q] = p[q];  // est_recover uses only the low 16 bits
        t[2 * q + 1] = p[q] >> 16;
      }
    } else if constexpr (VR_EST_ASM) {
      gather_issue_t(TB, stride, pa, h * EBB, lane_bt, t);
      gather_wait_t(t);
    } else {
#pragma unroll
      for (int q = 0; q < EBB; ++q) {
        const char* row = reinterpret_cast<const char*>(TB) + (size_t)readlane_u32(pa, h * EBB + q) * (stride * 2u);
        t[q] = __builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(row + lane_bt));
      }
    }
#pragma unroll
    for (int q = 0; q < EBB; ++q)  // EST 3: the join's precomputed low end (lane j = pair j)
      t[q] = est_recover(t[q], est_lo_b<EST>(el, pa, la, h * EBB + q, lane, t[q]));
    fn(h, t);
  }
}

// yA of the window's 64 pairs, batch by batch, handed to fn(h, ya[BB])
template <typename TBT, typename Fn>
__device__ inline void gather_window(const TBT* __restrict__ TB, const uint32_t* __restrict__ baseA,
                                     uint32_t stride, uint32_t pa, uint32_t ca, uint32_t lane_bt,
                                     uint32_t lane_b4, Fn&& fn) {
  if constexpr (VR_RANKB_PIPE) {
    uint32_t t[2][BB], b[2][BB];
    gather_issue<TBT>(TB, baseA, stride, pa, ca, 0, lane_bt, lane_b4, t[0], b[0]);
#pragma unroll
    for (int h = 0; h < 64 / BB; ++h) {
      const int cur = h & 1;
      if (h + 1 < 64 / BB) {
        gather_issue<TBT>(TB, baseA, stride, pa, ca, (h + 1) * BB, lane_bt, lane_b4, t[cur ^ 1], b[cur ^ 1]);
        gather_wait<2 * BB>(t[cur], b[cur]);
      } else {
        gather_wait<0>(t[cur], b[cur]);
      }
      uint32_t ya[BB];
#pragma unroll
      for (int q = 0; q < BB; ++q) ya[q] = 2u * b[cur][q] + t[cur][q];
      fn(h, ya);
    }
  } else {
#pragma unroll
    for (int h = 0; h < 64 / BB; ++h) {
      uint32_t t[BB], b[BB], ya[BB];
      gather_issue<TBT>(TB, baseA, stride, pa, ca, h * BB, lane_bt, lane_b4, t, b);
      gather_wait<0>(t, b);
#pragma unroll
      for (int q = 0; q < BB; ++q) ya[q] = 2u * b[q] + t[q];
      fn(h, ya);
    }
  }
}

#ifndef VR_XP
#define VR_XP 0  // timing probes of the prefetching walk's per-pair work (bitmask; wrong scores)
#endif
#ifndef VR_TAIL_CHECK
#define VR_TAIL_CHECK 1  // 0: probe builds only -- the tail invariants never flag
#endif
#ifndef VR_PROBE_WT
#define VR_PROBE_WT 0  // timing probe: per-wave start / end clocks of the last k_rankB launch
#endif
#if VR_PROBE_WT
__device__ uint64_t g_wt[2 * 16384];
#endif
#ifndef VR_XW_L2
#define VR_XW_L2 1  // the prefetching walk also with masks from L2 (n > 10,176); 0: the per-window walk there
#endif
#ifndef VR_XWIN
#define VR_XWIN 1  // EST 3 / 4 B walk: next window's streams and masks fetched inside the window (0: off)
#endif

// EST 3 / 4 B walk, prefetching form (VR_XWIN; the window low ends computed from the A
// positions in scalar registers, not streamed): every vector-memory load of the walk is
// issued from asm and retired by a counted asm `s_waitcnt vmcnt(N)`, so the compiler places
// no vmcnt wait of its own: the next window's streams S (codes, A positions: 2 loads) and
// its two L2 mask gathers M (when the masks are not in LDS) are issued between the window's
// TB row batches G[0..7] (8 loads each) and retired with them, and the next window's 64 x 64
// transpose runs while G[3] is in flight. A window boundary then costs only the drain of
// G[7] and the refill from G[0] -- no dependent mask round trip and no transpose with the
// gathers idle. Issue order:
//   S(w+1) G[0] G[1] G[2] M(w+1) G[3] ... G[7] | S(w+2) G'[0] ...
// (batch h is waited for once batch h+1 is issued: vmcnt(8); S is retired with G[0], M with
// G[2], the last batch with vmcnt(0)).
// Nothing is in flight across the loop's back edge (G[7] is retired with vmcnt(0)), so no
// register holding an asm load result is live there. tests/test_isa_guard.py checks the
// generated code for every register these asm loads define.
__device__ inline void xw_ld2(const uint32_t* a, const uint32_t* b, uint32_t voff, uint32_t& x, uint32_t& y) {
  asm volatile("global_load_dword %0, %1, %2" : "=v"(x) : "v"(voff), "s"(a) : "memory");
  asm volatile("global_load_dword %0, %1, %2" : "=v"(y) : "v"(voff), "s"(b) : "memory");
}
// (s_nop 4: five wait states between any VALU write of the base SGPRs -- an SGPR spill
// restored by v_readlane, round 5's fault -- and the loads reading them; hipcc pads nothing
// inside an asm statement. tests/test_isa_guard.py checks every asm load for it.)
__device__ inline void xw_ldm(const uint64_t* m, uint32_t code, uint64_t& a, uint64_t& b) {
  asm volatile("s_nop 4\n\tglobal_load_dwordx2 %0, %1, %2" : "=v"(a) : "v"((code >> 16) * 8u), "s"(m) : "memory");
  asm volatile("global_load_dwordx2 %0, %1, %2" : "=v"(b) : "v"((code & 0xffffu) * 8u), "s"(m) : "memory");
}

// B side. Exact form: yA = 2 baseA[chunkA] + TB[posA] (two gathers per pair). EST form:
// yA recovered from TB[posA] (absolute, modulo 2^16) and the LDS count table (one gather).
template <bool LDS, bool FULL, typename TBT, bool BIGT, int EST>
__global__ __launch_bounds__(ENG_THREADS, EST ? VR_RANKB_EST_MINW : VR_RANKB_MINW) void k_rankB(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gstart,
    const uint32_t* __restrict__ chunk_g, const uint32_t* __restrict__ gflag, uint32_t nchunks,
    const uint64_t* __restrict__ gmask, int64_t n, const TBT* __restrict__ TB, int lw,
    const uint32_t* __restrict__ posA_byB, const uint32_t* __restrict__ chunkA_byB,
    const uint32_t* __restrict__ baseA, uint32_t* __restrict__ seg_tot,
    uint64_t* __restrict__ seg_part, uint32_t nseg, const uint2* __restrict__ ftab,
    uint32_t tabrows, int bits, const uint32_t* __restrict__ segpos, uint32_t* __restrict__ queue) {
  static_assert(!EST || sizeof(TBT) == 2, "EST ranks are u16");
  constexpr int NB = EST ? EBB : BB;  // pairs per gather batch
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  EstLo el{nullptr, 0, 0.f, 0.f, 0u, 0u, 0u, 0u};
  if constexpr (EST != 0) el = est_setup<EST>(ftab, tabrows, bits, reinterpret_cast<uint2*>(smask + (LDS ? n : 0)));
  const int lane = threadIdx.x & 63;
  const bool active = FULL || lane < lw;
  const uint32_t stride = FULL ? (uint32_t)LANES : (uint32_t)lw;
  const uint32_t wave = wave_uniform(blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6));
#if VR_PROBE_WT
  if (lane == 0 && wave < 16384u) g_wt[wave] = wall_clock64();
#endif
  // One segment [P0, P1) of B positions (a B tie-group start each), partial sums at index
  // sidx. EST passes: segments of ~M / est_nseg positions (segpos, k_seg_table) taken from
  // a work queue until none is left, so waves that run slow take fewer of them and the
  // launch does not end on a tail of late waves; the partial sums stay indexed by segment,
  // so the scores do not depend on which wave walked what. Exact form: the wave's static
  // chunk range.
  auto walk_segment = [&](uint32_t sidx, uint32_t P0, uint32_t P1) {
    u128 acc = 0;       // sum over B groups of S y'_B
    uint64_t St = 0;    // sum of S (= sum of included yA)
    uint64_t tie = 0;   // sum of k^3 - k
    u128 tie_big = 0;
    uint32_t cw = 0;
    if (P0 < P1) {
      uint32_t cgs = 0;
      uint64_t S = 0;  // sum of included yA (absolute doubled A midranks) in the open group
      auto close = [&](uint32_t ce) {
        const uint32_t y = cgs + ce + 1u;
        acc += (u128)S * y;
        St += S;
        tie_add<BIGT>(tie, tie_big, ce - cgs);
        S = 0;
        cgs = ce;
      };
      // EST 3 / 4 (small tie groups): the prefetching walk, which computes the window low
      // ends from the A positions (a join's streamed low ends, VISREPS_ENGINE_LO_JOIN=1, hold
      // the same values and are not read)
      // (with masks from L2 -- n > 10,176 -- too, VR_XW_L2; round 5 restricted it to LDS masks
      // after a MEMORY_APERTURE_VIOLATION, whose cause was a probe build's SGPR spill restored
      // by v_readlane right before the asm mask load that reads it: see xw_ldm)
      constexpr bool XW = VR_XWIN && EST == 3 && !BIGT && (LDS || VR_XW_L2);
      constexpr bool walked = XW;
      if constexpr (XW) {
        static_assert(EBB == 8, "prefetching batches are 8 pairs");
        {
          const uint16_t* TB16 = reinterpret_cast<const uint16_t*>(TB);
          uint32_t lane_bt;
          asm("" : "=v"(lane_bt) : "0"((uint32_t)lane * 2u));
          // stream offset of window wv: lanes past the segment end re-read its last position
          auto voff_of = [&](uint32_t wv) -> uint32_t {
            const uint32_t lim = wave_uniform(min(63u, P1 - 1u - wv));
            return min((uint32_t)lane, lim) * 4u;
          };
          // inclusion bits of window wv from its two mask words per lane
          auto bits_of = [&](uint32_t wv, uint64_t ma, uint64_t mb) -> uint64_t {
            const uint32_t pos = wv + (uint32_t)lane;
            const uint64_t v = transpose64<VR_XPOSE_B>((pos >= P0 && pos < P1) ? (ma & mb) : 0ull, lane);
            return active ? v : 0ull;
          };
          uint32_t w = P0 & ~63u;
          uint32_t cd, pa;
          xw_ld2(codes + w, posA_byB + w, voff_of(w), cd, pa);
          asm volatile("s_waitcnt vmcnt(0)" : "+v"(cd), "+v"(pa) : : "memory");
          uint64_t x;
          if constexpr (!LDS) {
            uint64_t ma, mb;
            xw_ldm(m, cd, ma, mb);
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(ma), "+v"(mb) : : "memory");
            x = bits_of(w, ma, mb);
          } else {
            x = window_bits<VR_XPOSE_B>(m, cd, w, P0, P1, lane, active);
          }
          // group-start flags of the window (scalar loads), fetched one window ahead
          uint32_t f0 = sload(gflag + (w >> 5)), f1 = sload(gflag + (w >> 5) + 1);
          for (;;) {
            const bool more = w + 64 < P1;
            const uint32_t wn = more ? w + 64 : w;
            uint32_t cdn, pan;
            const uint64_t F = restrict_flags(((uint64_t)f1 << 32) | f0, w, P0, P1);
            f0 = sload(gflag + (wn >> 5));
            f1 = sload(gflag + (wn >> 5) + 1);
            uint64_t xn = 0;
            // the window's batch pipeline; proc(h, ya) consumes batch h's recovered A ranks
            // (issued inside each of its two instances: a load in flight across the branch into
            // them would be copied between registers before its wait)
            // batch issue: the TB row gathers of pairs j0 .. j0 + 7 (and, VR_XW_SLO, their low ends)
            auto issue = [&](uint32_t j0, uint32_t* t, uint32_t* lq) {
  #if VR_XW_SLO
              gather_issue_tl(TB16, stride, pa, j0, lane_bt, t, lq, el.Lu, el.Ru);
  #else
              (void)lq;
              gather_issue_t(TB16, stride, pa, j0, lane_bt, t);
  #endif
            };
            auto pipeline = [&](auto&& proc) {
              uint64_t ma = 0, mb = 0;
              uint32_t t[2][EBB], lq[2][EBB];
              xw_ld2(codes + wn, posA_byB + wn, voff_of(wn), cdn, pan);  // S(w+1)
              issue(0, t[0], lq[0]);
  #pragma unroll
              for (int h = 0; h < 64 / EBB; ++h) {
                uint32_t(&cur)[EBB] = t[h & 1];
                if (h + 1 < 64 / EBB) {
                  issue((h + 1) * EBB, t[(h + 1) & 1], lq[(h + 1) & 1]);
                  gather_wait_n<EBB>(cur);
                  if (h == 0) asm volatile("" : "+v"(cdn), "+v"(pan));  // S(w+1): older than G[0]
                  if constexpr (!LDS) {
                    if (h == 1) xw_ldm(m, cdn, ma, mb);  // M(w+1), behind G[2]
                  }
                  if (h == 2) {  // only G[3] may be in flight: M(w+1) is retired
                    if constexpr (!LDS) {
                      asm volatile("" : "+v"(ma), "+v"(mb));
                      xn = bits_of(wn, ma, mb);
                    } else {
  #if VR_XP & 8  // timing probe only (wrong scores): the mask lookups without the 64 x 64 transpose
                      const uint32_t pn = wn + (uint32_t)lane;
                      xn = (active && pn >= P0 && pn < P1) ? (m[cdn >> 16] & m[cdn & 0xffffu]) : 0ull;
  #else
                      xn = window_bits<VR_XPOSE_B>(m, cdn, wn, P0, P1, lane, active);
  #endif
                    }
                  }
                } else {
                  gather_wait_n<0>(cur);
                }
                proc(h, cur, lq[h & 1]);
              }
            };
  #if VR_XW_SLO
            // pair j's window low end (gather_issue_tl: scalar, from its row index)
            auto recover = [&](uint32_t v, uint32_t lo) -> uint32_t { return est_recover(v, lo); };
  #else
            // the window low ends of the window's A positions, lane j = pair j (3 VALU ops)
            const uint32_t la = el.Lu + __umulhi(pa << 1, el.Ru);
            auto recover = [&](uint32_t v, uint32_t j) -> uint32_t { return est_recover(v, readlane_u32(la, j)); };
  #endif
            auto fast_proc = [&](uint64_t& a64, uint32_t& c1) {
              return [&](int h, uint32_t* cur, const uint32_t* lo) {
  #pragma unroll
                for (int q = 0; q < EBB; ++q) {
                  const uint32_t j = h * EBB + q;
                  const uint32_t y = recover(cur[q], VR_XW_SLO ? lo[q] : j);
                  const uint32_t mk = (uint32_t)((int32_t)((uint32_t)(x >> (j & 32u)) << (31u - (j & 31u))) >> 31);
                  const uint32_t yb = y & mk;
                  if (j < 63) {
  #if VR_XP & 1  // timing probe only (wrong scores): no 64-bit multiply-add
                    a64 = (a64 & ~0xffffffffull) | (uint32_t)((uint32_t)a64 + (yb ^ c1));
  #else
                    a64 += (uint64_t)yb * c1;
  #endif
  #if VR_XP & 2  // timing probe only: no 64-bit running sum
                    c1 ^= yb & 1u;
  #else
                    St += yb;
  #endif
                    c1 -= mk;
                  } else {
                    S = yb;
                    cgs = c1 - 1u;
                  }
                }
              };
            };
            auto slow_proc = [&](int h, uint32_t* cur, const uint32_t* lo) {
  #pragma unroll
              for (int q = 0; q < EBB; ++q) {
                const uint32_t j = h * EBB + q;
                const uint32_t y = recover(cur[q], VR_XW_SLO ? lo[q] : j);
                if ((F >> j) & 1ull) close(cw + popc64(x & lowmask(j)));
                S += ((x >> j) & 1ull) ? (uint64_t)y : 0ull;
              }
            };
            if (F == ~0ull) {  // every position starts a group (the per-window form below explains)
              close(cw);
              uint64_t a64 = 0;
              uint32_t c1 = cw + 1u;
              pipeline(fast_proc(a64, c1));
              acc += (u128)a64 * 2u;
            } else {
              pipeline(slow_proc);
            }
            cw += popc64(x);
            if (!more) break;
            w = wn;
            cd = cdn;
            pa = pan;
            x = xn;
          }
        }
      }
      uint32_t w0 = P0 & ~63u;
      auto fetch = [&](uint32_t w, uint32_t& pa, uint32_t& ca, uint32_t& cd, uint32_t& f0,
                       uint32_t& f1) {
        const uint32_t pos = w + (uint32_t)lane;
        const bool valid = pos >= P0 && pos < P1;
        if constexpr (EST >= 5) {  // triangle-order TB: the row is the pair's triangle index
          cd = valid ? codes[pos] : 0u;
          pa = valid ? tri32(cd, (uint32_t)n) : 0u;
          ca = 0u;
          f0 = sload(gflag + (w >> 5));
          f1 = sload(gflag + (w >> 5) + 1);
          return;
        }
        pa = valid ? posA_byB[pos] : 0u;
        // EST 3/4: the window low end of the pair's A position, L + (2 posA R >> 32), computed
        // here per lane for the window's 64 pairs (three VALU ops per window lane, no stream),
        // or streamed from the join (VISREPS_ENGINE_LO_JOIN=1, A/B)
        if constexpr (EST >= 3)
          ca = !valid ? 0u : chunkA_byB ? chunkA_byB[pos] : el.Lu + __umulhi(pa << 1, el.Ru);
        else
          ca = (!EST && valid) ? chunkA_byB[pos] : 0u;
        cd = valid ? codes[pos] : 0u;
        f0 = sload(gflag + (w >> 5));
        f1 = sload(gflag + (w >> 5) + 1);
      };
      uint32_t pa = 0, ca = 0, cd = 0, f0 = 0, f1 = 0;
      if constexpr (!walked) fetch(w0, pa, ca, cd, f0, f1);
      for (; !walked && w0 < P1; w0 += 64) {
        const uint32_t pa_c = pa, ca_c = ca;
        uint32_t lane_b4, lane_bt;  // opaque per window, so the base + lane sum is not hoisted
        asm("" : "=v"(lane_b4) : "0"((uint32_t)lane * 4u));
        asm("" : "=v"(lane_bt) : "0"((uint32_t)lane * (uint32_t)sizeof(TBT)));
  #if VR_PROBE_WB  // timing probe only (wrong scores): no mask lookups, no transpose
        const uint64_t x = active ? (0xF7DFBEFDFBF7EFDFull ^ ((uint64_t)(cd & 7u) << 3)) : 0ull;
  #else
        const uint64_t x = window_bits<VR_XPOSE_B>(m, cd, w0, P0, P1, lane, active);
  #endif
        const uint64_t F = restrict_flags(((uint64_t)f1 << 32) | f0, w0, P0, P1);
        if (w0 + 64 < P1) fetch(w0 + 64, pa, ca, cd, f0, f1);
        auto gather = [&](auto&& fn) {
          if constexpr (EST)
            gather_window_est<EST>(reinterpret_cast<const uint16_t*>(TB), stride, el, pa_c, ca_c, lane_bt, lane, fn);
          else
            gather_window<TBT>(TB, baseA, stride, pa_c, ca_c, lane_bt, lane_b4, fn);
        };
        if (F == ~0ull) {
          // Every position starts a group (the normal case for continuous RDMs): after
          // closing the carried group, positions 0..62 are singletons, whose tie term is 0
          // and whose doubled midrank is 2 (c + 1) with c the included count before them;
          // position 63 opens the next group. The singleton products yA (c + 1) stay below
          // 2^50 (yA < 2^32, segment counts < 2^18), so a window sums them in 64 bits.
          close(cw);
          uint64_t a64 = 0;
          uint32_t c1 = cw + 1u;  // 1 + included count before position j
          gather([&](int h, uint32_t* ya) {
  #pragma unroll
            for (int q = 0; q < NB; ++q) {
              const uint32_t j = h * NB + q;
              // m = -(bit j of x): one sign-extending bit-field extract serves as the select
              // mask and the count increment (c1 - m = c1 + bit)
              const uint32_t m = (uint32_t)((int32_t)((uint32_t)(x >> (j & 32u)) << (31u - (j & 31u))) >> 31);
              const uint32_t yb = ya[q] & m;  // x is 0 on inactive lanes
              if (j < 63) {
  #if VR_PROBE_ACC == 1
                a64 += yb ^ c1;
                St += yb;
                c1 -= m;
  #elif VR_PROBE_ACC == 2
                a64 += yb ^ c1;
                c1 -= m;
  #elif VR_PROBE_ACC == 3
                c1 += yb;
  #else
                a64 += (uint64_t)yb * c1;
                St += yb;
                c1 -= m;
  #endif
              } else {
                S = yb;
                cgs = c1 - 1u;
              }
            }
          });
          acc += (u128)a64 * 2u;
        } else {
          gather([&](int h, uint32_t* ya) {
  #pragma unroll
            for (int q = 0; q < NB; ++q) {
              const uint32_t j = h * NB + q;
              if ((F >> j) & 1ull) close(cw + popc64(x & lowmask(j)));
              S += ((x >> j) & 1ull) ? (uint64_t)ya[q] : 0ull;  // x is 0 on inactive lanes
            }
          });
        }
        cw += popc64(x);
      }
      if ((P1 & 63u) == 0) close(cw);  // a 64-aligned segment end is in no window
    }
    const size_t o = (size_t)sidx * LANES + lane, fs = (size_t)nseg * LANES;
    const u128 tt = tie_big + tie;
    seg_tot[o] = cw;
    seg_part[PB_ACCL * fs + o] = (uint64_t)acc;
    seg_part[PB_ACCH * fs + o] = (uint64_t)(acc >> 64);
    seg_part[PB_ST * fs + o] = St;
    seg_part[PB_TIEL * fs + o] = (uint64_t)tt;
    seg_part[PB_TIEH * fs + o] = (uint64_t)(tt >> 64);
  };
  if constexpr (EST != 0) {
    for (;;) {
      const uint32_t s = next_segment(queue);
      if (s >= nseg) break;
      walk_segment(s, segpos[s], segpos[s + 1]);
    }
  } else {
    const Segment sg = my_segment(nchunks, nseg, wave);
    const bool any = sg.c0 < sg.c1;
    walk_segment(wave, any ? chunk_start(gstart, chunk_g, sg.c0) : 0u, any ? chunk_start(gstart, chunk_g, sg.c1) : 0u);
  }
#if VR_PROBE_WT
  if (lane == 0 && wave < 16384u) g_wt[16384u + wave] = wall_clock64();
#endif
}

// ---------------------------------------------------------------------------------
// Grid B walk: one B plan against R <= 4 A plans in one launch (the regions a model layer
// is scored against, evals.py:323-373). Every region's call draws the same bootstrap index
// sets (RandomState(42) is re-created per region, evals.py:356), so for one B plan and one
// pass the regions' B walks share everything but the A ranks: the pair order, the window
// inclusion bits x (mask lookups + 64 x 64 transpose), the group-start flags, the included
// counts c1 and the B tie terms. Per window those are done once; per pair each region adds
// its own TB row gather, window low end and sums. The regions' TB tables (one A walk each)
// are resident together. Same exact integer sums as k_rankB EST 3 (the segment partials go
// to each region's workspace, unit j), so the scores are bit-identical to the per-region
// calls. Tie groups < 2^16 (the caller checks). The launch runs one 16-wave workgroup per
// CU, so the masks (8 B per stimulus) sit in LDS up to n = 20,352 (LDS = true); larger n
// read them from L2 (LDS = false: two 8-B plain loads per window lane, compiler-counted).
// ---------------------------------------------------------------------------------
struct GridB {
  const uint16_t* TB[4];     // each region's TB (EST: absolute doubled ranks mod 2^16)
  const uint32_t* posA[4];   // B position -> A position, per region
  uint32_t* seg_tot[4];      // unit (j, region) segment partials (k_tail_part's inputs)
  uint64_t* seg_part[4];
};
#ifndef VR_GRID_NB
#define VR_GRID_NB 4  // pairs per gather batch (x R regions loads in flight, two batches)
#endif
#ifndef VR_GRID_NT
#define VR_GRID_NT 1  // TB rows read with nontemporal loads (each is read once per pass and region)
#endif
#ifndef VR_GRID_MASKMUL
#define VR_GRID_MASKMUL 0  // 1: mask the shared multipliers instead of each region's rank (A/B)
#endif
#ifndef VR_GRID_MINW
#define VR_GRID_MINW 4  // waves per SIMD the grid walk is compiled for (4: 128 VGPRs)
#endif
template <int R, bool LDS>
__global__ __launch_bounds__(ENG_THREADS, VR_GRID_MINW) void k_rankB_grid(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gflag, const uint64_t* __restrict__ gmask,
    int64_t n, GridB g, uint32_t nseg, const uint2* __restrict__ ftab, const uint32_t* __restrict__ segpos,
    uint32_t* __restrict__ queue) {
  constexpr int NB = VR_GRID_NB;
  static_assert(64 % NB == 0, "batch");
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const uint32_t Lu = wave_uniform(sload(&ftab->x)), Ru = wave_uniform(sload(&ftab->y));
  const int lane = threadIdx.x & 63;
  const uint32_t lane_off = (uint32_t)lane;
  for (;;) {
    const uint32_t sidx = next_segment(queue);
    if (sidx >= nseg) break;
    const uint32_t P0 = segpos[sidx], P1 = segpos[sidx + 1];
    u128 acc[R];
    uint64_t St[R], S[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0, St[r] = 0, S[r] = 0;
    uint64_t tie = 0;
    u128 tie_unused = 0;
    uint32_t cw = 0, cgs = 0;
    if (P0 < P1) {
      auto close = [&](uint32_t ce) {
        const uint32_t y = cgs + ce + 1u;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          acc[r] += (u128)S[r] * y;
          St[r] += S[r];
          S[r] = 0;
        }
        tie_add<false>(tie, tie_unused, ce - cgs);
        cgs = ce;
      };
      for (uint32_t w0 = P0 & ~63u; w0 < P1; w0 += 64) {
        const uint32_t pos = w0 + (uint32_t)lane;
        const bool valid = pos >= P0 && pos < P1;
        const uint32_t cd = valid ? codes[pos] : 0u;
        uint32_t pa[R], la[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          pa[r] = valid ? g.posA[r][pos] : 0u;
          la[r] = Lu + __umulhi(pa[r] << 1, Ru);
        }
        const uint64_t x = window_bits<VR_XPOSE_B>(m, cd, w0, P0, P1, lane, true);
        const uint64_t F =
            restrict_flags(((uint64_t)sload(gflag + (w0 >> 5) + 1) << 32) | sload(gflag + (w0 >> 5)), w0, P0, P1);
        // batch h's TB entries, t[r][q] = region r's row of pair h NB + q, lane's subset
        auto issue = [&](int h, uint32_t (&t)[R][NB]) {
#pragma unroll
          for (int q = 0; q < NB; ++q)
#pragma unroll
            for (int r = 0; r < R; ++r)
#if VR_GRID_NT
              t[r][q] = __builtin_nontemporal_load(g.TB[r] + (size_t)readlane_u32(pa[r], h * NB + q) * LANES + lane_off);
#else
              t[r][q] = g.TB[r][(size_t)readlane_u32(pa[r], h * NB + q) * LANES + lane_off];
#endif
        };
        uint32_t tb[2][R][NB];
        if (F == ~0ull) {  // every position starts a group (k_rankB's per-window form explains)
          close(cw);
          uint64_t a64[R];
#pragma unroll
          for (int r = 0; r < R; ++r) a64[r] = 0;
          uint32_t c1 = cw + 1u;
          issue(0, tb[0]);
#pragma unroll
          for (int h = 0; h < 64 / NB; ++h) {
            if (h + 1 < 64 / NB) issue(h + 1, tb[(h + 1) & 1]);
#pragma unroll
            for (int q = 0; q < NB; ++q) {
              const uint32_t j = h * NB + q;
              const uint32_t mk = (uint32_t)((int32_t)((uint32_t)(x >> (j & 32u)) << (31u - (j & 31u))) >> 31);
#if VR_GRID_MASKMUL
              // the inclusion mask on the shared multipliers: c1 & mk and mk & 1 (two 64-bit
              // multiply-adds per region, no per-region mask)
              const uint32_t c1m = c1 & mk, bit = mk & 1u;
#endif
#pragma unroll
              for (int r = 0; r < R; ++r) {
                const uint32_t y = est_recover(tb[h & 1][r][q], readlane_u32(la[r], j));
                if (j < 63) {
#if VR_GRID_MASKMUL
                  a64[r] += (uint64_t)y * c1m;
                  St[r] += (uint64_t)y * bit;
#else
                  const uint32_t yb = y & mk;
                  a64[r] += (uint64_t)yb * c1;
                  St[r] += yb;
#endif
                } else {
                  S[r] = y & mk;
                }
              }
              if (j < 63)
                c1 -= mk;
              else
                cgs = c1 - 1u;
            }
          }
#pragma unroll
          for (int r = 0; r < R; ++r) acc[r] += (u128)a64[r] * 2u;
        } else {
          issue(0, tb[0]);
#pragma unroll
          for (int h = 0; h < 64 / NB; ++h) {
            if (h + 1 < 64 / NB) issue(h + 1, tb[(h + 1) & 1]);
#pragma unroll
            for (int q = 0; q < NB; ++q) {
              const uint32_t j = h * NB + q;
              if ((F >> j) & 1ull) close(cw + popc64(x & lowmask(j)));
              const bool in = (x >> j) & 1ull;
#pragma unroll
              for (int r = 0; r < R; ++r) {
                const uint32_t y = est_recover(tb[h & 1][r][q], readlane_u32(la[r], j));
                S[r] += in ? (uint64_t)y : 0ull;
              }
            }
          }
        }
        cw += popc64(x);
      }
      if ((P1 & 63u) == 0) close(cw);  // a 64-aligned segment end is in no window
    }
    const size_t o = (size_t)sidx * LANES + lane, fs = (size_t)nseg * LANES;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      g.seg_tot[r][o] = cw;
      g.seg_part[r][PB_ACCL * fs + o] = (uint64_t)acc[r];
      g.seg_part[r][PB_ACCH * fs + o] = (uint64_t)(acc[r] >> 64);
      g.seg_part[r][PB_ST * fs + o] = St[r];
      g.seg_part[r][PB_TIEL * fs + o] = tie;
      g.seg_part[r][PB_TIEH * fs + o] = 0;
    }
  }
}

// ---------------------------------------------------------------------------------
// Exact grid B walk: k_rankB_grid's region fusion in the exact chunk-base form (every pass
// with VISREPS_ENGINE_EST=0, and the regions of a grid call whose estimate fails its up-front
// check). Per pair and region yA = 2 baseA[chunk] + TB[posA] (u16 chunk-relative ranks:
// narrow A plans), as in k_rankB's exact form; the A chunk of a position is found here from
// the region's chunk starts (cst: the last c <= pos / L whose start is <= pos, k_join's rule),
// so the shared joins' A positions serve the exact form too (no per-unit chunk joins). Same
// integer sums as the per-region exact walks: scores bit-identical to them.
// ---------------------------------------------------------------------------------
struct GridX {
  const uint16_t* TB[4];     // each region's chunk-relative doubled ranks (u16)
  const uint32_t* posA[4];   // B position -> A position, per region
  const uint32_t* base[4];   // [nch][64] absolute included count at each A chunk start
  const uint32_t* cst[4];    // [nch] A chunk start positions
  uint32_t* seg_tot[4];
  uint64_t* seg_part[4];
};
#ifndef VR_GRIDX_NB
#define VR_GRIDX_NB 2  // pairs per gather batch (x R regions x 2 loads in flight, two batches);
#endif                 // 1 at R = 4, whose 2-pair batches do not fit 128 VGPRs
// chunk of A position pa: q = pa / L from the reciprocal Lm = floor(2^32 / L) (q is exact or
// one low), then back over chunk starts above pa (group-aligned chunks start at or after c L)
__device__ inline uint32_t a_chunk(uint32_t pa, const uint32_t* __restrict__ cst, uint32_t L, uint32_t Lm,
                                   uint32_t nch) {
  uint32_t q = __umulhi(pa, Lm);
  if ((q + 1u) * L <= pa) ++q;
  q = min(q, nch - 1u);
  while (q > 0u && cst[q] > pa) --q;
  return q;
}
template <int R, bool LDS>
__global__ __launch_bounds__(ENG_THREADS, VR_GRID_MINW) void k_rankB_gridx(
    const uint32_t* __restrict__ codes, const uint32_t* __restrict__ gflag, const uint64_t* __restrict__ gmask,
    int64_t n, GridX g, uint32_t nseg, uint32_t L, uint32_t Lm, uint32_t nch, const uint32_t* __restrict__ segpos,
    uint32_t* __restrict__ queue) {
  constexpr int NB = R >= 4 ? 1 : VR_GRIDX_NB;
  static_assert(64 % NB == 0, "batch");
  extern __shared__ uint64_t smask[];
  const uint64_t* m = stage_masks<LDS>(gmask, n, smask);
  const int lane = threadIdx.x & 63;
  const uint32_t lane_off = (uint32_t)lane;
  for (;;) {
    const uint32_t sidx = next_segment(queue);
    if (sidx >= nseg) break;
    const uint32_t P0 = segpos[sidx], P1 = segpos[sidx + 1];
    u128 acc[R];
    uint64_t St[R], S[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0, St[r] = 0, S[r] = 0;
    uint64_t tie = 0;
    u128 tie_unused = 0;
    uint32_t cw = 0, cgs = 0;
    if (P0 < P1) {
      auto close = [&](uint32_t ce) {
        const uint32_t y = cgs + ce + 1u;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          acc[r] += (u128)S[r] * y;
          St[r] += S[r];
          S[r] = 0;
        }
        tie_add<false>(tie, tie_unused, ce - cgs);
        cgs = ce;
      };
      for (uint32_t w0 = P0 & ~63u; w0 < P1; w0 += 64) {
        const uint32_t pos = w0 + (uint32_t)lane;
        const bool valid = pos >= P0 && pos < P1;
        const uint32_t cd = valid ? codes[pos] : 0u;
        uint32_t pa[R], ca[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          pa[r] = valid ? g.posA[r][pos] : 0u;
          ca[r] = a_chunk(pa[r], g.cst[r], L, Lm, nch);
        }
        const uint64_t x = window_bits<VR_XPOSE_B>(m, cd, w0, P0, P1, lane, true);
        const uint64_t F =
            restrict_flags(((uint64_t)sload(gflag + (w0 >> 5) + 1) << 32) | sload(gflag + (w0 >> 5)), w0, P0, P1);
        // batch h's rows, t / b[r][q] = region r's TB entry / chunk base of pair h NB + q
        auto issue = [&](int h, uint32_t (&t)[R][NB], uint32_t (&b)[R][NB]) {
#pragma unroll
          for (int q = 0; q < NB; ++q)
#pragma unroll
            for (int r = 0; r < R; ++r) {
              t[r][q] = __builtin_nontemporal_load(g.TB[r] + (size_t)readlane_u32(pa[r], h * NB + q) * LANES + lane_off);
              b[r][q] = g.base[r][(size_t)readlane_u32(ca[r], h * NB + q) * LANES + lane_off];
            }
        };
        uint32_t tb[2][R][NB], bb[2][R][NB];
        if (F == ~0ull) {  // every position starts a group (k_rankB's per-window form explains)
          close(cw);
          uint64_t a64[R];
#pragma unroll
          for (int r = 0; r < R; ++r) a64[r] = 0;
          uint32_t c1 = cw + 1u;
          issue(0, tb[0], bb[0]);
#pragma unroll
          for (int h = 0; h < 64 / NB; ++h) {
            if (h + 1 < 64 / NB) issue(h + 1, tb[(h + 1) & 1], bb[(h + 1) & 1]);
#pragma unroll
            for (int q = 0; q < NB; ++q) {
              const uint32_t j = h * NB + q;
              const uint32_t mk = (uint32_t)((int32_t)((uint32_t)(x >> (j & 32u)) << (31u - (j & 31u))) >> 31);
#pragma unroll
              for (int r = 0; r < R; ++r) {
                const uint32_t y = 2u * bb[h & 1][r][q] + tb[h & 1][r][q];
                if (j < 63) {
                  const uint32_t yb = y & mk;
                  a64[r] += (uint64_t)yb * c1;
                  St[r] += yb;
                } else {
                  S[r] = y & mk;
                }
              }
              if (j < 63)
                c1 -= mk;
              else
                cgs = c1 - 1u;
            }
          }
#pragma unroll
          for (int r = 0; r < R; ++r) acc[r] += (u128)a64[r] * 2u;
        } else {
          issue(0, tb[0], bb[0]);
#pragma unroll
          for (int h = 0; h < 64 / NB; ++h) {
            if (h + 1 < 64 / NB) issue(h + 1, tb[(h + 1) & 1], bb[(h + 1) & 1]);
#pragma unroll
            for (int q = 0; q < NB; ++q) {
              const uint32_t j = h * NB + q;
              if ((F >> j) & 1ull) close(cw + popc64(x & lowmask(j)));
              const bool in = (x >> j) & 1ull;
#pragma unroll
              for (int r = 0; r < R; ++r) {
                const uint32_t y = 2u * bb[h & 1][r][q] + tb[h & 1][r][q];
                S[r] += in ? (uint64_t)y : 0ull;
              }
            }
          }
        }
        cw += popc64(x);
      }
      if ((P1 & 63u) == 0) close(cw);  // a 64-aligned segment end is in no window
    }
    const size_t o = (size_t)sidx * LANES + lane, fs = (size_t)nseg * LANES;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      g.seg_tot[r][o] = cw;
      g.seg_part[r][PB_ACCL * fs + o] = (uint64_t)acc[r];
      g.seg_part[r][PB_ACCH * fs + o] = (uint64_t)(acc[r] >> 64);
      g.seg_part[r][PB_ST * fs + o] = St[r];
      g.seg_part[r][PB_TIEL * fs + o] = tie;
      g.seg_part[r][PB_TIEH * fs + o] = 0;
    }
  }
}

// chunk start positions of an A plan: cst[c] = gstart[chunk_g[c]]
__global__ void k_chunk_starts(const uint32_t* __restrict__ gstart, const uint32_t* __restrict__ chunk_g,
                               uint32_t nch, uint32_t* __restrict__ cst) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < nch) cst[c] = gstart[chunk_g[c]];
}

// ---------------------------------------------------------------------------------
// final combination
// ---------------------------------------------------------------------------------
__device__ inline double i128_to_f64(i128 x) {
  const bool neg = x < 0;
  u128 u = neg ? (u128)(-x) : (u128)x;
  double d = (double)(uint64_t)(u >> 64) * 18446744073709551616.0 + (double)(uint64_t)u;
  return neg ? -d : d;
}

__device__ inline u128 ld128(const uint64_t* p, size_t lo, size_t hi) {
  return ((u128)p[hi] << 64) | p[lo];
}

// Tail of a pass for units u = blockIdx.y (all B walks of the pass first, one tail for all
// of them). Per block of SCAN_SEGS B segments, in segment order:
//   tA = sum (k^3 - k) over A groups,  tB = same over B groups,  T = included pairs,
//   S = sum St,  X = sum_seg (acc + 2 P St)  with P the included pairs of the block's
//   segments before this one
// so that ab = sum yA yB = sum_blk (X_blk + 2 P_blk S_blk) with P_blk the pairs of the
// blocks before (k_tail_top): no separate scan of the segment counts.
constexpr int FP_N = 8;  // fpart fields: tA lo/hi, tB lo/hi, X lo/hi, T, S
__global__ __launch_bounds__(1024) void k_tail_part(
    const uint64_t* __restrict__ segA_part, const uint64_t* __restrict__ segB_part0,
    const uint32_t* __restrict__ segB_tot0, uint32_t nseg, size_t ustride, uint64_t* __restrict__ fpart0,
    uint32_t ratioA) {
  __shared__ u128 red[3][16][LANES];
  __shared__ uint64_t red64[2][16][LANES];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const size_t fs = (size_t)nseg * LANES, fsA = fs * ratioA;
  const uint64_t* segB_part = segB_part0 + blockIdx.y * ustride * PB_N;
  const uint32_t* segB_tot = segB_tot0 + blockIdx.y * ustride;
  constexpr int PER = SCAN_SEGS / 16;
  const uint32_t s0 = blockIdx.x * SCAN_SEGS + v * PER;
  u128 tA = 0, tB = 0, X = 0;
  uint64_t T = 0, S = 0;
  for (int i = 0; i < PER; ++i) {
    if (s0 + i >= nseg) break;
    const size_t o = (size_t)(s0 + i) * LANES + lane;
    const uint64_t st = segB_part[PB_ST * fs + o];
    for (uint32_t r = 0; r < ratioA; ++r) {  // the A segments inside B segment s0 + i (any order: exact sums)
      const size_t oa = ((size_t)(s0 + i) * ratioA + r) * LANES + lane;
      tA += ld128(segA_part, PA_TIEL * fsA + oa, PA_TIEH * fsA + oa);
    }
    tB += ld128(segB_part, PB_TIEL * fs + o, PB_TIEH * fs + o);
    X += ld128(segB_part, PB_ACCL * fs + o, PB_ACCH * fs + o) + 2 * (u128)T * st;
    S += st;
    T += segB_tot[o];
  }
  red[0][v][lane] = tA;
  red[1][v][lane] = tB;
  red[2][v][lane] = X;
  red64[0][v][lane] = T;
  red64[1][v][lane] = S;
  __syncthreads();
  if (v != 0) return;
  for (int u = 1; u < 16; ++u) {  // waves in segment order
    tA += red[0][u][lane];
    tB += red[1][u][lane];
    X += red[2][u][lane] + 2 * (u128)T * red64[1][u][lane];
    S += red64[1][u][lane];
    T += red64[0][u][lane];
  }
  uint64_t* f = fpart0 + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * FP_N * LANES + lane;
  f[0 * LANES] = (uint64_t)tA;
  f[1 * LANES] = (uint64_t)(tA >> 64);
  f[2 * LANES] = (uint64_t)tB;
  f[3 * LANES] = (uint64_t)(tB >> 64);
  f[4 * LANES] = (uint64_t)X;
  f[5 * LANES] = (uint64_t)(X >> 64);
  f[6 * LANES] = T;
  f[7 * LANES] = S;
}

// rho from exact integers, one block per unit. With M' included pairs and doubled midranks y:
//   sum y = M'(M'+1),  mu = M'(M'+1)^2,
//   sum k y^2 = 4 M'(M'+1)(2M'+1)/6 - sum_g (k^3 - k)/3   (untied squares minus tie spread)
// nan_units bit u: unit u's B plan has a NaN (so does every unit when a_nan).
// Invariants (free: both sums are already here): the B walk's included-pair count P equals
// the A walk's M', and the sum of the yA it gathered equals sum y = M'(M'+1). A B-side
// recovery error (a wrong 2^16 window, a corrupted TB row) moves S and sets *viol, so the
// pass is re-run in the exact form (EST) or the call fails (exact form) -- never a silent
// wrong score.
// EST 4 pass (est4_shift): lane 0's shifted-away sums of one unit, sum_p d(posA(p)) and
// sum_p d(posA(p)) yB(p) over its B positions p, yB(p) = gs + ge + 1 for p's B tie group
// [gs, ge) (the full set's doubled midrank). Each wave walks a contiguous range of 64-position
// windows in order: lane j holds position w + j, the window's group-start bits F (two scalar
// loads) give every lane its group bounds inside the window, and the group open at a window's
// end is carried into the next (its members' d summed per lane until it ends). Only the
// range's first and last groups need a search, wave-uniform (a few flag words back or
// forward, else a binary search over the group starts). A fixed grid of CORR_BLK blocks,
// each writing its block's sums (sum d, then sum d yB as four 32-bit limb sums) to
// corr[field][block]; k_tail_top adds them up (exact integers: no order dependence).
__device__ inline uint32_t group_index(const uint32_t* __restrict__ gstart, uint32_t G, uint32_t p) {
  uint32_t lo = 0, hi = G;  // gstart[lo] <= p < gstart[hi] (gstart[G] = M)
  while (hi - lo > 1) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    if (sload(gstart + mid) <= p) lo = mid; else hi = mid;
  }
  return lo;
}
// the last group start < w (w a multiple of 64, > 0): wave-uniform
__device__ inline uint32_t start_before(const uint32_t* __restrict__ gflag, const uint32_t* __restrict__ gstart,
                                        uint32_t G, uint32_t w) {
  for (uint32_t k = w >> 5, i = 0; k > 0 && i < 8; ++i) {
    const uint32_t v = sload(gflag + (--k));
    if (v) return (k << 5) + 31u - (uint32_t)__clz(v);
  }
  return sload(gstart + group_index(gstart, G, w - 1u));
}
// the first group start >= e (a multiple of 64), or M: wave-uniform
__device__ inline uint32_t start_from(const uint32_t* __restrict__ gflag, const uint32_t* __restrict__ gstart,
                                      uint32_t G, int64_t M, uint32_t e) {
  if ((int64_t)e >= M) return (uint32_t)M;
  const uint32_t kend = (uint32_t)((M + 31) >> 5);
  for (uint32_t k = e >> 5, i = 0; k < kend && i < 8; ++k, ++i) {
    const uint32_t v = sload(gflag + k);
    if (v) {
      const uint32_t s = (k << 5) + (uint32_t)__ffs(v) - 1u;
      return (int64_t)s >= M ? (uint32_t)M : s;  // (bits past the last position are padding)
    }
  }
  const uint32_t gi = group_index(gstart, G, e);  // the group holding e (no start in 8 words)
  return sload(gstart + gi + 1u);
}
constexpr int CORR_UNROLL = 4;  // windows per round, their loads issued together
__global__ __launch_bounds__(256) void k_full_corr(const uint32_t* __restrict__ posA_byB,
                                                   const uint32_t* __restrict__ gflag,
                                                   const uint32_t* __restrict__ gstart, uint32_t G, int64_t M,
                                                   uint32_t Ru, uint64_t* __restrict__ corr) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t nwin = (uint64_t)(M + 63) / 64u;
  const uint64_t waves = (uint64_t)gridDim.x * 4u;
  const uint64_t wid = wave_uniform(blockIdx.x * 4u + (uint32_t)wv);
  // this wave's windows: a contiguous range, walked in order, so the group open at a window's
  // end is carried into the next one (no search per window)
  const uint64_t wb = nwin * wid / waves, we = nwin * (wid + 1) / waves;
  const uint64_t below = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);  // positions <= lane
  uint64_t c1 = 0;
  u128 c2 = 0;
  uint64_t dopen = 0;  // sum of d over this lane's positions in the group open at the window end
  uint32_t gsc = 0;    // the last group start before the current window (wave-uniform)
  if (wb < we && wb > 0 && !(sload(gflag + 2 * wb) & 1u)) gsc = start_before(gflag, gstart, G, (uint32_t)(wb * 64u));
  for (uint64_t w0 = wb; w0 < we; w0 += CORR_UNROLL) {
    uint32_t pa[CORR_UNROLL];
    uint64_t Fs[CORR_UNROLL];
#pragma unroll
    for (int i = 0; i < CORR_UNROLL; ++i) {
      const uint64_t win = w0 + i < we ? w0 + i : w0;
      const int64_t p = (int64_t)win * 64 + lane;
      pa[i] = p < M ? posA_byB[p] : 0u;
      Fs[i] = ((uint64_t)sload(gflag + 2 * win + 1) << 32) | sload(gflag + 2 * win);
    }
#pragma unroll
    for (int i = 0; i < CORR_UNROLL; ++i) {
      if (w0 + i >= we) break;
      const uint32_t w = (uint32_t)((w0 + i) * 64u);
      const int64_t left = M - (int64_t)w;
      uint64_t F = Fs[i];
      if (left < 64) F |= ~0ull << left;  // the triangle's end starts a (padding) group
      if (F) {  // the carried group (if any) ends at the window's first start
        const uint32_t ge0 = w + (uint32_t)__builtin_ctzll(F);
        c2 += (u128)dopen * ge0;
        dopen = 0;
      }
      const bool valid = (int64_t)lane < left;
      const uint32_t d = valid ? est4_shift(Ru, pa[i]) : 0u;
      const uint64_t lo = F & below, hi = F & ~below;
      const uint32_t gs = lo ? w + 63u - (uint32_t)__builtin_clzll(lo) : gsc;
      c1 += d;
      c2 += (u128)((uint64_t)d * (gs + 1u));  // the gs + 1 part of yB = gs + ge + 1
      if (hi)
        c2 += (u128)((uint64_t)d * (w + (uint32_t)__builtin_ctzll(hi)));  // ge inside the window
      else
        dopen += d;  // ge lies past the window: added when the group ends
      if (F) gsc = w + 63u - (uint32_t)__builtin_clzll(F);
    }
  }
  if (wb < we) {  // the group open at the range end ends at the next start (or M)
    const uint64_t any = __ballot(dopen != 0);
    if (any) c2 += (u128)dopen * start_from(gflag, gstart, G, M, (uint32_t)(we * 64u));
  }
  __shared__ uint64_t red[CORR_F][4];
  const uint64_t v[CORR_F] = {c1, (uint64_t)(uint32_t)c2, (uint64_t)(uint32_t)(c2 >> 32),
                              (uint64_t)(uint32_t)(c2 >> 64), (uint64_t)(c2 >> 96)};
#pragma unroll
  for (int f = 0; f < CORR_F; ++f) {
    uint64_t s = v[f];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += shfl_xor64(s, m);
    if (lane == 0) red[f][wv] = s;
  }
  __syncthreads();
  if (threadIdx.x < CORR_F)
    corr[(size_t)threadIdx.x * CORR_BLK + blockIdx.x] =
        red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
}

// corr (EST 4 pass, else null): per unit [CORR_F][CORR_BLK] k_full_corr block sums, added to lane 0's
__global__ void k_tail_top(const uint64_t* __restrict__ fpart0, uint32_t nblk,
                           const uint32_t* __restrict__ totA, int a_nan, uint64_t nan_units, int nl,
                           double* __restrict__ scores0, int64_t score_ld, uint32_t* __restrict__ viol,
                           const uint64_t* __restrict__ corr) {
  const int lane = threadIdx.x;
  const uint32_t u = blockIdx.x;
  const uint64_t* fpart = fpart0 + (size_t)u * nblk * FP_N * LANES;
  u128 tA = 0, tB = 0, ab = 0;
  uint64_t P = 0, Ssum = 0;
  // unrolled so the loads of several partial blocks are in flight at once (the loop is
  // otherwise one L2 round trip per block)
#pragma unroll 8
  for (uint32_t b = 0; b < nblk; ++b) {
    const uint64_t* f = fpart + (size_t)b * FP_N * LANES + lane;
    tA += ((u128)f[1 * LANES] << 64) | f[0 * LANES];
    tB += ((u128)f[3 * LANES] << 64) | f[2 * LANES];
    ab += (((u128)f[5 * LANES] << 64) | f[4 * LANES]) + 2 * (u128)P * f[7 * LANES];
    P += f[6 * LANES];
    Ssum += f[7 * LANES];
  }
  if (corr != nullptr) {  // lane 0: the full set's shifted ranks (est4_shift)
    const uint64_t* c = corr + (size_t)u * CORR_N;
    uint64_t s[CORR_F] = {0, 0, 0, 0, 0};
    for (int b = lane; b < CORR_BLK; b += LANES)
#pragma unroll
      for (int f = 0; f < CORR_F; ++f) s[f] += c[(size_t)f * CORR_BLK + b];
#pragma unroll
    for (int f = 0; f < CORR_F; ++f)
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) s[f] += shfl_xor64(s[f], m);
    if (lane == 0) {
      Ssum += s[0];
      ab += (u128)s[1] + ((u128)s[2] << 32) + ((u128)s[3] << 64) + ((u128)s[4] << 96);
    }
  }
  const bool forced_nan = a_nan || ((nan_units >> u) & 1ull);
  const bool broken = lane < nl && !forced_nan &&
                      (P != (uint64_t)totA[lane] || Ssum != (uint64_t)totA[lane] * ((uint64_t)totA[lane] + 1u));
  // bit 1 (the A walk's window checks set bit 0); benign race: every writer stores old | 2
  if (VR_TAIL_CHECK && __ballot(broken) != 0 && lane == 0) *viol |= 2u;
  if (lane >= nl) return;
  const u128 Mp = totA[lane];
  const u128 mu = Mp * (Mp + 1) * (Mp + 1);
  const u128 sq = 4 * (Mp * (Mp + 1) * (2 * Mp + 1) / 6);
  const i128 num = (i128)ab - (i128)mu;
  const i128 va = (i128)(sq - tA / 3) - (i128)mu;
  const i128 vb = (i128)(sq - tB / 3) - (i128)mu;
  double r;
  if (forced_nan || Mp < 2 || va <= 0 || vb <= 0) {
    r = __builtin_nan("");
  } else {
    r = i128_to_f64(num) / sqrt(i128_to_f64(va) * i128_to_f64(vb));
    r = r > 1.0 ? 1.0 : (r < -1.0 ? -1.0 : r);
  }
  scores0[(size_t)u * score_ld + lane] = r;
}

__global__ void k_fill_nan(double* out, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = __builtin_nan("");
}

// ---------------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------------
template <typename K>
static int allow_big_lds(K kernel) {
  VR_CHECK_HIP(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024));
  return VR_OK;
}

// A side of a pass (shared by every B plan of the call), exact form: TB rows in A order,
// chunk bases baseA, A segment tie sums and the included-pair totals totA.
template <bool LDS, bool FULL, typename TBT, bool BTA>
static int pass_a(const PlanView& A, int64_t n, const EngineWs& E, int lw, const EngineCfg& cfg,
                  hipStream_t st) {
  VR_ONCE(VR_TRY(allow_big_lds(k_rankA<LDS, FULL, TBT, BTA, false>)));
  const int64_t M = pairs_of(n);
  const uint32_t nch = plan_nchunks(M);
  const uint32_t nseg = (uint32_t)cfg.nwaves;
  {
    KtScope kt(KT_RANKA, (double)M, st);
    k_rankA<LDS, FULL, TBT, BTA, false><<<cfg.grid, ENG_THREADS, cfg.lds, st>>>(
        A.codes, A.gstart, A.chunk_g, A.gflag, nch, E.masks, n, static_cast<TBT*>(E.TB), lw, E.lpA,
        E.segA_tot, E.segA_part, nseg, EstA{}, nullptr, nullptr);
    VR_CHECK_LAUNCH();
  }
  VR_TRY(lane_scan(E.segA_tot, nseg, E.bsum, E.segA_pre, E.totA, st));
  const size_t nb = ((size_t)nch * LANES + 255) / 256;
  k_add_base<<<(unsigned)nb, 256, 0, st>>>(E.lpA, E.segA_pre, nch, nseg, E.baseA);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// A side of a pass, EST form: count pre-pass -> segment bases and the interval table ->
// absolute u16 ranks in A order (flagging *viol when one is not recoverable). The count
// pre-pass reads the masks from LDS when they fit (CL), the rank walk from L2.
template <int EM, bool CL, bool FULL, bool BTA>
static int pass_a_est(const PlanView& A, int64_t n, const EngineWs& E, int lw, int nl, const EngineCfg& cfg,
                      uint2 e3, uint2 tri, uint32_t* viol, hipStream_t st) {
  VR_ONCE(VR_TRY(allow_big_lds(k_countA<CL, FULL>)); VR_TRY(allow_big_lds(k_rankA<CL, FULL, uint16_t, BTA, EM>)));
  const int64_t M = pairs_of(n);
  const uint32_t nch = plan_nchunks(M);
  const uint32_t nseg = cfg.est_nsegA;
  const int bits = cfg.est_b;
  const uint32_t nc = cfg.est_rows;
  {
    KtScope kt(KT_COUNTA, (double)M, st);
    k_countA<CL, FULL><<<cfg.est_grid, ENG_THREADS, CL ? (size_t)n * sizeof(uint64_t) : 0, st>>>(
        A.codes, A.gstart, A.chunk_g, nch, E.masks, n, lw, bits, E.c0rel, E.c0seg, E.segA_tot, nseg, E.segposA);
    VR_CHECK_LAUNCH();
  }
  VR_TRY(lane_scan(E.segA_tot, nseg, E.bsum, E.segA_pre, E.totA, st));
  if constexpr (EM >= 3)
    k_c0_u<<<1, 1, 0, st>>>(e3.x, e3.y, tri.x, tri.y, E.ftab);
  else if constexpr (EM == 2)
    k_c0_lin<<<1, LANES, 0, st>>>(E.totA, M, E.ftab);
  else
    k_c0<<<nc, LANES, 0, st>>>(E.c0rel, E.c0seg, E.segA_pre, E.totA, nc, bits, M, E.ftab);
  VR_CHECK_LAUNCH();
  const EstA est{E.segA_pre, E.ftab, nc, bits, viol, nl};
  {
    KtScope kt(KT_RANKA, (double)M, st);
    k_rankA<CL, FULL, uint16_t, BTA, EM><<<cfg.est_grid, ENG_THREADS, cfg.tab, st>>>(
        A.codes, A.gstart, A.chunk_g, A.gflag, nch, E.masks, n, static_cast<uint16_t*>(E.TB), lw, E.lpA,
        E.segA_tot, E.segA_part, nseg, est, E.segposA, E.queue + QS_RANKA);
    VR_CHECK_LAUNCH();
  }
  return VR_OK;
}

// EST 3 up-front check of a call's first pass (masks already built): the count pre-pass at
// boundaries every 2^b positions (<= EST_NC of them), its scan, k_est_predict. bad <- the
// wave-uniform estimate cannot hold these A ranks (strongly structured RDMs: per-stimulus
// effects move a subset's count hundreds of thousands of pairs off the line), so the call
// goes to the exact form before spending an EST pass and its joins on a flag.
template <bool CL, bool FULL>
static int est_predict(const PlanView& A, int64_t n, const EngineWs& E, int lw, int nl, bool full0,
                       const EngineCfg& cfg, uint2 e3, hipStream_t st, bool& bad) {
  VR_ONCE(VR_TRY(allow_big_lds(k_countA<CL, FULL>)));
  const int64_t M = pairs_of(n);
  const uint32_t nch = plan_nchunks(M);
  const uint32_t nseg = cfg.est_nsegA;
  int b = 12;
  while (((M + ((int64_t)1 << b) - 1) >> b) > (int64_t)EST_NC) ++b;
  const uint32_t nc = est_intervals(M, b);
  {
    KtScope kt(KT_COUNTA, (double)M, st);
    k_countA<CL, FULL><<<cfg.est_grid, ENG_THREADS, CL ? (size_t)n * sizeof(uint64_t) : 0, st>>>(
        A.codes, A.gstart, A.chunk_g, nch, E.masks, n, lw, b, E.c0rel, E.c0seg, E.segA_tot, nseg, E.segposA);
    VR_CHECK_LAUNCH();
  }
  VR_TRY(lane_scan(E.segA_tot, nseg, E.bsum, E.segA_pre, E.totA, st));
  uint32_t* flag = E.viol;  // pass flags are cleared before the EST passes
  VR_CHECK_HIP(hipMemsetAsync(flag, 0, sizeof(uint32_t), st));
  k_est_predict<<<nc, LANES, 0, st>>>(E.c0rel, E.c0seg, E.segA_pre, b, e3.y, nl, full0 ? 1 : 0, flag);
  VR_CHECK_LAUNCH();
  uint32_t h = 0;
  VR_CHECK_HIP(hipMemcpyAsync(&h, flag, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VR_CHECK_HIP(hipStreamSynchronize(st));
  bad = h != 0;
  return VR_OK;
}

// B walk of a pass for one B plan (unit slot u of the segment partials), joined to A by
// posA_byB (and chunkA_byB: the A chunks in the exact form, EST 3's window low ends)
template <bool LDS, bool FULL, typename TBT, bool BTB, int EST>
static int walk_b(const PlanView& B, const uint32_t* posA_byB, const uint32_t* chunkA_byB, int64_t n,
                  const EngineWs& E, int lw, int64_t u, const EngineCfg& cfg, hipStream_t st, int kt_slot = -1) {
  VR_ONCE(VR_TRY(allow_big_lds(k_rankB<LDS, FULL, TBT, BTB, EST>)));
  const int64_t M = pairs_of(n);
  const uint32_t nch = plan_nchunks(M);
  const uint32_t nseg = EST ? cfg.est_nseg : (uint32_t)cfg.nwaves;
  const size_t us = (size_t)E.useg * (size_t)u;
  // EST: unit u's B segment starts and its queue counter (slots past QSLOTS are reused, each
  // cleared right before its launch)
  const uint32_t* segpos = EST ? E.segposB + E.segstride * (size_t)u : nullptr;
  uint32_t* q = nullptr;
  if constexpr (EST != 0) {
    q = E.queue + QS_RANKB + (size_t)u % (size_t)(QSLOTS - QS_RANKB);
    if (u >= QSLOTS - QS_RANKB) VR_CHECK_HIP(hipMemsetAsync(q, 0, sizeof(uint32_t), st));
  }
  {
    KtScope kt(kt_slot >= 0 ? kt_slot : EST == 6 ? KT_RANKB_FULL : EST ? KT_RANKB_EST : KT_RANKB_EXACT, (double)M, st);
    k_rankB<LDS, FULL, TBT, BTB, EST><<<EST ? cfg.est_grid : cfg.grid, ENG_THREADS, EST ? cfg.tab : cfg.lds, st>>>(
        B.codes, B.gstart, B.chunk_g, B.gflag, nch, E.masks, n, static_cast<const TBT*>(E.TB), lw,
        posA_byB, chunkA_byB, E.baseA, E.segB_tot + us, E.segB_part + us * PB_N, nseg, E.ftab,
        EST ? cfg.est_rows : 0, EST ? cfg.est_b : 0, segpos, q);
    VR_CHECK_LAUNCH();
  }
  return VR_OK;
}

// Tail of a pass for units [0, nb) (their B walks done): the nl scores of each, unit j's at
// scores + j * score_ld. nan_b[j]: unit j's B plan holds a NaN. *viol <- 1 when a unit's
// sums break the invariants (k_tail_top).
static int tail_units(const EngineWs& E, int64_t nb, uint32_t nseg, uint32_t ratioA, bool a_nan,
                      const std::vector<char>& nan_b, int nl, double* scores, int64_t score_ld, uint32_t* viol,
                      hipStream_t st, const uint64_t* corr = nullptr) {
  const uint32_t nsb = scan_blocks(nseg);
  for (int64_t u0 = 0; u0 < nb; u0 += 64) {  // 64 units per launch (the NaN bitmask)
    const int64_t cnt = std::min<int64_t>(64, nb - u0);
    uint64_t nan_units = 0;
    for (int64_t j = 0; j < cnt; ++j)
      if (nan_b[(size_t)(u0 + j)]) nan_units |= 1ull << j;
    const size_t us = (size_t)E.useg * (size_t)u0;
    k_tail_part<<<dim3(nsb, (unsigned)cnt), 1024, 0, st>>>(E.segA_part, E.segB_part + us * PB_N,
                                                            E.segB_tot + us, nseg, E.useg, E.fpart, ratioA);
    VR_CHECK_LAUNCH();
    k_tail_top<<<(unsigned)cnt, LANES, 0, st>>>(E.fpart, nsb, E.totA, a_nan ? 1 : 0, nan_units, nl,
                                                scores + u0 * score_ld, score_ld, viol,
                                                corr ? corr + (size_t)u0 * CORR_N : nullptr);
    VR_CHECK_LAUNCH();
  }
  return VR_OK;
}

// compile-time pass variant: masks in LDS, all 64 lanes, TB element type
template <bool L, bool F, typename T>
struct PassTag {
  static constexpr bool lds = L, full = F;
  using tbt = T;
};
template <class Fn>
static int with_pass_tag(bool lds, bool full, bool narrow, Fn&& fn) {
  if (lds) {
    if (full) return narrow ? fn(PassTag<true, true, uint16_t>{}) : fn(PassTag<true, true, uint32_t>{});
    return narrow ? fn(PassTag<true, false, uint16_t>{}) : fn(PassTag<true, false, uint32_t>{});
  }
  if (full) return narrow ? fn(PassTag<false, true, uint16_t>{}) : fn(PassTag<false, true, uint32_t>{});
  return narrow ? fn(PassTag<false, false, uint16_t>{}) : fn(PassTag<false, false, uint32_t>{});
}

// One A plan against nb B plans (one unit each). Per pass of 64 subsets the A side runs
// once and every B side reads its TB rows, so a plan shared by several units (a neural
// RDM against every model layer, evals.py:323-373 loops regions x layers) pays its rank
// walk once per pass. Spearman is symmetric in its two arguments and every sum is exact,
// so scores equal the per-unit calls bit for bit.
// Scores of B j: scores[j * score_ld + s] for the `total` subsets (full set first if
// full_first), 64 per pass. joins: nb pairs of M-element (posA_byB, chunkA_byB) arrays.
// Passes run in the EST form; the few it flags (and every pass, with VISREPS_ENGINE_EST=0)
// run in the exact chunk-base form, which needs the chunkA joins too.
// Test hook (vr_test_engine_inject(p), a test-only export; -1 = off, the default): after
// the A walk of EST pass p, add 1 to the TB entries of lanes 1..63 of one pair row -- a
// B-side recovery error the A walk's checks cannot see. The tail's invariants must flag
// the pass and the exact re-run must restore every score (tests/test_engine_est.py). No
// environment variable is read: the product path cannot be switched into it by accident.
static std::atomic<int64_t> g_test_inject{-1};

__global__ void k_inject_tb(uint16_t* __restrict__ TB, uint32_t row, int stride, int lanes) {
  const int lane = threadIdx.x;
  if (lane >= 1 && lane < lanes) TB[(size_t)row * stride + lane] += 1u;
}

// exact_passes (non-null): run only these passes, in the exact form (a grid call's flagged
// passes of one region; the rest of its scores stand)
static int run_engine_multi_impl(const PlanView& A, const PlanView* Bs, int64_t nb, int64_t n,
                                 const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                                 double* scores, int64_t score_ld, uint32_t* const* joins,
                                 const EngineWs& E, int lw, const EngineCfg& cfg, hipStream_t st,
                                 const std::vector<int64_t>* exact_passes = nullptr) {
  const int64_t M = pairs_of(n);
  uint32_t* const xbad = E.viol + EST_MAX_PASSES;  // exact-form passes' invariant flag
  const int64_t inject = g_test_inject.load(std::memory_order_relaxed);
  const int64_t total = n_sets + (full_first ? 1 : 0);
  if (total == 0 || nb == 0) return VR_OK;
  if (M == 0) {  // no pairs: every score is NaN (scipy on empty input)
    for (int64_t j = 0; j < nb; ++j) {
      k_fill_nan<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(scores + j * score_ld, total);
      VR_CHECK_LAUNCH();
    }
    return VR_OK;
  }
  // u16 chunk-relative ranks y~ <= 2 span + 1 need every chunk span (< L + largest tie
  // group of A) <= 32767; 64-bit tie sums need every group below 2^16
  std::vector<PlanHeader> h((size_t)nb + 1);
  VR_CHECK_HIP(hipMemcpyAsync(&h[0], A.hdr, sizeof(PlanHeader), hipMemcpyDeviceToHost, st));
  for (int64_t j = 0; j < nb; ++j)
    VR_CHECK_HIP(hipMemcpyAsync(&h[(size_t)j + 1], Bs[j].hdr, sizeof(PlanHeader),
                                hipMemcpyDeviceToHost, st));
  VR_CHECK_HIP(hipStreamSynchronize(st));
  const bool narrow = (uint64_t)PLAN_L + h[0].max_group <= 32767u;
  std::vector<char> nan_b((size_t)nb);
  for (int64_t j = 0; j < nb; ++j) nan_b[(size_t)j] = h[(size_t)j + 1].has_nan != 0;
  const bool bigA = h[0].max_group >= 65536u;
  const bool est = engine_est();
  // (a point-only call holds the full set alone: its window is the full set's, so lane 0's
  // EST 4 shift is at most 1 -- with k's window instead a group of > 3 tied pairs could
  // shift below 1 and flag the pass)
  const uint2 e3 = est3_params(n_sets > 0 ? k : n, M);
  int second = JOIN_NONE;  // what the joins' second arrays hold
  auto join = [&](int mode) -> int {
    for (int64_t j = 0; j < nb; ++j) {
      KtScope kt(KT_JOIN, (double)M, st);
      if (mode == JOIN_LO && second != JOIN_NONE) {  // the A positions are already there
        k_join_lo<<<(unsigned)((M + 255) / 256), 256, 0, st>>>(joins[2 * j], M, joins[2 * j + 1], e3.x, e3.y);
        VR_CHECK_LAUNCH();
        continue;
      }
      k_join<<<(unsigned)((M + 255) / 256), 256, 0, st>>>(Bs[j].codes, M, n, A.gstart, A.chunk_g,
                                                         plan_chunk_len(M), plan_nchunks(M), A.pos_map,
                                                         joins[2 * j], joins[2 * j + 1], mode, e3.x, e3.y);
      VR_CHECK_LAUNCH();
    }
    second = mode;
    return VR_OK;
  };
  // EST 5 / 6 (opt-in, VISREPS_ENGINE_TRI=1, in place of the EST 3 / 4 passes while
  // M <= 2^28): the A walk writes each pair's 128-B row at its triangle index, lane 63
  // holding the coarse A position, so the B walk finds the row from its own pair codes --
  // no per-unit join, no A-position / low-end streams (132 instead of 140 B per pair) -- at
  // the price of scattered (instead of sequential) row writes in the A walk and 63 subsets
  // per pass. Flagged passes re-run in the exact form, which joins on demand. Measured on
  // MI355X at configs[1] the scattered writes cost the A walk more (+0.70 ms
  // per pass) than the joins save, so the A-order TB stays the default.
  const bool tri = est && cfg.est_mode == 3 && lw == LANES && M <= ((int64_t)1 << 28) &&
                   env_int("VISREPS_ENGINE_TRI", 0) != 0;
  // EST 6 coarse position pos >> sh and EST 5 tag (low end + 2^15) >> g: both 16 bits
  uint32_t sh = 0, g = 0;
  while (((uint64_t)(M - 1) >> sh) >= 65536u) ++sh;
  {
    const uint64_t umax = 1u + (uint32_t)(((uint64_t)(2u * (uint32_t)(M - 1)) * e3.y) >> 32);
    while ((umax >> g) >= 65536u) ++g;
  }
  const uint2 trip = make_uint2(sh, g);
  // EST 3: the join precomputes the window low ends (JOIN_LO), the B walk streams them;
  // VISREPS_ENGINE_LO_JOIN=0 has the walk compute them from the A positions instead (4 B
  // fewer per pair and pass, but measured no faster: 1367 vs 1359 us per k_rankB launch,
  // profiles/r3_engine_lo_ab.log)
  const bool lo_join = !tri && cfg.est_mode == 3 && env_int("VISREPS_ENGINE_LO_JOIN", 0) != 0;
  // the EST 3 estimate checked against the first pass's A counts before any join or pass
  // (VISREPS_ENGINE_EST_PREDICT=0: skip the check; a failing estimate is then caught by the
  // first pass's flags, at the cost of that pass)
  // EST segment starts of the A plan and of every B plan (k_seg_table), once per call
  if (est) {
    const uint32_t ns = cfg.est_nseg, nsA = cfg.est_nsegA;
    k_seg_table<<<(nsA + 256) / 256, 256, 0, st>>>(A.gstart, A.hdr, M, nsA, E.segposA);
    VR_CHECK_LAUNCH();
    for (int64_t j = 0; j < nb; ++j) {
      k_seg_table<<<(ns + 256) / 256, 256, 0, st>>>(Bs[j].gstart, Bs[j].hdr, M, ns,
                                                    E.segposB + E.segstride * (size_t)j);
      VR_CHECK_LAUNCH();
    }
  }
  bool predicted_bad = false;
  // (only when some lane holds a bootstrap subset: the full-set lane is exact by
  // construction, and a point-only call -- phase 1's 56 -- would pay a host sync for nothing)
  if (est && cfg.est_mode == 3 && n_sets > 0 && !exact_passes && env_int("VISREPS_ENGINE_EST_PREDICT", 1) != 0) {
    const int64_t sub0 = tri ? LANES - 1 : lw;
    const int nl0 = (int)std::min<int64_t>(sub0, total);
    VR_TRY(build_pass_masks(idx, k, 0, nl0, full_first, E.masks, n, st));
    VR_TRY(with_pass_tag(cfg.est_lds, lw == LANES, true, [&](auto tag) -> int {
      using Tg = decltype(tag);
      return est_predict<Tg::lds, Tg::full>(A, n, E, lw, nl0, full_first != 0, cfg, e3, st, predicted_bad);
    }));
  }
  // (pre-joined units already hold their A positions: an EST call reading only those skips
  // the join; an exact-form one rewrites them with the same values beside the A chunks)
  if (!tri && !predicted_bad && !exact_passes && !(cfg.prejoined && est && !lo_join))
    VR_TRY(join(!est ? JOIN_CHUNK : (lo_join ? JOIN_LO : JOIN_NONE)));
  // the exact chunk-base form of subsets [set0, set0 + nl), nl <= lw
  auto exact_pass = [&](auto tag, int64_t set0, int nl) -> int {
    using Tg = decltype(tag);
    using TBT = typename Tg::tbt;
    VR_TRY(build_pass_masks(idx, k, set0, nl, full_first, E.masks, n, st));
    VR_TRY((bigA ? pass_a<Tg::lds, Tg::full, TBT, true>(A, n, E, lw, cfg, st)
                 : pass_a<Tg::lds, Tg::full, TBT, false>(A, n, E, lw, cfg, st)));
    for (int64_t j = 0; j < nb; ++j) {
      const uint32_t* pj = joins[2 * j];
      const uint32_t* cj = joins[2 * j + 1];
      VR_TRY((h[(size_t)j + 1].max_group >= 65536u
                  ? walk_b<Tg::lds, Tg::full, TBT, true, 0>(Bs[j], pj, cj, n, E, lw, j, cfg, st)
                  : walk_b<Tg::lds, Tg::full, TBT, false, 0>(Bs[j], pj, cj, n, E, lw, j, cfg, st)));
    }
    return tail_units(E, nb, (uint32_t)cfg.nwaves, 1u, h[0].has_nan != 0, nan_b, nl, scores + set0, score_ld, xbad,
                      st);
  };
  // subsets [s0, total) in exact passes of lw
  auto exact_from = [&](int64_t s0) -> int {
    if (second != JOIN_CHUNK) VR_TRY(join(JOIN_CHUNK));
    return with_pass_tag(cfg.use_lds, lw == LANES, narrow, [&](auto tag) -> int {
      for (int64_t set0 = s0; set0 < total; set0 += lw)
        VR_TRY(exact_pass(tag, set0, (int)std::min<int64_t>(lw, total - set0)));
      return VR_OK;
    });
  };
  if (exact_passes) {
    VR_TRY(join(JOIN_CHUNK));
    return with_pass_tag(cfg.use_lds, lw == LANES, narrow, [&](auto tag) -> int {
      for (int64_t p : *exact_passes) {
        const int64_t set0 = p * lw;
        if (set0 < total) VR_TRY(exact_pass(tag, set0, (int)std::min<int64_t>(lw, total - set0)));
      }
      return VR_OK;
    });
  }
  if (!est) return exact_from(0);
  if (predicted_bad) {
    g_est_predicted.fetch_add(1);
    // The lane-uniform EST 3 window cannot hold these counts (per-stimulus structure moves a
    // subset's included count further from the line than 2^14 pairs: it grows ~ n^1.5, so
    // large triangles cross it first). EST 1 follows each lane's own counts (an interpolated
    // table whose knots are the lane's counts at <= 144 boundaries, one LDS read per pair),
    // one gather per pair like EST 3; its flagged passes are re-run exact as ever. The exact
    // form from the start only with VISREPS_ENGINE_EST1_FALLBACK=0 or a point-only call.
    // (Only where the exact form reads its masks from L2 too, n > 20,352: below that the exact
    // walks keep the masks in LDS and EST 1, whose table takes that LDS, measured slower --
    // 79 vs 73 ms per unit on bench.structured_est_probe's RDM at N = 10k; at 20,500 EST 1
    // won, 215 vs 234 ms, profiles/r6_large_n_probe_v2.log.)
    if (lw == LANES && !cfg.use_lds && env_int("VISREPS_ENGINE_EST1_FALLBACK", 1) != 0) {
      EngineCfg c1 = engine_cfg(n, 1);
      c1.prejoined = cfg.prejoined;
      if (c1.nwaves == cfg.nwaves && c1.est_nsegA <= (uint32_t)cfg.nwaves * VR_SEGS_PER_WAVE) {
        g_est1_fallbacks.fetch_add(1);
        return run_engine_multi_impl(A, Bs, nb, n, idx, k, n_sets, full_first, scores, score_ld, joins, E, lw, c1,
                                     st);
      }
    }
    return exact_from(0);
  }
  const int64_t sub = tri ? LANES - 1 : lw;  // subsets per EST pass
  const int64_t npass = (total + sub - 1) / sub;
  const int64_t pfirst = 0;
  // The first EST pass runs alone: when the estimate cannot hold these A ranks (strongly
  // structured RDMs, giant tie groups) every pass is run in the exact form from there on.
  const int want = lo_join ? JOIN_LO : JOIN_NONE;  // what the EST passes read
  for (int64_t p0 = pfirst, p1 = pfirst; p0 < npass; p0 = p1) {
    p1 = std::min<int64_t>(npass, p0 == pfirst ? p0 + 1 : p0 + EST_MAX_PASSES);
    if (want != JOIN_NONE && second != want) VR_TRY(join(want));
    VR_CHECK_HIP(hipMemsetAsync(E.viol, 0, (size_t)(p1 - p0) * sizeof(uint32_t), st));
    VR_TRY(with_pass_tag(cfg.est_lds, lw == LANES, true, [&](auto tag) -> int {
      using Tg = decltype(tag);
      if constexpr (sizeof(typename Tg::tbt) == 2) {
        for (int64_t p = p0; p < p1; ++p) {
          const int64_t set0 = p * sub;
          const int nl = (int)std::min<int64_t>(sub, total - set0);
          VR_TRY(build_pass_masks(idx, k, set0, nl, full_first, E.masks, n, st));
          VR_CHECK_HIP(hipMemsetAsync(E.queue, 0, sizeof(uint32_t) * (size_t)std::min<int64_t>(QS_RANKB + nb, QSLOTS),
                                      st));  // this pass's work-queue counters
          uint32_t* viol = E.viol + (p - p0);
          auto run_pass = [&](auto em) -> int {
            constexpr int EM = decltype(em)::value;
            if constexpr (EM >= 5 && !Tg::full) {
              return VR_OK;  // (never taken: triangle-order passes are whole 64-lane rows)
            } else {
              VR_TRY((bigA ? pass_a_est<EM, Tg::lds, Tg::full, true>(A, n, E, lw, nl, cfg, e3, trip, viol, st)
                           : pass_a_est<EM, Tg::lds, Tg::full, false>(A, n, E, lw, nl, cfg, e3, trip, viol, st)));
              if (p == inject) {
                k_inject_tb<<<1, LANES, 0, st>>>(static_cast<uint16_t*>(E.TB), (uint32_t)(M / 2), lw,
                                                 (int)std::min<int64_t>(lw, sub));
                VR_CHECK_LAUNCH();
              }
              // EST 4: lane 0's ranks are stored shifted (est4_shift), so its B walks are the EST 3
              // kernel (timed on their own slot) and k_full_corr supplies lane 0's shift sums
              constexpr int EB = EM == 4 ? 3 : EM;
              const int kts = EM == 4 ? KT_RANKB_FULL : -1;
              for (int64_t j = 0; j < nb; ++j) {
                // EST 3/4: A positions and streamed low ends; EST 5/6: neither
                const uint32_t* pj = EM >= 5 ? nullptr : joins[2 * j];
                const uint32_t* lj = EM >= 3 && EM <= 4 && lo_join ? joins[2 * j + 1] : nullptr;
                VR_TRY((h[(size_t)j + 1].max_group >= 65536u
                            ? walk_b<Tg::lds, Tg::full, uint16_t, true, EB>(Bs[j], pj, lj, n, E, lw, j, cfg, st, kts)
                            : walk_b<Tg::lds, Tg::full, uint16_t, false, EB>(Bs[j], pj, lj, n, E, lw, j, cfg, st, kts)));
                if constexpr (EM == 4) {
                  KtScope kt(KT_FULL_CORR, (double)M, st);
                  k_full_corr<<<CORR_BLK, 256, 0, st>>>(pj, Bs[j].gflag, Bs[j].gstart, h[(size_t)j + 1].G, M, e3.y,
                                                    E.corr + (size_t)j * CORR_N);
                  VR_CHECK_LAUNCH();
                }
              }
              return tail_units(E, nb, cfg.est_nseg, cfg.est_ratioA, h[0].has_nan != 0, nan_b, nl, scores + set0,
                                score_ld, viol, st, EM == 4 ? E.corr : nullptr);
            }
          };
          // EST 3 needs every lane to hold k stimuli: the pass holding the full set runs EST 4
          const bool full0 = full_first && p == 0;
          if (tri)
            VR_TRY(full0 ? run_pass(std::integral_constant<int, 6>{}) : run_pass(std::integral_constant<int, 5>{}));
          else
            VR_TRY(cfg.est_mode == 3   ? (full0 ? run_pass(std::integral_constant<int, 4>{})
                                                : run_pass(std::integral_constant<int, 3>{}))
                   : cfg.est_mode == 2 ? run_pass(std::integral_constant<int, 2>{})
                                       : run_pass(std::integral_constant<int, 1>{}));
        }
      }
      return VR_OK;
    }));
    std::vector<uint32_t> flags((size_t)(p1 - p0));
    VR_CHECK_HIP(hipMemcpyAsync(flags.data(), E.viol, flags.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    VR_CHECK_HIP(hipStreamSynchronize(st));
    for (int64_t p = p0; p < p1; ++p) {
      if (!flags[(size_t)(p - p0)]) continue;
      // only the tail invariants flagged it: the A walk's window checks passed, so the B side
      // recovered a wrong rank (an A-flagged pass breaks the invariants too, as expected)
      if ((flags[(size_t)(p - p0)] & 3u) == 2u) g_est_tail_flags.fetch_add(1);
      if (second != JOIN_CHUNK) VR_TRY(join(JOIN_CHUNK));
      g_est_reruns.fetch_add(1);
      const int64_t set0 = p * sub;
      const int nl = (int)std::min<int64_t>(sub, total - set0);
      VR_TRY(with_pass_tag(cfg.use_lds, lw == LANES, narrow, [&](auto tag) { return exact_pass(tag, set0, nl); }));
    }
    if (p0 == pfirst && flags[0] && p1 < npass) return exact_from(p1 * sub);  // give up on the estimate
  }
  return VR_OK;
}

// run_engine_multi_impl, then the exact-form passes' invariant flag: a set flag means the
// exact arithmetic itself went wrong, so the call fails instead of returning the scores.
static int run_engine_multi(const PlanView& A, const PlanView* Bs, int64_t nb, int64_t n,
                            const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                            double* scores, int64_t score_ld, uint32_t* const* joins,
                            const EngineWs& E, int lw, const EngineCfg& cfg, hipStream_t st,
                            const std::vector<int64_t>* exact_passes = nullptr) {
  uint32_t* const xbad = E.viol + EST_MAX_PASSES;
  VR_CHECK_HIP(hipMemsetAsync(xbad, 0, sizeof(uint32_t), st));
  VR_TRY(run_engine_multi_impl(A, Bs, nb, n, idx, k, n_sets, full_first, scores, score_ld, joins, E, lw, cfg, st,
                               exact_passes));
  uint32_t bad = 0;
  VR_CHECK_HIP(hipMemcpyAsync(&bad, xbad, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  VR_CHECK_HIP(hipStreamSynchronize(st));
  if (bad) {
    set_error("bootstrap engine: an exact-form pass broke the rank-sum invariants (included pairs / sum of ranks)");
    return VR_EINTERNAL;
  }
  return VR_OK;
}

// R A plans (regions) x nb B plans (model layers), every unit pre-joined (joins[r][2 j] =
// unit (j, r)'s A positions; joins[r][2 j + 1] = region 0's second arrays): scores of unit
// (j, r) at scores + (r nb + j) score_ld. The EST passes run region-fused (k_rankB_grid: one
// B walk per B plan for all fused regions) on the happy path -- EST 3 with its 4 form for
// the full set, B tie groups < 2^16 -- for every region with A tie groups < 2^16 whose
// estimate passes its up-front check; a region failing that, or one whose pass is later
// flagged, leaves the fused set and runs on its own once the fused passes are done (EST with
// exact re-runs of its flagged passes, or the exact form), so the other regions stay fused.
// Es[0]: region 0's full workspace (multi_layout, prejoined), which also holds the shared
// masks and B segment tables and serves every region run on its own; Es[1..]: slim
// workspaces (u16 TB, no join arrays) beside it.
template <bool LDS>
static int launch_grid(int R, unsigned grid, size_t lds, const PlanView& B, const uint64_t* masks, int64_t n,
                       const GridB& g, uint32_t ns, const uint2* ftab, const uint32_t* segpos, uint32_t* q,
                       hipStream_t st) {
  VR_ONCE(VR_TRY(allow_big_lds(k_rankB_grid<2, LDS>)); VR_TRY(allow_big_lds(k_rankB_grid<3, LDS>));
          VR_TRY(allow_big_lds(k_rankB_grid<4, LDS>)));
  if (R == 2)
    k_rankB_grid<2, LDS><<<grid, ENG_THREADS, lds, st>>>(B.codes, B.gflag, masks, n, g, ns, ftab, segpos, q);
  else if (R == 3)
    k_rankB_grid<3, LDS><<<grid, ENG_THREADS, lds, st>>>(B.codes, B.gflag, masks, n, g, ns, ftab, segpos, q);
  else
    k_rankB_grid<4, LDS><<<grid, ENG_THREADS, lds, st>>>(B.codes, B.gflag, masks, n, g, ns, ftab, segpos, q);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// masks of the grid walk in LDS (one 16-wave workgroup per CU: up to 20,352 stimuli);
// VISREPS_ENGINE_GRID_LDS=0 reads them from L2 at any n (A/B, tests)
static bool grid_masks_lds(int64_t n) {
  return (size_t)n * sizeof(uint64_t) <= 160 * 1024 - 1024 && env_int("VISREPS_ENGINE_GRID_LDS", 1) != 0;
}

template <bool LDS>
static int launch_gridx(int R, unsigned grid, size_t lds, const PlanView& B, const uint64_t* masks, int64_t n,
                        const GridX& g, uint32_t ns, uint32_t L, uint32_t Lm, uint32_t nch, const uint32_t* segpos,
                        uint32_t* q, hipStream_t st) {
  VR_ONCE(VR_TRY(allow_big_lds(k_rankB_gridx<2, LDS>)); VR_TRY(allow_big_lds(k_rankB_gridx<3, LDS>));
          VR_TRY(allow_big_lds(k_rankB_gridx<4, LDS>)));
  if (R == 2)
    k_rankB_gridx<2, LDS><<<grid, ENG_THREADS, lds, st>>>(B.codes, B.gflag, masks, n, g, ns, L, Lm, nch, segpos, q);
  else if (R == 3)
    k_rankB_gridx<3, LDS><<<grid, ENG_THREADS, lds, st>>>(B.codes, B.gflag, masks, n, g, ns, L, Lm, nch, segpos, q);
  else
    k_rankB_gridx<4, LDS><<<grid, ENG_THREADS, lds, st>>>(B.codes, B.gflag, masks, n, g, ns, L, Lm, nch, segpos, q);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

// A region a grid call can walk in the exact grid form: u16 chunk-relative ranks (every A
// chunk span, < L + its largest tie group, <= 32767) and 64-bit tie sums (groups < 2^16)
static bool gridx_region_ok(const PlanHeader& h) {
  return (uint64_t)PLAN_L + h.max_group <= 32767u && h.max_group < 65536u;
}

// Every pass of regions rs (2..4 of them, gridx_region_ok; B tie groups < 2^16) in the exact
// chunk-base form, region-fused: per pass the masks once, each region's exact A walk
// (pass_a: TB, chunk bases), then one k_rankB_gridx launch per B plan for all of them, then
// each region's tail. B segments: cfg.nwaves per plan (the exact A side's count, so the tail
// pairs them as the per-region exact calls do). E: the grid's workspaces (E[r].masks = the
// shared masks); region 0's B segment tables and queue counters are rewritten.
static int grid_exact(const PlanView* As, const std::vector<int>& rs, const PlanView* Bs, int64_t nb, int64_t n,
                      const int32_t* idx, int64_t k, int64_t n_sets, int full_first, double* scores,
                      int64_t score_ld, uint32_t* const* const* joins, const std::vector<EngineWs>& E,
                      const std::vector<PlanHeader>& hA, const std::vector<char>& nan_b, const EngineCfg& cfg,
                      hipStream_t st) {
  const int64_t M = pairs_of(n);
  const int64_t total = n_sets + (full_first ? 1 : 0);
  const int RA = (int)rs.size();
  VR_REQUIRE(RA >= 2 && RA <= 4, "grid_exact: %d regions", RA);
  const uint32_t nch = plan_nchunks(M), L = plan_chunk_len(M);
  const uint32_t Lm = (uint32_t)(((uint64_t)1 << 32) / L);
  const uint32_t nsx = (uint32_t)cfg.nwaves;
  VR_REQUIRE(E[0].segstride >= (size_t)nsx + 1 && E[0].useg >= (size_t)nsx * LANES, "grid_exact: segment tables");
  for (int64_t j = 0; j < nb; ++j) {
    k_seg_table<<<(nsx + 256) / 256, 256, 0, st>>>(Bs[j].gstart, Bs[j].hdr, M, nsx,
                                                    E[0].segposB + E[0].segstride * (size_t)j);
    VR_CHECK_LAUNCH();
  }
  for (int r : rs) VR_CHECK_HIP(hipMemsetAsync(E[(size_t)r].viol + EST_MAX_PASSES, 0, sizeof(uint32_t), st));
  const unsigned ggrid = (unsigned)num_cus();
  const bool glds = grid_masks_lds(n);
  // regions per launch: all, or (VISREPS_ENGINE_GRIDX_MAXR < 4, A/B) 4 regions as 2 + 2
  const int maxr = (RA == 4 && env_int("VISREPS_ENGINE_GRIDX_MAXR", 4) < 4) ? 2 : RA;
  const int64_t npass = (total + LANES - 1) / LANES;
  for (int64_t p = 0; p < npass; ++p) {
    const int64_t set0 = p * LANES;
    const int nl = (int)std::min<int64_t>(LANES, total - set0);
    VR_TRY(build_pass_masks(idx, k, set0, nl, full_first, E[0].masks, n, st));
    for (int r : rs) {
      const EngineWs& e = E[(size_t)r];
      VR_TRY((cfg.use_lds ? pass_a<true, true, uint16_t, false>(As[r], n, e, LANES, cfg, st)
                          : pass_a<false, true, uint16_t, false>(As[r], n, e, LANES, cfg, st)));
      // the chunk starts go to lpA, dead once pass_a has turned it into baseA
      k_chunk_starts<<<(nch + 255) / 256, 256, 0, st>>>(As[r].gstart, As[r].chunk_g, nch, e.lpA);
      VR_CHECK_LAUNCH();
    }
    VR_CHECK_HIP(hipMemsetAsync(E[0].queue + QS_RANKB, 0,
                                sizeof(uint32_t) * (size_t)std::min<int64_t>(nb, QSLOTS - QS_RANKB), st));
    for (int64_t j = 0; j < nb; ++j) {
      const uint32_t* segpos = E[0].segposB + E[0].segstride * (size_t)j;
      for (int i0 = 0; i0 < RA; i0 += maxr) {  // region groups of <= maxr per launch
        const int ri = std::min(maxr, RA - i0);
        GridX g{};
        for (int i = 0; i < ri; ++i) {
          const int r = rs[(size_t)(i0 + i)];
          const EngineWs& e = E[(size_t)r];
          const size_t us = e.useg * (size_t)j;
          g.TB[i] = static_cast<const uint16_t*>(e.TB);
          g.posA[i] = joins[r][2 * j];
          g.base[i] = e.baseA;
          g.cst[i] = e.lpA;
          g.seg_tot[i] = e.segB_tot + us;
          g.seg_part[i] = e.segB_part + us * PB_N;
        }
        uint32_t* q = E[0].queue + QS_RANKB + (size_t)(j * 2 + i0 / maxr) % (size_t)(QSLOTS - QS_RANKB);
        VR_CHECK_HIP(hipMemsetAsync(q, 0, sizeof(uint32_t), st));
        KtScope kt(KT_RANKB_GRIDX, (double)M * ri, st);
        if (glds)
          VR_TRY(launch_gridx<true>(ri, ggrid, (size_t)n * sizeof(uint64_t), Bs[j], E[0].masks, n, g, nsx, L, Lm, nch,
                                    segpos, q, st));
        else
          VR_TRY(launch_gridx<false>(ri, ggrid, 0, Bs[j], E[0].masks, n, g, nsx, L, Lm, nch, segpos, q, st));
      }
    }
    for (int r : rs)
      VR_TRY(tail_units(E[(size_t)r], nb, nsx, 1u, hA[(size_t)r].has_nan != 0, nan_b, nl,
                        scores + (size_t)r * nb * score_ld + set0, score_ld, E[(size_t)r].viol + EST_MAX_PASSES, st));
  }
  for (int r : rs) {  // an exact pass that breaks the invariants is an error, as in run_engine_multi
    uint32_t bad = 0;
    VR_CHECK_HIP(hipMemcpyAsync(&bad, E[(size_t)r].viol + EST_MAX_PASSES, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    VR_CHECK_HIP(hipStreamSynchronize(st));
    if (bad) {
      set_error("bootstrap engine: an exact grid pass broke the rank-sum invariants (included pairs / sum of ranks)");
      return VR_EINTERNAL;
    }
  }
  return VR_OK;
}

static int run_engine_grid(const PlanView* As, int R, const PlanView* Bs, int64_t nb, int64_t n, const int32_t* idx,
                           int64_t k, int64_t n_sets, int full_first, double* scores, int64_t score_ld,
                           uint32_t* const* const* joins, const EngineWs* Es, const EngineCfg& cfg, hipStream_t st) {
  const int64_t M = pairs_of(n);
  const int64_t total = n_sets + (full_first ? 1 : 0);
  std::vector<int> solo;  // regions run on their own once the fused passes are done
  std::vector<std::vector<int64_t>> fix((size_t)R);  // fused regions' flagged passes (re-run exact)
  std::vector<int> xg;  // regions walked together in the exact grid form (grid_exact), before the solos
  std::vector<PlanHeader> hA((size_t)R), hB((size_t)nb);
  std::vector<char> nan_b((size_t)nb);
  std::vector<EngineWs> E(Es, Es + R);  // the masks of a pass are built once (region 0's buffer)
  for (int r = 1; r < R; ++r) E[(size_t)r].masks = E[0].masks;
  auto finish = [&]() -> int {
    if (!xg.empty())
      VR_TRY(grid_exact(As, xg, Bs, nb, n, idx, k, n_sets, full_first, scores, score_ld, joins, E, hA, nan_b, cfg, st));
    for (int r : solo)
      VR_TRY(run_engine_multi(As[r], Bs, nb, n, idx, k, n_sets, full_first, scores + (size_t)r * nb * score_ld,
                              score_ld, joins[r], Es[0], LANES, cfg, st));
    for (int r = 0; r < R; ++r)
      if (!fix[(size_t)r].empty())
        VR_TRY(run_engine_multi(As[r], Bs, nb, n, idx, k, n_sets, full_first, scores + (size_t)r * nb * score_ld,
                                score_ld, joins[r], Es[0], LANES, cfg, st, &fix[(size_t)r]));
    return VR_OK;
  };
  auto all_solo = [&]() -> int {
    solo.clear();
    for (int r = 0; r < R; ++r)
      if (std::find(xg.begin(), xg.end(), r) == xg.end()) solo.push_back(r);
    return finish();
  };
  if (total == 0 || nb == 0 || M == 0) return all_solo();
  for (int r = 0; r < R; ++r)
    VR_CHECK_HIP(hipMemcpyAsync(&hA[(size_t)r], As[r].hdr, sizeof(PlanHeader), hipMemcpyDeviceToHost, st));
  for (int64_t j = 0; j < nb; ++j)
    VR_CHECK_HIP(hipMemcpyAsync(&hB[(size_t)j], Bs[j].hdr, sizeof(PlanHeader), hipMemcpyDeviceToHost, st));
  VR_CHECK_HIP(hipStreamSynchronize(st));
  for (int64_t j = 0; j < nb; ++j) nan_b[(size_t)j] = hB[(size_t)j].has_nan != 0;
  bool b_small = true;  // B tie groups < 2^16 (the fused walks' 64-bit tie sums)
  for (int64_t j = 0; j < nb; ++j) b_small = b_small && hB[(size_t)j].max_group < 65536u;
  // the exact grid form (opt-in, VISREPS_ENGINE_GRIDX=1): measured slower than the per-region
  // exact calls on the bench RDMs (36.2-36.9 against 33.8 ms per unit, every pass exact,
  // profiles/r6_exact_grid_ab.log): one 16-wave workgroup per CU, which the LDS masks and
  // 128 VGPRs allow, cannot keep the two gathers per pair and region in flight that the
  // per-region walks' two workgroups per CU do
  const bool gridx = b_small && R >= 2 && R <= 4 && env_int("VISREPS_ENGINE_GRID", 1) != 0 &&
                     env_int("VISREPS_ENGINE_GRIDX", 0) != 0;
  auto take_exact_grid = [&](const std::vector<int>& rs) -> std::vector<int> {  // -> the regions left over
    std::vector<int> ok, rest;
    for (int r : rs) (gridx && gridx_region_ok(hA[(size_t)r]) ? ok : rest).push_back(r);
    if (ok.size() >= 2)
      xg.insert(xg.end(), ok.begin(), ok.end());
    else
      rest.insert(rest.end(), ok.begin(), ok.end());
    std::sort(xg.begin(), xg.end());
    return rest;
  };
  if (!engine_est()) {  // every pass exact: the exact grid where it applies
    std::vector<int> all;
    for (int r = 0; r < R; ++r) all.push_back(r);
    take_exact_grid(all);
    return all_solo();
  }
  bool fused = cfg.est_mode == 3 && R >= 2 && R <= 4 && env_int("VISREPS_ENGINE_TRI", 0) == 0 &&
               env_int("VISREPS_ENGINE_LO_JOIN", 0) == 0 && env_int("VISREPS_ENGINE_GRID", 1) != 0;
  // test hook (vr_test_engine_inject): the first fused region's TB gets the B-side error after
  // its A walk of that pass, so the region must be flagged and re-run on its own
  const int64_t inject = g_test_inject.load(std::memory_order_relaxed);
  fused = fused && b_small;
  if (!fused) return all_solo();
  std::vector<int> act;  // the fused regions
  for (int r = 0; r < R; ++r) (hA[(size_t)r].max_group < 65536u ? act : solo).push_back(r);
  // (a point-only call holds the full set alone: its window is the full set's, so lane 0's
  // EST 4 shift is at most 1 -- with k's window instead a group of > 3 tied pairs could
  // shift below 1 and flag the pass)
  const uint2 e3 = est3_params(n_sets > 0 ? k : n, M);
  const uint2 trip = make_uint2(0u, 0u);
  const uint32_t ns = cfg.est_nseg, nsA = cfg.est_nsegA;
  // A-side walks: masks in LDS when two 16-wave workgroups per CU hold them (n <= 10,176),
  // else from L2 (the per-region calls' choice, engine_cfg)
  auto est_a = [&](auto&& fn) -> int {
    return cfg.est_lds ? fn(std::integral_constant<bool, true>{}) : fn(std::integral_constant<bool, false>{});
  };
  for (int r : act) {
    k_seg_table<<<(nsA + 256) / 256, 256, 0, st>>>(As[r].gstart, As[r].hdr, M, nsA, E[(size_t)r].segposA);
    VR_CHECK_LAUNCH();
  }
  for (int64_t j = 0; j < nb; ++j) {  // B segments depend on the B plan only: region 0's table
    k_seg_table<<<(ns + 256) / 256, 256, 0, st>>>(Bs[j].gstart, Bs[j].hdr, M, ns, E[0].segposB + E[0].segstride * (size_t)j);
    VR_CHECK_LAUNCH();
  }
  // the up-front estimate check, per region (its counts are its own)
  if (n_sets > 0 && env_int("VISREPS_ENGINE_EST_PREDICT", 1) != 0) {
    const int nl0 = (int)std::min<int64_t>(LANES, total);
    VR_TRY(build_pass_masks(idx, k, 0, nl0, full_first, E[0].masks, n, st));
    std::vector<int> keep, pbad;
    for (int r : act) {
      bool bad = false;
      VR_TRY(est_a([&](auto cl) -> int {
        return est_predict<decltype(cl)::value, true>(As[r], n, E[(size_t)r], LANES, nl0, full_first != 0, cfg, e3,
                                                      st, bad);
      }));
      (bad ? pbad : keep).push_back(r);
    }
    act.swap(keep);
    // Regions off the estimate go to the exact form (run_engine_multi's choice while the exact
    // walks keep their masks in LDS; above that EST 1 serves them on their own): two or more of
    // them walk it region-fused
    if (cfg.use_lds || env_int("VISREPS_ENGINE_EST1_FALLBACK", 1) == 0) {
      for (int r : take_exact_grid(pbad)) solo.push_back(r);
      g_est_predicted.fetch_add((int64_t)xg.size());
    } else {
      for (int r : pbad) solo.push_back(r);
    }
  }
  if (act.size() < 2) return all_solo();  // fusing pays with two regions or more
  const int64_t npass = (total + LANES - 1) / LANES;
  const unsigned ggrid = (unsigned)num_cus();  // one 16-wave workgroup per CU (4 waves per SIMD)
  const bool glds = grid_masks_lds(n);
  for (int r : act)
    VR_CHECK_HIP(hipMemsetAsync(E[(size_t)r].viol, 0, (size_t)std::min<int64_t>(npass, EST_MAX_PASSES) * sizeof(uint32_t), st));
  for (int64_t p = 0; p < npass; ++p) {
    const int64_t set0 = p * LANES;
    const int nl = (int)std::min<int64_t>(LANES, total - set0);
    const bool full0 = full_first && p == 0;
    const int64_t vslot = p % EST_MAX_PASSES;
    VR_TRY(build_pass_masks(idx, k, set0, nl, full_first, E[0].masks, n, st));
    for (int r : act) {
      VR_CHECK_HIP(hipMemsetAsync(E[(size_t)r].queue, 0, sizeof(uint32_t) * (size_t)QS_RANKB, st));
      uint32_t* viol = E[(size_t)r].viol + vslot;
      VR_TRY(est_a([&](auto cl) -> int {
        constexpr bool CL = decltype(cl)::value;
        return full0 ? pass_a_est<4, CL, true, false>(As[r], n, E[(size_t)r], LANES, nl, cfg, e3, trip, viol, st)
                     : pass_a_est<3, CL, true, false>(As[r], n, E[(size_t)r], LANES, nl, cfg, e3, trip, viol, st);
      }));
      if (p == inject && r == act[0]) {
        k_inject_tb<<<1, LANES, 0, st>>>(static_cast<uint16_t*>(E[(size_t)r].TB), (uint32_t)(M / 2), LANES, nl);
        VR_CHECK_LAUNCH();
      }
    }
    VR_CHECK_HIP(hipMemsetAsync(E[0].queue + QS_RANKB, 0,
                                sizeof(uint32_t) * (size_t)std::min<int64_t>(nb, QSLOTS - QS_RANKB), st));
    const int RA = (int)act.size();
    for (int64_t j = 0; j < nb; ++j) {
      GridB g{};
      for (int i = 0; i < RA; ++i) {
        const EngineWs& e = E[(size_t)act[(size_t)i]];
        const size_t us = e.useg * (size_t)j;
        g.TB[i] = static_cast<const uint16_t*>(e.TB);
        g.posA[i] = joins[act[(size_t)i]][2 * j];
        g.seg_tot[i] = e.segB_tot + us;
        g.seg_part[i] = e.segB_part + us * PB_N;
      }
      uint32_t* q = E[0].queue + QS_RANKB + (size_t)j % (size_t)(QSLOTS - QS_RANKB);
      if (j >= QSLOTS - QS_RANKB) VR_CHECK_HIP(hipMemsetAsync(q, 0, sizeof(uint32_t), st));
      const uint32_t* segpos = E[0].segposB + E[0].segstride * (size_t)j;
      // the window parameters of this pass (k_c0_u: the same for every region) from a fused
      // region's workspace: region 0 may be running on its own
      const uint2* ftab = E[(size_t)act[0]].ftab;
      KtScope kt(full0 ? KT_RANKB_FULL : KT_RANKB_GRID, (double)M * RA, st);
      if (glds)
        VR_TRY(launch_grid<true>(RA, ggrid, (size_t)n * sizeof(uint64_t), Bs[j], E[0].masks, n, g, ns, ftab,
                                 segpos, q, st));
      else
        VR_TRY(launch_grid<false>(RA, ggrid, 0, Bs[j], E[0].masks, n, g, ns, ftab, segpos, q, st));
    }
    for (int r : act) {
      if (full0) {
        for (int64_t j = 0; j < nb; ++j) {
          KtScope kt(KT_FULL_CORR, (double)M, st);
          k_full_corr<<<CORR_BLK, 256, 0, st>>>(joins[r][2 * j], Bs[j].gflag, Bs[j].gstart, hB[(size_t)j].G, M, e3.y,
                                                E[(size_t)r].corr + (size_t)j * CORR_N);
          VR_CHECK_LAUNCH();
        }
      }
      VR_TRY(tail_units(E[(size_t)r], nb, ns, cfg.est_ratioA, hA[(size_t)r].has_nan != 0, nan_b, nl,
                        scores + (size_t)r * nb * score_ld + set0, score_ld, E[(size_t)r].viol + vslot, st,
                        full0 ? E[(size_t)r].corr : nullptr));
    }
    // flags: after the first pass, then every EST_MAX_PASSES passes and at the end. A region
    // whose first pass is flagged (its estimate is off: structured counts, giant tie groups)
    // leaves the fused set and runs on its own at the end, which rewrites all of its scores;
    // a later flagged pass (rare: a B-side recovery broke the tail invariants, or one subset
    // strayed) is re-run alone in the exact form at the end, the region staying fused. The
    // other regions' sums are their own and stand.
    if (p == 0 || vslot == EST_MAX_PASSES - 1 || p == npass - 1) {
      const int64_t cnt = vslot + 1, pbase = p - vslot;
      std::vector<int> keep;
      for (int r : act) {
        std::vector<uint32_t> flags((size_t)cnt);
        VR_CHECK_HIP(hipMemcpyAsync(flags.data(), E[(size_t)r].viol, flags.size() * sizeof(uint32_t),
                                    hipMemcpyDeviceToHost, st));
        VR_CHECK_HIP(hipStreamSynchronize(st));
        if (p == 0 && flags[0]) {
          solo.push_back(r);
          continue;
        }
        for (int64_t i = 0; i < cnt; ++i) {
          if (!flags[(size_t)i]) continue;
          fix[(size_t)r].push_back(pbase + i);
          g_est_reruns.fetch_add(1);
          if ((flags[(size_t)i] & 3u) == 2u) g_est_tail_flags.fetch_add(1);
        }
        keep.push_back(r);
      }
      act.swap(keep);
      if (act.size() < 2 && p + 1 < npass) {  // one region left: it runs on its own too
        for (int r : act) {
          solo.push_back(r);
          fix[(size_t)r].clear();
        }
        act.clear();
        break;
      }
      if (vslot == EST_MAX_PASSES - 1 && p + 1 < npass)
        for (int r : act)
          VR_CHECK_HIP(hipMemsetAsync(E[(size_t)r].viol, 0, (size_t)EST_MAX_PASSES * sizeof(uint32_t), st));
    }
  }
  std::sort(solo.begin(), solo.end());
  return finish();
}

// Scores for `total` subsets (full set first if full_first), 64 per pass.
static int run_engine(const PlanView& A, const PlanView& B, int64_t n, const int32_t* idx,
                      int64_t k, int64_t n_sets, int full_first, double* scores,
                      const EngineWs& E, int lw, const EngineCfg& cfg, hipStream_t st) {
  uint32_t* joins[2] = {E.posA_byB, E.chunkA_byB};
  return run_engine_multi(A, &B, 1, n, idx, k, n_sets, full_first, scores, 0, joins, E, lw, cfg, st);
}

// Workspace of the multi-B engine: the engine scratch, then the joins of B 1..nb-1 (B 0
// uses the engine's own join arrays). prejoined (the caller passes every unit's A positions,
// vr_bootstrap_spearman_multi_joined): only the second array of each later unit is carved.
static size_t multi_layout(void* base, int64_t n, int64_t nb, int nwaves, EngineWs* E,
                           std::vector<uint32_t*>* joins, bool prejoined = false) {
  size_t eb = 0;
  const EngineWs e = engine_layout(base, n, LANES, nwaves, &eb, nb);
  const int64_t M = pairs_of(n);
  Carver c(base ? static_cast<char*>(base) + eb : nullptr);
  if (joins) joins->assign((size_t)std::max<int64_t>(nb, 1) * 2, nullptr);
  if (joins && nb > 0) {
    (*joins)[0] = e.posA_byB;
    (*joins)[1] = e.chunkA_byB;
  }
  for (int64_t j = 1; j < nb; ++j) {
    uint32_t* p = prejoined ? nullptr : c.take<uint32_t>((size_t)M);
    uint32_t* q = c.take<uint32_t>((size_t)M);
    if (joins) {
      (*joins)[2 * j] = p;
      (*joins)[2 * j + 1] = q;
    }
  }
  if (E) *E = e;
  return eb + c.bytes();
}

static size_t oneshot_bytes(int64_t n, int lw, int nwaves, void* base, PlanView* A, PlanView* B,
                            PlanBuildWs* W, EngineWs* E) {
  Carver c(base);
  const size_t pb = plan_bytes(n);
  char* pa = c.take<char>(pb);
  char* pbb = c.take<char>(pb);
  size_t wb = 0, eb = 0;
  plan_build_layout(nullptr, n, &wb);
  engine_layout(nullptr, n, lw, nwaves, &eb);
  char* wsb = c.take<char>(std::max(wb, eb));  // plan-build scratch is dead once plans exist
  if (base) {
    *A = plan_layout(pa, n);
    *B = plan_layout(pbb, n);
    *W = plan_build_layout(wsb, n, nullptr);
    *E = engine_layout(wsb, n, lw, nwaves, nullptr);
  }
  return c.bytes();
}

}  // namespace vr

using namespace vr;

extern "C" {

int64_t vr_engine_est_reruns(void) { return g_est_reruns.load(); }
int64_t vr_engine_est_tail_flags(void) { return g_est_tail_flags.load(); }
int64_t vr_engine_est_predicted(void) { return g_est_predicted.load(); }
int64_t vr_engine_est1_fallbacks(void) { return g_est1_fallbacks.load(); }
int vr_test_engine_inject(int64_t pass) {
  g_test_inject.store(pass < 0 ? -1 : pass);
  return VR_OK;
}
#if VR_PROBE_WT
// probe builds only: the wave start / end clocks (wall_clock64, 100 MHz) of the last k_rankB
int vr_probe_wave_times(uint64_t* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wt), sizeof(uint64_t) * 2 * 16384) == hipSuccess ? 0 : -1;
}
#endif

size_t vr_bootstrap_workspace(int64_t n) {
  size_t b = 0;
  n = n < 0 ? 0 : n;
  engine_layout(nullptr, n, LANES, engine_cfg(n).nwaves, &b);
  return b;
}

int vr_bootstrap_spearman_plans(const void* planA, const void* planB, int64_t n,
                                const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                                double* scores, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535, "vr_bootstrap_spearman_plans: n=%lld out of range", (long long)n);
  VR_REQUIRE(planA && planB && scores, "vr_bootstrap_spearman_plans: null pointer");
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "vr_bootstrap_spearman_plans: bad k=%lld sets=%lld",
             (long long)k, (long long)n_sets);
  VR_REQUIRE(idx != nullptr || n_sets == 0 || k == 0, "vr_bootstrap_spearman_plans: null idx");
  const EngineCfg cfg = engine_cfg(n);
  size_t need = 0;
  EngineWs E = engine_layout(ws, n, LANES, cfg.nwaves, &need);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_bootstrap_spearman_plans: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView A = plan_layout(const_cast<void*>(planA), n);
  PlanView B = plan_layout(const_cast<void*>(planB), n);
  return run_engine(A, B, n, idx, k, n_sets, full_first, scores, E, LANES, cfg, as_stream(stream));
}

size_t vr_bootstrap_multi_workspace(int64_t n, int64_t n_b) {
  n = n < 0 ? 0 : n;
  n_b = n_b < 1 ? 1 : n_b;
  return multi_layout(nullptr, n, n_b, engine_cfg(n).nwaves, nullptr, nullptr);
}

int vr_bootstrap_spearman_multi(const void* planA, const void* const* planBs, int64_t n_b, int64_t n,
                                const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                                double* scores, int64_t ld_scores, void* ws, size_t ws_bytes,
                                void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535, "vr_bootstrap_spearman_multi: n=%lld out of range", (long long)n);
  VR_REQUIRE(n_b >= 0, "vr_bootstrap_spearman_multi: n_b=%lld", (long long)n_b);
  VR_REQUIRE(planA && (n_b == 0 || (planBs && scores)), "vr_bootstrap_spearman_multi: null pointer");
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "vr_bootstrap_spearman_multi: bad k=%lld sets=%lld",
             (long long)k, (long long)n_sets);
  VR_REQUIRE(idx != nullptr || n_sets == 0 || k == 0, "vr_bootstrap_spearman_multi: null idx");
  const int64_t total = n_sets + (full_first ? 1 : 0);
  VR_REQUIRE(n_b <= 1 || ld_scores >= total, "vr_bootstrap_spearman_multi: ld_scores %lld < %lld",
             (long long)ld_scores, (long long)total);
  for (int64_t j = 0; j < n_b; ++j)
    VR_REQUIRE(planBs[j] != nullptr, "vr_bootstrap_spearman_multi: planBs[%lld] is null", (long long)j);
  const EngineCfg cfg = engine_cfg(n);
  const size_t need = multi_layout(nullptr, n, n_b, cfg.nwaves, nullptr, nullptr);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_bootstrap_spearman_multi: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  EngineWs E;
  std::vector<uint32_t*> joins;
  multi_layout(ws, n, n_b, cfg.nwaves, &E, &joins);
  const PlanView A = plan_layout(const_cast<void*>(planA), n);
  std::vector<PlanView> Bs;
  for (int64_t j = 0; j < n_b; ++j) Bs.push_back(plan_layout(const_cast<void*>(planBs[j]), n));
  return run_engine_multi(A, Bs.data(), n_b, n, idx, k, n_sets, full_first, scores, ld_scores,
                          joins.data(), E, LANES, cfg, as_stream(stream));
}

size_t vr_bootstrap_multi_joined_workspace(int64_t n, int64_t n_b) {
  n = n < 0 ? 0 : n;
  n_b = n_b < 1 ? 1 : n_b;
  return multi_layout(nullptr, n, n_b, engine_cfg(n).nwaves, nullptr, nullptr, true);
}

int vr_bootstrap_spearman_multi_joined(const void* planA, const void* const* planBs, int64_t n_b, int64_t n,
                                const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                                double* scores, int64_t ld_scores, uint32_t* const* posA, void* ws,
                                size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535, "vr_bootstrap_spearman_multi_joined: n=%lld out of range", (long long)n);
  VR_REQUIRE(n_b >= 0, "vr_bootstrap_spearman_multi_joined: n_b=%lld", (long long)n_b);
  VR_REQUIRE(planA && (n_b == 0 || (planBs && scores)), "vr_bootstrap_spearman_multi_joined: null pointer");
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "vr_bootstrap_spearman_multi_joined: bad k=%lld sets=%lld",
             (long long)k, (long long)n_sets);
  VR_REQUIRE(idx != nullptr || n_sets == 0 || k == 0, "vr_bootstrap_spearman_multi_joined: null idx");
  const int64_t total = n_sets + (full_first ? 1 : 0);
  VR_REQUIRE(n_b <= 1 || ld_scores >= total, "vr_bootstrap_spearman_multi_joined: ld_scores %lld < %lld",
             (long long)ld_scores, (long long)total);
  for (int64_t j = 0; j < n_b; ++j)
    VR_REQUIRE(planBs[j] != nullptr, "vr_bootstrap_spearman_multi_joined: planBs[%lld] is null", (long long)j);
  VR_REQUIRE(n_b == 0 || posA != nullptr, "vr_bootstrap_spearman_multi_joined: null posA");
  for (int64_t j = 0; j < n_b; ++j)
    VR_REQUIRE(posA[j] != nullptr, "vr_bootstrap_spearman_multi_joined: posA[%lld] is null", (long long)j);
  EngineCfg cfg = engine_cfg(n);
  cfg.prejoined = true;
  const size_t need = multi_layout(nullptr, n, n_b, cfg.nwaves, nullptr, nullptr, true);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_bootstrap_spearman_multi_joined: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  EngineWs E;
  std::vector<uint32_t*> joins;
  multi_layout(ws, n, n_b, cfg.nwaves, &E, &joins, true);
  for (int64_t j = 0; j < n_b; ++j) joins[(size_t)(2 * j)] = posA[j];
  const PlanView A = plan_layout(const_cast<void*>(planA), n);
  std::vector<PlanView> Bs;
  for (int64_t j = 0; j < n_b; ++j) Bs.push_back(plan_layout(const_cast<void*>(planBs[j]), n));
  return run_engine_multi(A, Bs.data(), n_b, n, idx, k, n_sets, full_first, scores, ld_scores,
                          joins.data(), E, LANES, cfg, as_stream(stream));
}

// A grid call's workspace: region 0's full joined-multi layout, then one slim layout (u16 TB,
// no join arrays) per further region
static size_t grid_slim_bytes(int64_t n, int64_t n_b, int nwaves) {
  size_t b = 0;
  engine_layout(nullptr, n, LANES, nwaves, &b, n_b, true);
  return b;
}

size_t vr_bootstrap_grid_joined_workspace(int64_t n, int64_t n_a, int64_t n_b) {
  n = n < 0 ? 0 : n;
  n_a = n_a < 1 ? 1 : n_a;
  n_b = n_b < 1 ? 1 : n_b;
  const int nw = engine_cfg(n).nwaves;
  return multi_layout(nullptr, n, n_b, nw, nullptr, nullptr, true) + (size_t)(n_a - 1) * grid_slim_bytes(n, n_b, nw);
}

int vr_bootstrap_spearman_grid_joined(const void* const* planAs, int64_t n_a, const void* const* planBs, int64_t n_b,
                                      int64_t n, const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                                      double* scores, int64_t ld_scores, uint32_t* const* posA, void* ws,
                                      size_t ws_bytes, void* stream) {
  const char* fn = "vr_bootstrap_spearman_grid_joined";
  VR_REQUIRE(n >= 0 && n <= 65535, "%s: n=%lld out of range", fn, (long long)n);
  VR_REQUIRE(n_a >= 1 && n_a <= 4, "%s: n_a=%lld not in [1, 4]", fn, (long long)n_a);
  VR_REQUIRE(n_b >= 0, "%s: n_b=%lld", fn, (long long)n_b);
  VR_REQUIRE(planAs && (n_b == 0 || (planBs && scores && posA)), "%s: null pointer", fn);
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "%s: bad k=%lld sets=%lld", fn, (long long)k, (long long)n_sets);
  VR_REQUIRE(idx != nullptr || n_sets == 0 || k == 0, "%s: null idx", fn);
  const int64_t total = n_sets + (full_first ? 1 : 0);
  VR_REQUIRE(ld_scores >= total, "%s: ld_scores %lld < %lld", fn, (long long)ld_scores, (long long)total);
  for (int64_t i = 0; i < n_a; ++i) VR_REQUIRE(planAs[i] != nullptr, "%s: planAs[%lld] is null", fn, (long long)i);
  for (int64_t j = 0; j < n_b; ++j) VR_REQUIRE(planBs[j] != nullptr, "%s: planBs[%lld] is null", fn, (long long)j);
  for (int64_t u = 0; u < n_a * n_b; ++u) VR_REQUIRE(posA[u] != nullptr, "%s: posA[%lld] is null", fn, (long long)u);
  EngineCfg cfg = engine_cfg(n);
  cfg.prejoined = true;
  const size_t full = multi_layout(nullptr, n, n_b, cfg.nwaves, nullptr, nullptr, true);
  const size_t slim = grid_slim_bytes(n, n_b, cfg.nwaves);
  const size_t need = full + (size_t)(n_a - 1) * slim;
  if (ws == nullptr || ws_bytes < need) {
    set_error("%s: workspace %zu < %zu", fn, ws_bytes, need);
    return VR_EWORKSPACE;
  }
  std::vector<EngineWs> E((size_t)n_a);
  std::vector<uint32_t*> j0;
  multi_layout(ws, n, n_b, cfg.nwaves, &E[0], &j0, true);
  for (int64_t i = 1; i < n_a; ++i)
    E[(size_t)i] = engine_layout(static_cast<char*>(ws) + full + (size_t)(i - 1) * slim, n, LANES, cfg.nwaves,
                                 nullptr, n_b, true);
  // every region: its own A positions, region 0's second arrays (the exact form's A chunks,
  // written when a region runs on its own)
  std::vector<std::vector<uint32_t*>> jv((size_t)n_a, j0);
  std::vector<uint32_t* const*> joins((size_t)n_a);
  std::vector<PlanView> As;
  for (int64_t i = 0; i < n_a; ++i) {
    for (int64_t j = 0; j < n_b; ++j) jv[(size_t)i][(size_t)(2 * j)] = posA[i * n_b + j];
    joins[(size_t)i] = jv[(size_t)i].data();
    As.push_back(plan_layout(const_cast<void*>(planAs[i]), n));
  }
  std::vector<PlanView> Bs;
  for (int64_t j = 0; j < n_b; ++j) Bs.push_back(plan_layout(const_cast<void*>(planBs[j]), n));
  return run_engine_grid(As.data(), (int)n_a, Bs.data(), n_b, n, idx, k, n_sets, full_first, scores, ld_scores,
                         joins.data(), E.data(), cfg, as_stream(stream));
}

size_t vr_engine_posmap4_bytes(int64_t n) { return (size_t)pairs_of(n) * sizeof(uint4); }

int vr_engine_posmap4(const void* const* planAs, int64_t n_a, int64_t n, void* posmap4, void* stream) {
  VR_REQUIRE(n >= 2 && n <= 65535, "vr_engine_posmap4: n=%lld out of range", (long long)n);
  VR_REQUIRE(n_a >= 1 && n_a <= 4, "vr_engine_posmap4: n_a=%lld not in [1, 4]", (long long)n_a);
  VR_REQUIRE(planAs && posmap4, "vr_engine_posmap4: null pointer");
  Maps4 m{{nullptr, nullptr, nullptr, nullptr}};
  for (int64_t i = 0; i < n_a; ++i) {
    VR_REQUIRE(planAs[i] != nullptr, "vr_engine_posmap4: planAs[%lld] is null", (long long)i);
    m.p[i] = plan_layout(const_cast<void*>(planAs[i]), n).pos_map;
  }
  const int64_t M = pairs_of(n);
  k_posmap4<<<(unsigned)((M + 255) / 256), 256, 0, as_stream(stream)>>>(m, (int)n_a, M,
                                                                         static_cast<uint4*>(posmap4));
  VR_CHECK_LAUNCH();
  return VR_OK;
}

int vr_engine_join4(const void* posmap4, int64_t n_a, const void* planB, int64_t n, uint32_t* const* posA,
                    void* stream) {
  VR_REQUIRE(n >= 2 && n <= 65535, "vr_engine_join4: n=%lld out of range", (long long)n);
  VR_REQUIRE(n_a >= 1 && n_a <= 4, "vr_engine_join4: n_a=%lld not in [1, 4]", (long long)n_a);
  VR_REQUIRE(posmap4 && planB && posA, "vr_engine_join4: null pointer");
  Outs4 o{{nullptr, nullptr, nullptr, nullptr}};
  for (int64_t i = 0; i < n_a; ++i) {
    VR_REQUIRE(posA[i] != nullptr, "vr_engine_join4: posA[%lld] is null", (long long)i);
    o.p[i] = posA[i];
  }
  const int64_t M = pairs_of(n);
  const PlanView B = plan_layout(const_cast<void*>(planB), n);
  hipStream_t st = as_stream(stream);
  KtScope kt(KT_JOIN4, (double)M * (4.0 + 16.0 + 4.0 * (double)n_a), st);  // codes + record gather + writes
  k_join4<<<(unsigned)((M + 255) / 256), 256, 0, st>>>(B.codes, M, n, static_cast<const uint4*>(posmap4), (int)n_a,
                                                       o);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

size_t vr_bootstrap_spearman_workspace(int64_t n) {
  n = n < 0 ? 0 : n;
  return oneshot_bytes(n, LANES, engine_cfg(n).nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int vr_bootstrap_spearman_f32(const float* A, const float* B, int64_t n, int64_t ld,
                              const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                              double* scores, void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535 && ld >= n, "vr_bootstrap_spearman_f32: bad shape");
  VR_REQUIRE(k >= 0 && k <= n && n_sets >= 0, "vr_bootstrap_spearman_f32: bad k");
  VR_REQUIRE(scores != nullptr, "vr_bootstrap_spearman_f32: null scores");
  const EngineCfg cfg = engine_cfg(n);
  const size_t need = oneshot_bytes(n, LANES, cfg.nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_bootstrap_spearman_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView PA, PB;
  PlanBuildWs W;
  EngineWs E;
  oneshot_bytes(n, LANES, cfg.nwaves, ws, &PA, &PB, &W, &E);
  hipStream_t st = as_stream(stream);
  VR_TRY(build_plan(A, n, ld, PA, W, st));
  VR_TRY(build_plan(B, n, ld, PB, W, st));
  return run_engine(PA, PB, n, idx, k, n_sets, full_first, scores, E, LANES, cfg, st);
}

size_t vr_spearman_triu_workspace(int64_t n) {
  n = n < 0 ? 0 : n;
  return oneshot_bytes(n, 1, engine_cfg(n).nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int vr_spearman_triu_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out,
                         void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(n >= 0 && n <= 65535 && ld >= n, "vr_spearman_triu_f32: bad shape n=%lld ld=%lld",
             (long long)n, (long long)ld);
  VR_REQUIRE(out != nullptr, "vr_spearman_triu_f32: null out");
  const EngineCfg cfg = engine_cfg(n);
  const size_t need = oneshot_bytes(n, 1, cfg.nwaves, nullptr, nullptr, nullptr, nullptr, nullptr);
  if (ws_bytes < need || ws == nullptr) {
    set_error("vr_spearman_triu_f32: workspace %zu < %zu", ws_bytes, need);
    return VR_EWORKSPACE;
  }
  PlanView PA, PB;
  PlanBuildWs W;
  EngineWs E;
  oneshot_bytes(n, 1, cfg.nwaves, ws, &PA, &PB, &W, &E);
  hipStream_t st = as_stream(stream);
  VR_TRY(build_plan(A, n, ld, PA, W, st));
  VR_TRY(build_plan(B, n, ld, PB, W, st));
  return run_engine(PA, PB, n, nullptr, 0, 0, 1, out, E, 1, cfg, st);
}

}  // extern "C"
