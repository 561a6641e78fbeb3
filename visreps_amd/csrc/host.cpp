// Host-side pieces of libvisreps_hip.so:
//  - error reporting and device queries,
//  - the legacy numpy RandomState (MT19937) index stream, bit-exact, which draws the
//    bootstrap / selection subsets (visreps/evals.py:260-261,356,362-364;
//    visreps/analysis/rsa.py:169,176,248-250; evals.py:111-113),
//  - numpy.percentile(.., method='linear') for the bootstrap CI (evals.py:371-372).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

#include "common.h"

namespace vr {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
void clear_error() { g_err[0] = 0; }

int num_cus() {
  static std::mutex mu;
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  std::lock_guard<std::mutex> lk(mu);
  if (cache[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
            hipSuccess ||
        cus <= 0)
      cus = 256;
    cache[dev] = cus;
  }
  return cache[dev];
}

// ---------------------------------------------------------------------------------
// MT19937 as numpy's legacy RandomState uses it: integer seeds go through
// init_genrand (mt19937_seed), 32-bit draws are the standard tempered outputs, and
// bounded integers use masked rejection (legacy random_interval). permutation(n)
// shuffles arange(n) with i running n-1 .. 1, j = interval(i), swap(x[i], x[j]);
// choice(n, k, replace=False) is permutation(n)[:k].
// ---------------------------------------------------------------------------------
struct MTState {
  uint32_t mt[624];
  int pos;
};

static void mt_seed(MTState* s, uint32_t seed) {
  s->mt[0] = seed;
  for (int i = 1; i < 624; ++i)
    s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
  s->pos = 624;
}

static inline uint32_t mt_twist(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return c ^ (y >> 1) ^ (0u - (y & 1u) & 0x9908b0dfu);
}

// the same recurrence as mt[i] = twist(mt[i], mt[(i+1) % 624], mt[(i+397) % 624]) in
// order, split where the indices wrap so the loops carry no modulo
static void mt_regen(MTState* s) {
  uint32_t* mt = s->mt;
  int i = 0;
  for (; i < 624 - 397; ++i) mt[i] = mt_twist(mt[i], mt[i + 1], mt[i + 397]);
  for (; i < 623; ++i) mt[i] = mt_twist(mt[i], mt[i + 1], mt[i + 397 - 624]);
  mt[623] = mt_twist(mt[623], mt[0], mt[396]);
  s->pos = 0;
}

static inline uint32_t mt_next(MTState* s) {
  if (s->pos >= 624) mt_regen(s);
  uint32_t y = s->mt[s->pos++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// Bounded draw in [0, mx] for mx < 2^32 (every caller here bounds n by INT32_MAX).
static inline uint32_t mt_interval(MTState* s, uint32_t mx) {
  if (mx == 0) return 0;
  uint32_t mask = mx;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  uint32_t v;
  while ((v = (mt_next(s) & mask)) > mx) {
  }
  return v;
}

static void mt_permutation(MTState* s, int64_t n, int32_t* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)i;
  for (int64_t i = n - 1; i >= 1; --i) {
    int64_t j = (int64_t)mt_interval(s, (uint32_t)i);
    std::swap(out[i], out[j]);
  }
}

}  // namespace vr

using namespace vr;

extern "C" {

int vr_version(void) { return 100; }

const char* vr_last_error(void) { return g_err; }

size_t vr_rng_state_bytes(void) { return sizeof(MTState); }

int vr_rng_seed(void* state, uint32_t seed) {
  VR_REQUIRE(state != nullptr, "vr_rng_seed: null state");
  mt_seed(static_cast<MTState*>(state), seed);
  return VR_OK;
}

int vr_rng_permutation(void* state, int64_t n, int32_t* out) {
  VR_REQUIRE(state != nullptr && (out != nullptr || n == 0), "vr_rng_permutation: null pointer");
  VR_REQUIRE(n >= 0 && n <= INT32_MAX, "vr_rng_permutation: n=%lld out of range", (long long)n);
  mt_permutation(static_cast<MTState*>(state), n, out);
  return VR_OK;
}

int vr_rng_choice(void* state, int64_t n, int64_t k, int32_t* out) {
  VR_REQUIRE(state != nullptr, "vr_rng_choice: null state");
  VR_REQUIRE(n >= 0 && n <= INT32_MAX, "vr_rng_choice: n=%lld out of range", (long long)n);
  // numpy: "Cannot take a larger sample than population when 'replace=False'"
  VR_REQUIRE(k >= 0 && k <= n, "vr_rng_choice: sample size %lld > population %lld",
             (long long)k, (long long)n);
  std::vector<int32_t> perm((size_t)n);
  mt_permutation(static_cast<MTState*>(state), n, perm.data());
  if (k > 0) std::memcpy(out, perm.data(), (size_t)k * sizeof(int32_t));
  return VR_OK;
}

int vr_rng_random_u32(void* state, int64_t count, uint32_t* out) {
  VR_REQUIRE(state != nullptr && (out != nullptr || count == 0), "vr_rng_random_u32: null pointer");
  MTState* s = static_cast<MTState*>(state);
  for (int64_t i = 0; i < count; ++i) out[i] = mt_next(s);
  return VR_OK;
}

int vr_legacy_choice(uint32_t seed, int64_t n, int64_t k, int64_t n_draws, int32_t* out) {
  VR_REQUIRE(n >= 0 && n <= INT32_MAX && k >= 0 && k <= n && n_draws >= 0,
             "vr_legacy_choice: bad sizes n=%lld k=%lld draws=%lld", (long long)n,
             (long long)k, (long long)n_draws);
  VR_REQUIRE(out != nullptr || n_draws == 0 || k == 0, "vr_legacy_choice: null out");
  MTState s;
  mt_seed(&s, seed);
  const unsigned hw = std::thread::hardware_concurrency();
  const int64_t nt = std::min<int64_t>({(int64_t)(hw ? hw : 1), 16, n_draws});
  if (nt < 2 || n < 1024 || k == 0) {
    std::vector<int32_t> perm((size_t)n);
    for (int64_t d = 0; d < n_draws; ++d) {
      mt_permutation(&s, n, perm.data());
      if (k > 0) std::memcpy(out + d * k, perm.data(), (size_t)k * sizeof(int32_t));
    }
    return VR_OK;
  }
  // Many draws: the stream is split at draw boundaries. A sequential pass replays only the
  // bounded draws' accept/reject decisions (no shuffle; the accept test and the mask update
  // are branch-free), recording the generator state at the start of every draw; threads
  // then run the permutations from those states. Same outputs as the loop above.
  std::vector<MTState> snap((size_t)n_draws);
  for (int64_t d = 0; d < n_draws; ++d) {
    snap[(size_t)d] = s;
    uint32_t i = (uint32_t)(n - 1), mask = i;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t buf[624];
    while (i >= 1) {
      if (s.pos >= 624) mt_regen(&s);
      const int m = 624 - s.pos;
      for (int j = 0; j < m; ++j) {  // tempered outputs of the rest of this block
        uint32_t y = s.mt[s.pos + j];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        buf[j] = y ^ (y >> 18);
      }
      int j = 0;
      for (; j < m && i >= 1; ++j) {
        const uint32_t acc = (buf[j] & mask) <= i;
        i -= acc;
        mask = i <= (mask >> 1) ? mask >> 1 : mask;
      }
      s.pos += j;
    }
  }
  // Worker t draws d = t, t + nt, ...; its scratch is allocated here, so nothing inside a
  // thread can throw. If the system refuses a thread (a container's thread limit), the
  // stride classes not started run on this thread: same outputs, no exception through the
  // C ABI.
  std::vector<std::vector<int32_t>> perm((size_t)nt, std::vector<int32_t>((size_t)n));
  auto work = [&](int64_t t) {
    for (int64_t d = t; d < n_draws; d += nt) {
      MTState local = snap[(size_t)d];
      mt_permutation(&local, n, perm[(size_t)t].data());
      std::memcpy(out + d * k, perm[(size_t)t].data(), (size_t)k * sizeof(int32_t));
    }
  };
  std::vector<std::thread> pool;
  pool.reserve((size_t)nt);
  int64_t started = 0;
  try {
    for (; started < nt; ++started) pool.emplace_back(work, started);
  } catch (const std::system_error&) {
  }
  for (int64_t t = started; t < nt; ++t) work(t);
  for (auto& th : pool) th.join();
  return VR_OK;
}

// numpy.percentile(x, q), method='linear' (numpy/lib/_function_base_impl.py: q/100,
// virtual index (n-1)*q, neighbours floor/floor+1 clipped, gamma = frac, _lerp with
// the b - diff*(1-gamma) branch for gamma >= 0.5). NaN anywhere -> NaN.
double vr_percentile_linear(const double* x, int64_t n, double q) {
  if (n <= 0 || x == nullptr) return std::nan("");
  std::vector<double> v(x, x + n);
  for (double e : v)
    if (std::isnan(e)) return std::nan("");
  std::sort(v.begin(), v.end());
  const double qq = q / 100.0;
  const double vi = (double)(n - 1) * qq;
  int64_t prev, next;
  if (vi >= (double)(n - 1)) {
    prev = next = n - 1;
  } else if (vi < 0) {
    prev = next = 0;
  } else {
    prev = (int64_t)std::floor(vi);
    next = prev + 1;
  }
  const double gamma = vi - std::floor(vi);
  const double a = v[(size_t)prev], b = v[(size_t)next];
  const double diff = b - a;
  if (gamma >= 0.5) return b - diff * (1.0 - gamma);
  return a + diff * gamma;
}

}  // extern "C"
