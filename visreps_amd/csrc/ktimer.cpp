// Kernel-level HIP-event timing of the hot kernels (vr_ktimer_*; declared in
// include/visreps_hip.h). Used by bench.py to price the dominant kernel against its
// roofline on the stream it runs on: one event pair per launch, resolved on read.
#include <mutex>
#include <vector>

#include "internal.h"

namespace vr {
namespace {
struct Rec {
  int kernel;
  double units;
  hipEvent_t e0, e1;
};
std::mutex g_mu;
bool g_on = false;
std::vector<Rec> g_pending;
std::vector<hipEvent_t> g_pool;
double g_ms[KT_N] = {};
double g_units[KT_N] = {};
int64_t g_launches[KT_N] = {};

hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

int resolve_locked() {
  int rc = VR_OK;
  for (const Rec& r : g_pending) {
    float ms = 0.f;
    if (hipEventSynchronize(r.e1) != hipSuccess || hipEventElapsedTime(&ms, r.e0, r.e1) != hipSuccess) {
      rc = VR_EHIP;
    } else {
      g_ms[r.kernel] += ms;
      g_units[r.kernel] += r.units;
      g_launches[r.kernel] += 1;
    }
    g_pool.push_back(r.e0);
    g_pool.push_back(r.e1);
  }
  g_pending.clear();
  return rc;
}
}  // namespace

bool ktimer_on() { return g_on; }

KtScope::KtScope(int k, double u, hipStream_t s) : kernel(k), units(u), st(s) {
  if (!g_on) return;
  std::lock_guard<std::mutex> lk(g_mu);
  e0 = take_event();
  if (e0 && hipEventRecord(e0, st) != hipSuccess) e0 = nullptr;
}

KtScope::~KtScope() {
  if (!e0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t e1 = take_event();
  if (e1 && hipEventRecord(e1, st) == hipSuccess)
    g_pending.push_back(Rec{kernel, units, e0, e1});
  else
    g_pool.push_back(e0);
}

}  // namespace vr

using namespace vr;

extern "C" {

int vr_ktimer_enable(int on) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int rc = resolve_locked();
  for (int k = 0; k < KT_N; ++k) g_ms[k] = g_units[k] = 0.0, g_launches[k] = 0;
  g_on = on != 0;
  return rc;
}

int vr_ktimer_read(int kernel, double* ms, int64_t* launches, double* units) {
  if (kernel < 0 || kernel >= KT_N || !ms || !launches || !units) {
    set_error("vr_ktimer_read: bad kernel id %d or null output", kernel);
    return VR_EINVAL;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  const int rc = resolve_locked();
  *ms = g_ms[kernel];
  *launches = g_launches[kernel];
  *units = g_units[kernel];
  return rc;
}

}  // extern "C"
