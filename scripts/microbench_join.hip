// The shared join (k_join4) in three shapes, on MI355X, at M = 49,995,000 pairs (N = 10k):
//   G4   gather: B order, t = perm_inv[i], 16-B record pm4[t] -> 4 separate 4-B outputs [i]
//        (today's k_join4)
//   G16  gather, one interleaved 16-B output record per B position
//   S16  scatter: triangle order, p = perm[t] (the B plan's pos_map), pm4[t] (sequential)
//        -> one 16-B record at out4[p] (random 16-B stores)
//   S4   scatter into 4 separate 4-B outputs (random 4-B stores)
// perm is a random permutation (host std::mt19937_64 Fisher-Yates). Times from hipEvents
// over REPS launches; run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE for the bytes.
// hipcc --offload-arch=gfx950 -O3 scripts/microbench_join.hip -o scripts/bin/mb_join
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

__global__ void g4(const uint32_t* __restrict__ inv, const uint4* __restrict__ pm4, uint32_t M,
                   uint32_t* __restrict__ o0, uint32_t* __restrict__ o1, uint32_t* __restrict__ o2,
                   uint32_t* __restrict__ o3) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint4 r = pm4[__builtin_nontemporal_load(inv + i)];
  __builtin_nontemporal_store(r.x, o0 + i);
  __builtin_nontemporal_store(r.y, o1 + i);
  __builtin_nontemporal_store(r.z, o2 + i);
  __builtin_nontemporal_store(r.w, o3 + i);
}

__global__ void g16(const uint32_t* __restrict__ inv, const uint4* __restrict__ pm4, uint32_t M,
                    uint4* __restrict__ o) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint4 r = pm4[__builtin_nontemporal_load(inv + i)];
  const v4u v = {r.x, r.y, r.z, r.w};
  __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(o + i));
}

template <bool NT>
__global__ void s16(const uint32_t* __restrict__ perm, const uint4* __restrict__ pm4, uint32_t M,
                    uint4* __restrict__ o) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M) return;
  const uint32_t p = __builtin_nontemporal_load(perm + t);
  const v4u r = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(pm4) + t);
  if (NT)
    __builtin_nontemporal_store(r, reinterpret_cast<v4u*>(o) + p);
  else
    reinterpret_cast<v4u*>(o)[p] = r;
}

__global__ void s4(const uint32_t* __restrict__ perm, const uint4* __restrict__ pm4, uint32_t M,
                   uint32_t* __restrict__ o0, uint32_t* __restrict__ o1, uint32_t* __restrict__ o2,
                   uint32_t* __restrict__ o3) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M) return;
  const uint32_t p = __builtin_nontemporal_load(perm + t);
  const v4u r = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(pm4) + t);
  o0[p] = r.x;
  o1[p] = r.y;
  o2[p] = r.z;
  o3[p] = r.w;
}

// the consumer side: read the 4 positions per B position from 4 arrays or one record
__global__ void rd4(const uint32_t* __restrict__ a0, const uint32_t* __restrict__ a1,
                    const uint32_t* __restrict__ a2, const uint32_t* __restrict__ a3, uint32_t M,
                    uint32_t* __restrict__ sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t v = a0[i] ^ a1[i] ^ a2[i] ^ a3[i];
  if (v == 0x9e3779b9u) sink[0] = i;
}
__global__ void rd16(const uint4* __restrict__ a, uint32_t M, uint32_t* __restrict__ sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint4 r = a[i];
  const uint32_t v = r.x ^ r.y ^ r.z ^ r.w;
  if (v == 0x9e3779b9u) sink[0] = i;
}

int main(int argc, char** argv) {
  const uint32_t M = argc > 1 ? (uint32_t)atoll(argv[1]) : 49995000u;
  const int REPS = argc > 2 ? atoi(argv[2]) : 10;
  std::vector<uint32_t> perm(M), inv(M);
  for (uint32_t i = 0; i < M; ++i) perm[i] = i;
  std::mt19937_64 rng(12345);
  for (uint32_t i = M - 1; i > 0; --i) {
    const uint32_t j = (uint32_t)(rng() % (uint64_t)(i + 1));
    std::swap(perm[i], perm[j]);
  }
  for (uint32_t t = 0; t < M; ++t) inv[perm[t]] = t;
  std::vector<uint4> pm(M);
  for (uint32_t t = 0; t < M; ++t) pm[t] = make_uint4(t, t ^ 0x55555555u, t * 3u, ~t);
  uint32_t *dperm, *dinv, *o[4], *sink;
  uint4 *dpm, *o4;
  CK(hipMalloc(&dperm, (size_t)M * 4));
  CK(hipMalloc(&dinv, (size_t)M * 4));
  CK(hipMalloc(&dpm, (size_t)M * 16));
  CK(hipMalloc(&o4, (size_t)M * 16));
  for (int a = 0; a < 4; ++a) CK(hipMalloc(&o[a], (size_t)M * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMemcpy(dperm, perm.data(), (size_t)M * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dinv, inv.data(), (size_t)M * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpm, pm.data(), (size_t)M * 16, hipMemcpyHostToDevice));
  const unsigned grid = (M + 255) / 256;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto&& launch) -> int {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < REPS; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / REPS;
    printf("%-5s %9.1f us  %6.2f TB/s on %.0f B/pair\n", name, us, bytes * M / (us * 1e-6) / 1e12, bytes);
    return 0;
  };
  if (timeit("G4", 36, [&] { g4<<<grid, 256>>>(dinv, dpm, M, o[0], o[1], o[2], o[3]); })) return 1;
  if (timeit("G16", 36, [&] { g16<<<grid, 256>>>(dinv, dpm, M, o4); })) return 1;
  if (timeit("S16", 36, [&] { s16<false><<<grid, 256>>>(dperm, dpm, M, o4); })) return 1;
  if (timeit("S16nt", 36, [&] { s16<true><<<grid, 256>>>(dperm, dpm, M, o4); })) return 1;
  if (timeit("S4", 36, [&] { s4<<<grid, 256>>>(dperm, dpm, M, o[0], o[1], o[2], o[3]); })) return 1;
  if (timeit("RD4", 16, [&] { rd4<<<grid, 256>>>(o[0], o[1], o[2], o[3], M, sink); })) return 1;
  if (timeit("RD16", 16, [&] { rd16<<<grid, 256>>>(o4, M, sink); })) return 1;
  // check: S16's record at p is pm4[inv[p]] (G16's)
  std::vector<uint4> h(M);
  s16<false><<<grid, 256>>>(dperm, dpm, M, o4);
  CK(hipMemcpy(h.data(), o4, (size_t)M * 16, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (uint32_t p = 0; p < M; ++p) bad += h[p].x != inv[p];
  printf("S16 check: %zu mismatches\n", bad);
  return bad != 0;
}
