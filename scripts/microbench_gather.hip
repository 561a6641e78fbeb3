// Random row-gather rates on MI355X for the bootstrap engine's B-side shapes.
// Every pair gathers one row of `64 * sizeof(T)` bytes at a random (permuted) row index,
// lane l reading element l of the row; NB rows in flight per wave.
//   g<T>       : rows of 64 x T, table = ROWS x row bytes (each row read once)
//   g16+base   : the round-1 engine shape: a u16 row + a u32 row of a 2 MB base table
// Also prints FETCH_SIZE-calibration byte counts (one launch of each kernel at the end,
// bracketed by markers in the stdout so a --pmc run can be matched).
// hipcc --offload-arch=gfx950 -O3 scripts/microbench_gather.hip -o scripts/bin/mb_gather
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

// 128 subsets per pass: one u32 (two u16 subsets) per lane of a 256-B TB row and one u64
// (two u32 subsets) per lane of a 512-B chunk-base row
template <int NB>
__global__ __launch_bounds__(1024) void gather2(const uint32_t* __restrict__ tb, const uint32_t* __restrict__ perm,
                                                const uint2* __restrict__ base, uint32_t nbase,
                                                uint32_t rows, uint32_t per_wave, uint32_t* out) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  uint32_t acc = 0;
  for (uint32_t r = r0; r < r0 + per_wave; r += 64) {
    const uint32_t pr = (r + lane < rows) ? perm[r + lane] : 0u;
#pragma unroll
    for (int h = 0; h < 64; h += NB) {
      uint32_t v[NB];
      uint2 b[NB];
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        const uint32_t row = (uint32_t)__builtin_amdgcn_readlane((int)pr, h + t);
        v[t] = tb[(size_t)row * 64 + lane];
        b[t] = base[(size_t)(row % nbase) * 64 + lane];
      }
#pragma unroll
      for (int t = 0; t < NB; ++t) acc += (v[t] & 0xffff) + (v[t] >> 16) + b[t].x + b[t].y;
    }
  }
  out[wave * 64 + lane] = acc;
}

template <typename T, int NB, bool BASE>
__global__ __launch_bounds__(1024) void gather(const T* __restrict__ tb, const uint32_t* __restrict__ perm,
                                               const uint32_t* __restrict__ base, uint32_t nbase,
                                               uint32_t rows, uint32_t per_wave, uint32_t* out) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  uint32_t acc = 0;
  for (uint32_t r = r0; r < r0 + per_wave; r += 64) {
    const uint32_t pr = (r + lane < rows) ? perm[r + lane] : 0u;
#pragma unroll
    for (int h = 0; h < 64; h += NB) {
      uint32_t v[NB], b[NB];
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        const uint32_t row = (uint32_t)__builtin_amdgcn_readlane((int)pr, h + t);
        v[t] = (uint32_t)tb[(size_t)row * 64 + lane];
        if (BASE) b[t] = base[(size_t)(row % nbase) * 64 + lane];
      }
#pragma unroll
      for (int t = 0; t < NB; ++t) acc += v[t] + (BASE ? b[t] : 0u);
    }
  }
  out[wave * 64 + lane] = acc;
}

template <typename T>
__global__ void fill(T* tb, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    tb[i] = (T)(i * 2654435761u);
}

int main(int argc, char** argv) {
  const uint32_t pairs = 50000000;  // M at N = 10k
  const int grid = 512;             // 2 blocks of 16 waves per CU
  const uint32_t waves = grid * 16;
  const uint32_t per = ((pairs + waves - 1) / waves + 63) / 64 * 64;
  const bool once = argc > 1 && strcmp(argv[1], "once") == 0;  // one launch each (for --pmc)
  void* tb;
  uint32_t *perm, *out, *base;
  const size_t max_bytes = (size_t)pairs * 256;  // u32 rows, one per pair
  CK(hipMalloc(&tb, max_bytes));
  CK(hipMalloc(&perm, (size_t)pairs * 4));
  CK(hipMalloc(&out, (size_t)waves * 64 * 4));
  const uint32_t nbase = 8138;  // 2 MB of 256-B base rows (round-1 chunk table at N=10k)
  CK(hipMalloc(&base, (size_t)nbase * 512));
  fill<uint32_t><<<4096, 256>>>((uint32_t*)tb, max_bytes / 4);
  fill<uint32_t><<<64, 256>>>(base, (size_t)nbase * 64);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<uint32_t> h(pairs);
  auto make_perm = [&](uint32_t rows) -> int {
    uint64_t s = 88172645463325252ull;
    for (uint32_t i = 0; i < pairs; ++i) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      h[i] = (uint32_t)(s % rows);
    }
    CK(hipMemcpy(perm, h.data(), (size_t)pairs * 4, hipMemcpyHostToDevice));
    return 0;
  };
  auto run = [&](const char* name, double bytes_per_pair, auto launch) -> int {
    if (once) {
      printf("@@ %s\n", name);
      fflush(stdout);
      launch();
      CK(hipDeviceSynchronize());
      printf("@@ %s algorithmic bytes %.0f\n", name, bytes_per_pair * pairs);
      return 0;
    }
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < 5; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 5;
    printf("%-22s %8.3f ms  %7.2f TB/s (row bytes x pairs)\n", name, ms, bytes_per_pair * pairs / (ms * 1e9));
    return 0;
  };
  // u16 rows: 50M-row table (6.4 GB), each pair a random row
  if (make_perm(pairs)) return 1;
  run("g16 NB8", 128, [&] { gather<uint16_t, 8, false><<<grid, 1024>>>((uint16_t*)tb, perm, base, nbase, pairs, per, out); });
  run("g16 NB16", 128, [&] { gather<uint16_t, 16, false><<<grid, 1024>>>((uint16_t*)tb, perm, base, nbase, pairs, per, out); });
  run("g16+base NB8", 128, [&] { gather<uint16_t, 8, true><<<grid, 1024>>>((uint16_t*)tb, perm, base, nbase, pairs, per, out); });
  // u32 rows (256 B): 50M-row table (12.8 GB) -- absolute ranks, one gather per pair
  run("g32 NB8", 256, [&] { gather<uint32_t, 8, false><<<grid, 1024>>>((uint32_t*)tb, perm, base, nbase, pairs, per, out); });
  run("g32 NB16", 256, [&] { gather<uint32_t, 16, false><<<grid, 1024>>>((uint32_t*)tb, perm, base, nbase, pairs, per, out); });
  run("g32+base NB8", 256, [&] { gather<uint32_t, 8, true><<<grid, 1024>>>((uint32_t*)tb, perm, base, nbase, pairs, per, out); });
  run("g32x2+base64 NB8 (4 MB base)", 256, [&] { gather2<8><<<grid, 1024>>>((uint32_t*)tb, perm, (uint2*)base, nbase, pairs, per, out); });
  run("g32x2+base64 NB4 (4 MB base)", 256, [&] { gather2<4><<<grid, 1024>>>((uint32_t*)tb, perm, (uint2*)base, nbase, pairs, per, out); });
  run("g32x2+base64 NB8 (2 MB base)", 256, [&] { gather2<8><<<grid, 1024>>>((uint32_t*)tb, perm, (uint2*)base, nbase / 2, pairs, per, out); });
  // u64 rows (512 B) over the same 12.8 GB: 25M rows
  if (make_perm(pairs / 2)) return 1;
  run("g64 NB8 (25M rows)", 512, [&] { gather<uint64_t, 8, false><<<grid, 1024>>>((uint64_t*)tb, perm, base, nbase, pairs, per, out); });
  return 0;
}
