// Is k_rankB's gap to the random-row floor the access ORDER of a real B walk or the walk's
// own instruction stream? The same plain 128-B row gather (scripts/microbench_scatter.hip's
// `gather`, 32 waves per CU, 8 loads in flight per wave) over the TB-sized buffer, with the
// rows taken in three orders:
//   walk   : a real unit's A positions in B order (posA_byB of a bench unit, from a file
//            written by scripts/probe_walk_order.py),
//   random : a uniform random permutation (the microbench's order),
//   seq    : ascending rows.
// plus the walk order with the B walk's two 4-B streams and an 80-KB LDS table per
// workgroup (the engine's mask table: 2 workgroups per CU).
// hipcc --offload-arch=gfx950 -O3 scripts/microbench_walk.hip -o scripts/bin/mb_walk
// usage: mb_walk <posA.bin>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

template <int NB, bool STREAMS, bool LDSTAB>
__global__ __launch_bounds__(1024) void gather(const uint16_t* __restrict__ tb, const uint32_t* __restrict__ order,
                                               const uint32_t* __restrict__ codes, uint32_t rows, uint32_t per_wave,
                                               uint32_t* out) {
  extern __shared__ uint64_t tab[];
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if constexpr (LDSTAB) {
    for (uint32_t i = threadIdx.x; i < 10000; i += 1024) tab[i] = i * 0x9E3779B97F4A7C15ull;
    __syncthreads();
  }
  const uint32_t r0 = wave * per_wave;
  uint32_t acc = 0;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; r += 64) {
    const uint32_t pr = (r + lane < rows) ? order[r + lane] : 0u;
    if constexpr (STREAMS) {
      const uint32_t cd = (r + lane < rows) ? codes[r + lane] : 0u;
      if constexpr (LDSTAB) {
        acc ^= (uint32_t)(tab[(cd >> 16) % 10000u] & tab[(cd & 0xffffu) % 10000u]);
      } else {
        acc ^= cd;
      }
    }
#pragma unroll
    for (int h = 0; h < 64; h += NB) {
      uint32_t v[NB];
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        const uint32_t row = (uint32_t)__builtin_amdgcn_readlane((int)pr, h + t);
        v[t] = __builtin_nontemporal_load(tb + (size_t)row * 64 + lane);
      }
#pragma unroll
      for (int t = 0; t < NB; ++t) acc += v[t];
    }
  }
  out[wave * 64 + lane] = acc;
}

int main(int argc, char** argv) {
  std::vector<uint32_t> walk;
  if (argc > 1) {
    FILE* f = fopen(argv[1], "rb");
    if (!f) {
      printf("cannot open %s\n", argv[1]);
      return 1;
    }
    fseek(f, 0, SEEK_END);
    const long bytes = ftell(f);
    fseek(f, 0, SEEK_SET);
    walk.resize((size_t)bytes / 4);
    if (fread(walk.data(), 4, walk.size(), f) != walk.size()) return 1;
    fclose(f);
  }
  const uint32_t rows = walk.empty() ? 49995000u : (uint32_t)walk.size();
  std::vector<uint32_t> rnd(rows), seq(rows);
  for (uint32_t i = 0; i < rows; ++i) rnd[i] = seq[i] = i;
  uint64_t s = 88172645463325252ull;
  for (uint32_t i = rows - 1; i > 0; --i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    std::swap(rnd[i], rnd[(uint32_t)(s % (i + 1))]);
  }
  if (walk.empty()) walk = rnd;
  uint32_t mx = 0;
  for (uint32_t v : walk) mx = std::max(mx, v);
  printf("rows %u, max walk row %u\n", rows, mx);
  uint16_t* tb;
  uint32_t *d_walk, *d_rnd, *d_seq, *codes, *out;
  CK(hipMalloc(&tb, (size_t)rows * 128));
  CK(hipMemset(tb, 1, (size_t)rows * 128));
  CK(hipMalloc(&d_walk, (size_t)rows * 4));
  CK(hipMalloc(&d_rnd, (size_t)rows * 4));
  CK(hipMalloc(&d_seq, (size_t)rows * 4));
  CK(hipMalloc(&codes, (size_t)rows * 4));
  CK(hipMalloc(&out, (size_t)1 << 24));
  CK(hipMemcpy(d_walk, walk.data(), (size_t)rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rnd, rnd.data(), (size_t)rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_seq, seq.data(), (size_t)rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(codes, rnd.data(), (size_t)rows * 4, hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 2, waves = grid * 16;
  const uint32_t per_wave = ((rows + waves - 1) / waves + 63) / 64 * 64;
  CK(hipFuncSetAttribute((const void*)gather<8, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 80000));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) -> int {
    for (int w = 0; w < 2; ++w) launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-40s %8.3f ms  %6.2f TB/s (128 B x rows)\n", name, ms, (double)rows * 128 / (ms * 1e-3) / 1e12);
    return 0;
  };
  if (run("gather seq", [&] { gather<8, false, false><<<grid, 1024>>>(tb, d_seq, codes, rows, per_wave, out); })) return 1;
  if (run("gather random", [&] { gather<8, false, false><<<grid, 1024>>>(tb, d_rnd, codes, rows, per_wave, out); })) return 1;
  if (run("gather walk order", [&] { gather<8, false, false><<<grid, 1024>>>(tb, d_walk, codes, rows, per_wave, out); })) return 1;
  if (run("gather walk + streams", [&] { gather<8, true, false><<<grid, 1024>>>(tb, d_walk, codes, rows, per_wave, out); })) return 1;
  if (run("gather walk + streams + LDS table", [&] {
        gather<8, true, true><<<grid, 1024, 80000>>>(tb, d_walk, codes, rows, per_wave, out);
      })) return 1;
  if (run("gather random + streams + LDS table", [&] {
        gather<8, true, true><<<grid, 1024, 80000>>>(tb, d_rnd, codes, rows, per_wave, out);
      })) return 1;
  return 0;
}
