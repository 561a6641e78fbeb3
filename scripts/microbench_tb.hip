// Microbenchmark for the bootstrap engine's rank-table (TB) traffic shapes on MI355X.
//   store_u16   : wave writes consecutive 128-byte rows, one global_store_short per row
//   store_x4    : same bytes, 16 B per lane (global_store_dwordx4), 1 KB per instruction
//   gather_u16  : wave reads 128-byte rows at random row indices (u16 per lane), NB loads
//                 in flight per wave, sums them
// hipcc --offload-arch=gfx950 -O3 scripts/microbench_tb.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);     \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ __launch_bounds__(1024) void store_u16(uint16_t* tb, uint32_t rows, uint32_t per_wave) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; ++r) tb[(size_t)r * 64 + lane] = (uint16_t)(r + lane);
}

// as store_u16 but the wave drains its stores every 64 rows (s_waitcnt vmcnt(0)), and
// only the first `active` waves work
__global__ __launch_bounds__(1024) void store_u16_drain(uint16_t* tb, uint32_t rows, uint32_t per_wave,
                                                        uint32_t active, int drain) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wave >= active) return;
  const uint32_t r0 = wave * per_wave;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; ++r) {
    tb[(size_t)r * 64 + lane] = (uint16_t)(r + lane);
    if (drain && (r & 63) == 63) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

__global__ __launch_bounds__(1024) void store_x4(uint4* tb, uint32_t rows, uint32_t per_wave) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;  // rows of 128 B; 8 rows per 1 KB instruction
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; r += 8)
    tb[((size_t)r * 128) / 16 + lane] = make_uint4(r, lane, r ^ lane, 7);
}

template <int NB>
__global__ __launch_bounds__(1024) void gather_u16(const uint16_t* tb, const uint32_t* perm,
                                                   uint32_t rows, uint32_t per_wave, uint32_t* out) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  uint32_t acc = 0;
  for (uint32_t r = r0; r + NB <= r0 + per_wave && r + NB <= rows; r += NB) {
    const uint32_t pr = perm[r + (lane % NB)];
    uint32_t v[NB];
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const uint32_t row = __builtin_amdgcn_readlane(pr, t);
      v[t] = tb[(size_t)row * 64 + lane];
    }
#pragma unroll
    for (int t = 0; t < NB; ++t) acc += v[t];
  }
  out[wave * 64 + lane] = acc;
}

int main() {
  const uint32_t rows = 50000000;  // M at N = 10k
  const size_t bytes = (size_t)rows * 128;
  uint16_t* tb;
  uint32_t *perm, *out;
  CK(hipMalloc(&tb, bytes));
  CK(hipMalloc(&perm, (size_t)rows * 4));
  std::vector<uint32_t> h(rows);
  uint64_t s = 88172645463325252ull;
  for (uint32_t i = 0; i < rows; ++i) h[i] = i;
  for (uint32_t i = rows - 1; i > 0; --i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    std::swap(h[i], h[s % (i + 1)]);
  }
  CK(hipMemcpy(perm, h.data(), (size_t)rows * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int grid : {256, 512, 1024}) {
    const uint32_t waves = grid * 16, per = (rows + waves - 1) / waves;
    CK(hipMalloc(&out, (size_t)waves * 64 * 4));
    auto run = [&](const char* name, auto launch) -> int {
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      for (int i = 0; i < 5; ++i) launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= 5;
      printf("grid %5d %-14s %8.3f ms  %7.2f TB/s\n", grid, name, ms, bytes / (ms * 1e9));
      return 0;
    };
    run("store_u16", [&] { store_u16<<<grid, 1024>>>(tb, rows, per); });
    const uint32_t act = waves * 3 / 4, per_act = (rows + act - 1) / act;
    run("u16_3/4waves", [&] { store_u16_drain<<<grid, 1024>>>(tb, rows, per_act, act, 0); });
    run("u16_drain64", [&] { store_u16_drain<<<grid, 1024>>>(tb, rows, per, waves, 1); });
    run("u16_3/4+drain", [&] { store_u16_drain<<<grid, 1024>>>(tb, rows, per_act, act, 1); });
    run("store_x4", [&] { store_x4<<<grid, 1024>>>((uint4*)tb, rows, (per + 7) / 8 * 8); });
    run("gather16", [&] { gather_u16<16><<<grid, 1024>>>(tb, perm, rows, per, out); });
    run("gather32", [&] { gather_u16<32><<<grid, 1024>>>(tb, perm, rows, per, out); });
    run("gather64", [&] { gather_u16<64><<<grid, 1024>>>(tb, perm, rows, per, out); });
    CK(hipFree(out));
  }
  return 0;
}
