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

// same bytes with W-byte lanes: each instruction covers 64*W contiguous bytes
template <typename T>
__global__ __launch_bounds__(1024) void store_w(T* tb, uint32_t rows, uint32_t per_wave) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  constexpr uint32_t RPI = sizeof(T) / 2;  // 128-byte rows per instruction
  const uint32_t r0 = wave * per_wave;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; r += RPI) {
    T v;
    __builtin_memset(&v, (int)(r + lane), sizeof(T));
    __builtin_nontemporal_store(v, reinterpret_cast<T*>(reinterpret_cast<char*>(tb) + (size_t)r * 128) + lane);
  }
}

// u16 rows with ALU work between stores (a dependent chain of `work` fmas per row)
__global__ __launch_bounds__(1024) void store_u16_alu(uint16_t* tb, uint32_t rows, uint32_t per_wave,
                                                      int work, float* sink) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  float a = lane * 0.5f;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; ++r) {
    for (int i = 0; i < work; ++i) a = __builtin_fmaf(a, 1.0001f, 0.5f);
    __builtin_nontemporal_store((uint16_t)((uint32_t)a + r), tb + (size_t)r * 64 + lane);
  }
  if (a == 12345.f) sink[0] = a;
}

// wave-specialised: even waves store all the rows (twice the rows each), odd waves only
// run the fma chain (work per row of the full workload)
__global__ __launch_bounds__(1024) void store_split(uint16_t* tb, uint32_t rows, uint32_t per_wave2,
                                                    int work, float* sink) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = (wave >> 1) * per_wave2;
  if ((wave & 1) == 0) {
    for (uint32_t r = r0; r < r0 + per_wave2 && r < rows; ++r)
      __builtin_nontemporal_store((uint16_t)(r + lane), tb + (size_t)r * 64 + lane);
  } else {
    float a = lane * 0.5f;
    for (uint32_t r = r0; r < r0 + per_wave2 && r < rows; ++r)
      for (int i = 0; i < work; ++i) a = __builtin_fmaf(a, 1.0001f, 0.5f);
    if (a == 12345.f) sink[0] = a;
  }
}

// fma chain only (no stores), same per-row work as store_u16_alu
__global__ __launch_bounds__(1024) void alu_only(uint32_t rows, uint32_t per_wave, int work, float* sink) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  float a = lane * 0.5f;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; ++r)
    for (int i = 0; i < work; ++i) a = __builtin_fmaf(a, 1.0001f, 0.5f);
  if (a == 12345.f) sink[0] = a;
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
  for (int grid : {512}) {
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
    run("nt_u16", [&] { store_w<uint16_t><<<grid, 1024>>>(tb, rows, per); });
    run("nt_u32", [&] { store_w<uint32_t><<<grid, 1024>>>((uint32_t*)tb, rows, (per + 1) / 2 * 2); });
    run("nt_u64", [&] { store_w<uint64_t><<<grid, 1024>>>((uint64_t*)tb, rows, (per + 3) / 4 * 4); });
    for (int work : {4, 8})
      run(work == 4 ? "u16+4fma" : "u16+8fma",
          [&] { store_u16_alu<<<grid, 1024>>>(tb, rows, per, work, (float*)out); });
    run("alu8_only", [&] { alu_only<<<grid, 1024>>>(rows, per, 8, (float*)out); });
    run("split8", [&] { store_split<<<grid, 1024>>>(tb, rows, 2 * per, 16, (float*)out); });
    run("gather16", [&] { gather_u16<16><<<grid, 1024>>>(tb, perm, rows, per, out); });
    run("gather32", [&] { gather_u16<32><<<grid, 1024>>>(tb, perm, rows, per, out); });
    run("gather64", [&] { gather_u16<64><<<grid, 1024>>>(tb, perm, rows, per, out); });
    CK(hipFree(out));
  }
  return 0;
}
