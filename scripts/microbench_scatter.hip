// Row-write rates on MI355X for the bootstrap engine's A-side shapes: every pair writes one
// 128-byte TB row (64 lanes x u16) either at its own position (sequential, the A-order TB)
// or at a random permuted row (the triangle-order TB an A walk in A order would scatter).
// Also the same random rows read back (the B walk's gather) for reference.
// hipcc --offload-arch=gfx950 -O3 scripts/microbench_scatter.hip -o scripts/bin/mb_scatter
#include <hip/hip_runtime.h>

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

template <bool RANDOM, bool NT>
__global__ __launch_bounds__(1024) void scatter(uint16_t* __restrict__ tb, const uint32_t* __restrict__ perm,
                                                uint32_t rows, uint32_t per_wave) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; r += 64) {
    const uint32_t pr = (r + lane < rows) ? (RANDOM ? perm[r + lane] : r + lane) : 0xffffffffu;
#pragma unroll 8
    for (int j = 0; j < 64; ++j) {
      const uint32_t row = (uint32_t)__builtin_amdgcn_readlane((int)pr, j);
      if (row == 0xffffffffu) break;
      uint16_t* p = tb + (size_t)row * 64 + lane;
      const uint16_t v = (uint16_t)(row + lane);
      if (NT)
        __builtin_nontemporal_store(v, p);
      else
        *p = v;
    }
  }
}

template <int NB>
__global__ __launch_bounds__(1024) void gather(const uint16_t* __restrict__ tb, const uint32_t* __restrict__ perm,
                                               uint32_t rows, uint32_t per_wave, uint32_t* out) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  uint32_t acc = 0;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; r += 64) {
    const uint32_t pr = (r + lane < rows) ? perm[r + lane] : 0u;
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

// the same gather with narrower rows: T per lane (u8: 64-B rows, u16x2 per lane pair: 32-B
// rows read by 16 lanes as u16) -- what a u8-residue TB would cost
template <int NB, typename T, int ROWB>
__global__ __launch_bounds__(1024) void gather_n(const uint8_t* __restrict__ tb, const uint32_t* __restrict__ perm,
                                                 uint32_t rows, uint32_t per_wave, uint32_t* out) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  constexpr uint32_t LPR = ROWB / sizeof(T);  // lanes per row
  uint32_t acc = 0;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; r += 64) {
    const uint32_t pr = (r + lane < rows) ? perm[r + lane] : 0u;
#pragma unroll
    for (int h = 0; h < 64; h += NB) {
      T v[NB];
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        const uint32_t row = (uint32_t)__builtin_amdgcn_readlane((int)pr, h + t);
        v[t] = __builtin_nontemporal_load((const T*)(tb + (size_t)row * ROWB) + (lane % LPR));
      }
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        if constexpr (sizeof(T) == 8)
          acc += (uint32_t)v[t] ^ (uint32_t)(v[t] >> 32);
        else
          acc += v[t];
      }
    }
  }
  out[wave * 64 + lane] = acc;
}

// sequential TB writes with 16-B stores per lane: one instruction writes 8 rows (1 KB)
template <bool NT>
__global__ __launch_bounds__(1024) void write_x4(uint16_t* __restrict__ tb, uint32_t rows, uint32_t per_wave) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; r += 64) {
#pragma unroll
    for (int j = 0; j < 64; j += 8) {
      if (r + j + 8 > rows) break;
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      u32x4* p = reinterpret_cast<u32x4*>(tb + (size_t)(r + j) * 64) + lane;
      const u32x4 v = {r + lane, r + j, lane, (uint32_t)j};
      if (NT)
        __builtin_nontemporal_store(v, p);
      else
        *p = v;
    }
  }
}

// the gather with the B walk's two 4-B streams per pair (codes, A positions) read
// sequentially beside it: the rows come from the streamed positions, as in k_rankB
template <int NB>
__global__ __launch_bounds__(1024) void gather_streams(const uint16_t* __restrict__ tb, const uint32_t* __restrict__ perm,
                                                       const uint32_t* __restrict__ codes, uint32_t rows,
                                                       uint32_t per_wave, uint32_t* out) {
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t r0 = wave * per_wave;
  uint32_t acc = 0;
  for (uint32_t r = r0; r < r0 + per_wave && r < rows; r += 64) {
    const uint32_t pr = (r + lane < rows) ? perm[r + lane] : 0u;
    const uint32_t cd = (r + lane < rows) ? codes[r + lane] : 0u;
    acc ^= cd;
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

int main() {
  const uint32_t rows = 49995000u;  // M at N = 10k
  std::vector<uint32_t> h(rows);
  for (uint32_t i = 0; i < rows; ++i) h[i] = i;
  uint64_t s = 88172645463325252ull;
  for (uint32_t i = rows - 1; i > 0; --i) {  // Fisher-Yates with xorshift
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    const uint32_t j = (uint32_t)(s % (i + 1));
    std::swap(h[i], h[j]);
  }
  uint16_t* tb;
  uint32_t *perm, *out;
  CK(hipMalloc(&tb, (size_t)rows * 512));  // room for the 512-B row gathers
  CK(hipMalloc(&perm, (size_t)rows * 4));
  CK(hipMalloc(&out, (size_t)1 << 24));
  CK(hipMemcpy(perm, h.data(), (size_t)rows * 4, hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 2, waves = grid * 16;
  const uint32_t per_wave = ((rows + waves - 1) / waves + 63) / 64 * 64;
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
    printf("%-28s %8.3f ms  %6.2f TB/s (128 B x rows)\n", name, ms, (double)rows * 128 / (ms * 1e-3) / 1e12);
    return 0;
  };
  if (run("write seq", [&] { scatter<false, true><<<grid, 1024>>>(tb, perm, rows, per_wave); })) return 1;
  if (run("write seq (default policy)", [&] { scatter<false, false><<<grid, 1024>>>(tb, perm, rows, per_wave); })) return 1;
  if (run("write random", [&] { scatter<true, true><<<grid, 1024>>>(tb, perm, rows, per_wave); })) return 1;
  if (run("write random (default)", [&] { scatter<true, false><<<grid, 1024>>>(tb, perm, rows, per_wave); })) return 1;
  if (run("gather random NB8", [&] { gather<8><<<grid, 1024>>>(tb, perm, rows, per_wave, out); })) return 1;
  if (run("gather random NB16", [&] { gather<16><<<grid, 1024>>>(tb, perm, rows, per_wave, out); })) return 1;
  if (run("write seq x4 (16 B/lane)", [&] { write_x4<false><<<grid, 1024>>>(tb, rows, per_wave); })) return 1;
  if (run("write seq x4 NT", [&] { write_x4<true><<<grid, 1024>>>(tb, rows, per_wave); })) return 1;
  uint32_t* codes2;
  CK(hipMalloc(&codes2, (size_t)rows * 4));
  CK(hipMemset(codes2, 1, (size_t)rows * 4));
  if (run("gather random + 2 streams NB8", [&] { gather_streams<8><<<grid, 1024>>>(tb, perm, codes2, rows, per_wave, out); })) return 1;
  if (run("gather random + 2 streams NB16", [&] { gather_streams<16><<<grid, 1024>>>(tb, perm, codes2, rows, per_wave, out); })) return 1;
  auto gb = [&](auto k) { k<<<grid, 1024>>>((const uint8_t*)tb, perm, rows, per_wave, out); };
  if (run("gather random 64B u8 NB16", [&] { gb(gather_n<16, uint8_t, 64>); })) return 1;
  if (run("gather random 64B u16 NB16", [&] { gb(gather_n<16, uint16_t, 64>); })) return 1;
  if (run("gather random 32B u8 NB16", [&] { gb(gather_n<16, uint8_t, 32>); })) return 1;
  if (run("gather random 128B u16 NB16", [&] { gb(gather_n<16, uint16_t, 128>); })) return 1;
  // wider rows: two / four passes' subsets per row (u32 / u64 per lane)
  if (run("gather random 256B u32 NB16", [&] { gb(gather_n<16, uint32_t, 256>); })) return 1;
  if (run("gather random 256B u32 NB8", [&] { gb(gather_n<8, uint32_t, 256>); })) return 1;
  if (run("gather random 512B u64 NB8", [&] { gb(gather_n<8, uint64_t, 512>); })) return 1;
  return 0;
}
