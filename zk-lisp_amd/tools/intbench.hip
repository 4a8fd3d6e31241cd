// Integer VALU microbenchmarks on gfx950: throughput of the instructions the f128
// field arithmetic is built from, and of the full Poseidon permutation (round-1 numbers:
// profiles/r01/intbench.txt).  bench.py's VALU ceiling now comes from the per-class rates of
// tools/madbench.hip and the row hash's own instruction mix (tools/valu_mix.py).
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdio.h>
#include <stdint.h>
#include <chrono>
#include "../csrc/field.h"
using namespace zkl;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_mad64(uint64_t* out, uint32_t a, uint32_t b) {
  uint64_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = threadIdx.x + i;
  uint32_t x = a + threadIdx.x, y = b;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (uint64_t)(x + i) * y + acc[i];
    y += 1;
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mullo(uint32_t* out, uint32_t a, uint32_t b) {
  uint32_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = acc[i] * (a + i) + b;
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_add(uint32_t* out, uint32_t a) {
  uint32_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (acc[i] ^ a) + i;
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fmul(fe* out, fe a) {
  fe acc[4];
  for (int i = 0; i < 4; i++) acc[i] = fe{threadIdx.x + (uint64_t)i, (uint64_t)blockIdx.x};
  for (int it = 0; it < ITERS / 16; it++) {
#pragma unroll
    for (int i = 0; i < 4; i++) acc[i] = fe_mul(acc[i], a);
  }
  fe s = acc[0];
  for (int i = 1; i < 4; i++) s = fe_add(s, acc[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// launch f once to warm up, then time 5 launches; any HIP failure aborts the benchmark
#define MUST(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
template <class F>
double timeit(F f) {
  hipEvent_t a, b;
  MUST(hipEventCreate(&a));
  MUST(hipEventCreate(&b));
  f();
  MUST(hipGetLastError());
  MUST(hipDeviceSynchronize());
  MUST(hipEventRecord(a));
  for (int i = 0; i < 5; i++) f();
  MUST(hipEventRecord(b));
  MUST(hipEventSynchronize(b));
  float ms = 0;
  MUST(hipEventElapsedTime(&ms, a, b));
  MUST(hipEventDestroy(a));
  MUST(hipEventDestroy(b));
  return ms / 5;
}

int main() {
  const int blocks = 256 * 32, threads = 256;
  size_t nthr = (size_t)blocks * threads;
  void* d;
  CHECK(hipMalloc(&d, nthr * 16));
  double ms;
  ms = timeit([&] { k_mad64<<<blocks, threads>>>((uint64_t*)d, 3, 5); });
  printf("{\"op\":\"v_mad_u64_u32\",\"G_per_s\":%.1f}\n", nthr * (double)ITERS * 8 / ms / 1e6);
  ms = timeit([&] { k_mullo<<<blocks, threads>>>((uint32_t*)d, 3, 5); });
  printf("{\"op\":\"v_mul_lo_u32+add\",\"G_per_s\":%.1f}\n", nthr * (double)ITERS * 8 / ms / 1e6);
  ms = timeit([&] { k_add<<<blocks, threads>>>((uint32_t*)d, 3); });
  printf("{\"op\":\"xor+add(2 ops)\",\"G_per_s\":%.1f}\n", nthr * (double)ITERS * 8 / ms / 1e6);
  ms = timeit([&] { k_fmul<<<blocks, threads>>>((fe*)d, fe{0x123456789ull, 0x987654321ull}); });
  printf("{\"op\":\"f128_mulmod\",\"G_per_s\":%.2f}\n", nthr * (double)(ITERS / 16) * 4 / ms / 1e6);
  CHECK(hipFree(d));
  return 0;
}
