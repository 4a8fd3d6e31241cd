// Issue/latency microbenchmark of the integer multiply forms used by the field arithmetic
// (gfx950): v_mad_u64_u32, v_mul_lo_u32, v_mad_u32_u24, v_mul_hi_u32_u24, v_dot2_u32_u16,
// v_fma_f64, the 64-bit shifts and the 32-bit ops of the carries (round 5).  One wave (latency view: one wave per SIMD, no other wave to hide behind) and a
// full chip (throughput view).  Prints shader cycles and ns per wave-instruction.
//   hipcc --offload-arch=gfx950 -O3 tools/madbench.hip -o /tmp/madbench && /tmp/madbench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITERS = 4096;

#define CHAIN8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

template <int KIND, bool DEP>
__global__ void bench(uint64_t* out, uint32_t seed) {
  uint64_t acc[8];
  uint32_t a[8], b = seed * 2654435761u + threadIdx.x;
  double fa[8], fb = (double)seed;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc[i] = i + threadIdx.x;
    a[i] = seed + 17 * i + threadIdx.x;
    fa[i] = (double)a[i];
  }
  const uint64_t c0 = clock64(), w0 = wall_clock64();
  for (int it = 0; it < ITERS; it++) {
    if (KIND == 0) {  // v_mad_u64_u32
      if (DEP) {
#define OPD(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[0]) : "v"(a[i]), "v"(b) : "vcc");
        CHAIN8(OPD)
#undef OPD
      } else {
#define OPI(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a[i]), "v"(b) : "vcc");
        CHAIN8(OPI)
#undef OPI
      }
    } else if (KIND == 1) {  // v_mul_lo_u32
#define OPI(i) asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(a[DEP ? 0 : i]) : "v"(a[DEP ? 0 : i]), "v"(b));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 2) {  // v_mad_u32_u24
#define OPI(i) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(a[DEP ? 0 : i]) : "v"(a[(i + 1) & 7]), "v"(b));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 3) {  // v_mul_hi_u32_u24
#define OPI(i) asm volatile("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(a[DEP ? 0 : i]) : "v"(a[DEP ? 0 : i]), "v"(b));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 4) {  // v_dot2_u32_u16
#define OPI(i) asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(a[DEP ? 0 : i]) : "v"(a[(i + 1) & 7]), "v"(b));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 5) {  // v_fma_f64
#define OPI(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(fa[DEP ? 0 : i]) : "v"(fa[(i + 1) & 7]), "v"(fb));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 6) {  // v_add_u32 (reference full-rate op)
#define OPI(i) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[DEP ? 0 : i]) : "v"(b));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 7) {  // v_lshl_add_u64 (64-bit shift-add used by the REDC carries)
#define OPI(i) asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(acc[DEP ? 0 : i]) : "v"(acc[(i + 1) & 7]));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 8) {  // v_ashrrev_i64 (the REDC / fold carries)
#define OPI(i) asm volatile("v_ashrrev_i64 %0, 3, %0" : "+v"(acc[DEP ? 0 : i]));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 9) {  // v_lshrrev_b64
#define OPI(i) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(acc[DEP ? 0 : i]));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 10) {  // v_mad_i64_i32 (digit-column fold, REDC's -2^24 m)
#define OPI(i) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(acc[DEP ? 0 : i]) : "v"(a[i]), "v"(b) : "vcc");
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 11) {  // v_alignbit_b32 (a 64-bit shift's low word in one 32-bit op)
#define OPI(i) asm volatile("v_alignbit_b32 %0, %1, %0, 26" : "+v"(a[DEP ? 0 : i]) : "v"(b));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 12) {  // v_and_b32
#define OPI(i) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a[DEP ? 0 : i]) : "v"(b));
      CHAIN8(OPI)
#undef OPI
    } else if (KIND == 13) {  // v_mad_u64_u32 and v_add_u32 alternating (independent)
#define OPI(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n v_add_u32 %3, %2, %3" : "+v"(acc[i]), "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(b) : "vcc");
      CHAIN8(OPI)
#undef OPI
    }
  }
  const uint64_t c1 = clock64(), w1 = wall_clock64();
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += acc[i] + a[i] + (uint64_t)fa[i];
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
  }
  if (s == 0x1234567) out[2] = s;
}

static const char* names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mad_u32_u24", "v_mul_hi_u32_u24",
                              "v_dot2_u32_u16", "v_fma_f64", "v_add_u32", "v_lshl_add_u64",
                              "v_ashrrev_i64", "v_lshrrev_b64", "v_mad_i64_i32", "v_alignbit_b32",
                              "v_and_b32", "mad_u64+add_u32"};

template <int K, bool D>
static void run(uint64_t* d, int blocks, int threads) {
  uint64_t h[3] = {0, 0, 0};
  bench<K, D><<<blocks, threads>>>(d, 7);  // warm
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  bench<K, D><<<blocks, threads>>>(d, 7);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  const double n_instr = (K == 13 ? 16.0 : 8.0) * ITERS;
  int wall_mhz = 0;
  (void)hipDeviceGetAttribute(&wall_mhz, hipDeviceAttributeWallClockRate, 0);  // kHz
  const double wall_ns = (double)h[1] * 1e6 / (double)wall_mhz;
  const double waves = (double)blocks * threads / 64.0;
  printf("%-18s %-5s waves %6.0f: %6.2f cycles/instr/wave, %6.2f ns/instr (wave 0), clock %.0f MHz, chip %.1f G wave-instr/s\n",
         names[K], D ? "dep" : "indep", waves, h[0] / n_instr, wall_ns / n_instr, h[0] / wall_ns * 1e3,
         waves * n_instr / (ms * 1e-3) / 1e9);
}

template <int K>
static void kind(uint64_t* d, int cus) {
  run<K, false>(d, 1, 64);
  run<K, true>(d, 1, 64);
  run<K, false>(d, cus, 256);      // one wave per SIMD everywhere
  run<K, false>(d, cus * 2, 256);  // 2 waves per SIMD
  run<K, false>(d, cus * 3, 256);  // 3 waves per SIMD
  run<K, false>(d, cus * 8, 256);  // 8 waves per SIMD
}

int main() {
  uint64_t* d;
  (void)hipMalloc(&d, 64);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", cus);
  kind<0>(d, cus);
  kind<1>(d, cus);
  kind<2>(d, cus);
  kind<3>(d, cus);
  kind<4>(d, cus);
  kind<5>(d, cus);
  kind<6>(d, cus);
  kind<7>(d, cus);
  kind<8>(d, cus);
  kind<9>(d, cus);
  kind<10>(d, cus);
  kind<11>(d, cus);
  kind<12>(d, cus);
  kind<13>(d, cus);
  (void)hipFree(d);
  return 0;
}
