// Latency of one Poseidon permutation in the latency-bound form (the 48-lane wide group that
// the tree tops, FRI coins and transcript kernels use), measured on the device: each wave
// hashes merge(d, d) `reps` times in a dependent chain and times it with s_memtime (core clock)
// and s_memrealtime (100 MHz).  Configurations: waves per workgroup and workgroups, so one wave
// alone on a SIMD, two per SIMD (merkle_top's first level) and a full chip can be compared.
// Constants are random (timing only; the permutation's values are checked by the parity tests).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/latbench.hip -o tools/latbench
//   tools/latbench [reps]
#include "../zk-lisp_amd/csrc/poseidon.hip"

#include <cstdio>
#include <random>

using namespace zkl;

__global__ __launch_bounds__(512) void pw_chain_kernel(fe* io, int reps, int active, unsigned long long* cyc) {
  __shared__ __align__(16) uint32_t pw_lds[8 * PW_WAVE_WORDS];
  PWGroup P;
  pw_init(P, pw_lds);
  const int w = (int)(threadIdx.x >> 6);
  if (w >= active) return;  // wave-uniform
  const size_t slot = (size_t)blockIdx.x * 8 + w;
  fe d = io[slot];
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < reps; i++) {
    d = pw_sponge<DOM_MERGE>(P, true, 2, [&](int) { return d; });
    d = pw_bcast(P, d, 0);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    io[slot] = d;
    cyc[2 * slot] = c1 - c0;
    cyc[2 * slot + 1] = r1 - r0;
  }
}

// Parts of the 48-lane round, each timed as a chain of 27 x reps rounds on one wave:
// MODE 1 = the cube alone, 2 = the cube exchange through LDS alone, 3 = exchange + MDS columns
// + fold + DPP sums (no cube), 0 = the whole round (as pw_permute), 4 = the whole round with
// two of the three MDS columns per lane (50 instead of 75 multiply-adds; timing only), 5 / 6 =
// 0 / 2 with the cubes gathered by ds_bpermute instead of an LDS store and load, 7 / 9 = 0 / 2
// with the cubes laid out so that a lane's 15 words are four 128-bit reads, 8 = a copy of 0
// (code-placement noise).
template <int MODE>
__global__ __launch_bounds__(64) void pw_part_kernel(fe* io, int reps, unsigned long long* cyc) {
  __shared__ __align__(16) uint32_t pw_lds[2 * 64];  // room for the 64-word layout of MODE 7 / 9
  PWGroup P;
  pw_init(P, pw_lds);
  uint32_t s[5], s2[5];
  to_mont130(io[threadIdx.x & 63], s);
  to_mont130(io[(threadIdx.x + 1) & 63], s2);
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < reps; i++) {
    const uint32_t* rcp = &c_hm.rc130[0][P.e][0];
#pragma unroll 1
    for (int r = 0; r < 27; r++, rcp += 60) {
      uint32_t rc[5];
#pragma unroll
      for (int l = 0; l < 5; l++) rc[l] = rcp[l];
      uint32_t t[5];
      if (MODE == 10) {  // two independent cube chains per lane: issue-bound or dependency-bound?
        uint32_t t2[5];
        mont_cube130(s, t);
        mont_cube130(s2, t2);
#pragma unroll
        for (int l = 0; l < 5; l++) {
          s[l] = t[l] + rc[l];
          s2[l] = t2[l] + rc[l];
        }
        continue;
      }
      if (MODE == 2 || MODE == 3 || MODE == 6 || MODE == 9) {
#pragma unroll
        for (int l = 0; l < 5; l++) t[l] = s[l];
      } else {
        mont_cube130(s, t);
      }
      if (MODE == 1) {
#pragma unroll
        for (int l = 0; l < 5; l++) s[l] = t[l] + rc[l];
        continue;
      }
      uint32_t tk[PW_COLS][5];
      if (MODE == 7 || MODE == 9) {  // LDS, the 15 words a lane reads contiguous: 4 x 128-bit reads
        // element k at word 16 (k / 3) + 5 (k % 3) + l
        if (P.h == 0) {
          uint32_t* w = P.x + 16 * (P.e / 3) + 5 * (P.e % 3);
#pragma unroll
          for (int l = 0; l < 5; l++) w[l] = t[l];
        }
        wave_sync();
        const uint4* r = reinterpret_cast<const uint4*>(P.x + 16 * P.h);
        uint32_t v[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint4 a = r[q];
          v[4 * q] = a.x; v[4 * q + 1] = a.y; v[4 * q + 2] = a.z; v[4 * q + 3] = a.w;
        }
#pragma unroll
        for (int k = 0; k < PW_COLS; k++)
#pragma unroll
          for (int l = 0; l < 5; l++) tk[k][l] = v[5 * k + l];
        __builtin_amdgcn_wave_barrier();
      } else if (MODE == 5 || MODE == 6) {  // cross-lane reads instead of the LDS round trip
        const int base = PW_LANES * P.g + P.h;
#pragma unroll
        for (int k = 0; k < PW_COLS; k++) {
          const int addr = ((base + PW_SPLIT * (PW_COLS * P.h + k)) & 63) << 2;
#pragma unroll
          for (int l = 0; l < 5; l++) tk[k][l] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)t[l]);
        }
      } else {
        if (P.h == 0) {
#pragma unroll
          for (int l = 0; l < 5; l++) P.x[l * 12 + P.e] = t[l];
        }
        wave_sync();
#pragma unroll
        for (int l = 0; l < 5; l++)
#pragma unroll
          for (int k = 0; k < PW_COLS; k++) tk[k][l] = P.x[l * 12 + PW_COLS * P.h + k];
        __builtin_amdgcn_wave_barrier();
      }
      if (MODE == 2 || MODE == 6 || MODE == 9) {
#pragma unroll
        for (int l = 0; l < 5; l++) s[l] = (tk[0][l] ^ tk[1][l] ^ tk[2][l]) + rc[l];
        continue;
      }
      uint64_t col[5] = {0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < (MODE == 4 ? PW_COLS - 1 : PW_COLS); k++)
#pragma unroll
        for (int u = 0; u < 5; u++)
#pragma unroll
          for (int l = 0; l < 5; l++) col[l] += (uint64_t)tk[k][u] * P.c[k][u][l];
      uint32_t part[5];
      pw_fold(col, part);
#pragma unroll
      for (int l = 0; l < 5; l++) s[l] = pw_elem_sum(part[l]) + rc[l];
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  io[threadIdx.x & 63] = from_mont130(s);
  if (MODE == 10) io[(threadIdx.x & 63) + 64] = from_mont130(s2);
  if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

template <int MODE>
static void part_run(fe* io, unsigned long long* cyc, int reps, hipStream_t s, const char* what) {
  pw_part_kernel<MODE><<<1, 64, 0, s>>>(io, 2, cyc);
  pw_part_kernel<MODE><<<1, 64, 0, s>>>(io, reps, cyc);
  ZKL_HIPCHECK(hipStreamSynchronize(s));
  unsigned long long c = 0;
  ZKL_HIPCHECK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
  printf("{\"part\": \"%s\", \"cycles_per_round\": %.1f}\n", what, (double)c / reps / 27);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  HasherConsts hc{};
  std::mt19937_64 rng(7);
  auto rnd = [&] { return fe{rng(), rng() >> 1}; };
  for (auto& x : hc.mds) x = rnd();
  for (auto& x : hc.rc) x = rnd();
  hc.dom[0] = rnd(); hc.dom[1] = rnd();
  hc.dom_elems = rnd(); hc.dom_merge = rnd(); hc.dom_many = rnd(); hc.dom_int = rnd();
  hipStream_t s;
  ZKL_HIPCHECK(hipStreamCreate(&s));
  upload_hasher_mont(make_hasher_mont(hc), s);
  const int max_blocks = 512;
  fe* io;
  unsigned long long* cyc;
  ZKL_HIPCHECK(hipMalloc(&io, sizeof(fe) * 8 * max_blocks));
  ZKL_HIPCHECK(hipMalloc(&cyc, 16 * 8 * max_blocks));
  std::vector<fe> h(8 * max_blocks);
  for (auto& x : h) x = rnd();
  ZKL_HIPCHECK(hipMemcpy(io, h.data(), sizeof(fe) * h.size(), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  ZKL_HIPCHECK(hipEventCreate(&e0));
  ZKL_HIPCHECK(hipEventCreate(&e1));
  struct Cfg { int blocks, waves; const char* what; };
  const Cfg cfgs[] = {{1, 1, "1 wave alone"}, {1, 4, "4 waves, 1 per SIMD"}, {1, 8, "8 waves, 2 per SIMD"},
                      {256, 4, "256 CUs x 4 waves"}, {256, 8, "256 CUs x 8 waves (tree top level 1)"}};
  for (const Cfg& c : cfgs) {
    auto go = [&](int r) { pw_chain_kernel<<<c.blocks, 512, 0, s>>>(io, r, c.waves, cyc); };
    go(4);  // warm-up
    ZKL_HIPCHECK(hipEventRecord(e0, s));
    go(reps);
    ZKL_HIPCHECK(hipEventRecord(e1, s));
    ZKL_HIPCHECK(hipStreamSynchronize(s));
    float ms = 0;
    ZKL_HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> hc2(16 * max_blocks);
    ZKL_HIPCHECK(hipMemcpy(hc2.data(), cyc, 16 * 8 * max_blocks, hipMemcpyDeviceToHost));
    double cy = 0, rt = 0;
    int n = 0;
    for (int b = 0; b < c.blocks; b++)
      for (int w = 0; w < c.waves; w++, n++) {
        cy += (double)hc2[2 * (b * 8 + w)];
        rt += (double)hc2[2 * (b * 8 + w) + 1];
      }
    cy /= n;
    rt /= n;
    printf("{\"cfg\": \"%s\", \"reps\": %d, \"us_per_perm_event\": %.3f, \"us_per_perm_realtime\": %.3f, "
           "\"cycles_per_perm\": %.0f, \"cycles_per_round\": %.1f, \"clock_mhz\": %.0f}\n",
           c.what, reps, ms * 1e3 / reps, rt / 100.0 / reps, cy / reps, cy / reps / 27, cy / (rt / 100.0));
  }
  part_run<0>(io, cyc, reps, s, "whole round");
  part_run<1>(io, cyc, reps, s, "cube");
  part_run<10>(io, cyc, reps, s, "two independent cubes per lane (divide by 2)");
  part_run<2>(io, cyc, reps, s, "LDS exchange");
  part_run<3>(io, cyc, reps, s, "exchange + MDS + fold + sums");
  part_run<4>(io, cyc, reps, s, "whole round, 50 MDS multiply-adds");
  part_run<5>(io, cyc, reps, s, "whole round, bpermute exchange");
  part_run<6>(io, cyc, reps, s, "bpermute exchange");
  part_run<7>(io, cyc, reps, s, "whole round, 128-bit reads");
  part_run<9>(io, cyc, reps, s, "128-bit-read exchange");
  part_run<8>(io, cyc, reps, s, "whole round (copy)");
  part_run<0>(io, cyc, reps, s, "whole round (again)");
  return 0;
}
