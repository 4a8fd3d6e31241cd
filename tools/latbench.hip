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
  return 0;
}
