// gfx950 Poseidon kernels of the zk-lisp segment prover: hot loop A --
// partitioned row hashing of the trace and composition LDEs, Merkle levels, FRI layer leaves,
// transcript draws and grinding -- in the lane-group (latency) and matrix-core (throughput)
// forms.  A translation unit of its own so scheduler flags can differ from those of the NTT,
// constraint evaluator and DEEP (kernels.hip); the default scheduler measured best for both
// (Makefile: POSEIDON_SCHED).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "kernels.h"
#include "mont26.h"

namespace zkl {

// =====================================================================================
// Poseidon (poseidon/hasher.rs:173-190): 27 rounds of x^3 on all 12 lanes, dense MDS, +rc.
// The MDS row sum is accumulated unreduced (288-bit) and reduced once per lane.
// =====================================================================================
__constant__ HasherMont c_hm;

__device__ __forceinline__ void to_mont130(fe a, uint32_t out[5]) {
  uint32_t l[5];
  to26(a, l);
  uint64_t col[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  mac5(l, c_hm.r2_130, col);
  redc130(col, out);
}

__device__ __forceinline__ fe from_mont130(const uint32_t a[5]) {
  uint64_t col[10] = {a[0], a[1], a[2], a[3], a[4], 0, 0, 0, 0, 0};
  uint32_t l[5];
  redc130(col, l);  // < p + 2
  fe r;
  r.lo = (uint64_t)l[0] | ((uint64_t)l[1] << 26) | ((uint64_t)l[2] << 52);
  r.hi = ((uint64_t)l[2] >> 12) | ((uint64_t)l[3] << 14) | ((uint64_t)l[4] << 40);
  if (r.hi == P_HI && r.lo >= P_LO) r = fe{r.lo - P_LO, 0};
  return r;
}

__device__ __forceinline__ void to_mont(fe a, uint32_t out[5]) {
  uint32_t l[5];
  to26(a, l);
  mont_mul(l, c_hm.r2, out);
}

__device__ __forceinline__ fe from_mont(const uint32_t a[5]) {
  uint64_t col[10] = {a[0], a[1], a[2], a[3], a[4], 0, 0, 0, 0, 0};
  uint32_t l[5];
  redc(col, l);  // < p + 1
  fe r;
  r.lo = (uint64_t)l[0] | ((uint64_t)l[1] << 26) | ((uint64_t)l[2] << 52);
  r.hi = ((uint64_t)l[2] >> 12) | ((uint64_t)l[3] << 14) | ((uint64_t)l[4] << 40);
  if (r.hi == P_HI && r.lo >= P_LO) r = fe{r.lo - P_LO, 0};
  return r;
}

HasherMont make_hasher_mont(const HasherConsts& h) {
  HasherMont m{};
  fe R = fe_pow64(fe{2, 0}, 156);  // 2^156 mod p
  auto mont = [&](fe x, uint32_t out[5]) { limbs26(fe_mul(x, R), out); };
  for (int i = 0; i < 12; i++)
    for (int k = 0; k < 12; k++) mont(h.mds[i * 12 + k], m.mds[i][k]);
  for (int r = 0; r < 27; r++)
    for (int i = 0; i < 12; i++) mont(h.rc[r * 12 + i], m.rc[r][i]);
  mont(h.dom[0], m.dom[0]);
  mont(h.dom[1], m.dom[1]);
  limbs26(fe_mul(R, R), m.r2);
  mont(h.dom_elems, m.dfe[DOM_ELEMS]);
  mont(h.dom_merge, m.dfe[DOM_MERGE]);
  mont(h.dom_many, m.dfe[DOM_MANY]);
  mont(h.dom_int, m.dfe[DOM_INT]);
  const fe R130 = fe_pow64(fe{2, 0}, 130);
  auto mont130 = [&](fe x, uint32_t out[5]) { limbs26(fe_mul(x, R130), out); };
  mont130(h.dom[0], m.dom130[0]);
  mont130(h.dom[1], m.dom130[1]);
  limbs26(fe_mul(R130, R130), m.r2_130);
  mont130(h.dom_elems, m.dfe130[DOM_ELEMS]);
  mont130(h.dom_merge, m.dfe130[DOM_MERGE]);
  mont130(h.dom_many, m.dfe130[DOM_MANY]);
  mont130(h.dom_int, m.dfe130[DOM_INT]);
  fe w = fe_one();  // 2^(26u)
  for (int u = 0; u < 5; u++, w = fe_mul(w, fe{1ull << 26, 0}))
    for (int i = 0; i < 12; i++)
      for (int k = 0; k < 12; k++) limbs26(fe_mul(h.mds[i * 12 + k], w), m.mdsl[i][k][u]);
  for (int r = 0; r < 27; r++)
    for (int i = 0; i < 12; i++) mont130(h.rc[r * 12 + i], m.rc130[r][i]);
  {
    uint32_t c[5];
    const uint32_t z[5] = {0, 0, 0, 0, 0};
    mont_cube130(z, c);
    pm_pack_words(c, m.pmk0);
    for (int t = 0; t < 2; t++) {
      mont_cube130(m.dom130[t], c);
      pm_pack_words(c, m.pmkt[t]);
    }
  }
  return m;
}

void upload_hasher_mont(const HasherMont& m, hipStream_t s) {
  ZKL_HIPCHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_hm), &m, sizeof m, 0, hipMemcpyHostToDevice, s));
}

// ---- lane-group permutation ------------------------------------------------------------
// One Poseidon state is held by 12 lanes of a wave: lane j owns s_j (5 limbs) and row j of
// the MDS matrix (60 VGPRs, loaded once).  A round is: cube own lane -> publish it in LDS
// -> read all 12 cubes of the group -> own MDS row sum -> REDC -> +rc.  A wave holds five
// states (lanes 0..59); lanes 60..63 form a partial sixth group whose results are unused.
// Compared with one state per lane this keeps the MDS constants in registers instead of
// re-streaming them through SGPRs, and cuts the latency of one permutation twelve-fold,
// which is what bounds the upper Merkle levels and the FRI layers.
constexpr int PG_LANES = 12;
constexpr int PG_PER_WAVE = 5;
constexpr int PG_GROUP_WORDS = 60;  // 5 limbs x 12 lanes
constexpr int PG_WAVE_WORDS = 6 * PG_GROUP_WORDS;  // six groups

struct PGroup {
  uint32_t m[12][5];  // MDS row j (Montgomery)
  uint32_t* x;        // this group's exchange area: x[limb * 12 + lane]

  int j;              // lane within the group
  int g;              // group within the wave (5 = the partial group)
};

__device__ __forceinline__ void pg_init(PGroup& P, uint32_t* lds) {
  const int lane = (int)(threadIdx.x & 63);
  P.g = lane / PG_LANES;
  P.j = lane - PG_LANES * P.g;
  P.x = lds + (threadIdx.x >> 6) * PG_WAVE_WORDS + P.g * PG_GROUP_WORDS;

#pragma unroll
  for (int k = 0; k < 12; k++)
#pragma unroll
    for (int l = 0; l < 5; l++) P.m[k][l] = c_hm.mds[P.j][k][l];
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Poseidon permutation (poseidon/hasher.rs:173-190): 27 rounds of x^3 on all 12 lanes,
// dense 12x12 MDS, + round constants.  s = this lane's state element (Montgomery).
__device__ __forceinline__ void pg_permute(PGroup& P, uint32_t s[5]) {
  const uint4* xv = reinterpret_cast<const uint4*>(P.x);
  const uint32_t* rcp = &c_hm.rc[0][P.j][0];
#pragma unroll 1
  for (int r = 0; r < 27; r++, rcp += 60) {
    uint32_t rc[5];  // issued early; consumed after the MDS row sum
#pragma unroll
    for (int l = 0; l < 5; l++) rc[l] = rcp[l];
    uint32_t t[5];
    mont_cube(s, t);
#pragma unroll
    for (int l = 0; l < 5; l++) P.x[l * 12 + P.j] = t[l];
    wave_sync();
    uint64_t col[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint4 v[15];  // all twelve cubes of the group, limb-major: v[l*3+q] = limb l of lanes 4q..4q+3
#pragma unroll
    for (int i = 0; i < 15; i++) v[i] = xv[i];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 3; q++) {
      uint32_t a0[5] = {v[q].x, v[3 + q].x, v[6 + q].x, v[9 + q].x, v[12 + q].x};
      uint32_t a1[5] = {v[q].y, v[3 + q].y, v[6 + q].y, v[9 + q].y, v[12 + q].y};
      uint32_t a2[5] = {v[q].z, v[3 + q].z, v[6 + q].z, v[9 + q].z, v[12 + q].z};
      uint32_t a3[5] = {v[q].w, v[3 + q].w, v[6 + q].w, v[9 + q].w, v[12 + q].w};
      mac5(a0, P.m[4 * q + 0], col);
      mac5(a1, P.m[4 * q + 1], col);
      mac5(a2, P.m[4 * q + 2], col);
      mac5(a3, P.m[4 * q + 3], col);
    }
    redc(col, s);
#pragma unroll
    for (int l = 0; l < 5; l++) s[l] += rc[l];
  }
}

// ro_bytes_sponge_custom_rounds (hasher.rs:144-231) over pre-folded 32-byte chunks: the
// stream [dom_fe, msg_0, .., msg_{n-1}] is added into lanes 0..9 ten at a time, permuting
// after each block (the last one possibly partial).  nmsg must be uniform within a group;
// ld(i) is called only by the lane that absorbs message i, and only when live.  Returns
// the digest value (state[0]) in lane 0 of the group.
template <int D, class Loader>
__device__ __forceinline__ fe pg_sponge(PGroup& P, bool live, int nmsg, Loader ld) {
  uint32_t s[5];
#pragma unroll
  for (int l = 0; l < 5; l++)
    s[l] = P.j == 0 ? c_hm.dfe[D][l] : P.j == 10 ? c_hm.dom[0][l] : P.j == 11 ? c_hm.dom[1][l] : 0u;
  const int T = nmsg + 1;
  for (int b = 0; b * 10 < T; b++) {
    const int idx = b * 10 + P.j;
    if (live && P.j < 10 && idx >= 1 && idx < T) {
      uint32_t m[5];
      to_mont(ld(idx - 1), m);
#pragma unroll
      for (int l = 0; l < 5; l++) s[l] += m[l];
    }
    pg_permute(P, s);
  }
  return from_mont(s);
}

// broadcast lane `src` of this thread's group to every lane of the group
__device__ __forceinline__ fe pg_bcast(const PGroup& P, fe v, int src) {
  const int from = (int)(threadIdx.x & 63) - P.j + src;
  fe r;
  r.lo = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v.lo >> 32), from) << 32) | (uint32_t)__shfl((int)(uint32_t)v.lo, from);
  r.hi = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v.hi >> 32), from) << 32) | (uint32_t)__shfl((int)(uint32_t)v.hi, from);
  return r;
}

// ---- wide lane groups (latency-bound levels) ------------------------------------------
// PW_SPLIT (2 or 4) lanes per state element: lane SPLIT*e + h owns element e (every lane of
// the element holds it) and the MDS row-e constants of columns COLS*h .. COLS*h + COLS-1
// (COLS = 12 / SPLIT).  Used where a level has too few states to fill the SIMDs (upper Merkle
// levels, small FRI layers, the transcript kernels): one permutation's dependency chain bounds
// those levels, so the round is built for a short chain rather than few
// instructions per state.
//
// Radix R' = 2^130, as the matrix-core form: a state element is held as s R' (five 26-bit
// limbs, lazily reduced), the cube is mont_cube130 (two five-digit REDCs) and gives s^3 R'.
// The MDS layer needs no REDC at all: the cube y (limbs y_u) enters row e as
// sum_u y_u (M[e][k] 2^(26u) mod p) with the limb-weighted constants c_hm.mdsl (linear, so the
// R' factor passes through), i.e. 5 x 5 products per column into five 64-bit limb columns,
// which one carry pass and a fold of the bits >= 128 (2^128 == 45 2^40 - 1) bring back to
// five limbs of a value < 2^128 + 2^82.  The SPLIT lanes of an element add those parts with
// DPP quad permutes, plus the round constant: limbs < 2^28.4, value < 2^130.4, inside what
// mont_cube130 takes.  Against the R = 2^156 round this drops one REDC digit step from each of
// the cube's two reductions and the whole six-step REDC of the MDS sum.
#ifndef PW_SPLIT
#define PW_SPLIT 4
#endif
static_assert(PW_SPLIT == 2 || PW_SPLIT == 4, "PW_SPLIT must be 2 or 4");
constexpr int PW_COLS = 12 / PW_SPLIT;
constexpr int PW_LANES = 12 * PW_SPLIT;
constexpr int PW_PER_WAVE = 64 / PW_LANES;
constexpr int PW_GROUP_WORDS = 60;  // cubes [l][12]
constexpr int PW_WAVE_WORDS = (PW_PER_WAVE + 1) * PW_GROUP_WORDS;  // + the idle partial group

struct PWGroup {
  uint32_t c[PW_COLS][5][5];  // c[k][u][l] = limb l of M[e][COLS*h + k] * 2^(26u) mod p
  uint32_t* x;                // cubes: x[limb * 12 + e]
  int e, h, g;
};

// Issue priority of the latency-bound tail kernels (wide lane groups, tree tops, FRI coin):
// with several proofs in flight their waves share SIMDs with another proof's throughput
// kernels, and a raised wave priority lets the one permutation chain they carry issue first.
#ifndef TAIL_PRIO_CFG
#define TAIL_PRIO_CFG 0
#endif
__device__ __forceinline__ void tail_prio() {
  if (TAIL_PRIO_CFG) __builtin_amdgcn_s_setprio(TAIL_PRIO_CFG);
}

__device__ __forceinline__ void pw_init(PWGroup& P, uint32_t* lds) {
  tail_prio();
  const int lane = (int)(threadIdx.x & 63);
  P.g = lane / PW_LANES;
  const int j = lane - PW_LANES * P.g;
  P.e = min(j / PW_SPLIT, 11);
  P.h = j % PW_SPLIT;
  P.x = lds + (threadIdx.x >> 6) * PW_WAVE_WORDS + P.g * PW_GROUP_WORDS;
#pragma unroll
  for (int k = 0; k < PW_COLS; k++)
#pragma unroll
    for (int u = 0; u < 5; u++)
#pragma unroll
      for (int l = 0; l < 5; l++) P.c[k][u][l] = c_hm.mdsl[P.e][PW_COLS * P.h + k][u][l];
}

// sum of v over the SPLIT lanes of this lane's element (DPP quad_perm [1,0,3,2], [2,3,0,1]);
// the permuted operand's old value is 0, so each step can issue as one v_add_u32_dpp
__device__ __forceinline__ uint32_t pw_elem_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
  if (PW_SPLIT == 4) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
  return v;
}

// five 64-bit limb columns (each < 2^60) -> five limbs of a congruent value < 2^128 + 2^82:
// limbs 0, 1, 3 < 2^26, limb 2 < 2^26 + 8, limb 4 < 2^24.  The bits >= 128 of column 4 fold
// as t 2^128 == t (737279 2^26 + 2^26 - 1) for its low word's top byte t and as
// hi 2^136 == hi (188743680 2^26 - 2^8) for its high word hi (< 2^28).
__device__ __forceinline__ void pw_fold(uint64_t col[5], uint32_t x[5]) {
  uint32_t l[4];
#pragma unroll
  for (int t = 0; t < 4; t++) {
    col[t + 1] += col[t] >> 26;
    l[t] = (uint32_t)col[t] & M26;
  }
  const uint32_t lo4 = (uint32_t)col[4], hi4 = (uint32_t)(col[4] >> 32);
  const uint32_t t = lo4 >> 24;
  // a >= -2^36; b >= 188743680 whenever hi4 > 0, so b + (a >> 26) >= 0
  const int64_t a = (int64_t)((uint64_t)t * M26 + l[0]) - (int64_t)((uint64_t)hi4 << 8);
  const uint64_t b = (uint64_t)t * 737279u + (uint64_t)hi4 * 188743680u + l[1];
  const uint64_t bb = b + (uint64_t)(a >> 26);
  x[0] = (uint32_t)a & M26;
  x[1] = (uint32_t)bb & M26;
  const uint32_t x2 = l[2] + (uint32_t)(bb >> 26);
  x[2] = x2 & M26;
  x[3] = l[3] + (x2 >> 26);
  x[4] = lo4 & 0xFFFFFFu;
}

__device__ __forceinline__ void pw_permute(PWGroup& P, uint32_t s[5]) {
  const uint32_t* rcp = &c_hm.rc130[0][P.e][0];
#pragma unroll 1
  for (int r = 0; r < 27; r++, rcp += 60) {
    uint32_t rc[5];
#pragma unroll
    for (int l = 0; l < 5; l++) rc[l] = rcp[l];
    uint32_t t[5];
    mont_cube130(s, t);
    if (P.h == 0) {
#pragma unroll
      for (int l = 0; l < 5; l++) P.x[l * 12 + P.e] = t[l];
    }
    wave_sync();
    uint32_t tk[PW_COLS][5];
#pragma unroll
    for (int l = 0; l < 5; l++)
#pragma unroll
      for (int k = 0; k < PW_COLS; k++) tk[k][l] = P.x[l * 12 + PW_COLS * P.h + k];
    __builtin_amdgcn_wave_barrier();
    uint64_t col[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < PW_COLS; k++)
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

template <int D, class Loader>
__device__ __forceinline__ fe pw_sponge(PWGroup& P, bool live, int nmsg, Loader ld) {
  uint32_t s[5];
#pragma unroll
  for (int l = 0; l < 5; l++)
    s[l] = P.e == 0 ? c_hm.dfe130[D][l] : P.e == 10 ? c_hm.dom130[0][l] : P.e == 11 ? c_hm.dom130[1][l] : 0u;
  const int T = nmsg + 1;
  for (int b = 0; b * 10 < T; b++) {
    const int idx = b * 10 + P.e;
    if (live && P.e < 10 && idx >= 1 && idx < T) {
      uint32_t m[5];
      to_mont130(ld(idx - 1), m);
#pragma unroll
      for (int l = 0; l < 5; l++) s[l] += m[l];
    }
    pw_permute(P, s);
  }
  return from_mont130(s);  // state element 0 in lanes with e == 0
}

__device__ __forceinline__ fe pw_bcast(const PWGroup& P, fe v, int src_e) {
  const int from = PW_LANES * P.g + PW_SPLIT * src_e;
  fe r;
  r.lo = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v.lo >> 32), from) << 32) | (uint32_t)__shfl((int)(uint32_t)v.lo, from);
  r.hi = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v.hi >> 32), from) << 32) | (uint32_t)__shfl((int)(uint32_t)v.hi, from);
  return r;
}

#define PW_SETUP()                                            \
  __shared__ __align__(16) uint32_t pw_lds[4 * PW_WAVE_WORDS]; \
  PWGroup P;                                                  \
  pw_init(P, pw_lds);                                         \
  const size_t item = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * PW_PER_WAVE + (size_t)P.g;

static inline unsigned pw_blocks(size_t items) {
  const size_t per = 4 * PW_PER_WAVE;
  return (unsigned)((items + per - 1) / per);
}

// levels (and FRI layers) with at most this many states use the wide groups: up to one
// wide wave per SIMD, where per-state latency rather than issue throughput bounds the level
#ifndef PW_MAX_ITEMS_CFG
#define PW_MAX_ITEMS_CFG 2048
#endif
constexpr size_t PW_MAX_ITEMS = PW_MAX_ITEMS_CFG;

// levels (and FRI layers) of [lo, hi) states use the 16-state matrix-core form (with the
// matrix-core engine): there the 32-state form runs at most half a wave per SIMD (2^14 states)
// and the lane groups a wave on every other SIMD (2^13), so a level costs one permutation's
// latency, which the 16-state form, with half the VALU work per lane, shortens: 2^14 states
// 69.5 -> 47 us, 2^13 56 -> 47 us (lane groups); at 2^15 the 32-state form is faster (73 against
// 80 us, profiles/r05/pm16/).  ZKL_PM16=lo,hi (0 = off) for A/B; default 2^13, 2^15.
static bool pm16_range(size_t items) {
  static const size_t* lim = [] {
    static size_t v[2] = {(size_t)1 << 13, (size_t)1 << 15};
    if (const char* e = getenv("ZKL_PM16")) {
      if (!strcmp(e, "0")) v[0] = v[1] = 0;
      else if (sscanf(e, "%zu,%zu", &v[0], &v[1]) != 2) throw std::invalid_argument("ZKL_PM16: expected lo,hi");
    }
    return v;
  }();
  return items >= lim[0] && items < lim[1];
}

// Occupancy target of the lane-group kernels: 2 waves/SIMD lets the scheduler batch the 15
// LDS reads of a round; 3 forces them to serialise on a shared register window.
#ifndef PG_WAVES
#define PG_WAVES 2
#endif
#define PG_KERNEL __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PG_WAVES, PG_WAVES)))

#define PG_SETUP()                                          \
  __shared__ __align__(16) uint32_t pg_lds[4 * PG_WAVE_WORDS]; \
  PGroup P;                                                 \
  pg_init(P, pg_lds);                                       \
  const size_t item = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * PG_PER_WAVE + (size_t)P.g;

static inline unsigned pg_blocks(size_t items) {
  const size_t per = 4 * PG_PER_WAVE;
  return (unsigned)((items + per - 1) / per);
}

// PM_ROW_BIG_CFG: row hashing keeps the partition digests in LDS for every partition count
// (the <TAG, true> form) instead of in registers (fewer VGPRs, for PM_ROW_WAVES_CFG = 12)
#ifndef PM_ROW_BIG_CFG
#define PM_ROW_BIG_CFG 0
#endif
#include "poseidon_mfma.inc"

// ---- row hashing (Winterfell partitioned row hash): one group per row.  The row's
// partitions are hashed one after another (hash_elements over psize columns, chunked in
// folded pairs); with more than one partition their digests are merged with merge_many.
// TAG only separates the trace (0) and composition (1) commitments in profiles
template <int TAG>
__global__ PG_KERNEL void hash_rows_kernel(const fe* __restrict__ M, uint32_t ncols, size_t nrows,
                                                        uint32_t psize, uint32_t merge, fe* __restrict__ out, int split) {
  PG_SETUP();
  const bool live = P.g < PG_PER_WAVE && item < nrows;
  const size_t row = live ? item : 0;
  const uint32_t np = (ncols + psize - 1) / psize;
  fe keep0 = fe_zero(), keep1 = fe_zero(), d = fe_zero();
  for (uint32_t p = 0; p < np; p++) {
    const uint32_t c0 = p * psize;
    const uint32_t len = min(psize, ncols - c0);
    const fe* base = M + (size_t)c0 * nrows + row;  // position (split: the row is lde_row)
    d = pg_sponge<DOM_ELEMS>(P, live, (int)((len + 1) / 2), [&](int j) {
      fe a = base[(size_t)(2 * j) * nrows];
      fe b = (2u * j + 1 < len) ? base[(size_t)(2 * j + 1) * nrows] : fe_zero();
      return fold_pair(a, b);
    });
    if (merge) {  // message p of merge_many is absorbed by lane (p+1) % 10 of block (p+1) / 10
      fe v = pg_bcast(P, d, 0);
      if ((int)((p + 1) % 10) == P.j) {
        if (p + 1 < 10) keep0 = v; else keep1 = v;
      }
    }
  }
  if (merge) d = pg_sponge<DOM_MANY>(P, live, (int)np, [&](int i) { return i + 1 < 10 ? keep0 : keep1; });
  if (live && P.j == 0) out[lde_row(row, nrows, split)] = d;
}

__global__ PG_KERNEL void merkle_level_kernel(fe* nodes, size_t lvl) {
  PG_SETUP();
  const bool live = P.g < PG_PER_WAVE && item < lvl;
  const size_t i = lvl + (live ? item : 0);
  fe d = pg_sponge<DOM_MERGE>(P, live, 2, [&](int j) { return nodes[2 * i + j]; });
  if (live && P.j == 0) nodes[i] = d;
}

__global__ PG_KERNEL void draw_kernel(fe seed, const fe* seed_p, uint64_t base, size_t k, fe* out) {
  if (seed_p) seed = *seed_p;
  PG_SETUP();
  const bool live = P.g < PG_PER_WAVE && item < k;
  const uint64_t ctr = base + 1 + item;
  fe d = pg_sponge<DOM_INT>(P, live, 2, [&](int j) { return j == 0 ? seed : fe{ctr, 0}; });
  if (live && P.j == 0) out[item] = d;
}

__global__ PG_KERNEL void grind_kernel(fe seed, const fe* seed_p, uint64_t base, uint32_t count, uint32_t bits,
                                                    unsigned long long* best) {
  if (seed_p) seed = *seed_p;
  // an earlier window found one (every nonce of an earlier window is below base; a solution
  // this window's other blocks have already found is not a reason to stop)
  if (*(volatile unsigned long long*)best < base) return;
  PG_SETUP();
  const bool live = P.g < PG_PER_WAVE && item < count;
  const uint64_t nonce = base + item;
  fe h = pg_sponge<DOM_INT>(P, live, 2, [&](int j) { return j == 0 ? seed : fe{nonce, 0}; });
  if (live && P.j == 0) {
    uint32_t tz = h.lo ? (uint32_t)__builtin_ctzll(h.lo) : 64u;
    if (tz >= bits) atomicMin(best, (unsigned long long)nonce);
  }
}

// Row-digest rule for one-chunk partitioned rows (partition size > width): 0 = winterfell
// commit_to_rows (merge_many of the single chunk digest), 1 = agg/child.rs:1025-1045
// (the chunk digest itself).  DESIGN.md §3.1; the oracle has the same switch.
static std::atomic<int> g_row_rule{0};
void set_row_digest_rule(int r) { g_row_rule.store(r ? 1 : 0); }
int row_digest_rule() { return g_row_rule.load(); }

void launch_hash_rows(const fe* d_mat, uint32_t ncols, size_t nrows, uint32_t np, uint32_t rate, fe* d_tmp, fe* d_out,
                      hipStream_t s, int tag, int split) {
  (void)d_tmp;
  uint32_t psize = ncols;
  if (np > 1) {
    psize = (ncols + np - 1) / np;
    if (psize < rate) psize = rate;  // PartitionOptions::partition_size, ExtensionDegree 1
  }
  const uint32_t np_eff = (ncols + psize - 1) / psize;
  // partitioned rows end in merge_many (rule 0: even of one digest)
  const uint32_t merge = row_digest_rule() == 0 ? (psize != ncols) : (np_eff > 1);
  if (hash_engine() == 1 && nrows >= pm_min_items() && np_eff <= (uint32_t)PM_MAX_PARTS) {
    if (np_eff > 9 || PM_ROW_BIG_CFG)
      PM_GO((hash_rows_pm_kernel<0, true>), nrows, true, s)(d_mat, ncols, nrows, psize, merge, d_out, split);
    else if (tag == 1)
      PM_GO((hash_rows_pm_kernel<1, false>), nrows, true, s)(d_mat, ncols, nrows, psize, merge, d_out, split);
    else
      PM_GO((hash_rows_pm_kernel<0, false>), nrows, true, s)(d_mat, ncols, nrows, psize, merge, d_out, split);
    return;
  }
  if (tag == 1)
    hash_rows_kernel<1><<<pg_blocks(nrows), 256, 0, s>>>(d_mat, ncols, nrows, psize, merge, d_out, split);
  else
    hash_rows_kernel<0><<<pg_blocks(nrows), 256, 0, s>>>(d_mat, ncols, nrows, psize, merge, d_out, split);
}

// Tree top: several levels per launch.  Workgroup g (TOP_WAVES waves, one 48-lane state each)
// owns nodes [cnt*g, cnt*g + cnt) of level lvl and reduces them to one node of level
// lvl/cnt, with a workgroup barrier between levels; waves without a live node skip the
// permutation.  A launch per level would add ~10 us of dispatch latency to each of these
// permutation-latency-bound levels.
#ifndef TOP_LDS_CFG
#define TOP_LDS_CFG 1
#endif
// waves per workgroup (one state each): 8 gives four levels per launch, the first at two waves
// per SIMD; 4 gives three levels per launch, all but a tree's 2048-node level at one wave per SIMD
// (round 6 A/B, profiles/r06/top_waves: Merkle family 10.87 -> 10.69 ms per proof)
#ifndef TOP_WAVES_CFG
#define TOP_WAVES_CFG 4
#endif
static_assert(TOP_WAVES_CFG == 4 || TOP_WAVES_CFG == 8, "TOP_WAVES_CFG must be 4 or 8");
constexpr int TOP_WAVES = TOP_WAVES_CFG / PW_PER_WAVE;
constexpr int TOP_SLOTS = TOP_WAVES * PW_PER_WAVE;
// coin_mode (the launch that reaches the root, one workgroup): after the root, wave 0 runs the
// transcript step that follows the tree -- 1: coin[0] = merge(coin[0], root) (the trace and
// constraint roots), 2: that and coin[1] = merge_with_int(coin[0], 1) (a FRI layer: alpha) --
// and copies the root to *root_out, instead of a launch of its own.
__global__ __launch_bounds__(64 * TOP_WAVES) void merkle_top_kernel(fe* nodes, size_t lvl, int cnt, fe* coin,
                                                                    fe* root_out, int coin_mode) {
  __shared__ __align__(16) uint32_t pw_lds[TOP_WAVES * PW_WAVE_WORDS];
  // the level just computed, also kept in LDS (double-buffered): the next level takes its children
  // from here instead of a global store / barrier / load round trip (round 6)
  __shared__ fe tn[2][TOP_SLOTS];
  PWGroup P;
  pw_init(P, pw_lds);
  const int wave_slot0 = (int)(threadIdx.x >> 6) * PW_PER_WAVE;
  const int slot = wave_slot0 + P.g;
  size_t L = lvl, base = (size_t)blockIdx.x * cnt;
  int par = 0;
  for (int c = cnt; c >= 1; c >>= 1, L >>= 1, base >>= 1, par ^= 1) {
    if (wave_slot0 < c) {  // wave-uniform
      const bool live = P.g < PW_PER_WAVE && slot < c;
      const size_t i = L + base + (live ? slot : 0);
      const int sl = live ? slot : 0;
      fe d = pw_sponge<DOM_MERGE>(P, live, 2, [&](int j) {
        return (c == cnt || !TOP_LDS_CFG) ? nodes[2 * i + j] : tn[par ^ 1][2 * sl + j];
      });
      if (live && P.e == 0 && P.h == 0) {
        nodes[i] = d;
        tn[par][slot] = d;
      }
    }
    __syncthreads();
  }
  if (coin_mode && threadIdx.x < 64) {  // wave 0 of the single workgroup
    const bool live = P.g == 0;
    const fe seed = coin[0], r = TOP_LDS_CFG ? tn[par ^ 1][0] : nodes[1];
    fe s1 = pw_sponge<DOM_MERGE>(P, live, 2, [&](int j) { return j == 0 ? seed : r; });
    fe a = fe_zero();
    if (coin_mode == 2) {
      s1 = pw_bcast(P, s1, 0);
      a = pw_sponge<DOM_INT>(P, live, 2, [&](int j) { return j == 0 ? s1 : fe{1, 0}; });
    }
    if (threadIdx.x == 0) {
      coin[0] = s1;
      if (coin_mode == 2) coin[1] = a;
      if (root_out) *root_out = r;
    }
  }
}

void launch_merkle(fe* d_nodes, size_t n, hipStream_t s, fe* d_coin, fe* d_root_out, int coin_mode) {
  // the transcript step of coin_mode runs only in the launch that reaches the root: a tree that
  // never gets there (fewer than two leaves) would silently leave the coin unseeded
  if (coin_mode && n < 2) throw std::logic_error("launch_merkle: coin step requested on a tree without a root launch");
  bool reached = false;
  for (size_t lvl = n / 2; lvl >= 1;) {
    if (lvl <= PW_MAX_ITEMS) {
      const size_t cnt = std::min<size_t>(lvl, TOP_SLOTS);
      const bool last = lvl / (cnt * 2) == 0;  // this launch reaches the root
      reached |= last;
      merkle_top_kernel<<<(unsigned)(lvl / cnt), 64 * TOP_WAVES, 0, s>>>(d_nodes, lvl, (int)cnt, d_coin, d_root_out,
                                                                          last ? coin_mode : 0);
      lvl /= cnt * 2;
      continue;
    }
    if (hash_engine() == 1 && pm16_range(lvl))
      PM16_GO(merkle_level_pm16_kernel, lvl, s)(d_nodes, lvl);
    else if (hash_engine() == 1 && lvl >= pm_min_items())
      PM_GO(merkle_level_pm_kernel, lvl, false, s)(d_nodes, lvl);
    else
      merkle_level_kernel<<<pg_blocks(lvl), 256, 0, s>>>(d_nodes, lvl);
    lvl /= 2;
  }
  if (coin_mode && !reached) throw std::logic_error("launch_merkle: no launch reached the root; coin step dropped");
}

__global__ PG_KERNEL void pg_permute_kernel(fe* st, size_t n) {
  PG_SETUP();
  const bool live = P.g < PG_PER_WAVE && item < n;
  const size_t i = live ? item : 0;
  uint32_t x[5];
  to_mont(st[i * 12 + P.j], x);
  pg_permute(P, x);
  if (live) st[i * 12 + P.j] = from_mont(x);
}

void launch_permute(fe* d_states, size_t n, int engine, hipStream_t s) {
  if (!n) return;
  if (engine == 2)
    PM16_GO(pm16_permute_kernel, n, s)(d_states, n);
  else if (engine == 1)
    PM_GO(pm_permute_kernel, n, false, s)(d_states, n);
  else
    pg_permute_kernel<<<pg_blocks(n), 256, 0, s>>>(d_states, n);
}

// small draw batches (the query positions, the DEEP coefficients) are one permutation's latency:
// the 48-lane form (~20 us) instead of the 12-lane one (~34 us, round 6 kernel trace)
__global__ __launch_bounds__(256) void draw_wide_kernel(fe seed, const fe* seed_p, uint64_t base, size_t k, fe* out) {
  if (seed_p) seed = *seed_p;
  PW_SETUP();
  const bool live = P.g < PW_PER_WAVE && item < k;
  const uint64_t ctr = base + 1 + (live ? item : 0);
  fe d = pw_sponge<DOM_INT>(P, live, 2, [&](int j) { return j == 0 ? seed : fe{ctr, 0}; });
  if (live && P.e == 0 && P.h == 0) out[item] = d;
}

void launch_draws(fe seed, uint64_t base, size_t k, fe* d_out, hipStream_t s, const fe* d_seed) {
  if (!k) return;
  if (hash_engine() == 1 && k >= pm_min_items())
    PM_GO(draw_pm_kernel, k, false, s)(seed, d_seed, base, k, d_out);
  else if (k <= PW_MAX_ITEMS)
    draw_wide_kernel<<<pw_blocks(k), 256, 0, s>>>(seed, d_seed, base, k, d_out);
  else
    draw_kernel<<<pg_blocks(k), 256, 0, s>>>(seed, d_seed, base, k, d_out);
}

void launch_grind(fe seed, uint64_t base, uint32_t count, uint32_t bits, unsigned long long* d_best, hipStream_t s,
                  const fe* d_seed) {
  if (hash_engine() == 1 && count >= pm_min_items())
    PM_GO(grind_pm_kernel, count, false, s)(seed, d_seed, base, count, bits, d_best);
  else
    grind_kernel<<<pg_blocks(count), 256, 0, s>>>(seed, d_seed, base, count, bits, d_best);
}

// ---- device transcript steps (DefaultRandomCoin on the device; one wave, group 0) --------
// (the reseeds after the trace, constraint and FRI layer trees run in the tree's last launch,
// merkle_top_kernel's coin_mode)
// FRI remainder (agg/trace.rs:926-952 geometry): the rlen lowest coefficients of the Nr last
// evaluations over 3 <w_Nr> (c_k = sum_j ev_j w^-jk / Nr * 3^-k), stored highest degree first
// in rem[0..rlen), rem[rlen] = hash_elements(rem), then coin[0] = merge(coin[0], rem[rlen]).
struct RemArgs {
  fe wk[16];   // w^-k, k < rlen
  fe sk[16];   // 3^-k / Nr
};
__global__ __launch_bounds__(64) void fri_remainder_kernel(const fe* ev, uint32_t Nr, uint32_t rlen, RemArgs A, fe* coin,
                                                           fe* rem) {
  __shared__ __align__(16) uint32_t pw_lds[PW_WAVE_WORDS];
  __shared__ fe c[16];
  const uint32_t t = threadIdx.x;
  if (t < rlen) {
    fe acc = fe_zero(), p = fe_one();
    for (uint32_t j = 0; j < Nr; j++) {
      acc = fe_add(acc, fe_mul(ev[j], p));
      p = fe_mul(p, A.wk[t]);
    }
    c[rlen - 1 - t] = fe_mul(acc, A.sk[t]);
  }
  __syncthreads();
  PWGroup P;
  pw_init(P, pw_lds);
  const bool live = P.g == 0;
  fe d = pw_sponge<DOM_ELEMS>(P, live, (int)((rlen + 1) / 2), [&](int j) {
    return fold_pair(c[2 * j], (uint32_t)(2 * j + 1) < rlen ? c[2 * j + 1] : fe_zero());
  });
  d = pw_bcast(P, d, 0);
  const fe seed = coin[0];
  const fe s1 = pw_sponge<DOM_MERGE>(P, live, 2, [&](int j) { return j == 0 ? seed : d; });
  if (t == 0) {
    coin[0] = s1;
    rem[rlen] = d;
  }
  if (t < rlen) rem[t] = c[t];
}
void launch_fri_remainder(const fe* d_ev, uint32_t Nr, uint32_t rlen, const fe* wk, const fe* sk, fe* d_coin, fe* d_rem,
                          hipStream_t s) {
  if (rlen < 1 || rlen > 16 || rlen > Nr) throw std::invalid_argument("FRI remainder: rem_deg + 1 must be in 1..16");
  RemArgs A{};
  for (uint32_t k = 0; k < rlen; k++) { A.wk[k] = wk[k]; A.sk[k] = sk[k]; }
  fri_remainder_kernel<<<1, 64, 0, s>>>(d_ev, Nr, rlen, A, d_coin, d_rem);
}

// query seed: coin[1] = merge_with_int(coin[0], *best) when grinding found a nonce
__global__ __launch_bounds__(64) void query_seed_kernel(fe* coin, const unsigned long long* best) {
  __shared__ __align__(16) uint32_t pw_lds[PW_WAVE_WORDS];
  const unsigned long long b = *best;
  if (b == ~0ull) return;  // wave-uniform: no nonce yet, the host continues the search
  PWGroup P;
  pw_init(P, pw_lds);
  const bool live = P.g == 0;
  const fe seed = coin[0];
  const fe q = pw_sponge<DOM_INT>(P, live, 2, [&](int j) { return j == 0 ? seed : fe{(uint64_t)b, 0}; });
  if (threadIdx.x == 0) coin[1] = q;
}
void launch_query_seed(fe* d_coin, const unsigned long long* d_best, hipStream_t s) {
  query_seed_kernel<<<1, 64, 0, s>>>(d_coin, d_best);
}

// FRI layer leaves: hash_elements([e_i, e_{i+Nd/2}]) (FriProver::build_layer, folding 2)
__global__ PG_KERNEL void fri_leaf_kernel(const fe* ev, size_t half, fe* leaves) {
  PG_SETUP();
  const bool live = P.g < PG_PER_WAVE && item < half;
  const size_t i = live ? item : 0;
  fe d = pg_sponge<DOM_ELEMS>(P, live, 1, [&](int) { return fold_pair(ev[i], ev[i + half]); });
  if (live && P.j == 0) leaves[i] = d;
}
__global__ __launch_bounds__(256) void fri_leaf_wide_kernel(const fe* ev, size_t half, fe* leaves) {
  PW_SETUP();
  const bool live = P.g < PW_PER_WAVE && item < half;
  const size_t i = live ? item : 0;
  fe d = pw_sponge<DOM_ELEMS>(P, live, 1, [&](int) { return fold_pair(ev[i], ev[i + half]); });
  if (live && P.e == 0 && P.h == 0) leaves[i] = d;
}
void launch_fri_leaves(const fe* d_ev, size_t Nd, fe* d_leaves, hipStream_t s) {
  size_t h = Nd / 2;
  if (h <= PW_MAX_ITEMS)
    fri_leaf_wide_kernel<<<pw_blocks(h), 256, 0, s>>>(d_ev, h, d_leaves);
  else if (hash_engine() == 1 && pm16_range(h))
    PM16_GO(fri_leaf_pm16_kernel, h, s)(d_ev, h, d_leaves);
  else if (hash_engine() == 1 && h >= pm_min_items())
    PM_GO(fri_leaf_pm_kernel, h, false, s)(d_ev, h, d_leaves);
  else
    fri_leaf_kernel<<<pg_blocks(h), 256, 0, s>>>(d_ev, h, d_leaves);
}

}  // namespace zkl

// compiled-in tuning values of this translation unit (zkl_hip_build_config; every value is a
// supported configuration, tests/test_abi.py checks the shipped build carries the defaults)
#define ZKL_STR2(x) #x
#define ZKL_STR(x) ZKL_STR2(x)
#ifndef ZKL_POSEIDON_SCHED_NAME
#define ZKL_POSEIDON_SCHED_NAME default
#endif
namespace zkl {
const char* poseidon_build_config() {
  return "PM_WAVES=" ZKL_STR(PM_WAVES_CFG) ";PM_WIDE=" ZKL_STR(PM_WIDE_CFG) ";PM_ROW_WAVES=" ZKL_STR(
      PM_ROW_WAVES_CFG) ";PM_IGLP=" ZKL_STR(PM_IGLP_CFG) ";TAIL_PRIO=" ZKL_STR(TAIL_PRIO_CFG) ";PW_MAX_ITEMS=" ZKL_STR(
      PW_MAX_ITEMS_CFG) ";PM_ROW_BIG=" ZKL_STR(PM_ROW_BIG_CFG) ";POSEIDON_SCHED=" ZKL_STR(
      ZKL_POSEIDON_SCHED_NAME) ";PM_PRUNE=" ZKL_STR(PM_PRUNE_CFG)
      ";TOP_LDS=" ZKL_STR(TOP_LDS_CFG) ";TOP_WAVES=" ZKL_STR(TOP_WAVES_CFG);
}
}  // namespace zkl
