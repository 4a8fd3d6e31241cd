// gfx950 kernels for the zk-lisp segment prover.
//
// Hot loops: A = Poseidon row hashing + Merkle trees (hash_rows_kernel,
// merge_parts_kernel, merkle_level_kernel, fri_leaf_kernel), B = constraint evaluation
// (constraint_eval_kernel), C = NTTs (ntt_pass_kernel), D = grinding (grind_kernel).
// All arithmetic is exact f128 (field.h); bit-exactness against the oracle follows from
// computing the same residues, independent of evaluation order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <stdexcept>
#include <vector>

#include "kernels.h"
#include "air_eval.h"

namespace zkl {


void upload_air_consts(ProofConsts* dK, const AirDevice& a, hipStream_t s) {
  ZKL_HIPCHECK(hipMemcpyAsync(&dK->air, &a, sizeof a, hipMemcpyHostToDevice, s));
}
void upload_alphas_from_device(ProofConsts* dK, const fe* d, int n, hipStream_t s) {
  if (n > 1024) throw std::invalid_argument("more than 1024 transition constraints");
  ZKL_HIPCHECK(hipMemcpyAsync(dK->alpha, d, sizeof(fe) * n, hipMemcpyDeviceToDevice, s));
}
static void limbs26(fe a, uint32_t l[5]);
void upload_deep_coeffs(ProofConsts* dK, const fe* h, int n, hipStream_t s) {
  // deep_kernel's unreduced 64-bit digit columns stay below the 2^62 REDC bound for at most 256
  // terms (column 3 takes four 26 x 26-bit products per term, < 2^54)
  if (n > 256) throw std::invalid_argument("more than 256 DEEP coefficients (W + C)");
  ZKL_HIPCHECK(hipMemcpyAsync(dK->deep, h, sizeof(fe) * n, hipMemcpyHostToDevice, s));
  static thread_local std::vector<uint32_t> m;
  m.assign((size_t)n * 5, 0);
  const fe R = fe_pow64(fe{2, 0}, 156);
  for (int i = 0; i < n; i++) limbs26(fe_mul(h[i], R), &m[(size_t)i * 5]);
  ZKL_HIPCHECK(hipMemcpyAsync(dK->deep_m, m.data(), m.size() * 4, hipMemcpyHostToDevice, s));
  ZKL_HIPCHECK(hipStreamSynchronize(s));  // m is reused by the next proof on this thread
}

// =====================================================================================
// Poseidon (poseidon/hasher.rs:173-190): 27 rounds of x^3 on all 12 lanes, dense MDS, +rc.
// The MDS row sum is accumulated unreduced (288-bit) and reduced once per lane.
// =====================================================================================
// ---- Montgomery arithmetic on 5 x 26-bit limbs (R = 2^156) ---------------------------
// p = 1 + 0x3F4C000*2^26 + (2^26-1)*2^52 + (2^26-1)*2^78 + (2^24-1)*2^104, and p == 1
// (mod 2^26), so the REDC quotient digit is m = -x mod 2^26 with no multiplication.
// Products accumulate in 64-bit columns by v_mad_u64_u32 with no carry handling: with
// limbs < 2^28 a column holds at most 60 products < 2^56, far below 2^64.  Values are
// kept lazily reduced (< 2^130) inside the permutation and canonicalised on output.
__constant__ HasherMont c_hm;

constexpr uint32_t M26 = 0x3FFFFFFu;

__host__ __device__ __forceinline__ void to26(fe a, uint32_t l[5]) {
  l[0] = (uint32_t)a.lo & M26;
  l[1] = (uint32_t)(a.lo >> 26) & M26;
  l[2] = (uint32_t)((a.lo >> 52) | (a.hi << 12)) & M26;
  l[3] = (uint32_t)(a.hi >> 14) & M26;
  l[4] = (uint32_t)(a.hi >> 40);
}

// col[0..9] = X (< 2^262, columns < 2^62); out = X * 2^-156 mod p + (0 or p): normalised
// 26-bit limbs of a value in (0, 2^130).  p = 1 + 45*2^14*2^26 ... written in columns is
// p = 2^0 + 737280*2^26 - 2^24*2^104 (... - 45*2^40 + 2^128), so removing m*p*2^(26i)
// from X touches only three columns: col_i -= m (exact: m = col_i mod 2^26, the rest
// carries), col_{i+1} += 737280*m, col_{i+4} -= 2^24*m.  Columns are signed; adding
// p*2^156 up front (col_6 += 1, col_7 -= 737280, col_9 += 2^50) keeps the result positive.
__host__ __device__ __forceinline__ void redc(uint64_t colu[10], uint32_t out[5]) {
  int64_t col[10];
#pragma unroll
  for (int i = 0; i < 10; i++) col[i] = (int64_t)colu[i];
  col[6] += 1;
  col[7] -= 737280;
  col[9] += (int64_t)1 << 50;
  // opaque copies of the two reduction constants: keeps -2^24*m a single v_mad_i64_i32
  // instead of a 64-bit shift + subtract
  int32_t kneg = -16777216;
  uint32_t k45 = 737280u;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(kneg), "+s"(k45));
#endif
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint32_t m = (uint32_t)col[i] & M26;
    col[i + 1] += col[i] >> 26;
    col[i + 1] += (int64_t)((uint64_t)m * k45);
    col[i + 4] += (int64_t)(int32_t)m * (int64_t)kneg;
  }
  int64_t c = 0;
#pragma unroll
  for (int t = 0; t < 3; t++) {
    const int64_t v = col[6 + t] + c;
    out[t] = (uint32_t)v & M26;
    c = v >> 26;
  }
  const int64_t v = col[9] + c;
  out[3] = (uint32_t)v & M26;
  out[4] = (uint32_t)(v >> 26);
}

// REDC with R' = 2^130 (the matrix-core permutation's radix): five digit steps instead of
// six.  col[0..8] = X < 2^262 (columns < 2^62); out = X * 2^-130 mod p + (0 or p), the
// normalised limbs of a value in (0, X / 2^130 + p): inputs < 2^129 give outputs < 2^129
// (2^258 / 2^130 + p < 2^129), inputs < 2^130 outputs < 2^131.  The bias p * 2^130 is
// col_5 += 1, col_6 -= 737280, col_9 += 2^24; limb 4 of the output carries everything
// above bit 104 (< 2^28).
__host__ __device__ __forceinline__ void redc130(uint64_t colu[10], uint32_t out[5]) {
  int64_t col[10];
#pragma unroll
  for (int i = 0; i < 10; i++) col[i] = (int64_t)colu[i];
  col[5] += 1;
  col[6] -= 737280;
  col[9] += (int64_t)1 << 24;
  int32_t kneg = -16777216;
  uint32_t k45 = 737280u;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(kneg), "+s"(k45));
#endif
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint32_t m = (uint32_t)col[i] & M26;
    col[i + 1] += col[i] >> 26;
    col[i + 1] += (int64_t)((uint64_t)m * k45);
    col[i + 4] += (int64_t)(int32_t)m * (int64_t)kneg;
  }
  int64_t c = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const int64_t v = col[5 + t] + c;
    out[t] = (uint32_t)v & M26;
    c = v >> 26;
  }
  out[4] = (uint32_t)(col[9] + c);
}

__host__ __device__ __forceinline__ void mac5(const uint32_t a[5], const uint32_t b[5], uint64_t col[10]) {
#pragma unroll
  for (int u = 0; u < 5; u++)
#pragma unroll
    for (int v = 0; v < 5; v++) col[u + v] += (uint64_t)a[u] * b[v];
}

__host__ __device__ __forceinline__ void mont_mul(const uint32_t a[5], const uint32_t b[5], uint32_t out[5]) {
  uint64_t col[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  mac5(a, b, col);
  redc(col, out);
}

__host__ __device__ __forceinline__ void mont_cube(const uint32_t a[5], uint32_t out[5]) {
  uint64_t col[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t d[5];
#pragma unroll
  for (int u = 0; u < 5; u++) d[u] = a[u] << 1;
#pragma unroll
  for (int u = 0; u < 5; u++) {
    col[2 * u] += (uint64_t)a[u] * a[u];
#pragma unroll
    for (int v = u + 1; v < 5; v++) col[u + v] += (uint64_t)d[u] * a[v];
  }
  uint32_t sq[5];
  redc(col, sq);
  mont_mul(sq, a, out);
}

// x^3 R'^-2 (R' = 2^130) with the squaring shortcut; inputs < 2^129 give outputs < 2^129,
// inputs < 2^130 (a state element right after absorbing a message) outputs < 2^131
__host__ __device__ __forceinline__ void mont_cube130(const uint32_t a[5], uint32_t out[5]) {
  uint64_t col[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t d[5];
#pragma unroll
  for (int u = 0; u < 5; u++) d[u] = a[u] << 1;
#pragma unroll
  for (int u = 0; u < 5; u++) {
    col[2 * u] += (uint64_t)a[u] * a[u];
#pragma unroll
    for (int v = u + 1; v < 5; v++) col[u + v] += (uint64_t)d[u] * a[v];
  }
  uint32_t sq[5];
  redc130(col, sq);
  uint64_t c2[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  mac5(sq, a, c2);
  redc130(c2, out);
}

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

enum { DOM_ELEMS = 0, DOM_MERGE = 1, DOM_MANY = 2, DOM_INT = 3 };

static void limbs26(fe a, uint32_t l[5]) {
  l[0] = (uint32_t)a.lo & M26;
  l[1] = (uint32_t)(a.lo >> 26) & M26;
  l[2] = (uint32_t)((a.lo >> 52) | (a.hi << 12)) & M26;
  l[3] = (uint32_t)(a.hi >> 14) & M26;
  l[4] = (uint32_t)(a.hi >> 40);
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
// (COLS = 12 / SPLIT).  Each lane sums its COLS products and reduces them (REDC is linear:
// REDC(a) + REDC(b) == (a + b) R^-1 mod p, and each output is < p + 2^109 since R = 2^156
// >> p, so the sum of four plus a round constant keeps limbs < 2^28.4, inside the bounds
// mont_cube and redc assume); the lanes of an element add their reduced parts with DPP
// quad permutes instead of a second LDS exchange.  One state per wave at SPLIT 4 (lanes
// 48..63 idle), two at SPLIT 2.  Used where a level has too few states to fill the SIMDs
// (upper Merkle levels, small FRI layers, the FRI transcript): one permutation's dependency
// chain bounds those levels.
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
  uint32_t m[PW_COLS][5];  // MDS row e, columns COLS*h .. (Montgomery)
  uint32_t* x;             // cubes: x[limb * 12 + e]
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
    for (int l = 0; l < 5; l++) P.m[k][l] = c_hm.mds[P.e][PW_COLS * P.h + k][l];
}

// sum of v over the SPLIT lanes of this lane's element (DPP quad_perm [1,0,3,2], [2,3,0,1])
__device__ __forceinline__ uint32_t pw_elem_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  if (PW_SPLIT == 4) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  return v;
}

__device__ __forceinline__ void pw_permute(PWGroup& P, uint32_t s[5]) {
  const uint32_t* rcp = &c_hm.rc[0][P.e][0];
#pragma unroll 1
  for (int r = 0; r < 27; r++, rcp += 60) {
    uint32_t rc[5];
#pragma unroll
    for (int l = 0; l < 5; l++) rc[l] = rcp[l];
    uint32_t t[5];
    mont_cube(s, t);
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
    uint64_t col[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < PW_COLS; k++) mac5(tk[k], P.m[k], col);
    uint32_t part[5];
    redc(col, part);
#pragma unroll
    for (int l = 0; l < 5; l++) s[l] = pw_elem_sum(part[l]) + rc[l];
  }
}

template <int D, class Loader>
__device__ __forceinline__ fe pw_sponge(PWGroup& P, bool live, int nmsg, Loader ld) {
  uint32_t s[5];
#pragma unroll
  for (int l = 0; l < 5; l++)
    s[l] = P.e == 0 ? c_hm.dfe[D][l] : P.e == 10 ? c_hm.dom[0][l] : P.e == 11 ? c_hm.dom[1][l] : 0u;
  const int T = nmsg + 1;
  for (int b = 0; b * 10 < T; b++) {
    const int idx = b * 10 + P.e;
    if (live && P.e < 10 && idx >= 1 && idx < T) {
      uint32_t m[5];
      to_mont(ld(idx - 1), m);
#pragma unroll
      for (int l = 0; l < 5; l++) s[l] += m[l];
    }
    pw_permute(P, s);
  }
  return from_mont(s);  // state element 0 in lanes with e == 0
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

__global__ PG_KERNEL void draw_kernel(fe seed, uint64_t base, size_t k, fe* out) {
  PG_SETUP();
  const bool live = P.g < PG_PER_WAVE && item < k;
  const uint64_t ctr = base + 1 + item;
  fe d = pg_sponge<DOM_INT>(P, live, 2, [&](int j) { return j == 0 ? seed : fe{ctr, 0}; });
  if (live && P.j == 0) out[item] = d;
}

__global__ PG_KERNEL void grind_kernel(fe seed, uint64_t base, uint32_t count, uint32_t bits,
                                                    unsigned long long* best) {
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

__global__ __launch_bounds__(256) void merkle_level_wide_kernel(fe* nodes, size_t lvl) {
  PW_SETUP();
  const bool live = P.g < PW_PER_WAVE && item < lvl;
  const size_t i = lvl + (live ? item : 0);
  fe d = pw_sponge<DOM_MERGE>(P, live, 2, [&](int j) { return nodes[2 * i + j]; });
  if (live && P.e == 0 && P.h == 0) nodes[i] = d;
}

// Tree top: several levels per launch.  Workgroup g (4 waves, 8 wide groups, one wave per
// SIMD) owns nodes [cnt*g, cnt*g + cnt) of level lvl and reduces them to one node of level
// lvl/cnt, with a workgroup barrier between levels; waves without a live node skip the
// permutation.  A launch per level would add ~10 us of dispatch latency to each of these
// permutation-latency-bound levels.
constexpr int TOP_WAVES = 8 / PW_PER_WAVE;
constexpr int TOP_SLOTS = TOP_WAVES * PW_PER_WAVE;  // 8
__global__ __launch_bounds__(64 * TOP_WAVES) void merkle_top_kernel(fe* nodes, size_t lvl, int cnt) {
  __shared__ __align__(16) uint32_t pw_lds[TOP_WAVES * PW_WAVE_WORDS];
  PWGroup P;
  pw_init(P, pw_lds);
  const int wave_slot0 = (int)(threadIdx.x >> 6) * PW_PER_WAVE;
  const int slot = wave_slot0 + P.g;
  size_t L = lvl, base = (size_t)blockIdx.x * cnt;
  for (int c = cnt; c >= 1; c >>= 1, L >>= 1, base >>= 1) {
    if (wave_slot0 < c) {  // wave-uniform
      const bool live = P.g < PW_PER_WAVE && slot < c;
      const size_t i = L + base + (live ? slot : 0);
      fe d = pw_sponge<DOM_MERGE>(P, live, 2, [&](int j) { return nodes[2 * i + j]; });
      if (live && P.e == 0 && P.h == 0) nodes[i] = d;
    }
    __syncthreads();
  }
}

void launch_merkle(fe* d_nodes, size_t n, hipStream_t s) {
  for (size_t lvl = n / 2; lvl >= 1;) {
    if (lvl <= PW_MAX_ITEMS) {
      const size_t cnt = std::min<size_t>(lvl, TOP_SLOTS);
      merkle_top_kernel<<<(unsigned)(lvl / cnt), 64 * TOP_WAVES, 0, s>>>(d_nodes, lvl, (int)cnt);
      lvl /= cnt * 2;
      continue;
    }
    if (hash_engine() == 1 && lvl >= pm_min_items())
      PM_GO(merkle_level_pm_kernel, lvl, false, s)(d_nodes, lvl);
    else
      merkle_level_kernel<<<pg_blocks(lvl), 256, 0, s>>>(d_nodes, lvl);
    lvl /= 2;
  }
}

// FRI transcript step on the device (DefaultRandomCoin: reseed with the layer root, then
// draw alpha with counter 1): coin[0] = merge(coin[0], root); coin[1] = merge_with_int(
// coin[0], 1); the root is also copied to *root_out.  One wave, group 0.
__global__ __launch_bounds__(64) void fri_coin_kernel(fe* coin, const fe* root, fe* root_out) {
  __shared__ __align__(16) uint32_t pw_lds[PW_WAVE_WORDS];
  PWGroup P;
  pw_init(P, pw_lds);
  const bool live = P.g == 0;
  const fe seed = coin[0], r = *root;
  fe s1 = pw_sponge<DOM_MERGE>(P, live, 2, [&](int j) { return j == 0 ? seed : r; });
  s1 = pw_bcast(P, s1, 0);
  fe a = pw_sponge<DOM_INT>(P, live, 2, [&](int j) { return j == 0 ? s1 : fe{1, 0}; });
  if (threadIdx.x == 0) {
    coin[0] = s1;
    coin[1] = a;
    *root_out = r;
  }
}
void launch_fri_coin(fe* d_coin, const fe* d_root, fe* d_root_out, hipStream_t s) {
  fri_coin_kernel<<<1, 64, 0, s>>>(d_coin, d_root, d_root_out);
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
  if (engine == 1)
    PM_GO(pm_permute_kernel, n, false, s)(d_states, n);
  else
    pg_permute_kernel<<<pg_blocks(n), 256, 0, s>>>(d_states, n);
}

void launch_draws(fe seed, uint64_t base, size_t k, fe* d_out, hipStream_t s) {
  if (!k) return;
  if (hash_engine() == 1 && k >= pm_min_items())
    PM_GO(draw_pm_kernel, k, false, s)(seed, base, k, d_out);
  else
    draw_kernel<<<pg_blocks(k), 256, 0, s>>>(seed, base, k, d_out);
}

void launch_grind(fe seed, uint64_t base, uint32_t count, uint32_t bits, unsigned long long* d_best, hipStream_t s) {
  if (hash_engine() == 1 && count >= pm_min_items())
    PM_GO(grind_pm_kernel, count, false, s)(seed, base, count, bits, d_best);
  else
    grind_kernel<<<pg_blocks(count), 256, 0, s>>>(seed, base, count, bits, d_best);
}

// =====================================================================================
// NTT: in-place radix-2 passes, up to 8 stages per pass staged through LDS.
// A pass covers global half-sizes H in {S, 2S, .., 2^(r-1) S}.  Group q of 2^r elements:
// L = q mod S, Hb = q / S, element t at Hb*S*2^r + t*S + L.  4096 elements per workgroup.
// =====================================================================================
#ifndef NTT_ELEMS_CFG
#define NTT_ELEMS_CFG 1024
#endif
#ifndef NTT_THREADS_CFG
#define NTT_THREADS_CFG 256
#endif
constexpr int NTT_ELEMS = NTT_ELEMS_CFG;      // elements per workgroup (1024: 17 KB of LDS)
constexpr int NTT_THREADS = NTT_THREADS_CFG;  // threads per workgroup

__device__ __forceinline__ uint32_t bitrev(uint32_t x, int logn) { return logn ? (__brev(x) >> (32 - logn)) : 0; }

// x * w for a twiddle w given as limbs of w*2^156 (MontTab): REDC(x * wR) = x*w, then one
// conditional subtraction makes it canonical.
__host__ __device__ __forceinline__ fe mul_tw(fe a, MontTab t, size_t e) {
  const uint4 q = t.l4[e];
  const uint32_t wm[5] = {q.x, q.y, q.z, q.w, t.l1[e]};
  uint32_t l[5], o[5];
  to26(a, l);
  mont_mul(l, wm, o);
  // the REDC result lies in (0, p + 2^100): bit 128 (limb 4, bit 24) may be set
  typedef unsigned __int128 u128;
  const u128 v = (u128)o[0] + ((u128)o[1] << 26) + ((u128)o[2] << 52) + ((u128)o[3] << 78) + ((u128)o[4] << 104);
  const u128 P = ((u128)P_HI << 64) | P_LO;
  const u128 r = (o[4] >> 24) ? v + C_RED : (v >= P ? v - P : v);  // v wrapped mod 2^128: Y - p = v + C
#ifdef NTT_CHECK
  {
    uint64_t cc[10] = {wm[0], wm[1], wm[2], wm[3], wm[4], 0, 0, 0, 0, 0};
    uint32_t wl[5];
    redc(cc, wl);
    u128 wv = (u128)wl[0] + ((u128)wl[1] << 26) + ((u128)wl[2] << 52) + ((u128)wl[3] << 78) + ((u128)wl[4] << 104);
    if (wv >= P) wv -= P;
    fe want = fe_mul(a, fe{(uint64_t)wv, (uint64_t)(wv >> 64)});
    if (want.lo != (uint64_t)r || want.hi != (uint64_t)(r >> 64))
      printf("mul_tw mismatch e=%lu a=%016lx%016lx got=%016lx%016lx want=%016lx%016lx o=%x %x %x %x %x\n", (unsigned long)e,
             (unsigned long)a.hi, (unsigned long)a.lo, (unsigned long)(uint64_t)(r >> 64), (unsigned long)(uint64_t)r,
             (unsigned long)want.hi, (unsigned long)want.lo, o[0], o[1], o[2], o[3], o[4]);
  }
#endif
  return fe{(uint64_t)r, (uint64_t)(r >> 64)};
}

// Stage-major twiddle layout: entry H + j = w_(2H)^j for H = 1, 2, 4, .., N/2 and j < H, so
// the twiddles of one radix-2 stage are contiguous (coalesced across consecutive L, and the
// small stages of a pass share a few KB that stay in L2).  Valid for any NTT size <= N.
void build_mont_table(const fe* w, size_t N, void* d_buf, hipStream_t s) {
  const fe R = fe_pow64(fe{2, 0}, 156);
  std::vector<uint32_t> l4(4 * N, 0), l1(N, 0);
  for (size_t H = 1; H < N; H *= 2) {
    const size_t step = N / (2 * H);
    for (size_t j = 0; j < H; j++) {
      uint32_t l[5];
      limbs26(fe_mul(w[j * step], R), l);
      for (int t = 0; t < 4; t++) l4[4 * (H + j) + t] = l[t];
      l1[H + j] = l[4];
    }
  }
  ZKL_HIPCHECK(hipMemcpyAsync(d_buf, l4.data(), N * 16, hipMemcpyHostToDevice, s));
  ZKL_HIPCHECK(hipMemcpyAsync((char*)d_buf + N * 16, l1.data(), N * 4, hipMemcpyHostToDevice, s));
  ZKL_HIPCHECK(hipStreamSynchronize(s));
}

// src != nullptr (first DIT pass of an LDE): element i of column c is read from
// src[c * (N >> src_logb) + (i >> src_logb)] instead of data, i.e. the blowup copies of the
// (scaled, bit-reversed) coefficients are generated on load rather than materialised.
template <bool DIF>
__global__ __launch_bounds__(NTT_THREADS) void ntt_pass_kernel(fe* __restrict__ data, size_t ncols, int logN, int r,
                                                       int logS, MontTab roots, int logTab, const fe* __restrict__ src,
                                                       int src_logb) {
  __shared__ fe buf[NTT_ELEMS + NTT_ELEMS / 16];
  const int R = 1 << r;
  const int G = NTT_ELEMS >> r;
  const size_t S = (size_t)1 << logS;
  const int log_gpc = logN - r;  // groups per column = N / R
  const size_t gpc = (size_t)1 << log_gpc;
  const bool gfast = S >= (size_t)G;
  const int pitch = R >= 16 ? R + 1 : R;  // pad: conflict-free 16-byte accesses
  // Block -> groups.  When a column holds whole blocks, consecutive blocks walk the columns
  // at a fixed group range, so concurrently running blocks share twiddles (same L) in L2.
  size_t col_fixed = 0, qbase = 0;
  const bool whole = gpc >= (size_t)G;
  if (whole) {
    col_fixed = blockIdx.x % (unsigned)ncols;
    qbase = (size_t)(blockIdx.x / (unsigned)ncols) * G;
  }
  auto locate = [&](int g, size_t& col, size_t& q) -> bool {
    if (whole) {
      col = col_fixed;
      q = qbase + g;
      return true;
    }
    const size_t qg = (size_t)blockIdx.x * G + g;
    col = qg >> log_gpc;
    q = qg & (gpc - 1);
    return col < ncols;
  };
  auto addr = [&](int g, int t, bool& ok) -> size_t {
    size_t col, q;
    ok = locate(g, col, q);
    const size_t L = q & (S - 1), Hb = q >> logS;
    return (col << logN) + ((Hb << logS) << r) + (size_t)t * S + L;
  };
  const size_t Nmask = ((size_t)1 << logN) - 1;
  for (int e = threadIdx.x; e < NTT_ELEMS; e += NTT_THREADS) {
    int g = gfast ? (e % G) : (e >> r);
    int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    size_t a = addr(g, t, ok);
    fe v = fe_zero();
    if (ok) v = src ? src[((a >> logN) << (logN - src_logb)) + ((a & Nmask) >> src_logb)] : data[a];
    buf[g * pitch + t] = v;
  }
  __syncthreads();
  for (int st = 0; st < r; st++) {
    const int lh = DIF ? (r - 1 - st) : st;  // log2 of local half size
    const int h = 1 << lh;
    const size_t Hs = (size_t)h << logS;  // global half size: stage table base
    // the four butterflies of a thread are disjoint: load all operands, then compute and store
    constexpr int BPT = NTT_ELEMS / 2 / NTT_THREADS;
    fe x0[BPT], x1[BPT];
    size_t te[BPT];
    int o0[BPT];
#pragma unroll
    for (int i = 0; i < BPT; i++) {
      // groups vary fastest across lanes: consecutive lanes take consecutive L, so the
      // twiddle loads w_(2H)^(k*S + L) are contiguous in the root table
      const int u = threadIdx.x + NTT_THREADS * i;
      const int g = u % G;
      const int w = u / G;
      const int k = w & (h - 1);
      const int t0 = ((w >> lh) << (lh + 1)) + k;
      size_t colx, q;
      locate(g, colx, q);
      const size_t L = q & (S - 1);
      te[i] = Hs + ((size_t)k << logS) + L;
      o0[i] = g * pitch + t0;
      x0[i] = buf[o0[i]];
      x1[i] = buf[o0[i] + h];
    }
#pragma unroll
    for (int i = 0; i < BPT; i++) {
      if (DIF) {
        buf[o0[i]] = fe_add(x0[i], x1[i]);
        buf[o0[i] + h] = mul_tw(fe_sub(x0[i], x1[i]), roots, te[i]);
      } else {
        const fe v = mul_tw(x1[i], roots, te[i]);
        buf[o0[i]] = fe_add(x0[i], v);
        buf[o0[i] + h] = fe_sub(x0[i], v);
      }
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < NTT_ELEMS; e += NTT_THREADS) {
    int g = gfast ? (e % G) : (e >> r);
    int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    size_t a = addr(g, t, ok);
    if (ok) data[a] = buf[g * pitch + t];
  }
}

// DIT pass with lazily reduced 26-bit limbs (the LDE evaluation passes).  Elements enter
// LDS as five limbs (struct of arrays), every butterfly is v = REDC(x1 * wR) (normalised,
// < 2^130), y0 = x0 + v, y1 = x0 + Q - v with Q = 8p written with every limb >= 2^26, and
// only the pass output is reduced to canonical form.  Limbs grow by at most 2^27 per stage,
// so after 8 stages they stay below 2^31 and every product term stays below 2^57 (the
// REDC input bound).  ~40% fewer instructions per butterfly than the canonical form
// (no per-butterfly canonicalisation, limbwise add/sub).
constexpr uint32_t NTT_Q[5] = {67108872u, 128319487u, 134217726u, 134217726u, 134217726u};  // 8p

__device__ __forceinline__ fe ntt_canon(const uint32_t l[5]) {
  typedef unsigned __int128 u128;
  // limbs < 2^31: the low part is < 2^110, adding limb 4's low 24 bits at 2^104 may carry
  // past 2^128, and limb 4's high bits sit at 2^128 (t < 2^7)
  const u128 lo = (u128)l[0] + ((u128)l[1] << 26) + ((u128)l[2] << 52) + ((u128)l[3] << 78);
  const u128 v = lo + ((u128)(l[4] & 0xFFFFFFu) << 104);
  const uint32_t t = (l[4] >> 24) + (v < lo ? 1u : 0u);
  const u128 P = ((u128)P_HI << 64) | P_LO;
  u128 r = v + (u128)t * C_RED;  // 2^128 == C_RED
  if (r < v) r += C_RED;
  if (r >= P) r -= P;
  return fe{(uint64_t)r, (uint64_t)(r >> 64)};
}

// ELEMS elements per workgroup: NTT_ELEMS, or 2 * NTT_ELEMS for a pass whose groups would
// otherwise own only half of each 128-byte line they touch (G = ELEMS >> r < 8 consecutive L
// at a stride S >= G: the other half went to a workgroup on another XCD and the line was
// fetched twice -- the 8-stage top pass of the trace LDE fetched 7.1 GB for 3.4 GB)
template <int ELEMS, int THREADS>
__global__ __launch_bounds__(THREADS) void ntt_dit_lazy_kernel(fe* __restrict__ data, size_t ncols, int logN, int r,
                                                                  int logS, MontTab roots, const fe* __restrict__ src,
                                                                  int src_logb) {
  constexpr int PITCHED = ELEMS + ELEMS / 16;
  __shared__ uint4 bufA[PITCHED];     // limbs 0..3 (16-byte accesses, as the canonical kernel)
  __shared__ uint32_t bufB[PITCHED];  // limb 4
  const int R = 1 << r;
  const int G = ELEMS >> r;
  const size_t S = (size_t)1 << logS;
  const int log_gpc = logN - r;
  const size_t gpc = (size_t)1 << log_gpc;
  const bool gfast = S >= (size_t)G;
  const int pitch = R >= 16 ? R + 1 : R;
  size_t col_fixed = 0, qbase = 0;
  const bool whole = gpc >= (size_t)G;
  if (whole) {
    col_fixed = blockIdx.x % (unsigned)ncols;
    qbase = (size_t)(blockIdx.x / (unsigned)ncols) * G;
  }
  auto locate = [&](int g, size_t& col, size_t& q) -> bool {
    if (whole) {
      col = col_fixed;
      q = qbase + g;
      return true;
    }
    const size_t qg = (size_t)blockIdx.x * G + g;
    col = qg >> log_gpc;
    q = qg & (gpc - 1);
    return col < ncols;
  };
  auto addr = [&](int g, int t, bool& ok) -> size_t {
    size_t col, q;
    ok = locate(g, col, q);
    const size_t L = q & (S - 1), Hb = q >> logS;
    return (col << logN) + ((Hb << logS) << r) + (size_t)t * S + L;
  };
  const size_t Nmask = ((size_t)1 << logN) - 1;
  for (int e = threadIdx.x; e < ELEMS; e += THREADS) {
    const int g = gfast ? (e % G) : (e >> r);
    const int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    const size_t a = addr(g, t, ok);
    fe v = fe_zero();
    if (ok) v = src ? src[((a >> logN) << (logN - src_logb)) + ((a & Nmask) >> src_logb)] : data[a];
    uint32_t l[5];
    to26(v, l);
    bufA[g * pitch + t] = make_uint4(l[0], l[1], l[2], l[3]);
    bufB[g * pitch + t] = l[4];
  }
  __syncthreads();
  auto ld = [&](int o, uint32_t x[5]) {
    const uint4 a = bufA[o];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = bufB[o];
  };
  auto st = [&](int o, const uint32_t x[5]) {
    bufA[o] = make_uint4(x[0], x[1], x[2], x[3]);
    bufB[o] = x[4];
  };
  auto tw = [&](size_t e, uint32_t wm[5]) {
    const uint4 q4 = roots.l4[e];
    wm[0] = q4.x; wm[1] = q4.y; wm[2] = q4.z; wm[3] = q4.w; wm[4] = roots.l1[e];
  };
  // y0 = x0 + x1 w, y1 = x0 - x1 w (+Q), in place
  auto bfly = [&](uint32_t x0[5], uint32_t x1[5], const uint32_t wm[5]) {
    uint32_t v[5];
    mont_mul(x1, wm, v);
#pragma unroll
    for (int l = 0; l < 5; l++) {
      x1[l] = x0[l] + NTT_Q[l] - v[l];
      x0[l] = x0[l] + v[l];
    }
  };
  int lh = 0;
  // two stages per LDS round trip: a thread takes the quad t0, t0+h, t0+2h, t0+3h of one
  // group; stage lh pairs (0,1), (2,3) under one twiddle, stage lh+1 pairs (0,2), (1,3)
  for (; lh + 1 < r; lh += 2) {
    const int h = 1 << lh;
    constexpr int QPT = ELEMS / 4 / THREADS;
#pragma unroll
    for (int i = 0; i < QPT; i++) {
      const int u = threadIdx.x + THREADS * i;
      const int g = u % G;
      const int w = u / G;
      const int k = w & (h - 1);
      const int t0 = ((w >> lh) << (lh + 2)) + k;
      size_t colx, q;
      locate(g, colx, q);
      const size_t L = q & (S - 1);
      const int o = g * pitch + t0;
      uint32_t a0[5], a1[5], a2[5], a3[5], w1[5], w2[5], w3[5];
      ld(o, a0); ld(o + h, a1); ld(o + 2 * h, a2); ld(o + 3 * h, a3);
      tw(((size_t)h << logS) + ((size_t)k << logS) + L, w1);
      tw(((size_t)(2 * h) << logS) + ((size_t)k << logS) + L, w2);
      tw(((size_t)(2 * h) << logS) + ((size_t)(k + h) << logS) + L, w3);
      bfly(a0, a1, w1);
      bfly(a2, a3, w1);
      bfly(a0, a2, w2);
      bfly(a1, a3, w3);
      st(o, a0); st(o + h, a1); st(o + 2 * h, a2); st(o + 3 * h, a3);
    }
    __syncthreads();
  }
  if (lh < r) {  // odd stage count: one radix-2 stage
    const int h = 1 << lh;
    constexpr int BPT = ELEMS / 2 / THREADS;
#pragma unroll
    for (int i = 0; i < BPT; i++) {
      const int u = threadIdx.x + THREADS * i;
      const int g = u % G;
      const int w = u / G;
      const int k = w & (h - 1);
      const int t0 = ((w >> lh) << (lh + 1)) + k;
      size_t colx, q;
      locate(g, colx, q);
      const int o = g * pitch + t0;
      uint32_t x0[5], x1[5], wm[5];
      ld(o, x0); ld(o + h, x1);
      tw(((size_t)h << logS) + ((size_t)k << logS) + (q & (S - 1)), wm);
      bfly(x0, x1, wm);
      st(o, x0); st(o + h, x1);
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < ELEMS; e += THREADS) {
    const int g = gfast ? (e % G) : (e >> r);
    const int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    const size_t a = addr(g, t, ok);
    const uint4 a4 = bufA[g * pitch + t];
    const uint32_t l[5] = {a4.x, a4.y, a4.z, a4.w, bufB[g * pitch + t]};
    if (ok) data[a] = ntt_canon(l);
  }
}

// 8-stage DIT pass held in registers: 2048 elements (8 groups of 256 at consecutive L, whole
// 128-byte lines) on 256 threads, 8 elements per thread.  Stages 0-2 run on the elements a
// thread loads straight from HBM (t = 8j + u), stages 3-5 and 6-7 after one LDS exchange each
// (t = a + 8u + 64c, then two quads t = a' + 64u'), and the last quads go straight back to HBM:
// two LDS round trips and two barriers per pass instead of five, the twiddles of a phase
// fetched before the barrier that precedes it.  Same lazy 26-bit limb arithmetic as
// ntt_dit_lazy_kernel (limbs < 2^31 after 8 stages).  Needs S >= 8 and N >> 8 >= 8.
constexpr int NTT8_G = 8;
constexpr int NTT8_THREADS = 256;
constexpr int NTT8_PITCH = 257;
__global__ __launch_bounds__(NTT8_THREADS) __global__ __launch_bounds__(NTT8_THREADS) void ntt_dit8_kernel(fe* __restrict__ data, size_t ncols, int logN, int logS,
                                                                 MontTab roots, const fe* __restrict__ src, int src_logb,
                                                                 int lfast, int split) {
  __shared__ uint4 bufA[NTT8_G * NTT8_PITCH];
  __shared__ uint32_t bufB[NTT8_G * NTT8_PITCH];
  const int tid = (int)threadIdx.x;
  const int g = tid & (NTT8_G - 1), j = tid >> 3;
  // block -> (column, 8 consecutive groups).  lfast = 0: consecutive blocks walk the columns
  // at a fixed group range, so concurrently running blocks share twiddles in L2; lfast = 1:
  // consecutive blocks take consecutive group ranges of one column, so concurrently running
  // blocks read and write neighbouring lines of each row t (DRAM page locality)
  size_t col, q;
  if (lfast) {
    const unsigned gpb = (1u << (logN - 8)) / NTT8_G;
    col = blockIdx.x / gpb;
    q = (size_t)(blockIdx.x % gpb) * NTT8_G + g;
  } else {
    col = blockIdx.x % (unsigned)ncols;
    q = (size_t)(blockIdx.x / (unsigned)ncols) * NTT8_G + g;
  }
  const size_t S = (size_t)1 << logS;
  const size_t L = q & (S - 1), Hb = q >> logS;
  const size_t base = (col << logN) + ((Hb << logS) << 8) + L;
  auto tw = [&](size_t h, size_t k, uint32_t wm[5]) {
    const size_t e = ((h + k) << logS) + L;
    const uint4 q4 = roots.l4[e];
    wm[0] = q4.x; wm[1] = q4.y; wm[2] = q4.z; wm[3] = q4.w; wm[4] = roots.l1[e];
  };
  auto bfly = [&](uint32_t x0[5], uint32_t x1[5], const uint32_t wm[5]) {
    uint32_t v[5];
    mont_mul(x1, wm, v);
#pragma unroll
    for (int l = 0; l < 5; l++) {
      x1[l] = x0[l] + NTT_Q[l] - v[l];
      x0[l] = x0[l] + v[l];
    }
  };
  auto lds_st = [&](int t, const uint32_t x[5]) {
    bufA[g * NTT8_PITCH + t] = make_uint4(x[0], x[1], x[2], x[3]);
    bufB[g * NTT8_PITCH + t] = x[4];
  };
  auto lds_ld = [&](int t, uint32_t x[5]) {
    const uint4 a = bufA[g * NTT8_PITCH + t];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = bufB[g * NTT8_PITCH + t];
  };
  uint32_t x[8][5];
  uint32_t w[7][5];
  // ---- phase A: t = 8j + u, local half sizes 1, 2, 4 (twiddle k = u0 mod h)
  tw(1, 0, w[0]);
  tw(2, 0, w[1]); tw(2, 1, w[2]);
#pragma unroll
  for (int k = 0; k < 4; k++) tw(4, k, w[3 + k]);
  {
    const size_t Nmask = ((size_t)1 << logN) - 1;
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const size_t a = base + (size_t)(8 * j + u) * S;
      const fe v = src ? src[((a >> logN) << (logN - src_logb)) + ((a & Nmask) >> src_logb)] : data[a];
      to26(v, x[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < 8; u += 2) bfly(x[u], x[u + 1], w[0]);
#pragma unroll
  for (int u = 0; u < 8; u += 4) { bfly(x[u], x[u + 2], w[1]); bfly(x[u + 1], x[u + 3], w[2]); }
#pragma unroll
  for (int k = 0; k < 4; k++) bfly(x[k], x[k + 4], w[3 + k]);
#pragma unroll
  for (int u = 0; u < 8; u++) lds_st(8 * j + u, x[u]);
  // ---- phase B: t = a + 8u + 64c, local half sizes 8, 16, 32 (k = a + 8 (u0 mod 2^s))
  const int a = j & 7, c = j >> 3;
  tw(8, a, w[0]);
  tw(16, a, w[1]); tw(16, a + 8, w[2]);
#pragma unroll
  for (int k = 0; k < 4; k++) tw(32, a + 8 * k, w[3 + k]);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 8; u++) lds_ld(a + 8 * u + 64 * c, x[u]);
#pragma unroll
  for (int u = 0; u < 8; u += 2) bfly(x[u], x[u + 1], w[0]);
#pragma unroll
  for (int u = 0; u < 8; u += 4) { bfly(x[u], x[u + 2], w[1]); bfly(x[u + 1], x[u + 3], w[2]); }
#pragma unroll
  for (int k = 0; k < 4; k++) bfly(x[k], x[k + 4], w[3 + k]);
  // in place: the thread's phase-B locations are its own (a partition), no barrier needed
#pragma unroll
  for (int u = 0; u < 8; u++) lds_st(a + 8 * u + 64 * c, x[u]);
  // ---- phase C: two quads t = a' + 64u' (a' = j, j + 32), local half sizes 64, 128
  tw(64, j, w[0]); tw(128, j, w[1]); tw(128, j + 64, w[2]);
  tw(64, j + 32, w[3]); tw(128, j + 32, w[4]); tw(128, j + 96, w[5]);
  __syncthreads();
#pragma unroll
  for (int qd = 0; qd < 2; qd++) {
    const int a2 = j + 32 * qd;
#pragma unroll
    for (int u = 0; u < 4; u++) lds_ld(a2 + 64 * u, x[4 * qd + u]);
    uint32_t* y0 = x[4 * qd];
    uint32_t* y1 = x[4 * qd + 1];
    uint32_t* y2 = x[4 * qd + 2];
    uint32_t* y3 = x[4 * qd + 3];
    bfly(y0, y1, w[3 * qd]);
    bfly(y2, y3, w[3 * qd]);
    bfly(y0, y2, w[3 * qd + 1]);
    bfly(y1, y3, w[3 * qd + 2]);
    // split (last pass only, S = N / 256, so L & 7 = g): row L + t S with t = a2 + 64 u goes to
    // lde_pos = (L - g) + g / 2 + 4 (t & 1) + (t / 2 + 128 (g & 1)) S, i.e. 32 S apart in u
    const size_t at0 = split ? (col << logN) + (L - g) + (g >> 1) + 4 * (a2 & 1) +
                                   ((size_t)((a2 >> 1) + ((g & 1) << 7)) << logS)
                             : base + (size_t)a2 * S;
    const size_t du = split ? 32 * S : 64 * S;
#pragma unroll
    for (int u = 0; u < 4; u++) data[at0 + u * du] = ntt_canon(x[4 * qd + u]);
  }
}

#include "ntt_mfma.inc"

// DIT form: lazy limbs (default) or the canonical kernel (ZKL_NTT=classic, set_ntt_lazy)
static std::atomic<int> g_ntt_lazy{-1};
static bool ntt_lazy_enabled() {
  int v = g_ntt_lazy.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("ZKL_NTT");
    v = (e && !strcmp(e, "classic")) ? 0 : 1;
    g_ntt_lazy.store(v);
  }
  return v != 0;
}
void set_ntt_lazy(bool on) { g_ntt_lazy.store(on ? 1 : 0); }
// measured (profiles/r02, scripts/ab_ntt_wide.sh): the 2048-element / 256-thread form halves
// the top pass's fetch (7.1 -> 3.7 GB) but its passes run no faster (fewer waves per CU hide
// less of the butterfly chains); 2048 elements on 512 threads keeps the waves and gives NTT
// 8.3 -> 8.0 ms per proof: default 2
static int ntt_wide_mode() {
  static const int m = [] {
    const char* e = getenv("ZKL_NTT_WIDE");
    return e ? atoi(e) : 2;
  }();
  return m;
}

// 8-stage register pass (ntt_dit8_kernel) for the lazy DIT passes it covers; ZKL_NTT8=0 keeps
// the LDS-staged kernels (A/B)
static bool ntt8_enabled() {
  static const bool on = [] {
    const char* e = getenv("ZKL_NTT8");
    return !(e && !strcmp(e, "0"));
  }();
  return on;
}

// block order of ntt_dit8_kernel (ZKL_NTT8_MAP): 0 = columns fastest, 1 = group ranges
// fastest, 2 = group ranges fastest for the passes over strides S >= 2048 only
static int ntt8_lfast(int logS) {
  static const int m = [] {
    const char* e = getenv("ZKL_NTT8_MAP");
    return e ? atoi(e) : 0;
  }();
  return m == 1 || (m == 2 && logS >= 11) ? 1 : 0;
}

static int ilog2s(size_t n) { int k = 0; while (((size_t)1 << k) < n) k++; return k; }

// Stage split of one transform into LDS passes.  The pass over the largest stride S (the
// last DIT pass, the first DIF pass) takes at most NTT_TOP_R stages, so a workgroup owns
// G = 1024 >> r >= 8 consecutive L, i.e. whole 128-byte lines of every row it touches (with
// 4 consecutive L a line was split between two workgroups on different XCDs and fetched
// twice); the other passes take up to 10 stages (the lazy kernel's limbs stay below 2^31 for
// 10 stages: 2^26 + 10 * 2^27), split as evenly as possible.  NTT_SPLIT_MODE 0 restores the
// greedy 8-stage split.
#ifndef NTT_TOP_R
#define NTT_TOP_R 6
#endif
#ifndef NTT_SPLIT_MODE
#define NTT_SPLIT_MODE 0  // measured: 8 + 8 = 8.25 ms, 9 + 7 = 8.75 ms, 10 + 6 = 9.8 ms per proof (r02)
#endif
static std::vector<int> ntt_split(int K) {
  std::vector<int> rs;
  if (K <= 0) return rs;
  if (NTT_SPLIT_MODE == 0) {
    for (int left = K; left > 0; left -= std::min(8, left)) rs.push_back(std::min(8, left));
    return rs;  // greedy from the smallest stride
  }
  if (K <= 10) { rs.push_back(K); return rs; }
  int rest = K - NTT_TOP_R;
  const int np = (rest + 9) / 10;
  for (int i = 0; i < np; i++) {
    int r = (rest + (np - i) - 1) / (np - i);
    if ((r & 1) && r < rest && r < 10) r++;  // even stage counts: radix-4 LDS round trips only
    rs.push_back(r);
    rest -= r;
  }
  rs.push_back(NTT_TOP_R);  // ascending-S order (DIT); DIF walks it backwards
  return rs;
}

// DIT passes over stages [lo, hi]: can the last one store the split layout (it must be the
// 8-stage register pass, whose store is the only one that knows the layout)?
static bool dit_split_ok(size_t N, int lo, int hi) {
  if (hi < lo || !ntt_lazy_enabled() || !ntt8_enabled() || ntt_mfma_enabled()) return false;
  const std::vector<int> rs = ntt_split(hi - lo + 1);
  int cur = lo;
  for (size_t k = 0; k + 1 < rs.size(); k++) cur += rs[k];
  return rs.back() == 8 && ((size_t)1 << cur) >= (size_t)NTT8_G && (N >> 8) >= (size_t)NTT8_G;
}

static void ntt_passes(fe* d, size_t ncols, size_t N, bool dif, int lo, int hi, MontTab roots, size_t Ntab,
                       const fe* src, int src_logb, hipStream_t s, int split = 0) {
  int logN = ilog2s(N), logTab = ilog2s(Ntab);
  if (hi < lo) return;
  const std::vector<int> rs = ntt_split(hi - lo + 1);
  if (dif) {
    int cur = hi;
    for (size_t k = rs.size(); k-- > 0;) {
      const int r = rs[k];
      int logS = cur - r + 1;
      size_t groups = (N >> r) * ncols;
      size_t G = NTT_ELEMS >> r;
      ntt_pass_kernel<true><<<(unsigned)((groups + G - 1) / G), NTT_THREADS, 0, s>>>(d, ncols, logN, r, logS, roots, logTab,
                                                                             nullptr, 0);
      cur -= r;
    }
  } else {
    int cur = lo;
    for (size_t ri = 0; ri < rs.size(); ri++) {
      const int r = rs[ri];
      const int split_here = split && ri + 1 == rs.size();
      size_t groups = (N >> r) * ncols;
      size_t G = NTT_ELEMS >> r;
      if (ntt_lazy_enabled()) {
        // wide mode (ZKL_NTT_WIDE): 1 = 2048 elements / 256 threads, 2 = 2048 / 512 for the
        // passes whose 1024-element groups own only half lines (see ntt_dit_lazy_kernel)
        const int wm = ntt_wide_mode();
        const bool wide = wm > 0 && G < 8 && ((size_t)1 << cur) >= G;
        const size_t Gw = wide ? 2 * G : G;
        const unsigned grid = (unsigned)((groups + Gw - 1) / Gw);
        const fe* sp = cur == lo ? src : nullptr;
        if (!split_here && r == 8 && launch_ntt_dit8_mfma(d, ncols, logN, cur, sp, src_logb, s)) {
          cur += r;
          continue;
        }
        if (r == 8 && ntt8_enabled() && ((size_t)1 << cur) >= (size_t)NTT8_G && (N >> 8) >= (size_t)NTT8_G)
          ntt_dit8_kernel<<<(unsigned)(groups / NTT8_G), NTT8_THREADS, 0, s>>>(d, ncols, logN, cur, roots, sp, src_logb,
                                                                              ntt8_lfast(cur), split_here);
        else if (wide && wm == 2)
          ntt_dit_lazy_kernel<2 * NTT_ELEMS, 2 * NTT_THREADS><<<grid, 2 * NTT_THREADS, 0, s>>>(d, ncols, logN, r, cur, roots, sp, src_logb);
        else if (wide)
          ntt_dit_lazy_kernel<2 * NTT_ELEMS, NTT_THREADS><<<grid, NTT_THREADS, 0, s>>>(d, ncols, logN, r, cur, roots, sp, src_logb);
        else
          ntt_dit_lazy_kernel<NTT_ELEMS, NTT_THREADS><<<grid, NTT_THREADS, 0, s>>>(d, ncols, logN, r, cur, roots, sp, src_logb);
      } else
        ntt_pass_kernel<false><<<(unsigned)((groups + G - 1) / G), NTT_THREADS, 0, s>>>(
            d, ncols, logN, r, cur, roots, logTab, cur == lo ? src : nullptr, src_logb);
      cur += r;
    }
  }
}

void launch_ntt_stages(fe* d, size_t ncols, size_t N, bool dif, int lo, int hi, MontTab roots, size_t Ntab,
                       hipStream_t s) {
  ntt_passes(d, ncols, N, dif, lo, hi, roots, Ntab, nullptr, 0, s);
}

int launch_lde_from_coeffs(const fe* d_coef, size_t ncols, size_t n, size_t N, MontTab roots, size_t Ntab, fe* d_out,
                           hipStream_t s, bool want_split) {
  const int logB = ilog2s(N / n);
  if (logB == 0) {
    ZKL_HIPCHECK(hipMemcpyAsync(d_out, d_coef, ncols * n * sizeof(fe), hipMemcpyDeviceToDevice, s));
    ntt_passes(d_out, ncols, N, false, 0, ilog2s(N) - 1, roots, Ntab, nullptr, 0, s);
    return 0;
  }
  const int split = want_split && dit_split_ok(N, logB, ilog2s(N) - 1) ? 1 : 0;
  ntt_passes(d_out, ncols, N, false, logB, ilog2s(N) - 1, roots, Ntab, d_coef, logB, s, split);
  return split;
}

__global__ void broadcast_kernel(const fe* __restrict__ in, size_t in_col_stride, size_t in_elem_stride,
                                 size_t in_offset, size_t ncols, size_t n, int logn, int logB, const fe* __restrict__ scale,
                                 fe mult, bool reverse, fe* __restrict__ out) {
  size_t N = n << logB;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * ncols) return;
  size_t col = i / N, pos = i % N;
  size_t j = pos >> logB;
  size_t src = reverse ? (n - 1 - j) : j;
  fe v = in[col * in_col_stride + in_offset + src * in_elem_stride];
  if (scale) v = fe_mul(v, scale[bitrev((uint32_t)j, logn)]);
  if (!(mult.lo == 1 && mult.hi == 0)) v = fe_mul(v, mult);
  out[i] = v;
}

void launch_broadcast(const fe* d_in, size_t in_col_stride, size_t in_elem_stride, size_t in_offset, size_t ncols,
                      size_t n, size_t N, const fe* d_scale, fe mult, bool reverse, fe* d_out, hipStream_t s) {
  size_t tot = N * ncols;
  broadcast_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(d_in, in_col_stride, in_elem_stride, in_offset, ncols,
                                                                 n, ilog2s(n), ilog2s(N / n), d_scale, mult, reverse, d_out);
}

__global__ void scale_bitrev_kernel(fe* d, size_t ncols, size_t n, int logn, const fe* scale) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * ncols) return;
  d[i] = fe_mul(d[i], scale[bitrev((uint32_t)(i % n), logn)]);
}
void launch_scale_bitrev(fe* d, size_t ncols, size_t n, const fe* scale, hipStream_t s) {
  scale_bitrev_kernel<<<(unsigned)((n * ncols + 255) / 256), 256, 0, s>>>(d, ncols, n, ilog2s(n), scale);
}


// =====================================================================================
// Constraint evaluation over the CE coset (DefaultConstraintEvaluator restated):
//   C(x) = [sum_j alpha_j c_j(x) * (x - g^(n-1)) + sum_c P_c(x) M_c(x) - W(x)] / (x^n - 1)
// c_j = ZkLispAir::evaluate_transition (vm/air/mod.rs:324-378) in evaluation order.
// =====================================================================================

// POSE: the PoseidonAir block, RM: the RamAir / MerkleAir blocks; each is compiled into a
// separate instance so that VM-only segments keep the smaller register footprint
// CE_WAVES_CFG: occupancy target (waves per SIMD; 0 lets the compiler choose: 214 VGPRs, 2 waves
// per SIMD for the VM-only instance).  The evaluator is latency-bound (dependent f128 products,
// gathers of 2 x 204 columns): 3 waves per SIMD took it from 1.57 to 1.40 ms per proof and 4 to
// 1.39 (round 3, profiles/r03/ab_ce); 3 keeps the larger Poseidon / RAM instances from spilling
// much.
#ifndef CE_WAVES_CFG
#define CE_WAVES_CFG 3
#endif
#if CE_WAVES_CFG
#define CE_OCC __attribute__((amdgpu_waves_per_eu(CE_WAVES_CFG, CE_WAVES_CFG)))
#else
#define CE_OCC
#endif
template <bool POSE, bool RM>
__device__ __forceinline__ void constraint_eval_body(const fe* __restrict__ lde, const fe* __restrict__ roots,
                                                     int roots_shift, const fe* __restrict__ pertab,
                                                     const fe* __restrict__ bm, const ProofConsts* __restrict__ K,
                                                     const fe* __restrict__ xinv, fe* __restrict__ out, int split) {
  const AirDevice& c_air = K->air;
  const CeParams& c_ce = K->ce;
  const size_t ce = c_ce.ce, N = c_ce.N;
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ce) return;
  // split layout with N / ce <= 2 (the CE rows are the even rows, or all rows): thread k reads
  // position k, i.e. whole lines of the first half of each column, and evaluates the CE point
  // of the row stored there; a wave's CE indices form two runs of 32.  Otherwise thread k
  // evaluates CE point k.
  const bool by_pos = split && N <= 2 * ce;
  const size_t i = by_pos ? lde_row(k, N, 1) / (N / ce) : k;
  const size_t r0 = by_pos ? k : lde_pos(i * (N / ce), N, split);
  const size_t r1 = lde_pos((i * (N / ce) + c_ce.blowup) & (N - 1), N, split);
  auto cur = [&](int c) { return lde[(size_t)c * N + r0]; };
  // next rows: position k + blowup for all but the rows whose L wraps; in the split layout
  // they share the lines this wave's current rows just brought in (PMC: taking them from the
  // neighbouring lane with ds_bpermute instead fetched the same bytes, round 3)
  auto nxt = [&](int c) { return lde[(size_t)c * N + r1]; };
  fe x = fe_mul(fe{3, 0}, roots[i << roots_shift]);
  const size_t per_period = ce / (c_ce.n / 32);
  const fe* per = pertab + (i % per_period) * 31;
  const size_t blow = ce / c_ce.n;
  const fe xn_inv = c_ce.xn_inv[i % blow];
  // p_last = L_{n-1}(x) = g^(n-1)/n * (x^n - 1) / (x - g^(n-1))
  fe x_gl = fe_sub_sel(x, c_ce.gl);
  fe xn_m1 = c_ce.xn_m1[i % blow];
  fe p_last = fe_mul(fe_mul(c_ce.lagr, xn_m1), xinv[i]);  // xinv[i] = 1 / (x - g^(n-1))
  const fe tsum = air_transition_sum<POSE, RM>(c_air, cur, nxt, per, p_last, K->alpha);
  // boundary: sum_c P_c(x) M_c(x) - W(x)
  uint32_t bacc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t nb = c_ce.n_bcols;
  for (uint32_t u = 0; u < nb; u++) mul_acc(cur((int)c_ce.bcol[u]), bm[(size_t)u * ce + i], bacc);
  fe bsum2 = fe_sub_sel(reduce288(bacc), bm[(size_t)nb * ce + i]);
  fe v = fe_add_sel(fe_mul(tsum, x_gl), bsum2);
  out[i] = fe_mul(v, xn_inv);
}

// The VM-only and RAM / Merkle instances run at CE_WAVES_CFG waves per SIMD; the Poseidon
// instances (90+ spilled VGPRs at 3 waves) keep the compiler's occupancy.
template <bool RM>
__global__ __launch_bounds__(256) CE_OCC void constraint_eval_kernel(const fe* __restrict__ lde, const fe* __restrict__ roots,
                                                                    int roots_shift, const fe* __restrict__ pertab,
                                                                    const fe* __restrict__ bm,
                                                                    const ProofConsts* __restrict__ K,
                                                                    const fe* __restrict__ xinv, fe* __restrict__ out,
                                                                    int split) {
  constraint_eval_body<false, RM>(lde, roots, roots_shift, pertab, bm, K, xinv, out, split);
}
template <bool RM>
__global__ __launch_bounds__(256) void constraint_eval_pose_kernel(const fe* __restrict__ lde, const fe* __restrict__ roots,
                                                                  int roots_shift, const fe* __restrict__ pertab,
                                                                  const fe* __restrict__ bm,
                                                                  const ProofConsts* __restrict__ K,
                                                                  const fe* __restrict__ xinv, fe* __restrict__ out,
                                                                  int split) {
  constraint_eval_body<true, RM>(lde, roots, roots_shift, pertab, bm, K, xinv, out, split);
}

// out[i] = 1 / ((x_i - a1) (x_i - a2)^two) over the coset x_i = 3 w_M^i (w_M^i =
// roots[i << shift]): each thread inverts INV_PTS points T apart with one field inversion
// (Montgomery's trick), instead of one ~250-multiplication Fermat inversion per point.
constexpr int INV_PTS = 16;
__global__ __launch_bounds__(256) void coset_inv_kernel(const fe* __restrict__ roots, int shift, fe a1, fe a2, int two,
                                                        fe* __restrict__ out) {
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  fe den[INV_PTS], pre[INV_PTS];
#pragma unroll
  for (int k = 0; k < INV_PTS; k++) {
    const fe x = fe_mul(fe{3, 0}, roots[(i0 + k * T) << shift]);
    fe d = fe_sub(x, a1);
    if (two) d = fe_mul(d, fe_sub(x, a2));
    den[k] = d;
    pre[k] = k ? fe_mul(pre[k - 1], d) : d;
  }
  fe inv = fe_inv(pre[INV_PTS - 1]);
#pragma unroll
  for (int k = INV_PTS - 1; k > 0; k--) {
    out[i0 + k * T] = fe_mul(inv, pre[k - 1]);
    inv = fe_mul(inv, den[k]);
  }
  out[i0] = inv;
}
static void launch_coset_inv(const fe* d_roots, int shift, size_t M, fe a1, fe a2, int two, fe* d_out, hipStream_t s) {
  // M is a power of two >= INV_PTS
  const size_t threads = std::min<size_t>(256, M / INV_PTS);
  coset_inv_kernel<<<(unsigned)(M / (threads * INV_PTS)), (unsigned)threads, 0, s>>>(d_roots, shift, a1, a2, two, d_out);
}

void launch_constraint_eval(const fe* d_lde, const fe* d_roots, size_t Ntab, const fe* d_pertab, const fe* d_bm,
                            const CeParams& p, ProofConsts* dK, bool pose_block, bool ram_merkle, fe* d_xinv,
                            bool xinv_ready, fe* d_out, hipStream_t s, int split) {
  ZKL_HIPCHECK(hipMemcpyAsync(&dK->ce, &p, sizeof p, hipMemcpyHostToDevice, s));
  int shift = ilog2s(Ntab) - ilog2s(p.ce);
  // 1 / (x - g^(n-1)) over the CE coset depends on the shape only: the caller keeps it per context
  if (!xinv_ready) launch_coset_inv(d_roots, shift, p.ce, p.gl, fe_zero(), 0, d_xinv, s);
  const unsigned grid = (unsigned)((p.ce + 255) / 256);
  if (pose_block && ram_merkle)
    constraint_eval_pose_kernel<true><<<grid, 256, 0, s>>>(d_lde, d_roots, shift, d_pertab, d_bm, dK, d_xinv, d_out, split);
  else if (pose_block)
    constraint_eval_pose_kernel<false><<<grid, 256, 0, s>>>(d_lde, d_roots, shift, d_pertab, d_bm, dK, d_xinv, d_out, split);
  else if (ram_merkle)
    constraint_eval_kernel<true><<<grid, 256, 0, s>>>(d_lde, d_roots, shift, d_pertab, d_bm, dK, d_xinv, d_out, split);
  else
    constraint_eval_kernel<false><<<grid, 256, 0, s>>>(d_lde, d_roots, shift, d_pertab, d_bm, dK, d_xinv, d_out, split);
}

__global__ void boundary_scatter_kernel(const uint32_t* slot, const uint32_t* step, const fe* beta, size_t na, size_t n,
                                        fe* vecs) {
  size_t a = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= na) return;
  vecs[(size_t)slot[a] * n + step[a]] = beta[a];
}
void launch_boundary_scatter(const uint32_t* d_slot, const uint32_t* d_step, const fe* d_beta, size_t na, size_t n,
                             fe* d_vecs, hipStream_t s) {
  boundary_scatter_kernel<<<(unsigned)((na + 255) / 256), 256, 0, s>>>(d_slot, d_step, d_beta, na, n, d_vecs);
}
__global__ void boundary_w_kernel(const uint32_t* rs, const fe* beta, const fe* val, size_t n, fe* w) {
  size_t row = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t a = rs[row]; a < rs[row + 1]; a++) mul_acc(beta[a], val[a], acc);
  w[row] = reduce288(acc);
}
void launch_boundary_w(const uint32_t* d_rs, const fe* d_beta, const fe* d_val, size_t n, fe* d_w, hipStream_t s) {
  boundary_w_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(d_rs, d_beta, d_val, n, d_w);
}

__global__ void check_zero_kernel(const fe* d, size_t N, int logN, size_t lo, size_t hi, unsigned* flag) {
  size_t k = lo + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= hi) return;
  fe v = d[bitrev((uint32_t)k, logN)];
  if (!fe_is_zero(v)) atomicOr(flag, 1u);
}
void launch_check_zero_range_bitrev(const fe* d, size_t N, size_t lo, size_t hi, unsigned* flag, hipStream_t s) {
  if (hi > lo) check_zero_kernel<<<(unsigned)((hi - lo + 255) / 256), 256, 0, s>>>(d, N, ilog2s(N), lo, hi, flag);
}

// =====================================================================================
// OOD (TracePolyTable::get_ood_frame / CompositionPoly ood): dot products with powers
// =====================================================================================
// partial[(pt * ncols + c) * chunks + k] = sum over chunk k of coef(c, j) * pw_pt[j]; the
// host adds the chunk partials (the OOD frame is read back anyway)
__global__ __launch_bounds__(256) void ood_kernel(OodArgs A, fe* partial) {
  const uint32_t c = blockIdx.x, pt = blockIdx.y, k = blockIdx.z;
  const fe* pw = pt ? A.pw2 : A.pw1;
  const fe* col = A.coef + (A.use_off ? (size_t)A.off[c] : (size_t)c * A.col_stride);
  const size_t len = A.n / A.chunks, j0 = (size_t)k * len;
  uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (size_t j = j0 + threadIdx.x; j < j0 + len; j += 256) mul_acc(col[j * A.elem_stride], pw[j], acc);
  __shared__ fe red[256];
  red[threadIdx.x] = reduce288(acc);
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = fe_add(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[((size_t)pt * A.ncols + c) * A.chunks + k] = red[0];
}
void launch_ood(const OodArgs& A, fe* d_partial, hipStream_t s) {
  ood_kernel<<<dim3(A.ncols, 2, A.chunks), 256, 0, s>>>(A, d_partial);
}

// DEEP composition over the LDE domain (agg/trace.rs:1126-1218 restates the formula):
// sum_i g_i [(T_i(x)-T_i(z))/(x-z) + (T_i(x)-T_i(zg))/(x-zg)] + same for H_j
//   = [(S(x) - S(z)) (x - zg) + (S(x) - S(zg)) (x - z)] / ((x - z)(x - zg)),  S = sum_i g_i T_i.
// S(x) is one lazily reduced dot product per point: the coefficients as Montgomery limbs
// (g R, uniform -> SGPR operands), each column value split into 26-bit limbs, 25
// v_mad_u64_u32 per column into 64-bit columns (up to 256 terms of < 2^54 stay below the 2^62
// the REDC needs; upload_deep_coeffs enforces it, W + C <= 226 here) and a
// single REDC.  Each thread takes DEEP_PTS points T apart (coalesced), keeps
// DEEP_COLS x DEEP_PTS loads in flight, and shares one inversion among its points.
// points per thread: 2 keeps the kernel at 96 VGPRs (5 waves per SIMD, more loads in flight;
// 4 points needed 180 VGPRs, 2 waves): DEEP 0.91 -> 0.85 ms (profiles/r02/ab_deep)
#ifndef DEEP_PTS_CFG
#define DEEP_PTS_CFG 2
#endif
#ifndef DEEP_COLS_CFG
#define DEEP_COLS_CFG 4
#endif
constexpr int DEEP_PTS = DEEP_PTS_CFG, DEEP_COLS = DEEP_COLS_CFG;

// canonical element of the REDC output limbs (normalised, value < 2^130)
__device__ __forceinline__ fe limbs_canon(const uint32_t l[5]) {
  typedef unsigned __int128 u128;
  const u128 v = (u128)l[0] | ((u128)l[1] << 26) | ((u128)l[2] << 52) | ((u128)l[3] << 78) | ((u128)(l[4] & 0xFFFFFFu) << 104);
  const u128 P = ((u128)P_HI << 64) | P_LO;
  u128 r = v + (u128)(l[4] >> 24) * C_RED;  // bits >= 128: 2^128 == C_RED
  if (r < v) r += C_RED;
  if (r >= P) r -= P;
  return fe{(uint64_t)r, (uint64_t)(r >> 64)};
}

__global__ __launch_bounds__(256) void deep_kernel(const fe* __restrict__ lde, const fe* __restrict__ clde,
                                                   const fe* __restrict__ roots, int shift, DeepParams p,
                                                   const ProofConsts* __restrict__ K, const fe* __restrict__ dinv,
                                                   fe* out, int split) {
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t col[DEEP_PTS][10];
#pragma unroll
  for (int k = 0; k < DEEP_PTS; k++)
#pragma unroll
    for (int u = 0; u < 10; u++) col[k][u] = 0;
  const uint32_t ncol = p.W + p.C;
  for (uint32_t c0 = 0; c0 < ncol; c0 += DEEP_COLS) {
    fe v[DEEP_COLS][DEEP_PTS];
#pragma unroll
    for (int cc = 0; cc < DEEP_COLS; cc++) {
      const uint32_t c = c0 + cc;
      // thread point k is LDE position q = i0 + k T (whole lines of the trace columns, which may
      // be in the split layout), i.e. row lde_row(q); composition columns are in natural order
      const bool tr = c < p.W;
      const fe* src = tr ? lde + (size_t)c * p.N : clde + (size_t)(c - p.W) * p.N;
#pragma unroll
      for (int k = 0; k < DEEP_PTS; k++)
        v[cc][k] = c < ncol ? src[tr ? i0 + k * T : lde_row(i0 + k * T, p.N, split)] : fe_zero();
    }
#pragma unroll
    for (int cc = 0; cc < DEEP_COLS; cc++) {
      const uint32_t c = min(c0 + cc, ncol - 1);  // a padded column contributes g * 0
      const uint32_t* g = K->deep_m[c];
      const uint32_t gm[5] = {g[0], g[1], g[2], g[3], g[4]};
#pragma unroll
      for (int k = 0; k < DEEP_PTS; k++) {
        uint32_t l[5];
        to26(v[cc][k], l);
        mac5(l, gm, col[k]);
      }
    }
  }
  // 1 / ((x - z)(x - zg)) comes from coset_inv_kernel (x is never z or zg: z is drawn
  // outside the LDE domain, as Winterfell requires)
#pragma unroll
  for (int k = 0; k < DEEP_PTS; k++) {
    uint32_t l[5];
    redc(col[k], l);
    const fe sv = limbs_canon(l);
    const size_t i = lde_row(i0 + k * T, p.N, split);
    const fe x = fe_mul(fe{3, 0}, roots[i << shift]);
    const fe d1 = fe_sub(x, p.z), d2 = fe_sub(x, p.zg);
    const fe num = fe_add(fe_mul(fe_sub(sv, p.sz), d2), fe_mul(fe_sub(sv, p.szg), d1));
    out[i] = fe_mul(num, dinv[i]);
  }
}
void launch_deep_denoms(const fe* d_roots, size_t Ntab, size_t N, fe z, fe zg, fe* d_dinv, hipStream_t s) {
  launch_coset_inv(d_roots, ilog2s(Ntab) - ilog2s(N), N, z, zg, 1, d_dinv, s);
}

void launch_deep(const fe* d_lde, const fe* d_clde, const fe* d_roots, size_t Ntab, const DeepParams& p,
                 const ProofConsts* dK, const fe* d_dinv, fe* d_out, hipStream_t s, int split) {
  // N is a power of two >= 64: every thread gets exactly DEEP_PTS points
  const size_t threads = std::min<size_t>(256, p.N / DEEP_PTS);
  deep_kernel<<<(unsigned)(p.N / (threads * DEEP_PTS)), (unsigned)threads, 0, s>>>(
      d_lde, d_clde, d_roots, ilog2s(Ntab) - ilog2s(p.N), p, dK, d_dinv, d_out, split);
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
  else if (hash_engine() == 1 && h >= pm_min_items())
    PM_GO(fri_leaf_pm_kernel, h, false, s)(d_ev, h, d_leaves);
  else
    fri_leaf_kernel<<<pg_blocks(h), 256, 0, s>>>(d_ev, h, d_leaves);
}
// fold: (v0+v1)/2 + alpha (v0-v1) / (2 x0), x0 = GENERATOR * g_d^i (constant offset, agg/trace.rs:764-800)
__global__ void fri_fold_kernel(const fe* ev, size_t half, const fe* alpha_p, const fe* iroots, int shift, fe inv3,
                                fe inv2, fe* out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= half) return;
  const fe alpha = *alpha_p;
  fe v0 = ev[i], v1 = ev[i + half];
  fe ix = fe_mul(inv3, iroots[i << shift]);
  out[i] = fe_mul(fe_add(fe_add(v0, v1), fe_mul(alpha, fe_mul(fe_sub(v0, v1), ix))), inv2);
}
void launch_fri_fold(const fe* d_ev, size_t Nd, const fe* d_alpha, const fe* d_iroots, size_t Ntab, fe* d_out,
                     hipStream_t s) {
  size_t h = Nd / 2;
  fe inv3 = fe_inv(fe{3, 0}), inv2 = fe_inv(fe{2, 0});
  fri_fold_kernel<<<(unsigned)((h + 255) / 256), 256, 0, s>>>(d_ev, h, d_alpha, d_iroots, ilog2s(Ntab) - ilog2s(Nd),
                                                               inv3, inv2, d_out);
}

__global__ void gather_kernel(const uint64_t* addrs, size_t k, fe* out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  out[i] = *reinterpret_cast<const fe*>(addrs[i]);
}
void launch_gather(const uint64_t* d_addrs, size_t k, fe* d_out, hipStream_t s) {
  if (k) gather_kernel<<<(unsigned)((k + 255) / 256), 256, 0, s>>>(d_addrs, k, d_out);
}

}  // namespace zkl
