// Host Poseidon permutation on AVX-512 IFMA (52-bit limb multiply-add), for the transcript
// hashing the prover does on the host between device phases (coin reseeds and draws, the OOD
// frame hash, the FRI remainder commitment, the query seed) and for the aggregation prover.
// Same permutation as permute_with (host_hash.cpp; poseidon/hasher.rs:173-190): 27 rounds of
// x^3 on all 12 lanes, dense 12x12 MDS, + round constants -- here in Montgomery form with
// R = 2^156 on 3 x 52-bit limbs, the 12 state elements in the lanes of two zmm registers
// (elements 0-7, 8-11), the MDS rows likewise: per round and column k the cube c_k is broadcast
// and 18 vpmadd52{lo,hi}uq accumulate M[i][k] c_k for 8 rows at once, unreduced, then one REDC
// per row vector.  Values stay below 3p between rounds (Montgomery bounds: T < R p for every
// REDC input since 24 p^2 < 2^156 p), and are canonicalised on the way out.
//
// Used only where the CPU has AVX-512F + IFMA (checked at run time, EPYC 9005 / Xeon hosts);
// the scalar permutation stays the reference the vector form is checked against at start-up.
#include <immintrin.h>
#include <string.h>

#include "host_hash.h"

namespace zkl {

namespace {
constexpr uint64_t M52 = (1ull << 52) - 1;
typedef unsigned __int128 u128;

inline void limbs52(fe a, uint64_t l[3]) {
  l[0] = a.lo & M52;
  l[1] = ((a.lo >> 52) | (a.hi << 12)) & M52;
  l[2] = a.hi >> 40;
}
inline fe from52(const uint64_t l[3]) {
  // l0, l1 < 2^52, l2 small: value = l0 + l1 2^52 + l2 2^104 (< 2^130)
  const u128 v = (u128)l[0] + ((u128)l[1] << 52) + ((u128)l[2] << 104);
  return fe{(uint64_t)v, (uint64_t)(v >> 64)};
}
inline fe mont_of(fe a, fe R) { return fe_mul(a, R); }
}  // namespace

struct alignas(64) IfmaSuite {
  uint64_t mds[12][2][3][8];  // [k][row vector][limb][lane]: limbs of M[8v+lane][k] R mod p
  uint64_t rc[27][2][3][8];   // [round][vector][limb][lane]: limbs of rc[r][8v+lane] R mod p
  uint64_t r2[3], one[3], p[3], pinv;  // R^2 mod p, 1, p, -p^-1 mod 2^52
  int rounds;
};

IfmaSuite* ifma_new() { return new IfmaSuite; }
void ifma_delete(IfmaSuite* p) { delete p; }

bool ifma_available() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512ifma");
  return ok;
}

void ifma_prepare(const PoseidonSuite& s, IfmaSuite& out) {
  memset(&out, 0, sizeof out);
  const fe R = fe_pow64(fe{2, 0}, 156);
  for (int k = 0; k < 12; k++)
    for (int i = 0; i < 12; i++) {
      uint64_t l[3];
      limbs52(mont_of(s.mds[i][k], R), l);
      for (int t = 0; t < 3; t++) out.mds[k][i / 8][t][i % 8] = l[t];
    }
  for (int r = 0; r < s.rounds; r++)
    for (int i = 0; i < 12; i++) {
      uint64_t l[3];
      limbs52(mont_of(s.rc[r][i], R), l);
      for (int t = 0; t < 3; t++) out.rc[r][i / 8][t][i % 8] = l[t];
    }
  limbs52(fe_mul(R, R), out.r2);
  out.one[0] = 1;
  limbs52(fe{P_LO, P_HI}, out.p);
  // -p^-1 mod 2^52 by Newton iteration on 64-bit words (p odd)
  uint64_t inv = 1;
  for (int it = 0; it < 7; it++) inv *= 2 - P_LO * inv;
  out.pinv = (0 - inv) & M52;
  out.rounds = s.rounds;
}

#define IFMA_TARGET __attribute__((target("avx512f,avx512ifma")))

namespace {
struct V3 {
  __m512i l[3];
};

IFMA_TARGET inline __m512i lo52(__m512i acc, __m512i a, __m512i b) { return _mm512_madd52lo_epu64(acc, a, b); }
IFMA_TARGET inline __m512i hi52(__m512i acc, __m512i a, __m512i b) { return _mm512_madd52hi_epu64(acc, a, b); }

// Montgomery REDC of six unreduced columns (each < 2^62) -> three limbs (l0, l1 < 2^52)
IFMA_TARGET inline V3 redc(__m512i t[6], const __m512i P[3], __m512i pinv) {
  const __m512i mask = _mm512_set1_epi64((long long)M52), z = _mm512_setzero_si512();
#pragma GCC unroll 3
  for (int i = 0; i < 3; i++) {
    t[i + 1] = _mm512_add_epi64(t[i + 1], _mm512_srli_epi64(t[i], 52));
    t[i] = _mm512_and_si512(t[i], mask);
    const __m512i m = _mm512_and_si512(lo52(z, t[i], pinv), mask);
    for (int j = 0; j < 3; j++) {
      t[i + j] = lo52(t[i + j], m, P[j]);
      t[i + j + 1] = hi52(t[i + j + 1], m, P[j]);
    }
    t[i + 1] = _mm512_add_epi64(t[i + 1], _mm512_srli_epi64(t[i], 52));  // t[i] is 0 mod 2^52
  }
  V3 r;
  t[4] = _mm512_add_epi64(t[4], _mm512_srli_epi64(t[3], 52));
  r.l[0] = _mm512_and_si512(t[3], mask);
  t[5] = _mm512_add_epi64(t[5], _mm512_srli_epi64(t[4], 52));
  r.l[1] = _mm512_and_si512(t[4], mask);
  r.l[2] = t[5];
  return r;
}

IFMA_TARGET inline V3 mont_mul(const V3& a, const V3& b, const __m512i P[3], __m512i pinv) {
  __m512i t[6];
  for (int i = 0; i < 6; i++) t[i] = _mm512_setzero_si512();
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      t[i + j] = lo52(t[i + j], a.l[i], b.l[j]);
      t[i + j + 1] = hi52(t[i + j + 1], a.l[i], b.l[j]);
    }
  return redc(t, P, pinv);
}

IFMA_TARGET inline V3 bcast3(const uint64_t l[3]) {
  V3 r;
  for (int t = 0; t < 3; t++) r.l[t] = _mm512_set1_epi64((long long)l[t]);
  return r;
}
}  // namespace

IFMA_TARGET void ifma_permute(const IfmaSuite& S, fe st[12]) {
  __m512i P[3];
  for (int t = 0; t < 3; t++) P[t] = _mm512_set1_epi64((long long)S.p[t]);
  const __m512i pinv = _mm512_set1_epi64((long long)S.pinv);
  const __m512i mask = _mm512_set1_epi64((long long)M52);
  // state -> limbs -> Montgomery (x R^2 R^-1)
  alignas(64) uint64_t in[2][3][8] = {};
  for (int i = 0; i < 12; i++) {
    uint64_t l[3];
    limbs52(st[i], l);
    for (int t = 0; t < 3; t++) in[i / 8][t][i % 8] = l[t];
  }
  const V3 r2 = bcast3(S.r2);
  V3 x[2];
  for (int v = 0; v < 2; v++) {
    V3 a;
    for (int t = 0; t < 3; t++) a.l[t] = _mm512_load_si512((const void*)in[v][t]);
    x[v] = mont_mul(a, r2, P, pinv);
  }
  for (int r = 0; r < S.rounds; r++) {
    V3 c[2];
    for (int v = 0; v < 2; v++) {
      const V3 sq = mont_mul(x[v], x[v], P, pinv);
      c[v] = mont_mul(sq, x[v], P, pinv);
    }
    __m512i acc[2][6];
    for (int v = 0; v < 2; v++)
      for (int i = 0; i < 6; i++) acc[v][i] = _mm512_setzero_si512();
    for (int k = 0; k < 12; k++) {
      const __m512i idx = _mm512_set1_epi64(k % 8);
      __m512i ck[3];
      for (int t = 0; t < 3; t++) ck[t] = _mm512_permutexvar_epi64(idx, c[k / 8].l[t]);
      for (int v = 0; v < 2; v++) {
        const uint64_t(*mk)[8] = S.mds[k][v];
        for (int i = 0; i < 3; i++) {
          const __m512i mi = _mm512_load_si512((const void*)mk[i]);
          for (int j = 0; j < 3; j++) {
            acc[v][i + j] = lo52(acc[v][i + j], mi, ck[j]);
            acc[v][i + j + 1] = hi52(acc[v][i + j + 1], mi, ck[j]);
          }
        }
      }
    }
    for (int v = 0; v < 2; v++) {
      V3 y = redc(acc[v], P, pinv);
      // + rc (Montgomery form), limbs renormalised for the next round's multiplies
      __m512i s0 = _mm512_add_epi64(y.l[0], _mm512_load_si512((const void*)S.rc[r][v][0]));
      __m512i s1 = _mm512_add_epi64(y.l[1], _mm512_load_si512((const void*)S.rc[r][v][1]));
      __m512i s2 = _mm512_add_epi64(y.l[2], _mm512_load_si512((const void*)S.rc[r][v][2]));
      s1 = _mm512_add_epi64(s1, _mm512_srli_epi64(s0, 52));
      s0 = _mm512_and_si512(s0, mask);
      s2 = _mm512_add_epi64(s2, _mm512_srli_epi64(s1, 52));
      s1 = _mm512_and_si512(s1, mask);
      x[v].l[0] = s0;
      x[v].l[1] = s1;
      x[v].l[2] = s2;
    }
  }
  // out of Montgomery form: REDC(x * 1) <= p, then canonical
  const V3 one = bcast3(S.one);
  alignas(64) uint64_t out[2][3][8];
  for (int v = 0; v < 2; v++) {
    const V3 o = mont_mul(x[v], one, P, pinv);
    for (int t = 0; t < 3; t++) _mm512_store_si512((void*)out[v][t], o.l[t]);
  }
  const u128 Pv = ((u128)P_HI << 64) | P_LO;
  for (int i = 0; i < 12; i++) {
    const uint64_t l[3] = {out[i / 8][0][i % 8], out[i / 8][1][i % 8], out[i / 8][2][i % 8]};
    fe f = from52(l);
    u128 v = ((u128)f.hi << 64) | f.lo;
    if (v >= Pv) v -= Pv;
    st[i] = fe{(uint64_t)v, (uint64_t)(v >> 64)};
  }
}

}  // namespace zkl
