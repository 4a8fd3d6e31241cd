/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  Never linked into libzkl_hip.so.
 *
 * f128 prime field, restating winter-math 0.13.1 `fields::f128::BaseElement`
 * (third-party crate, not vendored; used at zk-lisp-proof-winterfell/src/lib.rs:40,
 * prove.rs:20,26).  p = 2^128 - 45*2^40 + 1, canonical representation, GENERATOR = 3,
 * TWO_ADICITY = 40, TWO_ADIC_ROOT_OF_UNITY = 3^((p-1)/2^40)
 * = 23953097886125630542083529559205016746 (checked in tests/test_oracle_field.py).
 * Every value is an exact residue, so any correct implementation yields identical bytes.
 */
#ifndef ORACLE_F128_H
#define ORACLE_F128_H
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 fe;

#define FE_C ((fe)0x2CFFFFFFFFFFULL) /* 2^128 mod p = 45*2^40 - 1 */
#define FE_P ((((fe)0xFFFFFFFFFFFFFFFFULL) << 64) | (fe)0xFFFFD30000000001ULL)

static inline fe fe_from_u64(uint64_t x) { return (fe)x; }
static inline fe fe_from_u128(fe x) { return x >= FE_P ? x - FE_P : x; }

static inline fe fe_add(fe a, fe b) {
  fe s = a + b;
  if (s < a) return s + FE_C; /* wrapped past 2^128: s + 2^128 - p */
  if (s >= FE_P) s -= FE_P;
  return s;
}
static inline fe fe_sub(fe a, fe b) { return a >= b ? a - b : a + (FE_P - b); }
static inline fe fe_neg(fe a) { return a == 0 ? 0 : FE_P - a; }

static inline void fe_mul_wide(fe a, fe b, fe *hi, fe *lo) {
  uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64);
  uint64_t b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
  fe p00 = (fe)a0 * b0, p01 = (fe)a0 * b1, p10 = (fe)a1 * b0, p11 = (fe)a1 * b1;
  fe mid = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
  *lo = (fe)(uint64_t)p00 | (mid << 64);
  *hi = p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);
}

/* reduce hi*2^128 + lo modulo p using 2^128 = C (mod p) */
static inline fe fe_reduce_wide(fe hi, fe lo) {
  uint64_t h0 = (uint64_t)hi, h1 = (uint64_t)(hi >> 64);
  fe t0 = (fe)h0 * (uint64_t)FE_C;
  fe t1 = (fe)h1 * (uint64_t)FE_C;
  fe lo2 = t0 + (t1 << 64);
  fe hi2 = (t1 >> 64) + (lo2 < t0);
  fe s = lo + lo2;
  fe r = hi2 * FE_C + ((s < lo) ? FE_C : 0);
  fe s2 = s + r;
  if (s2 < s) s2 += FE_C;
  if (s2 >= FE_P) s2 -= FE_P;
  return s2;
}

static inline fe fe_mul(fe a, fe b) {
  fe hi, lo;
  fe_mul_wide(a, b, &hi, &lo);
  return fe_reduce_wide(hi, lo);
}
static inline fe fe_sqr(fe a) { return fe_mul(a, a); }
static inline fe fe_cube(fe a) { return fe_mul(fe_mul(a, a), a); }

static inline fe fe_exp(fe b, fe e) {
  fe r = 1;
  while (e) {
    if (e & 1) r = fe_mul(r, b);
    b = fe_mul(b, b);
    e >>= 1;
  }
  return r;
}
static inline fe fe_inv(fe a) { return a == 0 ? 0 : fe_exp(a, FE_P - 2); }

/* get_root_of_unity(k): TWO_ADIC_ROOT_OF_UNITY^(2^(40-k)) */
static inline fe fe_root_of_unity(unsigned k) {
  fe g = fe_exp(3, (FE_P - 1) >> 40);
  for (unsigned i = k; i < 40; i++) g = fe_mul(g, g);
  return g;
}

static inline void fe_to_bytes(fe a, uint8_t out[16]) {
  for (int i = 0; i < 16; i++) out[i] = (uint8_t)(a >> (8 * i));
}
static inline fe fe_from_bytes_raw(const uint8_t in[16]) {
  fe v = 0;
  for (int i = 15; i >= 0; i--) v = (v << 8) | in[i];
  return v;
}

/* batch inversion (Montgomery trick); zeros map to zero */
void fe_batch_inv(fe *out, const fe *in, size_t n, fe *scratch);

#endif
