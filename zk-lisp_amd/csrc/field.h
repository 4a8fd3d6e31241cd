// f128 prime field for the MI355X prover: p = 2^128 - 45*2^40 + 1 (winter-math 0.13.1
// fields::f128, used by the reference at zk-lisp-proof-winterfell/src/lib.rs:40).
// Canonical representation (< p), two little-endian 64-bit words.  Device code works on
// 32-bit limbs (v_mad_u64_u32); host code uses unsigned __int128.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zkl {

struct alignas(16) fe {
  uint64_t lo, hi;
};

constexpr uint64_t P_LO = 0xFFFFD30000000001ull;
constexpr uint64_t P_HI = 0xFFFFFFFFFFFFFFFFull;
constexpr uint64_t C_RED = 0x2CFFFFFFFFFFull;  // 2^128 mod p = 45*2^40 - 1

__host__ __device__ inline fe fe_make(uint64_t lo, uint64_t hi) { return fe{lo, hi}; }
__host__ __device__ inline fe fe_zero() { return fe{0, 0}; }
__host__ __device__ inline fe fe_one() { return fe{1, 0}; }
__host__ __device__ inline bool fe_is_zero(fe a) { return (a.lo | a.hi) == 0; }
__host__ __device__ inline bool fe_eq(fe a, fe b) { return a.lo == b.lo && a.hi == b.hi; }

// a + b mod p (inputs canonical), branch-free: with s = a + b mod 2^128, the result is
// s + C (mod 2^128) exactly when a + b >= p, i.e. when either addition carries out.
__host__ __device__ inline fe fe_add(fe a, fe b) {
  unsigned long long c0, c1, d0, d1;
  const unsigned long long lo = __builtin_addcll(a.lo, b.lo, 0, &c0);
  const unsigned long long hi = __builtin_addcll(a.hi, b.hi, c0, &c1);
  const unsigned long long tlo = __builtin_addcll(lo, C_RED, 0, &d0);
  const unsigned long long thi = __builtin_addcll(hi, 0, d0, &d1);
  return (c1 | d1) ? fe{tlo, thi} : fe{lo, hi};
}

// a - b mod p: on borrow the wrapped difference d needs + p = - C (mod 2^128)
__host__ __device__ inline fe fe_sub(fe a, fe b) {
  unsigned long long b0, b1, e0, e1;
  const unsigned long long lo = __builtin_subcll(a.lo, b.lo, 0, &b0);
  const unsigned long long hi = __builtin_subcll(a.hi, b.hi, b0, &b1);
  const unsigned long long tlo = __builtin_subcll(lo, C_RED, 0, &e0);
  const unsigned long long thi = __builtin_subcll(hi, 0, e0, &e1);
  (void)e1;
  return b1 ? fe{tlo, thi} : fe{lo, hi};
}


// Branching forms: cheaper when operands are small (the constraint evaluator's selectors
// and flags rarely wrap, so whole wavefronts skip the reduction).
__host__ __device__ inline fe fe_add_sel(fe a, fe b) {
  uint64_t lo = a.lo + b.lo;
  uint64_t c0 = lo < a.lo;
  uint64_t t = a.hi + b.hi;
  uint64_t c1 = t < a.hi;
  uint64_t hi = t + c0;
  c1 |= hi < t;
  if (c1) {  // wrapped past 2^128: add 2^128 - p = C_RED
    uint64_t l2 = lo + C_RED;
    hi += l2 < lo;
    return fe{l2, hi};
  }
  if (hi == P_HI && lo >= P_LO) return fe{lo - P_LO, 0};
  return fe{lo, hi};
}

__host__ __device__ inline fe fe_sub_sel(fe a, fe b) {
  uint64_t lo = a.lo - b.lo;
  uint64_t br0 = a.lo < b.lo;
  uint64_t t = a.hi - b.hi;
  uint64_t br1 = a.hi < b.hi;
  uint64_t hi = t - br0;
  br1 |= t < br0;
  if (br1) {  // negative: add p == subtract C_RED modulo 2^128
    uint64_t l2 = lo - C_RED;
    hi -= lo < C_RED;
    return fe{l2, hi};
  }
  return fe{lo, hi};
}

__host__ __device__ inline fe fe_neg(fe a) { return fe_sub(fe_zero(), a); }

// ---------------------------------------------------------------- device multiply
// 128x128 -> 256 schoolbook on 32-bit limbs: 16 v_mad_u64_u32.
__host__ __device__ inline void mul_wide32(fe a, fe b, uint32_t r[8]) {
  uint32_t x[4] = {(uint32_t)a.lo, (uint32_t)(a.lo >> 32), (uint32_t)a.hi, (uint32_t)(a.hi >> 32)};
  uint32_t y[4] = {(uint32_t)b.lo, (uint32_t)(b.lo >> 32), (uint32_t)b.hi, (uint32_t)(b.hi >> 32)};
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint64_t t = (uint64_t)x[i] * y[j] + r[i + j] + carry;
      r[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    r[i + 4] = (uint32_t)carry;
  }
}

// reduce a 288-bit value r[0..9) (r[8] small) modulo p.
// x = H*2^128 + L ; 2^128 == 45*2^40 - 1.
__host__ __device__ inline fe reduce288(const uint32_t r[9]) {
  // H = r[4..9) (up to 160 bits), T = 45*H
  uint32_t T[6];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    uint64_t t = (uint64_t)r[4 + i] * 45u + c;
    T[i] = (uint32_t)t;
    c = t >> 32;
  }
  T[5] = (uint32_t)c;
  // S = T << 40 (limbs 1..7), value < 2^214 -> 7 limbs
  uint32_t S[8];
  S[0] = 0;
  S[1] = T[0] << 8;
#pragma unroll
  for (int i = 2; i < 7; i++) S[i] = (T[i - 1] << 8) | (T[i - 2] >> 24);
  S[7] = T[5] >> 24;
  // U = S - H  (H < S always since S = 45*2^40*H)
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t hv = (i < 5) ? r[4 + i] : 0;
    uint64_t t = (uint64_t)S[i] - hv - br;
    S[i] = (uint32_t)t;
    br = (t >> 63) & 1;
  }
  // X = L + U
  uint64_t cc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t lv = (i < 4) ? r[i] : 0;
    uint64_t t = (uint64_t)S[i] + lv + cc;
    S[i] = (uint32_t)t;
    cc = t >> 32;
  }
  // X = Xlo (S[0..4)) + Xhi*2^128, Xhi = S[4..8) < 2^87
  // Xhi * C_RED = Xhi*45*2^40 - Xhi  (< 2^133)
  uint32_t V[5];
  c = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    uint64_t t = (uint64_t)S[4 + i] * 45u + c;
    V[i] = (uint32_t)t;
    c = t >> 32;
  }
  V[3] = (uint32_t)c + S[7] * 45u;  // S[7] tiny
  // W = V << 40 - Xhi (limbs 0..5)
  uint32_t Wv[6];
  Wv[0] = 0;
  Wv[1] = V[0] << 8;
  Wv[2] = (V[1] << 8) | (V[0] >> 24);
  Wv[3] = (V[2] << 8) | (V[1] >> 24);
  Wv[4] = (V[3] << 8) | (V[2] >> 24);
  Wv[5] = V[3] >> 24;
  br = 0;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    uint64_t hv = (i < 4) ? S[4 + i] : 0;
    uint64_t t = (uint64_t)Wv[i] - hv - br;
    Wv[i] = (uint32_t)t;
    br = (t >> 63) & 1;
  }
  // Y = Xlo + W  (< 2^128 + 2^134)
  cc = 0;
  uint32_t Y[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    uint64_t xv = (i < 4) ? S[i] : 0;
    uint64_t t = (uint64_t)xv + Wv[i] + cc;
    Y[i] = (uint32_t)t;
    cc = t >> 32;
  }
  // Y = Ylo + Yhi*2^128 with Yhi < 2^7: fold once more (Yhi*C_RED < 2^53)
  uint64_t yhi = (uint64_t)Y[4] | ((uint64_t)Y[5] << 32);
  uint64_t add_lo = yhi * C_RED;                       // < 2^60: no overflow
  uint64_t lo = (uint64_t)Y[0] | ((uint64_t)Y[1] << 32);
  uint64_t hi = (uint64_t)Y[2] | ((uint64_t)Y[3] << 32);
  uint64_t l2 = lo + add_lo;
  uint64_t h2 = hi + (l2 < lo);
  if (h2 < hi) {  // overflow past 2^128 (only when hi was all ones)
    uint64_t l3 = l2 + C_RED;
    h2 += l3 < l2;
    l2 = l3;
  }
  if (h2 == P_HI && l2 >= P_LO) return fe{l2 - P_LO, 0};
  return fe{l2, h2};
}


// acc[0..9) += a*b (lazy accumulation for dot products, <= 2^32 terms)
__host__ __device__ inline void mul_acc(fe a, fe b, uint32_t acc[9]) {
  uint32_t r[8];
  mul_wide32(a, b, r);
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t t = (uint64_t)acc[i] + r[i] + c;
    acc[i] = (uint32_t)t;
    c = t >> 32;
  }
  acc[8] += (uint32_t)c;
}

// acc[0..9) += v (lazy sum of field elements, no multiplication; <= 2^32 terms)
__host__ __device__ inline void add_acc(fe v, uint32_t acc[9]) {
  const uint32_t w[4] = {(uint32_t)v.lo, (uint32_t)(v.lo >> 32), (uint32_t)v.hi, (uint32_t)(v.hi >> 32)};
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t t = (uint64_t)acc[i] + w[i] + c;
    acc[i] = (uint32_t)t;
    c = t >> 32;
  }
#pragma unroll
  for (int i = 4; i < 8; i++) {
    uint64_t t = (uint64_t)acc[i] + c;
    acc[i] = (uint32_t)t;
    c = t >> 32;
  }
  acc[8] += (uint32_t)c;
}

// ---------------------------------------------------------------- host multiply
typedef unsigned __int128 u128;
inline u128 to128(fe a) { return ((u128)a.hi << 64) | a.lo; }
inline fe from128(u128 v) { return fe{(uint64_t)v, (uint64_t)(v >> 64)}; }
inline fe host_reduce(u128 hi, u128 lo) {
  const u128 C = C_RED;
  const u128 P = ((u128)P_HI << 64) | P_LO;
  uint64_t h0 = (uint64_t)hi, h1 = (uint64_t)(hi >> 64);
  u128 t0 = (u128)h0 * C_RED, t1 = (u128)h1 * C_RED;
  u128 lo2 = t0 + (t1 << 64);
  u128 hi2 = (t1 >> 64) + (lo2 < t0);
  u128 s = lo + lo2;
  u128 r = hi2 * C + ((s < lo) ? C : 0);
  u128 s2 = s + r;
  if (s2 < s) s2 += C;
  if (s2 >= P) s2 -= P;
  return from128(s2);
}
inline void host_mul_wide(fe a, fe b, u128* hi, u128* lo) {
  u128 p00 = (u128)a.lo * b.lo, p01 = (u128)a.lo * b.hi, p10 = (u128)a.hi * b.lo, p11 = (u128)a.hi * b.hi;
  u128 mid = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
  *lo = (u128)(uint64_t)p00 | (mid << 64);
  *hi = p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);
}

__host__ __device__ inline fe fe_mul(fe a, fe b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r[9];
  mul_wide32(a, b, r);
  r[8] = 0;
  return reduce288(r);
#else
  u128 hi, lo;
  host_mul_wide(a, b, &hi, &lo);
  return host_reduce(hi, lo);
#endif
}

__host__ __device__ inline fe fe_sqr(fe a) { return fe_mul(a, a); }
__host__ __device__ inline fe fe_cube(fe a) { return fe_mul(fe_mul(a, a), a); }

__host__ __device__ inline fe fe_pow(fe b, uint64_t e_lo, uint64_t e_hi) {
  fe r = fe_one();
  for (int w = 0; w < 2; w++) {
    uint64_t e = w ? e_hi : e_lo;
    for (int i = 0; i < 64; i++) {
      if (e & 1) r = fe_mul(r, b);
      b = fe_sqr(b);
      e >>= 1;
    }
  }
  return r;
}
__host__ __device__ inline fe fe_pow64(fe b, uint64_t e) {
  fe r = fe_one();
  while (e) {
    if (e & 1) r = fe_mul(r, b);
    b = fe_sqr(b);
    e >>= 1;
  }
  return r;
}
// Fermat inverse a^(p-2); zero -> zero.  p - 2 = [80 ones][1101 0010][40 ones] in binary, so an
// addition chain over a^(2^k - 1) takes 127 squarings and 12 multiplications instead of the 128 +
// ~125 of square-and-multiply (round 6: the DEEP denominators' batch inversion, coset_inv_kernel).
__host__ __device__ inline fe fe_sqr_n(fe a, int n) {
  for (int i = 0; i < n; i++) a = fe_mul(a, a);
  return a;
}
__host__ __device__ inline fe fe_inv(fe a) {
  if (fe_is_zero(a)) return a;
  const fe a1 = a;
  const fe a2 = fe_mul(fe_sqr_n(a1, 1), a1);     // a^(2^2 - 1)
  const fe a4 = fe_mul(fe_sqr_n(a2, 2), a2);
  const fe a8 = fe_mul(fe_sqr_n(a4, 4), a4);
  const fe a16 = fe_mul(fe_sqr_n(a8, 8), a8);
  const fe a32 = fe_mul(fe_sqr_n(a16, 16), a16);
  const fe a40 = fe_mul(fe_sqr_n(a32, 8), a8);
  fe r = fe_mul(fe_sqr_n(a40, 40), a40);         // a^(2^80 - 1)
  const uint32_t mid = 0xD2;                      // bits 47..40 of p - 2
  for (int b = 7; b >= 0; b--) {
    r = fe_mul(r, r);
    if ((mid >> b) & 1) r = fe_mul(r, a1);
  }
  return fe_mul(fe_sqr_n(r, 40), a40);           // then 40 ones
}

// x * 2^64 mod p  (fold of the high half of a 32-byte sponge chunk, utils.rs:359-371)
__host__ __device__ inline fe fe_mul_2_64(fe b) {
  // b*2^64 = b.hi*2^128 + b.lo*2^64 == b.hi*C + (b.lo, 0)
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t plo = b.hi * C_RED;
  uint64_t phi = __umul64hi(b.hi, C_RED);
#else
  unsigned __int128 pr = (unsigned __int128)b.hi * C_RED;
  uint64_t plo = (uint64_t)pr, phi = (uint64_t)(pr >> 64);
#endif
  fe x = fe{0, b.lo};
  uint64_t lo = x.lo + plo;  // x.lo == 0
  uint64_t hi = x.hi + phi;
  if (hi < x.hi) {  // overflow
    uint64_t l2 = lo + C_RED;
    hi += l2 < lo;
    lo = l2;
  }
  if (hi == P_HI && lo >= P_LO) return fe{lo - P_LO, 0};
  return fe{lo, hi};
}

// fold of one 32-byte chunk made of two canonical elements: a + b*2^64
__host__ __device__ inline fe fold_pair(fe a, fe b) { return fe_add(a, fe_mul_2_64(b)); }

}  // namespace zkl
