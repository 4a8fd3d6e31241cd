// Montgomery arithmetic on 5 x 26-bit limbs shared by the Poseidon kernels (poseidon.hip)
// and the NTT / DEEP kernels (kernels.hip).  Device-inline, no device state.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.h"

namespace zkl {

// ---- Montgomery arithmetic on 5 x 26-bit limbs (R = 2^156) ---------------------------
// p = 1 + 0x3F4C000*2^26 + (2^26-1)*2^52 + (2^26-1)*2^78 + (2^24-1)*2^104, and p == 1
// (mod 2^26), so the REDC quotient digit is m = -x mod 2^26 with no multiplication.
// Products accumulate in 64-bit columns by v_mad_u64_u32 with no carry handling: with
// limbs < 2^28 a column holds at most 60 products < 2^56, far below 2^64.  Values are
// kept lazily reduced (< 2^130) inside the permutation and canonicalised on output.

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

// a cube's normalised limbs (< 2^131) as the matrix-core permutation's B words: four words of
// offset bytes (c = sum_j (b_j + 128) 2^(8j) + top 2^128) and the top
__host__ __device__ __forceinline__ void pm_pack_words(const uint32_t c[5], uint32_t w[5]) {
  w[0] = (c[0] | (c[1] << 26)) ^ 0x80808080u;
  w[1] = ((c[1] >> 6) | (c[2] << 20)) ^ 0x80808080u;
  w[2] = ((c[2] >> 12) | (c[3] << 14)) ^ 0x80808080u;
  w[3] = ((c[3] >> 18) | (c[4] << 8)) ^ 0x80808080u;
  w[4] = c[4] >> 24;
}

enum { DOM_ELEMS = 0, DOM_MERGE = 1, DOM_MANY = 2, DOM_INT = 3 };

static inline void limbs26(fe a, uint32_t l[5]) {
  l[0] = (uint32_t)a.lo & M26;
  l[1] = (uint32_t)(a.lo >> 26) & M26;
  l[2] = (uint32_t)((a.lo >> 52) | (a.hi << 12)) & M26;
  l[3] = (uint32_t)(a.hi >> 14) & M26;
  l[4] = (uint32_t)(a.hi >> 40);
}

}  // namespace zkl
