/*
 * ORACLE — test infrastructure only.
 *
 * Radix-2 NTT over f128 in natural order, restating the math of winter-math 0.13.1
 * `fft::{evaluate_poly, evaluate_poly_with_offset, interpolate_poly,
 * interpolate_poly_with_offset}` (used by the reference at vm/air/mod.rs:574-588 and by
 * Winterfell's trace LDE / composition polynomial).  Results are exact residues, so the
 * evaluation order of butterflies does not matter.
 */
#include <string.h>
#include "oracle.h"

void fe_batch_inv(fe *out, const fe *in, size_t n, fe *scratch) {
  fe acc = 1;
  for (size_t i = 0; i < n; i++) {
    scratch[i] = acc;
    if (in[i]) acc = fe_mul(acc, in[i]);
  }
  fe inv = fe_inv(acc);
  for (size_t i = n; i-- > 0;) {
    if (in[i]) {
      fe t = fe_mul(inv, scratch[i]);
      inv = fe_mul(inv, in[i]);
      out[i] = t;
    } else {
      out[i] = 0;
    }
  }
}

static unsigned ilog2(size_t n) { unsigned k = 0; while (((size_t)1 << k) < n) k++; return k; }

void ntt_inplace(fe *a, size_t n, int inverse) {
  unsigned logn = ilog2(n);
  for (size_t i = 1, j = 0; i < n; i++) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) { fe t = a[i]; a[i] = a[j]; a[j] = t; }
  }
  for (unsigned s = 1; s <= logn; s++) {
    size_t m = (size_t)1 << s, h = m >> 1;
    fe w = fe_root_of_unity(s);
    if (inverse) w = fe_inv(w);
    fe *tw = (fe *)malloc(h * sizeof(fe));
    tw[0] = 1;
    for (size_t k = 1; k < h; k++) tw[k] = fe_mul(tw[k - 1], w);
    for (size_t b = 0; b < n; b += m)
      for (size_t k = 0; k < h; k++) {
        fe u = a[b + k], v = fe_mul(a[b + k + h], tw[k]);
        a[b + k] = fe_add(u, v);
        a[b + k + h] = fe_sub(u, v);
      }
    free(tw);
  }
  if (inverse) {
    fe ninv = fe_inv((fe)n);
    for (size_t i = 0; i < n; i++) a[i] = fe_mul(a[i], ninv);
  }
}

/* values over offset*<w_n> (natural order) -> coefficients */
void coset_interpolate(fe *a, size_t n, fe offset) {
  ntt_inplace(a, n, 1);
  fe oi = fe_inv(offset), p = 1;
  for (size_t i = 0; i < n; i++) { a[i] = fe_mul(a[i], p); p = fe_mul(p, oi); }
}

/* coefficients (ncoef <= n) -> values over offset*<w_n> */
void coset_evaluate(const fe *c, size_t ncoef, fe *out, size_t n, fe offset) {
  fe p = 1;
  for (size_t i = 0; i < n; i++) {
    if (i < ncoef) { out[i] = fe_mul(c[i], p); p = fe_mul(p, offset); }
    else out[i] = 0;
  }
  ntt_inplace(out, n, 0);
}

fe poly_eval(const fe *c, size_t n, fe x) {
  fe acc = 0;
  for (size_t i = n; i-- > 0;) acc = fe_add(fe_mul(acc, x), c[i]);
  return acc;
}
