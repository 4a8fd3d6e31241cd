/*
 * ORACLE — test infrastructure only.
 *
 * Poseidon suite derivation and the PoseidonHasher sponge, restating
 *   zk-lisp-proof-winterfell/src/poseidon/mod.rs:56-75   get_poseidon_suite_with_rounds
 *   poseidon/mod.rs:111-184                              MDS Cauchy derivation
 *   poseidon/mod.rs:186-217                              ROM rc, RC, domain tags
 *   poseidon/mod.rs:421-440                              ro_from_slices (BLAKE3 -> fe)
 *   poseidon/hasher.rs:57-231                            Hasher / ElementHasher impls
 *   utils.rs:33-74,346-381                               byte <-> field helpers
 *   commit.rs:31-79                                      program_field_commitment
 */
#include <stdio.h>
#include <string.h>
#include "oracle.h"

fe ro_from_slices(const char *domain, const uint8_t *const *parts, const size_t *lens, int nparts) {
  const uint8_t *p[8];
  size_t l[8];
  p[0] = (const uint8_t *)domain;
  l[0] = strlen(domain);
  for (int i = 0; i < nparts; i++) { p[i + 1] = parts[i]; l[i + 1] = lens[i]; }
  uint8_t h[32];
  orc_blake3_parts(p, l, nparts + 1, h);
  return fe_from_u128(fe_from_bytes_raw(h)); /* BE::from(lo) + BE::from(hi)*2^64 */
}

fe be_from_le8(const uint8_t b32[32]) { return fe_from_u128(fe_from_bytes_raw(b32)); }

static const fe POW2_64 = ((fe)1) << 64;

fe fold_bytes32(const uint8_t b[32]) {
  fe a = fe_from_u128(fe_from_bytes_raw(b));
  fe c = fe_from_u128(fe_from_bytes_raw(b + 16));
  return fe_add(a, fe_mul(c, POW2_64));
}

static void derive_points(const char *dom, const uint8_t sid[32], int n, fe *pts) {
  int have = 0;
  uint32_t ctr = 0;
  while (have < n) {
    uint8_t idx = (uint8_t)have;
    uint8_t cb[4] = {(uint8_t)ctr, (uint8_t)(ctr >> 8), (uint8_t)(ctr >> 16), (uint8_t)(ctr >> 24)};
    const uint8_t *parts[3] = {sid, &idx, cb};
    size_t lens[3] = {32, 1, 4};
    fe cand = ro_from_slices(dom, parts, lens, 3);
    int dup = (cand == 0);
    for (int i = 0; i < have && !dup; i++) dup = (pts[i] == cand);
    if (!dup) pts[have++] = cand;
    else ctr++;
  }
}

void pos_suite_derive(const uint8_t sid[32], int rounds, pos_suite *s) {
  const uint8_t *p1[1] = {sid};
  size_t l1[1] = {32};
  s->dom[0] = ro_from_slices("zkl/poseidon2/dom/c0", p1, l1, 1);
  s->dom[1] = ro_from_slices("zkl/poseidon2/dom/c1", p1, l1, 1);
  fe x[12], y[12];
  derive_points("zkl/poseidon2/mds/x", sid, 12, x);
  derive_points("zkl/poseidon2/mds/y", sid, 12, y);
  uint32_t adj = 0;
  for (;;) {
    int ok = 1;
    for (int i = 0; i < 12 && ok; i++)
      for (int j = 0; j < 12 && ok; j++)
        if (fe_add(x[i], y[j]) == 0) ok = 0;
    if (ok) break;
    for (int j = 0; j < 12; j++) { /* poseidon/mod.rs:150-165 */
      uint8_t jb = (uint8_t)j;
      uint8_t ab[4] = {(uint8_t)adj, (uint8_t)(adj >> 8), (uint8_t)(adj >> 16), (uint8_t)(adj >> 24)};
      const uint8_t *parts[3] = {sid, &jb, ab};
      size_t lens[3] = {32, 1, 4};
      fe cand = ro_from_slices("zkl/poseidon2/mds/y", parts, lens, 3);
      y[j] = cand == 0 ? 1 : cand;
    }
    adj++;
  }
  for (int i = 0; i < 12; i++)
    for (int j = 0; j < 12; j++) s->mds[i][j] = fe_inv(fe_add(x[i], y[j]));
  s->rounds = rounds;
  for (int r = 0; r < rounds && r < POS_ROUNDS; r++)
    for (int lane = 0; lane < 12; lane++) {
      uint8_t rb = (uint8_t)r, lb = (uint8_t)lane;
      const uint8_t *parts[3] = {sid, &rb, &lb};
      size_t lens[3] = {32, 1, 1};
      s->rc[r][lane] = ro_from_slices("zkl/poseidon2/rc", parts, lens, 3);
    }
}

void rom_constants(const uint8_t sid[32], fe rc[POS_ROUNDS][3], fe mds[3][3]) {
  for (int r = 0; r < POS_ROUNDS; r++)
    for (int lane = 0; lane < 3; lane++) {
      uint8_t rb = (uint8_t)r, lb = (uint8_t)lane;
      const uint8_t *parts[3] = {sid, &rb, &lb};
      size_t lens[3] = {32, 1, 1};
      rc[r][lane] = ro_from_slices("zkl/rom3/rc", parts, lens, 3);
    }
  fe x[3], y[3];
  derive_points("zkl/rom3/mds/x", sid, 3, x);
  derive_points("zkl/rom3/mds/y", sid, 3, y);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) mds[i][j] = fe_inv(fe_add(x[i], y[j]));
}

/* one full permutation: per round x^3 on all lanes, then MDS, then + rc (hasher.rs:173-190) */
void pos_permute(const pos_suite *s, fe st[12]) {
  /* sum_k mds[i][k]*c[k] is accumulated as an unreduced 256+4-bit integer and reduced once
   * per lane; the residue is the same as the reference's per-term field additions. */
  for (int r = 0; r < s->rounds; r++) {
    fe c[12], n[12];
    for (int i = 0; i < 12; i++) c[i] = fe_cube(st[i]);
    for (int i = 0; i < 12; i++) {
      fe hi = 0, lo = 0;
      uint64_t e = 0;
      for (int k = 0; k < 12; k++) {
        fe ph, pl;
        fe_mul_wide(s->mds[i][k], c[k], &ph, &pl);
        lo += pl;
        ph += (lo < pl);
        hi += ph;
        e += (hi < ph);
      }
      fe t = fe_reduce_wide((fe)e, hi);
      n[i] = fe_add(fe_reduce_wide(t, lo), s->rc[r][i]);
    }
    memcpy(st, n, sizeof n);
  }
}

static fe domain_fe(const char *domain) {
  uint8_t d[32] = {0};
  size_t l = strlen(domain);
  memcpy(d, domain, l < 32 ? l : 32);
  return fold_bytes32(d);
}

/* sponge over pre-folded 32-byte chunks (ro_bytes_sponge_custom_rounds, hasher.rs:144-231) */
static fe sponge_fes(const pos_suite *s, fe dom_fe, const fe *msgs, size_t n) {
  fe st[12] = {0};
  st[10] = s->dom[0];
  st[11] = s->dom[1];
  int lane = 0;
  st[lane] = fe_add(st[lane], dom_fe);
  lane++;
  for (size_t i = 0; i < n; i++) {
    st[lane] = fe_add(st[lane], msgs[i]);
    if (++lane == POS_RATE) { pos_permute(s, st); lane = 0; }
  }
  if (lane != 0) pos_permute(s, st);
  return st[0];
}

fe sponge_bytes(const pos_suite *s, const char *domain, const uint8_t *data, size_t len) {
  size_t nch = (len + 31) / 32;
  fe *m = (fe *)malloc((nch ? nch : 1) * sizeof(fe));
  for (size_t i = 0; i < nch; i++) {
    uint8_t c[32] = {0};
    size_t l = len - 32 * i < 32 ? len - 32 * i : 32;
    memcpy(c, data + 32 * i, l);
    m[i] = fold_bytes32(c);
  }
  fe r = sponge_fes(s, domain_fe(domain), m, nch);
  free(m);
  return r;
}

static pos_suite g_hsuite;
static int g_hsuite_init = 0;
static fe g_dom_bytes, g_dom_merge, g_dom_many, g_dom_int, g_dom_elem;

const pos_suite *pos_hasher_suite(void) {
  if (!g_hsuite_init) {
    uint8_t z[32] = {0};
    pos_suite_derive(z, POS_ROUNDS, &g_hsuite);
    g_dom_bytes = domain_fe("zkl/winter/hash/bytes");
    g_dom_merge = domain_fe("zkl/winter/hash/merge");
    g_dom_many = domain_fe("zkl/winter/hash/merge_many");
    g_dom_int = domain_fe("zkl/winter/hash/merge_with_int");
    g_dom_elem = domain_fe("winter/hash/elements");
    g_hsuite_init = 1;
  }
  return &g_hsuite;
}

fe ph_hash_bytes(const uint8_t *data, size_t len) {
  return sponge_bytes(pos_hasher_suite(), "zkl/winter/hash/bytes", data, len);
}

/* a digest is fe_to_bytes(x) || 0^16, so its 32-byte chunk folds back to x */
fe ph_merge(fe a, fe b) {
  const pos_suite *s = pos_hasher_suite();
  fe m[2] = {a, b};
  return sponge_fes(s, g_dom_merge, m, 2);
}

fe ph_merge_many(const fe *d, size_t n) {
  const pos_suite *s = pos_hasher_suite();
  if (n == 0) return 0; /* zero digest (hasher.rs:88-90) */
  return sponge_fes(s, g_dom_many, d, n);
}

fe ph_merge_with_int(fe seed, uint64_t v) {
  const pos_suite *s = pos_hasher_suite();
  fe m[2] = {seed, (fe)v};
  return sponge_fes(s, g_dom_int, m, 2);
}

/* hash_elements: bytes = 16-byte LE elements; chunk j = e[2j] + e[2j+1]*2^64 */
fe ph_hash_elements(const fe *e, size_t n) {
  const pos_suite *s = pos_hasher_suite();
  size_t nch = (n + 1) / 2;
  fe stackbuf[64];
  fe *m = nch <= 64 ? stackbuf : (fe *)malloc(nch * sizeof(fe));
  for (size_t j = 0; j < nch; j++) {
    fe a = e[2 * j];
    fe b = (2 * j + 1 < n) ? e[2 * j + 1] : 0;
    m[j] = fe_add(a, fe_mul(b, POW2_64));
  }
  fe r = sponge_fes(s, g_dom_elem, m, nch);
  if (m != stackbuf) free(m);
  return r;
}

void program_field_commitment(const uint8_t b32[32], fe out[2]) {
  pos_suite s;
  pos_suite_derive(b32, POS_ROUNDS, &s);
  fe st[12] = {0};
  st[0] = fe_from_u128(fe_from_bytes_raw(b32));
  st[1] = fe_from_u128(fe_from_bytes_raw(b32 + 16));
  st[10] = s.dom[0];
  st[11] = s.dom[1];
  pos_permute(&s, st);
  out[0] = st[0];
  out[1] = st[1];
}
