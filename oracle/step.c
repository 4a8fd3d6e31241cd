/*
 * ORACLE — test infrastructure only.  CPU restatement of the zl1 step-proof wrapper that
 * prove_segment puts around the inner Winterfell proof:
 *   - StepProof::to_bytes         zk-lisp-proof-winterfell/src/proof/step.rs:79-151
 *   - StepProof::from_bytes       step.rs:153-493 (field order, errors, single-segment rule)
 *   - StepMeta::new / from_env    step.rs:496-533
 *   - zl1 root_trace              proof/format.rs:214-238
 *   - step_digest                 proof/digest.rs:16-68
 *   - poseidon_hash_two_lanes     poseidon/mod.rs:255-291
 * Parity: the library's encoder/digest (zk-lisp_amd/csrc/step.cpp) are checked against
 * this file byte for byte (tests/test_step.py).  The BLAKE3 and Poseidon primitives are
 * pinned as in oracle.h; the wrapper layout follows the reference source directly.
 */
#include <stdio.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  uint8_t *p;
  size_t n, cap;
} wbuf;

static void w_raw(wbuf *b, const void *src, size_t k) {
  if (b->n + k > b->cap) {
    b->cap = (b->n + k) * 2 + 64;
    b->p = (uint8_t *)realloc(b->p, b->cap);
  }
  memcpy(b->p + b->n, src, k);
  b->n += k;
}
static void w_le(wbuf *b, uint64_t x, int bytes) {
  uint8_t t[8];
  for (int i = 0; i < bytes; i++) t[i] = (uint8_t)(x >> (8 * i));
  w_raw(b, t, (size_t)bytes);
}
/* utils::fe_to_bytes_fold (utils.rs:375-381) */
static void w_fe_fold(wbuf *b, fe x) {
  uint8_t t[32] = {0};
  fe_to_bytes(x, t);
  w_raw(b, t, 32);
}

/* winter-utils read_usize: vint64 */
static int rd_usize(const uint8_t *p, size_t n, size_t *off, uint64_t *out) {
  if (*off >= n) return -1;
  uint8_t f = p[*off];
  if (f == 0) {
    if (*off + 9 > n) return -1;
    uint64_t x = 0;
    for (int i = 0; i < 8; i++) x |= (uint64_t)p[*off + 1 + i] << (8 * i);
    *off += 9;
    *out = x;
    return 0;
  }
  int len = 1;
  while (!(f & 1)) { f >>= 1; len++; }
  if (*off + (size_t)len > n) return -1;
  uint64_t e = 0;
  for (int i = 0; i < len; i++) e |= (uint64_t)p[*off + i] << (8 * i);
  *off += (size_t)len;
  *out = e >> len;
  return 0;
}

/* Proof::to_bytes fields the wrapper reads: TraceInfo (6 bytes, log2 length at [3]), the
 * field modulus (size-prefixed), ProofOptions (queries [0], blowup [1]), num_unique_queries,
 * then Commitments (length-prefixed 32-byte digests). */
typedef struct {
  unsigned logn, blowup, queries;
  const uint8_t *dig;
  size_t ndig;
} inner_view;

static int view_inner(const uint8_t *p, size_t n, inner_view *v) {
  size_t off = 0;
  if (n < 7) return -1;
  if (p[1] || p[2]) return -1;
  v->logn = p[3];
  off = 6;
  size_t flen = p[off];
  off += 1 + flen;
  if (off + 11 > n) return -1;
  v->queries = p[off];
  v->blowup = p[off + 1];
  off += 11;
  uint64_t clen;
  if (rd_usize(p, n, &off, &clen) || clen % 32 || clen < 64 || off + clen > n) return -1;
  v->dig = p + off;
  v->ndig = (size_t)(clen / 32);
  return 0;
}

int orc_step_encode(const zkl_air_public_inputs *pi, const zkl_step_info *s, const uint8_t *inner, size_t inner_len,
                    uint8_t **out, size_t *out_len) {
  inner_view v;
  if (s->n_main_args > ZKL_MAX_MAIN_SLOTS || view_inner(inner, inner_len, &v)) return -1;
  wbuf b = {0, 0, 0};
  w_raw(&b, "ZKLSTP1", 7);
  w_le(&b, s->lambda_bits, 4);
  w_raw(&b, s->suite_id, 32);
  w_raw(&b, pi->program_id, 32);
  w_raw(&b, pi->program_commitment, 32);
  w_raw(&b, pi->merkle_root, 32);
  w_le(&b, pi->feature_mask, 8);
  w_le(&b, s->n_main_args, 4);
  for (uint32_t i = 0; i < s->n_main_args; i++) {
    const zkl_vm_arg *a = &s->main_args[i];
    if (a->tag > 2) { free(b.p); return -1; }
    uint8_t t = (uint8_t)a->tag;
    w_raw(&b, &t, 1);
    w_raw(&b, a->bytes, a->tag == 0 ? 8 : a->tag == 1 ? 16 : 32);
  }
  w_le(&b, pi->vm_usage_mask, 4);
  w_le(&b, pi->ram_delta_clk_bits, 4);
  for (int i = 0; i < 3; i++) w_fe_fold(&b, ((fe)pi->rom_acc[i].hi << 64) | pi->rom_acc[i].lo);
  w_le(&b, s->segment_index, 4);
  w_le(&b, s->segments_total, 4);
  w_raw(&b, s->pc_init, 32);
  w_raw(&b, s->state_in_hash, 32);
  w_raw(&b, s->state_out_hash, 32);
  w_raw(&b, s->ram_gp_unsorted_in, 32);
  w_raw(&b, s->ram_gp_unsorted_out, 32);
  w_raw(&b, s->ram_gp_sorted_in, 32);
  w_raw(&b, s->ram_gp_sorted_out, 32);
  for (int i = 0; i < 3; i++) w_raw(&b, s->rom_s_in[i], 32);
  for (int i = 0; i < 3; i++) w_raw(&b, s->rom_s_out[i], 32);
  w_le(&b, inner_len, 4);
  w_raw(&b, inner, inner_len);
  *out = b.p;
  *out_len = b.n;
  return 0;
}

/* poseidon_hash_two_lanes: [l, r, 0 x 8, dom0, dom1] -> permutation -> lane 0 */
static fe two_lanes(const pos_suite *S, fe l, fe r) {
  fe st[12] = {l, r, 0, 0, 0, 0, 0, 0, 0, 0, S->dom[0], S->dom[1]};
  pos_permute(S, st);
  return st[0];
}

static fe ro1(const char *dom, const uint8_t *p, size_t n) {
  const uint8_t *parts[1] = {p};
  size_t lens[1] = {n};
  return ro_from_slices(dom, parts, lens, 1);
}

/* agg::child::children_root_from_compact (agg/child.rs:853-895) */
static int cmp32(const void *a, const void *b) { return memcmp(a, b, 32); }

int orc_children_root(const uint8_t suite[32], const uint8_t *digests, const uint8_t *roots, uint32_t n,
                      uint8_t out[32]) {
  memset(out, 0, 32);
  if (n == 0) return 0;
  pos_suite S;
  pos_suite_derive(suite, POS_ROUNDS, &S);
  uint8_t *items = (uint8_t *)calloc(n, 32);
  fe *layer = (fe *)malloc(sizeof(fe) * n);
  for (uint32_t i = 0; i < n; i++) {
    fe leaf = two_lanes(&S, fold_bytes32(digests + 32 * i), fold_bytes32(roots + 32 * i));
    fe_to_bytes(leaf, items + 32 * i); /* fe_to_bytes_fold: 16 LE bytes + 16 zero */
  }
  qsort(items, n, 32, cmp32);
  size_t m = n;
  for (size_t i = 0; i < m; i++) layer[i] = fold_bytes32(items + 32 * i);
  while (m > 1) {
    size_t k = 0;
    for (size_t i = 0; i < m; i += 2) layer[k++] = two_lanes(&S, layer[i], i + 1 < m ? layer[i + 1] : layer[i]);
    m = k;
  }
  fe_to_bytes(layer[0], out);
  free(items);
  free(layer);
  return 0;
}

/* error text follows step.rs ("step proof truncated before <field>") */
#define NEED(k, what)                                                        \
  do {                                                                       \
    if (off + (size_t)(k) > n) {                                             \
      snprintf(err, errlen, "step proof truncated before %s", what);         \
      return -1;                                                             \
    }                                                                        \
  } while (0)

int orc_step_digest(const uint8_t *p, size_t n, uint8_t digest[32], uint8_t rt[32], char *err, size_t errlen) {
  size_t off = 0;
  if (errlen) err[0] = 0;
  if (n < 7) { snprintf(err, errlen, "step proof too short to contain magic header"); return -1; }
  if (memcmp(p, "ZKLSTP1", 7)) { snprintf(err, errlen, "invalid step proof magic tag"); return -1; }
  off = 7;
#define U32(dst, what) do { NEED(4, what); dst = 0; for (int i_ = 0; i_ < 4; i_++) dst |= (uint32_t)p[off + i_] << (8 * i_); off += 4; } while (0)
  uint32_t lambda_bits, nargs, seg_index, seg_total, inner_len, tmp;
  U32(lambda_bits, "lambda_bits");
  NEED(128, "suite_id bytes");
  const uint8_t *suite = p + off, *program_id = p + off + 32, *program_commitment = p + off + 64;
  off += 128;
  NEED(8, "feature_mask");
  uint64_t feature_mask = 0;
  for (int i = 0; i < 8; i++) feature_mask |= (uint64_t)p[off + i] << (8 * i);
  off += 8;
  U32(nargs, "main_args length");
  size_t slots = 0;
  for (uint32_t a = 0; a < nargs; a++) {
    NEED(1, "VmArg tag");
    uint8_t tag = p[off++];
    if (tag > 2) { snprintf(err, errlen, "invalid VmArg tag in step proof encoding"); return -1; }
    size_t k = tag == 0 ? 8 : tag == 1 ? 16 : 32;
    NEED(k, tag == 0 ? "VmArg::U64" : tag == 1 ? "VmArg::U128" : "VmArg::Bytes32");
    off += k;
    slots += tag == 2 ? 2 : 1;
  }
  U32(tmp, "vm_usage_mask");
  U32(tmp, "ram_delta_clk_bits");
  (void)tmp;
  NEED(96, "rom_acc bytes");
  off += 96;
  U32(seg_index, "segment_index");
  U32(seg_total, "segments_total");
  NEED(32 * 13, "pc_init bytes");
  const uint8_t *pc_init = p + off, *bnd = p + off + 32;
  off += 32 * 13;
  U32(inner_len, "inner proof length");
  NEED(inner_len, "inner proof bytes");
  inner_view v;
  if (view_inner(p + off, inner_len, &v)) { snprintf(err, errlen, "failed to decode inner Winterfell proof"); return -1; }
#undef U32
  if (seg_total <= 1) { seg_index = 0; seg_total = 1; }

  /* root_trace = BLAKE3("zkl/step/root_trace" || suite || every commitment digest) */
  {
    const uint8_t *parts[3] = {(const uint8_t *)"zkl/step/root_trace", suite, v.dig};
    size_t lens[3] = {19, 32, 32 * v.ndig};
    uint8_t r[32];
    orc_blake3_parts(parts, lens, 3, r);
    if (rt) memcpy(rt, r, 32);
    if (!digest) return 0;

    pos_suite S;
    pos_suite_derive(suite, POS_ROUNDS, &S);
    uint32_t m = 1u << v.logn;
    uint32_t pi_len = (uint32_t)(5 + slots + 13);
    uint32_t lam = lambda_bits > 65535 ? 65535 : lambda_bits;
    wbuf mb = {0, 0, 0}, pb = {0, 0, 0};
    w_le(&mb, m, 4); w_le(&mb, v.blowup, 2); w_le(&mb, v.queries, 2); w_le(&mb, 2, 2); w_le(&mb, lam, 2);
    w_le(&mb, pi_len, 4); w_le(&mb, (uint64_t)m * v.queries, 8);
    w_raw(&pb, program_id, 32); w_raw(&pb, program_commitment, 32); w_le(&pb, feature_mask, 8);
    w_le(&pb, seg_index, 4); w_le(&pb, seg_total, 4); w_raw(&pb, pc_init, 32); w_raw(&pb, bnd, 32 * 12);
    fe suite_fe = ro1("zkl/step/digest/suite", suite, 32);
    fe h_meta = two_lanes(&S, ro1("zkl/step/digest/meta", mb.p, mb.n), 0);
    fe h_pi = two_lanes(&S, ro1("zkl/step/digest/pi", pb.p, pb.n), 0);
    fe h_roots = two_lanes(&S, fold_bytes32(r), 0);
    fe ch = two_lanes(&S, two_lanes(&S, two_lanes(&S, suite_fe, h_meta), h_pi), h_roots);
    memset(digest, 0, 32);
    fe_to_bytes(ch, digest);
    free(mb.p);
    free(pb.p);
  }
  return 0;
}
