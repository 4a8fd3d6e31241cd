/*
 * ORACLE — test infrastructure only.  Segment-proof verifier (winter-verifier 0.13.1
 * semantics restated): parses Proof::to_bytes, replays the
 * transcript, checks the out-of-domain constraint identity, every Merkle opening, the
 * DEEP values at the query positions, every FRI fold and the remainder, and the
 * proof-of-work.  It shares only the AIR and hash primitives with the oracle prover; the
 * checks themselves are the verifier-side formulas:
 *   transcript order               agg/fs.rs:67-237 (restated by the reference itself)
 *   OOD identity                   H(z) = sum_j H_j(z) z^(j n)
 *                                  = sum_k alpha_k c_k(z) (z - g^(n-1)) / (z^n - 1)
 *                                    + sum_a beta_a (t_a(z) - v_a) / (z - g^(s_a))
 *   DEEP at x = 3 w_N^p            agg/trace.rs:1126-1218
 *   FRI fold (folding factor 2)    agg/trace.rs:697-955, positions agg/child.rs:1072-1100
 *   batch Merkle openings          agg/child.rs:1049-1068 (even index: merge(acc, sib))
 */
#include <stdio.h>
#include <string.h>

#include "oracle.h"

void orc_context_elements(uint32_t W, size_t n, const zkl_proof_options *o, fe *out, int *nout);
int orc_pi_elements(const zkl_air_public_inputs *pi, fe *out);

typedef struct {
  const uint8_t *p;
  size_t len, off;
  int bad;
} rd_t;

static uint8_t rd_u8(rd_t *r) {
  if (r->off + 1 > r->len) { r->bad = 1; return 0; }
  return r->p[r->off++];
}
static uint64_t rd_u64(rd_t *r) {
  uint64_t v = 0;
  if (r->off + 8 > r->len) { r->bad = 1; return 0; }
  for (int i = 0; i < 8; i++) v |= (uint64_t)r->p[r->off + i] << (8 * i);
  r->off += 8;
  return v;
}
/* winter-utils read_usize (vint64): the first byte's trailing zeros give the length */
static uint64_t rd_usize(rd_t *r) {
  if (r->off >= r->len) { r->bad = 1; return 0; }
  uint8_t b0 = r->p[r->off];
  if (b0 == 0) { r->off++; return rd_u64(r); }
  int l = __builtin_ctz(b0) + 1;
  if (r->off + (size_t)l > r->len) { r->bad = 1; return 0; }
  uint64_t enc = 0;
  for (int i = 0; i < l; i++) enc |= (uint64_t)r->p[r->off + i] << (8 * i);
  r->off += (size_t)l;
  return enc >> l;
}
static fe rd_fe(rd_t *r) {
  if (r->off + 16 > r->len) { r->bad = 1; return 0; }
  fe v = fe_from_bytes_raw(r->p + r->off);
  r->off += 16;
  if (v >= FE_P) r->bad = 1;
  return v;
}
static fe rd_digest(rd_t *r) {
  fe v = rd_fe(r);
  for (int i = 0; i < 16 && !r->bad; i++)
    if (r->off + (size_t)i >= r->len || r->p[r->off + (size_t)i]) r->bad = 1;
  r->off += 16;
  return v;
}
/* a length-prefixed byte vector: returns a sub-reader */
static rd_t rd_vec(rd_t *r) {
  rd_t s = {0};
  uint64_t l = rd_usize(r);
  if (r->bad || r->off + l > r->len) { r->bad = 1; s.bad = 1; return s; }
  s.p = r->p + r->off;
  s.len = (size_t)l;
  r->off += (size_t)l;
  return s;
}

typedef struct { fe seed; uint64_t counter; } vcoin;
static void vc_reseed(vcoin *c, fe d) { c->seed = ph_merge(c->seed, d); c->counter = 0; }
static fe vc_draw(vcoin *c) { c->counter++; return ph_merge_with_int(c->seed, c->counter); }

static int cmp_size(const void *a, const void *b) {
  size_t x = *(const size_t *)a, y = *(const size_t *)b;
  return (x > y) - (x < y);
}

/* BatchMerkleProof::get_root: idx (sorted, unique) with leaf digests; proof lists in the
 * order MerkleTree::prove_batch wrote them.  Returns 0 and the root, or -1. */
static int batch_root(rd_t *pr, size_t n_leaves, const size_t *idx, const fe *leaf, size_t nidx, fe *root) {
  size_t depth = 0;
  while (((size_t)1 << depth) < n_leaves) depth++;
  if (rd_u8(pr) != depth) return -1;
  size_t m = rd_u8(pr);
  /* lists */
  fe **lists = (fe **)calloc(m ? m : 1, sizeof(fe *));
  size_t *cnt = (size_t *)calloc(m ? m : 1, sizeof(size_t)), *rpos = (size_t *)calloc(m ? m : 1, sizeof(size_t));
  int rc = 0;
  for (size_t k = 0; k < m && !pr->bad; k++) {
    cnt[k] = rd_u8(pr);
    lists[k] = (fe *)malloc((cnt[k] + 1) * sizeof(fe));
    for (size_t j = 0; j < cnt[k]; j++) lists[k][j] = rd_digest(pr);
  }
  if (pr->bad) rc = -1;
  /* normalized pairs */
  size_t *norm = (size_t *)malloc((nidx + 1) * sizeof(size_t));
  size_t nn = 0;
  for (size_t i = 0; i < nidx; i++) {
    size_t b = idx[i] & ~(size_t)1;
    if (nn == 0 || norm[nn - 1] != b) norm[nn++] = b;
  }
  if (nn != m) rc = -1;
  size_t *cur = (size_t *)malloc((nn + 1) * sizeof(size_t)), *nxt = (size_t *)malloc((nn + 1) * sizeof(size_t));
  fe *cv = (fe *)malloc((nn + 1) * sizeof(fe)), *nv = (fe *)malloc((nn + 1) * sizeof(fe));
#define POP(k, out)                                     \
  do {                                                  \
    if (rpos[k] >= cnt[k]) { rc = -1; (out) = 0; }      \
    else (out) = lists[k][rpos[k]++];                   \
  } while (0)
  for (size_t k = 0; k < nn && rc == 0; k++) {
    fe v[2];
    for (int t = 0; t < 2; t++) {
      size_t j = norm[k] + (size_t)t;
      size_t q = 0;
      while (q < nidx && idx[q] != j) q++;
      if (q < nidx) v[t] = leaf[q];
      else POP(k, v[t]);
    }
    cv[k] = ph_merge(v[0], v[1]);
    cur[k] = (norm[k] + n_leaves) >> 1;
  }
  size_t cn = nn;
  for (size_t lvl = 1; lvl < depth && rc == 0; lvl++) {
    size_t on = 0;
    for (size_t i = 0; i < cn && rc == 0; i++) {
      size_t sib = cur[i] ^ 1;
      fe parent;
      if (i + 1 < cn && cur[i + 1] == sib) {
        parent = ph_merge(cv[i], cv[i + 1]);
        i++;
      } else {
        fe s;
        POP(i, s);
        parent = (cur[i] & 1) ? ph_merge(s, cv[i]) : ph_merge(cv[i], s);
      }
      nxt[on] = sib >> 1;
      nv[on] = parent;
      on++;
    }
    memcpy(cur, nxt, on * sizeof(size_t));
    memcpy(cv, nv, on * sizeof(fe));
    cn = on;
  }
#undef POP
  if (rc == 0 && (cn != 1 || cur[0] != 1)) rc = -1;
  for (size_t k = 0; k < m && rc == 0; k++)
    if (rpos[k] != cnt[k]) rc = -1; /* every proof node consumed */
  if (rc == 0) *root = cv[0];
  for (size_t k = 0; k < m; k++) free(lists[k]);
  free(lists); free(cnt); free(rpos); free(norm); free(cur); free(nxt); free(cv); free(nv);
  return rc;
}

static size_t part_size(uint32_t np, uint32_t rate, size_t ncols) {
  if (np <= 1) return ncols;
  size_t a = (ncols + np - 1) / np;
  return a > rate ? a : rate;
}
static unsigned lg2(size_t n) { unsigned k = 0; while (((size_t)1 << k) < n) k++; return k; }

#define FAIL(msg)                                     \
  do {                                                \
    snprintf(err, errlen, "%s", msg);                 \
    rc = -1;                                          \
    goto done;                                        \
  } while (0)

int orc_verify_segment(const uint8_t *proof, size_t len, const zkl_air_public_inputs *pi,
                       const zkl_proof_options *opts, char *err, size_t errlen) {
  int rc = 0;
  zk_air air;
  int air_ok = 0;
  fe *tvals = NULL, *cvals = NULL, *ood_t = NULL, *alphas = NULL, *betas = NULL, *gam = NULL;
  fe *deep = NULL, *evals = NULL, *nevals = NULL, *lv = NULL, *leafd = NULL;
  size_t *pos = NULL, *fpos = NULL, *npos = NULL;
  rd_t r = {proof, len, 0, 0};
  if (errlen) err[0] = 0;

  /* ---- Context (TraceInfo, field modulus, ProofOptions) + num_unique_queries ---- */
  uint32_t W = rd_u8(&r);
  if (rd_u8(&r) != 0 || rd_u8(&r) != 0) FAIL("trace info: auxiliary segments are not supported");
  unsigned logn = rd_u8(&r);
  if (rd_u8(&r) != 0 || rd_u8(&r) != 0) FAIL("trace info: trace metadata must be empty");
  if (rd_u8(&r) != 16) FAIL("context: field element size must be 16");
  {
    uint8_t pb[16];
    fe_to_bytes(FE_P, pb);
    if (r.off + 16 > r.len || memcmp(r.p + r.off, pb, 16) != 0) FAIL("field modulus in the context is not f128");
    r.off += 16;
  }
  zkl_proof_options po;
  po.num_queries = rd_u8(&r); po.blowup_factor = rd_u8(&r); po.grinding_factor = rd_u8(&r);
  po.field_extension = rd_u8(&r); po.fri_folding_factor = rd_u8(&r); po.fri_remainder_max_degree = rd_u8(&r);
  po.batching_constraints = rd_u8(&r); po.batching_deep = rd_u8(&r);
  po.num_partitions = rd_u8(&r); po.hash_rate = rd_u8(&r);
  if (memcmp(&po, opts, sizeof po) != 0) FAIL("proof options in the proof differ from the expected options");
  size_t nq_proof = rd_u8(&r);
  if (r.bad) FAIL("truncated context");
  const size_t n = (size_t)1 << logn, N = n * opts->blowup_factor;
  if (air_new(&air, pi, W, n)) FAIL("AIR construction failed for these public inputs");
  air_ok = 1;
  const int C = air.n_comp_cols;
  const fe g = fe_root_of_unity(logn), wN = fe_root_of_unity(lg2(N));
  size_t rem_max = (size_t)(opts->fri_remainder_max_degree + 1) * opts->blowup_factor;
  int nl = 0;
  for (size_t d = N; d > rem_max; d /= 2) nl++;

  /* ---- Commitments ---- */
  fe troot, croot, froot[64], rem_commit;
  {
    rd_t cm = rd_vec(&r);
    troot = rd_digest(&cm);
    croot = rd_digest(&cm);
    for (int d = 0; d < nl; d++) froot[d] = rd_digest(&cm);
    rem_commit = rd_digest(&cm);
    if (cm.bad || cm.off != cm.len || r.bad) FAIL("malformed commitments");
  }

  /* ---- transcript replay up to the query positions ---- */
  fe seed_el[64];
  int ns;
  orc_context_elements(W, n, opts, seed_el, &ns);
  ns += orc_pi_elements(pi, seed_el + ns);
  vcoin coin = {ph_hash_elements(seed_el, (size_t)ns), 0};
  vc_reseed(&coin, troot);
  alphas = (fe *)malloc((size_t)air.n_tc * sizeof(fe));
  betas = (fe *)malloc((air.n_assert + 1) * sizeof(fe));
  for (int k = 0; k < air.n_tc; k++) alphas[k] = vc_draw(&coin);
  for (size_t a = 0; a < air.n_assert; a++) betas[a] = vc_draw(&coin);
  vc_reseed(&coin, croot);
  const fe z = vc_draw(&coin), zg = fe_mul(z, g);

  /* ---- the rest of the proof body ---- */
  if (rd_usize(&r) != 1) FAIL("trace queries: exactly one main segment expected");
  rd_t tq_v = rd_vec(&r), tq_p = rd_vec(&r), cq_v = rd_vec(&r), cq_p = rd_vec(&r);
  rd_t ood_ts = rd_vec(&r), ood_es = rd_vec(&r);
  if (r.bad) FAIL("malformed query / OOD sections");
  if (ood_ts.len != 2 * (size_t)W * 16 || ood_es.len != 2 * (size_t)C * 16) FAIL("OOD frame has the wrong shape");
  ood_t = (fe *)malloc(2 * ((size_t)W + C) * sizeof(fe)); /* t(z) | H(z) | t(zg) | H(zg) (prover order) */
  for (uint32_t c = 0; c < W; c++) ood_t[c] = rd_fe(&ood_ts);
  for (uint32_t c = 0; c < W; c++) ood_t[W + C + c] = rd_fe(&ood_ts);
  for (int j = 0; j < C; j++) ood_t[W + j] = rd_fe(&ood_es);
  for (int j = 0; j < C; j++) ood_t[2 * W + C + j] = rd_fe(&ood_es);
  if (ood_ts.bad || ood_es.bad) FAIL("non-canonical OOD values");

  /* OOD constraint identity */
  {
    fe per[32], tc[MAX_TC];
    air_periodic_at(&air, z, per);
    const fe gl = fe_exp(g, (fe)(n - 1)), zn = fe_exp(z, (fe)n);
    per[31] = fe_mul(fe_mul(gl, fe_sub(zn, 1)), fe_inv(fe_mul((fe)n, fe_sub(z, gl))));
    air_eval_transition(&air, ood_t, ood_t + W + C, per, tc);
    fe t = 0;
    for (int k = 0; k < air.n_tc; k++) t = fe_add(t, fe_mul(alphas[k], tc[k]));
    t = fe_mul(fe_mul(t, fe_sub(z, gl)), fe_inv(fe_sub(zn, 1)));
    /* boundary: sum_a beta_a (t_col(z) - v_a) / (z - g^step), grouped by step */
    fe b = 0;
    for (size_t a = 0; a < air.n_assert;) {
      size_t e = a;
      fe num = 0;
      while (e < air.n_assert && air.as_step[e] == air.as_step[a]) {
        num = fe_add(num, fe_mul(betas[e], fe_sub(ood_t[air.as_col[e]], air.as_val[e])));
        e++;
      }
      b = fe_add(b, fe_mul(num, fe_inv(fe_sub(z, fe_exp(g, (fe)air.as_step[a])))));
      a = e;
    }
    fe h = 0, zjn = 1;
    for (int j = 0; j < C; j++) { h = fe_add(h, fe_mul(ood_t[W + j], zjn)); zjn = fe_mul(zjn, zn); }
    if (fe_add(t, b) != h) FAIL("out-of-domain constraint identity does not hold");
  }
  vc_reseed(&coin, ph_hash_elements(ood_t, 2 * ((size_t)W + C)));
  gam = (fe *)malloc(((size_t)W + C) * sizeof(fe));
  for (size_t k = 0; k < (size_t)W + C; k++) gam[k] = vc_draw(&coin);
  fe alpha_l[64];
  for (int d = 0; d < nl; d++) { vc_reseed(&coin, froot[d]); alpha_l[d] = vc_draw(&coin); }
  vc_reseed(&coin, rem_commit);

  /* ---- FRI proof bytes, PoW nonce ---- */
  if ((int)rd_usize(&r) != nl) FAIL("FRI layer count mismatch");
  rd_t fl_v[64], fl_p[64];
  for (int d = 0; d < nl; d++) { fl_v[d] = rd_vec(&r); fl_p[d] = rd_vec(&r); }
  rd_t remv = rd_vec(&r);
  if (rd_u8(&r) != 0) FAIL("FRI remainder partitions must be 1");
  uint64_t nonce = rd_u64(&r);
  if (r.bad || r.off != r.len) FAIL("malformed FRI section or trailing bytes");
  {
    fe h = ph_merge_with_int(coin.seed, nonce);
    uint64_t lo = (uint64_t)h;
    unsigned tz = lo ? (unsigned)__builtin_ctzll(lo) : 64;
    if (tz < opts->grinding_factor) FAIL("proof-of-work nonce does not meet the grinding factor");
  }

  /* ---- query positions ---- */
  coin.seed = ph_merge_with_int(coin.seed, nonce);
  coin.counter = 0;
  size_t q = opts->num_queries, nq = 0;
  pos = (size_t *)malloc(q * sizeof(size_t));
  for (size_t k = 0; k < q; k++) pos[k] = (size_t)((uint64_t)vc_draw(&coin) & (N - 1));
  qsort(pos, q, sizeof(size_t), cmp_size);
  for (size_t k = 0; k < q; k++) if (nq == 0 || pos[nq - 1] != pos[k]) pos[nq++] = pos[k];
  if (nq != nq_proof) FAIL("num_unique_queries does not match the drawn positions");

  /* ---- trace and constraint openings ---- */
  if (tq_v.len != nq * W * 16 || cq_v.len != nq * (size_t)C * 16) FAIL("query value sections have the wrong size");
  tvals = (fe *)malloc(nq * W * sizeof(fe));
  cvals = (fe *)malloc(nq * (size_t)C * sizeof(fe));
  for (size_t k = 0; k < nq * W; k++) tvals[k] = rd_fe(&tq_v);
  for (size_t k = 0; k < nq * (size_t)C; k++) cvals[k] = rd_fe(&cq_v);
  if (tq_v.bad || cq_v.bad) FAIL("non-canonical query values");
  leafd = (fe *)malloc((nq + 1) * sizeof(fe));
  {
    fe root;
    size_t ps = part_size(opts->num_partitions, opts->hash_rate, W);
    for (size_t k = 0; k < nq; k++) leafd[k] = orc_row_digest(tvals + k * W, W, ps);
    if (batch_root(&tq_p, N, pos, leafd, nq, &root) || root != troot || tq_p.off != tq_p.len)
      FAIL("trace Merkle opening does not reproduce the trace commitment");
    ps = part_size(opts->num_partitions, opts->hash_rate, (size_t)C);
    for (size_t k = 0; k < nq; k++) leafd[k] = orc_row_digest(cvals + k * C, (size_t)C, ps);
    if (batch_root(&cq_p, N, pos, leafd, nq, &root) || root != croot || cq_p.off != cq_p.len)
      FAIL("constraint Merkle opening does not reproduce the constraint commitment");
  }

  /* ---- DEEP composition at the query positions ---- */
  deep = (fe *)malloc(nq * sizeof(fe));
  {
    fe sz = 0, szg = 0;
    for (uint32_t c = 0; c < W; c++) {
      sz = fe_add(sz, fe_mul(gam[c], ood_t[c]));
      szg = fe_add(szg, fe_mul(gam[c], ood_t[W + C + c]));
    }
    for (int j = 0; j < C; j++) {
      sz = fe_add(sz, fe_mul(gam[W + j], ood_t[W + j]));
      szg = fe_add(szg, fe_mul(gam[W + j], ood_t[2 * W + C + j]));
    }
    for (size_t k = 0; k < nq; k++) {
      fe x = fe_mul(3, fe_exp(wN, (fe)pos[k]));
      fe s = 0;
      for (uint32_t c = 0; c < W; c++) s = fe_add(s, fe_mul(gam[c], tvals[k * W + c]));
      for (int j = 0; j < C; j++) s = fe_add(s, fe_mul(gam[W + j], cvals[k * C + j]));
      deep[k] = fe_add(fe_mul(fe_sub(s, sz), fe_inv(fe_sub(x, z))), fe_mul(fe_sub(s, szg), fe_inv(fe_sub(x, zg))));
    }
  }

  /* ---- FRI: layer openings, folds, remainder ---- */
  {
    size_t np_ = nq, Nd = N;
    fpos = (size_t *)malloc((nq + 1) * sizeof(size_t));
    npos = (size_t *)malloc((nq + 1) * sizeof(size_t));
    evals = (fe *)malloc((nq + 1) * sizeof(fe));
    nevals = (fe *)malloc((nq + 1) * sizeof(fe));
    memcpy(fpos, pos, nq * sizeof(size_t));
    memcpy(evals, deep, nq * sizeof(fe));
    const fe inv2 = fe_inv(2);
    for (int d = 0; d < nl; d++) {
      size_t h = Nd / 2, m = 0;
      /* folded positions: p mod h, de-duplicated in order of first appearance */
      for (size_t k = 0; k < np_; k++) {
        size_t y = fpos[k] % h, j = 0;
        while (j < m && npos[j] != y) j++;
        if (j == m) npos[m++] = y;
      }
      if (fl_v[d].len != m * 32) FAIL("FRI layer values have the wrong size");
      lv = (fe *)malloc(2 * m * sizeof(fe));
      for (size_t k = 0; k < 2 * m; k++) lv[k] = rd_fe(&fl_v[d]);
      if (fl_v[d].bad) FAIL("non-canonical FRI layer values");
      /* the previous layer's values at this layer's positions */
      for (size_t k = 0; k < np_; k++) {
        size_t y = fpos[k] % h, j = 0;
        while (npos[j] != y) j++;
        if (lv[2 * j + (fpos[k] >= h ? 1 : 0)] != evals[k]) FAIL("FRI layer opening disagrees with the folded values");
      }
      /* Merkle: leaves hash_elements([e_y, e_{y+h}]) at index y, positions sorted */
      {
        size_t *sp = (size_t *)malloc((m + 1) * sizeof(size_t));
        fe *sl = (fe *)malloc((m + 1) * sizeof(fe));
        memcpy(sp, npos, m * sizeof(size_t));
        qsort(sp, m, sizeof(size_t), cmp_size);
        for (size_t k = 0; k < m; k++) {
          size_t j = 0;
          while (npos[j] != sp[k]) j++;
          sl[k] = ph_hash_elements(lv + 2 * j, 2);
        }
        fe root;
        int bad = batch_root(&fl_p[d], h, sp, sl, m, &root) || root != froot[d] || fl_p[d].off != fl_p[d].len;
        free(sp); free(sl);
        if (bad) FAIL("FRI layer Merkle opening does not reproduce the layer commitment");
      }
      /* fold: (v0+v1)/2 + alpha (v0-v1) / (2 x0), x0 = 3 * w_Nd^y (constant domain offset) */
      const fe gd = fe_root_of_unity(lg2(Nd));
      for (size_t j = 0; j < m; j++) {
        fe v0 = lv[2 * j], v1 = lv[2 * j + 1];
        fe x0 = fe_mul(3, fe_exp(gd, (fe)npos[j]));
        nevals[j] = fe_mul(fe_add(fe_add(v0, v1), fe_mul(alpha_l[d], fe_mul(fe_sub(v0, v1), fe_inv(x0)))), inv2);
      }
      free(lv);
      lv = NULL;
      memcpy(fpos, npos, m * sizeof(size_t));
      memcpy(evals, nevals, m * sizeof(fe));
      np_ = m;
      Nd = h;
    }
    /* remainder: rem = reversed coefficients of degree <= rem_deg over 3 * <w_Nd> */
    size_t rlen = opts->fri_remainder_max_degree + 1;
    if (remv.len != rlen * 16) FAIL("FRI remainder has the wrong size");
    fe rem[16];
    for (size_t k = 0; k < rlen; k++) rem[k] = rd_fe(&remv);
    if (remv.bad) FAIL("non-canonical remainder");
    if (ph_hash_elements(rem, rlen) != rem_commit) FAIL("remainder does not match its commitment");
    const fe gr = fe_root_of_unity(lg2(Nd));
    for (size_t k = 0; k < np_; k++) {
      fe x = fe_mul(3, fe_exp(gr, (fe)fpos[k])), v = 0, xp = 1;
      for (size_t c = 0; c < rlen; c++) { v = fe_add(v, fe_mul(rem[rlen - 1 - c], xp)); xp = fe_mul(xp, x); }
      if (v != evals[k]) FAIL("FRI remainder does not match the last layer");
    }
  }

done:
  if (air_ok) air_free(&air);
  free(tvals); free(cvals); free(ood_t); free(alphas); free(betas); free(gam); free(deep); free(evals);
  free(nevals); free(lv); free(leafd); free(pos); free(fpos); free(npos);
  return rc;
}
