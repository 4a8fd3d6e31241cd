/*
 * ORACLE — test infrastructure only.
 *
 * Single-threaded CPU restatement of winterfell 0.13.1 `Prover::prove` as instantiated by
 * the reference (prove.rs:425-517: ZkLispAir, PoseidonHasher, MerkleTree, DefaultRandomCoin,
 * DefaultTraceLde, DefaultConstraintEvaluator, DefaultConstraintCommitment), options
 * prove.rs:963-972 + with_partitions (prove.rs:1121).
 *
 * Conventions and where they are pinned:
 *   transcript order             agg/fs.rs:67-237 (reference's own replay of the verifier)
 *   OOD hash order               agg/fs.rs:152-164  z-row || H(z) || zg-row || H(zg)
 *   DEEP formula (z and zg terms for trace AND composition columns)  agg/trace.rs:1126-1218
 *   FRI fold / constant offset / remainder Horner order               agg/trace.rs:697-955
 *   FRI folded positions         agg/child.rs:1072-1100
 *   Merkle orientation           agg/child.rs:1049-1068
 *   LDE point of position i      x = GENERATOR * g^i                   agg/trace.rs:1126-1140
 *   everything else              winterfell 0.13.1 source as published (crate absent here):
 *                                Context::to_elements, row partitioning, BatchMerkleProof
 *                                layout, Proof::to_bytes field layout -> "parity unpinned".
 * Boundary constraints: boundary_mode 1 evaluates Winterfell's per-(stride,step) groups
 * literally (O(groups x CE)); mode 0 evaluates the algebraically identical column-wise
 * form sum_c [P_c(x) M_c(x) - W(x)] / (x^n - 1); tests check both agree.
 */
#include <stdio.h>
#include <string.h>
#include "oracle.h"

int g_orc_threads = 1;
void orc_set_threads(int t) { g_orc_threads = t < 1 ? 1 : t; }

/* ------------------------------------------------------------------ bytes */
typedef struct { uint8_t *p; size_t len, cap; } bbuf;
static void bb_put(bbuf *b, const void *d, size_t n) {
  if (b->len + n > b->cap) {
    size_t c = b->cap ? b->cap * 2 : 4096;
    while (c < b->len + n) c *= 2;
    b->p = (uint8_t *)realloc(b->p, c);
    b->cap = c;
  }
  memcpy(b->p + b->len, d, n);
  b->len += n;
}
static void bb_u8(bbuf *b, uint8_t v) { bb_put(b, &v, 1); }
static void bb_u64(bbuf *b, uint64_t v) {
  uint8_t t[8];
  for (int i = 0; i < 8; i++) t[i] = (uint8_t)(v >> (8 * i));
  bb_put(b, t, 8);
}
/* winter-utils ByteWriter::write_usize (vint64) */
static void bb_usize(bbuf *b, uint64_t v) {
  int lz = v ? __builtin_clzll(v) : 64;
  int l = (lz > 0 ? lz - 1 : 0) / 7;
  int len = 9 - (l < 8 ? l : 8);
  if (len == 9) { bb_u8(b, 0); bb_u64(b, v); return; }
  uint64_t enc = ((v << 1) | 1) << (len - 1);
  uint8_t t[8];
  for (int i = 0; i < 8; i++) t[i] = (uint8_t)(enc >> (8 * i));
  bb_put(b, t, (size_t)len);
}
static void bb_fe(bbuf *b, fe v) { uint8_t t[16]; fe_to_bytes(v, t); bb_put(b, t, 16); }
static void bb_digest(bbuf *b, fe v) { uint8_t t[32] = {0}; fe_to_bytes(v, t); bb_put(b, t, 32); }
static void bb_vec(bbuf *b, const bbuf *inner) { bb_usize(b, inner->len); bb_put(b, inner->p, inner->len); }

/* ------------------------------------------------------------------ coin */
typedef struct { fe seed; uint64_t counter; } coin_t;
static void coin_reseed(coin_t *c, fe d) { c->seed = ph_merge(c->seed, d); c->counter = 0; }
static fe coin_draw(coin_t *c) { c->counter++; return ph_merge_with_int(c->seed, c->counter); }

/* draw K consecutive elements (independent given seed: parallel-safe) */
static void coin_draw_many(coin_t *c, fe *out, size_t k) {
  uint64_t base = c->counter;
  fe seed = c->seed;
#pragma omp parallel for num_threads(g_orc_threads) schedule(static)
  for (size_t i = 0; i < k; i++) out[i] = ph_merge_with_int(seed, base + 1 + i);
  c->counter += k;
}

/* ------------------------------------------------------------------ merkle */
static fe *merkle_build(const fe *leaves, size_t n) {
  fe *nodes = (fe *)malloc(2 * n * sizeof(fe));
  memcpy(nodes + n, leaves, n * sizeof(fe));
  for (size_t lvl = n / 2; lvl >= 1; lvl /= 2) {
#pragma omp parallel for num_threads(g_orc_threads) schedule(static)
    for (size_t i = lvl; i < 2 * lvl; i++) nodes[i] = ph_merge(nodes[2 * i], nodes[2 * i + 1]);
  }
  nodes[0] = 0;
  return nodes;
}

static int cmp_sz(const void *a, const void *b) {
  size_t x = *(const size_t *)a, y = *(const size_t *)b;
  return (x > y) - (x < y);
}

/* MerkleTree::prove_batch (winter-crypto 0.13) -> BatchMerkleProof bytes:
 * depth u8, #node-lists u8, then per list: u8 count + 32-byte digests */
static void merkle_batch_proof(const fe *nodes, size_t n, const size_t *idx, size_t nidx, bbuf *out) {
  size_t depth = 0; while (((size_t)1 << depth) < n) depth++;
  size_t *norm = (size_t *)malloc(nidx * sizeof(size_t));
  for (size_t i = 0; i < nidx; i++) norm[i] = idx[i] & ~(size_t)1;
  qsort(norm, nidx, sizeof(size_t), cmp_sz);
  size_t m = 0;
  for (size_t i = 0; i < nidx; i++) if (m == 0 || norm[m - 1] != norm[i]) norm[m++] = norm[i];
  /* membership of requested leaves */
  fe **lists = (fe **)calloc(m, sizeof(fe *));
  size_t *cnt = (size_t *)calloc(m, sizeof(size_t));
  for (size_t k = 0; k < m; k++) lists[k] = (fe *)malloc((depth + 2) * sizeof(fe));
  size_t *next = (size_t *)malloc(m * sizeof(size_t));
  for (size_t k = 0; k < m; k++) {
    for (size_t j = norm[k]; j < norm[k] + 2; j++) {
      int requested = 0;
      for (size_t q = 0; q < nidx; q++) if (idx[q] == j) { requested = 1; break; }
      if (!requested) lists[k][cnt[k]++] = nodes[n + j];
    }
    next[k] = (norm[k] + n) >> 1;
  }
  size_t nn = m;
  size_t *cur = (size_t *)malloc(m * sizeof(size_t));
  for (size_t lvl = 1; lvl < depth; lvl++) {
    memcpy(cur, next, nn * sizeof(size_t));
    size_t cn = nn;
    nn = 0;
    for (size_t i = 0; i < cn; i++) {
      size_t sib = cur[i] ^ 1;
      if (i + 1 < cn && cur[i + 1] == sib) i++;
      else lists[i][cnt[i]++] = nodes[sib];
      next[nn++] = sib >> 1;
    }
  }
  bb_u8(out, (uint8_t)depth);
  bb_u8(out, (uint8_t)m);
  for (size_t k = 0; k < m; k++) {
    bb_u8(out, (uint8_t)cnt[k]);
    for (size_t j = 0; j < cnt[k]; j++) bb_digest(out, lists[k][j]);
    free(lists[k]);
  }
  free(lists); free(cnt); free(next); free(cur); free(norm);
}

/* ------------------------------------------------------------------ row hashing */
static size_t partition_size(uint32_t np, uint32_t rate, size_t ncols) {
  if (np <= 1) return ncols;
  size_t a = (ncols + np - 1) / np;
  return a > rate ? a : rate;
}
/* Row digest of a partitioned row (PartitionOptions).  Two rules differ only for
 * a row whose partition size exceeds its width, i.e. one chunk (composition rows at
 * n >= 2^14; any matrix narrower than its partition size):
 *   rule 0 (default) winterfell 0.13.1 RowMatrix::commit_to_rows [WF-recall]: hash_elements
 *          when partition_size == num_cols, otherwise merge_many over the chunk digests,
 *          even of a single digest;
 *   rule 1 the reference's own restatement agg/child.rs:1025-1045 (hash_row_poseidon):
 *          a single chunk digest is returned as is.
 * DESIGN.md §3.1 records why rule 0 is the default. */
int g_orc_row_digest_rule = 0;
void orc_set_row_digest_rule(int r) { g_orc_row_digest_rule = r ? 1 : 0; }
int orc_row_digest_rule(void) { return g_orc_row_digest_rule; }

fe orc_row_digest(const fe *row, size_t ncols, size_t psize) {
  if (psize == ncols) return ph_hash_elements(row, ncols);
  fe d[256];
  size_t np = 0;
  for (size_t s = 0; s < ncols; s += psize) {
    size_t l = ncols - s < psize ? ncols - s : psize;
    d[np++] = ph_hash_elements(row + s, l);
  }
  if (np == 1 && g_orc_row_digest_rule == 1) return d[0];
  return ph_merge_many(d, np);
}
static void hash_rows(const fe *rows, size_t nrows, size_t ncols, uint32_t np, uint32_t rate, fe *out) {
  size_t ps = partition_size(np, rate, ncols);
#pragma omp parallel for num_threads(g_orc_threads) schedule(dynamic, 64)
  for (size_t r = 0; r < nrows; r++) out[r] = orc_row_digest(rows + r * ncols, ncols, ps);
}

/* ------------------------------------------------------------------ proof */
static const char *g_err = "";
const char *orc_last_error(void) { return g_err; }
void orc_free(void *p) { free(p); }

static fe fe_of(zkl_f128 v) { return ((fe)v.hi << 64) | v.lo; }

void orc_context_elements(uint32_t W, size_t n, const zkl_proof_options *o, fe *out, int *nout) {
  int k = 0;
  out[k++] = (fe)((uint32_t)W << 8);              /* main width << 8 | num aux segments */
  out[k++] = (fe)(uint32_t)n;                      /* trace length */
  out[k++] = (fe)0xFFFFD30000000001ull;            /* modulus LE bytes [0..8) */
  out[k++] = (fe)0xFFFFFFFFFFFFFFFFull;            /* modulus LE bytes [8..16) */
  out[k++] = (fe)((o->field_extension << 16) | (o->fri_folding_factor << 8) | o->fri_remainder_max_degree);
  out[k++] = (fe)o->grinding_factor;
  out[k++] = (fe)o->blowup_factor;
  out[k++] = (fe)o->num_queries;
  *nout = k;
}

/* AirPublicInputs::to_elements (lib.rs:116-160) */
int orc_pi_elements(const zkl_air_public_inputs *pi, fe *out) {
  int k = 0;
  out[k++] = (fe)pi->feature_mask;
  out[k++] = be_from_le8(pi->program_commitment);
  out[k++] = be_from_le8(pi->merkle_root);
  int nz = 0;
  for (int i = 0; i < 32; i++) nz |= pi->program_commitment[i];
  if (nz) { fe fc[2]; program_field_commitment(pi->program_commitment, fc); out[k++] = fc[0]; out[k++] = fc[1]; }
  else { out[k++] = 0; out[k++] = 0; }
  for (uint32_t i = 0; i < pi->n_main_slots; i++) out[k++] = fe_of(pi->main_slots[i]);
  out[k++] = fe_of(pi->pc_init);
  out[k++] = fe_of(pi->ram_gp_unsorted_in);
  out[k++] = fe_of(pi->ram_gp_unsorted_out);
  out[k++] = fe_of(pi->ram_gp_sorted_in);
  out[k++] = fe_of(pi->ram_gp_sorted_out);
  for (int i = 0; i < 3; i++) out[k++] = fe_of(pi->rom_s_in[i]);
  for (int i = 0; i < 3; i++) out[k++] = fe_of(pi->rom_s_out[i]);
  out[k++] = (fe)pi->vm_usage_mask;
  out[k++] = (fe)pi->ram_delta_clk_bits;
  return k;
}

static unsigned ilog2z(size_t n) { unsigned k = 0; while (((size_t)1 << k) < n) k++; return k; }

/* boundary term on the whole CE domain, column-wise form */
static void boundary_columnwise(const zk_air *air, const fe *betas, const fe *lde, size_t W, size_t n,
                                size_t N, size_t ce, fe *out) {
  size_t step_lde = N / ce;
  /* collect asserted columns */
  int ucols[256]; int nu = 0;
  for (size_t a = 0; a < air->n_assert; a++) {
    int cidx = (int)air->as_col[a], found = 0;
    for (int u = 0; u < nu; u++) if (ucols[u] == cidx) { found = 1; break; }
    if (!found) ucols[nu++] = cidx;
  }
  fe *vec = (fe *)malloc(n * sizeof(fe));
  fe *mv = (fe *)malloc(ce * sizeof(fe));
  fe *acc = (fe *)calloc(ce, sizeof(fe));
  fe *wv = (fe *)calloc(n, sizeof(fe));
  fe *rev = (fe *)malloc(n * sizeof(fe));
  for (int u = 0; u < nu; u++) {
    memset(vec, 0, n * sizeof(fe));
    for (size_t a = 0; a < air->n_assert; a++)
      if ((int)air->as_col[a] == ucols[u]) {
        vec[air->as_step[a]] = betas[a];
        wv[air->as_step[a]] = fe_add(wv[air->as_step[a]], fe_mul(betas[a], air->as_val[a]));
      }
    ntt_inplace(vec, n, 0);
    for (size_t k = 0; k < n; k++) rev[k] = vec[n - 1 - k];
    coset_evaluate(rev, n, mv, ce, 3);
    for (size_t i = 0; i < ce; i++)
      acc[i] = fe_add(acc[i], fe_mul(lde[(i * step_lde) * W + ucols[u]], mv[i]));
  }
  ntt_inplace(wv, n, 0);
  for (size_t k = 0; k < n; k++) rev[k] = wv[n - 1 - k];
  coset_evaluate(rev, n, mv, ce, 3);
  /* 1/(x^n - 1): x^n = 3^n * w_ce^(i n), takes ce/n distinct values */
  size_t blow = ce / n;
  fe wb = fe_root_of_unity(ilog2z(blow));
  fe o_n = fe_exp(3, (fe)n);
  fe zinv[64];
  fe p = 1;
  for (size_t j = 0; j < blow; j++) { zinv[j] = fe_inv(fe_sub(fe_mul(o_n, p), 1)); p = fe_mul(p, wb); }
  for (size_t i = 0; i < ce; i++) out[i] = fe_mul(fe_sub(acc[i], mv[i]), zinv[i % blow]);
  free(vec); free(mv); free(acc); free(wv); free(rev);
}

/* Winterfell's literal per-group evaluation: groups keyed by (stride=0, first_step) */
static void boundary_groups(const zk_air *air, const fe *betas, const fe *lde, size_t W, size_t n,
                            size_t N, size_t ce, fe *out) {
  size_t step_lde = N / ce;
  fe g = fe_root_of_unity(ilog2z(n));
  fe wce = fe_root_of_unity(ilog2z(ce));
  fe *xs = (fe *)malloc(ce * sizeof(fe));
  fe *den = (fe *)malloc(ce * sizeof(fe));
  fe *inv = (fe *)malloc(ce * sizeof(fe));
  fe *scr = (fe *)malloc(ce * sizeof(fe));
  fe x = 3;
  for (size_t i = 0; i < ce; i++) { xs[i] = x; out[i] = 0; x = fe_mul(x, wce); }
  for (size_t a = 0; a < air->n_assert;) {
    size_t b = a;
    while (b < air->n_assert && air->as_step[b] == air->as_step[a]) b++;
    fe gs = fe_exp(g, (fe)air->as_step[a]);
    for (size_t i = 0; i < ce; i++) den[i] = fe_sub(xs[i], gs);
    fe_batch_inv(inv, den, ce, scr);
    for (size_t i = 0; i < ce; i++) {
      const fe *row = lde + (i * step_lde) * W;
      fe num = 0;
      for (size_t k = a; k < b; k++)
        num = fe_add(num, fe_mul(fe_sub(row[air->as_col[k]], air->as_val[k]), betas[k]));
      out[i] = fe_add(out[i], fe_mul(num, inv[i]));
    }
    a = b;
  }
  free(xs); free(den); free(inv); free(scr);
}

typedef struct {
  double t_lde, t_commit, t_eval, t_comp, t_deep, t_fri, t_grind, t_query;
} orc_times;
static orc_times g_times;
#include <time.h>
static double now_ms(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec * 1e3 + t.tv_nsec / 1e6; }
void orc_last_times(double *out) {
  out[0] = g_times.t_lde; out[1] = g_times.t_commit; out[2] = g_times.t_eval; out[3] = g_times.t_comp;
  out[4] = g_times.t_deep; out[5] = g_times.t_fri; out[6] = g_times.t_grind; out[7] = g_times.t_query;
}

int orc_prove_segment(const zkl_f128 *trace, uint32_t W, uint32_t n, const zkl_air_public_inputs *pi,
                      const zkl_proof_options *o, uint8_t **proof_out, size_t *len_out, int boundary_mode) {
  double t0 = now_ms();
  if (o->field_extension != 1 || o->fri_folding_factor != 2 || o->batching_constraints != 0 ||
      o->batching_deep != 0) { g_err = "unsupported proof options"; return ZKL_E_INVALID; }
  if (n < 32 || (n & (n - 1))) { g_err = "trace length must be a power of two >= 32"; return ZKL_E_INVALID; }
  zk_air air;
  int rc = air_new(&air, pi, W, n);
  if (rc) { g_err = "AIR construction failed (unsupported features or assertion count mismatch)"; air_free(&air); return ZKL_E_INVALID; }
  const size_t N = (size_t)n * o->blowup_factor, ce = (size_t)n * air.ce_blowup;
  const int C = air.n_comp_cols;
  if (o->blowup_factor < (uint32_t)air.ce_blowup) { g_err = "blowup below CE blowup"; air_free(&air); return ZKL_E_INVALID; }
  const fe offset = 3;
  const fe g = fe_root_of_unity(ilog2z(n));
  const fe wN = fe_root_of_unity(ilog2z(N));

  /* ---- coin seed: Context::to_elements || AirPublicInputs::to_elements ---- */
  fe seed_el[64];
  int ns;
  orc_context_elements(W, n, o, seed_el, &ns);
  ns += orc_pi_elements(pi, seed_el + ns);
  coin_t coin = {ph_hash_elements(seed_el, (size_t)ns), 0};

  /* ---- 1. trace LDE (DefaultTraceLde::new) ---- */
  fe *coef = (fe *)malloc((size_t)W * n * sizeof(fe));
  fe *lde = (fe *)malloc(N * W * sizeof(fe)); /* row-major */
  fe *col = (fe *)malloc(N * sizeof(fe));
#pragma omp parallel num_threads(g_orc_threads)
  {
    fe *colt = (fe *)malloc(N * sizeof(fe));
#pragma omp for schedule(dynamic, 1)
    for (uint32_t c = 0; c < W; c++) {
      fe *cc = coef + (size_t)c * n;
      for (size_t r = 0; r < n; r++) cc[r] = fe_of(trace[(size_t)c * n + r]);
      ntt_inplace(cc, n, 1);
      coset_evaluate(cc, n, colt, N, offset);
      for (size_t r = 0; r < N; r++) lde[r * W + c] = colt[r];
    }
    free(colt);
  }
  double t1 = now_ms();
  fe *leaves = (fe *)malloc(N * sizeof(fe));
  hash_rows(lde, N, W, o->num_partitions, o->hash_rate, leaves);
  fe *ttree = merkle_build(leaves, N);
  coin_reseed(&coin, ttree[1]);
  double t2 = now_ms();

  /* ---- 2. constraint evaluation ---- */
  fe *alphas = (fe *)malloc((size_t)air.n_tc * sizeof(fe));
  fe *betas = (fe *)malloc(air.n_assert * sizeof(fe));
  coin_draw_many(&coin, alphas, (size_t)air.n_tc);
  coin_draw_many(&coin, betas, air.n_assert);
  fe *cev = (fe *)malloc(ce * sizeof(fe));
  if (boundary_mode == 1) boundary_groups(&air, betas, lde, W, n, N, ce, cev);
  else boundary_columnwise(&air, betas, lde, W, n, N, ce, cev);
  {
    size_t step = N / ce;
    fe wce = fe_root_of_unity(ilog2z(ce));
    fe gl = fe_exp(g, (fe)(n - 1));
    size_t blow = ce / n;
    fe wb = fe_root_of_unity(ilog2z(blow)), o_n = fe_exp(offset, (fe)n), p = 1, zi[64];
    for (size_t j = 0; j < blow; j++) { zi[j] = fe_inv(fe_sub(fe_mul(o_n, p), 1)); p = fe_mul(p, wb); }
    /* periodic cycle-32 values repeat every 256 CE points: cache them */
    size_t per_period = ce / (n / 32);
    fe *pert = (fe *)malloc(per_period * 32 * sizeof(fe));
    for (size_t i = 0; i < per_period; i++) air_periodic_at(&air, fe_mul(offset, fe_exp(wce, (fe)i)), pert + i * 32);
#pragma omp parallel for num_threads(g_orc_threads) schedule(dynamic, 256)
    for (size_t i = 0; i < ce; i++) {
      fe x = fe_mul(offset, fe_exp(wce, (fe)i));
      fe per[32], tc[MAX_TC];
      memcpy(per, pert + (i % per_period) * 32, 31 * sizeof(fe));
      /* p_last = L_{n-1}(x) */
      fe xn = fe_exp(x, (fe)n);
      per[31] = fe_mul(fe_mul(gl, fe_sub(xn, 1)), fe_inv(fe_mul((fe)n, fe_sub(x, gl))));
      const fe *cur = lde + (i * step) * W;
      const fe *nxt = lde + ((i * step + o->blowup_factor) % N) * W;
      air_eval_transition(&air, cur, nxt, per, tc);
      fe acc = 0;
      for (int k = 0; k < air.n_tc; k++) acc = fe_add(acc, fe_mul(alphas[k], tc[k]));
      /* divide by Z(x) = (x^n - 1)/(x - g^{n-1}) */
      acc = fe_mul(fe_mul(acc, fe_sub(x, gl)), zi[i % blow]);
      cev[i] = fe_add(cev[i], acc);
    }
    free(pert);
  }
  double t3 = now_ms();

  /* ---- 3. composition polynomial + commitment ---- */
  coset_interpolate(cev, ce, offset);
  for (size_t k = (size_t)C * n; k < ce; k++)
    if (cev[k] != 0) {
      g_err = "constraint composition polynomial degree too large: trace does not satisfy the AIR";
      free(coef); free(lde); free(col); free(leaves); free(ttree); free(alphas); free(betas); free(cev);
      air_free(&air);
      return ZKL_E_INVALID;
    }
  fe *clde = (fe *)malloc(N * (size_t)C * sizeof(fe)); /* row-major N x C */
  for (int j = 0; j < C; j++) {
    coset_evaluate(cev + (size_t)j * n, n, col, N, offset);
    for (size_t r = 0; r < N; r++) clde[r * C + j] = col[r];
  }
  fe *cleaves = (fe *)malloc(N * sizeof(fe));
  hash_rows(clde, N, (size_t)C, o->num_partitions, o->hash_rate, cleaves);
  fe *ctree = merkle_build(cleaves, N);
  coin_reseed(&coin, ctree[1]);
  double t4 = now_ms();

  /* ---- 4. OOD ---- */
  fe z = coin_draw(&coin), zg = fe_mul(z, g);
  fe *ood = (fe *)malloc(2 * ((size_t)W + C) * sizeof(fe)); /* t(z) | H(z) | t(zg) | H(zg) */
  for (uint32_t c = 0; c < W; c++) {
    ood[c] = poly_eval(coef + (size_t)c * n, n, z);
    ood[W + C + c] = poly_eval(coef + (size_t)c * n, n, zg);
  }
  for (int j = 0; j < C; j++) {
    ood[W + j] = poly_eval(cev + (size_t)j * n, n, z);
    ood[2 * W + C + j] = poly_eval(cev + (size_t)j * n, n, zg);
  }
  coin_reseed(&coin, ph_hash_elements(ood, 2 * ((size_t)W + C)));
  fe *gam = (fe *)malloc(((size_t)W + C) * sizeof(fe));
  for (size_t k = 0; k < (size_t)W + C; k++) gam[k] = coin_draw(&coin);

  /* ---- 5. DEEP composition over the LDE domain ---- */
  fe sz = 0, szg = 0;
  for (uint32_t c = 0; c < W; c++) { sz = fe_add(sz, fe_mul(gam[c], ood[c])); szg = fe_add(szg, fe_mul(gam[c], ood[W + C + c])); }
  for (int j = 0; j < C; j++) { sz = fe_add(sz, fe_mul(gam[W + j], ood[W + j])); szg = fe_add(szg, fe_mul(gam[W + j], ood[2 * W + C + j])); }
  fe *deep = (fe *)malloc(N * sizeof(fe));
  {
    fe *d1 = (fe *)malloc(N * sizeof(fe)), *d2 = (fe *)malloc(N * sizeof(fe));
    fe *i1 = (fe *)malloc(N * sizeof(fe)), *i2 = (fe *)malloc(N * sizeof(fe)), *scr = (fe *)malloc(N * sizeof(fe));
    fe x = offset;
    for (size_t i = 0; i < N; i++) { d1[i] = fe_sub(x, z); d2[i] = fe_sub(x, zg); x = fe_mul(x, wN); }
    fe_batch_inv(i1, d1, N, scr);
    fe_batch_inv(i2, d2, N, scr);
#pragma omp parallel for num_threads(g_orc_threads) schedule(static)
    for (size_t i = 0; i < N; i++) {
      fe s = 0;
      const fe *row = lde + i * W;
      for (uint32_t c = 0; c < W; c++) s = fe_add(s, fe_mul(gam[c], row[c]));
      const fe *crow = clde + i * C;
      for (int j = 0; j < C; j++) s = fe_add(s, fe_mul(gam[W + j], crow[j]));
      deep[i] = fe_add(fe_mul(fe_sub(s, sz), i1[i]), fe_mul(fe_sub(s, szg), i2[i]));
    }
    free(d1); free(d2); free(i1); free(i2); free(scr);
  }
  double t5 = now_ms();

  /* ---- 6. FRI ---- */
  size_t rem_max = (size_t)(o->fri_remainder_max_degree + 1) * o->blowup_factor;
  int nlayers = 0;
  for (size_t d = N; d > rem_max; d /= 2) nlayers++;
  fe **ltrees = (fe **)calloc((size_t)nlayers + 1, sizeof(fe *));
  fe **lvals = (fe **)calloc((size_t)nlayers + 1, sizeof(fe *));
  fe fri_roots[64];
  fe *ev = deep;
  size_t Nd = N;
  for (int d = 0; d < nlayers; d++) {
    size_t h = Nd / 2;
    fe *lv = (fe *)malloc(Nd * sizeof(fe)); /* transposed [e_i, e_{i+h}] */
    fe *lf = (fe *)malloc(h * sizeof(fe));
    for (size_t i = 0; i < h; i++) { lv[2 * i] = ev[i]; lv[2 * i + 1] = ev[i + h]; }
#pragma omp parallel for num_threads(g_orc_threads) schedule(static)
    for (size_t i = 0; i < h; i++) lf[i] = ph_hash_elements(lv + 2 * i, 2);
    ltrees[d] = merkle_build(lf, h);
    free(lf);
    lvals[d] = lv;
    fri_roots[d] = ltrees[d][1];
    coin_reseed(&coin, fri_roots[d]);
    fe alpha = coin_draw(&coin);
    /* fold with the constant domain offset (agg/trace.rs:764-800) */
    fe gd = fe_root_of_unity(ilog2z(Nd));
    fe *nx = (fe *)malloc(h * sizeof(fe));
    fe xe = offset, inv2 = fe_inv(2);
    fe *den = (fe *)malloc(h * sizeof(fe)), *inv = (fe *)malloc(h * sizeof(fe)), *scr = (fe *)malloc(h * sizeof(fe));
    for (size_t i = 0; i < h; i++) { den[i] = xe; xe = fe_mul(xe, gd); }
    fe_batch_inv(inv, den, h, scr);
    for (size_t i = 0; i < h; i++) {
      fe v0 = ev[i], v1 = ev[i + h];
      /* (v0+v1)/2 + alpha (v0-v1)/(2 x0) == (v1(a-x0) - v0(a-x1))/(x1-x0), x1 = -x0 */
      nx[i] = fe_mul(fe_add(fe_add(v0, v1), fe_mul(alpha, fe_mul(fe_sub(v0, v1), inv[i]))), inv2);
    }
    free(den); free(inv); free(scr);
    if (ev != deep) free(ev);
    ev = nx;
    Nd = h;
  }
  /* remainder: interpolate with offset GENERATOR, keep rem_deg+1 coefficients, reversed */
  coset_interpolate(ev, Nd, offset);
  size_t rlen = o->fri_remainder_max_degree + 1;
  fe rem[16];
  for (size_t k = 0; k < rlen; k++) rem[k] = ev[rlen - 1 - k];
  fe rem_commit = ph_hash_elements(rem, rlen);
  coin_reseed(&coin, rem_commit);
  if (ev != deep) free(ev);
  double t6 = now_ms();

  /* ---- 7. grinding: smallest nonce >= 1 (no `concurrent` feature) ---- */
  uint64_t nonce = 0;
  if (o->grinding_factor == 0) nonce = 1; /* still the first candidate */
  {
    uint64_t B = 64;
    for (uint64_t base = 1; nonce == 0; base += B, B = B < 4096 ? 2 * B : B) {
      uint64_t best = UINT64_MAX;
#pragma omp parallel for num_threads(g_orc_threads) reduction(min : best) schedule(static)
      for (uint64_t k = base; k < base + B; k++) {
        fe h = ph_merge_with_int(coin.seed, k);
        uint64_t lo = (uint64_t)h;
        unsigned tz = lo ? (unsigned)__builtin_ctzll(lo) : 64;
        if (tz >= o->grinding_factor && k < best) best = k;
      }
      if (best != UINT64_MAX) nonce = best;
    }
  }
  double t7 = now_ms();

  /* ---- 8. query positions ---- */
  coin.seed = ph_merge_with_int(coin.seed, nonce);
  coin.counter = 0;
  size_t q = o->num_queries;
  size_t *pos = (size_t *)malloc(q * sizeof(size_t));
  for (size_t k = 0; k < q; k++) pos[k] = (size_t)((uint64_t)coin_draw(&coin) & (N - 1));
  qsort(pos, q, sizeof(size_t), cmp_sz);
  size_t nq = 0;
  for (size_t k = 0; k < q; k++) if (nq == 0 || pos[nq - 1] != pos[k]) pos[nq++] = pos[k];

  /* ---- 9. Proof::to_bytes ---- */
  bbuf out = {0};
  /* Context */
  bb_u8(&out, (uint8_t)W); bb_u8(&out, 0); bb_u8(&out, 0); bb_u8(&out, (uint8_t)ilog2z(n));
  bb_u8(&out, 0); bb_u8(&out, 0); /* trace_meta len u16 = 0 */
  bb_u8(&out, 16);
  bb_fe(&out, FE_P);
  bb_u8(&out, (uint8_t)o->num_queries); bb_u8(&out, (uint8_t)o->blowup_factor);
  bb_u8(&out, (uint8_t)o->grinding_factor); bb_u8(&out, (uint8_t)o->field_extension);
  bb_u8(&out, (uint8_t)o->fri_folding_factor); bb_u8(&out, (uint8_t)o->fri_remainder_max_degree);
  bb_u8(&out, (uint8_t)o->batching_constraints); bb_u8(&out, (uint8_t)o->batching_deep);
  bb_u8(&out, (uint8_t)o->num_partitions); bb_u8(&out, (uint8_t)o->hash_rate);
  bb_u8(&out, (uint8_t)nq);
  /* Commitments */
  {
    bbuf cm = {0};
    bb_digest(&cm, ttree[1]); bb_digest(&cm, ctree[1]);
    for (int d = 0; d < nlayers; d++) bb_digest(&cm, fri_roots[d]);
    bb_digest(&cm, rem_commit);
    bb_vec(&out, &cm); free(cm.p);
  }
  /* trace queries: Vec<Queries> with one segment */
  bb_usize(&out, 1);
  {
    bbuf v = {0}, pth = {0};
    for (size_t k = 0; k < nq; k++) for (uint32_t c = 0; c < W; c++) bb_fe(&v, lde[pos[k] * W + c]);
    merkle_batch_proof(ttree, N, pos, nq, &pth);
    bb_vec(&out, &v); bb_vec(&out, &pth); free(v.p); free(pth.p);
  }
  {
    bbuf v = {0}, pth = {0};
    for (size_t k = 0; k < nq; k++) for (int j = 0; j < C; j++) bb_fe(&v, clde[pos[k] * C + j]);
    merkle_batch_proof(ctree, N, pos, nq, &pth);
    bb_vec(&out, &v); bb_vec(&out, &pth); free(v.p); free(pth.p);
  }
  /* OOD frame */
  {
    bbuf ts = {0}, es = {0};
    for (uint32_t c = 0; c < W; c++) bb_fe(&ts, ood[c]);
    for (uint32_t c = 0; c < W; c++) bb_fe(&ts, ood[W + C + c]);
    for (int j = 0; j < C; j++) bb_fe(&es, ood[W + j]);
    for (int j = 0; j < C; j++) bb_fe(&es, ood[2 * W + C + j]);
    bb_vec(&out, &ts); bb_vec(&out, &es); free(ts.p); free(es.p);
  }
  /* FRI proof */
  double t8a = now_ms();
  bb_usize(&out, (uint64_t)nlayers);
  {
    size_t *fp = (size_t *)malloc(nq * sizeof(size_t)), nf = nq;
    memcpy(fp, pos, nq * sizeof(size_t));
    size_t dsz = N;
    for (int d = 0; d < nlayers; d++) {
      size_t h = dsz / 2;
      size_t m = 0;
      for (size_t k = 0; k < nf; k++) {
        size_t pk = fp[k] % h;
        int dup = 0;
        for (size_t j = 0; j < m; j++) if (fp[j] == pk) { dup = 1; break; }
        if (!dup) fp[m++] = pk;
      }
      nf = m;
      bbuf v = {0}, pth = {0};
      for (size_t k = 0; k < nf; k++) { bb_fe(&v, lvals[d][2 * fp[k]]); bb_fe(&v, lvals[d][2 * fp[k] + 1]); }
      merkle_batch_proof(ltrees[d], h, fp, nf, &pth);
      bb_vec(&out, &v); bb_vec(&out, &pth); free(v.p); free(pth.p);
      dsz = h;
    }
    free(fp);
    bbuf rv = {0};
    for (size_t k = 0; k < rlen; k++) bb_fe(&rv, rem[k]);
    bb_vec(&out, &rv); free(rv.p);
    bb_u8(&out, 0); /* num_partitions = 1, stored as log2 */
  }
  bb_u64(&out, nonce);
  double t8 = now_ms();
  (void)t8a;

  g_times.t_lde = t1 - t0; g_times.t_commit = t2 - t1; g_times.t_eval = t3 - t2; g_times.t_comp = t4 - t3;
  g_times.t_deep = t5 - t4; g_times.t_fri = t6 - t5; g_times.t_grind = t7 - t6; g_times.t_query = t8 - t7;

  for (int d = 0; d < nlayers; d++) { free(ltrees[d]); free(lvals[d]); }
  free(ltrees); free(lvals); free(pos); free(deep); free(gam); free(ood); free(clde); free(cleaves);
  free(ctree); free(cev); free(alphas); free(betas); free(coef); free(lde); free(col); free(leaves);
  free(ttree);
  air_free(&air);
  *proof_out = out.p;
  *len_out = out.len;
  return ZKL_OK;
}
