/* ORACLE — test infrastructure only.  Byte-level entry points for tests/ (ctypes). */
#include <string.h>
#include "oracle.h"

static fe rd(const uint8_t *b) { return fe_from_bytes_raw(b); }
static void wr(fe v, uint8_t *b) { fe_to_bytes(v, b); }

void orc_api_fe_add(const uint8_t *a, const uint8_t *b, uint8_t *o) { wr(fe_add(rd(a), rd(b)), o); }
void orc_api_fe_sub(const uint8_t *a, const uint8_t *b, uint8_t *o) { wr(fe_sub(rd(a), rd(b)), o); }
void orc_api_fe_mul(const uint8_t *a, const uint8_t *b, uint8_t *o) { wr(fe_mul(rd(a), rd(b)), o); }
void orc_api_fe_inv(const uint8_t *a, uint8_t *o) { wr(fe_inv(rd(a)), o); }
void orc_api_root_of_unity(unsigned k, uint8_t *o) { wr(fe_root_of_unity(k), o); }
void orc_api_suite(const uint8_t *sid, int rounds, uint8_t *dom, uint8_t *mds, uint8_t *rc) {
  pos_suite s;
  pos_suite_derive(sid, rounds, &s);
  wr(s.dom[0], dom); wr(s.dom[1], dom + 16);
  for (int i = 0; i < 144; i++) wr(s.mds[i / 12][i % 12], mds + 16 * i);
  for (int r = 0; r < rounds && r < POS_ROUNDS; r++)
    for (int l = 0; l < 12; l++) wr(s.rc[r][l], rc + 16 * (r * 12 + l));
}
void orc_api_permute(const uint8_t *st_in, uint8_t *st_out) {
  fe st[12];
  for (int i = 0; i < 12; i++) st[i] = rd(st_in + 16 * i);
  pos_permute(pos_hasher_suite(), st);
  for (int i = 0; i < 12; i++) wr(st[i], st_out + 16 * i);
}
void orc_api_hash_elements(const uint8_t *e, size_t n, uint8_t *o) {
  fe *v = (fe *)malloc((n ? n : 1) * sizeof(fe));
  for (size_t i = 0; i < n; i++) v[i] = rd(e + 16 * i);
  wr(ph_hash_elements(v, n), o);
  free(v);
}
void orc_api_merge(const uint8_t *a, const uint8_t *b, uint8_t *o) { wr(ph_merge(rd(a), rd(b)), o); }
void orc_api_merge_many(const uint8_t *d, size_t n, uint8_t *o) {
  fe *v = (fe *)malloc((n ? n : 1) * sizeof(fe));
  for (size_t i = 0; i < n; i++) v[i] = rd(d + 16 * i);
  wr(ph_merge_many(v, n), o);
  free(v);
}
void orc_api_merge_with_int(const uint8_t *s, uint64_t x, uint8_t *o) { wr(ph_merge_with_int(rd(s), x), o); }
void orc_api_hash_bytes(const uint8_t *d, size_t n, uint8_t *o) { wr(ph_hash_bytes(d, n), o); }
void orc_api_program_field_commitment(const uint8_t *b32, uint8_t *o) {
  fe r[2];
  program_field_commitment(b32, r);
  wr(r[0], o); wr(r[1], o + 16);
}
int orc_api_air_info(const zkl_air_public_inputs *pi, uint32_t w, size_t n, int *n_tc, size_t *n_assert,
                     int *ce_blowup, int *n_comp) {
  zk_air a;
  int rc = air_new(&a, pi, w, n);
  *n_tc = a.n_tc; *n_assert = a.n_assert; *ce_blowup = a.ce_blowup; *n_comp = a.n_comp_cols;
  air_free(&a);
  return rc;
}
/* evaluate transition constraints on trace rows (row, row+1) of a column-major trace: all
 * must vanish where the AIR's periodic selectors are taken at the trace-domain point */
int orc_api_check_trace(const zkl_f128 *t, uint32_t w, size_t n, const zkl_air_public_inputs *pi,
                        size_t *bad_row, int *bad_idx) {
  zk_air a;
  int rc = air_new(&a, pi, w, n);
  if (rc) { air_free(&a); return rc; }
  fe *cur = (fe *)malloc(w * sizeof(fe)), *nx = (fe *)malloc(w * sizeof(fe)), res[MAX_TC], per[32];
  int bad = 0;
  for (size_t r = 0; r + 1 < n && !bad; r++) {
    for (uint32_t c = 0; c < w; c++) {
      cur[c] = ((fe)t[(size_t)c * n + r].hi << 64) | t[(size_t)c * n + r].lo;
      nx[c] = ((fe)t[(size_t)c * n + r + 1].hi << 64) | t[(size_t)c * n + r + 1].lo;
    }
    size_t pos = r % 32;
    for (int k = 0; k < 31; k++) per[k] = 0;
    per[0] = pos == 0;
    if (pos >= 1 && pos <= 27) per[pos] = 1;
    per[28] = pos == 28;
    per[29] = pos >= 29;
    per[30] = pos == 31;
    per[31] = r == n - 1;
    air_eval_transition(&a, cur, nx, per, res);
    for (int k = 0; k < a.n_tc; k++)
      if (res[k] != 0) { *bad_row = r; *bad_idx = k; bad = 1; break; }
  }
  /* assertions */
  for (size_t k = 0; k < a.n_assert && !bad; k++) {
    size_t c = a.as_col[k], r = a.as_step[k];
    fe v = ((fe)t[c * n + r].hi << 64) | t[c * n + r].lo;
    if (v != a.as_val[k]) { *bad_row = r; *bad_idx = -1 - (int)k; bad = 1; }
  }
  free(cur); free(nx);
  air_free(&a);
  return bad ? 1 : 0;
}
/* digest of one row (ncols elements) partitioned into chunks of psize under the current rule */
void orc_api_row_digest(const uint8_t *row, size_t ncols, size_t psize, uint8_t *o) {
  fe *v = (fe *)malloc((ncols ? ncols : 1) * sizeof(fe));
  for (size_t i = 0; i < ncols; i++) v[i] = rd(row + 16 * i);
  wr(orc_row_digest(v, ncols, psize), o);
  free(v);
}
