/*
 * ORACLE — test infrastructure only.
 *
 * ZkLispAir restated for VM/ROM segments:
 *   vm/layout.rs:183-374        Columns::for_config
 *   vm/air/mod.rs:114-318       ZkLispAir::new (features, degrees, #assertions)
 *   vm/air/mod.rs:324-378       evaluate_transition (module order Poseidon, Ctrl, ALU, RAM, Merkle, ROM)
 *   vm/air/ctrl.rs:28-391       VmCtrlAir
 *   vm/air/alu.rs:29-355        VmAluAir
 *   vm/air/rom.rs:26-148        RomAir
 *   vm/air/mixers.rs:19-48      degree mixers
 *   vm/air/schedule.rs:28-141   ScheduleAir assertions
 *   vm/air/mod.rs:380-504       get_assertions + dedup by (column, step)
 *   vm/air/mod.rs:520-592       periodic column polynomials
 * Poseidon / RAM / Merkle blocks are outside this restatement: air_new rejects traces
 * whose effective feature mask enables them (the {vm, rom} layout of width 204 is the
 * published segment shape).
 */
#include <stdio.h>
#include <string.h>
#include "oracle.h"

#define NR 8
#define STEPS 32

enum { U_ASSERT = 0, U_ASSERT_BIT, U_ASSERT_RANGE, U_DIVMOD, U_MULWIDE, U_DIV128, U_EQ, U_SPONGE, U_RAM_DCLK };

void cols_for_config(int vm, int ram, int sponge, int merkle, int rom, zk_cols *c) {
  (void)vm; (void)sponge;
  c->lanes_start = 0;
  int cur = 12;
  c->g_map = cur; c->g_final = cur + 1; c->g_r_start = cur + 2;
  cur = c->g_r_start + POS_ROUNDS;
  c->mask = cur++;
  c->r_start = cur; cur += NR;
  for (int k = 0; k < 17; k++) c->op[k] = cur + k;
  cur += 17;
  c->sel_dst0 = cur; c->sel_a = cur + NR; c->sel_b = cur + 2 * NR; c->sel_c = cur + 3 * NR;
  c->sel_dst1 = cur + 4 * NR;
  cur += 5 * NR;
  c->sel_s_bits = cur; c->sel_s_active = cur + 30;
  cur += 40;
  c->imm = cur; c->eq_inv = cur + 1;
  cur += 2;
  c->ram_sorted = cur; c->ram_s_addr = cur + 1; c->ram_s_clk = cur + 2; c->ram_s_val = cur + 3;
  c->ram_s_is_write = cur + 4; c->ram_s_last_write = cur + 5; c->ram_gp_unsorted = cur + 6; c->ram_gp_sorted = cur + 7;
  if (ram) cur += 8;
  c->merkle_g = cur; c->merkle_dir = cur + 1; c->merkle_sib = cur + 2; c->merkle_acc = cur + 3;
  c->merkle_first = cur + 4; c->merkle_last = cur + 5; c->merkle_leaf = cur + 6;
  if (merkle) cur += 7;
  c->pi_prog = cur++;
  c->pc = cur++;
  c->rom_op_start = cur;
  if (rom) cur += 17;
  c->pose_active = cur++;
  c->gadget_b = cur;
  cur += 32;
  c->rom_s = cur;
  if (rom) cur += 3;
  c->width = rom ? cur : c->pc + 1;
}

static fe rom_w(uint32_t seed, fe out[59]) {
  fe acc = fe_exp(3, seed);
  fe cur = fe_mul(acc, 3);
  for (int i = 0; i < 59; i++) { out[i] = cur; cur = fe_mul(cur, 3); }
  return 0;
}

/* periodic cycle-32 column polynomial coefficients (31 columns), shared by all AIRs */
static fe g_percoef[31][32];
static int g_percoef_init = 0;
static void periodic_init(void) {
  if (g_percoef_init) return;
  for (int col = 0; col < 31; col++) {
    fe v[32];
    for (int pos = 0; pos < 32; pos++) {
      int one = 0;
      if (col == 0) one = (pos == 0);
      else if (col <= POS_ROUNDS) one = (pos == col);
      else if (col == 28) one = (pos == 28);
      else if (col == 29) one = (pos != 0 && pos != 28 && !(pos >= 1 && pos <= 27));
      else one = (pos == 31);
      v[pos] = one ? 1 : 0;
    }
    ntt_inplace(v, 32, 1);
    memcpy(g_percoef[col], v, sizeof v);
  }
  g_percoef_init = 1;
}

void air_periodic_at(const zk_air *air, fe x, fe out[32]) {
  size_t n = air->trace_len;
  fe y = fe_exp(x, (fe)(n / STEPS));
  for (int c = 0; c < 31; c++) out[c] = poly_eval(g_percoef[c], 32, y);
  /* p_last = L_{n-1}(x) = g^{n-1} (x^n - 1) / (n (x - g^{n-1})) */
  unsigned logn = 0; while (((size_t)1 << logn) < n) logn++;
  fe g = fe_root_of_unity(logn);
  fe gl = fe_exp(g, (fe)(n - 1));
  fe num = fe_mul(gl, fe_sub(fe_exp(x, (fe)n), 1));
  fe den = fe_mul((fe)n, fe_sub(x, gl));
  out[31] = fe_mul(num, fe_inv(den));
}

static int cmp_assert(const void *a, const void *b) {
  const uint64_t *x = (const uint64_t *)a, *y = (const uint64_t *)b;
  return (x[0] > y[0]) - (x[0] < y[0]);
}

int air_new(zk_air *air, const zkl_air_public_inputs *pi, uint32_t width, size_t n) {
  memset(air, 0, sizeof *air);
  periodic_init();
  uint64_t eff = pi->segment_feature_mask ? pi->segment_feature_mask : pi->feature_mask;
  air->feat_poseidon = !!(eff & FM_POSEIDON);
  air->feat_vm = !!(eff & FM_VM);
  air->feat_vm_expect = !!(eff & FM_VM_EXPECT);
  air->feat_sponge = !!(eff & FM_SPONGE);
  air->feat_merkle = !!(eff & FM_MERKLE);
  air->feat_ram = !!(eff & FM_RAM);
  int pid_nz = 0, com_nz = 0;
  for (int i = 0; i < 32; i++) { pid_nz |= pi->program_id[i]; com_nz |= pi->program_commitment[i]; }
  air->rom_enabled = pid_nz != 0;
  air->commit_nonzero = com_nz != 0;
  air->vm_usage_mask = pi->vm_usage_mask;
  air->ram_delta_clk_bits = pi->ram_delta_clk_bits;
  air->trace_len = n;
  zk_cols base;
  cols_for_config(1, 1, 1, 1, 1, &base);
  if ((int)width < base.width)
    cols_for_config(air->feat_vm, air->feat_ram, air->feat_sponge, air->feat_merkle, air->rom_enabled, &air->cols);
  else
    cols_for_config(1, 1, 1, 1, air->rom_enabled, &air->cols);
  if (air->cols.width != (int)width) return -2;

  pos_suite ps;
  pos_suite_derive(pi->program_id, POS_ROUNDS, &ps);
  air->dom[0] = ps.dom[0];
  air->dom[1] = ps.dom[1];
  memcpy(air->pose_mds, ps.mds, sizeof air->pose_mds);
  memcpy(air->pose_rc, ps.rc, sizeof air->pose_rc);
  rom_constants(pi->program_id, air->rom_rc, air->rom_mds);
  rom_w(17, air->rom_w0);
  rom_w(1037, air->rom_w1);
  if (pid_nz) program_field_commitment(pi->program_id, air->program_fe);

  air->merkle_root = be_from_le8(pi->merkle_root);
  /* degrees in module order (mod.rs:217-238); DEG(base, has the 32-cycle) */
  int nd = 0;
#define DEG(b, cyc) do { air->deg_base[nd] = (b); air->deg_cyc[nd] = (cyc); nd++; } while (0)
  uint32_t m = pi->vm_usage_mask;
  if (air->feat_poseidon) { /* PoseidonAir::push_degrees (poseidon.rs:26-62) */
    for (int i = 0; i < POS_ROUNDS * 12; i++) DEG(4, 1);
    for (int i = 0; i < 12; i++) DEG(1, 1);
    air->pose_bind = air->feat_vm && air->feat_sponge && (m & (1u << U_SPONGE));
    if (air->pose_bind) {
      static const int lane_bases[10] = {6, 6, 3, 3, 3, 3, 3, 3, 3, 3};
      for (int i = 0; i < 10; i++) DEG(lane_bases[i], 1);
    }
  }
  if (air->feat_vm) {
    for (int i = 0; i < 5 * NR; i++) DEG(2, 1);
    for (int i = 0; i < 5; i++) DEG(1, 1);
    for (int i = 0; i < NR; i++) DEG(2, 1);
    if (air->feat_sponge && (m & (1u << U_SPONGE)))
      for (int i = 0; i < 40; i++) DEG(2, 1);
    DEG(2, 1);
    for (int i = 0; i < 17; i++) DEG(2, 1);
    DEG(2, 1);
    for (int i = 0; i < 17; i++) DEG(2, 1);
    DEG(1, 1);
    DEG(1, 1);
    /* ALU */
    for (int i = 0; i < NR; i++) DEG(1, 1);
    for (int i = 0; i < NR; i++) DEG(7, 1);
    if (m & (1u << U_EQ)) for (int i = 0; i < 2; i++) DEG(5, 1);
    if (m & (1u << U_DIVMOD)) for (int i = 0; i < 2; i++) DEG(5, 1);
    if (m & (1u << U_ASSERT)) DEG(5, 1);
    if (m & (1u << U_ASSERT_BIT)) DEG(5, 1);
    if (m & (1u << U_ASSERT_RANGE)) for (int i = 0; i < 33; i++) DEG(5, 1);
    if (m & (1u << U_MULWIDE)) DEG(5, 1);
    if (m & (1u << U_DIV128)) for (int i = 0; i < 2; i++) DEG(5, 1);
  }
  if (air->feat_ram) { /* RamAir::push_degrees (ram.rs:26-79) */
    DEG(4, 1);
    DEG(2, 0); DEG(5, 0); DEG(3, 0); DEG(6, 0); DEG(5, 0);
    if (m & (1u << U_RAM_DCLK)) {
      for (int i = 0; i < 32; i++) if ((pi->ram_delta_clk_bits >> i) & 1) DEG(5, 0);
      DEG(5, 0);
    }
    DEG(2, 0);
  }
  if (air->feat_merkle) { /* MerkleAir::push_degrees (merkle.rs:26-58) */
    DEG(3, 1); DEG(3, 1); DEG(3, 1); DEG(2, 1); DEG(3, 1); DEG(3, 1); DEG(3, 1);
  }
  if (air->rom_enabled) {
    for (int i = 0; i < 81; i++) DEG(3, 1);
    for (int i = 0; i < 3; i++) DEG(1, 1);
    for (int i = 0; i < 2; i++) DEG(1, 1);
  }
  if (nd == 0) return -3; /* AIR with no constraints: not a VM segment */
  air->n_tc = nd;

#undef DEG
  /* AirContext: ce_blowup = max next_pow2(base + cycles - 1) (min 2); eval degree =
   * base (n-1) + cycles (n/32) 31; num composition columns = ceil((max_eval - (n-1)) / n) */
  int ceb = 2;
  size_t max_eval = 0;
  for (int i = 0; i < nd; i++) {
    int need = 1;
    while (need < air->deg_base[i] + air->deg_cyc[i] - 1) need <<= 1;
    if (need > ceb) ceb = need;
    size_t ev = (size_t)air->deg_base[i] * (n - 1) + (air->deg_cyc[i] ? (n / STEPS) * (STEPS - 1) : 0);
    if (ev > max_eval) max_eval = ev;
  }
  air->ce_blowup = ceb;
  air->n_comp_cols = (int)((max_eval - (n - 1) + n - 1) / n);

  /* ---- assertions ---- */
  size_t levels = n / STEPS; if (levels == 0) levels = 1;
  size_t cap = levels * 141 + 32;
  uint64_t *key = (uint64_t *)malloc(cap * 2 * sizeof(uint64_t)); /* (step<<32|col, idx) */
  fe *vals = (fe *)malloc(cap * sizeof(fe));
  size_t na = 0;
  const zk_cols *c = &air->cols;
#define PUSH(col, step, v) do { key[2 * na] = ((uint64_t)(step) << 32) | (uint32_t)(col); key[2 * na + 1] = na; vals[na] = (v); na++; } while (0)
  size_t last = n - 1;
  size_t lvls = (last + 1) / STEPS;
  for (size_t lvl = 0; lvl < lvls; lvl++) {
    size_t b = lvl * STEPS, rm = b, rf = b + 28;
    PUSH(c->lanes_start + 10, rm, air->dom[0]);
    PUSH(c->lanes_start + 11, rm, air->dom[1]);
    PUSH(c->g_map, rm, 1);
    PUSH(c->g_final, rf, 1);
    for (int j = 0; j < POS_ROUNDS; j++) PUSH(c->g_r_start + j, b + 1 + j, 1);
    PUSH(c->g_final, rm, 0);
    for (int j = 0; j < POS_ROUNDS; j++) PUSH(c->g_r_start + j, rm, 0);
    PUSH(c->g_map, rf, 0);
    for (int j = 0; j < POS_ROUNDS; j++) PUSH(c->g_r_start + j, rf, 0);
    for (int j = 0; j < POS_ROUNDS; j++) { PUSH(c->g_map, b + 1 + j, 0); PUSH(c->g_final, b + 1 + j, 0); }
    if (lvl == 0 && air->feat_vm) {
      fe pc_init = ((fe)pi->pc_init.hi << 64) | pi->pc_init.lo;
      if (pc_init == 0 && air->commit_nonzero) PUSH(c->pi_prog, rm, be_from_le8(pi->program_commitment));
      PUSH(c->pc, rm, pc_init);
    }
  }
  fe pc_init = ((fe)pi->pc_init.hi << 64) | pi->pc_init.lo;
  if (air->feat_vm) {
    if (air->feat_vm_expect) {
      size_t row = pi->vm_out_row < last ? pi->vm_out_row : last;
      int reg = pi->vm_out_reg < NR - 1 ? (int)pi->vm_out_reg : NR - 1;
      PUSH(c->r_start + reg, row, be_from_le8(pi->vm_expected_bytes));
    }
    if (pc_init == 0 && pi->n_main_slots > 0) {
      int slots = (int)pi->n_main_slots;
      if (slots > NR) { free(key); free(vals); return -4; }
      for (int j = 0; j < slots; j++) {
        fe v = ((fe)pi->main_slots[j].hi << 64) | pi->main_slots[j].lo;
        PUSH(c->r_start + NR - slots + j, 0, v);
      }
    }
  }
  if (air->commit_nonzero) {
    for (int i = 0; i < 3; i++) PUSH(c->rom_s + i, 0, ((fe)pi->rom_s_in[i].hi << 64) | pi->rom_s_in[i].lo);
    for (int i = 0; i < 3; i++) PUSH(c->rom_s + i, last, ((fe)pi->rom_s_out[i].hi << 64) | pi->rom_s_out[i].lo);
  }
  if (na == 0) PUSH(c->mask, last, 0);
#undef PUSH
  /* dedup by (column, step) keeping the first (mod.rs:448-475), then Winterfell's
   * BTreeSet order (stride, first_step, column) = (step, column) for single assertions.
   * Stable sort on the packed key; ties (duplicates) keep first-pushed order. */
  qsort(key, na, 2 * sizeof(uint64_t), cmp_assert);
  /* qsort is not stable: resolve duplicates by original index */
  air->as_col = (uint32_t *)malloc(na * sizeof(uint32_t));
  air->as_step = (uint32_t *)malloc(na * sizeof(uint32_t));
  air->as_val = (fe *)malloc(na * sizeof(fe));
  size_t out = 0;
  for (size_t i = 0; i < na;) {
    size_t j = i, best = key[2 * i + 1];
    while (j < na && key[2 * j] == key[2 * i]) { if (key[2 * j + 1] < best) best = key[2 * j + 1]; j++; }
    air->as_col[out] = (uint32_t)(key[2 * i] & 0xffffffffu);
    air->as_step[out] = (uint32_t)(key[2 * i] >> 32);
    air->as_val[out] = vals[best];
    out++;
    i = j;
  }
  air->n_assert = out;
  free(key);
  free(vals);

  /* context.num_assertions formula (mod.rs:248-290) must equal the deduped count */
  size_t expect = (2 + POS_ROUNDS) * levels + (4 * POS_ROUNDS + 2) * levels + 2 * levels;
  if (air->feat_vm) {
    expect += 1;
    if (pc_init == 0 && air->commit_nonzero) expect += 1;
    if (pi->n_main_slots > 0 && pc_init == 0) expect += pi->n_main_slots;
  }
  if (air->feat_vm && air->feat_vm_expect) expect += 1;
  if (expect == 0) expect = 1;
  if (air->rom_enabled) expect += 6;
  if (expect != air->n_assert) return -5;
  return 0;
}

void air_free(zk_air *air) {
  free(air->as_col); free(air->as_step); free(air->as_val);
  air->as_col = 0; air->as_step = 0; air->as_val = 0;
}

static const uint32_t ROM_ENC_OPS = 17;

static fe rom_encode(const zk_cols *c, const fe *row, const fe *w) {
  fe sum = 0;
  int k = 0;
  for (uint32_t i = 0; i < ROM_ENC_OPS; i++) sum = fe_add(sum, fe_mul(row[c->op[i]], w[k++]));
  const int starts[5] = {c->sel_dst0, c->sel_a, c->sel_b, c->sel_c, c->sel_dst1};
  for (int s = 0; s < 5; s++)
    for (int i = 0; i < NR; i++) sum = fe_add(sum, fe_mul(row[starts[s] + i], w[k++]));
  return sum;
}

void air_eval_transition(const zk_air *air, const fe *cur, const fe *nxt, const fe *per, fe *res) {
  const zk_cols *c = &air->cols;
  int ix = 0;
  uint32_t m = air->vm_usage_mask;
  fe p_map = per[0], p_final = per[28], p_pad = per[29], p_pad_last = per[30], p_last = per[31];
  fe s_low = fe_mul(p_last, p_map);
  fe g_carry = fe_add(p_map, fe_sub(p_pad, p_pad_last));
  for (int j = 0; j < POS_ROUNDS - 1; j++) g_carry = fe_add(g_carry, per[1 + j]);
  fe rom_on = air->commit_nonzero ? 1 : 0;

  if (air->feat_poseidon) {
    /* ---------------- PoseidonAir (poseidon.rs:65-162) ---------------- */
    const fe pa = cur[c->pose_active];
    fe s3[12], ms[12];
    for (int i = 0; i < 12; i++) s3[i] = fe_cube(cur[c->lanes_start + i]);
    for (int i = 0; i < 12; i++) {
      fe acc = 0;
      for (int k = 0; k < 12; k++) acc = fe_add(acc, fe_mul(air->pose_mds[i][k], s3[k]));
      ms[i] = acc;
    }
    for (int j = 0; j < POS_ROUNDS; j++) {
      fe g = fe_mul(pa, per[1 + j]);
      for (int i = 0; i < 12; i++)
        res[ix++] = fe_mul(g, fe_sub(nxt[c->lanes_start + i], fe_add(ms[i], air->pose_rc[j][i])));
    }
    fe g_hold = fe_sub(p_pad, p_pad_last);
    for (int i = 0; i < 12; i++) res[ix++] = fe_mul(g_hold, fe_sub(nxt[c->lanes_start + i], cur[c->lanes_start + i]));
    if (air->pose_bind) {
      fe b_sponge = cur[c->op[8]];
      for (int lane = 0; lane < 10; lane++) {
        fe b0 = cur[c->sel_s_bits + lane * 3], b1 = cur[c->sel_s_bits + lane * 3 + 1],
           b2 = cur[c->sel_s_bits + lane * 3 + 2], act = cur[c->sel_s_active + lane];
        const fe *rr = cur + c->r_start;
        fe nb0 = fe_sub(1, b0), nb1 = fe_sub(1, b1), nb2 = fe_sub(1, b2);
        fe s0 = fe_add(fe_mul(b0, rr[1]), fe_mul(nb0, rr[0]));
        fe s1 = fe_add(fe_mul(b0, rr[3]), fe_mul(nb0, rr[2]));
        fe s2 = fe_add(fe_mul(b0, rr[5]), fe_mul(nb0, rr[4]));
        fe s3v = fe_add(fe_mul(b0, rr[7]), fe_mul(nb0, rr[6]));
        fe t0 = fe_add(fe_mul(b1, s1), fe_mul(nb1, s0));
        fe t1 = fe_add(fe_mul(b1, s3v), fe_mul(nb1, s2));
        fe sel_val = fe_add(fe_mul(b2, t1), fe_mul(nb2, t0));
        fe expect = fe_mul(act, sel_val);
        res[ix++] = fe_mul(fe_mul(fe_mul(p_map, pa), b_sponge), fe_sub(cur[c->lanes_start + lane], expect));
      }
    }
  }

  if (air->feat_vm) {
    /* ---------------- VmCtrlAir (ctrl.rs:114-390) ---------------- */
    fe pi = cur[c->pi_prog];
    fe s_high = fe_mul(s_low, pi);
    const fe *b = cur; /* op bits */
    fe bo[17];
    for (int k = 0; k < 17; k++) bo[k] = b[c->op[k]];
    enum { CONST, MOV, ADD, SUB, MUL, NEG, EQ, SEL, SPONGE, ASSERT, ABIT, ARANGE, DIVMOD, DIV128, MULWIDE, LOAD, STORE };
    fe sum_d0 = 0, sum_a = 0, sum_b = 0, sum_c = 0, sum_d1 = 0;
    for (int i = 0; i < NR; i++) {
      fe sd0 = cur[c->sel_dst0 + i], sa = cur[c->sel_a + i], sb = cur[c->sel_b + i],
         sc = cur[c->sel_c + i], sd1 = cur[c->sel_dst1 + i];
      sum_d0 = fe_add(sum_d0, sd0); sum_a = fe_add(sum_a, sa); sum_b = fe_add(sum_b, sb);
      sum_c = fe_add(sum_c, sc); sum_d1 = fe_add(sum_d1, sd1);
      fe v[5] = {sd0, sa, sb, sc, sd1};
      for (int t = 0; t < 5; t++) res[ix++] = fe_add(fe_mul(p_map, fe_mul(v[t], fe_sub(v[t], 1))), s_high);
    }
    fe uses_a = 0, uses_b = 0, uses_c = 0, op_any = 0;
    const int ua[] = {MOV, ADD, SUB, MUL, NEG, EQ, SEL, DIVMOD, DIV128, MULWIDE, LOAD, STORE};
    for (unsigned i = 0; i < sizeof ua / sizeof ua[0]; i++) uses_a = fe_add(uses_a, bo[ua[i]]);
    const int ub[] = {ADD, SUB, MUL, EQ, SEL, DIVMOD, DIV128, MULWIDE, STORE};
    for (unsigned i = 0; i < sizeof ub / sizeof ub[0]; i++) uses_b = fe_add(uses_b, bo[ub[i]]);
    const int uc[] = {SEL, ASSERT, ABIT, ARANGE};
    for (unsigned i = 0; i < sizeof uc / sizeof uc[0]; i++) uses_c = fe_add(uses_c, bo[uc[i]]);
    const int oa[] = {CONST, MOV, ADD, SUB, MUL, NEG, EQ, SEL, SPONGE, ASSERT, ABIT, ARANGE, DIVMOD, DIV128, MULWIDE};
    for (unsigned i = 0; i < sizeof oa / sizeof oa[0]; i++) op_any = fe_add(op_any, bo[oa[i]]);
    fe uses_d0 = fe_add(fe_sub(op_any, bo[SPONGE]), bo[LOAD]);
    fe uses_d1 = fe_add(fe_add(bo[DIVMOD], bo[DIV128]), bo[MULWIDE]);
    res[ix++] = fe_add(fe_mul(p_map, fe_sub(sum_d0, uses_d0)), s_low);
    res[ix++] = fe_add(fe_mul(p_map, fe_sub(sum_a, uses_a)), s_low);
    res[ix++] = fe_add(fe_mul(p_map, fe_sub(sum_b, uses_b)), s_low);
    res[ix++] = fe_add(fe_mul(p_map, fe_sub(sum_c, uses_c)), s_low);
    res[ix++] = fe_add(fe_mul(p_map, fe_sub(sum_d1, uses_d1)), s_low);
    for (int i = 0; i < NR; i++)
      res[ix++] = fe_add(fe_mul(p_map, fe_mul(cur[c->sel_dst0 + i], cur[c->sel_dst1 + i])), s_high);
    if (air->feat_sponge && (m & (1u << U_SPONGE))) {
      for (int lane = 0; lane < 10; lane++) {
        for (int bit = 0; bit < 3; bit++) {
          fe v = cur[c->sel_s_bits + lane * 3 + bit];
          res[ix++] = fe_add(fe_mul(p_map, fe_mul(v, fe_sub(v, 1))), s_high);
        }
        fe a = cur[c->sel_s_active + lane];
        res[ix++] = fe_add(fe_mul(p_map, fe_mul(a, fe_sub(a, 1))), s_high);
      }
    }
    res[ix++] = s_high; /* select cond booleanity lives in ALU (ctrl.rs:280-290) */
    fe op_sum = 0;
    for (int k = 0; k < 17; k++) {
      res[ix++] = fe_add(fe_mul(p_map, fe_mul(bo[k], fe_sub(bo[k], 1))), s_high);
      op_sum = fe_add(op_sum, bo[k]);
    }
    res[ix++] = fe_add(fe_mul(p_map, fe_mul(op_sum, fe_sub(op_sum, 1))), s_high);
    for (int k = 0; k < 17; k++)
      res[ix++] = fe_add(fe_mul(rom_on, fe_mul(p_map, fe_sub(bo[k], cur[c->rom_op_start + k]))), s_high);
    fe pc_c = cur[c->pc], pc_n = nxt[c->pc];
    res[ix++] = fe_add(fe_mul(rom_on, fe_mul(g_carry, fe_sub(pc_n, pc_c))), s_low);
    res[ix++] = fe_add(fe_mul(rom_on, fe_mul(p_pad_last, fe_sub(pc_n, fe_add(pc_c, 1)))), s_low);

    /* ---------------- VmAluAir (alu.rs:108-354) ---------------- */
    int use_eq = !!(m & (1u << U_EQ)), use_divmod = !!(m & (1u << U_DIVMOD)),
        use_mulwide = !!(m & (1u << U_MULWIDE)), use_div128 = !!(m & (1u << U_DIV128)),
        use_assert = !!(m & (1u << U_ASSERT)), use_abit = !!(m & (1u << U_ASSERT_BIT)),
        use_arange = !!(m & (1u << U_ASSERT_RANGE));
    fe pi2 = fe_sqr(pi), pi4 = fe_sqr(pi2), pi6 = fe_mul(pi4, pi2);
    fe s_write = fe_mul(s_low, pi6), s_eq = fe_mul(s_low, pi4);
    fe a_val = 0, b_val = 0, c_val = 0;
    for (int i = 0; i < NR; i++) {
      fe r = cur[c->r_start + i];
      a_val = fe_add(a_val, fe_mul(cur[c->sel_a + i], r));
      b_val = fe_add(b_val, fe_mul(cur[c->sel_b + i], r));
      c_val = fe_add(c_val, fe_mul(cur[c->sel_c + i], r));
    }
    for (int i = 0; i < NR; i++)
      res[ix++] = fe_add(fe_mul(g_carry, fe_sub(nxt[c->r_start + i], cur[c->r_start + i])), s_low);
    fe imm = cur[c->imm];
    fe mode64 = cur[c->eq_inv];
    fe d0n = 0, d0c = 0, d1n = 0;
    for (int i = 0; i < NR; i++) {
      d0n = fe_add(d0n, fe_mul(cur[c->sel_dst0 + i], nxt[c->r_start + i]));
      d0c = fe_add(d0c, fe_mul(cur[c->sel_dst0 + i], cur[c->r_start + i]));
      d1n = fe_add(d1n, fe_mul(cur[c->sel_dst1 + i], nxt[c->r_start + i]));
    }
    fe r = fe_mul(bo[CONST], imm);
    r = fe_add(r, fe_mul(bo[MOV], a_val));
    r = fe_add(r, fe_mul(bo[ADD], fe_add(a_val, b_val)));
    r = fe_add(r, fe_mul(bo[SUB], fe_sub(a_val, b_val)));
    r = fe_add(r, fe_mul(bo[MUL], fe_mul(a_val, b_val)));
    r = fe_add(r, fe_mul(bo[NEG], fe_neg(a_val)));
    r = fe_add(r, fe_mul(bo[SEL], fe_add(fe_mul(c_val, a_val), fe_mul(fe_sub(1, c_val), b_val))));
    r = fe_add(r, fe_mul(bo[SPONGE], cur[c->lanes_start]));
    if (use_eq) r = fe_add(r, fe_mul(bo[EQ], d0n));
    if (use_assert) r = fe_add(r, bo[ASSERT]);
    if (use_abit) r = fe_add(r, bo[ABIT]);
    r = fe_add(r, fe_mul(bo[LOAD], imm));
    fe sum = 0, pow2 = 1;
    for (int i = 0; i < 32; i++) { sum = fe_add(sum, fe_mul(pow2, cur[c->gadget_b + i])); pow2 = fe_add(pow2, pow2); }
    if (use_arange) r = fe_add(r, fe_mul(bo[ARANGE], fe_add(fe_mul(fe_sub(1, imm), sum), imm)));
    int uses_two = use_divmod || use_mulwide || use_div128;
    fe b_two = uses_two ? fe_add(fe_add(bo[DIVMOD], bo[MULWIDE]), bo[DIV128]) : 0;
    fe w0 = fe_add(fe_mul(fe_sub(1, b_two), r), fe_mul(b_two, d0n));
    fe w1 = fe_mul(b_two, d1n);
    for (int i = 0; i < NR; i++) {
      fe sd0 = cur[c->sel_dst0 + i], sd1 = cur[c->sel_dst1 + i];
      fe keep = fe_sub(fe_sub(1, sd0), sd1);
      fe rhs = fe_add(fe_add(fe_mul(keep, cur[c->r_start + i]), fe_mul(sd0, w0)), fe_mul(sd1, w1));
      res[ix++] = fe_add(fe_mul(p_final, fe_sub(nxt[c->r_start + i], rhs)), s_write);
    }
    fe diff = fe_sub(a_val, b_val);
    fe inv = cur[c->eq_inv];
    if (use_eq) {
      res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[EQ], fe_mul(d0n, diff))), s_eq);
      res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[EQ], fe_sub(fe_sub(1, d0n), fe_mul(diff, inv)))), s_eq);
    }
    if (use_divmod) {
      res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[DIVMOD], fe_sub(fe_sub(a_val, fe_mul(b_val, d0n)), d1n))), s_eq);
      res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[DIVMOD], fe_sub(fe_mul(b_val, inv), 1))), s_eq);
    }
    fe p264 = ((fe)1) << 64;
    if (use_mulwide)
      res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[MULWIDE], fe_sub(fe_mul(a_val, b_val), fe_add(d0n, fe_mul(d1n, p264))))), s_eq);
    if (use_div128) {
      fe num128 = fe_add(fe_mul(a_val, p264), imm);
      res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[DIV128], fe_sub(num128, fe_add(fe_mul(b_val, d0n), d1n)))), s_eq);
      res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[DIV128], fe_sub(fe_mul(b_val, inv), 1))), s_eq);
    }
    if (use_assert)
      res[ix++] = fe_add(fe_mul(p_final, fe_add(fe_mul(bo[ASSERT], fe_sub(c_val, 1)),
                                                fe_mul(bo[SEL], fe_mul(c_val, fe_sub(c_val, 1))))), s_eq);
    if (use_abit)
      res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[ABIT], fe_mul(c_val, fe_sub(c_val, 1)))), s_eq);
    if (use_arange) {
      for (int i = 0; i < 32; i++) {
        fe bi = cur[c->gadget_b + i];
        res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[ARANGE], fe_mul(bi, fe_sub(bi, 1)))), s_eq);
      }
      fe p232 = ((fe)1) << 32;
      fe eq32 = fe_sub(c_val, sum);
      fe eq64 = fe_sub(c_val, fe_add(d0c, fe_mul(sum, p232)));
      fe eqt = fe_mul(imm, fe_add(fe_mul(mode64, eq64), fe_mul(fe_sub(1, mode64), eq32)));
      res[ix++] = fe_add(fe_mul(p_final, fe_mul(bo[ARANGE], eqt)), s_eq);
    }
  }

  if (air->feat_ram) {
    /* ---------------- RamAir (ram.rs:82-236) ---------------- */
    fe p_pad_ = per[29];
    fe g_hold = fe_sub(p_pad_, p_pad_last);
    fe op_load = cur[c->op[15]], op_store = cur[c->op[16]];
    fe event = fe_mul(p_final, fe_add(op_load, op_store));
    fe q0 = air->program_fe[0], q2 = fe_sqr(q0), q3 = fe_mul(q2, q0), q4 = fe_sqr(q2), q5 = fe_mul(q4, q0);
    fe r1 = fe_add(q2, 1), r2 = fe_add(q3, q0), r3 = fe_add(q5, 7);
    fe a_ev = 0, b_ev = 0;
    for (int i = 0; i < NR; i++) {
      fe ri = cur[c->r_start + i];
      a_ev = fe_add(a_ev, fe_mul(cur[c->sel_a + i], ri));
      b_ev = fe_add(b_ev, fe_mul(cur[c->sel_b + i], ri));
    }
    fe w_ev = op_store;
    fe val_ev = fe_add(fe_mul(w_ev, b_ev), fe_mul(fe_sub(1, w_ev), cur[c->imm]));
    fe comp_uns = fe_add(fe_add(fe_add(a_ev, fe_mul(r1, cur[c->pc])), fe_mul(r2, val_ev)), fe_mul(r3, w_ev));
    fe gu = cur[c->ram_gp_unsorted], gu_n = nxt[c->ram_gp_unsorted];
    res[ix++] = fe_add(fe_add(fe_mul(event, fe_sub(gu_n, fe_add(gu, comp_uns))), fe_mul(fe_sub(1, event), fe_sub(gu_n, gu))),
                       fe_mul(g_hold, fe_sub(gu_n, gu)));
    fe s_on = cur[c->ram_sorted], s_addr = cur[c->ram_s_addr], s_clk = cur[c->ram_s_clk], s_val = cur[c->ram_s_val],
       s_w = cur[c->ram_s_is_write], lastw = cur[c->ram_s_last_write];
    fe d_addr = fe_sub(nxt[c->ram_s_addr], s_addr);
    fe same = fe_sub(1, fe_mul(d_addr, cur[c->eq_inv]));
    fe comp = fe_add(fe_add(fe_add(s_addr, fe_mul(r1, s_clk)), fe_mul(r2, s_val)), fe_mul(r3, s_w));
    fe gs = cur[c->ram_gp_sorted], gs_n = nxt[c->ram_gp_sorted];
    res[ix++] = fe_add(fe_mul(s_on, fe_sub(gs_n, fe_add(gs, comp))), fe_mul(fe_sub(1, s_on), fe_sub(gs_n, gs)));
    fe sw_val = fe_mul(s_w, s_val);
    fe keep = fe_add(fe_mul(same, fe_add(fe_mul(fe_sub(1, s_w), lastw), sw_val)), fe_mul(fe_sub(1, same), sw_val));
    res[ix++] = fe_mul(s_on, fe_sub(nxt[c->ram_s_last_write], keep));
    res[ix++] = fe_mul(fe_mul(s_on, fe_sub(1, s_w)), fe_sub(s_val, lastw));
    fe s_on_n = nxt[c->ram_sorted];
    res[ix++] = fe_mul(fe_mul(fe_mul(fe_mul(s_on, s_on_n), fe_sub(1, same)), fe_sub(1, nxt[c->ram_s_is_write])),
                       nxt[c->ram_s_val]);
    res[ix++] = fe_mul(s_on, fe_mul(same, fe_sub(same, 1)));
    if (m & (1u << U_RAM_DCLK)) {
      fe d_clk = fe_sub(nxt[c->ram_s_clk], s_clk);
      fe sum = 0, pow2 = 1;
      fe g_same = fe_mul(s_on, same);
      for (int i = 0; i < 32; i++) {
        fe bi = cur[c->gadget_b + i];
        if ((air->ram_delta_clk_bits >> i) & 1) res[ix++] = fe_mul(g_same, fe_mul(bi, fe_sub(bi, 1)));
        sum = fe_add(sum, fe_mul(pow2, bi));
        pow2 = fe_add(pow2, pow2);
      }
      res[ix++] = fe_mul(fe_mul(fe_mul(s_on, s_on_n), same), fe_sub(d_clk, sum));
    }
    res[ix++] = fe_mul(p_last, fe_sub(gu, gs));
  }

  if (air->feat_merkle) {
    /* ---------------- MerkleAir (merkle.rs:60-134) ---------------- */
    fe g = cur[c->merkle_g], dir = cur[c->merkle_dir], acc = cur[c->merkle_acc], sib = cur[c->merkle_sib];
    fe pg = fe_mul(p_map, g);
    res[ix++] = fe_mul(pg, fe_mul(dir, fe_sub(dir, 1)));
    fe left = fe_add(fe_mul(fe_sub(1, dir), acc), fe_mul(dir, sib));
    fe right = fe_add(fe_mul(fe_sub(1, dir), sib), fe_mul(dir, acc));
    res[ix++] = fe_mul(pg, fe_sub(cur[c->lanes_start], left));
    res[ix++] = fe_mul(pg, fe_sub(cur[c->lanes_start + 1], right));
    res[ix++] = fe_mul(fe_mul(g, g_carry), fe_sub(nxt[c->merkle_acc], acc));
    res[ix++] = fe_mul(fe_mul(pg, cur[c->merkle_first]), fe_sub(acc, cur[c->merkle_leaf]));
    res[ix++] = fe_mul(fe_mul(fe_mul(p_final, g), cur[c->merkle_last]), fe_sub(acc, air->merkle_root));
    res[ix++] = fe_mul(fe_mul(fe_mul(p_pad_last, g), nxt[c->merkle_g]), fe_sub(nxt[c->merkle_acc], acc));
  }

  /* ---------------- RomAir (rom.rs:57-120); runs when program_commitment != 0 ------- */
  if (air->commit_nonzero) {
    fe s[3], s3[3];
    for (int i = 0; i < 3; i++) { s[i] = cur[c->rom_s + i]; s3[i] = fe_cube(s[i]); }
    fe ms[3];
    for (int i = 0; i < 3; i++) {
      fe acc = 0;
      for (int k = 0; k < 3; k++) acc = fe_add(acc, fe_mul(air->rom_mds[i][k], s3[k]));
      ms[i] = acc;
    }
    for (int j = 0; j < POS_ROUNDS; j++) {
      fe gr = per[1 + j];
      for (int i = 0; i < 3; i++)
        res[ix++] = fe_mul(gr, fe_sub(nxt[c->rom_s + i], fe_add(ms[i], air->rom_rc[j][i])));
    }
    fe g_hold = fe_sub(p_pad, p_pad_last);
    for (int i = 0; i < 3; i++) res[ix++] = fe_mul(g_hold, fe_sub(nxt[c->rom_s + i], cur[c->rom_s + i]));
    if (p_map != 0) {
      fe e0 = rom_encode(c, cur, air->rom_w0), e1 = rom_encode(c, cur, air->rom_w1);
      res[ix++] = fe_mul(p_map, fe_sub(cur[c->rom_s + 1], e0));
      res[ix++] = fe_mul(p_map, fe_sub(cur[c->rom_s + 2], e1));
    } else {
      res[ix++] = 0;
      res[ix++] = 0;
    }
  }
  (void)ix;
}
