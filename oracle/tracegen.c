/*
 * ORACLE — test infrastructure only.
 *
 * Synthetic VM segment built the way the reference builds traces:
 *   vm/trace/mod.rs:386-524     build_empty_trace / build_full_trace (schedule gates, pc, dom tags)
 *   vm/trace/vm.rs:58-888       VmTraceBuilder::fill_table (Const/Mov/Add/Sub/Mul/Neg/SAbsorbN/SSqueeze/
 *                               MerkleStepFirst/MerkleStep/MerkleStepLast/Load/Store/End)
 *   vm/trace/poseidon.rs:9-87   apply_level_absorb
 *   vm/trace/ram.rs:43-271      RamTraceBuilder (sorted table in pad rows, last-write, delta_clk bits,
 *                               grand-product compressors)
 *   vm/trace/vm.rs:890-921      op_to_one_hot (ROM mirror)
 *   vm/trace/rom.rs:29-108      RomTraceBuilder (t=3 accumulator)
 *   vm/trace/mod.rs:80-235      SegmentLayout projection (we build the segment layout directly)
 *   prove.rs:292-423,1289-1392  AIR public inputs, vm_usage_mask
 *   utils.rs:262-289            vm_output_from_trace
 * Program: levels-1 ALU ops cycling Const/Add/Mov/Mul over r0..r7 (splitmix64 choices,
 * immediates < 2^63) followed by End; program_id = BLAKE3 of a fixed descriptor string.
 * The product has its own generator (zk-lisp_amd/csrc/tracegen.cpp); tests pin it to this one.
 */
#include <stdio.h>
#include <string.h>
#include "oracle.h"

#define NR 8

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

enum { OP_CONST = 0, OP_MOV = 1, OP_ADD = 2, OP_SUB = 3, OP_MUL = 4, OP_NEG = 5, OP_EQ = 6, OP_SELECT = 7,
       OP_ASSERT = 9, OP_ASSERT_BIT = 10, OP_RANGE = 11, OP_DIVMOD = 12, OP_DIV128 = 13, OP_MULWIDE = 14,
       OP_ABSORB = 30, OP_SQUEEZE = 31, OP_CADDR = 32, OP_RANGE_LO = 33, OP_RANGE_HI = 34,
       OP_LOAD = 15, OP_STORE = 16, OP_MFIRST = 20, OP_MSTEP = 21, OP_MLAST = 22, OP_END = 99, OP_PAD = 100 };
/* dst2: DivMod r / DivMod128 r / MulWide hi; c: Select / Assert* / AssertRange* register, DivMod128 a_lo */
typedef struct { int kind; int dst, a, b; uint64_t imm; int nabs; int abs_regs[10]; int c, dst2, bits; } synth_op;

#define SYN_SPONGE 1u
#define SYN_RAM 2u
#define SYN_MERKLE 4u
#define RAM_ADDR_REG 7

/* Program generator.  flags 0: Const/Add/Mov/Mul cycle.  SYN_SPONGE: every 8 levels
 * absorb, const, absorb, squeeze, add, mov, mul, squeeze-with-nothing-pending (vm.rs:565-672).
 * SYN_RAM: 8-level block const-address (r7 <- 0..7), const, store, load, add, store, mul, load
 * (vm.rs:803-842); ALU destinations avoid r7 so addresses repeat; stores, adds and muls
 * read the latest result.  With both, the sponge block
 * is followed by the RAM block.  SYN_MERKLE: levels 1..5 are bit r5, bit r6, MerkleStepFirst
 * (leaf r0, dir r5, sib r1), MerkleStep (dir r6, sib r2), MerkleStepLast (dir r5, sib r3)
 * (vm.rs:675-800), a single path whose root becomes pi.merkle_root. */
static void synth_program(uint64_t seed, size_t levels, synth_op *ops, uint32_t flags) {
  uint64_t st = seed;
  static const int cyc[4] = {OP_CONST, OP_ADD, OP_MOV, OP_MUL};
  static const int cyc_s[8] = {OP_ABSORB, OP_CONST, OP_ABSORB, OP_SQUEEZE, OP_ADD, OP_MOV, OP_MUL, OP_SQUEEZE};
  static const int cyc_r[8] = {OP_CADDR, OP_CONST, OP_STORE, OP_LOAD, OP_ADD, OP_STORE, OP_MUL, OP_LOAD};
  int cycle[16], clen = 0;
  if (flags & SYN_SPONGE) for (int i = 0; i < 8; i++) cycle[clen++] = cyc_s[i];
  if (flags & SYN_RAM) for (int i = 0; i < 8; i++) cycle[clen++] = cyc_r[i];
  if (!clen) for (int i = 0; i < 4; i++) cycle[clen++] = cyc[i];
  int last_dst = 0;
  for (size_t l = 0; l + 1 < levels; l++) {
    uint64_t r = splitmix64(&st);
    synth_op *o = &ops[l];
    memset(o, 0, sizeof *o);
    o->kind = cycle[l % (size_t)clen];
    o->dst = (int)(r & 7);
    if (flags & SYN_RAM) o->dst %= RAM_ADDR_REG;
    o->a = (int)((r >> 3) & 7);
    o->b = (int)((r >> 6) & 7);
    o->imm = o->kind == OP_CONST ? (splitmix64(&st) >> 1) : 0;
    if (o->kind == OP_ABSORB) {
      o->nabs = 1 + (int)((r >> 9) % 3);
      for (int i = 0; i < 3; i++) o->abs_regs[i] = (int)((r >> (12 + 3 * i)) & 7);
    } else if (o->kind == OP_CADDR) {
      o->dst = RAM_ADDR_REG;
      o->imm = (r >> 9) & 7;
    } else if (o->kind == OP_LOAD || o->kind == OP_STORE) {
      o->a = RAM_ADDR_REG;
      if (o->kind == OP_STORE) o->b = last_dst; /* store the latest result */
    } else if ((flags & SYN_RAM) && (o->kind == OP_ADD || o->kind == OP_MUL)) {
      o->a = last_dst;
    }
    if (o->kind != OP_STORE && o->kind != OP_ABSORB && o->kind != OP_CADDR) last_dst = o->dst;
  }
  if ((flags & SYN_MERKLE) && levels >= 8) {
    uint64_t r = splitmix64(&st);
    synth_op m[5] = {{OP_CONST, 5, 0, 0, r & 1, 0, {0}, 0, 0, 0}, {OP_CONST, 6, 0, 0, (r >> 1) & 1, 0, {0}, 0, 0, 0},
                     {OP_MFIRST, 0, 5, 1, 0, 0, {0}, 0, 0, 0}, {OP_MSTEP, 0, 6, 2, 0, 0, {0}, 0, 0, 0},
                     {OP_MLAST, 0, 5, 3, 0, 0, {0}, 0, 0, 0}};
    for (int i = 0; i < 5; i++) ops[1 + i] = m[i]; /* MerkleStep*: dst = leaf reg, a = dir reg, b = sib reg */
  }
  memset(&ops[levels - 1], 0, sizeof ops[levels - 1]);
  ops[levels - 1].kind = OP_END;
}

static void set_fe(zkl_f128 *t, size_t n, int col, size_t row, fe v) {
  t[(size_t)col * n + row].lo = (uint64_t)v;
  t[(size_t)col * n + row].hi = (uint64_t)(v >> 64);
}
static fe get_fe(const zkl_f128 *t, size_t n, int col, size_t row) {
  const zkl_f128 *e = &t[(size_t)col * n + row];
  return ((fe)e->hi << 64) | e->lo;
}
static void set_sel(zkl_f128 *t, size_t n, size_t row, int start, int idx) {
  for (int i = 0; i < NR; i++) set_fe(t, n, start + i, row, 0);
  set_fe(t, n, start + idx, row, 1);
}

static fe rom_encode_row(const zk_cols *c, const zkl_f128 *t, size_t n, size_t row, const fe *w) {
  fe sum = 0;
  int k = 0;
  for (int i = 0; i < 17; i++) sum = fe_add(sum, fe_mul(get_fe(t, n, c->op[i], row), w[k++]));
  const int st[5] = {c->sel_dst0, c->sel_a, c->sel_b, c->sel_c, c->sel_dst1};
  for (int s = 0; s < 5; s++)
    for (int i = 0; i < NR; i++) sum = fe_add(sum, fe_mul(get_fe(t, n, st[s] + i, row), w[k++]));
  return sum;
}

int orc_synth_vm_segment(uint64_t seed, uint32_t log_n, zkl_f128 *t, zkl_air_public_inputs *pi,
                         uint32_t *width_out) {
  return orc_synth_vm_segment_ex(seed, log_n, 0, t, pi, width_out);
}

/* apply_level_absorb (vm/trace/poseidon.rs:9-87): lanes of one level hold the AIR-suite
 * permutation of [inputs (<= 10, zero padded), dom0, dom1]: map row = input state, round
 * row 1+j = state before round j, final and pad rows = output state */
static void apply_level_absorb(zkl_f128 *t, size_t n, const zk_cols *c, const pos_suite *ps, size_t level,
                               const fe *in, int nin) {
  size_t b = level * 32;
  fe st[12];
  for (int i = 0; i < 12; i++) st[i] = 0;
  for (int i = 0; i < nin && i < 10; i++) st[i] = in[i];
  st[10] = ps->dom[0];
  st[11] = ps->dom[1];
  for (int i = 0; i < 12; i++) set_fe(t, n, c->lanes_start + i, b, st[i]);
  for (int j = 0; j < POS_ROUNDS; j++) {
    for (int i = 0; i < 12; i++) set_fe(t, n, c->lanes_start + i, b + 1 + j, st[i]);
    fe s3[12], y[12];
    for (int i = 0; i < 12; i++) s3[i] = fe_cube(st[i]);
    for (int i = 0; i < 12; i++) {
      fe acc = 0;
      for (int k = 0; k < 12; k++) acc = fe_add(acc, fe_mul(ps->mds[i][k], s3[k]));
      y[i] = fe_add(acc, ps->rc[j][i]);
    }
    memcpy(st, y, sizeof st);
  }
  for (size_t r = b + 28; r < b + 32; r++)
    for (int i = 0; i < 12; i++) set_fe(t, n, c->lanes_start + i, r, st[i]);
}

static void set_sponge_sel(zkl_f128 *t, size_t n, const zk_cols *c, size_t row, const int *regs, int k) {
  for (int lane = 0; lane < 10; lane++) {
    int on = lane < k;
    int idx = on ? regs[lane] : 0;
    for (int bit = 0; bit < 3; bit++) set_fe(t, n, c->sel_s_bits + lane * 3 + bit, row, on ? (fe)((idx >> bit) & 1) : 0);
    set_fe(t, n, c->sel_s_active + lane, row, on ? 1 : 0);
  }
}

/* RamTraceBuilder::fill_table (vm/trace/ram.rs:43-271) */
static int cmp_event(const void *x, const void *y) {
  const fe *a = (const fe *)x, *b = (const fe *)y;
  if (a[0] != b[0]) return a[0] < b[0] ? -1 : 1;
  return (a[1] > b[1]) - (a[1] < b[1]);
}
static void ram_fill(zkl_f128 *t, size_t n, const zk_cols *c, const uint8_t pid[32], fe (*ev)[4], size_t n_ev) {
  qsort(ev, n_ev, sizeof *ev, cmp_event); /* (addr, clk) keys are unique: one event per level */
  size_t *ev_row = (size_t *)malloc((n_ev + 1) * sizeof(size_t));
  size_t k = 0;
  for (size_t row = 0; row < n; row++) {
    size_t pos = row % 32;
    if (pos >= 29 && k < n_ev) { /* pad rows hold the sorted table */
      set_fe(t, n, c->ram_sorted, row, 1);
      set_fe(t, n, c->ram_s_addr, row, ev[k][0]);
      set_fe(t, n, c->ram_s_clk, row, ev[k][1]);
      set_fe(t, n, c->ram_s_val, row, ev[k][2]);
      set_fe(t, n, c->ram_s_is_write, row, ev[k][3]);
      ev_row[k++] = row;
    }
  }
  for (size_t i = 0; i + 1 < n_ev; i++) { /* mirror same-address witnesses across the gap */
    if (ev[i][0] != ev[i + 1][0]) continue;
    for (size_t row = ev_row[i] + 1; row < ev_row[i + 1]; row++)
      if (!get_fe(t, n, c->ram_sorted, row)) {
        set_fe(t, n, c->ram_s_addr, row, ev[i][0]);
        set_fe(t, n, c->ram_s_clk, row, ev[i][1]);
        set_fe(t, n, c->ram_s_val, row, ev[i][2]);
        set_fe(t, n, c->ram_s_is_write, row, ev[i][3]);
      }
  }
  free(ev_row);
  fe fc[2];
  program_field_commitment(pid, fc);
  fe q0 = fc[0], q2 = fe_mul(q0, q0), q3 = fe_mul(q2, q0), q4 = fe_mul(q2, q2), q5 = fe_mul(q4, q0);
  fe r1 = fe_add(q2, 1), r2 = fe_add(q3, q0), r3 = fe_add(q5, 7);
  fe gp = 0, last = 0;
  for (size_t row = 0; row < n; row++) {
    if (row > 0 && get_fe(t, n, c->ram_sorted, row - 1)) {
      size_t p = row - 1;
      fe a = get_fe(t, n, c->ram_s_addr, p), clk = get_fe(t, n, c->ram_s_clk, p), v = get_fe(t, n, c->ram_s_val, p),
         w = get_fe(t, n, c->ram_s_is_write, p);
      gp = fe_add(gp, fe_add(fe_add(fe_add(a, fe_mul(r1, clk)), fe_mul(r2, v)), fe_mul(r3, w)));
      if (get_fe(t, n, c->ram_s_addr, row) == a) last = fe_add(fe_mul(fe_sub(1, w), last), fe_mul(w, v));
      else last = fe_mul(w, v);
    }
    set_fe(t, n, c->ram_gp_sorted, row, gp);
    set_fe(t, n, c->ram_s_last_write, row, last);
  }
  for (size_t row = 0; row + 1 < n; row++) {
    if (!get_fe(t, n, c->ram_sorted, row)) continue;
    fe a = get_fe(t, n, c->ram_s_addr, row), an = get_fe(t, n, c->ram_s_addr, row + 1);
    set_fe(t, n, c->eq_inv, row, fe_inv(fe_sub(an, a)));
    if (get_fe(t, n, c->ram_sorted, row + 1) && an == a) {
      fe clk = get_fe(t, n, c->ram_s_clk, row), clk_n = get_fe(t, n, c->ram_s_clk, row + 1);
      fe delta = clk_n > clk ? clk_n - clk : 0; /* as_int saturating_sub */
      for (int i = 0; i < 32; i++) set_fe(t, n, c->gadget_b + i, row, (delta >> i) & 1);
    }
  }
  fe gu = 0;
  for (size_t row = 0; row < n; row++) {
    if (row > 0 && (row - 1) % 32 == 28) {
      size_t p = row - 1;
      int ld = get_fe(t, n, c->op[15], p) == 1, stv = get_fe(t, n, c->op[16], p) == 1;
      if (ld || stv) {
        fe a_ev = 0, b_ev = 0;
        for (int i = 0; i < NR; i++) {
          fe ri = get_fe(t, n, c->r_start + i, p);
          a_ev = fe_add(a_ev, fe_mul(get_fe(t, n, c->sel_a + i, p), ri));
          b_ev = fe_add(b_ev, fe_mul(get_fe(t, n, c->sel_b + i, p), ri));
        }
        fe w = stv ? 1 : 0;
        fe val = stv ? b_ev : get_fe(t, n, c->imm, p);
        gu = fe_add(gu, fe_add(fe_add(fe_add(a_ev, fe_mul(r1, get_fe(t, n, c->pc, p))), fe_mul(r2, val)), fe_mul(r3, w)));
      }
    }
    set_fe(t, n, c->ram_gp_unsorted, row, gu);
  }
}

int orc_synth_vm_segment_ex(uint64_t seed, uint32_t log_n, uint32_t flags, zkl_f128 *t, zkl_air_public_inputs *pi,
                            uint32_t *width_out) {
  return orc_synth_vm_segment_chain(seed, seed, log_n, flags, NULL, t, pi, width_out);
}

/* The trace of a program of `levels` ops (OP_PAD past its last op) and its AIR public inputs:
 * build_full_trace (mod.rs:434-524) with the initial registers regs0 (vm.rs:64-104), ROM lane 0
 * entering the first level = rom0, written in the segment layout of the features. */
static int build_core(const synth_op *ops, size_t levels, const uint8_t pid[32], const uint8_t commit[32], int sponge,
                      int ram, int merkle, fe rom0, const fe regs0[NR], const fe *slots, uint32_t n_slots, zkl_f128 *t,
                      zkl_air_public_inputs *pi) {
  size_t n = levels * 32;
  zk_cols c;
  cols_for_config(1, ram, sponge, merkle, 1, &c);
  memset(t, 0, (size_t)c.width * n * sizeof(zkl_f128));
  memset(pi, 0, sizeof *pi);
  pos_suite ps;
  pos_suite_derive(pid, POS_ROUNDS, &ps);

  /* build_empty_trace + pc + dom tags (mod.rs:386-470) */
  for (size_t l = 0; l < levels; l++) {
    size_t b = l * 32;
    set_fe(t, n, c.g_map, b, 1);
    set_fe(t, n, c.g_final, b + 28, 1);
    for (int j = 0; j < POS_ROUNDS; j++) set_fe(t, n, c.g_r_start + j, b + 1 + j, 1);
    for (size_t r = b; r < b + 32; r++) set_fe(t, n, c.pc, r, (fe)l);
    set_fe(t, n, c.lanes_start + 10, b, ps.dom[0]);
    set_fe(t, n, c.lanes_start + 11, b, ps.dom[1]);
  }
  /* VmTraceBuilder (vm.rs:58-888) */
  fe regs[NR];
  memcpy(regs, regs0, sizeof regs);
  int pending[10], npending = 0;
  /* RAM: host memory (addr -> value) and the event log (addr, clk, val, is_write) */
  size_t n_ev = 0, n_mem = 0;
  fe (*ev)[4] = (fe(*)[4])malloc((levels + 1) * sizeof *ev);
  fe (*mem)[2] = (fe(*)[2])malloc((levels + 1) * sizeof *mem);
  int last_merkle = -1;
  for (size_t l = 0; l < levels; l++) {
    fe next[NR];
    memcpy(next, regs, sizeof next);
    size_t b = l * 32, rm = b, rf = b + 28;
    const synth_op *op = &ops[l];
    if (op->kind == OP_PAD) continue; /* registers stay zero past the program (build_empty_trace) */
    if (l == 0) set_fe(t, n, c.pi_prog, 0, be_from_le8(pid));
    int onehot = -1;
    switch (op->kind) {
      case OP_CONST: onehot = 0; break;
      case OP_MOV: onehot = 1; break;
      case OP_ADD: onehot = 2; break;
      case OP_SUB: onehot = 3; break;
      case OP_MUL: onehot = 4; break;
      case OP_NEG: onehot = 5; break;
      case OP_EQ: onehot = 6; break;
      case OP_SELECT: onehot = 7; break;
      case OP_ASSERT: onehot = 9; break;
      case OP_ASSERT_BIT: onehot = 10; break;
      case OP_RANGE:
      case OP_RANGE_LO:
      case OP_RANGE_HI: onehot = 11; break;
      case OP_DIVMOD: onehot = 12; break;
      case OP_DIV128: onehot = 13; break;
      case OP_MULWIDE: onehot = 14; break;
      case OP_ABSORB:
      case OP_SQUEEZE: onehot = 8; break;
      case OP_CADDR: onehot = 0; break;
      case OP_LOAD: onehot = 15; break;
      case OP_STORE: onehot = 16; break;
      default: break;
    }
    if (onehot >= 0) set_fe(t, n, c.rom_op_start + onehot, rm, 1);
    for (int i = 0; i < NR; i++) set_fe(t, n, c.r_start + i, rm, regs[i]);
    size_t rows[2] = {rm, rf};
    if (op->kind == OP_ABSORB || op->kind == OP_SQUEEZE) {
      /* SAbsorbN / SSqueeze (vm.rs:565-672): op_sponge and lane selectors at map and final */
      int sel_regs[10], k = 0;
      if (op->kind == OP_ABSORB) {
        for (int i = 0; i < op->nabs; i++) {
          if (npending == 10) { free(ev); free(mem); return -1; } /* push_absorb overflow (vm.rs:925-935) */
          sel_regs[k++] = op->abs_regs[i];
          pending[npending++] = op->abs_regs[i];
        }
      } else {
        for (int i = 0; i < npending; i++) sel_regs[k++] = pending[i];
      }
      for (int q = 0; q < 2; q++) {
        set_fe(t, n, c.op[8], rows[q], 1);
        set_sponge_sel(t, n, &c, rows[q], sel_regs, k);
      }
      if (op->kind == OP_SQUEEZE) {
        set_sel(t, n, rf, c.sel_dst0, op->dst);
        fe in[10];
        for (int i = 0; i < k; i++) in[i] = regs[sel_regs[i]];
        apply_level_absorb(t, n, &c, &ps, l, in, k);
        next[op->dst] = get_fe(t, n, c.lanes_start, rf);
        npending = 0;
        for (size_t r = b; r < b + 32; r++) set_fe(t, n, c.pose_active, r, 1);
      }
    }
    if (op->kind == OP_MFIRST || op->kind == OP_MSTEP || op->kind == OP_MLAST) {
      /* MerkleStepFirst / MerkleStep / MerkleStepLast (vm.rs:675-800) */
      for (size_t r = b; r < b + 32; r++) set_fe(t, n, c.merkle_g, r, 1);
      fe acc;
      if (op->kind == OP_MFIRST) {
        acc = regs[op->dst];
        set_fe(t, n, c.merkle_first, rm, 1);
        set_fe(t, n, c.merkle_leaf, rm, acc);
      } else {
        acc = last_merkle >= 0 ? get_fe(t, n, c.merkle_acc, (size_t)last_merkle * 32 + 28) : 0;
      }
      for (size_t r = rm; r < rf; r++) set_fe(t, n, c.merkle_acc, r, acc);
      fe d = regs[op->a], sib = regs[op->b];
      set_fe(t, n, c.merkle_dir, rm, d);
      set_fe(t, n, c.merkle_sib, rm, sib);
      fe in[2] = {fe_add(fe_mul(fe_sub(1, d), acc), fe_mul(d, sib)), fe_add(fe_mul(fe_sub(1, d), sib), fe_mul(d, acc))};
      apply_level_absorb(t, n, &c, &ps, l, in, 2);
      if (op->kind == OP_MLAST) set_fe(t, n, c.merkle_last, rf, 1);
      fe out = get_fe(t, n, c.lanes_start, rf);
      for (size_t r = rf; r < b + 32; r++) set_fe(t, n, c.merkle_acc, r, out);
      for (size_t r = b; r < b + 32; r++) set_fe(t, n, c.pose_active, r, 1);
      last_merkle = (int)l;
    }
    if (op->kind == OP_LOAD || op->kind == OP_STORE) {
      /* Load / Store (vm.rs:803-842): clk = level, loads read 0 from unwritten addresses */
      fe addr = regs[op->a], val = 0;
      size_t k = 0;
      while (k < n_mem && mem[k][0] != addr) k++;
      for (int q = 0; q < 2; q++) {
        set_fe(t, n, c.op[onehot], rows[q], 1);
        set_sel(t, n, rows[q], c.sel_a, op->a);
        if (op->kind == OP_LOAD) set_sel(t, n, rows[q], c.sel_dst0, op->dst);
        else set_sel(t, n, rows[q], c.sel_b, op->b);
      }
      if (op->kind == OP_LOAD) {
        val = k < n_mem ? mem[k][1] : 0;
        set_fe(t, n, c.imm, rm, val);
        set_fe(t, n, c.imm, rf, val);
        next[op->dst] = val;
      } else {
        val = regs[op->b];
        if (k == n_mem) { mem[k][0] = addr; n_mem++; }
        mem[k][1] = val;
      }
      ev[n_ev][0] = addr; ev[n_ev][1] = (fe)l; ev[n_ev][2] = val; ev[n_ev][3] = op->kind == OP_STORE;
      n_ev++;
    }
    /* ALU ops (vm.rs:199-564): op bit and selectors on map and final rows, imm / eq_inv /
     * range-gadget witnesses on both rows */
    const int k_ = op->kind;
    const fe M64 = (((fe)1) << 64) - 1;
    fe ra = regs[op->a], rb = regs[op->b], rc = regs[op->c];
    fe imm = 0, inv = 0, bitv[32];
    int gadget = 0;
    switch (k_) {
      case OP_CONST:
      case OP_CADDR: imm = (fe)op->imm; next[op->dst] = imm; break;
      case OP_MOV: next[op->dst] = ra; break;
      case OP_ADD: next[op->dst] = fe_add(ra, rb); break;
      case OP_SUB: next[op->dst] = fe_sub(ra, rb); break;
      case OP_MUL: next[op->dst] = fe_mul(ra, rb); break;
      case OP_NEG: next[op->dst] = fe_neg(ra); break;
      case OP_EQ: {
        fe d = fe_sub(ra, rb);
        inv = d ? fe_inv(d) : 0;
        next[op->dst] = d ? 0 : 1;
        break;
      }
      case OP_SELECT: next[op->dst] = fe_add(fe_mul(rc, ra), fe_mul(fe_sub(1, rc), rb)); break;
      case OP_ASSERT:
      case OP_ASSERT_BIT: next[op->dst] = 1; break;
      case OP_RANGE: { /* 32-bit form: imm 1, eq_inv 0, the low min(bits, 32) bits of r */
        int kb = op->bits < 32 ? op->bits : 32;
        for (int i = 0; i < 32; i++) bitv[i] = i < kb ? (rc >> i) & 1 : 0;
        imm = 1; gadget = 1;
        next[op->dst] = 1;
        break;
      }
      case OP_RANGE_LO: /* 64-bit stage 0: imm 0, eq_inv 1, low 32 bits; dst <- r mod 2^32 */
        for (int i = 0; i < 32; i++) bitv[i] = (rc >> i) & 1;
        inv = 1; gadget = 1;
        next[op->dst] = rc & 0xFFFFFFFFu;
        break;
      case OP_RANGE_HI: /* stage 1: imm 1, eq_inv 1, bits 32..63 */
        for (int i = 0; i < 32; i++) bitv[i] = (rc >> (32 + i)) & 1;
        imm = 1; inv = 1; gadget = 1;
        next[op->dst] = 1;
        break;
      case OP_DIVMOD: { /* canonical values as u128; results mod 2^64; eq_inv = (b mod 2^64)^-1 */
        fe q = rb ? ra / rb : 0, r = rb ? ra % rb : ra;
        next[op->dst] = q & M64;
        next[op->dst2] = r & M64;
        inv = rb ? fe_inv(rb & M64) : 0;
        break;
      }
      case OP_MULWIDE: {
        fe prod = (ra & M64) * (rb & M64);
        next[op->dst] = prod & M64;
        next[op->dst2] = prod >> 64;
        break;
      }
      case OP_DIV128: { /* ((a_hi << 64) | a_lo mod 2^64) / b; imm = a_lo */
        fe num = (ra << 64) | (rc & M64);
        fe q = rb ? num / rb : 0, r = rb ? num % rb : num;
        imm = rc;
        next[op->dst] = q & M64;
        next[op->dst2] = r & M64;
        inv = rb ? fe_inv(rb & M64) : 0;
        break;
      }
      default: break;
    }
    if (onehot >= 0 && onehot != 8 && onehot < 15) {
      int uses_a = k_ != OP_CONST && k_ != OP_CADDR && k_ != OP_ASSERT && k_ != OP_ASSERT_BIT && k_ != OP_RANGE &&
                   k_ != OP_RANGE_LO && k_ != OP_RANGE_HI;
      int uses_b = k_ == OP_ADD || k_ == OP_SUB || k_ == OP_MUL || k_ == OP_EQ || k_ == OP_SELECT || k_ == OP_DIVMOD ||
                   k_ == OP_DIV128 || k_ == OP_MULWIDE;
      int uses_c = k_ == OP_SELECT || k_ == OP_ASSERT || k_ == OP_ASSERT_BIT || k_ == OP_RANGE || k_ == OP_RANGE_LO ||
                   k_ == OP_RANGE_HI;
      int uses_d1 = k_ == OP_DIVMOD || k_ == OP_DIV128 || k_ == OP_MULWIDE;
      for (int q = 0; q < 2; q++) {
        size_t row = rows[q];
        set_fe(t, n, c.op[onehot], row, 1);
        set_sel(t, n, row, c.sel_dst0, op->dst);
        if (uses_d1) set_sel(t, n, row, c.sel_dst1, op->dst2);
        if (uses_a) set_sel(t, n, row, c.sel_a, op->a);
        if (uses_b) set_sel(t, n, row, c.sel_b, op->b);
        if (uses_c) set_sel(t, n, row, c.sel_c, op->c);
        set_fe(t, n, c.imm, row, imm);
        set_fe(t, n, c.eq_inv, row, inv);
        for (int i = 0; gadget && i < 32; i++) set_fe(t, n, c.gadget_b + i, row, bitv[i]);
      }
    }
    for (size_t r = rm + 1; r <= rf; r++)
      for (int i = 0; i < NR; i++) set_fe(t, n, c.r_start + i, r, regs[i]);
    for (size_t r = rf + 1; r < b + 32; r++)
      for (int i = 0; i < NR; i++) set_fe(t, n, c.r_start + i, r, next[i]);
    memcpy(regs, next, sizeof regs);
  }
  if (ram) ram_fill(t, n, &c, pid, ev, n_ev);
  free(ev);
  free(mem);
  /* RomTraceBuilder (rom.rs:37-106) */
  fe rc3[POS_ROUNDS][3], mds3[3][3], w0[59], w1[59];
  rom_constants(pid, rc3, mds3);
  {
    fe a = fe_exp(3, 17), cur = fe_mul(a, 3);
    for (int i = 0; i < 59; i++) { w0[i] = cur; cur = fe_mul(cur, 3); }
    a = fe_exp(3, 1037); cur = fe_mul(a, 3);
    for (int i = 0; i < 59; i++) { w1[i] = cur; cur = fe_mul(cur, 3); }
  }
  fe s0_prev = rom0;
  fe last_state[3] = {0, 0, 0};
  for (size_t l = 0; l < levels; l++) {
    size_t b = l * 32, rm = b, rf = b + 28;
    fe s1 = rom_encode_row(&c, t, n, rm, w0), s2 = rom_encode_row(&c, t, n, rm, w1);
    set_fe(t, n, c.rom_s, rm, s0_prev);
    set_fe(t, n, c.rom_s + 1, rm, s1);
    set_fe(t, n, c.rom_s + 2, rm, s2);
    fe s[3] = {s0_prev, s1, s2};
    for (int j = 0; j < POS_ROUNDS; j++) {
      size_t r = b + 1 + j;
      for (int i = 0; i < 3; i++) set_fe(t, n, c.rom_s + i, r, s[i]);
      fe s3[3] = {fe_cube(s[0]), fe_cube(s[1]), fe_cube(s[2])};
      fe y[3];
      for (int i = 0; i < 3; i++)
        y[i] = fe_add(fe_add(fe_add(fe_mul(mds3[i][0], s3[0]), fe_mul(mds3[i][1], s3[1])),
                             fe_mul(mds3[i][2], s3[2])), rc3[j][i]);
      for (int i = 0; i < 3; i++) set_fe(t, n, c.rom_s + i, r + 1, y[i]);
      memcpy(s, y, sizeof s);
    }
    for (size_t r = rf + 1; r < b + 32; r++)
      for (int i = 0; i < 3; i++) set_fe(t, n, c.rom_s + i, r, s[i]);
    s0_prev = s[0];
    memcpy(last_state, s, sizeof s);
  }

  /* AIR public inputs (prove.rs:292-423 with segment = whole trace) */
  memcpy(pi->program_id, pid, 32);
  memcpy(pi->program_commitment, commit, 32);
  pi->feature_mask = FM_VM | (sponge ? FM_SPONGE | FM_POSEIDON : 0) | (ram ? FM_RAM : 0) |
                     (merkle ? FM_MERKLE | FM_POSEIDON : 0);
  long mlast = -1;
  for (size_t l = 0; l < levels; l++) if (ops[l].kind == OP_MLAST) mlast = (long)l;
  if (merkle && mlast >= 0) { /* root = acc after the last MerkleStepLast level, 16 LE bytes (utils.rs:346-355) */
    fe root = get_fe(t, n, c.merkle_acc, (size_t)mlast * 32 + 28);
    for (int i = 0; i < 16; i++) pi->merkle_root[i] = (uint8_t)(root >> (8 * i));
  }
  pi->segment_feature_mask = pi->feature_mask;
  pi->n_main_slots = n_slots;
  for (uint32_t i = 0; i < n_slots; i++) { pi->main_slots[i].lo = (uint64_t)slots[i]; pi->main_slots[i].hi = (uint64_t)(slots[i] >> 64); }
  /* vm_output_from_trace_with_layout (utils.rs:262-289) */
  pi->vm_out_reg = 0; pi->vm_out_row = 29;
  for (size_t l = levels; l-- > 0;) {
    size_t rf = l * 32 + 28;
    int found = -1;
    for (int i = 0; i < NR; i++) if (get_fe(t, n, c.sel_dst0 + i, rf) == 1) { found = i; break; }
    if (found >= 0) { pi->vm_out_reg = (uint32_t)found; pi->vm_out_row = (uint32_t)(rf + 1); break; }
  }
  for (int i = 0; i < 3; i++) {
    fe v = last_state[i];
    pi->rom_acc[i].lo = (uint64_t)v; pi->rom_acc[i].hi = (uint64_t)(v >> 64);
    fe in = get_fe(t, n, c.rom_s + i, 0);
    pi->rom_s_in[i].lo = (uint64_t)in; pi->rom_s_in[i].hi = (uint64_t)(in >> 64);
    fe out = get_fe(t, n, c.rom_s + i, (levels - 1) * 32 + 28);
    pi->rom_s_out[i].lo = (uint64_t)out; pi->rom_s_out[i].hi = (uint64_t)(out >> 64);
  }
  fe pc0 = get_fe(t, n, c.pc, 0);
  pi->pc_init.lo = (uint64_t)pc0; pi->pc_init.hi = (uint64_t)(pc0 >> 64);
  /* compute_vm_usage_mask_for_trace (prove.rs:1289-1392): ALU-only program -> 0 */
  uint32_t mask = 0;
  for (size_t r = 0; r < n; r++) {
    int at_final = (r % 32) == 28;
    if (at_final && (get_fe(t, n, c.op[9], r) || get_fe(t, n, c.op[7], r))) mask |= 1u << 0;
    if (at_final && get_fe(t, n, c.op[10], r)) mask |= 1u << 1;
    if (at_final && get_fe(t, n, c.op[11], r)) mask |= 1u << 2;
    if (at_final && get_fe(t, n, c.op[12], r)) mask |= 1u << 3;
    if (at_final && get_fe(t, n, c.op[14], r)) mask |= 1u << 4;
    if (at_final && get_fe(t, n, c.op[13], r)) mask |= 1u << 5;
    if (at_final && get_fe(t, n, c.op[6], r)) mask |= 1u << 6;
    if (get_fe(t, n, c.op[8], r)) mask |= 1u << 7;
  }
  uint32_t ram_bits = 0;
  if (ram)
    for (size_t r = 0; r + 1 < n; r++)
      if (get_fe(t, n, c.ram_sorted, r) && get_fe(t, n, c.ram_sorted, r + 1) &&
          get_fe(t, n, c.ram_s_addr, r) == get_fe(t, n, c.ram_s_addr, r + 1)) {
        mask |= 1u << 8;
        for (int i = 0; i < 32; i++) if (get_fe(t, n, c.gadget_b + i, r)) ram_bits |= 1u << i;
      }
  pi->vm_usage_mask = mask;
  pi->ram_delta_clk_bits = ram_bits;
  return 0;
}

/* the synthetic program with ROM lane 0 entering the first level at *rom0_in (the accumulator
 * lane the aggregation chains across segments, agg/trace.rs:524-541) instead of 0 */
int orc_synth_vm_segment_chain(uint64_t program_seed, uint64_t seed, uint32_t log_n, uint32_t flags, const zkl_f128 *rom0_in, zkl_f128 *t,
                               zkl_air_public_inputs *pi, uint32_t *width_out) {
  if (log_n < 5 || log_n > 26 || (flags & ~7u)) return -1;
  if ((flags & SYN_MERKLE) && log_n < 8) return -1;
  size_t n = (size_t)1 << log_n, levels = n / 32;
  zk_cols c;
  cols_for_config(1, !!(flags & SYN_RAM), !!(flags & SYN_SPONGE), !!(flags & SYN_MERKLE), 1, &c);
  if (width_out) *width_out = (uint32_t)c.width;
  if (!t) return 0;
  char desc[160];
  snprintf(desc, sizeof desc, "zkl-hip/synthetic-vm-segment/v1 %s%s%sseed=0x%016llx levels=%zu",
           (flags & SYN_SPONGE) ? "sponge " : "", (flags & SYN_RAM) ? "ram " : "", (flags & SYN_MERKLE) ? "merkle " : "",
           (unsigned long long)program_seed, levels);
  uint8_t pid[32];
  orc_blake3((const uint8_t *)desc, strlen(desc), pid);
  synth_op *ops = (synth_op *)malloc(levels * sizeof(synth_op));
  synth_program(seed, levels, ops, flags);
  fe regs0[NR] = {0};
  int rc = build_core(ops, levels, pid, pid, !!(flags & SYN_SPONGE), !!(flags & SYN_RAM), !!(flags & SYN_MERKLE),
                      rom0_in ? ((fe)rom0_in->hi << 64 | rom0_in->lo) : 0, regs0, NULL, 0, t, pi);
  free(ops);
  return rc;
}

/* The op-list trace builder (zkl_build_trace's twin): builder::Op list (builder.rs:25-158)
 * -> build_full_trace (mod.rs:434-524) over next_pow2(n_ops) levels. */
int orc_build_trace(const zkl_op *zops, uint32_t n_ops, const uint8_t pid[32], const uint8_t commit[32],
                    const uint64_t *secret, uint32_t n_secret, const zkl_vm_arg *margs, uint32_t n_main,
                    const zkl_f128 *rom0_in, zkl_f128 *t, zkl_air_public_inputs *pi, uint32_t *width_out,
                    uint32_t *n_rows_out) {
  static const int kinds[] = {OP_CONST, OP_MOV, OP_ADD, OP_SUB, OP_MUL, OP_NEG, OP_EQ, OP_SELECT, OP_ASSERT,
                              OP_ASSERT_BIT, OP_RANGE, OP_RANGE_LO, OP_RANGE_HI, OP_DIVMOD, OP_DIV128, OP_MULWIDE,
                              OP_LOAD, OP_STORE, OP_ABSORB, OP_SQUEEZE, OP_MFIRST, OP_MSTEP, OP_MLAST, OP_END};
  if (!zops || !n_ops || n_main > ZKL_MAX_MAIN_SLOTS) return -1;
  size_t levels = 1;
  while (levels < n_ops) levels <<= 1;
  synth_op *ops = (synth_op *)calloc(levels, sizeof(synth_op));
  int sponge = 0, ram = 0, merkle = 0;
  for (size_t l = 0; l < levels; l++) {
    synth_op *o = &ops[l];
    if (l >= n_ops) { o->kind = OP_PAD; continue; }
    const zkl_op *z = &zops[l];
    if (z->kind >= sizeof kinds / sizeof kinds[0] || z->dst > 7 || z->dst2 > 7 || z->a > 7 || z->b > 7 || z->c > 7 ||
        z->n_regs > 10 || (z->kind == ZKL_OP_ASSERT_RANGE && (z->bits < 1 || z->bits > 64)) ||
        (z->kind == ZKL_OP_SABSORBN && z->n_regs < 1)) {
      free(ops);
      return -1;
    }
    o->kind = kinds[z->kind];
    o->dst = z->dst; o->dst2 = z->dst2; o->a = z->a; o->b = z->b; o->c = z->c; o->bits = z->bits; o->imm = z->imm;
    o->nabs = z->n_regs;
    for (int i = 0; i < z->n_regs; i++) {
      if (z->regs[i] > 7) { free(ops); return -1; }
      o->abs_regs[i] = z->regs[i];
    }
    sponge |= o->kind == OP_ABSORB || o->kind == OP_SQUEEZE;
    ram |= o->kind == OP_LOAD || o->kind == OP_STORE;
    merkle |= o->kind == OP_MFIRST || o->kind == OP_MSTEP || o->kind == OP_MLAST;
  }
  zk_cols c;
  cols_for_config(1, ram, sponge, merkle, 1, &c);
  if (width_out) *width_out = (uint32_t)c.width;
  if (n_rows_out) *n_rows_out = (uint32_t)(levels * 32);
  if (!t) { free(ops); return 0; }
  fe slots[8];
  uint32_t ns = 0;
  for (uint32_t i = 0; i < n_main; i++) { /* encode_vmarg_to_elements (utils.rs:79-97) */
    const zkl_vm_arg *a = &margs[i];
    int need = a->tag == 2 ? 2 : 1;
    if (a->tag > 2 || ns + need > 8) { free(ops); return -1; }
    if (a->tag == 0) { uint64_t x; memcpy(&x, a->bytes, 8); slots[ns++] = x; }
    else { slots[ns++] = be_from_le8(a->bytes); if (a->tag == 2) slots[ns++] = be_from_le8(a->bytes + 16); }
  }
  fe regs0[NR] = {0};
  uint32_t tail = NR - ns;
  for (uint32_t i = 0; i < n_secret && i < tail; i++) regs0[i] = secret[i];
  for (uint32_t j = 0; j < ns; j++) regs0[tail + j] = slots[j];
  int rc = build_core(ops, levels, pid, commit, sponge, ram, merkle, rom0_in ? ((fe)rom0_in->hi << 64 | rom0_in->lo) : 0,
                      regs0, slots, ns, t, pi);
  free(ops);
  return rc;
}
