// ZkLispAir::evaluate_transition (vm/air/mod.rs:324-378) folded with the composition
// coefficients: sum_j alpha_j c_j(x) over the transition constraints in the reference's
// evaluation order (PoseidonAir, VmCtrlAir, VmAluAir, RamAir, MerkleAir, RomAir).  One
// definition for the device constraint evaluator (constraint_eval_kernel, every CE point) and
// the host verifier (zkl_verify_segment, the out-of-domain point): cur(c) / nxt(c) read
// column c of the current / next frame, per[0..31) are the cycle-32 periodic columns at x
// and p_last = L_{n-1}(x).  POSE / RM compile the Poseidon and RAM/Merkle blocks in or out.
#pragma once
#include "air_host.h"
#include "field.h"

namespace zkl {

struct AirAcc {
  uint32_t a[9];
  int ix;
  const fe* al;
  __host__ __device__ __forceinline__ void emit(fe v) { mul_acc(al[ix++], v, a); }
};

// pose_k: K_j = sum_i alpha_{12j+i} rc[j][i] for the 27 Poseidon rounds (pose_k_kernel, once per
// proof), or nullptr to form them here (host verifier).
// PART: 0 = the whole sum; 1 = the PoseidonAir block alone; 2 = everything after it (its alphas
// skipped).  Parts 1 + 2 = part 0: the device evaluates the Poseidon block in a kernel of its own,
// whose register footprint does not add to the rest's.
constexpr int pose_block_constraints(const AirDevice& a) { return 27 * 12 + 12 + (a.pose_bind ? 10 : 0); }
template <bool POSE, bool RM, int PART = 0, class Cur, class Nxt>
__host__ __device__ __forceinline__ fe air_transition_sum(const AirDevice& c_air, Cur cur, Nxt nxt, const fe* per,
                                                          fe p_last, const fe* alpha, const fe* pose_k = nullptr) {
  const Layout& C = c_air.cols;
  fe p_map = per[0], p_final = per[28], p_pad = per[29], p_pad_last = per[30];
  fe s_low = fe_mul(p_last, p_map);
  fe g_carry = fe_add_sel(p_map, fe_sub_sel(p_pad, p_pad_last));
  for (int j = 0; j < 26; j++) g_carry = fe_add_sel(g_carry, per[1 + j]);
  const fe rom_on = c_air.commit_nonzero ? fe_one() : fe_zero();
  const uint32_t m = c_air.vm_usage_mask;

  AirAcc A;
#pragma unroll
  for (int k = 0; k < 9; k++) A.a[k] = 0;
  A.ix = 0;
  A.al = alpha;
  const fe one = fe_one();

  if (POSE && PART == 2) A.ix += pose_block_constraints(c_air);
  if (POSE && PART != 2) {
    // ---------------- PoseidonAir (poseidon.rs:65-162): y = MDS s^3 (+ rc_j) is the same
    // for all 27 rounds but the round constant, so it is formed once per point
    const fe pa = cur(C.pose_active);
    fe s3[12];
#pragma unroll
    for (int i = 0; i < 12; i++) s3[i] = fe_cube(cur(C.lanes_start + i));
    fe ms[12];
    for (int i = 0; i < 12; i++) {
      uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 12; k++) mul_acc(c_air.pose_mds[i][k], s3[k], acc);
      ms[i] = reduce288(acc);
    }
    // constraint (j, i) = g_j (nxt_i - ms_i - rc_ji), g_j = pa per_j; its alpha-weighted sum over
    // i is g_j (sum_i alpha_ji d_i - K_j) with d_i = nxt_i - ms_i: one lazy dot product and one
    // product per round instead of 12 reduced products (the sum is the same field element)
    fe d[12];
#pragma unroll
    for (int i = 0; i < 12; i++) d[i] = fe_sub(nxt(C.lanes_start + i), ms[i]);
    const fe* al = A.al + A.ix;
    for (int j = 0; j < 27; j++) {
      uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 12; i++) mul_acc(al[12 * j + i], d[i], acc);
      fe kj;
      if (pose_k) {
        kj = pose_k[j];
      } else {
        uint32_t ka[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < 12; i++) mul_acc(al[12 * j + i], c_air.pose_rc[j][i], ka);
        kj = reduce288(ka);
      }
      mul_acc(fe_mul(pa, per[1 + j]), fe_sub(reduce288(acc), kj), A.a);
    }
    A.ix += 27 * 12;
    const fe g_hold = fe_sub_sel(p_pad, p_pad_last);
    for (int i = 0; i < 12; i++) A.emit(fe_mul(g_hold, fe_sub(nxt(C.lanes_start + i), cur(C.lanes_start + i))));
    if (c_air.pose_bind) {
      const fe gate = fe_mul(fe_mul(p_map, pa), cur(C.op[8]));
      fe rr[8];
#pragma unroll
      for (int i = 0; i < 8; i++) rr[i] = cur(C.r_start + i);
      for (int lane = 0; lane < 10; lane++) {
        const fe b0 = cur(C.sel_s_bits + lane * 3), b1 = cur(C.sel_s_bits + lane * 3 + 1),
                 b2 = cur(C.sel_s_bits + lane * 3 + 2), act = cur(C.sel_s_active + lane);
        const fe nb0 = fe_sub_sel(one, b0), nb1 = fe_sub_sel(one, b1), nb2 = fe_sub_sel(one, b2);
        const fe s0 = fe_add(fe_mul(b0, rr[1]), fe_mul(nb0, rr[0]));
        const fe s1 = fe_add(fe_mul(b0, rr[3]), fe_mul(nb0, rr[2]));
        const fe s2 = fe_add(fe_mul(b0, rr[5]), fe_mul(nb0, rr[4]));
        const fe s3v = fe_add(fe_mul(b0, rr[7]), fe_mul(nb0, rr[6]));
        const fe t0 = fe_add(fe_mul(b1, s1), fe_mul(nb1, s0));
        const fe t1 = fe_add(fe_mul(b1, s3v), fe_mul(nb1, s2));
        const fe sel_val = fe_add(fe_mul(b2, t1), fe_mul(nb2, t0));
        A.emit(fe_mul(gate, fe_sub(cur(C.lanes_start + lane), fe_mul(act, sel_val))));
      }
    }
  }
  if (PART == 1) return reduce288(A.a);

  if (c_air.feat_vm) {
    // ---------------- VmCtrlAir (ctrl.rs:114-390)
    fe pi = cur(C.pi_prog);
    fe s_high = fe_mul(s_low, pi);
    fe sum_d0 = fe_zero(), sum_a = fe_zero(), sum_b = fe_zero(), sum_c = fe_zero(), sum_d1 = fe_zero();
    for (int r = 0; r < 8; r++) {
      const fe v0 = cur(C.sel_dst0 + r), v1 = cur(C.sel_a + r), v2 = cur(C.sel_b + r), v3 = cur(C.sel_c + r),
               v4 = cur(C.sel_dst1 + r);
      sum_d0 = fe_add_sel(sum_d0, v0); sum_a = fe_add_sel(sum_a, v1); sum_b = fe_add_sel(sum_b, v2);
      sum_c = fe_add_sel(sum_c, v3); sum_d1 = fe_add_sel(sum_d1, v4);
      auto bit = [&](fe v) { A.emit(fe_add_sel(fe_mul(p_map, fe_mul(v, fe_sub_sel(v, one))), s_high)); };
      bit(v0); bit(v1); bit(v2); bit(v3); bit(v4);
    }
    // op bits read through cur() wherever used: a local fe[17] indexed in the loops below was
    // placed in scratch (288 B per lane)
    auto bo = [&](int k) { return cur(C.op[k]); };
    enum { CONST, MOV, ADD, SUB, MUL, NEG, EQ, SEL, SPONGE, ASSERT, ABIT, ARANGE, DIVMOD, DIV128, MULWIDE, LOAD, STORE };
    fe uses_a = fe_add_sel(fe_add_sel(fe_add_sel(bo(MOV), bo(ADD)), fe_add_sel(bo(SUB), bo(MUL))), fe_add_sel(fe_add_sel(bo(NEG), bo(EQ)), bo(SEL)));
    uses_a = fe_add_sel(uses_a, fe_add_sel(fe_add_sel(bo(DIVMOD), bo(DIV128)), fe_add_sel(fe_add_sel(bo(MULWIDE), bo(LOAD)), bo(STORE))));
    fe uses_b = fe_add_sel(fe_add_sel(fe_add_sel(bo(ADD), bo(SUB)), fe_add_sel(bo(MUL), bo(EQ))), fe_add_sel(bo(SEL), bo(DIVMOD)));
    uses_b = fe_add_sel(uses_b, fe_add_sel(fe_add_sel(bo(DIV128), bo(MULWIDE)), bo(STORE)));
    fe uses_c = fe_add_sel(fe_add_sel(bo(SEL), bo(ASSERT)), fe_add_sel(bo(ABIT), bo(ARANGE)));
    fe op_any = fe_zero();
#pragma unroll
    for (int k = 0; k <= MULWIDE; k++) op_any = fe_add_sel(op_any, bo(k));
    fe uses_d0 = fe_add_sel(fe_sub_sel(op_any, bo(SPONGE)), bo(LOAD));
    fe uses_d1 = fe_add_sel(fe_add_sel(bo(DIVMOD), bo(DIV128)), bo(MULWIDE));
    A.emit(fe_add_sel(fe_mul(p_map, fe_sub_sel(sum_d0, uses_d0)), s_low));
    A.emit(fe_add_sel(fe_mul(p_map, fe_sub_sel(sum_a, uses_a)), s_low));
    A.emit(fe_add_sel(fe_mul(p_map, fe_sub_sel(sum_b, uses_b)), s_low));
    A.emit(fe_add_sel(fe_mul(p_map, fe_sub_sel(sum_c, uses_c)), s_low));
    A.emit(fe_add_sel(fe_mul(p_map, fe_sub_sel(sum_d1, uses_d1)), s_low));
    for (int r = 0; r < 8; r++)
      A.emit(fe_add_sel(fe_mul(p_map, fe_mul(cur(C.sel_dst0 + r), cur(C.sel_dst1 + r))), s_high));
    if (c_air.sponge_block) {
      for (int lane = 0; lane < 10; lane++) {
        for (int bit = 0; bit < 3; bit++) {
          fe v = cur(C.sel_s_bits + lane * 3 + bit);
          A.emit(fe_add_sel(fe_mul(p_map, fe_mul(v, fe_sub_sel(v, one))), s_high));
        }
        fe a = cur(C.sel_s_active + lane);
        A.emit(fe_add_sel(fe_mul(p_map, fe_mul(a, fe_sub_sel(a, one))), s_high));
      }
    }
    A.emit(s_high);
    fe op_sum = fe_zero();
#pragma unroll
    for (int k = 0; k < 17; k++) {
      A.emit(fe_add_sel(fe_mul(p_map, fe_mul(bo(k), fe_sub_sel(bo(k), one))), s_high));
      op_sum = fe_add_sel(op_sum, bo(k));
    }
    A.emit(fe_add_sel(fe_mul(p_map, fe_mul(op_sum, fe_sub_sel(op_sum, one))), s_high));
#pragma unroll
    for (int k = 0; k < 17; k++)
      A.emit(fe_add_sel(fe_mul(rom_on, fe_mul(p_map, fe_sub_sel(bo(k), cur(C.rom_op_start + k)))), s_high));
    fe pc_c = cur(C.pc), pc_n = nxt(C.pc);
    A.emit(fe_add_sel(fe_mul(rom_on, fe_mul(g_carry, fe_sub_sel(pc_n, pc_c))), s_low));
    A.emit(fe_add_sel(fe_mul(rom_on, fe_mul(p_pad_last, fe_sub_sel(pc_n, fe_add_sel(pc_c, one)))), s_low));

    // ---------------- VmAluAir (alu.rs:108-354)
    const bool use_eq = m & (1u << 6), use_divmod = m & (1u << 3), use_mulwide = m & (1u << 4),
               use_div128 = m & (1u << 5), use_assert = m & 1u, use_abit = m & 2u, use_arange = m & 4u;
    fe pi2 = fe_sqr(pi), pi4 = fe_sqr(pi2), pi6 = fe_mul(pi4, pi2);
    fe s_write = fe_mul(s_low, pi6), s_eq = fe_mul(s_low, pi4);
    fe a_val = fe_zero(), b_val = fe_zero(), c_val = fe_zero(), d0n = fe_zero(), d0c = fe_zero(), d1n = fe_zero();
    for (int r = 0; r < 8; r++) {
      fe rc = cur(C.r_start + r), rn = nxt(C.r_start + r);
      a_val = fe_add_sel(a_val, fe_mul(cur(C.sel_a + r), rc));
      b_val = fe_add_sel(b_val, fe_mul(cur(C.sel_b + r), rc));
      c_val = fe_add_sel(c_val, fe_mul(cur(C.sel_c + r), rc));
      fe sd0 = cur(C.sel_dst0 + r);
      d0n = fe_add_sel(d0n, fe_mul(sd0, rn));
      d0c = fe_add_sel(d0c, fe_mul(sd0, rc));
      d1n = fe_add_sel(d1n, fe_mul(cur(C.sel_dst1 + r), rn));
    }
    for (int r = 0; r < 8; r++)
      A.emit(fe_add_sel(fe_mul(g_carry, fe_sub_sel(nxt(C.r_start + r), cur(C.r_start + r))), s_low));
    fe imm = cur(C.imm);
    fe mode64 = cur(C.eq_inv);
    fe res = fe_mul(bo(CONST), imm);
    res = fe_add_sel(res, fe_mul(bo(MOV), a_val));
    res = fe_add_sel(res, fe_mul(bo(ADD), fe_add_sel(a_val, b_val)));
    res = fe_add_sel(res, fe_mul(bo(SUB), fe_sub_sel(a_val, b_val)));
    res = fe_add_sel(res, fe_mul(bo(MUL), fe_mul(a_val, b_val)));
    res = fe_add_sel(res, fe_mul(bo(NEG), fe_neg(a_val)));
    res = fe_add_sel(res, fe_mul(bo(SEL), fe_add_sel(fe_mul(c_val, a_val), fe_mul(fe_sub_sel(one, c_val), b_val))));
    res = fe_add_sel(res, fe_mul(bo(SPONGE), cur(C.lanes_start)));
    if (use_eq) res = fe_add_sel(res, fe_mul(bo(EQ), d0n));
    if (use_assert) res = fe_add_sel(res, bo(ASSERT));
    if (use_abit) res = fe_add_sel(res, bo(ABIT));
    res = fe_add_sel(res, fe_mul(bo(LOAD), imm));
    fe bsum = fe_zero();
    if (use_arange) {
      fe pow2 = one;
      for (int k = 0; k < 32; k++) { bsum = fe_add_sel(bsum, fe_mul(pow2, cur(C.gadget_b + k))); pow2 = fe_add_sel(pow2, pow2); }
      res = fe_add_sel(res, fe_mul(bo(ARANGE), fe_add_sel(fe_mul(fe_sub_sel(one, imm), bsum), imm)));
    }
    bool uses_two = use_divmod || use_mulwide || use_div128;
    fe b_two = uses_two ? fe_add_sel(fe_add_sel(bo(DIVMOD), bo(MULWIDE)), bo(DIV128)) : fe_zero();
    fe w0 = fe_add_sel(fe_mul(fe_sub_sel(one, b_two), res), fe_mul(b_two, d0n));
    fe w1 = fe_mul(b_two, d1n);
    for (int r = 0; r < 8; r++) {
      fe sd0 = cur(C.sel_dst0 + r), sd1 = cur(C.sel_dst1 + r);
      fe keep = fe_sub_sel(fe_sub_sel(one, sd0), sd1);
      fe rhs = fe_add_sel(fe_add_sel(fe_mul(keep, cur(C.r_start + r)), fe_mul(sd0, w0)), fe_mul(sd1, w1));
      A.emit(fe_add_sel(fe_mul(p_final, fe_sub_sel(nxt(C.r_start + r), rhs)), s_write));
    }
    fe diff = fe_sub_sel(a_val, b_val);
    fe inv = cur(C.eq_inv);
    if (use_eq) {
      A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(EQ), fe_mul(d0n, diff))), s_eq));
      A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(EQ), fe_sub_sel(fe_sub_sel(one, d0n), fe_mul(diff, inv)))), s_eq));
    }
    if (use_divmod) {
      A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(DIVMOD), fe_sub_sel(fe_sub_sel(a_val, fe_mul(b_val, d0n)), d1n))), s_eq));
      A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(DIVMOD), fe_sub_sel(fe_mul(b_val, inv), one))), s_eq));
    }
    const fe p264 = fe{0, 1};
    if (use_mulwide)
      A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(MULWIDE), fe_sub_sel(fe_mul(a_val, b_val), fe_add_sel(d0n, fe_mul(d1n, p264))))), s_eq));
    if (use_div128) {
      fe num128 = fe_add_sel(fe_mul(a_val, p264), imm);
      A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(DIV128), fe_sub_sel(num128, fe_add_sel(fe_mul(b_val, d0n), d1n)))), s_eq));
      A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(DIV128), fe_sub_sel(fe_mul(b_val, inv), one))), s_eq));
    }
    if (use_assert)
      A.emit(fe_add_sel(fe_mul(p_final, fe_add_sel(fe_mul(bo(ASSERT), fe_sub_sel(c_val, one)), fe_mul(bo(SEL), fe_mul(c_val, fe_sub_sel(c_val, one))))), s_eq));
    if (use_abit) A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(ABIT), fe_mul(c_val, fe_sub_sel(c_val, one)))), s_eq));
    if (use_arange) {
      for (int k = 0; k < 32; k++) {
        fe bi = cur(C.gadget_b + k);
        A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(ARANGE), fe_mul(bi, fe_sub_sel(bi, one)))), s_eq));
      }
      const fe p232 = fe{1ull << 32, 0};
      fe eq32 = fe_sub_sel(c_val, bsum);
      fe eq64 = fe_sub_sel(c_val, fe_add_sel(d0c, fe_mul(bsum, p232)));
      fe eqt = fe_mul(imm, fe_add_sel(fe_mul(mode64, eq64), fe_mul(fe_sub_sel(one, mode64), eq32)));
      A.emit(fe_add_sel(fe_mul(p_final, fe_mul(bo(ARANGE), eqt)), s_eq));
    }
  }
  if (RM && c_air.ram_block) {
    // ---------------- RamAir (ram.rs:82-236)
    const fe g_hold = fe_sub_sel(p_pad, p_pad_last);
    const fe op_load = cur(C.op[15]), op_store = cur(C.op[16]);
    const fe event = fe_mul(p_final, fe_add_sel(op_load, op_store));
    const fe r1 = c_air.ram_r[0], r2 = c_air.ram_r[1], r3 = c_air.ram_r[2];
    fe a_ev = fe_zero(), b_ev = fe_zero();
    for (int r = 0; r < 8; r++) {
      const fe rc = cur(C.r_start + r);
      a_ev = fe_add_sel(a_ev, fe_mul(cur(C.sel_a + r), rc));
      b_ev = fe_add_sel(b_ev, fe_mul(cur(C.sel_b + r), rc));
    }
    const fe val_ev = fe_add_sel(fe_mul(op_store, b_ev), fe_mul(fe_sub_sel(one, op_store), cur(C.imm)));
    const fe comp_uns =
        fe_add_sel(fe_add_sel(fe_add_sel(a_ev, fe_mul(r1, cur(C.pc))), fe_mul(r2, val_ev)), fe_mul(r3, op_store));
    const fe gu = cur(C.ram_gp_unsorted), du = fe_sub_sel(nxt(C.ram_gp_unsorted), gu);
    A.emit(fe_add_sel(fe_add_sel(fe_mul(event, fe_sub_sel(du, comp_uns)), fe_mul(fe_sub_sel(one, event), du)),
                      fe_mul(g_hold, du)));
    const fe s_on = cur(C.ram_sorted), s_addr = cur(C.ram_s_addr), s_clk = cur(C.ram_s_clk), s_val = cur(C.ram_s_val),
             s_w = cur(C.ram_s_is_write), lastw = cur(C.ram_s_last_write);
    const fe same = fe_sub_sel(one, fe_mul(fe_sub_sel(nxt(C.ram_s_addr), s_addr), cur(C.eq_inv)));
    const fe comp = fe_add_sel(fe_add_sel(fe_add_sel(s_addr, fe_mul(r1, s_clk)), fe_mul(r2, s_val)), fe_mul(r3, s_w));
    const fe gs = cur(C.ram_gp_sorted), ds = fe_sub_sel(nxt(C.ram_gp_sorted), gs);
    A.emit(fe_add_sel(fe_mul(s_on, fe_sub_sel(ds, comp)), fe_mul(fe_sub_sel(one, s_on), ds)));
    const fe sw_val = fe_mul(s_w, s_val);
    const fe keep = fe_add_sel(fe_mul(same, fe_add_sel(fe_mul(fe_sub_sel(one, s_w), lastw), sw_val)),
                               fe_mul(fe_sub_sel(one, same), sw_val));
    A.emit(fe_mul(s_on, fe_sub_sel(nxt(C.ram_s_last_write), keep)));
    A.emit(fe_mul(fe_mul(s_on, fe_sub_sel(one, s_w)), fe_sub_sel(s_val, lastw)));
    const fe s_on_n = nxt(C.ram_sorted);
    const fe on2 = fe_mul(s_on, s_on_n);
    A.emit(fe_mul(fe_mul(fe_mul(on2, fe_sub_sel(one, same)), fe_sub_sel(one, nxt(C.ram_s_is_write))), nxt(C.ram_s_val)));
    A.emit(fe_mul(s_on, fe_mul(same, fe_sub_sel(same, one))));
    if (c_air.ram_dclk) {
      const fe g_same = fe_mul(s_on, same);
      const uint32_t bits = c_air.ram_dclk_bits;
      fe sum = fe_zero(), pow2 = one;
      for (int k = 0; k < 32; k++) {
        const fe bk = cur(C.gadget_b + k);
        if ((bits >> k) & 1u) A.emit(fe_mul(g_same, fe_mul(bk, fe_sub_sel(bk, one))));
        sum = fe_add_sel(sum, fe_mul(pow2, bk));
        pow2 = fe_add_sel(pow2, pow2);
      }
      A.emit(fe_mul(fe_mul(on2, same), fe_sub_sel(fe_sub_sel(nxt(C.ram_s_clk), s_clk), sum)));
    }
    A.emit(fe_mul(p_last, fe_sub_sel(gu, gs)));
  }
  if (RM && c_air.merkle_block) {
    // ---------------- MerkleAir (merkle.rs:60-134)
    const fe g = cur(C.merkle_g), dir = cur(C.merkle_dir), acc = cur(C.merkle_acc), sib = cur(C.merkle_sib);
    const fe pg = fe_mul(p_map, g);
    const fe ndir = fe_sub_sel(one, dir);
    A.emit(fe_mul(pg, fe_mul(dir, fe_sub_sel(dir, one))));
    A.emit(fe_mul(pg, fe_sub_sel(cur(C.lanes_start), fe_add_sel(fe_mul(ndir, acc), fe_mul(dir, sib)))));
    A.emit(fe_mul(pg, fe_sub_sel(cur(C.lanes_start + 1), fe_add_sel(fe_mul(ndir, sib), fe_mul(dir, acc)))));
    const fe acc_n = nxt(C.merkle_acc);
    A.emit(fe_mul(fe_mul(g, g_carry), fe_sub_sel(acc_n, acc)));
    A.emit(fe_mul(fe_mul(pg, cur(C.merkle_first)), fe_sub_sel(acc, cur(C.merkle_leaf))));
    A.emit(fe_mul(fe_mul(fe_mul(p_final, g), cur(C.merkle_last)), fe_sub_sel(acc, c_air.merkle_root)));
    A.emit(fe_mul(fe_mul(fe_mul(p_pad_last, g), nxt(C.merkle_g)), fe_sub_sel(acc_n, acc)));
  }
  // ---------------- RomAir (rom.rs:57-120)
  if (c_air.commit_nonzero) {
    fe s3[3];
#pragma unroll
    for (int k = 0; k < 3; k++) s3[k] = fe_cube(cur(C.rom_s + k));
    fe ms[3];
#pragma unroll
    for (int k = 0; k < 3; k++)
      ms[k] = fe_add_sel(fe_add_sel(fe_mul(c_air.rom_mds[k][0], s3[0]), fe_mul(c_air.rom_mds[k][1], s3[1])),
                     fe_mul(c_air.rom_mds[k][2], s3[2]));
    fe sn[3] = {nxt(C.rom_s), nxt(C.rom_s + 1), nxt(C.rom_s + 2)};
    for (int j = 0; j < 27; j++) {
      fe gr = per[1 + j];
#pragma unroll
      for (int k = 0; k < 3; k++) A.emit(fe_mul(gr, fe_sub_sel(sn[k], fe_add_sel(ms[k], c_air.rom_rc[j][k]))));
    }
    fe g_hold = fe_sub_sel(p_pad, p_pad_last);
#pragma unroll
    for (int k = 0; k < 3; k++) A.emit(fe_mul(g_hold, fe_sub_sel(sn[k], cur(C.rom_s + k))));
    if (!fe_is_zero(p_map)) {
      uint32_t e0[9] = {0}, e1[9] = {0};
      int w = 0;
#pragma unroll
      for (int k = 0; k < 17; k++, w++) {
        fe v = cur(C.op[k]);
        mul_acc(v, c_air.rom_w0[w], e0);
        mul_acc(v, c_air.rom_w1[w], e1);
      }
      const int starts[5] = {C.sel_dst0, C.sel_a, C.sel_b, C.sel_c, C.sel_dst1};
#pragma unroll
      for (int s5 = 0; s5 < 5; s5++)
#pragma unroll
        for (int r = 0; r < 8; r++, w++) {
          fe v = cur(starts[s5] + r);
          mul_acc(v, c_air.rom_w0[w], e0);
          mul_acc(v, c_air.rom_w1[w], e1);
        }
      A.emit(fe_mul(p_map, fe_sub_sel(cur(C.rom_s + 1), reduce288(e0))));
      A.emit(fe_mul(p_map, fe_sub_sel(cur(C.rom_s + 2), reduce288(e1))));
    } else {
      A.ix += 2;
    }
  }
  return reduce288(A.a);
}

}  // namespace zkl
