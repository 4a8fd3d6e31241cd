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

// Constraints that share a factor f and an addend s, c_i = f X_i + s, are summed as
// f (sum_i alpha_i X_i) + s (sum_i alpha_i): one product by f and one by s per group instead of one
// product by f per constraint (the same field element, so the same composition values).  A group's
// alphas are consecutive index ranges; their sum comes from the per-proof prefix sums of the alphas
// (apre[i] = alpha_0 + .. + alpha_(i-1), DerivedConsts::apre), or is added up here (host verifier).
// CE_BRANCHFREE_CFG: the evaluator's additions and subtractions in the branch-free form (fe_add /
// fe_sub) instead of the branching one (fe_add_sel / fe_sub_sel, cheaper when a wave's operands
// rarely wrap).  At LDE points the trace values are uniformly distributed, so the branching form's
// wrap branch diverges in most waves.  Both give the canonical sum.
#ifndef CE_BRANCHFREE_CFG
#define CE_BRANCHFREE_CFG 0
#endif
#if CE_BRANCHFREE_CFG
#define AE_ADD fe_add
#define AE_SUB fe_sub
#else
#define AE_ADD fe_add_sel
#define AE_SUB fe_sub_sel
#endif
#ifndef CE_DOT_CFG
#define CE_DOT_CFG 0
#endif
// CE_GROUPS_CFG: which groups are formed (A/B; 0 = one product per constraint): 1 VmCtrlAir
// p_map / s_high, 2 g_carry / s_low, 4 p_final / s_write, 8 p_final / s_eq, 16 RomAir rounds
#ifndef CE_GROUPS_CFG
#define CE_GROUPS_CFG 31
#endif
struct AirGroup {
  uint32_t x[9];
  fe asum;
  int start;
  __host__ __device__ __forceinline__ AirGroup() : asum(fe{0, 0}), start(0) {
#pragma unroll
    for (int k = 0; k < 9; k++) x[k] = 0;
  }
};

struct AirAcc {
  uint32_t a[9];
  int ix;
  const fe* al;
  const fe* apre;  // alpha prefix sums, or nullptr
  __host__ __device__ __forceinline__ void emit(fe v) { mul_acc(al[ix++], v, a); }
  __host__ __device__ __forceinline__ fe alpha_range(int b, int e) const {
    if (apre) return fe_sub(apre[e], apre[b]);
    fe t = fe{0, 0};
    for (int i = b; i < e; i++) t = fe_add(t, al[i]);
    return t;
  }
  // a run of constraints f X + s of group G starts / ends at the current alpha index
  __host__ __device__ __forceinline__ void open(AirGroup& G) const { G.start = ix; }
  __host__ __device__ __forceinline__ void close(AirGroup& G) const { G.asum = fe_add(G.asum, alpha_range(G.start, ix)); }
  __host__ __device__ __forceinline__ void emit_g(AirGroup& G, fe X) { mul_acc(al[ix++], X, G.x); }
  __host__ __device__ __forceinline__ void emit_g0(AirGroup&) { ix++; }  // X = 0: the constraint is s
  __host__ __device__ __forceinline__ void flush(const AirGroup& G, fe f, fe s) {
    add_acc(fe_mul(f, reduce288(G.x)), a);
    add_acc(fe_mul(s, G.asum), a);
  }
};

// pose_k: K_j = sum_i alpha_{12j+i} rc[j][i] for the 27 Poseidon rounds (pose_k_kernel, once per
// proof), or nullptr to form them here (host verifier).
// PART: 0 = the whole sum; 1 = the PoseidonAir block alone; 2 = everything after it (its alphas
// skipped).  Parts 1 + 2 = part 0: the device evaluates the Poseidon block in a kernel of its own,
// whose register footprint does not add to the rest's.
constexpr int pose_block_constraints(const AirDevice& a) { return 27 * 12 + 12 + (a.pose_bind ? 10 : 0); }
template <bool POSE, bool RM, int PART = 0, class Cur, class Nxt>
__host__ __device__ __forceinline__ fe air_transition_sum(const AirDevice& c_air, Cur cur, Nxt nxt, const fe* per,
                                                          fe p_last, const fe* alpha, const fe* pose_k = nullptr,
                                                          const fe* apre = nullptr) {
  const Layout& C = c_air.cols;
  fe p_map = per[0], p_final = per[28], p_pad = per[29], p_pad_last = per[30];
  fe s_low = fe_mul(p_last, p_map);
  fe g_carry = AE_ADD(p_map, AE_SUB(p_pad, p_pad_last));
  for (int j = 0; j < 26; j++) g_carry = AE_ADD(g_carry, per[1 + j]);
  const fe rom_on = c_air.commit_nonzero ? fe_one() : fe_zero();
  const uint32_t m = c_air.vm_usage_mask;

  AirAcc A;
#pragma unroll
  for (int k = 0; k < 9; k++) A.a[k] = 0;
  A.ix = 0;
  A.al = alpha;
  A.apre = apre;
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
    const fe g_hold = AE_SUB(p_pad, p_pad_last);
    for (int i = 0; i < 12; i++) A.emit(fe_mul(g_hold, fe_sub(nxt(C.lanes_start + i), cur(C.lanes_start + i))));
    if (c_air.pose_bind) {
      const fe gate = fe_mul(fe_mul(p_map, pa), cur(C.op[8]));
      fe rr[8];
#pragma unroll
      for (int i = 0; i < 8; i++) rr[i] = cur(C.r_start + i);
      for (int lane = 0; lane < 10; lane++) {
        const fe b0 = cur(C.sel_s_bits + lane * 3), b1 = cur(C.sel_s_bits + lane * 3 + 1),
                 b2 = cur(C.sel_s_bits + lane * 3 + 2), act = cur(C.sel_s_active + lane);
        const fe nb0 = AE_SUB(one, b0), nb1 = AE_SUB(one, b1), nb2 = AE_SUB(one, b2);
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
    // every VmCtrlAir constraint of the form p_map X + s_high (the selector / op bits and their
    // one-hot sums, the ROM op binding) goes through this group
    AirGroup gh;
    A.open(gh);
    fe sum_d0 = fe_zero(), sum_a = fe_zero(), sum_b = fe_zero(), sum_c = fe_zero(), sum_d1 = fe_zero();
    for (int r = 0; r < 8; r++) {
      const fe v0 = cur(C.sel_dst0 + r), v1 = cur(C.sel_a + r), v2 = cur(C.sel_b + r), v3 = cur(C.sel_c + r),
               v4 = cur(C.sel_dst1 + r);
      sum_d0 = AE_ADD(sum_d0, v0); sum_a = AE_ADD(sum_a, v1); sum_b = AE_ADD(sum_b, v2);
      sum_c = AE_ADD(sum_c, v3); sum_d1 = AE_ADD(sum_d1, v4);
      auto bit = [&](fe v) {
        if (CE_GROUPS_CFG & 1) A.emit_g(gh, fe_mul(v, AE_SUB(v, one)));
        else A.emit(AE_ADD(fe_mul(p_map, fe_mul(v, AE_SUB(v, one))), s_high));
      };
      bit(v0); bit(v1); bit(v2); bit(v3); bit(v4);
    }
    // op bits read through cur() wherever used: a local fe[17] indexed in the loops below was
    // placed in scratch (288 B per lane)
    auto bo = [&](int k) { return cur(C.op[k]); };
    enum { CONST, MOV, ADD, SUB, MUL, NEG, EQ, SEL, SPONGE, ASSERT, ABIT, ARANGE, DIVMOD, DIV128, MULWIDE, LOAD, STORE };
    fe uses_a = AE_ADD(AE_ADD(AE_ADD(bo(MOV), bo(ADD)), AE_ADD(bo(SUB), bo(MUL))), AE_ADD(AE_ADD(bo(NEG), bo(EQ)), bo(SEL)));
    uses_a = AE_ADD(uses_a, AE_ADD(AE_ADD(bo(DIVMOD), bo(DIV128)), AE_ADD(AE_ADD(bo(MULWIDE), bo(LOAD)), bo(STORE))));
    fe uses_b = AE_ADD(AE_ADD(AE_ADD(bo(ADD), bo(SUB)), AE_ADD(bo(MUL), bo(EQ))), AE_ADD(bo(SEL), bo(DIVMOD)));
    uses_b = AE_ADD(uses_b, AE_ADD(AE_ADD(bo(DIV128), bo(MULWIDE)), bo(STORE)));
    fe uses_c = AE_ADD(AE_ADD(bo(SEL), bo(ASSERT)), AE_ADD(bo(ABIT), bo(ARANGE)));
    fe op_any = fe_zero();
#pragma unroll
    for (int k = 0; k <= MULWIDE; k++) op_any = AE_ADD(op_any, bo(k));
    fe uses_d0 = AE_ADD(AE_SUB(op_any, bo(SPONGE)), bo(LOAD));
    fe uses_d1 = AE_ADD(AE_ADD(bo(DIVMOD), bo(DIV128)), bo(MULWIDE));
    A.close(gh);
    A.emit(AE_ADD(fe_mul(p_map, AE_SUB(sum_d0, uses_d0)), s_low));
    A.emit(AE_ADD(fe_mul(p_map, AE_SUB(sum_a, uses_a)), s_low));
    A.emit(AE_ADD(fe_mul(p_map, AE_SUB(sum_b, uses_b)), s_low));
    A.emit(AE_ADD(fe_mul(p_map, AE_SUB(sum_c, uses_c)), s_low));
    A.emit(AE_ADD(fe_mul(p_map, AE_SUB(sum_d1, uses_d1)), s_low));
    if (CE_GROUPS_CFG & 1) {
    A.open(gh);
    for (int r = 0; r < 8; r++) A.emit_g(gh, fe_mul(cur(C.sel_dst0 + r), cur(C.sel_dst1 + r)));
    if (c_air.sponge_block) {
      for (int lane = 0; lane < 10; lane++) {
        for (int bit = 0; bit < 3; bit++) {
          fe v = cur(C.sel_s_bits + lane * 3 + bit);
          A.emit_g(gh, fe_mul(v, AE_SUB(v, one)));
        }
        fe a = cur(C.sel_s_active + lane);
        A.emit_g(gh, fe_mul(a, AE_SUB(a, one)));
      }
    }
    A.emit_g0(gh);
    fe op_sum = fe_zero();
#pragma unroll
    for (int k = 0; k < 17; k++) {
      A.emit_g(gh, fe_mul(bo(k), AE_SUB(bo(k), one)));
      op_sum = AE_ADD(op_sum, bo(k));
    }
    A.emit_g(gh, fe_mul(op_sum, AE_SUB(op_sum, one)));
    // rom_on (0 or 1) * p_map * (b_k - rom_op_k) + s_high: with rom_on = 0 only s_high remains
#pragma unroll
    for (int k = 0; k < 17; k++) {
      if (c_air.commit_nonzero)
        A.emit_g(gh, AE_SUB(bo(k), cur(C.rom_op_start + k)));
      else
        A.emit_g0(gh);
    }
    A.close(gh);
    A.flush(gh, p_map, s_high);
    } else {
    for (int r = 0; r < 8; r++)
      A.emit(AE_ADD(fe_mul(p_map, fe_mul(cur(C.sel_dst0 + r), cur(C.sel_dst1 + r))), s_high));
    if (c_air.sponge_block) {
      for (int lane = 0; lane < 10; lane++) {
        for (int bit = 0; bit < 3; bit++) {
          fe v = cur(C.sel_s_bits + lane * 3 + bit);
          A.emit(AE_ADD(fe_mul(p_map, fe_mul(v, AE_SUB(v, one))), s_high));
        }
        fe a = cur(C.sel_s_active + lane);
        A.emit(AE_ADD(fe_mul(p_map, fe_mul(a, AE_SUB(a, one))), s_high));
      }
    }
    A.emit(s_high);
    fe op_sum = fe_zero();
#pragma unroll
    for (int k = 0; k < 17; k++) {
      A.emit(AE_ADD(fe_mul(p_map, fe_mul(bo(k), AE_SUB(bo(k), one))), s_high));
      op_sum = AE_ADD(op_sum, bo(k));
    }
    A.emit(AE_ADD(fe_mul(p_map, fe_mul(op_sum, AE_SUB(op_sum, one))), s_high));
#pragma unroll
    for (int k = 0; k < 17; k++)
      A.emit(AE_ADD(fe_mul(rom_on, fe_mul(p_map, AE_SUB(bo(k), cur(C.rom_op_start + k)))), s_high));
    }
    fe pc_c = cur(C.pc), pc_n = nxt(C.pc);
    A.emit(AE_ADD(fe_mul(rom_on, fe_mul(g_carry, AE_SUB(pc_n, pc_c))), s_low));
    A.emit(AE_ADD(fe_mul(rom_on, fe_mul(p_pad_last, AE_SUB(pc_n, AE_ADD(pc_c, one)))), s_low));

    // ---------------- VmAluAir (alu.rs:108-354)
    const bool use_eq = m & (1u << 6), use_divmod = m & (1u << 3), use_mulwide = m & (1u << 4),
               use_div128 = m & (1u << 5), use_assert = m & 1u, use_abit = m & 2u, use_arange = m & 4u;
    fe pi2 = fe_sqr(pi), pi4 = fe_sqr(pi2), pi6 = fe_mul(pi4, pi2);
    fe s_write = fe_mul(s_low, pi6), s_eq = fe_mul(s_low, pi4);
    // the selected operands are dot products of selector and register columns.  CE_DOT_CFG = 1
    // forms them as lazy 288-bit sums with one reduction each, two at a time: 0.5% faster on the
    // headline evaluator but it reads the register columns three times (PMC fetch 3.16 -> 3.80 GB
    // per launch, profiles/r06/final), so the default keeps one pass of reduced products.
    fe a_val, b_val, c_val, d0n, d0c, d1n;
    if (CE_DOT_CFG) {
      auto dot2 = [&](int sx, int sy, bool nx, bool ny, fe& vx, fe& vy) {
        uint32_t ax[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, ay[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int r = 0; r < 8; r++) {
          mul_acc(cur(sx + r), nx ? nxt(C.r_start + r) : cur(C.r_start + r), ax);
          mul_acc(cur(sy + r), ny ? nxt(C.r_start + r) : cur(C.r_start + r), ay);
        }
        vx = reduce288(ax);
        vy = reduce288(ay);
      };
      dot2(C.sel_a, C.sel_b, false, false, a_val, b_val);
      dot2(C.sel_c, C.sel_dst0, false, true, c_val, d0n);
      dot2(C.sel_dst0, C.sel_dst1, false, true, d0c, d1n);
    } else {
      a_val = fe_zero(), b_val = fe_zero(), c_val = fe_zero(), d0n = fe_zero(), d0c = fe_zero(), d1n = fe_zero();
      for (int r = 0; r < 8; r++) {
        fe rc = cur(C.r_start + r), rn = nxt(C.r_start + r);
        a_val = AE_ADD(a_val, fe_mul(cur(C.sel_a + r), rc));
        b_val = AE_ADD(b_val, fe_mul(cur(C.sel_b + r), rc));
        c_val = AE_ADD(c_val, fe_mul(cur(C.sel_c + r), rc));
        fe sd0 = cur(C.sel_dst0 + r);
        d0n = AE_ADD(d0n, fe_mul(sd0, rn));
        d0c = AE_ADD(d0c, fe_mul(sd0, rc));
        d1n = AE_ADD(d1n, fe_mul(cur(C.sel_dst1 + r), rn));
      }
    }
    if (CE_GROUPS_CFG & 2) {
      AirGroup gc;  // g_carry (r' - r) + s_low
      A.open(gc);
      for (int r = 0; r < 8; r++) A.emit_g(gc, AE_SUB(nxt(C.r_start + r), cur(C.r_start + r)));
      A.close(gc);
      A.flush(gc, g_carry, s_low);
    } else {
      for (int r = 0; r < 8; r++)
        A.emit(AE_ADD(fe_mul(g_carry, AE_SUB(nxt(C.r_start + r), cur(C.r_start + r))), s_low));
    }
    fe imm = cur(C.imm);
    fe mode64 = cur(C.eq_inv);
    fe res = fe_mul(bo(CONST), imm);
    res = AE_ADD(res, fe_mul(bo(MOV), a_val));
    res = AE_ADD(res, fe_mul(bo(ADD), AE_ADD(a_val, b_val)));
    res = AE_ADD(res, fe_mul(bo(SUB), AE_SUB(a_val, b_val)));
    res = AE_ADD(res, fe_mul(bo(MUL), fe_mul(a_val, b_val)));
    res = AE_ADD(res, fe_mul(bo(NEG), fe_neg(a_val)));
    res = AE_ADD(res, fe_mul(bo(SEL), AE_ADD(fe_mul(c_val, a_val), fe_mul(AE_SUB(one, c_val), b_val))));
    res = AE_ADD(res, fe_mul(bo(SPONGE), cur(C.lanes_start)));
    if (use_eq) res = AE_ADD(res, fe_mul(bo(EQ), d0n));
    if (use_assert) res = AE_ADD(res, bo(ASSERT));
    if (use_abit) res = AE_ADD(res, bo(ABIT));
    res = AE_ADD(res, fe_mul(bo(LOAD), imm));
    fe bsum = fe_zero();
    if (use_arange) {
      fe pow2 = one;
      // sum_k 2^k b_k by Horner's rule: doublings and additions, no products
      for (int k = 31; k >= 0; k--) bsum = AE_ADD(AE_ADD(bsum, bsum), cur(C.gadget_b + k));
      (void)pow2;
      res = AE_ADD(res, fe_mul(bo(ARANGE), AE_ADD(fe_mul(AE_SUB(one, imm), bsum), imm)));
    }
    bool uses_two = use_divmod || use_mulwide || use_div128;
    fe b_two = uses_two ? AE_ADD(AE_ADD(bo(DIVMOD), bo(MULWIDE)), bo(DIV128)) : fe_zero();
    fe w0 = AE_ADD(fe_mul(AE_SUB(one, b_two), res), fe_mul(b_two, d0n));
    fe w1 = fe_mul(b_two, d1n);
    {
      AirGroup gw;  // p_final (r' - rhs) + s_write
      A.open(gw);
      for (int r = 0; r < 8; r++) {
        fe sd0 = cur(C.sel_dst0 + r), sd1 = cur(C.sel_dst1 + r);
        fe keep = AE_SUB(AE_SUB(one, sd0), sd1);
        fe rhs = AE_ADD(AE_ADD(fe_mul(keep, cur(C.r_start + r)), fe_mul(sd0, w0)), fe_mul(sd1, w1));
        if (CE_GROUPS_CFG & 4) A.emit_g(gw, AE_SUB(nxt(C.r_start + r), rhs));
        else A.emit(AE_ADD(fe_mul(p_final, AE_SUB(nxt(C.r_start + r), rhs)), s_write));
      }
      if (CE_GROUPS_CFG & 4) {
        A.close(gw);
        A.flush(gw, p_final, s_write);
      }
    }
    fe diff = AE_SUB(a_val, b_val);
    fe inv = cur(C.eq_inv);
    AirGroup ge;  // p_final X + s_eq: the ALU checks below
    A.open(ge);
#define CE_EQ(X) do { if (CE_GROUPS_CFG & 8) A.emit_g(ge, (X)); else A.emit(AE_ADD(fe_mul(p_final, (X)), s_eq)); } while (0)
    if (use_eq) {
      CE_EQ(fe_mul(bo(EQ), fe_mul(d0n, diff)));
      CE_EQ(fe_mul(bo(EQ), AE_SUB(AE_SUB(one, d0n), fe_mul(diff, inv))));
    }
    if (use_divmod) {
      CE_EQ(fe_mul(bo(DIVMOD), AE_SUB(AE_SUB(a_val, fe_mul(b_val, d0n)), d1n)));
      CE_EQ(fe_mul(bo(DIVMOD), AE_SUB(fe_mul(b_val, inv), one)));
    }
    const fe p264 = fe{0, 1};
    if (use_mulwide)
      CE_EQ(fe_mul(bo(MULWIDE), AE_SUB(fe_mul(a_val, b_val), AE_ADD(d0n, fe_mul(d1n, p264)))));
    if (use_div128) {
      fe num128 = AE_ADD(fe_mul(a_val, p264), imm);
      CE_EQ(fe_mul(bo(DIV128), AE_SUB(num128, AE_ADD(fe_mul(b_val, d0n), d1n))));
      CE_EQ(fe_mul(bo(DIV128), AE_SUB(fe_mul(b_val, inv), one)));
    }
    if (use_assert)
      CE_EQ(AE_ADD(fe_mul(bo(ASSERT), AE_SUB(c_val, one)), fe_mul(bo(SEL), fe_mul(c_val, AE_SUB(c_val, one)))));
    if (use_abit) CE_EQ(fe_mul(bo(ABIT), fe_mul(c_val, AE_SUB(c_val, one))));
    if (use_arange) {
      for (int k = 0; k < 32; k++) {
        fe bi = cur(C.gadget_b + k);
        CE_EQ(fe_mul(bo(ARANGE), fe_mul(bi, AE_SUB(bi, one))));
      }
      const fe p232 = fe{1ull << 32, 0};
      fe eq32 = AE_SUB(c_val, bsum);
      fe eq64 = AE_SUB(c_val, AE_ADD(d0c, fe_mul(bsum, p232)));
      fe eqt = fe_mul(imm, AE_ADD(fe_mul(mode64, eq64), fe_mul(AE_SUB(one, mode64), eq32)));
      CE_EQ(fe_mul(bo(ARANGE), eqt));
    }
    if (CE_GROUPS_CFG & 8) {
      A.close(ge);
      A.flush(ge, p_final, s_eq);
    }
#undef CE_EQ
  }
  if (RM && c_air.ram_block) {
    // ---------------- RamAir (ram.rs:82-236)
    const fe g_hold = AE_SUB(p_pad, p_pad_last);
    const fe op_load = cur(C.op[15]), op_store = cur(C.op[16]);
    const fe event = fe_mul(p_final, AE_ADD(op_load, op_store));
    const fe r1 = c_air.ram_r[0], r2 = c_air.ram_r[1], r3 = c_air.ram_r[2];
    fe a_ev = fe_zero(), b_ev = fe_zero();
    for (int r = 0; r < 8; r++) {
      const fe rc = cur(C.r_start + r);
      a_ev = AE_ADD(a_ev, fe_mul(cur(C.sel_a + r), rc));
      b_ev = AE_ADD(b_ev, fe_mul(cur(C.sel_b + r), rc));
    }
    const fe val_ev = AE_ADD(fe_mul(op_store, b_ev), fe_mul(AE_SUB(one, op_store), cur(C.imm)));
    const fe comp_uns =
        AE_ADD(AE_ADD(AE_ADD(a_ev, fe_mul(r1, cur(C.pc))), fe_mul(r2, val_ev)), fe_mul(r3, op_store));
    const fe gu = cur(C.ram_gp_unsorted), du = AE_SUB(nxt(C.ram_gp_unsorted), gu);
    A.emit(AE_ADD(AE_ADD(fe_mul(event, AE_SUB(du, comp_uns)), fe_mul(AE_SUB(one, event), du)),
                      fe_mul(g_hold, du)));
    const fe s_on = cur(C.ram_sorted), s_addr = cur(C.ram_s_addr), s_clk = cur(C.ram_s_clk), s_val = cur(C.ram_s_val),
             s_w = cur(C.ram_s_is_write), lastw = cur(C.ram_s_last_write);
    const fe same = AE_SUB(one, fe_mul(AE_SUB(nxt(C.ram_s_addr), s_addr), cur(C.eq_inv)));
    const fe comp = AE_ADD(AE_ADD(AE_ADD(s_addr, fe_mul(r1, s_clk)), fe_mul(r2, s_val)), fe_mul(r3, s_w));
    const fe gs = cur(C.ram_gp_sorted), ds = AE_SUB(nxt(C.ram_gp_sorted), gs);
    A.emit(AE_ADD(fe_mul(s_on, AE_SUB(ds, comp)), fe_mul(AE_SUB(one, s_on), ds)));
    const fe sw_val = fe_mul(s_w, s_val);
    const fe keep = AE_ADD(fe_mul(same, AE_ADD(fe_mul(AE_SUB(one, s_w), lastw), sw_val)),
                               fe_mul(AE_SUB(one, same), sw_val));
    A.emit(fe_mul(s_on, AE_SUB(nxt(C.ram_s_last_write), keep)));
    A.emit(fe_mul(fe_mul(s_on, AE_SUB(one, s_w)), AE_SUB(s_val, lastw)));
    const fe s_on_n = nxt(C.ram_sorted);
    const fe on2 = fe_mul(s_on, s_on_n);
    A.emit(fe_mul(fe_mul(fe_mul(on2, AE_SUB(one, same)), AE_SUB(one, nxt(C.ram_s_is_write))), nxt(C.ram_s_val)));
    A.emit(fe_mul(s_on, fe_mul(same, AE_SUB(same, one))));
    if (c_air.ram_dclk) {
      const fe g_same = fe_mul(s_on, same);
      const uint32_t bits = c_air.ram_dclk_bits;
      // the bit checks g_same b_k (b_k - 1) share g_same: one lazy dot product, one product
      uint32_t gacc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (int k = 0; k < 32; k++) {
        const fe bk = cur(C.gadget_b + k);
        if ((bits >> k) & 1u) mul_acc(A.al[A.ix++], fe_mul(bk, AE_SUB(bk, one)), gacc);
      }
      add_acc(fe_mul(g_same, reduce288(gacc)), A.a);
      fe sum = fe_zero();  // sum_k 2^k b_k by Horner's rule
      for (int k = 31; k >= 0; k--) sum = AE_ADD(AE_ADD(sum, sum), cur(C.gadget_b + k));
      A.emit(fe_mul(fe_mul(on2, same), AE_SUB(AE_SUB(nxt(C.ram_s_clk), s_clk), sum)));
    }
    A.emit(fe_mul(p_last, AE_SUB(gu, gs)));
  }
  if (RM && c_air.merkle_block) {
    // ---------------- MerkleAir (merkle.rs:60-134)
    const fe g = cur(C.merkle_g), dir = cur(C.merkle_dir), acc = cur(C.merkle_acc), sib = cur(C.merkle_sib);
    const fe pg = fe_mul(p_map, g);
    const fe ndir = AE_SUB(one, dir);
    A.emit(fe_mul(pg, fe_mul(dir, AE_SUB(dir, one))));
    A.emit(fe_mul(pg, AE_SUB(cur(C.lanes_start), AE_ADD(fe_mul(ndir, acc), fe_mul(dir, sib)))));
    A.emit(fe_mul(pg, AE_SUB(cur(C.lanes_start + 1), AE_ADD(fe_mul(ndir, sib), fe_mul(dir, acc)))));
    const fe acc_n = nxt(C.merkle_acc);
    A.emit(fe_mul(fe_mul(g, g_carry), AE_SUB(acc_n, acc)));
    A.emit(fe_mul(fe_mul(pg, cur(C.merkle_first)), AE_SUB(acc, cur(C.merkle_leaf))));
    A.emit(fe_mul(fe_mul(fe_mul(p_final, g), cur(C.merkle_last)), AE_SUB(acc, c_air.merkle_root)));
    A.emit(fe_mul(fe_mul(fe_mul(p_pad_last, g), nxt(C.merkle_g)), AE_SUB(acc_n, acc)));
  }
  // ---------------- RomAir (rom.rs:57-120)
  if (c_air.commit_nonzero) {
    fe s3[3];
#pragma unroll
    for (int k = 0; k < 3; k++) s3[k] = fe_cube(cur(C.rom_s + k));
    fe ms[3];
#pragma unroll
    for (int k = 0; k < 3; k++)
      ms[k] = AE_ADD(AE_ADD(fe_mul(c_air.rom_mds[k][0], s3[0]), fe_mul(c_air.rom_mds[k][1], s3[1])),
                     fe_mul(c_air.rom_mds[k][2], s3[2]));
    fe sn[3] = {nxt(C.rom_s), nxt(C.rom_s + 1), nxt(C.rom_s + 2)};
    if (CE_GROUPS_CFG & 16) {
    // round j's three constraints g_j (s'_k - ms_k - rc_jk) share g_j: one lazy dot product of
    // the alphas with (s'_k - ms_k - rc_jk) and one product by g_j per round
    fe d[3];
#pragma unroll
    for (int k = 0; k < 3; k++) d[k] = AE_SUB(sn[k], ms[k]);
    for (int j = 0; j < 27; j++) {
      uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 3; k++) mul_acc(A.al[A.ix++], fe_sub(d[k], c_air.rom_rc[j][k]), acc);
      add_acc(fe_mul(per[1 + j], reduce288(acc)), A.a);
    }
    fe g_hold = AE_SUB(p_pad, p_pad_last);
    {
      uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 3; k++) mul_acc(A.al[A.ix++], AE_SUB(sn[k], cur(C.rom_s + k)), acc);
      add_acc(fe_mul(g_hold, reduce288(acc)), A.a);
    }
    } else {
    for (int j = 0; j < 27; j++) {
      fe gr = per[1 + j];
#pragma unroll
      for (int k = 0; k < 3; k++) A.emit(fe_mul(gr, AE_SUB(sn[k], AE_ADD(ms[k], c_air.rom_rc[j][k]))));
    }
    fe g_hold = AE_SUB(p_pad, p_pad_last);
#pragma unroll
    for (int k = 0; k < 3; k++) A.emit(fe_mul(g_hold, AE_SUB(sn[k], cur(C.rom_s + k))));
    }
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
      A.emit(fe_mul(p_map, AE_SUB(cur(C.rom_s + 1), reduce288(e0))));
      A.emit(fe_mul(p_map, AE_SUB(cur(C.rom_s + 2), reduce288(e1))));
    } else {
      A.ix += 2;
    }
  }
  return reduce288(A.a);
}

}  // namespace zkl
