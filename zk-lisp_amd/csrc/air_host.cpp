// Host side of ZkLispAir (zk-lisp-proof-winterfell/src/vm/air/mod.rs and modules).
#include "air_host.h"

#include <string.h>

#include <algorithm>
#include <map>
#include <stdexcept>

#include "host_hash.h"

namespace zkl {

static constexpr int NR = 8;
static constexpr int ROUNDS = 27;
static constexpr int STEPS = 32;
enum { U_ASSERT = 0, U_ASSERT_BIT, U_ASSERT_RANGE, U_DIVMOD, U_MULWIDE, U_DIV128, U_EQ, U_SPONGE, U_RAM_DCLK };

fe fe_from(const zkl_f128& v) { return fe{v.lo, v.hi}; }
zkl_f128 to_abi(fe v) { return zkl_f128{v.lo, v.hi}; }

fe root_of_unity(unsigned k) {
  // TWO_ADIC_ROOT_OF_UNITY = 3^((p-1)/2^40); get_root_of_unity(k) = that^(2^(40-k))
  static fe g40 = [] {
    // (p-1) >> 40 = 2^88 - 45
    uint64_t e_lo = (0ull - 45ull), e_hi = (1ull << 24) - 1;  // 2^88 - 45
    return fe_pow(fe{3, 0}, e_lo, e_hi);
  }();
  fe g = g40;
  for (unsigned i = k; i < 40; i++) g = fe_sqr(g);
  return g;
}

Layout make_layout(bool vm, bool ram, bool sponge, bool merkle, bool rom) {
  (void)vm; (void)sponge;
  Layout c{};
  int cur = 12;
  c.lanes_start = 0;
  c.g_map = cur; c.g_final = cur + 1; c.g_r_start = cur + 2;
  cur = c.g_r_start + ROUNDS;
  c.mask = cur++;
  c.r_start = cur; cur += NR;
  for (int k = 0; k < 17; k++) c.op[k] = cur + k;
  cur += 17;
  c.sel_dst0 = cur; c.sel_a = cur + NR; c.sel_b = cur + 2 * NR; c.sel_c = cur + 3 * NR; c.sel_dst1 = cur + 4 * NR;
  cur += 5 * NR;
  c.sel_s_bits = cur; c.sel_s_active = cur + 30;
  cur += 40;
  c.imm = cur; c.eq_inv = cur + 1;
  cur += 2;
  c.ram_sorted = cur; c.ram_s_addr = cur + 1; c.ram_s_clk = cur + 2; c.ram_s_val = cur + 3;
  c.ram_s_is_write = cur + 4; c.ram_s_last_write = cur + 5; c.ram_gp_unsorted = cur + 6; c.ram_gp_sorted = cur + 7;
  if (ram) cur += 8;
  c.merkle_g = cur; c.merkle_dir = cur + 1; c.merkle_sib = cur + 2; c.merkle_acc = cur + 3;
  c.merkle_first = cur + 4; c.merkle_last = cur + 5; c.merkle_leaf = cur + 6;
  if (merkle) cur += 7;
  c.pi_prog = cur++;
  c.pc = cur++;
  c.rom_op_start = cur;
  if (rom) cur += 17;
  c.pose_active = cur++;
  c.gadget_b = cur;
  cur += 32;
  c.rom_s = cur;
  if (rom) cur += 3;
  c.width = rom ? cur : c.pc + 1;
  return c;
}

static void rom_weights(uint32_t seed, fe out[59]) {  // utils.rs:95-121
  fe cur = fe_mul(fe_pow64(fe{3, 0}, seed), fe{3, 0});
  for (int i = 0; i < 59; i++) { out[i] = cur; cur = fe_mul(cur, fe{3, 0}); }
}

// check_width false: the aggregation's child replay (agg/fs.rs:38-80), which rebuilds the AIR
// with segment_feature_mask 0 as the reference does: ZkLispAir::new then takes the layout of the
// program's mask for a narrow trace without comparing widths (vm/air/mod.rs:141-163); only the
// constraint degrees (composition column count) are used.
std::string build_air(const zkl_air_public_inputs& pi, uint32_t width, size_t n, AirInstance& A, bool check_width) {
  {  // a fresh instance on the vectors' capacity (a prover context rebuilds it every proof)
    std::vector<int> db = std::move(A.degree_base), dc = std::move(A.degree_cycle);
    std::vector<Assertion> as = std::move(A.assertions);
    A = AirInstance{};
    db.clear(); dc.clear(); as.clear();
    A.degree_base = std::move(db);
    A.degree_cycle = std::move(dc);
    A.assertions = std::move(as);
  }
  A.n = n;
  uint64_t eff = pi.segment_feature_mask ? pi.segment_feature_mask : pi.feature_mask;
  bool f_pose = eff & FM_POSEIDON, f_vm = eff & FM_VM, f_exp = eff & FM_VM_EXPECT, f_sponge = eff & FM_SPONGE,
       f_merkle = eff & FM_MERKLE, f_ram = eff & FM_RAM;
  bool pid_nz = false, com_nz = false;
  for (int i = 0; i < 32; i++) { pid_nz |= pi.program_id[i] != 0; com_nz |= pi.program_commitment[i] != 0; }
  Layout base = make_layout(true, true, true, true, true);
  Layout cols = (int)width < base.width ? make_layout(f_vm, f_ram, f_sponge, f_merkle, pid_nz)
                                        : make_layout(true, true, true, true, pid_nz);
  if (check_width && cols.width != (int)width) return "trace width does not match the layout implied by the feature mask";
  if (com_nz != pid_nz) return "program_id / program_commitment zero-ness differs (ROM block would be inconsistent)";

  AirDevice& d = A.dev;
  d.cols = cols;
  d.feat_vm = f_vm;
  d.commit_nonzero = com_nz;
  d.vm_usage_mask = pi.vm_usage_mask;
  uint32_t m = pi.vm_usage_mask;
  d.sponge_block = f_sponge && (m & (1u << U_SPONGE));
  derive_rom_constants(pi.program_id, d.rom_rc, d.rom_mds);
  rom_weights(17, d.rom_w0);
  rom_weights(1037, d.rom_w1);
  PoseidonSuite ps = derive_poseidon_suite(pi.program_id, 27);
  A.suite_dom[0] = ps.dom[0];
  A.suite_dom[1] = ps.dom[1];
  d.pose_block = f_pose;
  d.pose_bind = f_pose && f_vm && f_sponge && (m & (1u << U_SPONGE));
  for (int i = 0; i < 12; i++)
    for (int k = 0; k < 12; k++) d.pose_mds[i][k] = ps.mds[i][k];
  for (int r = 0; r < 27; r++)
    for (int i = 0; i < 12; i++) d.pose_rc[r][i] = ps.rc[r][i];
  d.ram_block = f_ram;
  d.ram_dclk = f_ram && (m & (1u << U_RAM_DCLK));
  d.ram_dclk_bits = pi.ram_delta_clk_bits;
  {
    fe pfe[2] = {fe_zero(), fe_zero()};
    if (pid_nz) program_field_commitment(pi.program_id, pfe);  // vm/air/mod.rs:184-188
    fe q0 = pfe[0], q2 = fe_mul(q0, q0), q3 = fe_mul(q2, q0), q5 = fe_mul(fe_mul(q2, q2), q0);
    d.ram_r[0] = fe_add(q2, fe_one());
    d.ram_r[1] = fe_add(q3, q0);
    d.ram_r[2] = fe_add(q5, fe{7, 0});
  }
  d.merkle_block = f_merkle;
  d.merkle_root = be_from_le16(pi.merkle_root);

  // degrees in module order: Poseidon, Ctrl, ALU (vm), RAM, Merkle, ROM (vm/air/mod.rs:217-238)
  auto& deg = A.degree_base;
  auto& cyc = A.degree_cycle;
  auto push = [&](int cnt, int b, int c = 1) {
    for (int i = 0; i < cnt; i++) { deg.push_back(b); cyc.push_back(c); }
  };
  if (f_pose) {  // PoseidonAir::push_degrees (poseidon.rs:26-62)
    push(27 * 12, 4);
    push(12, 1);
    if (d.pose_bind) { push(2, 6); push(8, 3); }
  }
  if (f_vm) {
    push(5 * NR, 2); push(5, 1); push(NR, 2);
    if (d.sponge_block) push(40, 2);
    push(1, 2); push(17, 2); push(1, 2); push(17, 2); push(2, 1);
    push(NR, 1); push(NR, 7);
    if (m & (1u << U_EQ)) push(2, 5);
    if (m & (1u << U_DIVMOD)) push(2, 5);
    if (m & (1u << U_ASSERT)) push(1, 5);
    if (m & (1u << U_ASSERT_BIT)) push(1, 5);
    if (m & (1u << U_ASSERT_RANGE)) push(33, 5);
    if (m & (1u << U_MULWIDE)) push(1, 5);
    if (m & (1u << U_DIV128)) push(2, 5);
  }
  if (f_ram) {  // RamAir::push_degrees (ram.rs:26-79): only the unsorted carry has the cycle
    push(1, 4); push(1, 2, 0); push(1, 5, 0); push(1, 3, 0); push(1, 6, 0); push(1, 5, 0);
    if (d.ram_dclk) { push(__builtin_popcount(pi.ram_delta_clk_bits), 5, 0); push(1, 5, 0); }
    push(1, 2, 0);
  }
  if (f_merkle) { push(3, 3); push(1, 2); push(3, 3); }  // MerkleAir (merkle.rs:26-58)
  if (pid_nz) { push(81, 3); push(3, 1); push(2, 1); }
  if (deg.empty()) return "AIR without transition constraints is not a VM segment";
  A.n_tc = d.n_tc = (int)deg.size();
  // ce_blowup = max (base + #cycles - 1).next_power_of_two(), min 2; eval degree
  // base (n-1) + #cycles (n/32) 31 (winter-air TransitionConstraintDegree)
  int ceb = 2;
  size_t max_eval = 0;
  for (size_t i = 0; i < deg.size(); i++) {
    int need = 1;
    while (need < deg[i] + cyc[i] - 1) need <<= 1;
    ceb = std::max(ceb, need);
    max_eval = std::max(max_eval, (size_t)deg[i] * (n - 1) + (cyc[i] ? (n / STEPS) * (STEPS - 1) : 0));
  }
  A.ce_blowup = ceb;
  A.num_comp_cols = (int)((max_eval - (n - 1) + n - 1) / n);

  // ---- assertions (ScheduleAir, VM PI, RomAir), dedup by (col, step), Winterfell order
  static thread_local std::vector<Assertion> raw;  // scratch kept by the thread (no per-proof heap churn)
  raw.clear();
  size_t last = n - 1, lvls = n / STEPS;
  if (pi.n_main_slots > ZKL_MAX_MAIN_SLOTS) return "n_main_slots exceeds ZKL_MAX_MAIN_SLOTS";
  fe pc_init = fe_from(pi.pc_init);
  for (size_t l = 0; l < lvls; l++) {
    uint32_t b = (uint32_t)(l * STEPS), rm = b, rf = b + 28;
    raw.push_back({(uint32_t)cols.lanes_start + 10, rm, ps.dom[0]});
    raw.push_back({(uint32_t)cols.lanes_start + 11, rm, ps.dom[1]});
    raw.push_back({(uint32_t)cols.g_map, rm, fe_one()});
    raw.push_back({(uint32_t)cols.g_final, rf, fe_one()});
    for (int j = 0; j < ROUNDS; j++) raw.push_back({(uint32_t)(cols.g_r_start + j), b + 1 + j, fe_one()});
    raw.push_back({(uint32_t)cols.g_final, rm, fe_zero()});
    for (int j = 0; j < ROUNDS; j++) raw.push_back({(uint32_t)(cols.g_r_start + j), rm, fe_zero()});
    raw.push_back({(uint32_t)cols.g_map, rf, fe_zero()});
    for (int j = 0; j < ROUNDS; j++) raw.push_back({(uint32_t)(cols.g_r_start + j), rf, fe_zero()});
    for (int j = 0; j < ROUNDS; j++) {
      raw.push_back({(uint32_t)cols.g_map, b + 1 + j, fe_zero()});
      raw.push_back({(uint32_t)cols.g_final, b + 1 + j, fe_zero()});
    }
    if (l == 0 && f_vm) {
      if (fe_is_zero(pc_init) && com_nz) raw.push_back({(uint32_t)cols.pi_prog, rm, be_from_le16(pi.program_commitment)});
      raw.push_back({(uint32_t)cols.pc, rm, pc_init});
    }
  }
  if (f_vm) {
    if (f_exp) {
      uint32_t row = (uint32_t)std::min<size_t>(pi.vm_out_row, last);
      int reg = std::min<int>((int)pi.vm_out_reg, NR - 1);
      raw.push_back({(uint32_t)(cols.r_start + reg), row, be_from_le16(pi.vm_expected_bytes)});
    }
    if (fe_is_zero(pc_init) && pi.n_main_slots > 0) {
      if (pi.n_main_slots > (uint32_t)NR) return "main_args must fit into NR registers";
      int s = (int)pi.n_main_slots;
      for (int j = 0; j < s; j++) raw.push_back({(uint32_t)(cols.r_start + NR - s + j), 0, fe_from(pi.main_slots[j])});
    }
  }
  if (com_nz) {
    for (int i = 0; i < 3; i++) raw.push_back({(uint32_t)(cols.rom_s + i), 0, fe_from(pi.rom_s_in[i])});
    for (int i = 0; i < 3; i++) raw.push_back({(uint32_t)(cols.rom_s + i), (uint32_t)last, fe_from(pi.rom_s_out[i])});
  }
  if (raw.empty()) raw.push_back({(uint32_t)cols.mask, (uint32_t)last, fe_zero()});
  // keep-first dedup by (col, step) then sort by (step, col) -- stable on the key
  static thread_local std::vector<size_t> idx;
  idx.resize(raw.size());
  for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
    if (raw[a].step != raw[b].step) return raw[a].step < raw[b].step;
    return raw[a].col < raw[b].col;
  });
  A.assertions.reserve(raw.size());
  for (size_t k = 0; k < idx.size(); k++) {
    const Assertion& a = raw[idx[k]];
    if (!A.assertions.empty() && A.assertions.back().step == a.step && A.assertions.back().col == a.col) continue;
    A.assertions.push_back(a);
  }
  // context.num_assertions (vm/air/mod.rs:248-290) must equal the deduped count
  size_t levels = std::max<size_t>(n / STEPS, 1);
  size_t expect = (2 + ROUNDS) * levels + (4 * ROUNDS + 2) * levels + 2 * levels;
  if (f_vm) {
    expect += 1;
    if (fe_is_zero(pc_init) && com_nz) expect += 1;
    if (pi.n_main_slots > 0 && fe_is_zero(pc_init)) expect += pi.n_main_slots;
  }
  if (f_vm && f_exp) expect += 1;
  if (pid_nz) expect += 6;
  if (expect != A.assertions.size()) return "assertion count differs from AirContext::num_assertions";
  return "";
}

std::vector<fe> pi_elements(const zkl_air_public_inputs& pi) {
  if (pi.n_main_slots > ZKL_MAX_MAIN_SLOTS) throw std::invalid_argument("n_main_slots exceeds ZKL_MAX_MAIN_SLOTS");
  std::vector<fe> out;
  out.push_back(fe{pi.feature_mask, 0});
  out.push_back(be_from_le16(pi.program_commitment));
  out.push_back(be_from_le16(pi.merkle_root));
  bool nz = false;
  for (int i = 0; i < 32; i++) nz |= pi.program_commitment[i] != 0;
  if (nz) {
    fe fc[2];
    program_field_commitment(pi.program_commitment, fc);
    out.push_back(fc[0]); out.push_back(fc[1]);
  } else {
    out.push_back(fe_zero()); out.push_back(fe_zero());
  }
  for (uint32_t i = 0; i < pi.n_main_slots; i++) out.push_back(fe_from(pi.main_slots[i]));
  out.push_back(fe_from(pi.pc_init));
  out.push_back(fe_from(pi.ram_gp_unsorted_in));
  out.push_back(fe_from(pi.ram_gp_unsorted_out));
  out.push_back(fe_from(pi.ram_gp_sorted_in));
  out.push_back(fe_from(pi.ram_gp_sorted_out));
  for (int i = 0; i < 3; i++) out.push_back(fe_from(pi.rom_s_in[i]));
  for (int i = 0; i < 3; i++) out.push_back(fe_from(pi.rom_s_out[i]));
  out.push_back(fe{pi.vm_usage_mask, 0});
  out.push_back(fe{pi.ram_delta_clk_bits, 0});
  return out;
}

std::vector<fe> context_elements(uint32_t width, size_t n, const zkl_proof_options& o) {
  return {fe{(uint64_t)width << 8, 0},  // TraceInfo: main width << 8 | #aux segments
          fe{(uint64_t)(uint32_t)n, 0},
          fe{P_LO, 0}, fe{P_HI, 0},    // field modulus LE bytes, two halves
          fe{((uint64_t)o.field_extension << 16) | ((uint64_t)o.fri_folding_factor << 8) | o.fri_remainder_max_degree, 0},
          fe{o.grinding_factor, 0}, fe{o.blowup_factor, 0}, fe{o.num_queries, 0}};
}

// coefficients (over y, degree < 32) of the 31 cycle-32 selector columns: q_col(y)
// interpolates the column's 32 values over <w_32> (inverse DFT)
static const std::vector<fe>& periodic_coeffs() {
  static const std::vector<fe> coef = [] {
    fe w32 = root_of_unity(5), w32i = fe_inv(w32), inv32 = fe_inv(fe{32, 0});
    std::vector<fe> c(31 * 32);
    for (int col = 0; col < 31; col++) {
      fe v[32];
      for (int pos = 0; pos < 32; pos++) {
        bool one;
        if (col == 0) one = pos == 0;
        else if (col <= 27) one = pos == col;
        else if (col == 28) one = pos == 28;
        else if (col == 29) one = pos >= 29;
        else one = pos == 31;
        v[pos] = one ? fe_one() : fe_zero();
      }
      for (int k = 0; k < 32; k++) {
        fe acc = fe_zero(), wk = fe_pow64(w32i, k), pw = fe_one();
        for (int j = 0; j < 32; j++) { acc = fe_add(acc, fe_mul(v[j], pw)); pw = fe_mul(pw, wk); }
        c[col * 32 + k] = fe_mul(acc, inv32);
      }
    }
    return c;
  }();
  return coef;
}

static void periodic_eval(size_t n, fe x, fe* out) {
  const std::vector<fe>& coef = periodic_coeffs();
  const fe y = fe_pow64(x, n / 32);
  for (int col = 0; col < 31; col++) {
    fe acc = fe_zero();
    for (int k = 31; k >= 0; k--) acc = fe_add(fe_mul(acc, y), coef[col * 32 + k]);
    out[col] = acc;
  }
}

std::vector<fe> periodic_table(size_t n, size_t ce, fe offset) {
  unsigned logce = 0;
  while (((size_t)1 << logce) < ce) logce++;
  fe wce = root_of_unity(logce);
  size_t period = ce / (n / 32);
  std::vector<fe> tab(period * 31);
  for (size_t i = 0; i < period; i++) periodic_eval(n, fe_mul(offset, fe_pow64(wce, i)), &tab[i * 31]);
  return tab;
}

std::vector<fe> periodic_at(size_t n, fe x) {
  std::vector<fe> v(31);
  periodic_eval(n, x, v.data());
  return v;
}

}  // namespace zkl
