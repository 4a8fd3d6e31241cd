// Workload generator (host): a synthetic zk-lisp VM segment built the way the reference's
// trace builder lays it out (vm/trace/mod.rs:386-524, vm/trace/vm.rs:58-888,
// vm/trace/rom.rs:29-108) with the {vm, rom} segment layout (vm/trace/mod.rs:80-235),
// plus the AIR public inputs prove_segment derives (prove.rs:292-423, 1197-1392).
// Program: (levels-1) ALU ops cycling Const/Add/Mov/Mul over r0..r7, splitmix64 choices,
// immediates < 2^63, then End.  flags bit 0 interleaves SAbsorbN / SSqueeze sponge ops
// (vm/trace/vm.rs:565-672, vm/trace/poseidon.rs:9-87) so the Poseidon AIR block
// (poseidon.rs:26-162) is exercised.  This is input preparation, not the measured path.
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/zkl_hip.h"
#include "air_host.h"
#include "host_hash.h"

using namespace zkl;

namespace {
uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
enum Kind { K_CONST = 0, K_MOV = 1, K_ADD = 2, K_SUB = 3, K_MUL = 4, K_ABSORB = 10, K_SQUEEZE = 11, K_END = 99 };
struct Op { Kind k; int dst, a, b; uint64_t imm; int nabs; int abs_regs[3]; };

struct Table {
  zkl_f128* t;
  size_t n;
  void set(int col, size_t row, fe v) { t[(size_t)col * n + row] = to_abi(v); }
  fe get(int col, size_t row) const { return fe_from(t[(size_t)col * n + row]); }
  void sel(size_t row, int start, int idx) {
    for (int i = 0; i < 8; i++) set(start + i, row, fe_zero());
    set(start + idx, row, fe_one());
  }
  // sponge lane selectors: lane j < k reads register regs[j] (3 index bits + active flag)
  void sponge_sel(const Layout& L, size_t row, const int* regs, int k) {
    for (int lane = 0; lane < 10; lane++) {
      bool on = lane < k;
      int idx = on ? regs[lane] : 0;
      for (int bit = 0; bit < 3; bit++) set(L.sel_s_bits + lane * 3 + bit, row, on ? fe{(uint64_t)((idx >> bit) & 1), 0} : fe_zero());
      set(L.sel_s_active + lane, row, on ? fe_one() : fe_zero());
    }
  }
};

// One level's Poseidon lanes (vm/trace/poseidon.rs:9-87): map row = [inputs (zero padded
// to 10), dom0, dom1]; round row 1+j = state before round j; final and pad rows = output.
void level_absorb(Table& T, const Layout& L, const PoseidonSuite& ps, size_t level, const fe* in, int nin) {
  size_t b = level * 32;
  fe st[12];
  for (int i = 0; i < 12; i++) st[i] = fe_zero();
  for (int i = 0; i < nin && i < 10; i++) st[i] = in[i];
  st[10] = ps.dom[0];
  st[11] = ps.dom[1];
  for (int i = 0; i < 12; i++) T.set(L.lanes_start + i, b, st[i]);
  for (int j = 0; j < 27; j++) {
    for (int i = 0; i < 12; i++) T.set(L.lanes_start + i, b + 1 + j, st[i]);
    fe s3[12], y[12];
    for (int i = 0; i < 12; i++) s3[i] = fe_cube(st[i]);
    for (int i = 0; i < 12; i++) {
      fe acc = fe_zero();
      for (int k = 0; k < 12; k++) acc = fe_add(acc, fe_mul(ps.mds[i][k], s3[k]));
      y[i] = fe_add(acc, ps.rc[j][i]);
    }
    memcpy(st, y, sizeof st);
  }
  for (size_t r = b + 28; r < b + 32; r++)
    for (int i = 0; i < 12; i++) T.set(L.lanes_start + i, r, st[i]);
}
}  // namespace

extern "C" int zkl_synth_vm_segment(uint64_t seed, uint32_t log_n, zkl_f128* trace, zkl_air_public_inputs* pi,
                                    uint32_t* width_out) {
  return zkl_synth_vm_segment_ex(seed, log_n, 0, trace, pi, width_out);
}

extern "C" int zkl_synth_vm_segment_ex(uint64_t seed, uint32_t log_n, uint32_t flags, zkl_f128* trace,
                                       zkl_air_public_inputs* pi, uint32_t* width_out) {
  if (flags & ~1u) return ZKL_E_INVALID;
  const bool sponge = flags & 1;
  if (log_n < 5 || log_n > 26) return ZKL_E_INVALID;
  const Layout L = make_layout(true, false, false, false, true);
  if (width_out) *width_out = (uint32_t)L.width;
  if (!trace) return ZKL_OK;
  if (!pi) return ZKL_E_INVALID;
  const size_t n = (size_t)1 << log_n, levels = n / 32;
  memset(trace, 0, sizeof(zkl_f128) * L.width * n);
  memset(pi, 0, sizeof *pi);
  Table T{trace, n};

  char desc[128];
  snprintf(desc, sizeof desc, "zkl-hip/synthetic-vm-segment/v1 %sseed=0x%016llx levels=%zu", sponge ? "sponge " : "",
           (unsigned long long)seed, levels);
  uint8_t pid[32];
  blake3_hash((const uint8_t*)desc, strlen(desc), pid);
  PoseidonSuite ps = derive_poseidon_suite(pid, 27);

  std::vector<Op> ops(levels);
  {
    uint64_t st = seed;
    const Kind cyc[4] = {K_CONST, K_ADD, K_MOV, K_MUL};
    // every 8 levels: absorb, const, absorb, squeeze, add, mov, mul, squeeze-with-nothing-pending
    const Kind cyc_s[8] = {K_ABSORB, K_CONST, K_ABSORB, K_SQUEEZE, K_ADD, K_MOV, K_MUL, K_SQUEEZE};
    for (size_t l = 0; l + 1 < levels; l++) {
      uint64_t r = splitmix(st);
      Op& o = ops[l];
      o = Op{};
      o.k = sponge ? cyc_s[l % 8] : cyc[l % 4];
      o.dst = (int)(r & 7); o.a = (int)((r >> 3) & 7); o.b = (int)((r >> 6) & 7);
      o.imm = o.k == K_CONST ? (splitmix(st) >> 1) : 0;
      if (o.k == K_ABSORB) {
        o.nabs = 1 + (int)((r >> 9) % 3);
        for (int i = 0; i < 3; i++) o.abs_regs[i] = (int)((r >> (12 + 3 * i)) & 7);
      }
    }
    ops[levels - 1] = Op{};
    ops[levels - 1].k = K_END;
  }
  // schedule gates, pc, domain tags (mod.rs:386-470)
  for (size_t l = 0; l < levels; l++) {
    size_t b = l * 32;
    T.set(L.g_map, b, fe_one());
    T.set(L.g_final, b + 28, fe_one());
    for (int j = 0; j < 27; j++) T.set(L.g_r_start + j, b + 1 + j, fe_one());
    for (size_t r = b; r < b + 32; r++) T.set(L.pc, r, fe{l, 0});
    T.set(L.lanes_start + 10, b, ps.dom[0]);
    T.set(L.lanes_start + 11, b, ps.dom[1]);
  }
  // VmTraceBuilder
  fe regs[8] = {};
  int pending[10], npending = 0;
  for (size_t l = 0; l < levels; l++) {
    fe next[8];
    memcpy(next, regs, sizeof next);
    size_t b = l * 32, rm = b, rf = b + 28;
    if (l == 0) T.set(L.pi_prog, 0, be_from_le16(pid));
    const Op& o = ops[l];
    if (o.k == K_ABSORB || o.k == K_SQUEEZE) {  // SAbsorbN / SSqueeze (vm.rs:565-672)
      T.set(L.rom_op_start + 8, rm, fe_one());
      int sel_regs[10], k = 0;
      if (o.k == K_ABSORB) {
        for (int i = 0; i < o.nabs; i++) { sel_regs[k++] = o.abs_regs[i]; pending[npending++] = o.abs_regs[i]; }
      } else {
        for (int i = 0; i < npending; i++) sel_regs[k++] = pending[i];
      }
      for (size_t row : {rm, rf}) {
        T.set(L.op[8], row, fe_one());
        T.sponge_sel(L, row, sel_regs, k);
      }
      if (o.k == K_SQUEEZE) {
        T.sel(rf, L.sel_dst0, o.dst);
        fe in[10];
        for (int i = 0; i < k; i++) in[i] = regs[sel_regs[i]];
        level_absorb(T, L, ps, l, in, k);
        next[o.dst] = T.get(L.lanes_start, rf);
        npending = 0;
        for (size_t r = b; r < b + 32; r++) T.set(L.pose_active, r, fe_one());
      }
    } else if (o.k != K_END) {
      int oh = (int)o.k;
      T.set(L.rom_op_start + oh, rm, fe_one());
      for (size_t row : {rm, rf}) {
        T.set(L.op[oh], row, fe_one());
        T.sel(row, L.sel_dst0, o.dst);
        if (o.k == K_CONST) T.set(L.imm, row, fe{o.imm, 0});
        else T.sel(row, L.sel_a, o.a);
        if (o.k == K_ADD || o.k == K_SUB || o.k == K_MUL) T.sel(row, L.sel_b, o.b);
      }
      switch (o.k) {
        case K_CONST: next[o.dst] = fe{o.imm, 0}; break;
        case K_MOV: next[o.dst] = regs[o.a]; break;
        case K_ADD: next[o.dst] = fe_add(regs[o.a], regs[o.b]); break;
        case K_SUB: next[o.dst] = fe_sub(regs[o.a], regs[o.b]); break;
        case K_MUL: next[o.dst] = fe_mul(regs[o.a], regs[o.b]); break;
        default: break;
      }
    }
    for (size_t r = rm; r <= rf; r++) for (int i = 0; i < 8; i++) T.set(L.r_start + i, r, regs[i]);
    for (size_t r = rf + 1; r < b + 32; r++) for (int i = 0; i < 8; i++) T.set(L.r_start + i, r, next[i]);
    memcpy(regs, next, sizeof regs);
  }
  // RomTraceBuilder
  fe rc3[27][3], mds3[3][3], w0[59], w1[59];
  derive_rom_constants(pid, rc3, mds3);
  {
    fe c = fe_mul(fe_pow64(fe{3, 0}, 17), fe{3, 0});
    for (int i = 0; i < 59; i++) { w0[i] = c; c = fe_mul(c, fe{3, 0}); }
    c = fe_mul(fe_pow64(fe{3, 0}, 1037), fe{3, 0});
    for (int i = 0; i < 59; i++) { w1[i] = c; c = fe_mul(c, fe{3, 0}); }
  }
  auto enc = [&](size_t row, const fe* w) {
    fe s = fe_zero();
    int k = 0;
    for (int i = 0; i < 17; i++) s = fe_add(s, fe_mul(T.get(L.op[i], row), w[k++]));
    const int st[5] = {L.sel_dst0, L.sel_a, L.sel_b, L.sel_c, L.sel_dst1};
    for (int q = 0; q < 5; q++) for (int i = 0; i < 8; i++) s = fe_add(s, fe_mul(T.get(st[q] + i, row), w[k++]));
    return s;
  };
  fe s0_prev = fe_zero();
  fe last[3] = {};
  for (size_t l = 0; l < levels; l++) {
    size_t b = l * 32, rm = b, rf = b + 28;
    fe s[3] = {s0_prev, enc(rm, w0), enc(rm, w1)};
    for (int i = 0; i < 3; i++) T.set(L.rom_s + i, rm, s[i]);
    for (int j = 0; j < 27; j++) {
      size_t r = b + 1 + j;
      for (int i = 0; i < 3; i++) T.set(L.rom_s + i, r, s[i]);
      fe c3[3] = {fe_cube(s[0]), fe_cube(s[1]), fe_cube(s[2])};
      fe y[3];
      for (int i = 0; i < 3; i++)
        y[i] = fe_add(fe_add(fe_add(fe_mul(mds3[i][0], c3[0]), fe_mul(mds3[i][1], c3[1])), fe_mul(mds3[i][2], c3[2])), rc3[j][i]);
      for (int i = 0; i < 3; i++) T.set(L.rom_s + i, r + 1, y[i]);
      memcpy(s, y, sizeof s);
    }
    for (size_t r = rf + 1; r < b + 32; r++) for (int i = 0; i < 3; i++) T.set(L.rom_s + i, r, s[i]);
    s0_prev = s[0];
    memcpy(last, s, sizeof last);
  }
  // AIR public inputs for the whole-trace segment
  memcpy(pi->program_id, pid, 32);
  memcpy(pi->program_commitment, pid, 32);
  pi->feature_mask = sponge ? (2 | 32 | 1) : 2;  // FM_VM (+ FM_SPONGE | FM_POSEIDON)
  pi->segment_feature_mask = pi->feature_mask;
  pi->vm_out_reg = 0;
  pi->vm_out_row = 29;
  for (size_t l = levels; l-- > 0;) {  // vm_output_from_trace_with_layout (utils.rs:262-289)
    size_t rf = l * 32 + 28;
    int found = -1;
    for (int i = 0; i < 8 && found < 0; i++) if (fe_eq(T.get(L.sel_dst0 + i, rf), fe_one())) found = i;
    if (found >= 0) { pi->vm_out_reg = (uint32_t)found; pi->vm_out_row = (uint32_t)(rf + 1); break; }
  }
  for (int i = 0; i < 3; i++) {
    pi->rom_acc[i] = to_abi(last[i]);
    pi->rom_s_in[i] = to_abi(T.get(L.rom_s + i, 0));
    pi->rom_s_out[i] = to_abi(T.get(L.rom_s + i, (levels - 1) * 32 + 28));
  }
  pi->pc_init = to_abi(T.get(L.pc, 0));
  uint32_t mask = 0;  // compute_vm_usage_mask_for_trace (prove.rs:1289-1392)
  for (size_t r = 0; r < n; r++) {
    bool fin = (r % 32) == 28;
    auto nz = [&](int k) { return !fe_is_zero(T.get(L.op[k], r)); };
    if (fin && (nz(9) || nz(7))) mask |= 1u << 0;
    if (fin && nz(10)) mask |= 1u << 1;
    if (fin && nz(11)) mask |= 1u << 2;
    if (fin && nz(12)) mask |= 1u << 3;
    if (fin && nz(14)) mask |= 1u << 4;
    if (fin && nz(13)) mask |= 1u << 5;
    if (fin && nz(6)) mask |= 1u << 6;
    if (nz(8)) mask |= 1u << 7;
  }
  pi->vm_usage_mask = mask;
  return ZKL_OK;
}
