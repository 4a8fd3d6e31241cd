// Workload generator (host): a synthetic zk-lisp VM segment built the way the reference's
// trace builder lays it out (vm/trace/mod.rs:386-524, vm/trace/vm.rs:58-888,
// vm/trace/ram.rs:43-271, vm/trace/rom.rs:29-108) directly in the segment layout the feature
// set implies (vm/trace/mod.rs:80-235), plus the AIR public inputs prove_segment derives
// (prove.rs:292-423, 1197-1392).
//
// Program (splitmix64 choices, immediates < 2^63, End on the last level):
//   flags 0            Const/Add/Mov/Mul over r0..r7
//   ZKL_SYN_SPONGE     8-level block absorb, const, absorb, squeeze, add, mov, mul, squeeze
//                      (SAbsorbN / SSqueeze, vm.rs:565-672) -> PoseidonAir block
//   ZKL_SYN_RAM        8-level block addr const (r7 <- 0..7), const, store, load, add, store,
//                      mul, load (vm.rs:803-842); ALU destinations avoid r7 -> RamAir block
//   ZKL_SYN_MERKLE     levels 1..5: bit r5, bit r6, MerkleStepFirst(leaf r0, dir r5, sib r1),
//                      MerkleStep(dir r6, sib r2), MerkleStepLast(dir r5, sib r3)
//                      (vm.rs:675-800) -> MerkleAir block, root in pi.merkle_root
// This is input preparation, not the measured path.
#include <stdio.h>
#include <string.h>

#include <algorithm>
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
enum Kind {
  K_CONST = 0, K_MOV = 1, K_ADD = 2, K_SUB = 3, K_MUL = 4, K_ABSORB = 10, K_SQUEEZE = 11, K_ADDR = 12,
  K_LOAD = 15, K_STORE = 16, K_MFIRST = 20, K_MSTEP = 21, K_MLAST = 22,
  K_NEG = 40, K_EQ, K_SELECT, K_ASSERT, K_ASSERT_BIT, K_RANGE, K_RANGE_LO, K_RANGE_HI, K_DIVMOD, K_DIV128, K_MULWIDE,
  K_END = 99, K_PAD = 100  // K_PAD: a level past the program's last op (build_empty_trace rows only)
};
// Merkle steps: dst = leaf register, a = dir register, b = sibling register.  dst2: the second
// destination (DivMod r, MulWide hi, DivMod128 r); c: condition / range register (Select,
// Assert*, AssertRange*) or a_lo (DivMod128); bits: AssertRange width.
struct Op { Kind k; int dst, a, b; uint64_t imm; int nabs; int abs_regs[10]; int c, dst2, bits; };
// op_to_one_hot (vm.rs:890-922): the op column / ROM one-hot index of a kind, -1 for none
int onehot_of(Kind k) {
  switch (k) {
    case K_CONST: case K_ADDR: return 0;
    case K_MOV: return 1;
    case K_ADD: return 2;
    case K_SUB: return 3;
    case K_MUL: return 4;
    case K_NEG: return 5;
    case K_EQ: return 6;
    case K_SELECT: return 7;
    case K_ABSORB: case K_SQUEEZE: return 8;
    case K_ASSERT: return 9;
    case K_ASSERT_BIT: return 10;
    case K_RANGE: case K_RANGE_LO: case K_RANGE_HI: return 11;
    case K_DIVMOD: return 12;
    case K_DIV128: return 13;
    case K_MULWIDE: return 14;
    case K_LOAD: return 15;
    case K_STORE: return 16;
    default: return -1;
  }
}
unsigned __int128 as_u128(fe v) { return ((unsigned __int128)v.hi << 64) | v.lo; }
fe from_u64(uint64_t x) { return fe{x, 0}; }
constexpr int ADDR_REG = 7;

struct RamEvent { fe addr, clk, val, w; };

struct Table {
  zkl_f128* t;
  size_t n;
  void set(int col, size_t row, fe v) { t[(size_t)col * n + row] = to_abi(v); }
  fe get(int col, size_t row) const { return fe_from(t[(size_t)col * n + row]); }
  bool nz(int col, size_t row) const { return !fe_is_zero(get(col, row)); }
  void sel(size_t row, int start, int idx) {
    for (int i = 0; i < 8; i++) set(start + i, row, fe_zero());
    set(start + idx, row, fe_one());
  }
  // sponge lane selectors: lane j < k reads register regs[j] (3 index bits + active flag)
  void sponge_sel(const Layout& L, size_t row, const int* regs, int k) {
    for (int lane = 0; lane < 10; lane++) {
      bool on = lane < k;
      int idx = on ? regs[lane] : 0;
      for (int bit = 0; bit < 3; bit++)
        set(L.sel_s_bits + lane * 3 + bit, row, on ? fe{(uint64_t)((idx >> bit) & 1), 0} : fe_zero());
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

std::vector<Op> make_program(uint64_t seed, size_t levels, uint32_t flags) {
  std::vector<Op> ops(levels);
  uint64_t st = seed;
  std::vector<Kind> cycle;
  if (flags & ZKL_SYN_SPONGE) cycle.insert(cycle.end(), {K_ABSORB, K_CONST, K_ABSORB, K_SQUEEZE, K_ADD, K_MOV, K_MUL, K_SQUEEZE});
  if (flags & ZKL_SYN_RAM) cycle.insert(cycle.end(), {K_ADDR, K_CONST, K_STORE, K_LOAD, K_ADD, K_STORE, K_MUL, K_LOAD});
  if (cycle.empty()) cycle = {K_CONST, K_ADD, K_MOV, K_MUL};
  const bool ram = flags & ZKL_SYN_RAM;
  int last_dst = 0;  // RAM programs: stores / adds / muls read the latest result
  for (size_t l = 0; l + 1 < levels; l++) {
    uint64_t r = splitmix(st);
    Op& o = ops[l];
    o = Op{};
    o.k = cycle[l % cycle.size()];
    o.dst = (int)(r & 7);
    if (ram) o.dst %= ADDR_REG;
    o.a = (int)((r >> 3) & 7);
    o.b = (int)((r >> 6) & 7);
    o.imm = o.k == K_CONST ? (splitmix(st) >> 1) : 0;
    switch (o.k) {
      case K_ABSORB:
        o.nabs = 1 + (int)((r >> 9) % 3);
        for (int i = 0; i < 3; i++) o.abs_regs[i] = (int)((r >> (12 + 3 * i)) & 7);
        break;
      case K_ADDR: o.dst = ADDR_REG; o.imm = (r >> 9) & 7; break;
      case K_STORE: o.a = ADDR_REG; o.b = last_dst; break;
      case K_LOAD: o.a = ADDR_REG; break;
      case K_ADD:
      case K_MUL: if (ram) o.a = last_dst; break;
      default: break;
    }
    if (o.k != K_STORE && o.k != K_ABSORB && o.k != K_ADDR) last_dst = o.dst;
  }
  if ((flags & ZKL_SYN_MERKLE) && levels >= 8) {
    uint64_t r = splitmix(st);
    const Op m[5] = {{K_CONST, 5, 0, 0, r & 1, 0, {}, 0, 0, 0}, {K_CONST, 6, 0, 0, (r >> 1) & 1, 0, {}, 0, 0, 0},
                     {K_MFIRST, 0, 5, 1, 0, 0, {}, 0, 0, 0}, {K_MSTEP, 0, 6, 2, 0, 0, {}, 0, 0, 0},
                     {K_MLAST, 0, 5, 3, 0, 0, {}, 0, 0, 0}};
    for (int i = 0; i < 5; i++) ops[1 + i] = m[i];
  }
  ops[levels - 1] = Op{};
  ops[levels - 1].k = K_END;
  return ops;
}

// RamTraceBuilder::fill_table (vm/trace/ram.rs:43-271)
void fill_ram(Table& T, const Layout& L, const uint8_t pid[32], std::vector<RamEvent> ev) {
  const size_t n = T.n;
  auto key_less = [](fe a, fe b) { return a.hi != b.hi ? a.hi < b.hi : a.lo < b.lo; };
  std::stable_sort(ev.begin(), ev.end(), [&](const RamEvent& x, const RamEvent& y) {
    if (!fe_eq(x.addr, y.addr)) return key_less(x.addr, y.addr);
    return key_less(x.clk, y.clk);
  });
  std::vector<size_t> at(ev.size());
  size_t k = 0;
  for (size_t row = 0; row < n && k < ev.size(); row++) {
    if (row % 32 < 29) continue;  // sorted table lives in the pad rows
    T.set(L.ram_sorted, row, fe_one());
    T.set(L.ram_s_addr, row, ev[k].addr);
    T.set(L.ram_s_clk, row, ev[k].clk);
    T.set(L.ram_s_val, row, ev[k].val);
    T.set(L.ram_s_is_write, row, ev[k].w);
    at[k++] = row;
  }
  for (size_t i = 0; i + 1 < ev.size(); i++) {  // mirror same-address witnesses across the gap
    if (!fe_eq(ev[i].addr, ev[i + 1].addr)) continue;
    for (size_t row = at[i] + 1; row < at[i + 1]; row++) {
      if (T.nz(L.ram_sorted, row)) continue;
      T.set(L.ram_s_addr, row, ev[i].addr);
      T.set(L.ram_s_clk, row, ev[i].clk);
      T.set(L.ram_s_val, row, ev[i].val);
      T.set(L.ram_s_is_write, row, ev[i].w);
    }
  }
  fe pfe[2];
  program_field_commitment(pid, pfe);
  const fe q0 = pfe[0], q2 = fe_mul(q0, q0), q3 = fe_mul(q2, q0), q5 = fe_mul(fe_mul(q2, q2), q0);
  const fe r1 = fe_add(q2, fe_one()), r2 = fe_add(q3, q0), r3 = fe_add(q5, fe{7, 0});
  auto compress = [&](fe a, fe clk, fe v, fe w) {
    return fe_add(fe_add(fe_add(a, fe_mul(r1, clk)), fe_mul(r2, v)), fe_mul(r3, w));
  };
  fe gp = fe_zero(), last = fe_zero();
  for (size_t row = 0; row < n; row++) {
    if (row > 0 && T.nz(L.ram_sorted, row - 1)) {
      const size_t p = row - 1;
      const fe a = T.get(L.ram_s_addr, p), v = T.get(L.ram_s_val, p), w = T.get(L.ram_s_is_write, p);
      gp = fe_add(gp, compress(a, T.get(L.ram_s_clk, p), v, w));
      last = fe_eq(T.get(L.ram_s_addr, row), a) ? fe_add(fe_mul(fe_sub(fe_one(), w), last), fe_mul(w, v))
                                                 : fe_mul(w, v);
    }
    T.set(L.ram_gp_sorted, row, gp);
    T.set(L.ram_s_last_write, row, last);
  }
  for (size_t row = 0; row + 1 < n; row++) {
    if (!T.nz(L.ram_sorted, row)) continue;
    const fe a = T.get(L.ram_s_addr, row), an = T.get(L.ram_s_addr, row + 1);
    T.set(L.eq_inv, row, fe_inv(fe_sub(an, a)));
    if (T.nz(L.ram_sorted, row + 1) && fe_eq(an, a)) {  // delta_clk bits (saturating as_int difference)
      const fe c0 = T.get(L.ram_s_clk, row), c1 = T.get(L.ram_s_clk, row + 1);
      const bool pos = c1.hi != c0.hi ? c1.hi > c0.hi : c1.lo > c0.lo;
      const uint64_t d = pos ? c1.lo - c0.lo : 0;  // clocks are level indices (< 2^64)
      for (int i = 0; i < 32; i++) T.set(L.gadget_b + i, row, fe{(d >> i) & 1, 0});
    }
  }
  fe gu = fe_zero();
  for (size_t row = 0; row < n; row++) {
    if (row > 0 && (row - 1) % 32 == 28) {
      const size_t p = row - 1;
      const bool ld = fe_eq(T.get(L.op[15], p), fe_one()), stv = fe_eq(T.get(L.op[16], p), fe_one());
      if (ld || stv) {
        fe a_ev = fe_zero(), b_ev = fe_zero();
        for (int i = 0; i < 8; i++) {
          const fe ri = T.get(L.r_start + i, p);
          a_ev = fe_add(a_ev, fe_mul(T.get(L.sel_a + i, p), ri));
          b_ev = fe_add(b_ev, fe_mul(T.get(L.sel_b + i, p), ri));
        }
        gu = fe_add(gu, compress(a_ev, T.get(L.pc, p), stv ? b_ev : T.get(L.imm, p), stv ? fe_one() : fe_zero()));
      }
    }
    T.set(L.ram_gp_unsorted, row, gu);
  }
}
}  // namespace

extern "C" int zkl_synth_vm_segment(uint64_t seed, uint32_t log_n, zkl_f128* trace, zkl_air_public_inputs* pi,
                                    uint32_t* width_out) {
  return zkl_synth_vm_segment_ex(seed, log_n, 0, trace, pi, width_out);
}

extern "C" int zkl_synth_vm_segment_ex(uint64_t seed, uint32_t log_n, uint32_t flags, zkl_f128* trace,
                                       zkl_air_public_inputs* pi, uint32_t* width_out) {
  return zkl_synth_vm_segment_chain(seed, seed, log_n, flags, nullptr, trace, pi, width_out);
}

namespace {
// vm_output_from_trace_with_layout (utils.rs:262-289) and compute_vm_usage_mask_for_trace
// (prove.rs:1289-1392) of a (segment) trace in layout L
void derive_trace_pi(const Table& T, const Layout& L, bool ram, size_t levels, zkl_air_public_inputs* pi) {
  const size_t n = T.n;
  pi->vm_out_reg = 0;
  pi->vm_out_row = 29;
  for (size_t l = levels; l-- > 0;) {  // vm_output_from_trace_with_layout (utils.rs:262-289)
    size_t rf = l * 32 + 28;
    int found = -1;
    for (int i = 0; i < 8 && found < 0; i++) if (fe_eq(T.get(L.sel_dst0 + i, rf), fe_one())) found = i;
    if (found >= 0) { pi->vm_out_reg = (uint32_t)found; pi->vm_out_row = (uint32_t)(rf + 1); break; }
  }
  uint32_t mask = 0, ram_bits = 0;  // compute_vm_usage_mask_for_trace (prove.rs:1289-1392)
  for (size_t r = 0; r < n; r++) {
    bool fin = (r % 32) == 28;
    auto nz = [&](int k) { return T.nz(L.op[k], r); };
    if (fin && (nz(9) || nz(7))) mask |= 1u << 0;
    if (fin && nz(10)) mask |= 1u << 1;
    if (fin && nz(11)) mask |= 1u << 2;
    if (fin && nz(12)) mask |= 1u << 3;
    if (fin && nz(14)) mask |= 1u << 4;
    if (fin && nz(13)) mask |= 1u << 5;
    if (fin && nz(6)) mask |= 1u << 6;
    if (nz(8)) mask |= 1u << 7;
    if (ram && r + 1 < n && T.nz(L.ram_sorted, r) && T.nz(L.ram_sorted, r + 1) &&
        fe_eq(T.get(L.ram_s_addr, r), T.get(L.ram_s_addr, r + 1))) {
      mask |= 1u << 8;
      for (int i = 0; i < 32; i++) if (T.nz(L.gadget_b + i, r)) ram_bits |= 1u << i;
    }
  }
  pi->vm_usage_mask = mask;
  pi->ram_delta_clk_bits = ram_bits;
}

// The trace of one program (ops.size() == n / 32 levels; K_PAD past the last op) in the
// segment layout of its features: build_full_trace (vm/trace/mod.rs:434-524) with the
// VmTraceBuilder (vm.rs:58-888), RamTraceBuilder (ram.rs:43-271), RomTraceBuilder
// (rom.rs:29-108), plus the AIR public inputs prove_segment derives (prove.rs:292-423).
// regs0: the initial register file (secret args, then main-arg slots in the tail registers,
// vm.rs:64-104); rom0: ROM lane 0 entering the first level.
int build_core(const std::vector<Op>& ops, const uint8_t pid[32], const uint8_t commit[32], bool sponge, bool ram,
               bool merkle, fe rom0, const fe regs0[8], const std::vector<fe>& slots, size_t n, zkl_f128* trace,
               zkl_air_public_inputs* pi) {
  const Layout L = make_layout(true, ram, sponge, merkle, true);
  const size_t levels = n / 32;
  memset(trace, 0, sizeof(zkl_f128) * L.width * n);
  memset(pi, 0, sizeof *pi);
  Table T{trace, n};
  PoseidonSuite ps = derive_poseidon_suite(pid, 27);

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
  fe regs[8];
  memcpy(regs, regs0, sizeof regs);
  int pending[10], npending = 0;
  std::vector<RamEvent> events;
  std::vector<std::pair<fe, fe>> mem;  // host memory: address -> last stored value
  long last_merkle = -1;
  for (size_t l = 0; l < levels; l++) {
    fe next[8];
    memcpy(next, regs, sizeof next);
    size_t b = l * 32, rm = b, rf = b + 28;
    const Op& o = ops[l];
    if (o.k == K_PAD) continue;  // levels past the program: build_empty_trace rows only
    if (l == 0) T.set(L.pi_prog, 0, be_from_le16(pid));
    {
      const int oh = onehot_of(o.k);
      if (oh >= 0) T.set(L.rom_op_start + oh, rm, fe_one());
    }
    switch (o.k) {
      case K_ABSORB:
      case K_SQUEEZE: {  // SAbsorbN / SSqueeze (vm.rs:565-672)
        int sel_regs[10], k = 0;
        if (o.k == K_ABSORB) {
          for (int i = 0; i < o.nabs; i++) {
            if (npending >= 10) return ZKL_E_INVALID;  // push_absorb: sponge rate overflow (vm.rs:925-935)
            sel_regs[k++] = o.abs_regs[i];
            pending[npending++] = o.abs_regs[i];
          }
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
        break;
      }
      case K_MFIRST:
      case K_MSTEP:
      case K_MLAST: {  // MerkleStepFirst / MerkleStep / MerkleStepLast (vm.rs:675-800)
        for (size_t r = b; r < b + 32; r++) T.set(L.merkle_g, r, fe_one());
        fe acc;
        if (o.k == K_MFIRST) {
          acc = regs[o.dst];
          T.set(L.merkle_first, rm, fe_one());
          T.set(L.merkle_leaf, rm, acc);
        } else {
          acc = last_merkle >= 0 ? T.get(L.merkle_acc, (size_t)last_merkle * 32 + 28) : fe_zero();
        }
        for (size_t r = rm; r < rf; r++) T.set(L.merkle_acc, r, acc);
        const fe d = regs[o.a], sib = regs[o.b], nd = fe_sub(fe_one(), d);
        T.set(L.merkle_dir, rm, d);
        T.set(L.merkle_sib, rm, sib);
        const fe in[2] = {fe_add(fe_mul(nd, acc), fe_mul(d, sib)), fe_add(fe_mul(nd, sib), fe_mul(d, acc))};
        level_absorb(T, L, ps, l, in, 2);
        if (o.k == K_MLAST) T.set(L.merkle_last, rf, fe_one());
        const fe out = T.get(L.lanes_start, rf);
        for (size_t r = rf; r < b + 32; r++) T.set(L.merkle_acc, r, out);
        for (size_t r = b; r < b + 32; r++) T.set(L.pose_active, r, fe_one());
        last_merkle = (long)l;
        break;
      }
      case K_LOAD:
      case K_STORE: {  // Load / Store (vm.rs:803-842): clk = level; unwritten addresses read 0
        const int oh = o.k == K_LOAD ? 15 : 16;
        const fe addr = regs[o.a];
        auto it = std::find_if(mem.begin(), mem.end(), [&](const std::pair<fe, fe>& e) { return fe_eq(e.first, addr); });
        for (size_t row : {rm, rf}) {
          T.set(L.op[oh], row, fe_one());
          T.sel(row, L.sel_a, o.a);
          if (o.k == K_LOAD) T.sel(row, L.sel_dst0, o.dst);
          else T.sel(row, L.sel_b, o.b);
        }
        fe val;
        if (o.k == K_LOAD) {
          val = it != mem.end() ? it->second : fe_zero();
          T.set(L.imm, rm, val);
          T.set(L.imm, rf, val);
          next[o.dst] = val;
        } else {
          val = regs[o.b];
          if (it != mem.end()) it->second = val;
          else mem.push_back({addr, val});
        }
        events.push_back({addr, fe{l, 0}, val, o.k == K_STORE ? fe_one() : fe_zero()});
        break;
      }
      case K_END: break;
      default: {  // ALU (vm.rs:199-564): op bit, selectors and witnesses on the map and final rows
        const int oh = onehot_of(o.k);
        const Kind k = o.k;
        const bool is_const = k == K_CONST || k == K_ADDR;
        const bool has_a = !is_const && k != K_ASSERT && k != K_ASSERT_BIT && k != K_RANGE && k != K_RANGE_LO &&
                           k != K_RANGE_HI;
        const bool has_b = k == K_ADD || k == K_SUB || k == K_MUL || k == K_EQ || k == K_SELECT || k == K_DIVMOD ||
                           k == K_DIV128 || k == K_MULWIDE;
        const bool has_c = k == K_SELECT || k == K_ASSERT || k == K_ASSERT_BIT || k == K_RANGE || k == K_RANGE_LO ||
                           k == K_RANGE_HI;
        const bool has_d2 = k == K_DIVMOD || k == K_DIV128 || k == K_MULWIDE;
        fe imm = fe_zero(), eqinv = fe_zero();
        fe bitsv[32];
        bool gadget = false;
        const fe va = regs[o.a], vb = regs[o.b], vc = regs[o.c];
        const unsigned __int128 M64 = ((unsigned __int128)1 << 64) - 1;
        switch (k) {
          case K_CONST:
          case K_ADDR: imm = fe{o.imm, 0}; next[o.dst] = imm; break;
          case K_MOV: next[o.dst] = va; break;
          case K_ADD: next[o.dst] = fe_add(va, vb); break;
          case K_SUB: next[o.dst] = fe_sub(va, vb); break;
          case K_MUL: next[o.dst] = fe_mul(va, vb); break;
          case K_NEG: next[o.dst] = fe_sub(fe_zero(), va); break;
          case K_EQ: {
            const fe diff = fe_sub(va, vb);
            eqinv = fe_is_zero(diff) ? fe_zero() : fe_inv(diff);
            next[o.dst] = fe_is_zero(diff) ? fe_one() : fe_zero();
            break;
          }
          case K_SELECT: next[o.dst] = fe_add(fe_mul(vc, va), fe_mul(fe_sub(fe_one(), vc), vb)); break;
          case K_ASSERT:
          case K_ASSERT_BIT: next[o.dst] = fe_one(); break;
          case K_RANGE: {  // 32-bit mode: stage 1 (imm 1), mode64 0 (eq_inv 0); low min(bits, 32) bits
            imm = fe_one();
            unsigned __int128 x = as_u128(vc);
            const int kb = std::min(o.bits, 32);
            for (int i = 0; i < 32; i++) {
              bitsv[i] = from_u64(i < kb ? (uint64_t)(x & 1) : 0);
              if (i < kb) x >>= 1;
            }
            gadget = true;
            next[o.dst] = fe_one();
            break;
          }
          case K_RANGE_LO:
          case K_RANGE_HI: {  // 64-bit stages 0 / 1: imm 0 / 1, mode64 (eq_inv 1), low / high 32 bits
            imm = k == K_RANGE_HI ? fe_one() : fe_zero();
            eqinv = fe_one();
            unsigned __int128 x = as_u128(vc) >> (k == K_RANGE_HI ? 32 : 0);
            for (int i = 0; i < 32; i++) { bitsv[i] = from_u64((uint64_t)(x & 1)); x >>= 1; }
            gadget = true;
            next[o.dst] = k == K_RANGE_HI ? fe_one() : from_u64((uint64_t)(as_u128(vc) & 0xFFFFFFFFu));
            break;
          }
          case K_DIVMOD: {  // u128 division of the canonical values; q, r truncated to 64 bits
            const unsigned __int128 av = as_u128(va), bv = as_u128(vb);
            const unsigned __int128 q = bv == 0 ? 0 : av / bv, r = bv == 0 ? av : av % bv;
            next[o.dst] = from_u64((uint64_t)(q & M64));
            next[o.dst2] = from_u64((uint64_t)(r & M64));
            eqinv = bv != 0 ? fe_inv(from_u64((uint64_t)bv)) : fe_zero();
            break;
          }
          case K_MULWIDE: {  // (a mod 2^64)(b mod 2^64): lo -> dst0 (dst), hi -> dst1 (dst2)
            const unsigned __int128 prod = (as_u128(va) & M64) * (as_u128(vb) & M64);
            next[o.dst] = from_u64((uint64_t)(prod & M64));
            next[o.dst2] = from_u64((uint64_t)(prod >> 64));
            break;
          }
          case K_DIV128: {  // (a_hi 2^64 | a_lo mod 2^64) / b; a_lo rides in imm
            imm = vc;
            const unsigned __int128 num = (as_u128(va) << 64) | (as_u128(vc) & M64), cu = as_u128(vb);
            const unsigned __int128 q = cu == 0 ? 0 : num / cu, r = cu == 0 ? num : num % cu;
            next[o.dst] = from_u64((uint64_t)(q & M64));
            next[o.dst2] = from_u64((uint64_t)(r & M64));
            eqinv = cu != 0 ? fe_inv(from_u64((uint64_t)cu)) : fe_zero();
            break;
          }
          default: return ZKL_E_INVALID;
        }
        for (size_t row : {rm, rf}) {
          T.set(L.op[oh], row, fe_one());
          T.sel(row, L.sel_dst0, o.dst);
          if (has_d2) T.sel(row, L.sel_dst1, o.dst2);
          if (has_a) T.sel(row, L.sel_a, o.a);
          if (has_b) T.sel(row, L.sel_b, o.b);
          if (has_c) T.sel(row, L.sel_c, o.c);
          T.set(L.imm, row, imm);
          T.set(L.eq_inv, row, eqinv);
          if (gadget)
            for (int i = 0; i < 32; i++) T.set(L.gadget_b + i, row, bitsv[i]);
        }
      }
    }
    for (size_t r = rm; r <= rf; r++) for (int i = 0; i < 8; i++) T.set(L.r_start + i, r, regs[i]);
    for (size_t r = rf + 1; r < b + 32; r++) for (int i = 0; i < 8; i++) T.set(L.r_start + i, r, next[i]);
    memcpy(regs, next, sizeof regs);
  }
  if (ram) fill_ram(T, L, pid, events);
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
  fe s0_prev = rom0;  // ROM lane 0 carries across segments
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
  memcpy(pi->program_commitment, commit, 32);
  pi->feature_mask = FM_VM | (sponge ? FM_SPONGE | FM_POSEIDON : 0) | (ram ? FM_RAM : 0) |
                     (merkle ? FM_MERKLE | FM_POSEIDON : 0);
  pi->n_main_slots = (uint32_t)slots.size();
  for (size_t i = 0; i < slots.size(); i++) pi->main_slots[i] = to_abi(slots[i]);
  pi->segment_feature_mask = pi->feature_mask;
  long last_mlast = -1;
  for (size_t l = 0; l < levels; l++) if (ops[l].k == K_MLAST) last_mlast = (long)l;
  if (merkle && last_mlast >= 0) {  // root = acc after the (last) MerkleStepLast level, 16 LE bytes
    const fe root = T.get(L.merkle_acc, (size_t)last_mlast * 32 + 28);
    for (int i = 0; i < 8; i++) {
      pi->merkle_root[i] = (uint8_t)(root.lo >> (8 * i));
      pi->merkle_root[8 + i] = (uint8_t)(root.hi >> (8 * i));
    }
  }
  for (int i = 0; i < 3; i++) {
    pi->rom_acc[i] = to_abi(last[i]);
    pi->rom_s_in[i] = to_abi(T.get(L.rom_s + i, 0));
    pi->rom_s_out[i] = to_abi(T.get(L.rom_s + i, (levels - 1) * 32 + 28));
  }
  pi->pc_init = to_abi(T.get(L.pc, 0));
  derive_trace_pi(T, L, ram, levels, pi);
  return ZKL_OK;
}

// SegmentFeatures::from_ops: sponge ops need the PoseidonAir block, Merkle steps the MerkleAir
// block (with Poseidon), Load / Store the RamAir block.
void features_of(const std::vector<Op>& ops, bool& sponge, bool& ram, bool& merkle) {
  sponge = ram = merkle = false;
  for (const Op& o : ops) {
    sponge |= o.k == K_ABSORB || o.k == K_SQUEEZE;
    ram |= o.k == K_LOAD || o.k == K_STORE;
    merkle |= o.k == K_MFIRST || o.k == K_MSTEP || o.k == K_MLAST;
  }
}
}  // namespace

extern "C" int zkl_synth_vm_segment_chain(uint64_t program_seed, uint64_t seed, uint32_t log_n, uint32_t flags,
                                          const zkl_f128* rom0_in, zkl_f128* trace, zkl_air_public_inputs* pi,
                                          uint32_t* width_out) {
  const uint32_t all = ZKL_SYN_SPONGE | ZKL_SYN_RAM | ZKL_SYN_MERKLE;
  if ((flags & ~all) || log_n < 5 || log_n > 26) return ZKL_E_INVALID;
  if ((flags & ZKL_SYN_MERKLE) && log_n < 8) return ZKL_E_INVALID;  // the path needs 8 levels
  const bool sponge = flags & ZKL_SYN_SPONGE, ram = flags & ZKL_SYN_RAM, merkle = flags & ZKL_SYN_MERKLE;
  const Layout L = make_layout(true, ram, sponge, merkle, true);
  if (width_out) *width_out = (uint32_t)L.width;
  if (!trace) return ZKL_OK;
  if (!pi) return ZKL_E_INVALID;
  const size_t n = (size_t)1 << log_n, levels = n / 32;
  char desc[160];
  snprintf(desc, sizeof desc, "zkl-hip/synthetic-vm-segment/v1 %s%s%sseed=0x%016llx levels=%zu",
           sponge ? "sponge " : "", ram ? "ram " : "", merkle ? "merkle " : "", (unsigned long long)program_seed, levels);
  uint8_t pid[32];
  blake3_hash((const uint8_t*)desc, strlen(desc), pid);
  const fe regs0[8] = {};
  return build_core(make_program(seed, levels, flags), pid, pid, sponge, ram, merkle,
                    rom0_in ? fe_from(*rom0_in) : fe_zero(), regs0, {}, n, trace, pi);
}

namespace {
// zkl_op list -> Op per level, K_PAD past the last op (levels = next_pow2(n_ops), mod.rs:439)
int to_ops(const zkl_op* ops_in, uint32_t n_ops, std::vector<Op>& ops) {
  size_t levels = 1;
  while (levels < n_ops) levels <<= 1;  // total_levels = levels.next_power_of_two() (mod.rs:439)
  if (levels > ((size_t)1 << 21)) return ZKL_E_INVALID;
  ops.assign(levels, Op{});
  for (size_t l = 0; l < levels; l++) {
    Op& o = ops[l];
    o = Op{};
    if (l >= n_ops) { o.k = K_PAD; continue; }
    const zkl_op& z = ops_in[l];
    if (z.dst > 7 || z.dst2 > 7 || z.a > 7 || z.b > 7 || z.c > 7 || z.n_regs > 10) return ZKL_E_INVALID;
    o.dst = z.dst; o.dst2 = z.dst2; o.a = z.a; o.b = z.b; o.c = z.c; o.bits = z.bits; o.imm = z.imm;
    switch (z.kind) {
      case ZKL_OP_CONST: o.k = K_CONST; break;
      case ZKL_OP_MOV: o.k = K_MOV; break;
      case ZKL_OP_ADD: o.k = K_ADD; break;
      case ZKL_OP_SUB: o.k = K_SUB; break;
      case ZKL_OP_MUL: o.k = K_MUL; break;
      case ZKL_OP_NEG: o.k = K_NEG; break;
      case ZKL_OP_EQ: o.k = K_EQ; break;
      case ZKL_OP_SELECT: o.k = K_SELECT; break;
      case ZKL_OP_ASSERT: o.k = K_ASSERT; break;
      case ZKL_OP_ASSERT_BIT: o.k = K_ASSERT_BIT; break;
      case ZKL_OP_ASSERT_RANGE:
        if (z.bits < 1 || z.bits > 64) return ZKL_E_INVALID;
        o.k = K_RANGE;
        break;
      case ZKL_OP_ASSERT_RANGE_LO: o.k = K_RANGE_LO; break;
      case ZKL_OP_ASSERT_RANGE_HI: o.k = K_RANGE_HI; break;
      case ZKL_OP_DIVMOD: o.k = K_DIVMOD; break;
      case ZKL_OP_DIVMOD128: o.k = K_DIV128; break;
      case ZKL_OP_MULWIDE: o.k = K_MULWIDE; break;
      case ZKL_OP_SABSORBN:
        if (z.n_regs < 1) return ZKL_E_INVALID;
        o.k = K_ABSORB;
        o.nabs = z.n_regs;
        for (int i = 0; i < z.n_regs; i++) {
          if (z.regs[i] > 7) return ZKL_E_INVALID;
          o.abs_regs[i] = z.regs[i];
        }
        break;
      case ZKL_OP_SSQUEEZE: o.k = K_SQUEEZE; break;
      case ZKL_OP_MERKLE_FIRST: o.k = K_MFIRST; break;
      case ZKL_OP_MERKLE_STEP: o.k = K_MSTEP; break;
      case ZKL_OP_MERKLE_LAST: o.k = K_MLAST; break;
      case ZKL_OP_LOAD: o.k = K_LOAD; break;
      case ZKL_OP_STORE: o.k = K_STORE; break;
      case ZKL_OP_END: o.k = K_END; break;
      default: return ZKL_E_INVALID;
    }
  }
  return ZKL_OK;
}
}  // namespace

extern "C" int zkl_build_trace(const zkl_op* ops_in, uint32_t n_ops, const uint8_t program_id[32],
                               const uint8_t program_commitment[32], const uint64_t* secret_args, uint32_t n_secret,
                               const zkl_vm_arg* main_args, uint32_t n_main, const zkl_f128* rom0_in,
                               zkl_f128* trace, zkl_air_public_inputs* pi, uint32_t* width_out,
                               uint32_t* n_rows_out) {
  if (!ops_in || n_ops == 0 || !program_id || !program_commitment) return ZKL_E_INVALID;
  if ((n_secret && !secret_args) || (n_main && !main_args) || n_main > ZKL_MAX_MAIN_SLOTS) return ZKL_E_INVALID;
  std::vector<Op> ops;
  if (int rc = to_ops(ops_in, n_ops, ops)) return rc;
  const size_t levels = ops.size();
  bool sponge, ram, merkle;
  features_of(ops, sponge, ram, merkle);
  const Layout L = make_layout(true, ram, sponge, merkle, true);
  const size_t n = levels * 32;
  if (width_out) *width_out = (uint32_t)L.width;
  if (n_rows_out) *n_rows_out = (uint32_t)n;
  if (!trace) return ZKL_OK;
  if (!pi) return ZKL_E_INVALID;
  std::vector<fe> slots;  // encode_main_args_to_slots (utils.rs:79-109)
  for (uint32_t i = 0; i < n_main; i++) {
    const zkl_vm_arg& a = main_args[i];
    if (a.tag == 0) { uint64_t x; memcpy(&x, a.bytes, 8); slots.push_back(fe{x, 0}); }
    else if (a.tag == 1) slots.push_back(be_from_le16(a.bytes));
    else if (a.tag == 2) { slots.push_back(be_from_le16(a.bytes)); slots.push_back(be_from_le16(a.bytes + 16)); }
    else return ZKL_E_INVALID;
  }
  if (slots.size() > 8) return ZKL_E_INVALID;  // "too many main_args for VM register file" (vm.rs:68-74)
  fe regs0[8] = {};
  const size_t tail = 8 - slots.size();  // secret args fill r0.., main-arg slots the tail (vm.rs:64-104)
  for (size_t i = 0; i < n_secret && i < tail; i++) regs0[i] = fe{secret_args[i], 0};
  for (size_t j = 0; j < slots.size(); j++) regs0[tail + j] = slots[j];
  return build_core(ops, program_id, program_commitment, sponge, ram, merkle, rom0_in ? fe_from(*rom0_in) : fe_zero(),
                    regs0, slots, n, trace, pi);
}

// rom_acc_from_program (romacc.rs:22-80): the ROM accumulator from the ops alone, over virtual
// map rows that hold each op's opcode bit and register selectors (encode_map_row_for_op,
// romacc.rs:82-260) — what the verifier recomputes for pi.rom_acc (prove.rs:815-821).
extern "C" int zkl_rom_acc_from_program(const zkl_op* ops_in, uint32_t n_ops, const uint8_t program_id[32],
                                        zkl_f128 out[3]) {
  if (!ops_in || !n_ops || !program_id || !out) return ZKL_E_INVALID;
  std::vector<Op> ops;
  if (int rc = to_ops(ops_in, n_ops, ops)) return rc;
  fe rc3[27][3], mds3[3][3], w0[59], w1[59];
  derive_rom_constants(program_id, rc3, mds3);
  {
    fe c = fe_mul(fe_pow64(fe{3, 0}, 17), fe{3, 0});
    for (int i = 0; i < 59; i++) { w0[i] = c; c = fe_mul(c, fe{3, 0}); }
    c = fe_mul(fe_pow64(fe{3, 0}, 1037), fe{3, 0});
    for (int i = 0; i < 59; i++) { w1[i] = c; c = fe_mul(c, fe{3, 0}); }
  }
  fe s[3] = {fe_zero(), fe_zero(), fe_zero()};
  for (const Op& o : ops) {
    // weights: 17 opcode bits, then dst0, a, b, c, dst1 selector groups of 8 (rom.rs encode order)
    int hot[6], nh = 0;
    const int oh = onehot_of(o.k);
    if (oh >= 0) hot[nh++] = oh;
    auto sel = [&](int group, int reg) { hot[nh++] = 17 + group * 8 + reg; };
    switch (o.k) {
      case K_CONST: case K_ADDR: case K_LOAD: sel(0, o.dst); if (o.k == K_LOAD) sel(1, o.a); break;
      case K_MOV: case K_NEG: sel(0, o.dst); sel(1, o.a); break;
      case K_ADD: case K_SUB: case K_MUL: case K_EQ: sel(0, o.dst); sel(1, o.a); sel(2, o.b); break;
      case K_SELECT: sel(0, o.dst); sel(1, o.a); sel(2, o.b); sel(3, o.c); break;
      case K_ASSERT: case K_ASSERT_BIT: case K_RANGE: case K_RANGE_LO: case K_RANGE_HI: sel(0, o.dst); sel(3, o.c); break;
      case K_DIVMOD: case K_DIV128: case K_MULWIDE: sel(0, o.dst); sel(4, o.dst2); sel(1, o.a); sel(2, o.b); break;
      case K_STORE: sel(1, o.a); sel(2, o.b); break;
      default: break;  // sponge: opcode bit only; Merkle steps, End, padding: nothing
    }
    fe e0 = fe_zero(), e1 = fe_zero();
    for (int i = 0; i < nh; i++) { e0 = fe_add(e0, w0[hot[i]]); e1 = fe_add(e1, w1[hot[i]]); }
    fe st[3] = {s[0], e0, e1};
    for (int j = 0; j < 27; j++) {
      const fe c3[3] = {fe_cube(st[0]), fe_cube(st[1]), fe_cube(st[2])};
      fe y[3];
      for (int i = 0; i < 3; i++)
        y[i] = fe_add(fe_add(fe_add(fe_mul(mds3[i][0], c3[0]), fe_mul(mds3[i][1], c3[1])), fe_mul(mds3[i][2], c3[2])),
                      rc3[j][i]);
      memcpy(st, y, sizeof st);
    }
    memcpy(s, st, sizeof s);
  }
  for (int i = 0; i < 3; i++) out[i] = to_abi(s[i]);
  return ZKL_OK;
}

// WinterfellSegmentPlanner::plan_segments (segment_planner.rs:93-276): the level ranges tile
// [0, next_pow2(n_ops)) contiguously, so the segments are consecutive runs of
// max(max_rows / 32, 1) levels (one segment when the trace fits).
extern "C" int zkl_plan_segments(uint32_t n_ops, uint32_t max_rows, uint32_t* r_starts, uint32_t* r_ends,
                                 uint32_t cap, uint32_t* count) {
  if (!n_ops || !count) return ZKL_E_INVALID;
  size_t levels = 1;
  while (levels < n_ops) levels <<= 1;
  const size_t rows = levels * 32;
  const size_t per = rows <= max_rows ? levels : std::max<size_t>(max_rows / 32, 1);
  const size_t k = (levels + per - 1) / per;
  *count = (uint32_t)k;
  if (!r_starts || !r_ends) return ZKL_OK;
  if (cap < k) return ZKL_E_INVALID;
  for (size_t i = 0; i < k; i++) {
    r_starts[i] = (uint32_t)(i * per * 32);
    r_ends[i] = (uint32_t)(std::min(levels, (i + 1) * per) * 32);
  }
  return ZKL_OK;
}

namespace {
// utils::vm_state_hash_row_with_layout (utils.rs:312-339): BLAKE3("zkl/vm/state-v1" | r0..r7 as
// 16-byte LE integers) of one row
void vm_state_hash(const Table& T, const Layout& L, size_t row, uint8_t out[32]) {
  uint8_t buf[15 + 8 * 16];
  memcpy(buf, "zkl/vm/state-v1", 15);
  for (int i = 0; i < 8; i++) {
    const fe v = T.get(L.r_start + i, row);
    for (int b = 0; b < 8; b++) {
      buf[15 + 16 * i + b] = (uint8_t)(v.lo >> (8 * b));
      buf[15 + 16 * i + 8 + b] = (uint8_t)(v.hi >> (8 * b));
    }
  }
  blake3_hash(buf, sizeof buf, out);
}
}  // namespace

// prove_segment's trace and public inputs for rows [r_start, r_end) of a full trace
// (prove.rs:1057-1134): the segment's own feature mask from the ops of its levels
// (compute_segment_features_for_levels / compute_segment_feature_mask, segment_planner.rs:283-334;
// used when it differs from the program's), the columns of that layout sliced out of the full
// trace (slice_trace_segment_with_layout, mod.rs), the boundary values
// (compute_segment_boundary_bytes, prove.rs:1197-1287), the segment-local VM output and usage
// mask (build_air_pi_for_trace, prove.rs:292-423) and the VM state hashes at its first and last
// rows (build_segment_trace_with_state_without_full).
extern "C" int zkl_slice_segment(const zkl_f128* full, uint32_t full_width, uint32_t n_full, const zkl_op* ops_in,
                                 uint32_t n_ops, const zkl_air_public_inputs* pi_full, uint32_t r_start,
                                 uint32_t r_end, zkl_f128* trace_out, zkl_air_public_inputs* pi_out,
                                 uint32_t* width_out, uint8_t state_in[32], uint8_t state_out[32]) {
  if (!full || !ops_in || !pi_full || r_start >= r_end || r_end > n_full) return ZKL_E_INVALID;
  if (r_start % 32 || r_end % 32) return ZKL_E_INVALID;  // segments aligned to full levels
  const size_t m = r_end - r_start;
  if (m & (m - 1)) return ZKL_E_INVALID;  // a Winterfell trace length
  std::vector<Op> ops;
  if (int rc = to_ops(ops_in, n_ops, ops)) return rc;
  if (ops.size() * 32 != n_full) return ZKL_E_INVALID;
  bool sp, rm, mk;
  features_of(ops, sp, rm, mk);
  const Layout LF = make_layout(true, rm, sp, mk, true);
  if (LF.width != (int)full_width) return ZKL_E_INVALID;
  // segment features over the program levels it covers (pad levels contribute none)
  const size_t l0 = r_start / 32, l1 = std::min<size_t>(r_end / 32, n_ops);
  std::vector<Op> seg_ops;
  for (size_t l = l0; l < l1; l++) seg_ops.push_back(ops[l]);
  bool ssp, srm, smk;
  features_of(seg_ops, ssp, srm, smk);
  const uint64_t base = pi_full->feature_mask;
  uint64_t seg = 0;
  if (base & FM_VM) seg |= FM_VM;
  if (base & FM_VM_EXPECT) seg |= FM_VM_EXPECT;
  if ((base & FM_RAM) && srm) seg |= FM_RAM;
  if ((base & FM_MERKLE) && smk) seg |= FM_MERKLE;
  if ((base & FM_SPONGE) && ssp) seg |= FM_SPONGE;
  if ((base & FM_POSEIDON) && (ssp || smk)) seg |= FM_POSEIDON;
  const uint64_t eff = (seg != 0 && seg != base) ? seg : base;
  const bool e_ram = eff & FM_RAM, e_merkle = eff & FM_MERKLE;
  const Layout LS = make_layout(true, e_ram, (eff & FM_SPONGE) != 0, e_merkle, true);
  if (width_out) *width_out = (uint32_t)LS.width;
  if (!trace_out) return ZKL_OK;
  if (!pi_out) return ZKL_E_INVALID;
  if ((e_ram && !rm) || (e_merkle && !mk)) return ZKL_E_INVALID;  // a block the full trace lacks
  // segment column -> full column: identical prefix, the optional RAM / Merkle blocks, then the
  // tail from pi_prog on
  auto full_col = [&](int c) {
    if (c < LS.ram_sorted) return c;
    if (e_ram && c < LS.ram_sorted + 8) return LF.ram_sorted + (c - LS.ram_sorted);
    if (e_merkle && c >= LS.merkle_g && c < LS.merkle_g + 7) return LF.merkle_g + (c - LS.merkle_g);
    return LF.pi_prog + (c - LS.pi_prog);
  };
  for (int c = 0; c < LS.width; c++)
    memcpy(trace_out + (size_t)c * m, full + (size_t)full_col(c) * n_full + r_start, m * sizeof(zkl_f128));
  const Table TF{const_cast<zkl_f128*>(full), n_full};
  const Table TS{trace_out, m};
  *pi_out = *pi_full;  // core inputs: ids, commitment, merkle root, base mask, main slots, rom_acc
  pi_out->segment_feature_mask = eff;
  pi_out->pc_init = to_abi(TF.get(LF.pc, r_start));
  if (rm) {
    pi_out->ram_gp_unsorted_in = to_abi(TF.get(LF.ram_gp_unsorted, r_start));
    pi_out->ram_gp_unsorted_out = to_abi(TF.get(LF.ram_gp_unsorted, r_end - 1));
    pi_out->ram_gp_sorted_in = to_abi(TF.get(LF.ram_gp_sorted, r_start));
    pi_out->ram_gp_sorted_out = to_abi(TF.get(LF.ram_gp_sorted, r_end - 1));
  } else {
    pi_out->ram_gp_unsorted_in = pi_out->ram_gp_unsorted_out = to_abi(fe_zero());
    pi_out->ram_gp_sorted_in = pi_out->ram_gp_sorted_out = to_abi(fe_zero());
  }
  for (int i = 0; i < 3; i++) {
    pi_out->rom_s_in[i] = to_abi(TF.get(LF.rom_s + i, r_start));
    pi_out->rom_s_out[i] = to_abi(TF.get(LF.rom_s + i, r_end - 32 + 28));
  }
  derive_trace_pi(TS, LS, e_ram, m / 32, pi_out);
  if (state_in) vm_state_hash(TS, LS, 0, state_in);
  if (state_out) vm_state_hash(TS, LS, m - 1, state_out);
  return ZKL_OK;
}
