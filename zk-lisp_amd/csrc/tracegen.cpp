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
  K_LOAD = 15, K_STORE = 16, K_MFIRST = 20, K_MSTEP = 21, K_MLAST = 22, K_END = 99
};
// Merkle steps: dst = leaf register, a = dir register, b = sibling register
struct Op { Kind k; int dst, a, b; uint64_t imm; int nabs; int abs_regs[3]; };
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
    const Op m[5] = {{K_CONST, 5, 0, 0, r & 1, 0, {}}, {K_CONST, 6, 0, 0, (r >> 1) & 1, 0, {}},
                     {K_MFIRST, 0, 5, 1, 0, 0, {}}, {K_MSTEP, 0, 6, 2, 0, 0, {}}, {K_MLAST, 0, 5, 3, 0, 0, {}}};
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

extern "C" int zkl_synth_vm_segment_chain(uint64_t program_seed, uint64_t seed, uint32_t log_n, uint32_t flags, const zkl_f128* rom0_in,
                                          zkl_f128* trace, zkl_air_public_inputs* pi, uint32_t* width_out) {
  const uint32_t all = ZKL_SYN_SPONGE | ZKL_SYN_RAM | ZKL_SYN_MERKLE;
  if ((flags & ~all) || log_n < 5 || log_n > 26) return ZKL_E_INVALID;
  if ((flags & ZKL_SYN_MERKLE) && log_n < 8) return ZKL_E_INVALID;  // the path needs 8 levels
  const bool sponge = flags & ZKL_SYN_SPONGE, ram = flags & ZKL_SYN_RAM, merkle = flags & ZKL_SYN_MERKLE;
  const Layout L = make_layout(true, ram, sponge, merkle, true);
  if (width_out) *width_out = (uint32_t)L.width;
  if (!trace) return ZKL_OK;
  if (!pi) return ZKL_E_INVALID;
  const size_t n = (size_t)1 << log_n, levels = n / 32;
  memset(trace, 0, sizeof(zkl_f128) * L.width * n);
  memset(pi, 0, sizeof *pi);
  Table T{trace, n};

  char desc[160];
  snprintf(desc, sizeof desc, "zkl-hip/synthetic-vm-segment/v1 %s%s%sseed=0x%016llx levels=%zu",
           sponge ? "sponge " : "", ram ? "ram " : "", merkle ? "merkle " : "", (unsigned long long)program_seed, levels);
  uint8_t pid[32];
  blake3_hash((const uint8_t*)desc, strlen(desc), pid);
  PoseidonSuite ps = derive_poseidon_suite(pid, 27);
  const std::vector<Op> ops = make_program(seed, levels, flags);

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
  std::vector<RamEvent> events;
  std::vector<std::pair<fe, fe>> mem;  // host memory: address -> last stored value
  long last_merkle = -1;
  for (size_t l = 0; l < levels; l++) {
    fe next[8];
    memcpy(next, regs, sizeof next);
    size_t b = l * 32, rm = b, rf = b + 28;
    if (l == 0) T.set(L.pi_prog, 0, be_from_le16(pid));
    const Op& o = ops[l];
    switch (o.k) {
      case K_ABSORB:
      case K_SQUEEZE: {  // SAbsorbN / SSqueeze (vm.rs:565-672)
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
        T.set(L.rom_op_start + oh, rm, fe_one());
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
      default: {  // ALU: Const / address const / Mov / Add / Sub / Mul
        const int oh = o.k == K_ADDR ? (int)K_CONST : (int)o.k;
        const bool is_const = o.k == K_CONST || o.k == K_ADDR;
        T.set(L.rom_op_start + oh, rm, fe_one());
        for (size_t row : {rm, rf}) {
          T.set(L.op[oh], row, fe_one());
          T.sel(row, L.sel_dst0, o.dst);
          if (is_const) T.set(L.imm, row, fe{o.imm, 0});
          else T.sel(row, L.sel_a, o.a);
          if (o.k == K_ADD || o.k == K_SUB || o.k == K_MUL) T.sel(row, L.sel_b, o.b);
        }
        switch (o.k) {
          case K_CONST:
          case K_ADDR: next[o.dst] = fe{o.imm, 0}; break;
          case K_MOV: next[o.dst] = regs[o.a]; break;
          case K_ADD: next[o.dst] = fe_add(regs[o.a], regs[o.b]); break;
          case K_SUB: next[o.dst] = fe_sub(regs[o.a], regs[o.b]); break;
          case K_MUL: next[o.dst] = fe_mul(regs[o.a], regs[o.b]); break;
          default: break;
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
  fe s0_prev = rom0_in ? fe_from(*rom0_in) : fe_zero();  // ROM lane 0 carries across segments
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
  pi->feature_mask = FM_VM | (sponge ? FM_SPONGE | FM_POSEIDON : 0) | (ram ? FM_RAM : 0) |
                     (merkle ? FM_MERKLE | FM_POSEIDON : 0);
  pi->segment_feature_mask = pi->feature_mask;
  if (merkle) {  // root = acc after the MerkleStepLast level, 16 LE bytes (utils.rs:346-355)
    const fe root = T.get(L.merkle_acc, 5 * 32 + 28);
    for (int i = 0; i < 8; i++) {
      pi->merkle_root[i] = (uint8_t)(root.lo >> (8 * i));
      pi->merkle_root[8 + i] = (uint8_t)(root.hi >> (8 * i));
    }
  }
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
  return ZKL_OK;
}
