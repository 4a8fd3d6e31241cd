// Trace builder (host): zk-lisp programs -- the compiler's builder::Op lists and the synthetic
// generator below -- executed and laid out the way the reference's trace builder does it
// (vm/trace/mod.rs:386-524, vm/trace/vm.rs:58-888, vm/trace/ram.rs:43-271,
// vm/trace/rom.rs:29-108), directly in the segment layout the feature set implies
// (vm/trace/mod.rs:80-235), plus the AIR public inputs prove_segment derives (prove.rs:292-423,
// 1197-1392).
//
// One program run (Run) executes the ops once and keeps what any window of levels needs: the VM
// carry (registers, pending absorbs, Merkle accumulator, memory-event count, ROM lane 0) every
// CK levels, the RAM event log with the sorted table's running sums, the final ROM state and the
// Merkle root.  A window of levels is then written from the nearest checkpoint: the whole trace
// (zkl_build_trace) or one segment in its own layout (zkl_build_segment_trace), which is what
// build_full_trace followed by slice_trace_segment_with_layout gives (mod.rs:316-380,
// prove.rs:1103-1113) without the full trace in memory -- examples/fib-2pow16.zlisp has 2^24
// rows (~55 GB at 204 columns) in 256 segments of 2^16.
//
// Synthetic program (splitmix64 choices, immediates < 2^63, End on the last level):
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
#include <map>
#include <string>
#include <utility>
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
bool fe_less(fe a, fe b) { return a.hi != b.hi ? a.hi < b.hi : a.lo < b.lo; }
constexpr int ADDR_REG = 7;
constexpr size_t CK = 32;  // levels between two carry checkpoints

struct RamEvent { fe addr, clk, val, w; };

// Rows [base, base + n) of a column-major trace.  map (optional): layout column -> column of
// t, -1 where t's (segment) layout drops it; writes to dropped columns are ignored.
struct Table {
  zkl_f128* t;
  size_t n;
  size_t base = 0;
  const int* map = nullptr;
  int col_of(int col) const { return map ? map[col] : col; }
  void set(int col, size_t row, fe v) {
    const int c = col_of(col);
    if (c >= 0) t[(size_t)c * n + (row - base)] = to_abi(v);
  }
  fe get(int col, size_t row) const {
    const int c = col_of(col);
    return c >= 0 ? fe_from(t[(size_t)c * n + (row - base)]) : fe_zero();
  }
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

// The VM carry entering a level.
struct Carry {
  fe regs[8];
  int pending[10];
  int npending;
  fe merkle_out;  // accumulator after the last Merkle level (MerkleStep reads it, vm.rs:700-720)
  size_t ev;      // memory events of the levels before
  fe rom0;        // ROM lane 0 entering the level (rom.rs:37-106)
};

// One program: ops, layout, constants and the pre-pass (prepass()).
struct Run {
  std::vector<Op> ops;
  size_t levels = 0;
  bool sponge = false, ram = false, merkle = false;
  Layout L{};
  uint8_t pid[32], commit[32];
  std::vector<fe> slots;
  Carry init{};
  PoseidonSuite ps;
  fe rc3[27][3], mds3[3][3], w0[59], w1[59];
  fe ram_r[3];  // RAM compressor coefficients (ram.rs:112-121)
  // pre-pass
  std::vector<Carry> cks;         // carry entering level i * CK
  std::vector<RamEvent> events;   // memory events in level order (clk = level)
  std::vector<RamEvent> sorted;   // the same by (addr, clk): the sorted table
  std::vector<fe> gp_sorted;      // gp_sorted[k]: sum of the first k sorted compressions
  std::vector<fe> last_write;     // ram_s_last_write after k sorted rows
  std::vector<fe> gp_unsorted;    // gp_unsorted[k]: sum of the first k level-order compressions
  fe rom_final[3];
  fe merkle_root = fe_zero();
  bool has_root = false;
};

void rom_weights(uint64_t seed, fe out[59]) {  // utils.rs:95-121
  fe c = fe_mul(fe_pow64(fe{3, 0}, seed), fe{3, 0});
  for (int i = 0; i < 59; i++) { out[i] = c; c = fe_mul(c, fe{3, 0}); }
}

void init_run(Run& R, const uint8_t pid[32], const uint8_t commit[32], bool sponge, bool ram, bool merkle) {
  R.sponge = sponge;
  R.ram = ram;
  R.merkle = merkle;
  R.L = make_layout(true, ram, sponge, merkle, true);
  memcpy(R.pid, pid, 32);
  memcpy(R.commit, commit, 32);
  R.ps = derive_poseidon_suite(pid, 27);
  derive_rom_constants(pid, R.rc3, R.mds3);
  rom_weights(17, R.w0);
  rom_weights(1037, R.w1);
  fe pfe[2];
  program_field_commitment(pid, pfe);
  const fe q0 = pfe[0], q2 = fe_mul(q0, q0), q3 = fe_mul(q2, q0), q5 = fe_mul(fe_mul(q2, q2), q0);
  R.ram_r[0] = fe_add(q2, fe_one());
  R.ram_r[1] = fe_add(q3, q0);
  R.ram_r[2] = fe_add(q5, fe{7, 0});
}

fe ram_compress(const Run& R, const RamEvent& e) {
  return fe_add(fe_add(fe_add(e.addr, fe_mul(R.ram_r[0], e.clk)), fe_mul(R.ram_r[1], e.val)), fe_mul(R.ram_r[2], e.w));
}

// One level's Poseidon lanes (vm/trace/poseidon.rs:9-87): map row = [inputs (zero padded
// to 10), dom0, dom1]; round row 1+j = state before round j; final and pad rows = output.
// Returns lane 0 of the output (written only when T is given).
fe level_absorb(Table* T, const Layout& L, const PoseidonSuite& ps, size_t level, const fe* in, int nin) {
  const size_t b = level * 32;
  fe st[12];
  for (int i = 0; i < 12; i++) st[i] = fe_zero();
  for (int i = 0; i < nin && i < 10; i++) st[i] = in[i];
  st[10] = ps.dom[0];
  st[11] = ps.dom[1];
  if (T) for (int i = 0; i < 12; i++) T->set(L.lanes_start + i, b, st[i]);
  for (int j = 0; j < 27; j++) {
    if (T) for (int i = 0; i < 12; i++) T->set(L.lanes_start + i, b + 1 + j, st[i]);
    fe s3[12], y[12];
    for (int i = 0; i < 12; i++) s3[i] = fe_cube(st[i]);
    for (int i = 0; i < 12; i++) {
      fe acc = fe_zero();
      for (int k = 0; k < 12; k++) acc = fe_add(acc, fe_mul(ps.mds[i][k], s3[k]));
      y[i] = fe_add(acc, ps.rc[j][i]);
    }
    memcpy(st, y, sizeof st);
  }
  if (T)
    for (size_t r = b + 28; r < b + 32; r++)
      for (int i = 0; i < 12; i++) T->set(L.lanes_start + i, r, st[i]);
  return st[0];
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

using MemMap = std::map<std::pair<uint64_t, uint64_t>, fe>;  // (hi, lo) address -> last stored value

// One level of build_full_trace: schedule gates, pc and domain tags (mod.rs:386-470) and
// VmTraceBuilder::fill_table for its op (vm.rs:58-888).  T: the rows to write (nullptr: only
// advance the carry).  mem: the pre-pass memory (unwritten addresses read 0); its loads and
// stores append to *log.  Without it a load reads its value from R.events.
int vm_level(const Run& R, size_t l, Carry& c, Table* T, MemMap* mem, std::vector<RamEvent>* log) {
  const Layout& L = R.L;
  const size_t b = l * 32, rm = b, rf = b + 28;
  if (T) {
    T->set(L.g_map, b, fe_one());
    T->set(L.g_final, b + 28, fe_one());
    for (int j = 0; j < 27; j++) T->set(L.g_r_start + j, b + 1 + j, fe_one());
    for (size_t r = b; r < b + 32; r++) T->set(L.pc, r, fe{l, 0});
    T->set(L.lanes_start + 10, b, R.ps.dom[0]);
    T->set(L.lanes_start + 11, b, R.ps.dom[1]);
  }
  const Op& o = R.ops[l];
  if (o.k == K_PAD) return ZKL_OK;  // levels past the program: build_empty_trace rows only
  fe next[8];
  memcpy(next, c.regs, sizeof next);
  const fe* regs = c.regs;
  if (T) {
    if (l == 0) T->set(L.pi_prog, 0, be_from_le16(R.pid));
    const int oh = onehot_of(o.k);
    if (oh >= 0) T->set(L.rom_op_start + oh, rm, fe_one());
  }
  switch (o.k) {
    case K_ABSORB:
    case K_SQUEEZE: {  // SAbsorbN / SSqueeze (vm.rs:565-672)
      int sel_regs[10], k = 0;
      if (o.k == K_ABSORB) {
        for (int i = 0; i < o.nabs; i++) {
          if (c.npending >= 10) return ZKL_E_INVALID;  // push_absorb: sponge rate overflow (vm.rs:925-935)
          sel_regs[k++] = o.abs_regs[i];
          c.pending[c.npending++] = o.abs_regs[i];
        }
      } else {
        for (int i = 0; i < c.npending; i++) sel_regs[k++] = c.pending[i];
      }
      if (T)
        for (size_t row : {rm, rf}) {
          T->set(L.op[8], row, fe_one());
          T->sponge_sel(L, row, sel_regs, k);
        }
      if (o.k == K_SQUEEZE) {
        if (T) T->sel(rf, L.sel_dst0, o.dst);
        fe in[10];
        for (int i = 0; i < k; i++) in[i] = regs[sel_regs[i]];
        next[o.dst] = level_absorb(T, L, R.ps, l, in, k);
        c.npending = 0;
        if (T) for (size_t r = b; r < b + 32; r++) T->set(L.pose_active, r, fe_one());
      }
      break;
    }
    case K_MFIRST:
    case K_MSTEP:
    case K_MLAST: {  // MerkleStepFirst / MerkleStep / MerkleStepLast (vm.rs:675-800)
      const fe acc = o.k == K_MFIRST ? regs[o.dst] : c.merkle_out;
      const fe d = regs[o.a], sib = regs[o.b], nd = fe_sub(fe_one(), d);
      if (T) {
        for (size_t r = b; r < b + 32; r++) T->set(L.merkle_g, r, fe_one());
        if (o.k == K_MFIRST) {
          T->set(L.merkle_first, rm, fe_one());
          T->set(L.merkle_leaf, rm, acc);
        }
        for (size_t r = rm; r < rf; r++) T->set(L.merkle_acc, r, acc);
        T->set(L.merkle_dir, rm, d);
        T->set(L.merkle_sib, rm, sib);
      }
      const fe in[2] = {fe_add(fe_mul(nd, acc), fe_mul(d, sib)), fe_add(fe_mul(nd, sib), fe_mul(d, acc))};
      const fe out = level_absorb(T, L, R.ps, l, in, 2);
      if (T) {
        if (o.k == K_MLAST) T->set(L.merkle_last, rf, fe_one());
        for (size_t r = rf; r < b + 32; r++) T->set(L.merkle_acc, r, out);
        for (size_t r = b; r < b + 32; r++) T->set(L.pose_active, r, fe_one());
      }
      c.merkle_out = out;
      break;
    }
    case K_LOAD:
    case K_STORE: {  // Load / Store (vm.rs:803-842): clk = level; unwritten addresses read 0
      const int oh = o.k == K_LOAD ? 15 : 16;
      const fe addr = regs[o.a];
      fe val;
      if (o.k == K_STORE) {
        val = regs[o.b];
        if (mem) (*mem)[{addr.hi, addr.lo}] = val;
      } else if (mem) {
        auto it = mem->find({addr.hi, addr.lo});
        val = it != mem->end() ? it->second : fe_zero();
      } else {
        if (c.ev >= R.events.size()) return ZKL_E_INTERNAL;
        val = R.events[c.ev].val;  // the value the pre-pass logged for this level
      }
      if (T) {
        for (size_t row : {rm, rf}) {
          T->set(L.op[oh], row, fe_one());
          T->sel(row, L.sel_a, o.a);
          if (o.k == K_LOAD) T->sel(row, L.sel_dst0, o.dst);
          else T->sel(row, L.sel_b, o.b);
        }
        if (o.k == K_LOAD) {
          T->set(L.imm, rm, val);
          T->set(L.imm, rf, val);
        }
      }
      if (o.k == K_LOAD) next[o.dst] = val;
      if (log) log->push_back({addr, fe{l, 0}, val, o.k == K_STORE ? fe_one() : fe_zero()});
      c.ev++;
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
          if (T) eqinv = fe_is_zero(diff) ? fe_zero() : fe_inv(diff);
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
          if (T) eqinv = bv != 0 ? fe_inv(from_u64((uint64_t)bv)) : fe_zero();
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
          if (T) eqinv = cu != 0 ? fe_inv(from_u64((uint64_t)cu)) : fe_zero();
          break;
        }
        default: return ZKL_E_INVALID;
      }
      if (T)
        for (size_t row : {rm, rf}) {
          T->set(L.op[oh], row, fe_one());
          T->sel(row, L.sel_dst0, o.dst);
          if (has_d2) T->sel(row, L.sel_dst1, o.dst2);
          if (has_a) T->sel(row, L.sel_a, o.a);
          if (has_b) T->sel(row, L.sel_b, o.b);
          if (has_c) T->sel(row, L.sel_c, o.c);
          T->set(L.imm, row, imm);
          T->set(L.eq_inv, row, eqinv);
          if (gadget)
            for (int i = 0; i < 32; i++) T->set(L.gadget_b + i, row, bitsv[i]);
        }
    }
  }
  if (T) {
    for (size_t r = rm; r <= rf; r++) for (int i = 0; i < 8; i++) T->set(L.r_start + i, r, regs[i]);
    for (size_t r = rf + 1; r < b + 32; r++) for (int i = 0; i < 8; i++) T->set(L.r_start + i, r, next[i]);
  }
  memcpy(c.regs, next, sizeof next);
  return ZKL_OK;
}

// encode_map_row_for_op (romacc.rs:82-260): the 59 ROM weights of an op's map row -- its
// one-hot opcode bit (vm.rs:890-922) and the register selectors the VM writes there, in
// rom.rs's order (17 opcode bits, then the dst0, a, b, c, dst1 groups of 8).
void rom_enc_op(const Run& R, const Op& o, fe e[2]) {
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
  e[0] = e[1] = fe_zero();
  for (int i = 0; i < nh; i++) { e[0] = fe_add(e[0], R.w0[hot[i]]); e[1] = fe_add(e[1], R.w1[hot[i]]); }
}

// RomTraceBuilder (rom.rs:37-106) over level l: state (lane 0 carried in, the two encodings of
// the map row) at the map row, the state before round j on row 1 + j, the output on the final
// and pad rows.  With T the encodings are read from the level's map row, else from the op.
void rom_level(const Run& R, size_t l, fe s0, Table* T, fe out[3]) {
  const Layout& L = R.L;
  const size_t b = l * 32;
  fe s[3] = {s0, fe_zero(), fe_zero()};
  if (T) {
    const int st[5] = {L.sel_dst0, L.sel_a, L.sel_b, L.sel_c, L.sel_dst1};
    for (int q = 0; q < 2; q++) {
      const fe* w = q ? R.w1 : R.w0;
      fe acc = fe_zero();
      int k = 0;
      for (int i = 0; i < 17; i++) acc = fe_add(acc, fe_mul(T->get(L.op[i], b), w[k++]));
      for (int g = 0; g < 5; g++) for (int i = 0; i < 8; i++) acc = fe_add(acc, fe_mul(T->get(st[g] + i, b), w[k++]));
      s[1 + q] = acc;
    }
    for (int i = 0; i < 3; i++) T->set(L.rom_s + i, b, s[i]);
  } else {
    rom_enc_op(R, R.ops[l], s + 1);
  }
  for (int j = 0; j < 27; j++) {
    const size_t r = b + 1 + j;
    if (T) for (int i = 0; i < 3; i++) T->set(L.rom_s + i, r, s[i]);
    const fe c3[3] = {fe_cube(s[0]), fe_cube(s[1]), fe_cube(s[2])};
    fe y[3];
    for (int i = 0; i < 3; i++)
      y[i] = fe_add(fe_add(fe_add(fe_mul(R.mds3[i][0], c3[0]), fe_mul(R.mds3[i][1], c3[1])), fe_mul(R.mds3[i][2], c3[2])),
                    R.rc3[j][i]);
    if (T) for (int i = 0; i < 3; i++) T->set(L.rom_s + i, r + 1, y[i]);
    memcpy(s, y, sizeof s);
  }
  if (T) for (size_t r = b + 29; r < b + 32; r++) for (int i = 0; i < 3; i++) T->set(L.rom_s + i, r, s[i]);
  memcpy(out, s, sizeof s);
}

void ram_last_writes(Run& R, size_t n);

// Executes the whole program once: carry checkpoints, the memory-event log, ROM lane 0 per
// checkpoint and the final ROM state (rom_acc), the Merkle root (the accumulator after the last
// MerkleStepLast, utils.rs:346-355), and the RAM table's running sums (ram.rs:43-271).
int prepass(Run& R) {
  Carry c = R.init;
  MemMap mem;
  R.cks.clear();
  R.events.clear();
  fe s[3] = {c.rom0, fe_zero(), fe_zero()};
  for (size_t l = 0; l < R.levels; l++) {
    if (l % CK == 0) R.cks.push_back(c);
    if (int rc = vm_level(R, l, c, nullptr, &mem, &R.events)) return rc;
    if (R.ops[l].k == K_MLAST) { R.merkle_root = c.merkle_out; R.has_root = true; }
    rom_level(R, l, c.rom0, nullptr, s);
    c.rom0 = s[0];
  }
  memcpy(R.rom_final, s, sizeof s);
  // the sorted table: (addr, clk) keys, clocks unique per address (one event per level)
  R.sorted = R.events;
  std::stable_sort(R.sorted.begin(), R.sorted.end(), [](const RamEvent& x, const RamEvent& y) {
    if (!fe_eq(x.addr, y.addr)) return fe_less(x.addr, y.addr);
    return fe_less(x.clk, y.clk);
  });
  const size_t E = R.sorted.size();
  R.gp_sorted.assign(E + 1, fe_zero());
  R.last_write.assign(E + 1, fe_zero());
  R.gp_unsorted.assign(R.events.size() + 1, fe_zero());
  for (size_t k = 0; k < E; k++) R.gp_sorted[k + 1] = fe_add(R.gp_sorted[k], ram_compress(R, R.sorted[k]));
  for (size_t k = 0; k < R.events.size(); k++)
    R.gp_unsorted[k + 1] = fe_add(R.gp_unsorted[k], ram_compress(R, R.events[k]));
  ram_last_writes(R, R.levels * 32);
  return ZKL_OK;
}

// The sorted RAM table as rows (ram.rs:43-271): event k sits on row 32 (k / 3) + 29 + k % 3 (the
// pad rows of consecutive levels); the rows between two same-address events of neighbouring
// levels (rows 0..28 of the later level) mirror the earlier one.  Returns the event shown on
// row r (nullptr: zeros) and whether r is a sorted row.
const RamEvent* ram_row(const Run& R, size_t r, bool* sorted) {
  const size_t p = r % 32, lv = r / 32, E = R.sorted.size();
  *sorted = false;
  if (p >= 29) {
    const size_t k = 3 * lv + (p - 29);
    if (k < E) { *sorted = true; return &R.sorted[k]; }
    return nullptr;
  }
  if (lv == 0) return nullptr;
  const size_t i = 3 * lv - 1;
  if (i + 1 < E && fe_eq(R.sorted[i].addr, R.sorted[i + 1].addr)) return &R.sorted[i];
  return nullptr;
}
// sorted rows above row r
size_t ram_sorted_before(const Run& R, size_t r) {
  const size_t p = r % 32;
  return std::min(R.sorted.size(), 3 * (r / 32) + (p > 29 ? p - 29 : 0));
}
// level-order events whose final row lies above row r (the unsorted sum adds a level's event on
// the row after its final row)
size_t ram_events_before(const Run& R, size_t r) {
  if (r < 29) return 0;
  const uint64_t last_level = (r - 29) / 32;
  return std::upper_bound(R.events.begin(), R.events.end(), last_level,
                          [](uint64_t v, const RamEvent& e) { return v < e.clk.lo; }) -
         R.events.begin();
}
fe ram_gp_sorted_at(const Run& R, size_t r) { return R.gp_sorted[ram_sorted_before(R, r)]; }
fe ram_gp_unsorted_at(const Run& R, size_t r) { return R.gp_unsorted[ram_events_before(R, r)]; }

// ram_s_last_write after each sorted row: updated on the row after a sorted row, continued when
// that row shows the same address, restarted otherwise
void ram_last_writes(Run& R, size_t n) {
  const size_t E = R.sorted.size();
  for (size_t k = 0; k < E; k++) {
    const RamEvent& e = R.sorted[k];
    const size_t row = 32 * (k / 3) + 29 + k % 3 + 1;
    bool s;
    const RamEvent* nx = row < n ? ram_row(R, row, &s) : nullptr;
    const fe a_next = nx ? nx->addr : fe_zero();
    const fe prev = R.last_write[k];
    R.last_write[k + 1] = fe_eq(a_next, e.addr) ? fe_add(fe_mul(fe_sub(fe_one(), e.w), prev), fe_mul(e.w, e.val))
                                                : fe_mul(e.w, e.val);
  }
}

// RamTraceBuilder::fill_table (ram.rs:43-271) on rows [r0, r1) of an n-row trace
void ram_window(const Run& R, Table& T, size_t r0, size_t r1, size_t n) {
  const Layout& L = R.L;
  size_t ev = ram_events_before(R, r0);
  for (size_t r = r0; r < r1; r++) {
    bool sorted;
    const RamEvent* e = ram_row(R, r, &sorted);
    if (sorted) T.set(L.ram_sorted, r, fe_one());
    if (e) {
      T.set(L.ram_s_addr, r, e->addr);
      T.set(L.ram_s_clk, r, e->clk);
      T.set(L.ram_s_val, r, e->val);
      T.set(L.ram_s_is_write, r, e->w);
    }
    const size_t k = ram_sorted_before(R, r);
    T.set(L.ram_gp_sorted, r, R.gp_sorted[k]);
    T.set(L.ram_s_last_write, r, R.last_write[k]);
    if (sorted && r + 1 < n) {
      bool sn;
      const RamEvent* en = ram_row(R, r + 1, &sn);
      const fe an = en ? en->addr : fe_zero();
      T.set(L.eq_inv, r, fe_inv(fe_sub(an, e->addr)));
      if (sn && fe_eq(an, e->addr)) {  // delta_clk bits (saturating as_int difference)
        const bool pos = fe_less(e->clk, en->clk);
        const uint64_t d = pos ? en->clk.lo - e->clk.lo : 0;  // clocks are level indices (< 2^64)
        for (int i = 0; i < 32; i++) T.set(L.gadget_b + i, r, fe{(d >> i) & 1, 0});
      }
    }
    while (ev < R.events.size() && r >= 32 * R.events[ev].clk.lo + 29) ev++;
    T.set(L.ram_gp_unsorted, r, R.gp_unsorted[ev]);
  }
}

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

uint64_t program_mask(const Run& R) {
  return FM_VM | (R.sponge ? FM_SPONGE | FM_POSEIDON : 0) | (R.ram ? FM_RAM : 0) |
         (R.merkle ? FM_MERKLE | FM_POSEIDON : 0);
}

// The program-level public inputs every segment shares: ids, commitment, feature mask, main-arg
// slots, Merkle root, rom_acc (prove.rs:292-423)
void core_pi(const Run& R, zkl_air_public_inputs* pi) {
  memset(pi, 0, sizeof *pi);
  memcpy(pi->program_id, R.pid, 32);
  memcpy(pi->program_commitment, R.commit, 32);
  pi->feature_mask = pi->segment_feature_mask = program_mask(R);
  pi->n_main_slots = (uint32_t)R.slots.size();
  for (size_t i = 0; i < R.slots.size(); i++) pi->main_slots[i] = to_abi(R.slots[i]);
  if (R.merkle && R.has_root)  // root = acc after the (last) MerkleStepLast level, 16 LE bytes
    for (int i = 0; i < 8; i++) {
      pi->merkle_root[i] = (uint8_t)(R.merkle_root.lo >> (8 * i));
      pi->merkle_root[8 + i] = (uint8_t)(R.merkle_root.hi >> (8 * i));
    }
  for (int i = 0; i < 3; i++) pi->rom_acc[i] = to_abi(R.rom_final[i]);
}

// Rows of levels [l0, l1) written into out (m = 32 (l1 - l0) rows, column-major in the layout
// whose columns map gives, or R.L), with the VM and ROM carried in from the checkpoint before l0.
int build_window(const Run& R, size_t l0, size_t l1, zkl_f128* out, int out_width, const int* map) {
  const size_t m = (l1 - l0) * 32, n = R.levels * 32;
  memset(out, 0, sizeof(zkl_f128) * (size_t)out_width * m);
  Table T{out, m, l0 * 32, map};
  Carry c = R.cks[l0 / CK];
  fe s[3];
  for (size_t l = (l0 / CK) * CK; l < l0; l++) {  // replay from the checkpoint without writing
    if (int rc = vm_level(R, l, c, nullptr, nullptr, nullptr)) return rc;
    rom_level(R, l, c.rom0, nullptr, s);
    c.rom0 = s[0];
  }
  for (size_t l = l0; l < l1; l++) {
    if (int rc = vm_level(R, l, c, &T, nullptr, nullptr)) return rc;
    rom_level(R, l, c.rom0, &T, s);
    c.rom0 = s[0];
  }
  if (R.ram) ram_window(R, T, l0 * 32, l1 * 32, n);
  return ZKL_OK;
}

// The program's trace as one segment (build_full_trace, mod.rs:434-524) and its AIR public inputs
int build_full(const Run& R, zkl_f128* trace, zkl_air_public_inputs* pi) {
  if (int rc = build_window(R, 0, R.levels, trace, R.L.width, nullptr)) return rc;
  const size_t n = R.levels * 32;
  const Table T{trace, n};
  core_pi(R, pi);
  for (int i = 0; i < 3; i++) {
    pi->rom_s_in[i] = to_abi(T.get(R.L.rom_s + i, 0));
    pi->rom_s_out[i] = to_abi(T.get(R.L.rom_s + i, (R.levels - 1) * 32 + 28));
  }
  pi->pc_init = to_abi(T.get(R.L.pc, 0));
  derive_trace_pi(T, R.L, R.ram, R.levels, pi);
  return ZKL_OK;
}

int prepare(Run& R, const fe regs0[8], fe rom0) {
  R.levels = R.ops.size();
  memcpy(R.init.regs, regs0, sizeof R.init.regs);
  R.init.rom0 = rom0;
  return prepass(R);
}

// SegmentFeatures::from_ops: sponge ops need the PoseidonAir block, Merkle steps the MerkleAir
// block (with Poseidon), Load / Store the RamAir block.
void features_of(const Op* ops, size_t n, bool& sponge, bool& ram, bool& merkle) {
  sponge = ram = merkle = false;
  for (size_t i = 0; i < n; i++) {
    const Kind k = ops[i].k;
    sponge |= k == K_ABSORB || k == K_SQUEEZE;
    ram |= k == K_LOAD || k == K_STORE;
    merkle |= k == K_MFIRST || k == K_MSTEP || k == K_MLAST;
  }
}

// prove_segment's effective feature mask for levels [l0, l1) (compute_segment_features_for_levels /
// compute_segment_feature_mask, segment_planner.rs:283-334; prove.rs:1078-1083): the program's
// mask cut to the blocks the ops of those levels use (pad levels use none); the program's when the
// cut is empty or equal.
uint64_t segment_mask(uint64_t base, const std::vector<Op>& ops, size_t n_ops, size_t l0, size_t l1) {
  l1 = std::min(l1, n_ops);
  bool ssp, srm, smk;
  features_of(ops.data() + std::min(l0, l1), l1 > l0 ? l1 - l0 : 0, ssp, srm, smk);
  uint64_t seg = 0;
  if (base & FM_VM) seg |= FM_VM;
  if (base & FM_VM_EXPECT) seg |= FM_VM_EXPECT;
  if ((base & FM_RAM) && srm) seg |= FM_RAM;
  if ((base & FM_MERKLE) && smk) seg |= FM_MERKLE;
  if ((base & FM_SPONGE) && ssp) seg |= FM_SPONGE;
  if ((base & FM_POSEIDON) && (ssp || smk)) seg |= FM_POSEIDON;
  return (seg != 0 && seg != base) ? seg : base;
}

// segment column -> full column (SegmentLayout::from_full_columns, mod.rs:80-235): identical
// prefix, the optional RAM / Merkle blocks, then the tail from pi_prog on
int full_col_of(const Layout& LF, const Layout& LS, bool e_ram, bool e_merkle, int c) {
  if (c < LS.ram_sorted) return c;
  if (e_ram && c < LS.ram_sorted + 8) return LF.ram_sorted + (c - LS.ram_sorted);
  if (e_merkle && c >= LS.merkle_g && c < LS.merkle_g + 7) return LF.merkle_g + (c - LS.merkle_g);
  return LF.pi_prog + (c - LS.pi_prog);
}
}  // namespace

// ---- synthetic segments ----------------------------------------------------------------------
extern "C" int zkl_synth_vm_segment(uint64_t seed, uint32_t log_n, zkl_f128* trace, zkl_air_public_inputs* pi,
                                    uint32_t* width_out) {
  return zkl_synth_vm_segment_ex(seed, log_n, 0, trace, pi, width_out);
}

extern "C" int zkl_synth_vm_segment_ex(uint64_t seed, uint32_t log_n, uint32_t flags, zkl_f128* trace,
                                       zkl_air_public_inputs* pi, uint32_t* width_out) {
  return zkl_synth_vm_segment_chain(seed, seed, log_n, flags, nullptr, trace, pi, width_out);
}

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
  Run R;
  init_run(R, pid, pid, sponge, ram, merkle);
  const fe regs0[8] = {};
  R.ops = make_program(seed, levels, flags);
  if (int rc = prepare(R, regs0, rom0_in ? fe_from(*rom0_in) : fe_zero())) return rc;
  return build_full(R, trace, pi);
}

// ---- op lists ----------------------------------------------------------------------------------
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

// The run of an op list: features, layout, initial registers -- secret u64 args from r0,
// main-arg slots (encode_main_args_to_slots, utils.rs:79-109) in the tail registers
// (vm.rs:64-104) -- and the pre-pass.
int make_run(Run& R, const zkl_op* ops_in, uint32_t n_ops, const uint8_t program_id[32],
             const uint8_t program_commitment[32], const uint64_t* secret_args, uint32_t n_secret,
             const zkl_vm_arg* main_args, uint32_t n_main, const zkl_f128* rom0_in, bool run) {
  if (!ops_in || n_ops == 0 || !program_id || !program_commitment) return ZKL_E_INVALID;
  if ((n_secret && !secret_args) || (n_main && !main_args) || n_main > ZKL_MAX_MAIN_SLOTS) return ZKL_E_INVALID;
  std::vector<Op> ops;
  if (int rc = to_ops(ops_in, n_ops, ops)) return rc;
  bool sponge, ram, merkle;
  features_of(ops.data(), ops.size(), sponge, ram, merkle);
  init_run(R, program_id, program_commitment, sponge, ram, merkle);
  R.slots.clear();
  for (uint32_t i = 0; i < n_main; i++) {
    const zkl_vm_arg& a = main_args[i];
    if (a.tag == 0) { uint64_t x; memcpy(&x, a.bytes, 8); R.slots.push_back(fe{x, 0}); }
    else if (a.tag == 1) R.slots.push_back(be_from_le16(a.bytes));
    else if (a.tag == 2) { R.slots.push_back(be_from_le16(a.bytes)); R.slots.push_back(be_from_le16(a.bytes + 16)); }
    else return ZKL_E_INVALID;
  }
  if (R.slots.size() > 8) return ZKL_E_INVALID;  // "too many main_args for VM register file" (vm.rs:68-74)
  fe regs0[8] = {};
  const size_t tail = 8 - R.slots.size();  // secret args fill r0.., main-arg slots the tail (vm.rs:64-104)
  for (size_t i = 0; i < n_secret && i < tail; i++) regs0[i] = fe{secret_args[i], 0};
  for (size_t j = 0; j < R.slots.size(); j++) regs0[tail + j] = R.slots[j];
  R.ops = std::move(ops);
  R.levels = R.ops.size();
  if (!run) return ZKL_OK;
  return prepare(R, regs0, rom0_in ? fe_from(*rom0_in) : fe_zero());
}
}  // namespace

extern "C" int zkl_build_trace(const zkl_op* ops_in, uint32_t n_ops, const uint8_t program_id[32],
                               const uint8_t program_commitment[32], const uint64_t* secret_args, uint32_t n_secret,
                               const zkl_vm_arg* main_args, uint32_t n_main, const zkl_f128* rom0_in,
                               zkl_f128* trace, zkl_air_public_inputs* pi, uint32_t* width_out,
                               uint32_t* n_rows_out) {
  Run R;
  const bool run = trace != nullptr;
  if (int rc = make_run(R, ops_in, n_ops, program_id, program_commitment, secret_args, n_secret, main_args, n_main,
                        rom0_in, false))
    return rc;
  if (width_out) *width_out = (uint32_t)R.L.width;
  if (n_rows_out) *n_rows_out = (uint32_t)(R.levels * 32);
  if (!run) return ZKL_OK;
  if (!pi) return ZKL_E_INVALID;
  if (int rc = make_run(R, ops_in, n_ops, program_id, program_commitment, secret_args, n_secret, main_args, n_main,
                        rom0_in, true))
    return rc;
  return build_full(R, trace, pi);
}

// rom_acc_from_program (romacc.rs:22-80): the ROM accumulator from the ops alone, over virtual
// map rows that hold each op's opcode bit and register selectors (encode_map_row_for_op,
// romacc.rs:82-260) — what the verifier recomputes for pi.rom_acc (prove.rs:815-821).
extern "C" int zkl_rom_acc_from_program(const zkl_op* ops_in, uint32_t n_ops, const uint8_t program_id[32],
                                        zkl_f128 out[3]) {
  if (!ops_in || !n_ops || !program_id || !out) return ZKL_E_INVALID;
  Run R;
  if (int rc = to_ops(ops_in, n_ops, R.ops)) return rc;
  R.levels = R.ops.size();
  init_run(R, program_id, program_id, false, false, false);
  fe s[3] = {fe_zero(), fe_zero(), fe_zero()};
  for (size_t l = 0; l < R.levels; l++) rom_level(R, l, s[0], nullptr, s);
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
  features_of(ops.data(), ops.size(), sp, rm, mk);
  const Layout LF = make_layout(true, rm, sp, mk, true);
  if (LF.width != (int)full_width) return ZKL_E_INVALID;
  const uint64_t eff = segment_mask(pi_full->feature_mask, ops, n_ops, r_start / 32, r_end / 32);
  const bool e_ram = eff & FM_RAM, e_merkle = eff & FM_MERKLE;
  const Layout LS = make_layout(true, e_ram, (eff & FM_SPONGE) != 0, e_merkle, true);
  if (width_out) *width_out = (uint32_t)LS.width;
  if (!trace_out) return ZKL_OK;
  if (!pi_out) return ZKL_E_INVALID;
  if ((e_ram && !rm) || (e_merkle && !mk)) return ZKL_E_INVALID;  // a block the full trace lacks
  for (int c = 0; c < LS.width; c++)
    memcpy(trace_out + (size_t)c * m, full + (size_t)full_col_of(LF, LS, e_ram, e_merkle, c) * n_full + r_start,
           m * sizeof(zkl_f128));
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

// ---- per-segment builder ------------------------------------------------------------------------
struct zkl_program {
  Run R;
};

extern "C" int zkl_program_new(const zkl_op* ops, uint32_t n_ops, const uint8_t program_id[32],
                               const uint8_t program_commitment[32], const uint64_t* secret_args, uint32_t n_secret,
                               const zkl_vm_arg* main_args, uint32_t n_main, const zkl_f128* rom0_in,
                               zkl_program** out, uint32_t* full_width_out, uint32_t* n_rows_out) {
  if (!out) return ZKL_E_INVALID;
  *out = nullptr;
  zkl_program* p = new (std::nothrow) zkl_program;
  if (!p) return ZKL_E_OOM;
  if (int rc = make_run(p->R, ops, n_ops, program_id, program_commitment, secret_args, n_secret, main_args, n_main,
                        rom0_in, true)) {
    delete p;
    return rc;
  }
  if (full_width_out) *full_width_out = (uint32_t)p->R.L.width;
  if (n_rows_out) *n_rows_out = (uint32_t)(p->R.levels * 32);
  *out = p;
  return ZKL_OK;
}

extern "C" void zkl_program_free(zkl_program* p) { delete p; }

extern "C" int zkl_build_segment_trace(const zkl_program* p, uint32_t r_start, uint32_t r_end, zkl_f128* trace_out,
                                       zkl_air_public_inputs* pi_out, uint32_t* width_out, uint8_t state_in[32],
                                       uint8_t state_out[32]) {
  if (!p) return ZKL_E_INVALID;
  const Run& R = p->R;
  const size_t n = R.levels * 32;
  if (r_start >= r_end || r_end > n || r_start % 32 || r_end % 32) return ZKL_E_INVALID;
  const size_t m = r_end - r_start;
  if (m & (m - 1)) return ZKL_E_INVALID;  // a Winterfell trace length
  size_t n_ops = R.levels;
  while (n_ops > 0 && R.ops[n_ops - 1].k == K_PAD) n_ops--;
  const size_t l0 = r_start / 32, l1 = r_end / 32;
  const uint64_t eff = segment_mask(program_mask(R), R.ops, n_ops, l0, l1);
  const bool e_ram = eff & FM_RAM, e_merkle = eff & FM_MERKLE;
  const Layout LS = make_layout(true, e_ram, (eff & FM_SPONGE) != 0, e_merkle, true);
  if (width_out) *width_out = (uint32_t)LS.width;
  if (!trace_out) return ZKL_OK;
  if (!pi_out) return ZKL_E_INVALID;
  std::vector<int> map(R.L.width, -1);
  for (int c = 0; c < LS.width; c++) map[full_col_of(R.L, LS, e_ram, e_merkle, c)] = c;
  if (int rc = build_window(R, l0, l1, trace_out, LS.width, map.data())) return rc;
  const Table TS{trace_out, m};
  core_pi(R, pi_out);
  pi_out->segment_feature_mask = eff;
  pi_out->pc_init = to_abi(fe{l0, 0});
  if (R.ram) {  // compute_segment_boundary_bytes (prove.rs:1197-1287): the running sums at both ends
    pi_out->ram_gp_unsorted_in = to_abi(ram_gp_unsorted_at(R, r_start));
    pi_out->ram_gp_unsorted_out = to_abi(ram_gp_unsorted_at(R, r_end - 1));
    pi_out->ram_gp_sorted_in = to_abi(ram_gp_sorted_at(R, r_start));
    pi_out->ram_gp_sorted_out = to_abi(ram_gp_sorted_at(R, r_end - 1));
  }
  for (int i = 0; i < 3; i++) {
    pi_out->rom_s_in[i] = to_abi(TS.get(LS.rom_s + i, 0));
    pi_out->rom_s_out[i] = to_abi(TS.get(LS.rom_s + i, m - 32 + 28));
  }
  derive_trace_pi(TS, LS, e_ram, m / 32, pi_out);
  if (state_in) vm_state_hash(TS, LS, 0, state_in);
  if (state_out) vm_state_hash(TS, LS, m - 1, state_out);
  return ZKL_OK;
}
