// Host side of ZkLispAir for the MI355X prover: layout, constraint degrees, assertions,
// public-input elements.  The transition constraints themselves are evaluated on the GPU
// (kernels.hip, constraint_eval_kernel) using AirDevice.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>
#include "../../include/zkl_hip.h"
#include "field.h"

namespace zkl {

// feature bits (zk-lisp-proof/src/pi.rs:23-28)
constexpr uint64_t FM_POSEIDON = 1, FM_VM = 2, FM_VM_EXPECT = 16, FM_SPONGE = 32, FM_MERKLE = 64, FM_RAM = 128;

// Columns::for_config (vm/layout.rs:183-374)
struct Layout {
  int lanes_start, g_map, g_final, g_r_start, mask, r_start;
  int op[17];  // const mov add sub mul neg eq select sponge assert assert_bit assert_range divmod div128 mulwide load store
  int sel_dst0, sel_a, sel_b, sel_c, sel_dst1, sel_s_bits, sel_s_active, imm, eq_inv;
  int pi_prog, pc, rom_op_start, pose_active, gadget_b, rom_s;
  int ram_sorted, ram_s_addr, ram_s_clk, ram_s_val, ram_s_is_write, ram_s_last_write, ram_gp_unsorted,
      ram_gp_sorted;                                                             // layout.rs:247-256
  int merkle_g, merkle_dir, merkle_sib, merkle_acc, merkle_first, merkle_last, merkle_leaf;  // :262-270
  int width;
};
Layout make_layout(bool vm, bool ram, bool sponge, bool merkle, bool rom);

// Parameters the constraint-evaluation kernel reads from __constant__ memory.
struct AirDevice {
  Layout cols;
  int feat_vm, sponge_block, commit_nonzero, n_tc;
  int pose_block, pose_bind;  // PoseidonAir present; its VM->lane bindings present
  uint32_t vm_usage_mask;
  int ram_block, ram_dclk, merkle_block;  // RamAir / its delta_clk gadget / MerkleAir present
  uint32_t ram_dclk_bits;                 // pi.ram_delta_clk_bits (bits with a booleanity constraint)
  fe ram_r[3];                            // compressor coefficients r1, r2, r3 (ram.rs:112-121)
  fe merkle_root;                         // be_from_le8(pi.merkle_root) (merkle.rs:118)
  fe pose_mds[12][12];  // AIR Poseidon suite (suite_id = program_id, vm/air/mod.rs:129-137)
  fe pose_rc[27][12];
  fe rom_mds[3][3];
  fe rom_rc[27][3];
  fe rom_w0[59];
  fe rom_w1[59];
};

struct Assertion {
  uint32_t col, step;
  fe value;
};

struct AirInstance {
  AirDevice dev;
  size_t n = 0;
  int ce_blowup = 0, num_comp_cols = 0, n_tc = 0;
  std::vector<int> degree_base;          // per transition constraint
  std::vector<int> degree_cycle;         // 1 if the constraint carries the 32-row cycle
  std::vector<Assertion> assertions;     // deduped, Winterfell order (step, column)
  fe suite_dom[2];
};

// ZkLispAir::new + get_assertions (vm/air/mod.rs:114-318, 380-504).
// Returns empty string on success, error text otherwise.
std::string build_air(const zkl_air_public_inputs& pi, uint32_t width, size_t n, AirInstance& out,
                      bool check_width = true);

// AirPublicInputs::to_elements (lib.rs:116-160)
std::vector<fe> pi_elements(const zkl_air_public_inputs& pi);
// Context::to_elements (winter-air 0.13.1, [WF-recall])
std::vector<fe> context_elements(uint32_t width, size_t n, const zkl_proof_options& o);

// Periodic cycle-32 selector values p_map, p_r[27], p_final, p_pad, p_pad_last evaluated at
// y = x^(n/32) for the 256 distinct y of the CE coset: table[256][31] (vm/air/mod.rs:520-592).
std::vector<fe> periodic_table(size_t n, size_t ce_size, fe offset);
// the same 31 values at one point x (the verifier's out-of-domain point)
std::vector<fe> periodic_at(size_t n, fe x);

fe fe_from(const zkl_f128& v);
zkl_f128 to_abi(fe v);
fe root_of_unity(unsigned log2n);

}  // namespace zkl
