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

// Columns::for_config (vm/layout.rs:183-374)
struct Layout {
  int lanes_start, g_map, g_final, g_r_start, mask, r_start;
  int op[17];  // const mov add sub mul neg eq select sponge assert assert_bit assert_range divmod div128 mulwide load store
  int sel_dst0, sel_a, sel_b, sel_c, sel_dst1, sel_s_bits, sel_s_active, imm, eq_inv;
  int pi_prog, pc, rom_op_start, pose_active, gadget_b, rom_s;
  int width;
};
Layout make_layout(bool vm, bool ram, bool sponge, bool merkle, bool rom);

// Parameters the constraint-evaluation kernel reads from __constant__ memory.
struct AirDevice {
  Layout cols;
  int feat_vm, sponge_block, commit_nonzero, n_tc;
  int pose_block, pose_bind;  // PoseidonAir present; its VM->lane bindings present
  uint32_t vm_usage_mask;
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
  std::vector<int> degree_base;          // per transition constraint (all with one 32-cycle)
  std::vector<Assertion> assertions;     // deduped, Winterfell order (step, column)
  fe suite_dom[2];
};

// ZkLispAir::new + get_assertions (vm/air/mod.rs:114-318, 380-504).
// Returns empty string on success, error text otherwise.
std::string build_air(const zkl_air_public_inputs& pi, uint32_t width, size_t n, AirInstance& out);

// AirPublicInputs::to_elements (lib.rs:116-160)
std::vector<fe> pi_elements(const zkl_air_public_inputs& pi);
// Context::to_elements (winter-air 0.13.1, [WF-recall])
std::vector<fe> context_elements(uint32_t width, size_t n, const zkl_proof_options& o);

// Periodic cycle-32 selector values p_map, p_r[27], p_final, p_pad, p_pad_last evaluated at
// y = x^(n/32) for the 256 distinct y of the CE coset: table[256][31] (vm/air/mod.rs:520-592).
std::vector<fe> periodic_table(size_t n, size_t ce_size, fe offset);

fe fe_from(const zkl_f128& v);
zkl_f128 to_abi(fe v);
fe root_of_unity(unsigned log2n);

}  // namespace zkl
