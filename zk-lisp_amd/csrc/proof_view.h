// Host-side reading of segment proofs: Proof::to_bytes() of a ZkLispAir proof parsed, its
// Fiat-Shamir transcript replayed and every check of winter-verifier 0.13.1 applied
// (the reference calls it at prove.rs:802-941 and replays the same
// transcript in agg/fs.rs:38-245).  The parsed and replayed values stay available to the
// aggregation (agg.cpp: the child transcripts of agg/child.rs:531-850).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

#include "../../include/zkl_hip.h"
#include "field.h"

namespace zkl {

// winter-utils ByteReader over a byte slice; `bad` latches on any overrun or non-canonical value
struct Rd {
  const uint8_t* p = nullptr;
  size_t len = 0, off = 0;
  bool bad = false;
  uint8_t u8();
  uint64_t u64();
  uint64_t usize();  // vint64 (ByteReader::read_usize)
  fe felem();        // 16-byte LE canonical element
  fe digest();       // 32-byte digest: value + 16 zero bytes
  Rd vec();          // length-prefixed sub-slice
  bool done() const { return !bad && off == len; }
};

// BatchMerkleProof::get_root (winter-crypto 0.13) for sorted unique leaf indices with their
// digests; consumes the proof bytes from r.  Returns false if the proof is malformed.
bool batch_merkle_root(Rd& r, size_t n_leaves, const std::vector<size_t>& idx, const std::vector<fe>& leaves,
                       fe* root);

struct SegmentView {
  // context
  uint32_t width = 0;
  size_t n = 0, lde = 0;
  int comp_cols = 0;
  zkl_proof_options opts{};
  // commitments
  fe trace_root{}, constraint_root{}, remainder_commit{};
  std::vector<fe> fri_roots;
  // out-of-domain frame: trace at z and z*g, composition columns at z and z*g
  std::vector<fe> ood_trace_z, ood_trace_zg, ood_comp_z, ood_comp_zg;
  // transcript
  fe z{};
  std::vector<fe> deep_coeffs;  // W trace then C composition coefficients
  std::vector<fe> fri_alphas;   // one per FRI layer
  std::vector<size_t> positions;  // unique, sorted query positions in the LDE domain
  uint64_t pow_nonce = 0;
  // openings
  std::vector<fe> trace_rows;   // positions x W
  std::vector<fe> comp_rows;    // positions x C
  std::vector<std::vector<size_t>> fri_positions;  // per layer: folded positions (order of first use)
  std::vector<std::vector<fe>> fri_values;         // per layer: [e_y, e_{y+h}] per folded position
  std::vector<fe> remainder;                       // reversed coefficients, degree <= rem_deg
  // the roots the trace / constraint openings reproduce when each opened row is hashed as the
  // reference's hash_row_poseidon does (agg/child.rs:1025-1045: a one-chunk row is not merged)
  // and the batch proof is decompressed with those leaves; equal to trace_root /
  // constraint_root unless a row is one chunk narrower than its partition
  fe trace_root_ref{}, constraint_root_ref{};
};

// ProofOptions bounds winterfell enforces when it builds or reads options (ProofOptions::new
// [WF-recall]): queries 1..255, blowup a power of two in 2..128, grinding <= 32, folding 2,
// remainder degree 2^k - 1 below the blowup, partitions 1..16, hash rate 1..255.  "" or the
// first violated bound.
std::string check_proof_options(const zkl_proof_options& o);

// Parses and verifies one segment proof under the given public inputs and options (the
// options must equal those recorded in the proof).  Returns "" when the proof verifies, the
// first failing check otherwise; `view` (optional) receives the parsed/replayed values.
std::string verify_segment(const uint8_t* proof, size_t len, const zkl_air_public_inputs& pi,
                           const zkl_proof_options& opts, SegmentView* view);
// The same with the options taken from the proof (opts == nullptr) and, when check_ood is
// false, without the out-of-domain constraint identity: the Fiat-Shamir replay plus every
// opening / DEEP / FRI / remainder / PoW check, which is what the aggregation re-derives from
// a step proof alone (agg/fs.rs:38-245 rebuilds the AIR public inputs without the expected
// VM output, so the identity is not available there either).
std::string verify_segment_ex(const uint8_t* proof, size_t len, const zkl_air_public_inputs& pi,
                              const zkl_proof_options* opts, SegmentView* view, bool check_ood);

// A decoded ZKLSTP1 step proof (StepProof::from_bytes, proof/step.rs:153-493) with the
// derived StepMeta (step.rs:516-533), zl1 root_trace (format.rs:214-238) and step digest
// (proof/digest.rs:16-68).  `inner` points into the caller's buffer.
struct StepDecoded {
  uint32_t lambda_bits = 0;
  uint8_t suite[32], program_id[32], program_commitment[32], merkle_root[32];
  uint64_t feature_mask = 0;
  std::vector<zkl_vm_arg> main_args;
  uint32_t vm_usage_mask = 0, ram_delta_clk_bits = 0;
  fe rom_acc[3];
  uint32_t segment_index = 0, segments_total = 1;  // new_single_segment normalises to (0, 1)
  uint8_t pc_init[32];
  // state_in, state_out, ram_gp_unsorted_in/out, ram_gp_sorted_in/out, rom_s_in[3], rom_s_out[3]
  uint8_t bnd[12][32];
  const uint8_t* inner = nullptr;
  size_t inner_len = 0;
  uint32_t m = 0, pi_len = 0;
  uint16_t rho = 0, q = 0, o = 0, lambda = 0;
  uint64_t v_units = 0;
  uint8_t digest[32], root_trace[32];
};
StepDecoded decode_step(const uint8_t* p, size_t n);

// runs f, mapping exceptions to ZKL_E_* codes and zkl_hip_last_error(NULL) (prover.cpp)
int guarded_call(const std::function<void()>& f);

}  // namespace zkl
