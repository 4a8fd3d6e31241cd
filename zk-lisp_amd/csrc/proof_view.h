// Host-side reading of segment proofs: Proof::to_bytes() of a ZkLispAir proof parsed, its
// Fiat-Shamir transcript replayed and every check of winter-verifier 0.13.1 applied
// (the reference calls it at prove.rs:802-941 and replays the same
// transcript in agg/fs.rs:38-245).  The parsed and replayed values stay available to the
// aggregation (agg.cpp: the child transcripts of agg/child.rs:531-850).
#pragma once
#include <stddef.h>
#include <stdint.h>

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
};

// Parses and verifies one segment proof under the given public inputs and options (the
// options must equal those recorded in the proof).  Returns "" when the proof verifies, the
// first failing check otherwise; `view` (optional) receives the parsed/replayed values.
std::string verify_segment(const uint8_t* proof, size_t len, const zkl_air_public_inputs& pi,
                           const zkl_proof_options& opts, SegmentView* view);

}  // namespace zkl
