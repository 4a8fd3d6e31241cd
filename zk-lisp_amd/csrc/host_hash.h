// Host-side hashing for the prover: BLAKE3 (program ids, Poseidon constant derivation)
// and the PoseidonHasher sponge for transcript-sized inputs.  Device-side hashing of
// matrices lives in kernels.hip.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string>
#include <vector>
#include "field.h"

namespace zkl {

void blake3_hash(const uint8_t* in, size_t len, uint8_t out[32]);

// PoseidonSuite (poseidon/mod.rs:31-35): dom tags, 12x12 Cauchy MDS, per-round constants.
struct PoseidonSuite {
  fe dom[2];
  fe mds[12][12];
  fe rc[27][12];
  int rounds;
};

// get_poseidon_suite_with_rounds (poseidon/mod.rs:56-75)
PoseidonSuite derive_poseidon_suite(const uint8_t suite_id[32], int rounds = 27);
// derive_rom_round_constants_3 / derive_rom_mds_cauchy_3x3 (poseidon/mod.rs:186-261)
void derive_rom_constants(const uint8_t suite_id[32], fe rc[27][3], fe mds[3][3]);
// ro_from_slices (poseidon/mod.rs:421-440)
fe ro_from_parts(const std::string& domain, const std::vector<std::vector<uint8_t>>& parts);
// fold_bytes32_to_fe (utils.rs:359-371) and be_from_le8 (utils.rs:346-357)
fe fold_bytes32(const uint8_t b[32]);
fe be_from_le16(const uint8_t b[16]);
// commit::program_field_commitment (commit.rs:31-79)
void program_field_commitment(const uint8_t b32[32], fe out[2]);

// The commitment/coin hasher: suite [0;32], 27 rounds (poseidon/hasher.rs:23,235-241).
struct IfmaSuite;  // host_poseidon_ifma.cpp
bool ifma_available();
void ifma_prepare(const PoseidonSuite& s, IfmaSuite& out);
void ifma_permute(const IfmaSuite& s, fe st[12]);
IfmaSuite* ifma_new();
void ifma_delete(IfmaSuite* p);

struct Hasher {
  PoseidonSuite suite;
  IfmaSuite* ifma = nullptr;  // the AVX-512 IFMA form of suite when the CPU has it (checked)
  fe dom_bytes, dom_merge, dom_many, dom_int, dom_elems;  // folded domain labels
  Hasher();
  void permute(fe st[12]) const;
  fe sponge(fe dom_fe, const fe* msgs, size_t n) const;
  fe merge(fe a, fe b) const;                   // hasher.rs:72-85
  fe merge_many(const fe* d, size_t n) const;   // hasher.rs:87-105
  fe merge_with_int(fe seed, uint64_t v) const; // hasher.rs:107-120
  fe hash_elements(const fe* e, size_t n) const;  // hasher.rs:126-139
};
const Hasher& hasher();
fe domain_fe(const char* domain);

}  // namespace zkl
