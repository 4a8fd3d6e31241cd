/*
 * ORACLE — test infrastructure only.  CPU restatement of the reference algorithm for
 * the zk-lisp segment-proof hot path (zk-lisp-proof-winterfell + winterfell 0.13.1).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity status: BLAKE3 pinned by the spec vectors; f128 and Poseidon by
 * an independent big-integer Python restatement (tests/pyref.py) and committed golden
 * vectors; the AIR by trace satisfaction; the Poseidon/AIR/transcript layers follow the
 * reference sources cited per function.  The Winterfell 0.13.1 byte/transcript conventions
 * (third-party crate, absent here, no reference fixtures) are a restatement and are
 * "parity unpinned" against real Winterfell output.
 */
#ifndef ORACLE_H
#define ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include "f128.h"
#include "../include/zkl_hip.h"

/* ---------------- BLAKE3 ---------------- */
void orc_blake3(const uint8_t *in, size_t len, uint8_t out32[32]);
void orc_blake3_parts(const uint8_t *const *parts, const size_t *lens, int nparts, uint8_t out32[32]);

/* ---------------- Poseidon (poseidon/mod.rs, poseidon/hasher.rs) ---------------- */
#define POS_T 12
#define POS_RATE 10
#define POS_ROUNDS 27
typedef struct {
  fe dom[2];
  fe mds[12][12];
  fe rc[POS_ROUNDS][12];
  int rounds;
} pos_suite;

void pos_suite_derive(const uint8_t suite_id[32], int rounds, pos_suite *out);
const pos_suite *pos_hasher_suite(void); /* suite_id = [0;32], 27 rounds (hasher.rs:23) */
void pos_permute(const pos_suite *s, fe st[12]);
fe ro_from_slices(const char *domain, const uint8_t *const *parts, const size_t *lens, int nparts);
fe fold_bytes32(const uint8_t b[32]);                     /* utils.rs:359-371 */
fe be_from_le8(const uint8_t b32[32]);                      /* utils.rs:346-357 */
fe sponge_bytes(const pos_suite *s, const char *domain, const uint8_t *data, size_t len); /* hasher.rs:144-231 */

/* PoseidonHasher digests are 32 bytes: state[0] LE16 || 16 zero bytes; we carry the fe */
fe ph_hash_bytes(const uint8_t *data, size_t len);          /* Hasher::hash       hasher.rs:62 */
fe ph_merge(fe a, fe b);                                   /* Hasher::merge      hasher.rs:72 */
fe ph_merge_many(const fe *d, size_t n);                   /* merge_many         hasher.rs:87 (n>0) */
fe ph_merge_with_int(fe seed, uint64_t v);                 /* merge_with_int     hasher.rs:107 */
fe ph_hash_elements(const fe *e, size_t n);                /* hash_elements      hasher.rs:126 */

/* ROM t=3 constants (poseidon/mod.rs:186-261) */
void rom_constants(const uint8_t suite_id[32], fe rc[POS_ROUNDS][3], fe mds[3][3]);
/* commit::program_field_commitment (commit.rs:31-79) */
void program_field_commitment(const uint8_t blake32[32], fe out[2]);

/* ---------------- NTT helpers ---------------- */
void ntt_inplace(fe *a, size_t n, int inverse);            /* natural order in/out */
void coset_interpolate(fe *a, size_t n, fe offset);        /* evals over offset*<w_n> -> coeffs */
void coset_evaluate(const fe *coeffs, size_t ncoef, fe *out, size_t n, fe offset);
fe poly_eval(const fe *c, size_t n, fe x);

/* ---------------- AIR (vm/air/ (all modules), vm/layout.rs) ---------------- */
/* feature bits (zk-lisp-proof/src/pi.rs:23-28) */
#define FM_POSEIDON 1ull
#define FM_VM 2ull
#define FM_VM_EXPECT 16ull
#define FM_SPONGE 32ull
#define FM_MERKLE 64ull
#define FM_RAM 128ull

typedef struct {
  int lanes_start, g_map, g_final, g_r_start, mask, r_start;
  int op[17];         /* const, mov, add, sub, mul, neg, eq, select, sponge, assert, assert_bit,
                         assert_range, divmod, div128, mulwide, load, store */
  int sel_dst0, sel_a, sel_b, sel_c, sel_dst1, sel_s_bits, sel_s_active, imm, eq_inv;
  int pi_prog, pc, rom_op_start, pose_active, gadget_b, rom_s;
  int ram_sorted, ram_s_addr, ram_s_clk, ram_s_val, ram_s_is_write, ram_s_last_write, ram_gp_unsorted,
      ram_gp_sorted;                                       /* layout.rs:247-256 */
  int merkle_g, merkle_dir, merkle_sib, merkle_acc, merkle_first, merkle_last, merkle_leaf; /* :262-270 */
  int width;
} zk_cols;
void cols_for_config(int vm, int ram, int sponge, int merkle, int rom, zk_cols *c);

#define MAX_TC 1024
typedef struct {
  zk_cols cols;
  int feat_poseidon, feat_vm, feat_vm_expect, feat_sponge, feat_merkle, feat_ram, rom_enabled;
  uint32_t vm_usage_mask, ram_delta_clk_bits;
  int commit_nonzero;
  fe rom_rc[POS_ROUNDS][3], rom_mds[3][3];
  fe rom_w0[59], rom_w1[59];
  fe dom[2];
  fe pose_mds[12][12], pose_rc[POS_ROUNDS][12]; /* AIR Poseidon suite (suite_id = program_id) */
  int pose_bind;                                 /* VM->lane bindings present (poseidon.rs:48-62) */
  fe program_fe[2];
  fe merkle_root;                                /* be_from_le8(pi.merkle_root) (merkle.rs:118) */
  /* transition constraint degrees (base, has_cycle32) */
  int n_tc;
  int deg_base[MAX_TC];
  unsigned char deg_cyc[MAX_TC];
  /* assertions sorted (step, column) after dedup */
  size_t n_assert;
  uint32_t *as_col, *as_step;
  fe *as_val;
  size_t trace_len;
  int ce_blowup, n_comp_cols;
} zk_air;

int air_new(zk_air *air, const zkl_air_public_inputs *pi, uint32_t width, size_t n);
void air_free(zk_air *air);
/* evaluate all transition constraints at a frame; periodic = 32 values */
void air_eval_transition(const zk_air *air, const fe *cur, const fe *nxt, const fe *periodic, fe *out);
void air_periodic_at(const zk_air *air, fe x, fe out[32]);

/* ---------------- trace generator (vm/trace/ (vm, rom) subset) ---------------- */
int orc_synth_vm_segment(uint64_t seed, uint32_t log_n, zkl_f128 *trace_out,
                         zkl_air_public_inputs *pi_out, uint32_t *width_out);
/* flags bit 0: program with SAbsorbN / SSqueeze sponge ops (features VM | SPONGE | POSEIDON) */
int orc_synth_vm_segment_ex(uint64_t seed, uint32_t log_n, uint32_t flags, zkl_f128 *trace_out,
                            zkl_air_public_inputs *pi_out, uint32_t *width_out);

/* ---------------- prover / verifier ---------------- */
int orc_synth_vm_segment_chain(uint64_t program_seed, uint64_t seed, uint32_t log_n, uint32_t flags, const zkl_f128 *rom0_in,
                               zkl_f128 *trace_out, zkl_air_public_inputs *pi_out, uint32_t *width_out);
/* op-list trace builder, zkl_build_trace's twin (same arguments; 0 / -1) */
int orc_build_trace(const zkl_op *ops, uint32_t n_ops, const uint8_t program_id[32], const uint8_t commitment[32],
                    const uint64_t *secret_args, uint32_t n_secret, const zkl_vm_arg *main_args, uint32_t n_main,
                    const zkl_f128 *rom0_in, zkl_f128 *trace_out, zkl_air_public_inputs *pi_out, uint32_t *width_out,
                    uint32_t *n_rows_out);
/* per-segment builder, zkl_build_segment_trace's twin (program arguments as orc_build_trace,
 * then the segment's rows; streams every level, no full trace) */
int orc_build_segment_trace(const zkl_op *ops, uint32_t n_ops, const uint8_t program_id[32],
                            const uint8_t commitment[32], const uint64_t *secret_args, uint32_t n_secret,
                            const zkl_vm_arg *main_args, uint32_t n_main, const zkl_f128 *rom0_in, uint32_t r_start,
                            uint32_t r_end, zkl_f128 *trace_out, zkl_air_public_inputs *pi_out, uint32_t *width_out,
                            uint8_t state_in[32], uint8_t state_out[32]);
int orc_prove_segment(const zkl_f128 *trace, uint32_t width, uint32_t n,
                      const zkl_air_public_inputs *pi, const zkl_proof_options *opts,
                      uint8_t **proof, size_t *len, int boundary_mode);
int orc_verify_segment(const uint8_t *proof, size_t len, const zkl_air_public_inputs *pi,
                       const zkl_proof_options *opts, char *err, size_t errlen);
void orc_free(void *p);
/* row digest of a (partitioned) row; rule 0 winterfell commit_to_rows, rule 1 agg/child.rs
 * hash_row_poseidon (differ only for one-chunk rows, prover.c) */
fe orc_row_digest(const fe *row, size_t ncols, size_t psize);
void orc_set_row_digest_rule(int rule);
int orc_row_digest_rule(void);

/* ---------------- zl1 step proof (proof/step.rs, format.rs, digest.rs) ---------------- */
int orc_step_encode(const zkl_air_public_inputs *pi, const zkl_step_info *s, const uint8_t *inner, size_t inner_len,
                    uint8_t **out, size_t *out_len);
int orc_step_digest(const uint8_t *p, size_t n, uint8_t digest[32], uint8_t rt[32], char *err, size_t errlen);
int orc_children_root(const uint8_t suite[32], const uint8_t *digests, const uint8_t *roots, uint32_t n,
                      uint8_t out[32]);

#endif
