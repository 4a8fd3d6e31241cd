/*
 * zkl_hip.h — C ABI of the MI355X-native zk-lisp segment prover (libzkl_hip.so).
 *
 * One call proves one zk-lisp execution segment and returns the bytes of the
 * inner STARK proof, i.e. what the reference gets from
 *   ZkWinterfellProver.prove(trace)           zk-lisp-proof-winterfell/src/prove.rs:225
 * inside
 *   prove_segment(...)                        zk-lisp-proof-winterfell/src/prove.rs:1057-1175
 * (the call at prove.rs:1142, `prover.prove(trace)?`).  The Rust side would
 * `Proof::from_bytes` the result and continue at prove.rs:1144.  The binding a
 * maintainer adds on the Rust side is shown in INTEGRATION.md.
 *
 * Conventions
 *  - field elements are f128 (p = 2^128 - 45*2^40 + 1), canonical (< p),
 *    little-endian limbs {lo, hi}; the same value `BaseElement::as_int()` gives.
 *  - traces are column-major: element (col, row) at trace[col * n_rows + row].
 *  - every function returns 0 on success and a negative ZKL_E_* code on failure;
 *    zkl_hip_last_error() then returns a message (the reference maps failures to
 *    prove::Error::Backend(String), prove.rs:225-227; same shape here).
 *  - the library owns nothing the caller passed in; proof buffers it returns are
 *    released with zkl_hip_free().
 *  - one zkl_ctx per device; calls on one ctx are serialised internally, calls
 *    on different ctx run concurrently (reference calls prove_segment from a
 *    rayon pool, prove.rs:1020-1048).
 */
#ifndef ZKL_HIP_H
#define ZKL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZKL_ABI_VERSION 1

enum {
  ZKL_OK = 0,
  ZKL_E_INVALID = -1,   /* bad argument / unsupported configuration */
  ZKL_E_DEVICE = -2,    /* HIP runtime error */
  ZKL_E_OOM = -3,       /* device or host allocation failed */
  ZKL_E_INTERNAL = -4,  /* internal consistency check failed */
};

typedef struct { uint64_t lo, hi; } zkl_f128;

/* winterfell::ProofOptions as built at prove.rs:963-972 + with_partitions(prove.rs:1121).
 * field_extension: 1 = None (FieldExtension discriminant); only None is supported for
 * step proofs.  batching_*: 0 = Linear (BatchingMethod discriminant). */
typedef struct {
  uint32_t num_queries;              /* CLI default 64 (zk-lisp-cli/src/main.rs:124-132) */
  uint32_t blowup_factor;            /* 16 */
  uint32_t grinding_factor;          /* 16 */
  uint32_t field_extension;          /* 1 = None */
  uint32_t fri_folding_factor;       /* 2 */
  uint32_t fri_remainder_max_degree; /* 1 */
  uint32_t batching_constraints;     /* 0 = Linear */
  uint32_t batching_deep;            /* 0 = Linear */
  uint32_t num_partitions;           /* select_partitions_for_trace, utils.rs:394-409 */
  uint32_t hash_rate;                /* idem */
} zkl_proof_options;

#define ZKL_MAX_MAIN_SLOTS 8

/* crate::AirPublicInputs (zk-lisp-proof-winterfell/src/lib.rs:75-95) flattened.
 * `core` fields are the subset of zk_lisp_proof::pi::PublicInputs (pi.rs:62-88)
 * that ZkLispAir::new / get_assertions / to_elements read.  main_args are given
 * already flattened into base-field slots (utils::encode_main_args_to_slots). */
typedef struct {
  uint8_t program_id[32];
  uint8_t program_commitment[32];
  uint8_t merkle_root[32];
  uint64_t feature_mask;          /* core.feature_mask (FM_* bits, pi.rs:23-28) */
  uint64_t segment_feature_mask;  /* effective per-segment mask (prove.rs:1078-1083) */
  uint32_t n_main_slots;
  zkl_f128 main_slots[ZKL_MAX_MAIN_SLOTS];
  uint32_t vm_out_reg;
  uint32_t vm_out_row;
  uint8_t vm_expected_bytes[32];
  zkl_f128 rom_acc[3];
  zkl_f128 pc_init;
  zkl_f128 ram_gp_unsorted_in, ram_gp_unsorted_out, ram_gp_sorted_in, ram_gp_sorted_out;
  zkl_f128 rom_s_in[3];
  zkl_f128 rom_s_out[3];
  uint32_t vm_usage_mask;
  uint32_t ram_delta_clk_bits;
} zkl_air_public_inputs;

/* ---- zl1 step proof (a18) --------------------------------------------------------
 * zk_lisp_proof::pi::VmArg (pi.rs) for the ZKLSTP1 encoding: tag 0 = U64 (bytes[0..8] LE),
 * 1 = U128 (bytes[0..16] LE), 2 = Bytes32. */
typedef struct {
  uint32_t tag;
  uint8_t bytes[32];
} zkl_vm_arg;

/* What prove_segment (prove.rs:1057-1175) feeds Proof::new_multi_segment (format.rs:105-148)
 * and StepProof besides the inner proof and the AirPublicInputs: the suite id (= program_id,
 * prove.rs:985), the security target echoed as lambda (opts.min_security_bits, prove.rs:634),
 * the segment position, the VM state hashes from the trace builder and the
 * SegmentBoundaryBytes (prove.rs:1112), and the typed main_args of the core public inputs. */
typedef struct {
  uint8_t suite_id[32];
  uint32_t lambda_bits;
  uint32_t segment_index, segments_total;
  uint8_t pc_init[32];
  uint8_t state_in_hash[32], state_out_hash[32];
  uint8_t ram_gp_unsorted_in[32], ram_gp_unsorted_out[32], ram_gp_sorted_in[32], ram_gp_sorted_out[32];
  uint8_t rom_s_in[3][32];
  uint8_t rom_s_out[3][32];
  uint32_t n_main_args;
  zkl_vm_arg main_args[ZKL_MAX_MAIN_SLOTS];
} zkl_step_info;

/* Per-stage wall times of the last proof on a ctx, milliseconds; stage names follow
 * the reference's tracing events (prove.rs:464-513): trace_lde, trace_commit,
 * coefficients, evaluator, constraint_commitment, ood, deep, fri, grind, queries. */
#define ZKL_NUM_STAGES 10

typedef struct zkl_ctx zkl_ctx;

/* ---- lifecycle ---------------------------------------------------------- */
int zkl_hip_init(int device, zkl_ctx** out);
void zkl_hip_destroy(zkl_ctx* ctx);
const char* zkl_hip_last_error(const zkl_ctx* ctx); /* ctx may be NULL */
void zkl_hip_free(uint8_t* buf);
int zkl_hip_abi_version(void);
/* compiled-in tuning values of the kernels ("NAME=value;..."): every value is a supported,
 * parity-tested configuration (no timing probes are compiled in; tests/test_abi.py) */
const char* zkl_hip_build_config(void);

/* ---- process-level settings (opt-in) --------------------------------------------------
 * zkl_hip_init changes nothing outside the library.  These process-wide settings helped the
 * prover on some hosts and are the embedding application's choice:
 *   ZKL_TUNE_SPIN    hipSetDeviceFlags(hipDeviceScheduleSpin) on every visible device: host waits
 *                    on the device spin instead of sleeping (a blocking wait was seen to wake
 *                    20-30 ms late); costs one host core per waiting context.  Takes effect only
 *                    before the first zkl_hip_init / HIP context of the process.
 *   ZKL_TUNE_MALLOC  glibc mallopt: mmap threshold 32 MiB, top pad 64 MiB, trim threshold 2 GiB --
 *                    the process keeps freed heap memory instead of returning it to the kernel
 *                    (memory returned while a proof ran was followed by idle GPU time).
 *                    Changes the allocator of the whole host process.
 * *applied receives the flags that took effect; ZKL_OK if all requested did. */
#define ZKL_TUNE_SPIN 1u
#define ZKL_TUNE_MALLOC 2u
int zkl_hip_process_tuning(uint32_t flags, uint32_t* applied);

/* ---- the drop-in: one segment proof ----------------------------------------
 * Replaces ZkProver::prove -> winterfell::Prover::prove (prove.rs:174-257) for
 * ZkLispAir + PoseidonHasher + MerkleTree + DefaultRandomCoin (prove.rs:425-437).
 * trace: host pointer, column-major width x n_rows.  Output: Proof::to_bytes(). */
int zkl_hip_prove_segment(zkl_ctx* ctx, const zkl_f128* trace, uint32_t width, uint32_t n_rows,
                          const zkl_air_public_inputs* pi, const zkl_proof_options* opts,
                          uint8_t** proof_out, size_t* proof_len);

/* Pinned host buffers owned by ctx for the next traces: slot 0 .. ZKL_TRACE_BUFFERS - 1, each at
 * least `bytes` (grown when needed, kept across proofs, freed by zkl_hip_destroy).  The caller
 * fills one -- zkl_build_segment_trace can write a segment straight into it -- and passes it as
 * `trace` to zkl_hip_prove_segment, which then DMAs the columns from it with no staging copy and no
 * per-proof host allocation on the caller's side (prove.rs:1103-1142 allocates a fresh TraceTable
 * per segment and drops it after the proof).  Two slots let the next segment be built while the
 * current one proves.  A slot must not be written while a proof reads it; valid until the next
 * call that grows it. */
#define ZKL_TRACE_BUFFERS 2
int zkl_hip_trace_buffer(zkl_ctx* ctx, uint32_t slot, size_t bytes, zkl_f128** out);
/* Pinned host memory the library holds across all contexts of the process (trace buffers,
 * upload slots, transcript / gather / proof staging): bytes now and the peak since load.  No
 * device work; for capacity planning (8 ranks x in-flight contexts on one host). */
int zkl_hip_pinned_bytes(uint64_t* current, uint64_t* peak);

/* Same, with the trace already resident in HBM (device pointer on ctx's device,
 * column-major).  Used by the multi-segment pipeline and by bench.py. */
int zkl_hip_prove_segment_device(zkl_ctx* ctx, const void* d_trace, uint32_t width, uint32_t n_rows,
                                 const zkl_air_public_inputs* pi, const zkl_proof_options* opts,
                                 uint8_t** proof_out, size_t* proof_len);

/* The same proof written into caller memory (no allocation, one copy): for a binding that keeps
 * one buffer across segments (e.g. a Vec<u8> reserved once and set_len'd; the reference's
 * Proof::to_bytes at prove.rs:1142 allocates per proof).  *proof_len receives the size; with
 * cap too small (or buf NULL, a size query) the call returns ZKL_E_INVALID (NULL: ZKL_OK) and
 * the bytes stay on the context for zkl_hip_last_proof. */
int zkl_hip_prove_segment_device_into(zkl_ctx* ctx, const void* d_trace, uint32_t width, uint32_t n_rows,
                                      const zkl_air_public_inputs* pi, const zkl_proof_options* opts,
                                      uint8_t* buf, size_t cap, size_t* proof_len);

/* The last proof made on ctx (any zkl_hip_prove_segment* call), valid until the next one:
 * *len = its size; copied into buf when buf != NULL and cap >= *len (ZKL_E_INVALID when cap is
 * too small or no proof is held). */
int zkl_hip_last_proof(zkl_ctx* ctx, uint8_t* buf, size_t cap, size_t* len);

/* The request checks zkl_hip_prove_segment* run before any device work, without a device:
 * ProofOptions / PartitionOptions bounds (num_queries 1..255, blowup a power of two >= 2 and
 * >= the AIR's constraint-evaluation blowup, num_partitions 1..16, hash_rate 1..256, FRI
 * folding 2, remainder degree 2^k - 1), the supported options (FieldExtension::None,
 * BatchingMethod::Linear), the trace shape (n_rows a power of two >= 32, width = the segment
 * layout's width) and the public-input shape (n_main_slots <= ZKL_MAX_MAIN_SLOTS, assertion
 * count = AirContext::num_assertions).  ZKL_OK or ZKL_E_INVALID + zkl_hip_last_error(NULL). */
int zkl_hip_check_request(uint32_t width, uint32_t n_rows, const zkl_air_public_inputs* pi,
                          const zkl_proof_options* opts);

/* Host-side wall times (ms) of the last proof on ctx: [0] host setup before the first
 * kernel (AIR instance, assertions, uploads), [1] host time between the first and last
 * stage marks not covered by device work, [2] the whole call, [3] the host-trace upload loop
 * of zkl_hip_prove_segment (pinned staging + DMA issue; 0 for the device entry point).
 * Returns number written. */
int zkl_hip_host_times(const zkl_ctx* ctx, double* out_ms, int max_n);

/* Stage timings (ms) of the last proof on ctx; returns number written.  Recorded only for
 * proofs run with zkl_hip_set_kernel_timing(ctx, 2) (zeros otherwise: each stage event
 * costs queue time on the proof stream). */
int zkl_hip_stage_times(const zkl_ctx* ctx, double* out_ms, int max_n);

/* Per-kernel-family device time of the last proof, measured with HIP events on the
 * ctx stream around each launch: out_ms[i] = summed ms, out_launches[i] = launches.
 * *names receives a static '\n'-separated list of the family names. */
#define ZKL_NUM_KFAMILIES 9
int zkl_hip_kernel_times(const zkl_ctx* ctx, double* out_ms, int* out_launches, int max_n, const char** names);
/* Which kernel families zkl_hip_kernel_times covers for the following proofs: 0 none,
 * 1 the trace row hash only (default: every bracket costs ~10 us of queue time), 2 all
 * families and the stage boundaries of zkl_hip_stage_times. */
int zkl_hip_set_kernel_timing(zkl_ctx* ctx, int mode);

/* ---- device memory (the library's own HIP runtime; callers need no torch) --- */
int zkl_hip_device_count(int* count);
int zkl_hip_device_alloc(zkl_ctx* ctx, size_t bytes, void** d_ptr);
int zkl_hip_device_free(zkl_ctx* ctx, void* d_ptr);
/* kind: 1 = host->device, 2 = device->host, 3 = device->device; synchronous */
int zkl_hip_memcpy(zkl_ctx* ctx, void* dst, const void* src, size_t bytes, int kind);
int zkl_hip_synchronize(zkl_ctx* ctx);

/* ---- reference helpers the host needs on its side ------------------------ */
/* utils::select_partitions_for_trace (utils.rs:394-409). */
void zkl_select_partitions(uint32_t trace_width, uint32_t trace_length,
                           uint32_t* num_partitions, uint32_t* hash_rate);

/* ---- stage entry points (parity tests call these through the same ABI) ----- */
/* PoseidonHasher::hash_elements over each row of a column-major matrix, with the
 * row partitioning Winterfell applies (partition_size, merge_many); d_* are device
 * pointers on ctx's device.  digests_out: n_rows field elements (digest low 16 B). */
int zkl_hip_hash_rows(zkl_ctx* ctx, const void* d_matrix, uint32_t n_cols, uint32_t n_rows,
                      uint32_t num_partitions, uint32_t hash_rate, void* d_digests_out);
/* MerkleTree::new over n_leaves digests (field-element form); writes all 2*n nodes
 * (nodes[1] = root, nodes[n+i] = leaf i) to d_nodes_out. */
int zkl_hip_merkle_tree(zkl_ctx* ctx, const void* d_leaves, uint32_t n_leaves, void* d_nodes_out);
/* n_states Poseidon permutations (poseidon/hasher.rs:173-190, suite [0;32]) of 12-element
 * canonical states, in place.  engine 1 = matrix-core form (the one the commitment kernels
 * use on large levels), 2 = its 16-state form (levels of 2^13 and 2^14 states), 0 = lane-group
 * form.  Stage entry point for parity tests. */
int zkl_hip_poseidon_permute(zkl_ctx* ctx, void* d_states, uint32_t n_states, int engine);
/* Process-wide hashing policy: engine 1 (default) runs Poseidon levels of at least
 * pm_min_items states (default 16384) on the 32-state matrix-core permutation, and Merkle
 * levels and FRI leaf layers inside the 16-state band (default [2^13, 2^15) states,
 * ZKL_PM16=lo,hi moves it, ZKL_PM16=0 disables it) on the 16-state matrix-core form whatever
 * pm_min_items is; engine 0 keeps every level on lane groups.  All forms give identical
 * digests; this only moves time. */
int zkl_hip_set_hash_policy(int engine, uint32_t pm_min_items);
/* Process-wide row-digest rule for partitioned rows that form a single chunk (partition
 * size > row width: the 7-column composition rows from 2^14 trace rows up, any matrix
 * narrower than its partition size).  0 (default): winterfell 0.13.1
 * RowMatrix::commit_to_rows — merge_many over the chunk digests whenever partition_size !=
 * num_cols, even of one digest; 1: the reference's own re-implementation
 * hash_row_poseidon (agg/child.rs:1025-1045), which returns a single chunk digest as is.
 * Rows of several chunks and unpartitioned rows hash identically under both (DESIGN.md
 * §3.1).  zkl_hip_row_digest_rule() returns the rule in force. */
int zkl_hip_set_row_digest_rule(int rule);
int zkl_hip_row_digest_rule(void);
/* Process-wide NTT form for evaluation (DIT) passes: 1 (default) lazily reduced 26-bit limbs
 * inside a pass, 0 the canonical-form kernel, 2 the lazy form with its 8-stage passes on the
 * matrix cores (slower on gfx950).  Identical results; for parity tests /
 * A-B. */
int zkl_hip_set_ntt_mode(int mode);
/* Coset low-degree extension of column-major n_cols x n_rows evaluations over
 * GENERATOR * <w_{n*blowup}>; writes coefficients (n_cols x n_rows) and the LDE
 * (n_cols x n_rows*blowup), both column-major, natural order. */
int zkl_hip_lde(zkl_ctx* ctx, const void* d_values, uint32_t n_cols, uint32_t n_rows,
                uint32_t blowup, void* d_coeffs_out, void* d_lde_out);

/* Raw in-place radix-2 NTT on n_cols contiguous device columns of length n (stage test
 * entry point).  dif != 0: natural order in, bit-reversed out (Gentleman-Sande);
 * dif == 0: bit-reversed in, natural out (Cooley-Tukey).  inverse selects w_n^-1; no 1/n
 * scaling.  out[k] = sum_j in[j] * w^(j*k) in the respective orders. */
int zkl_hip_ntt(zkl_ctx* ctx, void* d_data, uint32_t n_cols, uint32_t n, int dif, int inverse);

/* ---- verification (host, no device work) ------------------------------------
 * winter-verifier 0.13.1 for one segment proof (verify_proof, prove.rs:802-941): context and
 * options (must equal opts), commitments, transcript replay (agg/fs.rs:67-237), the
 * out-of-domain constraint identity (transition constraints of ZkLispAir + every assertion),
 * proof of work, query positions, trace / constraint / FRI Merkle openings, DEEP values, FRI
 * folds and remainder.  ZKL_OK when the proof verifies; ZKL_E_INVALID with
 * zkl_hip_last_error(NULL) naming the first failing check otherwise. */
int zkl_verify_segment(const uint8_t* proof, size_t len, const zkl_air_public_inputs* pi,
                       const zkl_proof_options* opts);

/* ---- workload generator (host, not the measured path) -------------------- */
/* Synthetic VM-only straight-line segment: 2^log_n rows, width 204
 * ({vm, rom} layout), ops cycling Const/Add/Mov/Mul over r0..r7 with splitmix64
 * immediates; trace built the way vm/trace/{mod,vm,rom}.rs build it.  Writes the
 * column-major trace (204 x 2^log_n) and the AIR public inputs. */
int zkl_synth_vm_segment(uint64_t seed, uint32_t log_n, zkl_f128* trace_out,
                         zkl_air_public_inputs* pi_out, uint32_t* width_out);
/* Same with program flags (flags = 0 is zkl_synth_vm_segment); the trace is built in the
 * segment layout the features imply ({vm, rom} 204, {vm, ram, rom} 212, {vm, merkle, rom} 211,
 * all 219, vm/layout.rs:183-313):
 *   ZKL_SYN_SPONGE  SAbsorbN / SSqueeze ops (vm/trace/vm.rs:565-672): FM_SPONGE | FM_POSEIDON,
 *                   PoseidonAir block (vm/air/poseidon.rs:26-162)
 *   ZKL_SYN_RAM     Load / Store over 8 addresses (vm.rs:803-842): FM_RAM, RamAir block
 *                   (vm/air/ram.rs:26-236) incl. the delta_clk range gadget
 *   ZKL_SYN_MERKLE  one MerkleStepFirst/Step/Last path (vm.rs:675-800): FM_MERKLE | FM_POSEIDON,
 *                   MerkleAir block (vm/air/merkle.rs:26-134); needs log_n >= 8 */
#define ZKL_SYN_SPONGE 1u
#define ZKL_SYN_RAM 2u
#define ZKL_SYN_MERKLE 4u
int zkl_synth_vm_segment_ex(uint64_t seed, uint32_t log_n, uint32_t flags, zkl_f128* trace_out,
                            zkl_air_public_inputs* pi_out, uint32_t* width_out);
/* Same with the program identity taken from program_seed (the ops still from seed) and ROM
 * lane 0 entering the first level at *rom0_in (NULL: 0), so that consecutive synthetic
 * segments are segments of one program and form the accumulator chain the aggregation checks
 * (agg/trace.rs:524-541: rom_s_in[0] of segment i+1 == rom_s_out[0] of segment i). */
int zkl_synth_vm_segment_chain(uint64_t program_seed, uint64_t seed, uint32_t log_n, uint32_t flags, const zkl_f128* rom0_in,
                               zkl_f128* trace_out, zkl_air_public_inputs* pi_out, uint32_t* width_out);

/* ---- op-list trace builder ------------------------------------------
 * zk_lisp_compiler::builder::Op (builder.rs:25-158), one op per 32-row level.  Field use:
 *   CONST dst imm | MOV dst a(=src) | ADD/SUB/MUL/EQ dst a b | NEG dst a | SELECT dst c a b
 *   ASSERT dst c | ASSERT_BIT, ASSERT_RANGE_LO, ASSERT_RANGE_HI dst c(=r)
 *   ASSERT_RANGE dst c(=r) bits | DIVMOD dst(=dst_q) dst2(=dst_r) a b
 *   DIVMOD128 a(=a_hi) c(=a_lo) b dst(=dst_q) dst2(=dst_r) | MULWIDE dst(=dst_lo) dst2(=dst_hi) a b
 *   LOAD dst a(=addr) | STORE a(=addr) b(=src) | SABSORBN n_regs regs[] | SSQUEEZE dst
 *   MERKLE_FIRST dst(=leaf_reg) a(=dir_reg) b(=sib_reg) | MERKLE_STEP, MERKLE_LAST a(=dir) b(=sib)
 *   END
 * Register indices < 8. */
enum {
  ZKL_OP_CONST = 0, ZKL_OP_MOV, ZKL_OP_ADD, ZKL_OP_SUB, ZKL_OP_MUL, ZKL_OP_NEG, ZKL_OP_EQ, ZKL_OP_SELECT,
  ZKL_OP_ASSERT, ZKL_OP_ASSERT_BIT, ZKL_OP_ASSERT_RANGE, ZKL_OP_ASSERT_RANGE_LO, ZKL_OP_ASSERT_RANGE_HI,
  ZKL_OP_DIVMOD, ZKL_OP_DIVMOD128, ZKL_OP_MULWIDE, ZKL_OP_LOAD, ZKL_OP_STORE, ZKL_OP_SABSORBN, ZKL_OP_SSQUEEZE,
  ZKL_OP_MERKLE_FIRST, ZKL_OP_MERKLE_STEP, ZKL_OP_MERKLE_LAST, ZKL_OP_END
};
typedef struct {
  uint32_t kind;
  uint8_t dst, dst2, a, b, c, bits, n_regs, reserved;
  uint8_t regs[10];
  uint64_t imm;
} zkl_op;
/* build_full_trace (vm/trace/mod.rs:434-524) of a program: n_rows = 32 * next_pow2(n_ops)
 * (levels past the last op keep only the schedule gates, pc and domain tags), initial registers
 * from secret_args (u64, r0..) and main_args flattened into slots in the tail registers
 * (vm.rs:64-104), the VM, RAM and ROM builders (vm.rs, ram.rs, rom.rs), written in the segment
 * layout of the features the ops use (sponge ops: FM_SPONGE | FM_POSEIDON, Load / Store:
 * FM_RAM, Merkle steps: FM_MERKLE | FM_POSEIDON; vm/layout.rs:183-313).  Also the AIR public
 * inputs prove_segment derives for the whole trace as one segment (prove.rs:292-423; merkle_root
 * = the accumulator after the last MerkleStepLast).  rom0_in: ROM lane 0 entering the first
 * level (NULL: 0).  trace_out NULL: only *width_out / *n_rows_out.  ZKL_E_INVALID on a register
 * index > 7, more than 10 pending absorbs (push_absorb, vm.rs:925-935), more than 8 main-arg
 * slots, or an unknown kind. */
int zkl_build_trace(const zkl_op* ops, uint32_t n_ops, const uint8_t program_id[32],
                    const uint8_t program_commitment[32], const uint64_t* secret_args, uint32_t n_secret,
                    const zkl_vm_arg* main_args, uint32_t n_main, const zkl_f128* rom0_in, zkl_f128* trace_out,
                    zkl_air_public_inputs* pi_out, uint32_t* width_out, uint32_t* n_rows_out);
/* rom_acc_from_program (romacc.rs:22-80): the t=3 ROM accumulator over the ops' virtual map rows
 * (opcode bit + register selectors, romacc.rs:82-260), next_pow2(n_ops) levels from state 0 —
 * what the verifier recomputes for pi.rom_acc when the commitment is non-zero (prove.rs:815-821,
 * lib.rs:210-214).  Equals the trace's rom_acc for a one-segment trace built from rom0 = 0. */
int zkl_rom_acc_from_program(const zkl_op* ops, uint32_t n_ops, const uint8_t program_id[32], zkl_f128 out[3]);

/* WinterfellSegmentPlanner::plan_segments (segment_planner.rs:93-276): the row ranges
 * [r_starts[i], r_ends[i]) of the segments of an n_ops program with at most max_rows rows per
 * segment (the reference's default is 1 << 12, ZKL_MAX_SEGMENT_ROWS).  r_starts / r_ends NULL:
 * only *count; otherwise cap >= *count entries are written. */
int zkl_plan_segments(uint32_t n_ops, uint32_t max_rows, uint32_t* r_starts, uint32_t* r_ends, uint32_t cap,
                      uint32_t* count);
/* prove_segment's inputs for rows [r_start, r_end) of a zkl_build_trace trace (prove.rs:1057-1134):
 * the segment feature mask from the ops of its levels (segment_planner.rs:283-334), the columns of
 * that layout (slice_trace_segment_with_layout), the AIR public inputs with the boundary values
 * (compute_segment_boundary_bytes, prove.rs:1197-1287) and the segment-local VM output / usage
 * mask (build_air_pi_for_trace), and the VM state hashes of its first and last rows
 * (utils::vm_state_hash_row_with_layout, for the zl1 step).  r_start, r_end multiples of 32,
 * r_end - r_start a power of two.  trace_out NULL: only *width_out. */
int zkl_slice_segment(const zkl_f128* full, uint32_t full_width, uint32_t n_full, const zkl_op* ops, uint32_t n_ops,
                      const zkl_air_public_inputs* pi_full, uint32_t r_start, uint32_t r_end, zkl_f128* trace_out,
                      zkl_air_public_inputs* pi_out, uint32_t* width_out, uint8_t state_in[32], uint8_t state_out[32]);

/* Per-segment trace builder: what prove_segment's input side (prove.rs:1057-1134,
 * build_segment_trace_with_state_without_full mod.rs:316-365 over build_full_trace mod.rs:434-524)
 * produces, without the full trace in memory.  zkl_program_new executes the program once (same
 * arguments as zkl_build_trace) and keeps the VM carry every 32 levels, the RAM event log with the
 * sorted table's running sums, ROM lane 0, rom_acc and the Merkle root; *full_width_out /
 * *n_rows_out receive the full trace's shape.  zkl_build_segment_trace then writes rows [r_start,
 * r_end) in the segment's layout with its AIR public inputs and VM state hashes -- bit for bit
 * what zkl_slice_segment(zkl_build_trace(..), .., r_start, r_end, ..) returns (same alignment
 * rules; trace_out NULL: only *width_out).  Calls on one program may run concurrently.
 * examples/fib-2pow16.zlisp (2^24 rows) is built this way segment by segment. */
typedef struct zkl_program zkl_program;
int zkl_program_new(const zkl_op* ops, uint32_t n_ops, const uint8_t program_id[32],
                    const uint8_t program_commitment[32], const uint64_t* secret_args, uint32_t n_secret,
                    const zkl_vm_arg* main_args, uint32_t n_main, const zkl_f128* rom0_in, zkl_program** out,
                    uint32_t* full_width_out, uint32_t* n_rows_out);
int zkl_build_segment_trace(const zkl_program* prog, uint32_t r_start, uint32_t r_end, zkl_f128* trace_out,
                            zkl_air_public_inputs* pi_out, uint32_t* width_out, uint8_t state_in[32],
                            uint8_t state_out[32]);
void zkl_program_free(zkl_program* prog);

/* ---- zl1 step proof (host-side, no device work) ----------------------------------
 * StepProof::to_bytes (proof/step.rs:79-151) of the step proof prove_segment builds around
 * an inner proof from zkl_hip_prove_segment*: "ZKLSTP1" | lambda | suite | core pi |
 * main_args | vm_usage_mask | ram_delta_clk_bits | rom_acc | segment index/total | pc_init |
 * state hashes | boundary bytes | inner proof (length-prefixed).  Buffer released with
 * zkl_hip_free. */
int zkl_step_proof_encode(const zkl_air_public_inputs* pi, const zkl_step_info* info, const uint8_t* inner,
                          size_t inner_len, uint8_t** out, size_t* out_len);
/* Decode a ZKLSTP1 encoding (StepProof::from_bytes, step.rs:153-493) and return the zl1
 * commitment echo root_trace = BLAKE3("zkl/step/root_trace" | suite | trace roots |
 * constraint root | FRI roots) (format.rs:214-238) and the step digest
 * (proof/digest.rs:16-68).  Either output may be NULL.  Errors: ZKL_E_INVALID with
 * zkl_hip_last_error(NULL) naming the truncated/invalid field, as step.rs does. */
int zkl_step_proof_digest(const uint8_t* step, size_t len, uint8_t digest_out[32], uint8_t root_trace_out[32]);
/* agg::child::children_root_from_compact (agg/child.rs:853-895): the aggregation's root
 * over n children given as n x 32-byte step digests and n x 32-byte zl1 root_trace values
 * (what zkl_step_proof_digest returns), under the Poseidon suite of suite_id.  Rank 0 of
 * a multi-GPU run computes it after gathering the step proofs. */
int zkl_children_root(const uint8_t suite_id[32], const uint8_t* digests, const uint8_t* root_traces, uint32_t n,
                      uint8_t root_out[32]);

/* ---- aggregation proof -------------------------------------
 * zk_lisp_proof::ProverOptions as the aggregation reads it (zk-lisp-proof/src/lib.rs:40-66). */
typedef struct {
  uint32_t queries;           /* the aggregation proves with max(queries, 16) (prove.rs:645) */
  uint32_t blowup;
  uint32_t grind;
  uint32_t min_security_bits; /* >= 128: FieldExtension::Quadratic, else None (prove.rs:647-651);
                                 >= 64: conjectured-security check (prove.rs:664-681) */
  uint32_t trace_mode;        /* ZKL_AGG_TRACE_VALID (0) or ZKL_AGG_TRACE_REFERENCE (1), below */
} zkl_agg_options;

/* Aggregation trace modes.
 * ZKL_AGG_TRACE_VALID: next_pow2(max(children + 1, 8)) rows (one padding row always, so the
 *   last-row assertions of agg/air.rs:276-304 can hold) and zero root-error columns (every
 *   opening was verified against its root under the library's row-digest rule); the batch must
 *   satisfy ZlAggAir, otherwise ZKL_E_INVALID.  This is what zkl_agg_prove writes to proof.bin.
 * ZKL_AGG_TRACE_REFERENCE: the trace agg/trace.rs:397-398,553-690 builds -- PARITY UNPINNED:
 *   checked only against the Python restatement oracle/agg_ref.py (no fixture from the reference
 *   exists; its batch-proof decompression order and partition_size are [WF-recall] rules), so
 *   "the reference's trace" means "the restatement of agg/trace.rs", not bytes seen from it:
 *   next_pow2(max(children, 8)) rows and root-error columns sum_k(root_k - root) where root_k is
 *   reproduced from the opening's row under hash_row_poseidon (agg/child.rs:1025-1045, one chunk
 *   not merged).  No AIR check, like the reference's release prover: for a power-of-two child
 *   count >= 8, or children whose composition rows are one chunk (n >= 2^14), the proof does
 *   not verify, as the reference's would not. */
#define ZKL_AGG_TRACE_VALID 0u
#define ZKL_AGG_TRACE_REFERENCE 1u

/* What `zk-lisp prove` does after the segment proofs (replaces the Rust calls
 * RecursionPublicBuilder::build_public lib.rs:404-482, RecursionBackend::prove lib.rs:295-344
 * -> prove_agg_proof prove.rs:629-719, RecursionArtifactCodec::encode lib.rs:486-551):
 * n ZKLSTP1 step proofs in, the ZKLRC1 artifact (the aggregation proof inside) out, plus the
 * recursion digest (recursion_digest_from_agg_pi, prove.rs:585-616) when digest_out != NULL.
 * Each child's Fiat-Shamir transcript is replayed from its step proof alone (agg/fs.rs:38-245)
 * and every opening, DEEP value, FRI fold, remainder and PoW is checked; a child that fails
 * is rejected (ZKL_E_INVALID) rather than aggregated into an unsatisfiable trace.  The
 * artifact is freed with zkl_hip_free.  Host-only (no ctx, no device). */
int zkl_agg_prove(const uint8_t* const* steps, const size_t* step_lens, uint32_t n_steps,
                  const zkl_agg_options* opts, uint8_t** artifact_out, size_t* artifact_len,
                  uint8_t digest_out[32]);
/* RecursionArtifactCodec::decode (lib.rs:552-660) + RecursionBackend::verify (lib.rs:346-372)
 * -> verify_agg_proof (prove.rs:732-791): decodes a ZKLRC1 artifact and verifies the
 * aggregation proof under ZlAggAir and the artifact's public inputs, accepting proof options
 * whose conjectured security (estimate_conjectured_security_bits, prove.rs:1177-1195) is at
 * least min_security_bits.  ZKL_OK, or ZKL_E_INVALID with zkl_hip_last_error(NULL) naming the
 * failing check.  Host-only. */
int zkl_agg_verify(const uint8_t* artifact, size_t len, uint32_t min_security_bits);
/* The aggregation trace of the same batch (build_agg_trace_from_transcripts,
 * agg/trace.rs:155-238): 31 columns x rows, column-major; rows_out receives the row count
 * (a power of two >= 8); out may be NULL to query it.  zkl_agg_trace builds the
 * ZKL_AGG_TRACE_VALID trace; zkl_agg_trace_mode takes the mode. */
int zkl_agg_trace(const uint8_t* const* steps, const size_t* step_lens, uint32_t n_steps,
                  zkl_f128* out, uint32_t max_rows, uint32_t* rows_out);
int zkl_agg_trace_mode(const uint8_t* const* steps, const size_t* step_lens, uint32_t n_steps,
                       uint32_t trace_mode, zkl_f128* out, uint32_t max_rows, uint32_t* rows_out);

/* ---- multi-GPU boundary exchange --------------------------
 * One process per GPU proves its own segments; the step proofs (zl1 ZKLSTP1 bytes with the
 * boundary fields the aggregation chains: state hashes, RAM grand products, ROM lanes) are
 * gathered on the aggregating rank with RCCL point-to-point transfers over xGMI.  Replaces the
 * reference's in-process Vec<StepProof> hand-off (prove.rs:1018-1050 -> lib.rs:382-482).
 * RCCL is opened at run time; without it these calls fail with ZKL_E_INVALID and
 * zkl_hip_last_error(NULL) says why (the single-GPU path does not need it). */
typedef struct zkl_comm zkl_comm;
/* ZKL_OK when RCCL can be opened here (checked by every rank before the collective init, so
 * that no rank enters ncclCommInitRank alone). */
int zkl_comm_available(void);
/* ncclGetUniqueId on the root rank; the 128 bytes go to the other ranks out of band
 * (bench.py / zkl_hip.dist use the torch.distributed store). */
int zkl_comm_unique_id(uint8_t id_out[128]);
/* ncclCommInitRank on `device` (collective over the world). */
int zkl_comm_init(int device, int world, int rank, const uint8_t id[128], zkl_comm** out);
/* Collective: every rank contributes `len` host bytes; on `root`, *out (free with
 * zkl_hip_free) receives the world blobs concatenated in rank order and lens_out[world] their
 * lengths (other ranks may pass NULL).  Lengths are all-gathered first, then each rank's blob
 * is sent to the root (grouped ncclSend / ncclRecv on the comm's stream). */
int zkl_comm_gather_bytes(zkl_comm* comm, const uint8_t* data, size_t len, int root, uint8_t** out,
                          size_t* lens_out);
/* Device time (ms, HIP events on the comm stream) of the last gather: length exchange + sends. */
double zkl_comm_last_ms(const zkl_comm* comm);
void zkl_comm_destroy(zkl_comm* comm);

#ifdef __cplusplus
}
#endif
#endif
