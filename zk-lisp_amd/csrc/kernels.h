// Launch wrappers for the gfx950 kernels of the segment prover (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>
#include "air_host.h"
#include "field.h"

namespace zkl {

// HIP runtime failure (mapped to ZKL_E_DEVICE at the C ABI, with the failing call or kernel)
struct DeviceError : std::runtime_error { using std::runtime_error::runtime_error; };
#define ZKL_HIPCHECK(x)                                                                       \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) throw ::zkl::DeviceError(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
// after a group of kernel launches: a failed launch (bad configuration, resources) surfaces
// here with the group's name instead of at some later synchronisation
inline void check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw DeviceError(std::string("kernel launch failed (") + what + "): " + hipGetErrorString(e));
}

struct HasherConsts {  // PoseidonHasher suite [0;32] + folded domain labels
  fe mds[144];
  fe rc[27 * 12];
  fe dom[2];
  fe dom_elems, dom_merge, dom_many, dom_int;
};

// Montgomery/26-bit-limb form of the hasher constants used by the device permutation
// (R = 2^156 mod p; every constant stored as 5 little-endian 26-bit limbs of x*R mod p).
struct HasherMont {
  uint32_t mds[12][12][5];
  uint32_t rc[27][12][5];
  uint32_t dom[2][5];
  uint32_t r2[5];      // R^2 mod p (converts a canonical element into Montgomery form)
  uint32_t dfe[4][5];  // Montgomery domain labels: elements, merge, merge_many, merge_with_int
  // the same entry constants for the matrix-core permutation, whose Montgomery radix is
  // R' = 2^130 (five REDC digit steps instead of six; poseidon_mfma.inc)
  uint32_t dom130[2][5];
  uint32_t r2_130[5];  // R'^2 mod p
  uint32_t dfe130[4][5];
  // the 48-lane permutation (poseidon.hip pw_permute): MDS entries weighted by limb position,
  // mdsl[i][k][u] = limbs of M[i][k] * 2^(26u) mod p (plain, canonical), and the round
  // constants in R' form
  uint32_t mdsl[12][12][5][5];
  uint32_t rc130[27][12][5];
  // round-1 cubes of the constant state elements of a sponge's first block, packed as the
  // matrix-core form's B words (four offset-byte words + the top): zero (element with no
  // message) and the two tag lanes dom130[0], dom130[1] (poseidon_mfma.inc pm_permute)
  uint32_t pmk0[5];
  uint32_t pmkt[2][5];
};
HasherMont make_hasher_mont(const HasherConsts& h);
void upload_hasher_mont(const HasherMont& m, hipStream_t s);
// matrix-core permutation tables (A digits of the MDS, round constants), built once
void upload_pm_tables(const HasherConsts& h, hipStream_t s);
// 1 = matrix-core permutation on throughput-bound levels (default), 0 = lane groups only
int hash_engine();
void set_hash_policy(int engine, size_t min_items);
// one-chunk row digest rule (launch_hash_rows): 0 winterfell commit_to_rows, 1 agg/child.rs
void set_row_digest_rule(int rule);
int row_digest_rule();
// DIT passes on lazily reduced limbs (default) or the canonical kernel
void set_ntt_lazy(bool on);
const char* poseidon_build_config();  // poseidon.hip
const char* kernels_build_config();   // kernels.hip
// n Poseidon permutations of 12-element canonical states in place (engine as above)
void launch_permute(fe* d_states, size_t n, int engine, hipStream_t s);
struct CeParams;
struct DerivedConsts;
struct ProofConsts;  // per-proof constants in device memory, one block per context (below)
void upload_air_consts(ProofConsts* dK, const AirDevice& a, hipStream_t s);
// transition composition coefficients alpha_j: copied device->device from the draw buffer
void upload_alphas_from_device(ProofConsts* dK, const fe* d_alphas, int n, hipStream_t s);
// dK->pose_k from dK->alpha and the AIR's round constants (after upload_alphas_from_device; the
// Poseidon block's alphas come first in the evaluation order), and the prefix sums dD->apre of
// the first n_tc alphas (the constraint groups of air_eval.h)
void launch_pose_k(const ProofConsts* dK, DerivedConsts* dD, int n_tc, bool pose, hipStream_t s);
// The DEEP coefficients straight from the draw buffer (no host round trip): dD->deep,
// dD->deep_m (limbs of g * 2^156) and dD->deep_sz from the OOD frame d_frame (t(z) [W] | H(z) [C]
// | t(zg) [W] | H(zg) [C]).  n = W + C <= 256.
void launch_deep_coeffs(const fe* d_gam, uint32_t W, uint32_t C, const fe* d_frame, DerivedConsts* dD, hipStream_t s);

// ---- hashing --------------------------------------------------------------
// Row digests of a column-major matrix (ld = rows per column) with Winterfell partitioning.
// d_tmp: scratch of n_parts * n_rows elements (unused when a single hash covers the row).
// tag: 0 = trace commitment, 1 = composition commitment (distinct kernel symbols in profiles)
// split: d_mat is a trace LDE in the split layout; the kernels walk positions q (whole lines)
// and write each digest to its row lde_row(q).
void launch_hash_rows(const fe* d_mat, uint32_t n_cols, size_t n_rows, uint32_t num_partitions,
                      uint32_t hash_rate, fe* d_tmp, fe* d_out, hipStream_t s, int tag = 0, int split = 0);
// Merkle tree: d_nodes[n..2n) must hold the leaves; fills d_nodes[1..n).
// coin_mode (d_coin, d_root_out): the transcript step after the tree runs in the launch that
// reaches the root -- 1: coin[0] = merge(coin[0], root) (the trace / constraint root reseed), 2:
// that and coin[1] = merge_with_int(coin[0], 1) (a FRI layer's alpha); the root is copied to
// *d_root_out when that is not null
void launch_merkle(fe* d_nodes, size_t n_leaves, hipStream_t s, fe* d_coin = nullptr, fe* d_root_out = nullptr,
                   int coin_mode = 0);
// out[i] = merge_with_int(seed, base + 1 + i)   (RandomCoin::draw, counter base+1+i)
// d_seed != nullptr: the seed is read from device memory (the device-side transcript)
void launch_draws(fe seed, uint64_t base, size_t k, fe* d_out, hipStream_t s, const fe* d_seed = nullptr);
// smallest nonce in [base, base+count) with trailing_zeros(merge_with_int(seed, nonce)) >= bits
void launch_grind(fe seed, uint64_t base, uint32_t count, uint32_t bits, unsigned long long* d_best, hipStream_t s,
                  const fe* d_seed = nullptr);
// Device-side transcript (DefaultRandomCoin with the seed in device memory):
// coin[0] = merge(coin[0], *value) and *value_out = *value (nullable)
// FRI remainder coefficients (rem[0..rlen), highest degree first), their hash_elements
// commitment rem[rlen], and coin[0] = merge(coin[0], rem[rlen]); wk[k] = w^-k, sk[k] = 3^-k / Nr
void launch_fri_remainder(const fe* d_ev, uint32_t Nr, uint32_t rlen, const fe* wk, const fe* sk, fe* d_coin,
                          fe* d_rem, hipStream_t s);
// coin[1] = merge_with_int(coin[0], *d_best) when *d_best != ~0 (the query seed)
void launch_query_seed(fe* d_coin, const unsigned long long* d_best, hipStream_t s);

// ---- NTT ---------------------------------------------------------------------
// Twiddle table in Montgomery/26-bit-limb form (entry = limbs of w * 2^156 mod p),
// split into limbs 0..3 (l4) and limb 4 (l1); a twiddle product is then one REDC.
struct MontTab {
  const uint4* l4;
  const uint32_t* l1;
};
// host: fill a device buffer of N*20 bytes (l4 then l1) from the canonical table w[0..N)
void build_mont_table(const fe* h_w, size_t N, void* d_buf, hipStream_t s);
inline MontTab mont_tab(const void* d_buf, size_t N) {
  return MontTab{(const uint4*)d_buf, (const uint32_t*)((const char*)d_buf + N * 16)};
}
// In-place radix-2 stages on n_cols contiguous columns of length N (power of two).
// dif=true : stages H = 2^hi_log .. 2^lo_log (descending), natural -> bit-reversed
// dif=false: stages H = 2^lo_log .. 2^hi_log (ascending),  bit-reversed -> natural
// roots: stage-major Montgomery table (build_mont_table) of size Ntab >= N; tables built from
// inverse roots give inverse transforms.
void launch_ntt_stages(fe* d_data, size_t n_cols, size_t N, bool dif, int lo_log, int hi_log,
                       MontTab roots, size_t Ntab, hipStream_t s);
// Coset LDE evaluation: d_coef holds per column the bit-reversed coefficients already scaled
// by the coset shift (c_k * 3^k at position bitrev(k)); d_out (N per column, natural order)
// = evaluations over 3*<w_N>.  The first DIT pass reads the blowup copies straight from
// d_coef.
// want_split: store the evaluations in the split layout (lde_pos below) when the last pass
// supports it; returns 1 when the output is split, 0 when it is in natural order.
// all stages of a DIF iNTT of n-element columns (natural in, bit-reversed out), reading src
// (nullptr: in place in d) and storing element i of each column times scale[bitrev(i)]
void launch_intt_scaled(const fe* d_src, fe* d_data, size_t n_cols, size_t n, MontTab iroots, size_t Ntab,
                        const fe* d_scale, hipStream_t s);
int launch_lde_from_coeffs(const fe* d_coef, size_t n_cols, size_t n, size_t N, MontTab roots, size_t Ntab, fe* d_out,
                           hipStream_t s, bool want_split = false);
// Even/odd split layout of a trace LDE column.  Write the N = 256 S rows as
// r = L + t S (L < S, t < 256); the last DIT pass owns, per block, 8 consecutive L (L0 + l)
// and all t, and must store in place, so the layout permutes within that set: row (L, t) goes
// to L' = L0 + l / 2 + 4 (t & 1), t' = t / 2 + 128 (l & 1).  Every even row thus sits in the
// first half of its column (the constraint evaluator reads only those, in whole 128-byte
// lines) and every line holds eight rows of one parity.  Needs S >= 8.
__host__ __device__ inline size_t lde_pos(size_t r, size_t N, int split) {
  if (!split) return r;
  const int logS = __builtin_ctzll((unsigned long long)N) - 8;
  const size_t S = (size_t)1 << logS;
  const size_t L = r & (S - 1), t = r >> logS, l = L & 7;
  return (L - l) + (l >> 1) + ((t & 1) << 2) + (((t >> 1) + ((l & 1) << 7)) << logS);
}
// inverse of lde_pos: the row stored at position q
__host__ __device__ inline size_t lde_row(size_t q, size_t N, int split) {
  if (!split) return q;
  const int logS = __builtin_ctzll((unsigned long long)N) - 8;
  const size_t S = (size_t)1 << logS;
  const size_t Lp = q & (S - 1), tp = q >> logS, m = Lp & 7;
  const size_t l = ((m & 3) << 1) | (tp >> 7), t = ((tp & 127) << 1) | (m >> 2);
  return (Lp - m) + l + (t << logS);
}
// out[c*N + B*j + t] = in[c*stride + off + src(j)*estride] * scale[bitrev_n(j)] * mult for t < B (B = N/n);
// src(j) = j or n-1-j
void launch_broadcast(const fe* d_in, size_t in_col_stride, size_t in_elem_stride, size_t in_offset,
                      size_t n_cols, size_t n, size_t N, const fe* d_scale, fe mult, bool reverse, fe* d_out, hipStream_t s);
// data[i] *= scale[bitrev(i)] on contiguous columns (post-DIF scaling)
void launch_scale_bitrev(fe* d_data, size_t n_cols, size_t n, const fe* d_scale, hipStream_t s);

// ---- constraint evaluation ---------------------------------------------------
struct CeParams {
  size_t n, N, ce;            // trace length, LDE size, CE size
  uint32_t blowup;            // LDE blowup (row step between cur and next)
  fe gl;                      // g^(n-1)
  fe inv_n;                   // 1/n
  fe xn_inv[64];              // 1/(x^n - 1) for x^n = 3^n * w_(ce/n)^j
  fe xn_m1[64];               // x^n - 1
  fe lagr;                    // g^(n-1)/n
  uint32_t n_bcols;           // number of asserted columns in the boundary tables
  uint32_t bcol[64];          // their trace column indices
};
// Per-proof constants live in a per-context device block (not __constant__ symbols) so that
// several contexts can prove concurrently on one device.
struct ProofConsts {
  AirDevice air;
  CeParams ce;
  fe alpha[1024];  // transition composition coefficients
};
// Per-proof constants the device derives itself (written by kernels, read by later kernels),
// kept apart from ProofConsts, which only host/device copies write.
struct DerivedConsts {
  fe pose_k[27];            // sum_i alpha_{12j+i} rc[j][i] per Poseidon round (launch_pose_k)
  fe apre[1025];            // alpha prefix sums: apre[i] = alpha_0 + .. + alpha_(i-1) (launch_pose_k)
  fe deep[512];             // DEEP coefficients (trace then composition columns)
  uint32_t deep_m[512][5];  // the same as 26-bit limbs of g * 2^156 mod p (deep_kernel)
  fe deep_sz[2];            // sum_i g_i * frame_i(z), sum_i g_i * frame_i(z g) (deep_coeffs_kernel)
};
void launch_constraint_eval(const fe* d_lde, const fe* d_roots, size_t Ntab, const fe* d_pertab,
                            const fe* d_bm /* (n_bcols + 1) x ce */, const CeParams& p, ProofConsts* dK,
                            const DerivedConsts* dD, bool pose_block, bool ram_merkle,
                            fe* d_xinv /* ce entries: 1 / (x_i - g^(n-1)) */, bool xinv_ready, fe* d_out,
                            hipStream_t s, int split = 0, fe* d_pose_part /* ce entries, Poseidon layouts */ = nullptr);
// boundary vectors: vec[slot*n + step] = beta_a ; wv[s] = sum beta_a*value_a over assertions at step s
void launch_boundary_scatter(const uint32_t* d_slot, const uint32_t* d_step, const fe* d_beta, size_t n_assert,
                             size_t n, fe* d_vecs, hipStream_t s);
void launch_boundary_w(const uint32_t* d_row_start, const fe* d_beta, const fe* d_val, size_t n, fe* d_w, hipStream_t s);
// any nonzero in data[lo, hi) on a bit-reversed vector of length N -> *d_flag = 1
void launch_check_zero_range_bitrev(const fe* d_data, size_t N, size_t lo, size_t hi, unsigned* d_flag, hipStream_t s);

// ---- OOD / DEEP / FRI ---------------------------------------------------------
// OOD evaluations as dot products with bit-reversed power vectors: for column c and point
// pt (pw1 / pw2), sum_j coef[base(c) + j * elem_stride] * pw_pt[j], j < n, where base(c) =
// off[c] (use_off) or c * col_stride; split into `chunks` partial sums per (pt, c).
struct OodArgs {
  const fe* coef;
  size_t col_stride, elem_stride, n;
  const fe* pw1;
  const fe* pw2;
  uint32_t ncols, chunks, use_off;
  uint32_t off[16];
};
void launch_ood(const OodArgs& a, fe* d_partial, hipStream_t s);
// The OOD frame from the two launch_ood partial sets: chunk sums, composition columns scaled by
// mult[j]; written in transcript order t(z) [W] | H(z) [C] | t(zg) [W] | H(zg) [C].
void launch_ood_frame(const fe* d_partial_trace, const fe* d_partial_comp, uint32_t W, uint32_t C, uint32_t chunks,
                      const fe* mult /* C host values */, fe* d_frame, hipStream_t s);
struct DeepParams {  // the frame dot products come from DerivedConsts::deep_sz (launch_deep_coeffs)
  size_t N;
  uint32_t W, C;
  fe z, zg;
};
// d_dinv[i] = 1/((x_i - z)(x_i - zg)) over the LDE coset x_i = 3*w_N^i (launch before launch_deep)
void launch_deep_denoms(const fe* d_roots, size_t Ntab, size_t N, fe z, fe zg, fe* d_dinv, hipStream_t s);
void launch_deep(const fe* d_lde, const fe* d_clde, const fe* d_roots, size_t Ntab, const DeepParams& p,
                 const DerivedConsts* dD, const fe* d_dinv /* from launch_deep_denoms */, fe* d_out, hipStream_t s,
                 int split = 0);
void launch_fri_leaves(const fe* d_ev, size_t Nd, fe* d_leaves, hipStream_t s);
// alpha read from device memory (coin[1], written by the layer tree's launch_merkle)
void launch_fri_fold(const fe* d_ev, size_t Nd, const fe* d_alpha, const fe* d_iroots, size_t Ntab, fe* d_out,
                     hipStream_t s);
// device transcript step of one FRI layer: coin[0] = merge(coin[0], *root); coin[1] = alpha
// = merge_with_int(coin[0], 1); *root_out = *root
// gather 16-byte elements from absolute device addresses
void launch_gather(const uint64_t* d_addrs, size_t k, fe* d_out, hipStream_t s);

}  // namespace zkl
