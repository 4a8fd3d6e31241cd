// gfx950 kernels for the zk-lisp segment prover.
//
// Hot loops: B = constraint evaluation (constraint_eval_kernel), C = NTTs
// (ntt_dit8_kernel, ntt_dit_lazy_kernel, ntt_pass_kernel), DEEP, FRI folds.  Hot loop A (the
// Poseidon row hashing, Merkle trees, FRI leaves, draws and grinding) is poseidon.hip.
// All arithmetic is exact f128 (field.h); bit-exactness against the oracle follows from
// computing the same residues, independent of evaluation order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <stdexcept>
#include <vector>

#include "kernels.h"
#include "air_eval.h"
#include "mont26.h"

namespace zkl {


void upload_air_consts(ProofConsts* dK, const AirDevice& a, hipStream_t s) {
  ZKL_HIPCHECK(hipMemcpyAsync(&dK->air, &a, sizeof a, hipMemcpyHostToDevice, s));
}
void upload_alphas_from_device(ProofConsts* dK, const fe* d, int n, hipStream_t s) {
  if (n > 1024) throw std::invalid_argument("more than 1024 transition constraints");
  ZKL_HIPCHECK(hipMemcpyAsync(dK->alpha, d, sizeof(fe) * n, hipMemcpyDeviceToDevice, s));
}
// one workgroup of 1024 threads: the Poseidon round constants' alpha sums (when the layout has the
// block) and the inclusive scan of the n_tc alphas in LDS (Hillis-Steele, 10 steps)
__global__ __launch_bounds__(1024) void pose_k_kernel(const ProofConsts* K, DerivedConsts* D, int n_tc, int pose) {
  const int j = (int)threadIdx.x;
  if (pose && j < 27) {
    uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 12; i++) mul_acc(K->alpha[12 * j + i], K->air.pose_rc[j][i], acc);
    D->pose_k[j] = reduce288(acc);
  }
  __shared__ fe sc[1024];
  sc[j] = j < n_tc ? K->alpha[j] : fe_zero();
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const fe add = j >= d ? sc[j - d] : fe_zero();
    __syncthreads();
    sc[j] = fe_add(sc[j], add);
    __syncthreads();
  }
  D->apre[j + 1] = sc[j];
  if (j == 0) D->apre[0] = fe_zero();
}
void launch_pose_k(const ProofConsts* dK, DerivedConsts* dD, int n_tc, bool pose, hipStream_t s) {
  if (n_tc < 0 || n_tc > 1024) throw std::invalid_argument("launch_pose_k: more than 1024 transition constraints");
  pose_k_kernel<<<1, 1024, 0, s>>>(dK, dD, n_tc, pose ? 1 : 0);
}

// =====================================================================================
// NTT: in-place radix-2 passes, up to 8 stages per pass staged through LDS.
// A pass covers global half-sizes H in {S, 2S, .., 2^(r-1) S}.  Group q of 2^r elements:
// L = q mod S, Hb = q / S, element t at Hb*S*2^r + t*S + L.  4096 elements per workgroup.
// =====================================================================================
#ifndef NTT_ELEMS_CFG
#define NTT_ELEMS_CFG 1024
#endif
#ifndef NTT_THREADS_CFG
#define NTT_THREADS_CFG 256
#endif
constexpr int NTT_ELEMS = NTT_ELEMS_CFG;      // elements per workgroup (1024: 17 KB of LDS)
constexpr int NTT_THREADS = NTT_THREADS_CFG;  // threads per workgroup

__device__ __forceinline__ uint32_t bitrev(uint32_t x, int logn) { return logn ? (__brev(x) >> (32 - logn)) : 0; }

// x * w for a twiddle w given as limbs of w*2^156 (MontTab): REDC(x * wR) = x*w, then one
// conditional subtraction makes it canonical.
__host__ __device__ __forceinline__ fe mul_tw(fe a, MontTab t, size_t e) {
  const uint4 q = t.l4[e];
  const uint32_t wm[5] = {q.x, q.y, q.z, q.w, t.l1[e]};
  uint32_t l[5], o[5];
  to26(a, l);
  mont_mul(l, wm, o);
  // the REDC result lies in (0, p + 2^100): bit 128 (limb 4, bit 24) may be set
  typedef unsigned __int128 u128;
  const u128 v = (u128)o[0] + ((u128)o[1] << 26) + ((u128)o[2] << 52) + ((u128)o[3] << 78) + ((u128)o[4] << 104);
  const u128 P = ((u128)P_HI << 64) | P_LO;
  const u128 r = (o[4] >> 24) ? v + C_RED : (v >= P ? v - P : v);  // v wrapped mod 2^128: Y - p = v + C
#ifdef NTT_CHECK
  {
    uint64_t cc[10] = {wm[0], wm[1], wm[2], wm[3], wm[4], 0, 0, 0, 0, 0};
    uint32_t wl[5];
    redc(cc, wl);
    u128 wv = (u128)wl[0] + ((u128)wl[1] << 26) + ((u128)wl[2] << 52) + ((u128)wl[3] << 78) + ((u128)wl[4] << 104);
    if (wv >= P) wv -= P;
    fe want = fe_mul(a, fe{(uint64_t)wv, (uint64_t)(wv >> 64)});
    if (want.lo != (uint64_t)r || want.hi != (uint64_t)(r >> 64))
      printf("mul_tw mismatch e=%lu a=%016lx%016lx got=%016lx%016lx want=%016lx%016lx o=%x %x %x %x %x\n", (unsigned long)e,
             (unsigned long)a.hi, (unsigned long)a.lo, (unsigned long)(uint64_t)(r >> 64), (unsigned long)(uint64_t)r,
             (unsigned long)want.hi, (unsigned long)want.lo, o[0], o[1], o[2], o[3], o[4]);
  }
#endif
  return fe{(uint64_t)r, (uint64_t)(r >> 64)};
}

// Stage-major twiddle layout: entry H + j = w_(2H)^j for H = 1, 2, 4, .., N/2 and j < H, so
// the twiddles of one radix-2 stage are contiguous (coalesced across consecutive L, and the
// small stages of a pass share a few KB that stay in L2).  Valid for any NTT size <= N.
void build_mont_table(const fe* w, size_t N, void* d_buf, hipStream_t s) {
  const fe R = fe_pow64(fe{2, 0}, 156);
  std::vector<uint32_t> l4(4 * N, 0), l1(N, 0);
  for (size_t H = 1; H < N; H *= 2) {
    const size_t step = N / (2 * H);
    for (size_t j = 0; j < H; j++) {
      uint32_t l[5];
      limbs26(fe_mul(w[j * step], R), l);
      for (int t = 0; t < 4; t++) l4[4 * (H + j) + t] = l[t];
      l1[H + j] = l[4];
    }
  }
  ZKL_HIPCHECK(hipMemcpyAsync(d_buf, l4.data(), N * 16, hipMemcpyHostToDevice, s));
  ZKL_HIPCHECK(hipMemcpyAsync((char*)d_buf + N * 16, l1.data(), N * 4, hipMemcpyHostToDevice, s));
  ZKL_HIPCHECK(hipStreamSynchronize(s));
}

// src != nullptr (first DIT pass of an LDE, first DIF pass of an out-of-place iNTT): element i
// of column c is read from src[c * (N >> src_logb) + (i >> src_logb)] instead of data, i.e. the
// blowup copies of the (scaled, bit-reversed) coefficients are generated on load rather than
// materialised.  scale != nullptr (last DIF pass): element i of a column is stored multiplied by
// scale[bitrev(i)] (the coefficient scaling of an iNTT whose output is bit-reversed).
template <bool DIF>
__global__ __launch_bounds__(NTT_THREADS) void ntt_pass_kernel(fe* __restrict__ data, size_t ncols, int logN, int r,
                                                       int logS, MontTab roots, int logTab, const fe* __restrict__ src,
                                                       int src_logb, const fe* __restrict__ scale = nullptr) {
  __shared__ fe buf[NTT_ELEMS + NTT_ELEMS / 16];
  const int R = 1 << r;
  const int G = NTT_ELEMS >> r;
  const size_t S = (size_t)1 << logS;
  const int log_gpc = logN - r;  // groups per column = N / R
  const size_t gpc = (size_t)1 << log_gpc;
  const bool gfast = S >= (size_t)G;
  const int pitch = R >= 16 ? R + 1 : R;  // pad: conflict-free 16-byte accesses
  // Block -> groups.  When a column holds whole blocks, consecutive blocks walk the columns
  // at a fixed group range, so concurrently running blocks share twiddles (same L) in L2.
  size_t col_fixed = 0, qbase = 0;
  const bool whole = gpc >= (size_t)G;
  if (whole) {
    col_fixed = blockIdx.x % (unsigned)ncols;
    qbase = (size_t)(blockIdx.x / (unsigned)ncols) * G;
  }
  auto locate = [&](int g, size_t& col, size_t& q) -> bool {
    if (whole) {
      col = col_fixed;
      q = qbase + g;
      return true;
    }
    const size_t qg = (size_t)blockIdx.x * G + g;
    col = qg >> log_gpc;
    q = qg & (gpc - 1);
    return col < ncols;
  };
  auto addr = [&](int g, int t, bool& ok) -> size_t {
    size_t col, q;
    ok = locate(g, col, q);
    const size_t L = q & (S - 1), Hb = q >> logS;
    return (col << logN) + ((Hb << logS) << r) + (size_t)t * S + L;
  };
  const size_t Nmask = ((size_t)1 << logN) - 1;
  for (int e = threadIdx.x; e < NTT_ELEMS; e += NTT_THREADS) {
    int g = gfast ? (e % G) : (e >> r);
    int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    size_t a = addr(g, t, ok);
    fe v = fe_zero();
    if (ok) v = src ? src[((a >> logN) << (logN - src_logb)) + ((a & Nmask) >> src_logb)] : data[a];
    buf[g * pitch + t] = v;
  }
  __syncthreads();
  for (int st = 0; st < r; st++) {
    const int lh = DIF ? (r - 1 - st) : st;  // log2 of local half size
    const int h = 1 << lh;
    const size_t Hs = (size_t)h << logS;  // global half size: stage table base
    // the four butterflies of a thread are disjoint: load all operands, then compute and store
    constexpr int BPT = NTT_ELEMS / 2 / NTT_THREADS;
    fe x0[BPT], x1[BPT];
    size_t te[BPT];
    int o0[BPT];
#pragma unroll
    for (int i = 0; i < BPT; i++) {
      // groups vary fastest across lanes: consecutive lanes take consecutive L, so the
      // twiddle loads w_(2H)^(k*S + L) are contiguous in the root table
      const int u = threadIdx.x + NTT_THREADS * i;
      const int g = u % G;
      const int w = u / G;
      const int k = w & (h - 1);
      const int t0 = ((w >> lh) << (lh + 1)) + k;
      size_t colx, q;
      locate(g, colx, q);
      const size_t L = q & (S - 1);
      te[i] = Hs + ((size_t)k << logS) + L;
      o0[i] = g * pitch + t0;
      x0[i] = buf[o0[i]];
      x1[i] = buf[o0[i] + h];
    }
#pragma unroll
    for (int i = 0; i < BPT; i++) {
      if (DIF) {
        buf[o0[i]] = fe_add(x0[i], x1[i]);
        buf[o0[i] + h] = mul_tw(fe_sub(x0[i], x1[i]), roots, te[i]);
      } else {
        const fe v = mul_tw(x1[i], roots, te[i]);
        buf[o0[i]] = fe_add(x0[i], v);
        buf[o0[i] + h] = fe_sub(x0[i], v);
      }
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < NTT_ELEMS; e += NTT_THREADS) {
    int g = gfast ? (e % G) : (e >> r);
    int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    size_t a = addr(g, t, ok);
    if (ok) data[a] = scale ? fe_mul(buf[g * pitch + t], scale[bitrev((uint32_t)(a & Nmask), logN)]) : buf[g * pitch + t];
  }
}

// DIT pass with lazily reduced 26-bit limbs (the LDE evaluation passes).  Elements enter
// LDS as five limbs (struct of arrays), every butterfly is v = REDC(x1 * wR) (normalised,
// < 2^130), y0 = x0 + v, y1 = x0 + Q - v with Q = 8p written with every limb >= 2^26, and
// only the pass output is reduced to canonical form.  Limbs grow by at most 2^27 per stage,
// so after 8 stages they stay below 2^31 and every product term stays below 2^57 (the
// REDC input bound).  ~40% fewer instructions per butterfly than the canonical form
// (no per-butterfly canonicalisation, limbwise add/sub).
constexpr uint32_t NTT_Q[5] = {67108872u, 128319487u, 134217726u, 134217726u, 134217726u};  // 8p

__device__ __forceinline__ fe ntt_canon(const uint32_t l[5]) {
  typedef unsigned __int128 u128;
  // limbs < 2^31: the low part is < 2^110, adding limb 4's low 24 bits at 2^104 may carry
  // past 2^128, and limb 4's high bits sit at 2^128 (t < 2^7)
  const u128 lo = (u128)l[0] + ((u128)l[1] << 26) + ((u128)l[2] << 52) + ((u128)l[3] << 78);
  const u128 v = lo + ((u128)(l[4] & 0xFFFFFFu) << 104);
  const uint32_t t = (l[4] >> 24) + (v < lo ? 1u : 0u);
  const u128 P = ((u128)P_HI << 64) | P_LO;
  u128 r = v + (u128)t * C_RED;  // 2^128 == C_RED
  if (r < v) r += C_RED;
  if (r >= P) r -= P;
  return fe{(uint64_t)r, (uint64_t)(r >> 64)};
}

// ELEMS elements per workgroup: NTT_ELEMS, or 2 * NTT_ELEMS for a pass whose groups would
// otherwise own only half of each 128-byte line they touch (G = ELEMS >> r < 8 consecutive L
// at a stride S >= G: the other half went to a workgroup on another XCD and the line was
// fetched twice -- the 8-stage top pass of the trace LDE fetched 7.1 GB for 3.4 GB)
template <int ELEMS, int THREADS>
__global__ __launch_bounds__(THREADS) void ntt_dit_lazy_kernel(fe* __restrict__ data, size_t ncols, int logN, int r,
                                                                  int logS, MontTab roots, const fe* __restrict__ src,
                                                                  int src_logb) {
  constexpr int PITCHED = ELEMS + ELEMS / 16;
  __shared__ uint4 bufA[PITCHED];     // limbs 0..3 (16-byte accesses, as the canonical kernel)
  __shared__ uint32_t bufB[PITCHED];  // limb 4
  const int R = 1 << r;
  const int G = ELEMS >> r;
  const size_t S = (size_t)1 << logS;
  const int log_gpc = logN - r;
  const size_t gpc = (size_t)1 << log_gpc;
  const bool gfast = S >= (size_t)G;
  const int pitch = R >= 16 ? R + 1 : R;
  size_t col_fixed = 0, qbase = 0;
  const bool whole = gpc >= (size_t)G;
  if (whole) {
    col_fixed = blockIdx.x % (unsigned)ncols;
    qbase = (size_t)(blockIdx.x / (unsigned)ncols) * G;
  }
  auto locate = [&](int g, size_t& col, size_t& q) -> bool {
    if (whole) {
      col = col_fixed;
      q = qbase + g;
      return true;
    }
    const size_t qg = (size_t)blockIdx.x * G + g;
    col = qg >> log_gpc;
    q = qg & (gpc - 1);
    return col < ncols;
  };
  auto addr = [&](int g, int t, bool& ok) -> size_t {
    size_t col, q;
    ok = locate(g, col, q);
    const size_t L = q & (S - 1), Hb = q >> logS;
    return (col << logN) + ((Hb << logS) << r) + (size_t)t * S + L;
  };
  const size_t Nmask = ((size_t)1 << logN) - 1;
  for (int e = threadIdx.x; e < ELEMS; e += THREADS) {
    const int g = gfast ? (e % G) : (e >> r);
    const int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    const size_t a = addr(g, t, ok);
    fe v = fe_zero();
    if (ok) v = src ? src[((a >> logN) << (logN - src_logb)) + ((a & Nmask) >> src_logb)] : data[a];
    uint32_t l[5];
    to26(v, l);
    bufA[g * pitch + t] = make_uint4(l[0], l[1], l[2], l[3]);
    bufB[g * pitch + t] = l[4];
  }
  __syncthreads();
  auto ld = [&](int o, uint32_t x[5]) {
    const uint4 a = bufA[o];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = bufB[o];
  };
  auto st = [&](int o, const uint32_t x[5]) {
    bufA[o] = make_uint4(x[0], x[1], x[2], x[3]);
    bufB[o] = x[4];
  };
  auto tw = [&](size_t e, uint32_t wm[5]) {
    const uint4 q4 = roots.l4[e];
    wm[0] = q4.x; wm[1] = q4.y; wm[2] = q4.z; wm[3] = q4.w; wm[4] = roots.l1[e];
  };
  // y0 = x0 + x1 w, y1 = x0 - x1 w (+Q), in place
  auto bfly = [&](uint32_t x0[5], uint32_t x1[5], const uint32_t wm[5]) {
    uint32_t v[5];
    mont_mul(x1, wm, v);
#pragma unroll
    for (int l = 0; l < 5; l++) {
      x1[l] = x0[l] + NTT_Q[l] - v[l];
      x0[l] = x0[l] + v[l];
    }
  };
  int lh = 0;
  // two stages per LDS round trip: a thread takes the quad t0, t0+h, t0+2h, t0+3h of one
  // group; stage lh pairs (0,1), (2,3) under one twiddle, stage lh+1 pairs (0,2), (1,3)
  for (; lh + 1 < r; lh += 2) {
    const int h = 1 << lh;
    constexpr int QPT = ELEMS / 4 / THREADS;
#pragma unroll
    for (int i = 0; i < QPT; i++) {
      const int u = threadIdx.x + THREADS * i;
      const int g = u % G;
      const int w = u / G;
      const int k = w & (h - 1);
      const int t0 = ((w >> lh) << (lh + 2)) + k;
      size_t colx, q;
      locate(g, colx, q);
      const size_t L = q & (S - 1);
      const int o = g * pitch + t0;
      uint32_t a0[5], a1[5], a2[5], a3[5], w1[5], w2[5], w3[5];
      ld(o, a0); ld(o + h, a1); ld(o + 2 * h, a2); ld(o + 3 * h, a3);
      tw(((size_t)h << logS) + ((size_t)k << logS) + L, w1);
      tw(((size_t)(2 * h) << logS) + ((size_t)k << logS) + L, w2);
      tw(((size_t)(2 * h) << logS) + ((size_t)(k + h) << logS) + L, w3);
      bfly(a0, a1, w1);
      bfly(a2, a3, w1);
      bfly(a0, a2, w2);
      bfly(a1, a3, w3);
      st(o, a0); st(o + h, a1); st(o + 2 * h, a2); st(o + 3 * h, a3);
    }
    __syncthreads();
  }
  if (lh < r) {  // odd stage count: one radix-2 stage
    const int h = 1 << lh;
    constexpr int BPT = ELEMS / 2 / THREADS;
#pragma unroll
    for (int i = 0; i < BPT; i++) {
      const int u = threadIdx.x + THREADS * i;
      const int g = u % G;
      const int w = u / G;
      const int k = w & (h - 1);
      const int t0 = ((w >> lh) << (lh + 1)) + k;
      size_t colx, q;
      locate(g, colx, q);
      const int o = g * pitch + t0;
      uint32_t x0[5], x1[5], wm[5];
      ld(o, x0); ld(o + h, x1);
      tw(((size_t)h << logS) + ((size_t)k << logS) + (q & (S - 1)), wm);
      bfly(x0, x1, wm);
      st(o, x0); st(o + h, x1);
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < ELEMS; e += THREADS) {
    const int g = gfast ? (e % G) : (e >> r);
    const int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    const size_t a = addr(g, t, ok);
    const uint4 a4 = bufA[g * pitch + t];
    const uint32_t l[5] = {a4.x, a4.y, a4.z, a4.w, bufB[g * pitch + t]};
    if (ok) data[a] = ntt_canon(l);
  }
}

// Natural -> bit-reversed transforms (the iNTTs and the forward DIF passes) with the DIT kernel's
// lazy limbs: Cooley-Tukey butterflies y0 = x0 + x1 w, y1 = x0 - x1 w (+Q) in decreasing-stride
// order, where the twiddle of a stage depends only on the butterfly's block: at global half size H
// (m = N / 2H blocks) block b takes w_(2m)^brv(b) (entry m + brv_(log m)(b) of the stage-major
// table), and the result equals the Gentleman-Sande DIF output exactly (round 6; the canonical DIF
// kernel reduced every sum, and its a + b chains cannot stay lazy).  Same pass split, element
// mapping, src / scale conventions and two-stages-per-LDS-round-trip quads as the kernels above.
template <int ELEMS, int THREADS>
__global__ __launch_bounds__(THREADS) void ntt_ct_lazy_kernel(fe* __restrict__ data, size_t ncols, int logN, int r,
                                                                 int logS, MontTab roots, const fe* __restrict__ src,
                                                                 int src_logb, const fe* __restrict__ scale) {
  constexpr int PITCHED = ELEMS + ELEMS / 16;
  __shared__ uint4 bufA[PITCHED];
  __shared__ uint32_t bufB[PITCHED];
  const int R = 1 << r;
  const int G = ELEMS >> r;
  const size_t S = (size_t)1 << logS;
  const int log_gpc = logN - r;
  const size_t gpc = (size_t)1 << log_gpc;
  const bool gfast = S >= (size_t)G;
  const int pitch = R >= 16 ? R + 1 : R;
  size_t col_fixed = 0, qbase = 0;
  const bool whole = gpc >= (size_t)G;
  if (whole) {
    col_fixed = blockIdx.x % (unsigned)ncols;
    qbase = (size_t)(blockIdx.x / (unsigned)ncols) * G;
  }
  auto locate = [&](int g, size_t& col, size_t& q) -> bool {
    if (whole) {
      col = col_fixed;
      q = qbase + g;
      return true;
    }
    const size_t qg = (size_t)blockIdx.x * G + g;
    col = qg >> log_gpc;
    q = qg & (gpc - 1);
    return col < ncols;
  };
  auto addr = [&](int g, int t, bool& ok) -> size_t {
    size_t col, q;
    ok = locate(g, col, q);
    const size_t L = q & (S - 1), Hb = q >> logS;
    return (col << logN) + ((Hb << logS) << r) + (size_t)t * S + L;
  };
  const size_t Nmask = ((size_t)1 << logN) - 1;
  for (int e = threadIdx.x; e < ELEMS; e += THREADS) {
    const int g = gfast ? (e % G) : (e >> r);
    const int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    const size_t a = addr(g, t, ok);
    fe v = fe_zero();
    if (ok) v = src ? src[((a >> logN) << (logN - src_logb)) + ((a & Nmask) >> src_logb)] : data[a];
    uint32_t l[5];
    to26(v, l);
    bufA[g * pitch + t] = make_uint4(l[0], l[1], l[2], l[3]);
    bufB[g * pitch + t] = l[4];
  }
  __syncthreads();
  auto ld = [&](int o, uint32_t x[5]) {
    const uint4 a = bufA[o];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = bufB[o];
  };
  auto st = [&](int o, const uint32_t x[5]) {
    bufA[o] = make_uint4(x[0], x[1], x[2], x[3]);
    bufB[o] = x[4];
  };
  // twiddle of block b at local stage lh of group q: w_(2m)^brv(b), m = N / 2H, H = 2^lh S
  auto tw = [&](int lh, size_t q, int t0, uint32_t wm[5]) {
    const int logm = logN - 1 - lh - logS;
    const size_t b = (q >> logS) * ((size_t)R >> (lh + 1)) + (size_t)(t0 >> (lh + 1));
    const size_t e = ((size_t)1 << logm) + (logm ? (size_t)(__brevll((unsigned long long)b) >> (64 - logm)) : 0);
    const uint4 q4 = roots.l4[e];
    wm[0] = q4.x; wm[1] = q4.y; wm[2] = q4.z; wm[3] = q4.w; wm[4] = roots.l1[e];
  };
  auto bfly = [&](uint32_t x0[5], uint32_t x1[5], const uint32_t wm[5]) {
    uint32_t v[5];
    mont_mul(x1, wm, v);
#pragma unroll
    for (int l = 0; l < 5; l++) {
      x1[l] = x0[l] + NTT_Q[l] - v[l];
      x0[l] = x0[l] + v[l];
    }
  };
  int lh = r - 1;
  // two stages per LDS round trip: a thread takes the quad t0, t0+hl, t0+2hl, t0+3hl (hl = 2^(lh-1));
  // stage lh pairs (0,2), (1,3) under one twiddle, stage lh-1 pairs (0,1) and (2,3)
  for (; lh >= 1; lh -= 2) {
    const int hl = 1 << (lh - 1);
    constexpr int QPT = ELEMS / 4 / THREADS;
#pragma unroll
    for (int i = 0; i < QPT; i++) {
      const int u = threadIdx.x + THREADS * i;
      const int g = u % G;
      const int w = u / G;
      const int k = w & (hl - 1);
      const int t0 = ((w >> (lh - 1)) << (lh + 1)) + k;
      size_t colx, q;
      locate(g, colx, q);
      const int o = g * pitch + t0;
      uint32_t a0[5], a1[5], a2[5], a3[5], w1[5], w2[5], w3[5];
      ld(o, a0); ld(o + hl, a1); ld(o + 2 * hl, a2); ld(o + 3 * hl, a3);
      tw(lh, q, t0, w1);
      tw(lh - 1, q, t0, w2);
      tw(lh - 1, q, t0 + 2 * hl, w3);
      bfly(a0, a2, w1);
      bfly(a1, a3, w1);
      bfly(a0, a1, w2);
      bfly(a2, a3, w3);
      st(o, a0); st(o + hl, a1); st(o + 2 * hl, a2); st(o + 3 * hl, a3);
    }
    __syncthreads();
  }
  if (lh == 0) {  // odd stage count: the last radix-2 stage
    constexpr int BPT = ELEMS / 2 / THREADS;
#pragma unroll
    for (int i = 0; i < BPT; i++) {
      const int u = threadIdx.x + THREADS * i;
      const int g = u % G;
      const int t0 = (u / G) << 1;
      size_t colx, q;
      locate(g, colx, q);
      const int o = g * pitch + t0;
      uint32_t x0[5], x1[5], wm[5];
      ld(o, x0); ld(o + 1, x1);
      tw(0, q, t0, wm);
      bfly(x0, x1, wm);
      st(o, x0); st(o + 1, x1);
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < ELEMS; e += THREADS) {
    const int g = gfast ? (e % G) : (e >> r);
    const int t = gfast ? (e / G) : (e & (R - 1));
    bool ok;
    const size_t a = addr(g, t, ok);
    const uint4 a4 = bufA[g * pitch + t];
    const uint32_t l[5] = {a4.x, a4.y, a4.z, a4.w, bufB[g * pitch + t]};
    if (ok) {
      const fe v = ntt_canon(l);
      data[a] = scale ? fe_mul(v, scale[bitrev((uint32_t)(a & Nmask), logN)]) : v;
    }
  }
}

// 8-stage DIT pass held in registers: 2048 elements (8 groups of 256 at consecutive L, whole
// 128-byte lines) on 256 threads, 8 elements per thread.  Stages 0-2 run on the elements a
// thread loads straight from HBM (t = 8j + u), stages 3-5 and 6-7 after one LDS exchange each
// (t = a + 8u + 64c, then two quads t = a' + 64u'), and the last quads go straight back to HBM:
// two LDS round trips and two barriers per pass instead of five, the twiddles of a phase
// fetched before the barrier that precedes it.  Same lazy 26-bit limb arithmetic as
// ntt_dit_lazy_kernel (limbs < 2^31 after 8 stages).  Needs S >= 8 and N >> 8 >= 8.
constexpr int NTT8_G = 8;
constexpr int NTT8_THREADS = 256;
constexpr int NTT8_PITCH = 257;
__global__ __launch_bounds__(NTT8_THREADS) __global__ __launch_bounds__(NTT8_THREADS) void ntt_dit8_kernel(fe* __restrict__ data, size_t ncols, int logN, int logS,
                                                                 MontTab roots, const fe* __restrict__ src, int src_logb,
                                                                 int lfast, int split) {
  __shared__ uint4 bufA[NTT8_G * NTT8_PITCH];
  __shared__ uint32_t bufB[NTT8_G * NTT8_PITCH];
  const int tid = (int)threadIdx.x;
  const int g = tid & (NTT8_G - 1), j = tid >> 3;
  // block -> (column, 8 consecutive groups).  lfast = 0: consecutive blocks walk the columns
  // at a fixed group range, so concurrently running blocks share twiddles in L2; lfast = 1:
  // consecutive blocks take consecutive group ranges of one column, so concurrently running
  // blocks read and write neighbouring lines of each row t (DRAM page locality)
  size_t col, q;
  if (lfast) {
    const unsigned gpb = (1u << (logN - 8)) / NTT8_G;
    col = blockIdx.x / gpb;
    q = (size_t)(blockIdx.x % gpb) * NTT8_G + g;
  } else {
    col = blockIdx.x % (unsigned)ncols;
    q = (size_t)(blockIdx.x / (unsigned)ncols) * NTT8_G + g;
  }
  const size_t S = (size_t)1 << logS;
  const size_t L = q & (S - 1), Hb = q >> logS;
  const size_t base = (col << logN) + ((Hb << logS) << 8) + L;
  auto tw = [&](size_t h, size_t k, uint32_t wm[5]) {
    const size_t e = ((h + k) << logS) + L;
    const uint4 q4 = roots.l4[e];
    wm[0] = q4.x; wm[1] = q4.y; wm[2] = q4.z; wm[3] = q4.w; wm[4] = roots.l1[e];
  };
  auto bfly = [&](uint32_t x0[5], uint32_t x1[5], const uint32_t wm[5]) {
    uint32_t v[5];
    mont_mul(x1, wm, v);
#pragma unroll
    for (int l = 0; l < 5; l++) {
      x1[l] = x0[l] + NTT_Q[l] - v[l];
      x0[l] = x0[l] + v[l];
    }
  };
  auto lds_st = [&](int t, const uint32_t x[5]) {
    bufA[g * NTT8_PITCH + t] = make_uint4(x[0], x[1], x[2], x[3]);
    bufB[g * NTT8_PITCH + t] = x[4];
  };
  auto lds_ld = [&](int t, uint32_t x[5]) {
    const uint4 a = bufA[g * NTT8_PITCH + t];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = bufB[g * NTT8_PITCH + t];
  };
  uint32_t x[8][5];
  uint32_t w[7][5];
  // ---- phase A: t = 8j + u, local half sizes 1, 2, 4 (twiddle k = u0 mod h)
  tw(1, 0, w[0]);
  tw(2, 0, w[1]); tw(2, 1, w[2]);
#pragma unroll
  for (int k = 0; k < 4; k++) tw(4, k, w[3 + k]);
  {
    const size_t Nmask = ((size_t)1 << logN) - 1;
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const size_t a = base + (size_t)(8 * j + u) * S;
      const fe v = src ? src[((a >> logN) << (logN - src_logb)) + ((a & Nmask) >> src_logb)] : data[a];
      to26(v, x[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < 8; u += 2) bfly(x[u], x[u + 1], w[0]);
#pragma unroll
  for (int u = 0; u < 8; u += 4) { bfly(x[u], x[u + 2], w[1]); bfly(x[u + 1], x[u + 3], w[2]); }
#pragma unroll
  for (int k = 0; k < 4; k++) bfly(x[k], x[k + 4], w[3 + k]);
#pragma unroll
  for (int u = 0; u < 8; u++) lds_st(8 * j + u, x[u]);
  // ---- phase B: t = a + 8u + 64c, local half sizes 8, 16, 32 (k = a + 8 (u0 mod 2^s))
  const int a = j & 7, c = j >> 3;
  tw(8, a, w[0]);
  tw(16, a, w[1]); tw(16, a + 8, w[2]);
#pragma unroll
  for (int k = 0; k < 4; k++) tw(32, a + 8 * k, w[3 + k]);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 8; u++) lds_ld(a + 8 * u + 64 * c, x[u]);
#pragma unroll
  for (int u = 0; u < 8; u += 2) bfly(x[u], x[u + 1], w[0]);
#pragma unroll
  for (int u = 0; u < 8; u += 4) { bfly(x[u], x[u + 2], w[1]); bfly(x[u + 1], x[u + 3], w[2]); }
#pragma unroll
  for (int k = 0; k < 4; k++) bfly(x[k], x[k + 4], w[3 + k]);
  // in place: the thread's phase-B locations are its own (a partition), no barrier needed
#pragma unroll
  for (int u = 0; u < 8; u++) lds_st(a + 8 * u + 64 * c, x[u]);
  // ---- phase C: two quads t = a' + 64u' (a' = j, j + 32), local half sizes 64, 128
  tw(64, j, w[0]); tw(128, j, w[1]); tw(128, j + 64, w[2]);
  tw(64, j + 32, w[3]); tw(128, j + 32, w[4]); tw(128, j + 96, w[5]);
  __syncthreads();
#pragma unroll
  for (int qd = 0; qd < 2; qd++) {
    const int a2 = j + 32 * qd;
#pragma unroll
    for (int u = 0; u < 4; u++) lds_ld(a2 + 64 * u, x[4 * qd + u]);
    uint32_t* y0 = x[4 * qd];
    uint32_t* y1 = x[4 * qd + 1];
    uint32_t* y2 = x[4 * qd + 2];
    uint32_t* y3 = x[4 * qd + 3];
    bfly(y0, y1, w[3 * qd]);
    bfly(y2, y3, w[3 * qd]);
    bfly(y0, y2, w[3 * qd + 1]);
    bfly(y1, y3, w[3 * qd + 2]);
    // split (last pass only, S = N / 256, so L & 7 = g): row L + t S with t = a2 + 64 u goes to
    // lde_pos = (L - g) + g / 2 + 4 (t & 1) + (t / 2 + 128 (g & 1)) S, i.e. 32 S apart in u
    const size_t at0 = split ? (col << logN) + (L - g) + (g >> 1) + 4 * (a2 & 1) +
                                   ((size_t)((a2 >> 1) + ((g & 1) << 7)) << logS)
                             : base + (size_t)a2 * S;
    const size_t du = split ? 32 * S : 64 * S;
#pragma unroll
    for (int u = 0; u < 4; u++) data[at0 + u * du] = ntt_canon(x[4 * qd + u]);
  }
}

// DIT form: lazy limbs (default) or the canonical kernel (ZKL_NTT=classic, set_ntt_lazy)
static std::atomic<int> g_ntt_lazy{-1};
static bool ntt_lazy_enabled() {
  int v = g_ntt_lazy.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("ZKL_NTT");
    v = (e && !strcmp(e, "classic")) ? 0 : 1;
    g_ntt_lazy.store(v);
  }
  return v != 0;
}
void set_ntt_lazy(bool on) { g_ntt_lazy.store(on ? 1 : 0); }
// measured (profiles/r02, scripts/ab_ntt_wide.sh): the 2048-element / 256-thread form halves
// the top pass's fetch (7.1 -> 3.7 GB) but its passes run no faster (fewer waves per CU hide
// less of the butterfly chains); 2048 elements on 512 threads keeps the waves and gives NTT
// 8.3 -> 8.0 ms per proof: default 2
static int ntt_wide_mode() {
  static const int m = [] {
    const char* e = getenv("ZKL_NTT_WIDE");
    return e ? atoi(e) : 2;
  }();
  return m;
}

// 8-stage register pass (ntt_dit8_kernel) for the lazy DIT passes it covers; ZKL_NTT8=0 keeps
// the LDS-staged kernels (A/B)
static bool ntt8_enabled() {
  static const bool on = [] {
    const char* e = getenv("ZKL_NTT8");
    return !(e && !strcmp(e, "0"));
  }();
  return on;
}

// block order of ntt_dit8_kernel (ZKL_NTT8_MAP): 0 = columns fastest, 1 = group ranges
// fastest, 2 = group ranges fastest for the passes over strides S >= 2048 only
static int ntt8_lfast(int logS) {
  static const int m = [] {
    const char* e = getenv("ZKL_NTT8_MAP");
    return e ? atoi(e) : 0;
  }();
  return m == 1 || (m == 2 && logS >= 11) ? 1 : 0;
}

// natural -> bit-reversed passes in the lazy Cooley-Tukey form (default) or the canonical DIF
// kernel (ZKL_NTT_CT=0, A/B); both give the same output
static bool ntt_ct_enabled() {
  static const bool on = [] {
    const char* e = getenv("ZKL_NTT_CT");
    return !(e && !strcmp(e, "0"));
  }();
  return on;
}

static int ilog2s(size_t n) { int k = 0; while (((size_t)1 << k) < n) k++; return k; }

// Stage split of one transform into LDS passes.  The pass over the largest stride S (the
// last DIT pass, the first DIF pass) takes at most NTT_TOP_R stages, so a workgroup owns
// G = 1024 >> r >= 8 consecutive L, i.e. whole 128-byte lines of every row it touches (with
// 4 consecutive L a line was split between two workgroups on different XCDs and fetched
// twice); the other passes take up to 10 stages (the lazy kernel's limbs stay below 2^31 for
// 10 stages: 2^26 + 10 * 2^27), split as evenly as possible.  NTT_SPLIT_MODE 0 restores the
// greedy 8-stage split.
#ifndef NTT_TOP_R
#define NTT_TOP_R 6
#endif
#ifndef NTT_SPLIT_MODE
#define NTT_SPLIT_MODE 0  // measured: 8 + 8 = 8.25 ms, 9 + 7 = 8.75 ms, 10 + 6 = 9.8 ms per proof (r02)
#endif
static std::vector<int> ntt_split(int K) {
  std::vector<int> rs;
  if (K <= 0) return rs;
  if (NTT_SPLIT_MODE == 0) {
    for (int left = K; left > 0; left -= std::min(8, left)) rs.push_back(std::min(8, left));
    return rs;  // greedy from the smallest stride
  }
  if (K <= 10) { rs.push_back(K); return rs; }
  int rest = K - NTT_TOP_R;
  const int np = (rest + 9) / 10;
  for (int i = 0; i < np; i++) {
    int r = (rest + (np - i) - 1) / (np - i);
    if ((r & 1) && r < rest && r < 10) r++;  // even stage counts: radix-4 LDS round trips only
    rs.push_back(r);
    rest -= r;
  }
  rs.push_back(NTT_TOP_R);  // ascending-S order (DIT); DIF walks it backwards
  return rs;
}

// DIT passes over stages [lo, hi]: can the last one store the split layout (it must be the
// 8-stage register pass, whose store is the only one that knows the layout)?
static bool dit_split_ok(size_t N, int lo, int hi) {
  if (hi < lo || !ntt_lazy_enabled() || !ntt8_enabled()) return false;
  const std::vector<int> rs = ntt_split(hi - lo + 1);
  int cur = lo;
  for (size_t k = 0; k + 1 < rs.size(); k++) cur += rs[k];
  return rs.back() == 8 && ((size_t)1 << cur) >= (size_t)NTT8_G && (N >> 8) >= (size_t)NTT8_G;
}

// DIF: src (out of place) feeds the first pass, scale the last pass's stores (see ntt_pass_kernel)
static void ntt_passes(fe* d, size_t ncols, size_t N, bool dif, int lo, int hi, MontTab roots, size_t Ntab,
                       const fe* src, int src_logb, hipStream_t s, int split = 0, const fe* scale = nullptr) {
  int logN = ilog2s(N), logTab = ilog2s(Ntab);
  if (hi < lo) return;
  const std::vector<int> rs = ntt_split(hi - lo + 1);
  if (dif) {
    int cur = hi;
    for (size_t k = rs.size(); k-- > 0;) {
      const int r = rs[k];
      int logS = cur - r + 1;
      size_t groups = (N >> r) * ncols;
      size_t G = NTT_ELEMS >> r;
      const fe* sp = k + 1 == rs.size() ? src : nullptr;
      const fe* sc = k == 0 ? scale : nullptr;
      if (ntt_lazy_enabled() && ntt_ct_enabled()) {
        // lazy Cooley-Tukey passes (ntt_ct_lazy_kernel); half-line groups take the wide form
        const int wm = ntt_wide_mode();
        const bool wide = wm > 0 && G < 8 && ((size_t)1 << logS) >= G;
        const size_t Gw = wide ? 2 * G : G;
        const unsigned grid = (unsigned)((groups + Gw - 1) / Gw);
        if (wide && wm == 2)
          ntt_ct_lazy_kernel<2 * NTT_ELEMS, 2 * NTT_THREADS><<<grid, 2 * NTT_THREADS, 0, s>>>(d, ncols, logN, r, logS, roots, sp, 0, sc);
        else if (wide)
          ntt_ct_lazy_kernel<2 * NTT_ELEMS, NTT_THREADS><<<grid, NTT_THREADS, 0, s>>>(d, ncols, logN, r, logS, roots, sp, 0, sc);
        else
          ntt_ct_lazy_kernel<NTT_ELEMS, NTT_THREADS><<<grid, NTT_THREADS, 0, s>>>(d, ncols, logN, r, logS, roots, sp, 0, sc);
      } else {
        ntt_pass_kernel<true><<<(unsigned)((groups + G - 1) / G), NTT_THREADS, 0, s>>>(d, ncols, logN, r, logS, roots,
                                                                                      logTab, sp, 0, sc);
      }
      cur -= r;
    }
  } else {
    int cur = lo;
    for (size_t ri = 0; ri < rs.size(); ri++) {
      const int r = rs[ri];
      const int split_here = split && ri + 1 == rs.size();
      size_t groups = (N >> r) * ncols;
      size_t G = NTT_ELEMS >> r;
      if (ntt_lazy_enabled()) {
        // wide mode (ZKL_NTT_WIDE): 1 = 2048 elements / 256 threads, 2 = 2048 / 512 for the
        // passes whose 1024-element groups own only half lines (see ntt_dit_lazy_kernel)
        const int wm = ntt_wide_mode();
        const bool wide = wm > 0 && G < 8 && ((size_t)1 << cur) >= G;
        const size_t Gw = wide ? 2 * G : G;
        const unsigned grid = (unsigned)((groups + Gw - 1) / Gw);
        const fe* sp = cur == lo ? src : nullptr;
        if (r == 8 && ntt8_enabled() && ((size_t)1 << cur) >= (size_t)NTT8_G && (N >> 8) >= (size_t)NTT8_G)
          ntt_dit8_kernel<<<(unsigned)(groups / NTT8_G), NTT8_THREADS, 0, s>>>(d, ncols, logN, cur, roots, sp, src_logb,
                                                                              ntt8_lfast(cur), split_here);
        else if (wide && wm == 2)
          ntt_dit_lazy_kernel<2 * NTT_ELEMS, 2 * NTT_THREADS><<<grid, 2 * NTT_THREADS, 0, s>>>(d, ncols, logN, r, cur, roots, sp, src_logb);
        else if (wide)
          ntt_dit_lazy_kernel<2 * NTT_ELEMS, NTT_THREADS><<<grid, NTT_THREADS, 0, s>>>(d, ncols, logN, r, cur, roots, sp, src_logb);
        else
          ntt_dit_lazy_kernel<NTT_ELEMS, NTT_THREADS><<<grid, NTT_THREADS, 0, s>>>(d, ncols, logN, r, cur, roots, sp, src_logb);
      } else
        ntt_pass_kernel<false><<<(unsigned)((groups + G - 1) / G), NTT_THREADS, 0, s>>>(
            d, ncols, logN, r, cur, roots, logTab, cur == lo ? src : nullptr, src_logb);
      cur += r;
    }
  }
}

void launch_ntt_stages(fe* d, size_t ncols, size_t N, bool dif, int lo, int hi, MontTab roots, size_t Ntab,
                       hipStream_t s) {
  ntt_passes(d, ncols, N, dif, lo, hi, roots, Ntab, nullptr, 0, s);
}

void launch_intt_scaled(const fe* src, fe* d, size_t ncols, size_t n, MontTab iroots, size_t Ntab, const fe* scale,
                        hipStream_t s) {
  const int logn = ilog2s(n);
  if (logn == 0) throw std::invalid_argument("launch_intt_scaled: n must be at least 2");
  ntt_passes(d, ncols, n, true, 0, logn - 1, iroots, Ntab, src, 0, s, 0, scale);
}

int launch_lde_from_coeffs(const fe* d_coef, size_t ncols, size_t n, size_t N, MontTab roots, size_t Ntab, fe* d_out,
                           hipStream_t s, bool want_split) {
  const int logB = ilog2s(N / n);
  if (logB == 0) {
    ZKL_HIPCHECK(hipMemcpyAsync(d_out, d_coef, ncols * n * sizeof(fe), hipMemcpyDeviceToDevice, s));
    ntt_passes(d_out, ncols, N, false, 0, ilog2s(N) - 1, roots, Ntab, nullptr, 0, s);
    return 0;
  }
  const int split = want_split && dit_split_ok(N, logB, ilog2s(N) - 1) ? 1 : 0;
  ntt_passes(d_out, ncols, N, false, logB, ilog2s(N) - 1, roots, Ntab, d_coef, logB, s, split);
  return split;
}

__global__ void broadcast_kernel(const fe* __restrict__ in, size_t in_col_stride, size_t in_elem_stride,
                                 size_t in_offset, size_t ncols, size_t n, int logn, int logB, const fe* __restrict__ scale,
                                 fe mult, bool reverse, fe* __restrict__ out) {
  size_t N = n << logB;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * ncols) return;
  size_t col = i / N, pos = i % N;
  size_t j = pos >> logB;
  size_t src = reverse ? (n - 1 - j) : j;
  fe v = in[col * in_col_stride + in_offset + src * in_elem_stride];
  if (scale) v = fe_mul(v, scale[bitrev((uint32_t)j, logn)]);
  if (!(mult.lo == 1 && mult.hi == 0)) v = fe_mul(v, mult);
  out[i] = v;
}

void launch_broadcast(const fe* d_in, size_t in_col_stride, size_t in_elem_stride, size_t in_offset, size_t ncols,
                      size_t n, size_t N, const fe* d_scale, fe mult, bool reverse, fe* d_out, hipStream_t s) {
  size_t tot = N * ncols;
  broadcast_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(d_in, in_col_stride, in_elem_stride, in_offset, ncols,
                                                                 n, ilog2s(n), ilog2s(N / n), d_scale, mult, reverse, d_out);
}

__global__ void scale_bitrev_kernel(fe* d, size_t ncols, size_t n, int logn, const fe* scale) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * ncols) return;
  d[i] = fe_mul(d[i], scale[bitrev((uint32_t)(i % n), logn)]);
}
void launch_scale_bitrev(fe* d, size_t ncols, size_t n, const fe* scale, hipStream_t s) {
  scale_bitrev_kernel<<<(unsigned)((n * ncols + 255) / 256), 256, 0, s>>>(d, ncols, n, ilog2s(n), scale);
}


// =====================================================================================
// Constraint evaluation over the CE coset (DefaultConstraintEvaluator restated):
//   C(x) = [sum_j alpha_j c_j(x) * (x - g^(n-1)) + sum_c P_c(x) M_c(x) - W(x)] / (x^n - 1)
// c_j = ZkLispAir::evaluate_transition (vm/air/mod.rs:324-378) in evaluation order.
// =====================================================================================

// POSE: the PoseidonAir block, RM: the RamAir / MerkleAir blocks; each is compiled into a
// separate instance so that VM-only segments keep the smaller register footprint
// CE_WAVES_CFG: occupancy target (waves per SIMD; 0 lets the compiler choose: 214 VGPRs, 2 waves
// per SIMD for the VM-only instance).  The evaluator is latency-bound (dependent f128 products,
// gathers of 2 x 204 columns): 3 waves per SIMD took it from 1.57 to 1.40 ms per proof and 4 to
// 1.39 (round 3, profiles/r03/ab_ce); 3 keeps the larger Poseidon / RAM instances from spilling
// much.
#ifndef CE_WAVES_CFG
#define CE_WAVES_CFG 3
#endif
#if CE_WAVES_CFG
#define CE_OCC __attribute__((amdgpu_waves_per_eu(CE_WAVES_CFG, CE_WAVES_CFG)))
#else
#define CE_OCC
#endif
// PART 0: the whole transition sum; PART 2: all but the PoseidonAir block, whose sum pose_part[i]
// (constraint_eval_pose_part_kernel) is added; PART 1: that block alone, written to out[i]
template <bool POSE, bool RM, int PART = 0>
__device__ __forceinline__ void constraint_eval_body(const fe* __restrict__ lde, const fe* __restrict__ roots,
                                                     int roots_shift, const fe* __restrict__ pertab,
                                                     const fe* __restrict__ bm, const ProofConsts* __restrict__ K,
                                                     const DerivedConsts* __restrict__ D, const fe* __restrict__ xinv,
                                                     fe* __restrict__ out, int split,
                                                     const fe* __restrict__ pose_part = nullptr) {
  const AirDevice& c_air = K->air;
  const CeParams& c_ce = K->ce;
  const size_t ce = c_ce.ce, N = c_ce.N;
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ce) return;
  // split layout with N / ce <= 2 (the CE rows are the even rows, or all rows): thread k reads
  // position k, i.e. whole lines of the first half of each column, and evaluates the CE point
  // of the row stored there; a wave's CE indices form two runs of 32.  Otherwise thread k
  // evaluates CE point k.
  const bool by_pos = split && N <= 2 * ce;
  const size_t i = by_pos ? lde_row(k, N, 1) / (N / ce) : k;
  const size_t r0 = by_pos ? k : lde_pos(i * (N / ce), N, split);
  const size_t r1 = lde_pos((i * (N / ce) + c_ce.blowup) & (N - 1), N, split);
  auto cur = [&](int c) { return lde[(size_t)c * N + r0]; };
  // next rows: position k + blowup for all but the rows whose L wraps; in the split layout
  // they share the lines this wave's current rows just brought in (PMC: taking them from the
  // neighbouring lane with ds_bpermute instead fetched the same bytes, round 3)
  auto nxt = [&](int c) { return lde[(size_t)c * N + r1]; };
  fe x = fe_mul(fe{3, 0}, roots[i << roots_shift]);
  const size_t per_period = ce / (c_ce.n / 32);
  const fe* per = pertab + (i % per_period) * 31;
  if (PART == 1) {
    out[i] = air_transition_sum<POSE, RM, 1>(c_air, cur, nxt, per, fe_zero(), K->alpha, D->pose_k, D->apre);
    return;
  }
  const size_t blow = ce / c_ce.n;
  const fe xn_inv = c_ce.xn_inv[i % blow];
  // p_last = L_{n-1}(x) = g^(n-1)/n * (x^n - 1) / (x - g^(n-1))
  fe x_gl = fe_sub_sel(x, c_ce.gl);
  fe xn_m1 = c_ce.xn_m1[i % blow];
  fe p_last = fe_mul(fe_mul(c_ce.lagr, xn_m1), xinv[i]);  // xinv[i] = 1 / (x - g^(n-1))
  fe tsum = air_transition_sum<POSE, RM, PART>(c_air, cur, nxt, per, p_last, K->alpha, D->pose_k, D->apre);
  if (PART == 2) tsum = fe_add(tsum, pose_part[i]);
  // boundary: sum_c P_c(x) M_c(x) - W(x)
  uint32_t bacc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t nb = c_ce.n_bcols;
  for (uint32_t u = 0; u < nb; u++) mul_acc(cur((int)c_ce.bcol[u]), bm[(size_t)u * ce + i], bacc);
  fe bsum2 = fe_sub_sel(reduce288(bacc), bm[(size_t)nb * ce + i]);
  fe v = fe_add_sel(fe_mul(tsum, x_gl), bsum2);
  out[i] = fe_mul(v, xn_inv);
}

// The VM-only and RAM / Merkle instances run at CE_WAVES_CFG waves per SIMD; the PoseidonAir
// block's own kernel at CE_POSE_WAVES_CFG (3: 48 spilled VGPRs, 3.33 against 3.42 ms of
// evaluation per rollup-bench proof at the compiler's 2, profiles/r04/ab_cepose.json).  The
// evaluator kernels are the library's only ones with a private segment (spills at 3 waves per
// SIMD, a stack object in the Poseidon block at any occupancy): the listed exceptions of
// tests/test_abi.py::test_only_listed_kernels_need_scratch.
#ifndef CE_POSE_WAVES_CFG
#define CE_POSE_WAVES_CFG 3
#endif
#if CE_POSE_WAVES_CFG
#define CE_POSE_OCC __attribute__((amdgpu_waves_per_eu(CE_POSE_WAVES_CFG, CE_POSE_WAVES_CFG)))
#else
#define CE_POSE_OCC
#endif
template <bool RM>
__global__ __launch_bounds__(256) CE_OCC void constraint_eval_kernel(const fe* __restrict__ lde, const fe* __restrict__ roots,
                                                                    int roots_shift, const fe* __restrict__ pertab,
                                                                    const fe* __restrict__ bm,
                                                                    const ProofConsts* __restrict__ K,
                                                                    const DerivedConsts* __restrict__ D,
                                                                    const fe* __restrict__ xinv, fe* __restrict__ out,
                                                                    int split) {
  constraint_eval_body<false, RM>(lde, roots, roots_shift, pertab, bm, K, D, xinv, out, split);
}
// Poseidon layouts in two kernels: the PoseidonAir block's alpha-weighted sum per CE point
// (pose_part), then every other block plus that sum, at the VM-only kernel's occupancy.  One
// kernel for both needed 256+ VGPRs (1 wave per SIMD).
__global__ __launch_bounds__(256) CE_POSE_OCC void constraint_eval_pose_part_kernel(
    const fe* __restrict__ lde, const fe* __restrict__ roots, int roots_shift, const fe* __restrict__ pertab,
    const fe* __restrict__ bm, const ProofConsts* __restrict__ K, const DerivedConsts* __restrict__ D,
    const fe* __restrict__ xinv, fe* __restrict__ pose_part, int split) {
  constraint_eval_body<true, false, 1>(lde, roots, roots_shift, pertab, bm, K, D, xinv, pose_part, split);
}
template <bool RM>
__global__ __launch_bounds__(256) CE_OCC void constraint_eval_pose_kernel(const fe* __restrict__ lde, const fe* __restrict__ roots,
                                                                  int roots_shift, const fe* __restrict__ pertab,
                                                                  const fe* __restrict__ bm,
                                                                  const ProofConsts* __restrict__ K,
                                                                  const DerivedConsts* __restrict__ D,
                                                                  const fe* __restrict__ xinv, fe* __restrict__ out,
                                                                  int split, const fe* __restrict__ pose_part) {
  constraint_eval_body<true, RM, 2>(lde, roots, roots_shift, pertab, bm, K, D, xinv, out, split, pose_part);
}

// out[i] = 1 / ((x_i - a1) (x_i - a2)^two) over the coset x_i = 3 w_M^i (w_M^i =
// roots[i << shift]): each thread inverts INV_PTS points T apart with one field inversion
// (Montgomery's trick), instead of one ~250-multiplication Fermat inversion per point.  The
// prefix products are not kept in a private array (with the denominators, both live across the
// inversion, the compiler placed them in scratch: 528 B per lane); they go to the output slots (each slot k > 0 holds prefix k-1 until it is overwritten
// with its inverse on the way back): 32 extra bytes per point of HBM traffic, no private array.
constexpr int INV_PTS = 16;
__device__ inline fe coset_den(const fe* __restrict__ roots, size_t i, int shift, fe a1, fe a2, int two) {
  const fe x = fe_mul(fe{3, 0}, roots[i << shift]);
  fe d = fe_sub(x, a1);
  if (two) d = fe_mul(d, fe_sub(x, a2));
  return d;
}
__global__ __launch_bounds__(256) void coset_inv_kernel(const fe* __restrict__ roots, int shift, fe a1, fe a2, int two,
                                                        fe* __restrict__ out) {
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  fe pre = coset_den(roots, i0, shift, a1, a2, two);
  for (int k = 1; k < INV_PTS; k++) {
    out[i0 + k * T] = pre;  // prefix k-1
    pre = fe_mul(pre, coset_den(roots, i0 + k * T, shift, a1, a2, two));
  }
  fe inv = fe_inv(pre);
  for (int k = INV_PTS - 1; k > 0; k--) {
    const fe p = out[i0 + k * T];
    out[i0 + k * T] = fe_mul(inv, p);
    inv = fe_mul(inv, coset_den(roots, i0 + k * T, shift, a1, a2, two));
  }
  out[i0] = inv;
}
static void launch_coset_inv(const fe* d_roots, int shift, size_t M, fe a1, fe a2, int two, fe* d_out, hipStream_t s) {
  // M is a power of two >= INV_PTS
  const size_t threads = std::min<size_t>(256, M / INV_PTS);
  coset_inv_kernel<<<(unsigned)(M / (threads * INV_PTS)), (unsigned)threads, 0, s>>>(d_roots, shift, a1, a2, two, d_out);
}

void launch_constraint_eval(const fe* d_lde, const fe* d_roots, size_t Ntab, const fe* d_pertab, const fe* d_bm,
                            const CeParams& p, ProofConsts* dK, const DerivedConsts* dD, bool pose_block,
                            bool ram_merkle, fe* d_xinv,
                            bool xinv_ready, fe* d_out, hipStream_t s, int split, fe* d_pose_part) {
  ZKL_HIPCHECK(hipMemcpyAsync(&dK->ce, &p, sizeof p, hipMemcpyHostToDevice, s));
  int shift = ilog2s(Ntab) - ilog2s(p.ce);
  // 1 / (x - g^(n-1)) over the CE coset depends on the shape only: the caller keeps it per context
  if (!xinv_ready) launch_coset_inv(d_roots, shift, p.ce, p.gl, fe_zero(), 0, d_xinv, s);
  const unsigned grid = (unsigned)((p.ce + 255) / 256);
  if (pose_block) {
    if (!d_pose_part) throw std::invalid_argument("constraint evaluation: Poseidon layout needs the pose_part buffer");
    constraint_eval_pose_part_kernel<<<grid, 256, 0, s>>>(d_lde, d_roots, shift, d_pertab, d_bm, dK, dD, d_xinv,
                                                           d_pose_part, split);
  }
  if (pose_block && ram_merkle)
    constraint_eval_pose_kernel<true><<<grid, 256, 0, s>>>(d_lde, d_roots, shift, d_pertab, d_bm, dK, dD, d_xinv, d_out,
                                                           split, d_pose_part);
  else if (pose_block)
    constraint_eval_pose_kernel<false><<<grid, 256, 0, s>>>(d_lde, d_roots, shift, d_pertab, d_bm, dK, dD, d_xinv, d_out,
                                                            split, d_pose_part);
  else if (ram_merkle)
    constraint_eval_kernel<true><<<grid, 256, 0, s>>>(d_lde, d_roots, shift, d_pertab, d_bm, dK, dD, d_xinv, d_out, split);
  else
    constraint_eval_kernel<false><<<grid, 256, 0, s>>>(d_lde, d_roots, shift, d_pertab, d_bm, dK, dD, d_xinv, d_out, split);
}

__global__ void boundary_scatter_kernel(const uint32_t* slot, const uint32_t* step, const fe* beta, size_t na, size_t n,
                                        fe* vecs) {
  size_t a = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= na) return;
  vecs[(size_t)slot[a] * n + step[a]] = beta[a];
}
void launch_boundary_scatter(const uint32_t* d_slot, const uint32_t* d_step, const fe* d_beta, size_t na, size_t n,
                             fe* d_vecs, hipStream_t s) {
  boundary_scatter_kernel<<<(unsigned)((na + 255) / 256), 256, 0, s>>>(d_slot, d_step, d_beta, na, n, d_vecs);
}
__global__ void boundary_w_kernel(const uint32_t* rs, const fe* beta, const fe* val, size_t n, fe* w) {
  size_t row = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t a = rs[row]; a < rs[row + 1]; a++) mul_acc(beta[a], val[a], acc);
  w[row] = reduce288(acc);
}
void launch_boundary_w(const uint32_t* d_rs, const fe* d_beta, const fe* d_val, size_t n, fe* d_w, hipStream_t s) {
  boundary_w_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(d_rs, d_beta, d_val, n, d_w);
}

__global__ void check_zero_kernel(const fe* d, size_t N, int logN, size_t lo, size_t hi, unsigned* flag) {
  size_t k = lo + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= hi) return;
  fe v = d[bitrev((uint32_t)k, logN)];
  if (!fe_is_zero(v)) atomicOr(flag, 1u);
}
void launch_check_zero_range_bitrev(const fe* d, size_t N, size_t lo, size_t hi, unsigned* flag, hipStream_t s) {
  if (hi > lo) check_zero_kernel<<<(unsigned)((hi - lo + 255) / 256), 256, 0, s>>>(d, N, ilog2s(N), lo, hi, flag);
}

// =====================================================================================
// OOD (TracePolyTable::get_ood_frame / CompositionPoly ood): dot products with powers
// =====================================================================================
// partial[(pt * ncols + c) * chunks + k] = sum over chunk k of coef(c, j) * pw_pt[j] for both
// points pt = 0 (z) and 1 (z g); the host adds the chunk partials (the OOD frame is read back
// anyway).  Each coefficient is read once for both dot products (round 6: one launch dimension
// per point read every coefficient twice, 445 MB per launch for 214 MB of coefficients).
__global__ __launch_bounds__(256) void ood_kernel(OodArgs A, fe* partial) {
  const uint32_t c = blockIdx.x, k = blockIdx.z;
  const fe* col = A.coef + (A.use_off ? (size_t)A.off[c] : (size_t)c * A.col_stride);
  const size_t len = A.n / A.chunks, j0 = (size_t)k * len;
  uint32_t acc1[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, acc2[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (size_t j = j0 + threadIdx.x; j < j0 + len; j += 256) {
    const fe v = col[j * A.elem_stride];
    mul_acc(v, A.pw1[j], acc1);
    mul_acc(v, A.pw2[j], acc2);
  }
  __shared__ fe red[2][256];
  red[0][threadIdx.x] = reduce288(acc1);
  red[1][threadIdx.x] = reduce288(acc2);
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] = fe_add(red[0][threadIdx.x], red[0][threadIdx.x + w]);
      red[1][threadIdx.x] = fe_add(red[1][threadIdx.x], red[1][threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 2) partial[((size_t)threadIdx.x * A.ncols + c) * A.chunks + k] = red[threadIdx.x][0];
}
void launch_ood(const OodArgs& A, fe* d_partial, hipStream_t s) {
  ood_kernel<<<dim3(A.ncols, 1, A.chunks), 256, 0, s>>>(A, d_partial);
}

// DEEP composition over the LDE domain (agg/trace.rs:1126-1218 restates the formula):
// sum_i g_i [(T_i(x)-T_i(z))/(x-z) + (T_i(x)-T_i(zg))/(x-zg)] + same for H_j
//   = [(S(x) - S(z)) (x - zg) + (S(x) - S(zg)) (x - z)] / ((x - z)(x - zg)),  S = sum_i g_i T_i.
// S(x) is one lazily reduced dot product per point: the coefficients as Montgomery limbs
// (g R, uniform -> SGPR operands), each column value split into 26-bit limbs, 25
// v_mad_u64_u32 per column into 64-bit columns (up to 256 terms of < 2^54 stay below the 2^62
// the REDC needs; upload_deep_coeffs enforces it, W + C <= 226 here) and a
// single REDC.  Each thread takes DEEP_PTS points T apart (coalesced), keeps
// DEEP_COLS x DEEP_PTS loads in flight, and shares one inversion among its points.
// points per thread: 2 keeps the kernel at 96 VGPRs (5 waves per SIMD, more loads in flight;
// 4 points needed 180 VGPRs, 2 waves): DEEP 0.91 -> 0.85 ms (profiles/r02/ab_deep)
#ifndef DEEP_PTS_CFG
#define DEEP_PTS_CFG 2
#endif
#ifndef DEEP_COLS_CFG
#define DEEP_COLS_CFG 4
#endif
constexpr int DEEP_PTS = DEEP_PTS_CFG, DEEP_COLS = DEEP_COLS_CFG;

// canonical element of the REDC output limbs (normalised, value < 2^130)
__device__ __forceinline__ fe limbs_canon(const uint32_t l[5]) {
  typedef unsigned __int128 u128;
  const u128 v = (u128)l[0] | ((u128)l[1] << 26) | ((u128)l[2] << 52) | ((u128)l[3] << 78) | ((u128)(l[4] & 0xFFFFFFu) << 104);
  const u128 P = ((u128)P_HI << 64) | P_LO;
  u128 r = v + (u128)(l[4] >> 24) * C_RED;  // bits >= 128: 2^128 == C_RED
  if (r < v) r += C_RED;
  if (r >= P) r -= P;
  return fe{(uint64_t)r, (uint64_t)(r >> 64)};
}

__global__ __launch_bounds__(256) void deep_kernel(const fe* __restrict__ lde, const fe* __restrict__ clde,
                                                   const fe* __restrict__ roots, int shift, DeepParams p,
                                                   const DerivedConsts* __restrict__ K, const fe* __restrict__ dinv,
                                                   fe* out, int split) {
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t col[DEEP_PTS][10];
#pragma unroll
  for (int k = 0; k < DEEP_PTS; k++)
#pragma unroll
    for (int u = 0; u < 10; u++) col[k][u] = 0;
  const uint32_t ncol = p.W + p.C;
  for (uint32_t c0 = 0; c0 < ncol; c0 += DEEP_COLS) {
    fe v[DEEP_COLS][DEEP_PTS];
#pragma unroll
    for (int cc = 0; cc < DEEP_COLS; cc++) {
      const uint32_t c = c0 + cc;
      // thread point k is LDE position q = i0 + k T (whole lines of the trace columns, which may
      // be in the split layout), i.e. row lde_row(q); composition columns are in natural order
      const bool tr = c < p.W;
      const fe* src = tr ? lde + (size_t)c * p.N : clde + (size_t)(c - p.W) * p.N;
#pragma unroll
      for (int k = 0; k < DEEP_PTS; k++)
        v[cc][k] = c < ncol ? src[tr ? i0 + k * T : lde_row(i0 + k * T, p.N, split)] : fe_zero();
    }
#pragma unroll
    for (int cc = 0; cc < DEEP_COLS; cc++) {
      const uint32_t c = min(c0 + cc, ncol - 1);  // a padded column contributes g * 0
      const uint32_t* g = K->deep_m[c];
      const uint32_t gm[5] = {g[0], g[1], g[2], g[3], g[4]};
#pragma unroll
      for (int k = 0; k < DEEP_PTS; k++) {
        uint32_t l[5];
        to26(v[cc][k], l);
        mac5(l, gm, col[k]);
      }
    }
  }
  // 1 / ((x - z)(x - zg)) comes from coset_inv_kernel (x is never z or zg: z is drawn
  // outside the LDE domain, as Winterfell requires)
#pragma unroll
  for (int k = 0; k < DEEP_PTS; k++) {
    uint32_t l[5];
    redc(col[k], l);
    const fe sv = limbs_canon(l);
    const size_t i = lde_row(i0 + k * T, p.N, split);
    const fe x = fe_mul(fe{3, 0}, roots[i << shift]);
    const fe d1 = fe_sub(x, p.z), d2 = fe_sub(x, p.zg);
    const fe num = fe_add(fe_mul(fe_sub(sv, K->deep_sz[0]), d2), fe_mul(fe_sub(sv, K->deep_sz[1]), d1));
    out[i] = fe_mul(num, dinv[i]);
  }
}
// One block: thread i < W + C stores coefficient i and its Montgomery limbs; both frame dot
// products are summed by a tree reduction in LDS.
__global__ __launch_bounds__(256) void deep_coeffs_kernel(const fe* __restrict__ gam, uint32_t W, uint32_t C,
                                                          const fe* __restrict__ frame, fe R156, DerivedConsts* K) {
  __shared__ fe red[2][256];
  const uint32_t i = threadIdx.x, n = W + C;
  fe a = fe_zero(), b = fe_zero();
  if (i < n) {
    const fe g = gam[i];
    K->deep[i] = g;
    uint32_t l[5];
    to26(fe_mul(g, R156), l);
#pragma unroll
    for (int t = 0; t < 5; t++) K->deep_m[i][t] = l[t];
    a = fe_mul(g, frame[i]);
    b = fe_mul(g, frame[n + i]);
  }
  red[0][i] = a;
  red[1][i] = b;
  __syncthreads();
  for (uint32_t h = 128; h > 0; h >>= 1) {
    if (i < h) {
      red[0][i] = fe_add(red[0][i], red[0][i + h]);
      red[1][i] = fe_add(red[1][i], red[1][i + h]);
    }
    __syncthreads();
  }
  if (i == 0) {
    K->deep_sz[0] = red[0][0];
    K->deep_sz[1] = red[1][0];
  }
}
void launch_deep_coeffs(const fe* d_gam, uint32_t W, uint32_t C, const fe* d_frame, DerivedConsts* dK, hipStream_t s) {
  if (W + C > 256) throw std::invalid_argument("more than 256 DEEP coefficients (W + C)");
  deep_coeffs_kernel<<<1, 256, 0, s>>>(d_gam, W, C, d_frame, fe_pow64(fe{2, 0}, 156), dK);
}

struct OodMult {
  fe m[16];
};
__global__ void ood_frame_kernel(const fe* __restrict__ pt, const fe* __restrict__ pc, uint32_t W, uint32_t C,
                                 uint32_t chunks, OodMult mult, fe* __restrict__ frame) {
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;  // output slot in transcript order
  const uint32_t n = W + C;
  if (o >= 2 * n) return;
  const uint32_t pt_ = o / n, r = o % n;  // point (z, zg), column in t | H
  const bool tr = r < W;
  const fe* src = tr ? pt + ((size_t)pt_ * W + r) * chunks : pc + ((size_t)pt_ * C + (r - W)) * chunks;
  fe acc = fe_zero();
  for (uint32_t k = 0; k < chunks; k++) acc = fe_add(acc, src[k]);
  frame[o] = tr ? acc : fe_mul(acc, mult.m[r - W]);
}
void launch_ood_frame(const fe* d_pt, const fe* d_pc, uint32_t W, uint32_t C, uint32_t chunks, const fe* mult,
                      fe* d_frame, hipStream_t s) {
  if (C > 16) throw std::invalid_argument("more than 16 composition columns");
  OodMult m{};
  for (uint32_t j = 0; j < C; j++) m.m[j] = mult[j];
  const uint32_t outs = 2 * (W + C);
  ood_frame_kernel<<<(outs + 127) / 128, 128, 0, s>>>(d_pt, d_pc, W, C, chunks, m, d_frame);
}

void launch_deep_denoms(const fe* d_roots, size_t Ntab, size_t N, fe z, fe zg, fe* d_dinv, hipStream_t s) {
  launch_coset_inv(d_roots, ilog2s(Ntab) - ilog2s(N), N, z, zg, 1, d_dinv, s);
}

void launch_deep(const fe* d_lde, const fe* d_clde, const fe* d_roots, size_t Ntab, const DeepParams& p,
                 const DerivedConsts* dK, const fe* d_dinv, fe* d_out, hipStream_t s, int split) {
  // N is a power of two >= 64: every thread gets exactly DEEP_PTS points
  const size_t threads = std::min<size_t>(256, p.N / DEEP_PTS);
  deep_kernel<<<(unsigned)(p.N / (threads * DEEP_PTS)), (unsigned)threads, 0, s>>>(
      d_lde, d_clde, d_roots, ilog2s(Ntab) - ilog2s(p.N), p, dK, d_dinv, d_out, split);
}

// fold: (v0+v1)/2 + alpha (v0-v1) / (2 x0), x0 = GENERATOR * g_d^i (constant offset, agg/trace.rs:764-800)
__global__ void fri_fold_kernel(const fe* ev, size_t half, const fe* alpha_p, const fe* iroots, int shift, fe inv3,
                                fe inv2, fe* out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= half) return;
  const fe alpha = *alpha_p;
  fe v0 = ev[i], v1 = ev[i + half];
  fe ix = fe_mul(inv3, iroots[i << shift]);
  out[i] = fe_mul(fe_add(fe_add(v0, v1), fe_mul(alpha, fe_mul(fe_sub(v0, v1), ix))), inv2);
}
void launch_fri_fold(const fe* d_ev, size_t Nd, const fe* d_alpha, const fe* d_iroots, size_t Ntab, fe* d_out,
                     hipStream_t s) {
  size_t h = Nd / 2;
  fe inv3 = fe_inv(fe{3, 0}), inv2 = fe_inv(fe{2, 0});
  fri_fold_kernel<<<(unsigned)((h + 255) / 256), 256, 0, s>>>(d_ev, h, d_alpha, d_iroots, ilog2s(Ntab) - ilog2s(Nd),
                                                               inv3, inv2, d_out);
}

__global__ void gather_kernel(const uint64_t* addrs, size_t k, fe* out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  out[i] = *reinterpret_cast<const fe*>(addrs[i]);
}
void launch_gather(const uint64_t* d_addrs, size_t k, fe* d_out, hipStream_t s) {
  if (k) gather_kernel<<<(unsigned)((k + 255) / 256), 256, 0, s>>>(d_addrs, k, d_out);
}

}  // namespace zkl

// compiled-in tuning values of this translation unit (zkl_hip_build_config)
#define ZKL_STR2(x) #x
#define ZKL_STR(x) ZKL_STR2(x)
namespace zkl {
const char* kernels_build_config() {
  return "NTT_ELEMS=" ZKL_STR(NTT_ELEMS_CFG) ";NTT_THREADS=" ZKL_STR(NTT_THREADS_CFG) ";CE_WAVES=" ZKL_STR(
      CE_WAVES_CFG) ";CE_POSE_WAVES=" ZKL_STR(CE_POSE_WAVES_CFG) ";DEEP_PTS=" ZKL_STR(DEEP_PTS_CFG) ";DEEP_COLS=" ZKL_STR(
      DEEP_COLS_CFG) ";CE_GROUPS=" ZKL_STR(CE_GROUPS_CFG) ";CE_DOT=" ZKL_STR(CE_DOT_CFG) ";CE_BRANCHFREE=" ZKL_STR(
      CE_BRANCHFREE_CFG);
}
}  // namespace zkl
