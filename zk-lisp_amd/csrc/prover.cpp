// MI355X segment prover: host orchestration of winterfell 0.13.1 `Prover::prove` for
// ZkLispAir + PoseidonHasher (reference instantiation prove.rs:425-517), exposed through
// the C ABI in include/zkl_hip.h.  Every heavy stage runs on the GPU (kernels.hip); the
// host keeps the Fiat-Shamir transcript (a few dozen permutations), builds Merkle
// multiproof index sets and serialises Proof::to_bytes().
#include <hip/hip_runtime.h>
#include <malloc.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <algorithm>
#include <chrono>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/zkl_hip.h"
#include "air_host.h"
#include "host_hash.h"
#include "kernels.h"
#include "host_proof.h"
#include "proof_view.h"

using namespace zkl;

namespace zkl {  // step.cpp
std::vector<uint8_t> step_encode(const zkl_air_public_inputs& pi, const zkl_step_info& s, const uint8_t* inner,
                                 size_t inner_len);
void step_digest(const uint8_t* p, size_t n, uint8_t digest[32], uint8_t rt[32]);
void children_root(const uint8_t suite[32], const uint8_t* digests, const uint8_t* roots, size_t n, uint8_t out[32]);
}  // namespace zkl

namespace {

#define HIPCHECK(x) ZKL_HIPCHECK(x)

struct InvalidArg : std::runtime_error { using std::runtime_error::runtime_error; };

uint32_t bitrev_u(uint32_t x, int logn) { uint32_t r = 0; for (int i = 0; i < logn; i++) r |= ((x >> i) & 1u) << (logn - 1 - i); return r; }

// ------------------------------------------------------------------ device buffers
struct DBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t b) {
    if (b <= bytes) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    HIPCHECK(hipMalloc(&p, b));
    bytes = b;
  }
  fe* f() const { return (fe*)p; }
  ~DBuf() { if (p) (void)hipFree(p); }
};

// Process-wide account of the pinned host memory the library holds (zkl_hip_pinned_bytes):
// every hipHostMalloc / hipHostFree of the library goes through these two.
std::atomic<uint64_t> g_pin_cur{0}, g_pin_peak{0};
void pin_alloc(void** p, size_t b) {
  HIPCHECK(hipHostMalloc(p, b, hipHostMallocDefault));
  const uint64_t c = g_pin_cur.fetch_add(b) + b;
  uint64_t pk = g_pin_peak.load();
  while (c > pk && !g_pin_peak.compare_exchange_weak(pk, c)) {
  }
}
hipError_t pin_free(void* p, size_t b) {
  if (!p) return hipSuccess;
  g_pin_cur.fetch_sub(b);
  return hipHostFree(p);
}

// Pinned host staging: copies from/to it are asynchronous DMA that neither blocks the host
// until the stream drains nor goes through the runtime's pageable bounce buffers.
struct HBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t b) {
    if (b <= bytes) return;
    (void)release();
    b += b / 4;  // sizes vary a little from proof to proof (query count, assertions)
    pin_alloc(&p, b);
    bytes = b;
  }
  hipError_t release() {
    const hipError_t e = pin_free(p, bytes);
    p = nullptr;
    bytes = 0;
    return e;
  }
  template <class T>
  T* at(size_t off = 0) const { return (T*)((char*)p + off); }
  ~HBuf() { (void)release(); }
};

}  // namespace

// pinned transcript staging (h_tx), in field elements: [0..4) seed + roots, [4..21) FRI
// remainder + commitment, [32] seed upload, [40] best nonce, [48..80) FRI coins/roots,
// [80..336) query draws, [336] FRI seed upload
constexpr size_t TX_CS = 48, TX_CS_MAX = 32, TX_QD = 80, TX_QD_MAX = 256, TX_FRI_SEED = 336, TX_WORDS = 344;

// ====================================================================== context
struct zkl_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::string err;
  double stage_ms[ZKL_NUM_STAGES] = {0};
  double host_ms[3] = {0, 0, 0};  // host setup before the first kernel, host tail after the last, whole call
  // tables
  size_t tab_n = 0, tab_N = 0;
  DBuf roots, iroots, mroots, miroots, opow, opow_n, pertab;
  // work buffers
  DBuf trace, coef, lde, parts, tree, ce, bvec, bm, clde, ctree, deep, draws, pw, oodv, oodf, txs, asl, ast, asv, ars;
  DBuf lcoef;  // coefficients (scaled, in LDE input order) of the boundary and composition column LDEs
  DBuf fri_ev, fri_tree, best, gaddr, gout, flag;
  DBuf xinv;    // batch-inverted coset denominators of DEEP (z-dependent)
  DBuf posep;   // PoseidonAir block's share of the transition sum per CE point (Poseidon layouts)
  DBuf cexinv;  // 1 / (x - g^(n-1)) over the CE coset: shape-only, kept while the key matches
  size_t cexinv_key_n = 0, cexinv_key_ce = 0, cexinv_key_tab = 0;
  const void* cexinv_key_roots = nullptr;
  DBuf kconst;  // ProofConsts of the proof in flight on this context (written by copies only)
  DBuf dconst;  // DerivedConsts: what the device derives per proof (pose_k, DEEP coefficients)
  DBuf fri_coin;  // device transcript of the FRI layers: seed, alpha, layer roots
  HBuf h_asrt, h_ood, h_addr, h_gv, h_tx, h_air;  // pinned staging: assertions, OOD frame, gather plan/values, transcript
  hipStream_t aux = nullptr;         // copy stream: assertion upload overlapped with the trace commitment
  hipEvent_t aux_ev = nullptr, hev = nullptr;
  // host-trace upload (zkl_hip_prove_segment): a ring of pinned slots, each filled from the
  // caller's pageable trace by host threads and DMA'd on its own copy stream while the compute
  // stream transforms the columns that already landed
  hipStream_t up = nullptr;
  std::vector<void*> up_slot;
  std::vector<hipEvent_t> up_ev;
  size_t up_slot_bytes = 0;
  double up_ms = 0;  // host wall time of the last proof's upload loop
  hipEvent_t stage_ev[ZKL_NUM_STAGES + 1] = {};
  bool stage_ev_ready = false;
  size_t pert_key_n = 0, pert_key_ce = 0;
  // kernel-family timers (HIP events on `stream` around each launch group)
  std::vector<hipEvent_t> evpool;
  std::vector<std::pair<int, size_t>> kmarks;  // (family, index of start event; stop = +1)
  size_t evnext = 0;
  int ktiming = 1;  // 0: no kernel-family events, 1: trace row hash only, 2: every family
  double kfam_ms[ZKL_NUM_KFAMILIES] = {0};
  int kfam_n[ZKL_NUM_KFAMILIES] = {0};
  // host scratch kept across proofs (gather plan, proof bytes, the AIR instance with its ~2.9e5
  // assertions): no per-proof allocation of the large host buffers
  std::vector<uint8_t> proof_s;
  Plan tplan_s;                              // trace / constraint tree query plan
  std::vector<Plan> fplan_s;                 // FRI layer plans
  std::vector<std::vector<size_t>> fpos_s;   // FRI layer query positions
  AirInstance air;
  // zkl_hip_trace_buffer: pinned host traces the caller fills in place (two slots: one filled
  // while the other's proof runs); zkl_hip_prove_segment DMAs columns straight from them
  HBuf tbuf[ZKL_TRACE_BUFFERS];
};

static const char* kFamilyNames =
    "ntt\ntrace_hash_rows\nmerkle\nconstraint_eval\ncomp_hash_rows\ndeep\nfri\ngrind\nmisc";
enum { KF_NTT = 0, KF_TRACE_HASH, KF_MERKLE, KF_CEVAL, KF_COMP_HASH, KF_DEEP, KF_FRI, KF_GRIND, KF_MISC };

namespace {

struct KScope {
  zkl_ctx* C;
  size_t i;
  // Each event record costs ~10 us of queue time between kernels, so by default only the
  // dominant family (the trace row hash) is bracketed; zkl_hip_set_kernel_timing(ctx, 2)
  // times every family (breakdown runs outside the timed region).
  KScope(zkl_ctx* c, int fam) : C(c), i(SIZE_MAX) {
    if (!(C->ktiming == 2 || (C->ktiming == 1 && fam == KF_TRACE_HASH))) return;
    if (C->evnext + 2 > C->evpool.size()) {
      size_t old = C->evpool.size();
      C->evpool.resize(old + 256);
      for (size_t k = old; k < C->evpool.size(); k++) HIPCHECK(hipEventCreate(&C->evpool[k]));
    }
    i = C->evnext;
    C->evnext += 2;
    C->kmarks.push_back({fam, i});
    HIPCHECK(hipEventRecord(C->evpool[i], C->stream));
  }
  ~KScope() {  // a failed stop record shows up as an error of hipEventElapsedTime in resolve_kernel_times
    if (i != SIZE_MAX) (void)hipEventRecord(C->evpool[i + 1], C->stream);
  }
};

void resolve_kernel_times(zkl_ctx* C) {
  for (int f = 0; f < ZKL_NUM_KFAMILIES; f++) { C->kfam_ms[f] = 0; C->kfam_n[f] = 0; }
  for (auto& m : C->kmarks) {
    float ms = 0;
    HIPCHECK(hipEventElapsedTime(&ms, C->evpool[m.second], C->evpool[m.second + 1]));
    C->kfam_ms[m.first] += ms;
    C->kfam_n[m.first]++;
  }
  C->kmarks.clear();
  C->evnext = 0;
}

const char* g_global_err = "";
thread_local std::string g_tls_err;

void set_err(zkl_ctx* c, const std::string& m) {
  if (c) c->err = m;
  g_tls_err = m;
  g_global_err = g_tls_err.c_str();
}

// PoseidonHasher constants (suite [0;32]) in both device forms: device globals, uploaded once
// per device (every context of a device shares them; they never change), then synchronised, so
// no proof carries a host-to-device copy of pageable memory (the runtime stages those)
void upload_hasher(hipStream_t s) {
  static HasherConsts hc;
  static HasherMont hm;
  static std::once_flag once;
  std::call_once(once, [] {
    const Hasher& H = hasher();
    for (int i = 0; i < 144; i++) hc.mds[i] = H.suite.mds[i / 12][i % 12];
    for (int r = 0; r < 27; r++) for (int l = 0; l < 12; l++) hc.rc[r * 12 + l] = H.suite.rc[r][l];
    hc.dom[0] = H.suite.dom[0]; hc.dom[1] = H.suite.dom[1];
    hc.dom_elems = H.dom_elems; hc.dom_merge = H.dom_merge; hc.dom_many = H.dom_many; hc.dom_int = H.dom_int;
    hm = make_hasher_mont(hc);
  });
  static std::mutex mu;
  static std::set<int> done;
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  if (done.count(dev)) return;
  upload_hasher_mont(hm, s);
  upload_pm_tables(hc, s);
  HIPCHECK(hipStreamSynchronize(s));
  done.insert(dev);
}

void ensure_tables(zkl_ctx* C, size_t n, size_t N) {
  hipStream_t s = C->stream;
  if (C->tab_N < N) {
    std::vector<fe> w(N), wi(N);
    fe g = root_of_unity(ilog2(N)), gi = fe_inv(g);
    w[0] = wi[0] = fe_one();
    for (size_t i = 1; i < N; i++) { w[i] = fe_mul(w[i - 1], g); wi[i] = fe_mul(wi[i - 1], gi); }
    C->roots.ensure(N * sizeof(fe));
    C->iroots.ensure(N * sizeof(fe));
    HIPCHECK(hipMemcpyAsync(C->roots.p, w.data(), N * sizeof(fe), hipMemcpyHostToDevice, s));
    HIPCHECK(hipMemcpyAsync(C->iroots.p, wi.data(), N * sizeof(fe), hipMemcpyHostToDevice, s));
    C->mroots.ensure(N * 20);
    C->miroots.ensure(N * 20);
    build_mont_table(w.data(), N, C->mroots.p, s);
    build_mont_table(wi.data(), N, C->miroots.p, s);
    HIPCHECK(hipStreamSynchronize(s));
    C->tab_N = N;
  }
  if (C->tab_n != n) {
    std::vector<fe> o(n), on(n);
    fe inv_n = fe_inv(fe{n, 0}), p = fe_one();
    for (size_t k = 0; k < n; k++) { o[k] = p; on[k] = fe_mul(p, inv_n); p = fe_mul(p, fe{3, 0}); }
    C->opow.ensure(n * sizeof(fe));
    C->opow_n.ensure(n * sizeof(fe));
    HIPCHECK(hipMemcpyAsync(C->opow.p, o.data(), n * sizeof(fe), hipMemcpyHostToDevice, s));
    HIPCHECK(hipMemcpyAsync(C->opow_n.p, on.data(), n * sizeof(fe), hipMemcpyHostToDevice, s));
    HIPCHECK(hipStreamSynchronize(s));
    C->tab_n = n;
  }
}

// Stage boundaries as HIP events on the proof stream.  Each record costs ~10 us of queue time,
// so the inner boundaries are recorded only with zkl_hip_set_kernel_timing(ctx, 2); the first
// and last (whole-proof device time) always are.  Events live in the context.
struct StageTimer {
  zkl_ctx* C;
  hipEvent_t* ev;
  bool inner;
  explicit StageTimer(zkl_ctx* c) : C(c), ev(c->stage_ev), inner(c->ktiming == 2) {
    if (!C->stage_ev_ready) {
      for (int i = 0; i <= ZKL_NUM_STAGES; i++) HIPCHECK(hipEventCreate(&C->stage_ev[i]));
      C->stage_ev_ready = true;
    }
  }
  void mark(int i) {
    if (inner || i == 0 || i == ZKL_NUM_STAGES) HIPCHECK(hipEventRecord(ev[i], C->stream));
  }
  void finish() {
    HIPCHECK(hipEventSynchronize(ev[ZKL_NUM_STAGES]));
    for (int i = 0; i < ZKL_NUM_STAGES; i++) {
      float ms = 0;
      if (inner) HIPCHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
      C->stage_ms[i] = ms;
    }
  }
};

// ZKL_HOST_TRACE=1: host timestamps (us since the call) of the phases around host round trips
static const bool g_host_trace = getenv("ZKL_HOST_TRACE") != nullptr;
// trace LDE in the even/odd split layout (kernels.h lde_pos): ZKL_LDE_SPLIT=0
// keeps natural order (A/B)
static const bool g_lde_split = [] {
  const char* e = getenv("ZKL_LDE_SPLIT");
  return !(e && !strcmp(e, "0"));
}();
#define HT(label)                                                                                   \
  do {                                                                                              \
    if (g_host_trace)                                                                               \
      fprintf(stderr, "[ht] %-24s %9.1f\n", label,                                                  \
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_call0).count()); \
  } while (0)

template <class T>
void d2h(zkl_ctx* C, T* dst, const void* src, size_t bytes) {
  HIPCHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, C->stream));
  HIPCHECK(hipStreamSynchronize(C->stream));
}

// powers kernel on host side is cheap enough only for small n: use geometric via GPU
__global__ void powers_kernel(fe base, fe mult, size_t n, int logn, fe* out) {
  size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  uint32_t k = logn ? (__brev((uint32_t)j) >> (32 - logn)) : 0;
  out[j] = fe_mul(mult, fe_pow64(base, k));
}

// Request checks that need no device (winterfell ProofOptions / PartitionOptions bounds, the
// options this backend supports, the public-input shape).  Shared by the prover and
// zkl_hip_check_request.
void validate_request(uint32_t W, uint32_t n32, const zkl_air_public_inputs& pi, const zkl_proof_options& o) {
  const size_t n = n32;
  if (n < 32 || (n & (n - 1))) throw InvalidArg("trace length must be a power of two >= 32");
  if (o.field_extension != 1) throw InvalidArg("only FieldExtension::None is supported for segment proofs");
  if (o.fri_folding_factor != 2) throw InvalidArg("only FRI folding factor 2 is supported");
  if (o.batching_constraints != 0 || o.batching_deep != 0) throw InvalidArg("only BatchingMethod::Linear is supported");
  // winterfell ProofOptions::new bounds [WF-recall]: blowup a power of two in 2..=128, grinding
  // factor <= 32 (the proof's context stores both as u8; a grind above 64 could never be met)
  if (o.blowup_factor < 2 || (o.blowup_factor & (o.blowup_factor - 1))) throw InvalidArg("blowup must be a power of two");
  if (o.blowup_factor > 128) throw InvalidArg("blowup must be at most 128");
  if (o.grinding_factor > 32) throw InvalidArg("grinding_factor must be at most 32");
  if (o.num_queries == 0 || o.num_queries > 255) throw InvalidArg("num_queries must be in 1..255");
  // winter-air PartitionOptions::new bounds (num_partitions 1..=16, min_partition_size 1..=256)
  if (o.num_partitions < 1 || o.num_partitions > 16) throw InvalidArg("num_partitions must be in 1..16");
  if (o.hash_rate < 1 || o.hash_rate > 255) throw InvalidArg("hash_rate must be in 1..255 (a u8 in the proof context)");
  if (o.fri_remainder_max_degree > 15 || ((o.fri_remainder_max_degree + 1) & o.fri_remainder_max_degree))
    throw InvalidArg("fri_remainder_max_degree must be one less than a power of two, at most 15");
  // the bounds the verifier applies to the options it decodes from the proof (verifier.cpp): a
  // request the library's own verifier, and the aggregation's child replay, would reject is
  // refused here rather than proved (remainder degree >= blowup)
  {
    const std::string e = check_proof_options(o);
    if (!e.empty()) throw InvalidArg(e);
  }
  if (pi.n_main_slots > ZKL_MAX_MAIN_SLOTS) throw InvalidArg("n_main_slots exceeds ZKL_MAX_MAIN_SLOTS");
  if (W == 0 || W > 4096) throw InvalidArg("trace width must be in 1..4096");
}

// Host-resident trace -> coefficient buffer, column chunk by column chunk, with the trace LDE of
// each chunk (iNTT over <g>, coset shift, DIT evaluation, all per-column transforms) issued on
// the compute stream as soon as its DMA lands.  The caller's trace is pageable memory (the Rust
// binding passes its Vec): host threads copy each chunk into a pinned slot (ZKL_UP_SLOTS slots of
// ZKL_UP_SLOT_MB), the copy stream DMAs the slot, the compute stream waits on that copy's event.
// The PCIe upload thus overlaps the LDE of the chunks before it, and the host copy of chunk j+1
// overlaps the DMA of chunk j.
constexpr int UP_SLOTS = 4;
constexpr size_t UP_SLOT_BYTES = (size_t)16 << 20;

// host copy threads of the upload ring (ZKL_UP_THREADS, default 8) and ZKL_UP_MODE=direct (each
// chunk straight from pageable memory; HIP stages it) for A/B on the GPU box
static unsigned up_threads() {
  static const unsigned t = [] {
    const char* e = getenv("ZKL_UP_THREADS");
    const unsigned d = std::max(1u, std::min(8u, std::thread::hardware_concurrency() / 2));
    return e ? std::max(1, atoi(e)) : (int)d;
  }();
  return t;
}
static bool up_direct() {
  static const bool d = [] {
    const char* e = getenv("ZKL_UP_MODE");
    return e && !strcmp(e, "direct");
  }();
  return d;
}

void parallel_copy(void* dst, const void* src, size_t bytes, unsigned nt) {
  if (nt <= 1 || bytes < ((size_t)1 << 20)) { memcpy(dst, src, bytes); return; }
  const size_t per = ((bytes + nt - 1) / nt + 63) & ~(size_t)63;
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt && t * per < bytes; t++)
    th.emplace_back([=] { memcpy((char*)dst + t * per, (const char*)src + t * per, std::min(per, bytes - t * per)); });
  memcpy(dst, src, std::min(per, bytes));
  for (auto& x : th) x.join();
}

template <class F>
void upload_trace_chunked(zkl_ctx* C, const void* h_trace, uint32_t W, size_t n, hipStream_t s, F&& on_chunk) {
  if (!C->up) {
    HIPCHECK(hipStreamCreateWithFlags(&C->up, hipStreamNonBlocking));
    C->up_slot.assign(UP_SLOTS, nullptr);
    C->up_ev.assign(UP_SLOTS, nullptr);
    for (int k = 0; k < UP_SLOTS; k++) {
      pin_alloc(&C->up_slot[k], UP_SLOT_BYTES);
      HIPCHECK(hipEventCreateWithFlags(&C->up_ev[k], hipEventDisableTiming));
    }
    C->up_slot_bytes = UP_SLOT_BYTES;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const size_t col_bytes = n * sizeof(fe);
  const uint32_t per = (uint32_t)std::max<size_t>(1, C->up_slot_bytes / col_bytes);
  const unsigned nt = up_threads();
  // a trace in one of the context's own pinned buffers (zkl_hip_trace_buffer) is DMA'd in place
  bool in_tbuf = false;
  for (const HBuf& b : C->tbuf)
    in_tbuf |= b.p && (const char*)h_trace >= (const char*)b.p &&
               (const char*)h_trace + (size_t)W * col_bytes <= (const char*)b.p + b.bytes;
  const bool direct = in_tbuf || up_direct();
  bool used[UP_SLOTS] = {false, false, false, false};
  double copy_ms = 0, wait_ms = 0;
  auto ms_since = [](std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  };
  int k = 0;
  for (uint32_t c0 = 0; c0 < W; c0 += per, k = (k + 1) % UP_SLOTS) {
    const uint32_t nc = std::min(per, W - c0);
    if (direct || col_bytes * nc > C->up_slot_bytes) {  // pageable copy (HIP stages it), or a column larger than a slot
      HIPCHECK(hipMemcpyAsync(C->coef.f() + (size_t)c0 * n, (const char*)h_trace + c0 * col_bytes, col_bytes * nc,
                              hipMemcpyHostToDevice, direct ? C->up : s));
      if (direct) {
        HIPCHECK(hipEventRecord(C->up_ev[k], C->up));
        HIPCHECK(hipStreamWaitEvent(s, C->up_ev[k], 0));
      }
      on_chunk(c0, nc);
      continue;
    }
    auto tw = std::chrono::steady_clock::now();
    if (used[k]) HIPCHECK(hipEventSynchronize(C->up_ev[k]));  // the slot's previous DMA has read it
    wait_ms += ms_since(tw);
    auto tc = std::chrono::steady_clock::now();
    parallel_copy(C->up_slot[k], (const char*)h_trace + c0 * col_bytes, col_bytes * nc, nt);
    copy_ms += ms_since(tc);
    HIPCHECK(hipMemcpyAsync(C->coef.f() + (size_t)c0 * n, C->up_slot[k], col_bytes * nc, hipMemcpyHostToDevice, C->up));
    HIPCHECK(hipEventRecord(C->up_ev[k], C->up));
    used[k] = true;
    HIPCHECK(hipStreamWaitEvent(s, C->up_ev[k], 0));
    on_chunk(c0, nc);
  }
  C->up_ms = ms_since(t0);
  if (getenv("ZKL_UP_DEBUG"))
    fprintf(stderr, "[zkl upload] %u cols x %zu rows: loop %.2f ms (host copy %.2f ms on %u threads, slot waits %.2f ms)%s\n",
            W, n, C->up_ms, copy_ms, nt, wait_ms, in_tbuf ? " pinned trace buffer" : direct ? " direct" : "");
}

// proofs running in any context: the row-digest rule (a process-wide test switch, DESIGN.md
// §3.1) may only change while this is zero
std::atomic<int> g_proofs_in_flight{0};
struct InFlight {
  InFlight() { g_proofs_in_flight.fetch_add(1); }
  ~InFlight() { g_proofs_in_flight.fetch_sub(1); }
};

// the proof bytes are left in C->proof_s (zkl_hip_last_proof), valid until the next proof
void prove_impl(zkl_ctx* C, const void* d_trace_in, bool trace_on_host, uint32_t W, uint32_t n32,
                const zkl_air_public_inputs& pi, const zkl_proof_options& o) {
  const InFlight in_flight;
  const auto t_call0 = std::chrono::steady_clock::now();
  hipStream_t s = C->stream;
  const size_t n = n32;
  validate_request(W, n32, pi, o);
  const size_t N = n * o.blowup_factor;
  const int logn = ilog2(n), logN = ilog2(N);
  const uint32_t B = o.blowup_factor;
  const fe g = root_of_unity(logn), three{3, 0};
  const Hasher& H = hasher();

  upload_hasher(s);
  ensure_tables(C, n, N);
  const fe* roots = C->roots.f();
  const fe* iroots = C->iroots.f();
  const MontTab mroots = mont_tab(C->mroots.p, C->tab_N), miroots = mont_tab(C->miroots.p, C->tab_N);
  const size_t Ntab = C->tab_N;

  StageTimer T(C);
  T.mark(0);
  C->host_ms[0] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call0).count();
  // ---- 1. trace LDE (DefaultTraceLde::new): iNTT over <g>, coset LDE over 3*<w_N>
  C->coef.ensure((size_t)W * n * sizeof(fe));
  C->lde.ensure((size_t)W * N * sizeof(fe));
  // columns [c0, c0 + nc): iNTT -> n*coef bit-reversed, scale c_k * 3^k (coset shift), DIT
  // every chunk takes the same pass split, so all columns share one layout
  int split = -1;
  // src: the caller's resident trace, read by the iNTT's first pass (nullptr: already in coef)
  auto lde_cols = [&](uint32_t c0, uint32_t nc, const fe* src) {
    fe* cf = C->coef.f() + (size_t)c0 * n;
    launch_intt_scaled(src, cf, nc, n, miroots, Ntab, C->opow_n.f(), s);
    const int sp = launch_lde_from_coeffs(cf, nc, n, N, mroots, Ntab, C->lde.f() + (size_t)c0 * N, s, g_lde_split);
    // the row hash, evaluator and DEEP read every column with one layout (the NTT mode cannot
    // change during a proof: zkl_hip_set_ntt_mode refuses while one is in flight)
    if (split >= 0 && sp != split) throw std::runtime_error("internal: trace LDE chunks in different layouts");
    split = sp;
  };
  if (trace_on_host) {
    KScope k(C, KF_NTT);
    upload_trace_chunked(C, d_trace_in, W, n, s, [&](uint32_t c0, uint32_t nc) { lde_cols(c0, nc, nullptr); });
  } else {
    C->up_ms = 0;
    KScope k(C, KF_NTT);
    lde_cols(0, W, (const fe*)d_trace_in);
  }
  check_launch("trace LDE");
  if (split < 0) split = 0;
  T.mark(1);
  // ---- trace commitment (commit_to_rows + MerkleTree)
  C->parts.ensure((size_t)o.num_partitions * N * sizeof(fe) + N * sizeof(fe));
  C->tree.ensure(2 * N * sizeof(fe));
  {
    KScope k(C, KF_TRACE_HASH);
    launch_hash_rows(C->lde.f(), W, N, o.num_partitions, o.hash_rate, C->parts.f(), C->tree.f() + N, s, 0, split);
  }
  check_launch("trace row hash");
  // ---- coin seed: Context::to_elements || AirPublicInputs::to_elements (agg/fs.rs:67-73),
  // hashed on the host while the device runs the trace LDE and row hash queued above
  std::vector<fe> seed_el = context_elements(W, n, o);
  auto pie = pi_elements(pi);
  seed_el.insert(seed_el.end(), pie.begin(), pie.end());
  Coin coin{H.hash_elements(seed_el.data(), seed_el.size()), 0};
  // The transcript up to the OOD point runs on the device: the seed goes up once, and the
  // trace-root reseed and the composition-coefficient draws follow the trace tree with no host
  // round trip (tx: [0] coin seed, [1] query seed, [2] trace root, [3] constraint root,
  // [4..] FRI remainder + its commitment; h_tx mirrors it, h_tx[32] stages the upload).
  // every per-proof copy goes through pinned memory (h_tx): an asynchronous copy to or from
  // pageable memory makes the runtime stage it, which was seen to stall the stream
  C->txs.ensure(64 * sizeof(fe));
  C->h_tx.ensure(TX_WORDS * sizeof(fe));
  fe* tx = C->txs.f();
  fe* htx = C->h_tx.at<fe>();
  htx[32] = coin.seed;
  HIPCHECK(hipMemcpyAsync(tx, htx + 32, sizeof(fe), hipMemcpyHostToDevice, s));
  {
    KScope k(C, KF_MERKLE);
    launch_merkle(C->tree.f(), N, s, tx, tx + 2, 1);  // + the trace-root reseed
  }
  check_launch("trace Merkle tree and trace-root reseed");
  coin.counter = 0;  // coin.seed is on the device until the constraint root
  // The AIR instance (layout, degrees, ~2.9e5 assertions at n = 2^16) is built on the host
  // meanwhile too.
  AirInstance& air = C->air;
  {
    std::string e = build_air(pi, W, n, air);
    if (e.empty() && o.blowup_factor < (uint32_t)air.ce_blowup) e = "blowup factor below constraint-evaluation blowup";
    if (!e.empty()) {
      (void)hipStreamSynchronize(s);
      throw InvalidArg(e);
    }
  }
  const size_t ce = n * air.ce_blowup;
  const int logce = ilog2(ce);
  const int Cc = air.num_comp_cols;
  C->kconst.ensure(sizeof(ProofConsts));
  ProofConsts* dK = (ProofConsts*)C->kconst.p;
  C->dconst.ensure(sizeof(DerivedConsts));
  DerivedConsts* dD = (DerivedConsts*)C->dconst.p;
  C->h_air.ensure(sizeof(AirDevice));
  memcpy(C->h_air.p, &air.dev, sizeof(AirDevice));
  upload_air_consts(dK, *C->h_air.at<AirDevice>(), s);
  const size_t na = air.assertions.size();
  // boundary tables: per asserted column c, M_c = coset-LDE of
  // reverse(NTT_n(beta_c)); W likewise from sum_c beta*value.
  std::map<uint32_t, uint32_t> slot_of;
  std::vector<uint32_t> bcols;
  for (auto& a : air.assertions)
    if (!slot_of.count(a.col)) { slot_of[a.col] = (uint32_t)bcols.size(); bcols.push_back(a.col); }
  if (bcols.size() > 64) throw InvalidArg("too many asserted columns");
  const uint32_t nb = (uint32_t)bcols.size();
  // assertion tables written straight into pinned memory and uploaded on the copy stream,
  // so the DMA runs under the trace commitment instead of after it
  const size_t off_st = na * 4, off_sv = (na * 8 + 15) & ~(size_t)15, off_rs = off_sv + na * sizeof(fe);
  C->h_asrt.ensure(off_rs + (n + 1) * 4);
  uint32_t* hslot = C->h_asrt.at<uint32_t>(0);
  uint32_t* hstep = C->h_asrt.at<uint32_t>(off_st);
  fe* hval = C->h_asrt.at<fe>(off_sv);
  uint32_t* rowstart = C->h_asrt.at<uint32_t>(off_rs);
  memset(rowstart, 0, (n + 1) * 4);
  for (size_t k = 0; k < na; k++) {
    hslot[k] = slot_of[air.assertions[k].col];
    hstep[k] = air.assertions[k].step;
    hval[k] = air.assertions[k].value;
    rowstart[hstep[k] + 1]++;
  }
  for (size_t r = 0; r < n; r++) rowstart[r + 1] += rowstart[r];
  C->asl.ensure(na * 4); C->ast.ensure(na * 4); C->asv.ensure(na * sizeof(fe)); C->ars.ensure((n + 1) * 4);
  if (!C->aux) {
    HIPCHECK(hipStreamCreateWithFlags(&C->aux, hipStreamNonBlocking));
    HIPCHECK(hipEventCreateWithFlags(&C->aux_ev, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&C->hev, hipEventDisableTiming));
  }
  HIPCHECK(hipMemcpyAsync(C->asl.p, hslot, na * 4, hipMemcpyHostToDevice, C->aux));
  HIPCHECK(hipMemcpyAsync(C->ast.p, hstep, na * 4, hipMemcpyHostToDevice, C->aux));
  HIPCHECK(hipMemcpyAsync(C->asv.p, hval, na * sizeof(fe), hipMemcpyHostToDevice, C->aux));
  HIPCHECK(hipMemcpyAsync(C->ars.p, rowstart, (n + 1) * 4, hipMemcpyHostToDevice, C->aux));
  HIPCHECK(hipEventRecord(C->aux_ev, C->aux));
  HIPCHECK(hipStreamWaitEvent(s, C->aux_ev, 0));
  C->bvec.ensure((size_t)(nb + 1) * n * sizeof(fe));
  C->bm.ensure((size_t)(nb + 1) * ce * sizeof(fe));
  HT("air_built");
  T.mark(2);

  // ---- 2. composition coefficients (Linear): transition then boundary, one draw each
  const size_t ndraw = (size_t)air.n_tc + na;
  C->draws.ensure((ndraw + 1024) * sizeof(fe));
  {
    KScope k(C, KF_MISC);
    launch_draws(fe_zero(), coin.counter, ndraw, C->draws.f(), s, tx);
  }
  check_launch("composition coefficient draws");
  coin.counter += ndraw;
  upload_alphas_from_device(dK, C->draws.f(), air.n_tc, s);
  launch_pose_k(dK, dD, air.n_tc, air.dev.pose_block != 0, s);

  HIPCHECK(hipMemsetAsync(C->bvec.p, 0, (size_t)(nb + 1) * n * sizeof(fe), s));
  const fe* betas = C->draws.f() + air.n_tc;
  {
    KScope k(C, KF_CEVAL);
    launch_boundary_scatter((const uint32_t*)C->asl.p, (const uint32_t*)C->ast.p, betas, na, n, C->bvec.f(), s);
    launch_boundary_w((const uint32_t*)C->ars.p, betas, C->asv.f(), n, C->bvec.f() + (size_t)nb * n, s);
  }
  {
    KScope k(C, KF_NTT);
    launch_ntt_stages(C->bvec.f(), nb + 1, n, true, 0, logn - 1, mroots, Ntab, s);  // forward, bit-reversed out
    // reversed, scaled coefficients, then the DIT over the CE coset whose first pass reads each
    // of them blowup times (the copies are not materialised; same values as a broadcast)
    C->lcoef.ensure((size_t)std::max<uint32_t>(nb + 1, Cc) * n * sizeof(fe));
    launch_broadcast(C->bvec.f(), n, 1, 0, nb + 1, n, n, C->opow.f(), fe_one(), true, C->lcoef.f(), s);
    launch_lde_from_coeffs(C->lcoef.f(), nb + 1, n, ce, mroots, Ntab, C->bm.f(), s, false);
  }
  check_launch("boundary tables");

  // periodic table
  if (C->pert_key_n != n || C->pert_key_ce != ce) {
    auto tab = periodic_table(n, ce, three);
    C->pertab.ensure(tab.size() * sizeof(fe));
    HIPCHECK(hipMemcpyAsync(C->pertab.p, tab.data(), tab.size() * sizeof(fe), hipMemcpyHostToDevice, s));
    HIPCHECK(hipStreamSynchronize(s));
    C->pert_key_n = n; C->pert_key_ce = ce;
  }
  CeParams cp{};
  cp.n = n; cp.N = N; cp.ce = ce; cp.blowup = B;
  cp.gl = fe_pow64(g, n - 1);
  cp.inv_n = fe_inv(fe{n, 0});
  cp.lagr = fe_mul(cp.gl, cp.inv_n);
  {
    size_t blow = ce / n;
    fe wb = root_of_unity(ilog2(blow)), on = fe_pow64(three, n), p = fe_one();
    for (size_t j = 0; j < blow; j++) {
      cp.xn_m1[j] = fe_sub(fe_mul(on, p), fe_one());
      cp.xn_inv[j] = fe_inv(cp.xn_m1[j]);
      p = fe_mul(p, wb);
    }
  }
  cp.n_bcols = nb;
  for (uint32_t u = 0; u < nb; u++) cp.bcol[u] = bcols[u];
  C->ce.ensure(ce * sizeof(fe));
  {
    KScope k(C, KF_CEVAL);
    const bool ready = C->cexinv_key_n == n && C->cexinv_key_ce == ce && C->cexinv_key_tab == Ntab &&
                       C->cexinv_key_roots == (const void*)roots && C->cexinv.bytes >= ce * sizeof(fe);
    if (!ready) {
      C->cexinv_key_n = 0;  // invalid until the launch below has been queued
      C->cexinv.ensure(ce * sizeof(fe));
    }
    if (air.dev.pose_block) C->posep.ensure(ce * sizeof(fe));
    launch_constraint_eval(C->lde.f(), roots, Ntab, C->pertab.f(), C->bm.f(), cp, dK, dD, air.dev.pose_block != 0,
                           (air.dev.ram_block | air.dev.merkle_block) != 0, C->cexinv.f(), ready, C->ce.f(), s, split,
                           air.dev.pose_block ? C->posep.f() : nullptr);
    C->cexinv_key_n = n; C->cexinv_key_ce = ce; C->cexinv_key_tab = Ntab; C->cexinv_key_roots = roots;
  }
  check_launch("constraint evaluation");
  T.mark(3);

  // ---- 3. composition polynomial: coset interpolation, degree check, column LDE, commit
  C->flag.ensure(16);
  C->clde.ensure((size_t)Cc * N * sizeof(fe));
  const int loge = ilog2(ce / n);
  const fe inv3 = fe_inv(three), inv_ce = fe_inv(fe{ce, 0});
  {
    KScope k(C, KF_NTT);
    launch_ntt_stages(C->ce.f(), 1, ce, true, 0, logce - 1, miroots, Ntab, s);  // ce * c_k * 3^k (bitrev)
    HIPCHECK(hipMemsetAsync(C->flag.p, 0, 4, s));
    launch_check_zero_range_bitrev(C->ce.f(), ce, (size_t)Cc * n, ce, (unsigned*)C->flag.p, s);
    for (int j = 0; j < Cc; j++) {
      // column j coefficient k' = chat[j n + k'] * 3^(-(j n + k')) / ce; LDE multiplies by 3^k'
      fe mult = fe_mul(fe_pow64(inv3, (uint64_t)j * n), inv_ce);
      launch_broadcast(C->ce.f(), 0, ce / n, bitrev_u((uint32_t)j, loge), 1, n, n, nullptr, mult, false,
                       C->lcoef.f() + (size_t)j * n, s);
    }
    launch_lde_from_coeffs(C->lcoef.f(), Cc, n, N, mroots, Ntab, C->clde.f(), s, false);
  }
  check_launch("composition polynomial LDE");
  C->ctree.ensure(2 * N * sizeof(fe));
  {
    KScope k(C, KF_COMP_HASH);
    launch_hash_rows(C->clde.f(), Cc, N, o.num_partitions, o.hash_rate, C->parts.f(), C->ctree.f() + N, s, 1);
  }
  {
    KScope k(C, KF_MERKLE);
    launch_merkle(C->ctree.f(), N, s, tx, tx + 3, 1);  // + the constraint-root reseed
  }
  check_launch("composition commitment");
  // one round trip: degree flag, both roots and the coin seed after the constraint root
  HIPCHECK(hipMemcpyAsync(htx, tx, 4 * sizeof(fe), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipMemcpyAsync(htx + 4, C->flag.p, 4, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  HT("croot");
  unsigned bad = 0;
  memcpy(&bad, htx + 4, 4);
  if (bad) throw InvalidArg("constraint composition polynomial degree too large: trace does not satisfy the AIR");
  const fe troot = htx[2], croot = htx[3];
  coin.seed = htx[0];
  coin.counter = 0;
  T.mark(4);

  // ---- 4. OOD frame at z and z*g
  fe z = coin.draw(), zg = fe_mul(z, g);
  C->pw.ensure(4 * n * sizeof(fe));
  fe* pw = C->pw.f();
  // both the trace coefficients (c_k 3^k) and the composition columns carry the coset
  // shift, so one pair of bit-reversed power vectors of z/3 and zg/3 serves both
  powers_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(fe_mul(z, inv3), fe_one(), n, logn, pw + 2 * n);
  powers_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(fe_mul(zg, inv3), fe_one(), n, logn, pw + 3 * n);
  const uint32_t chunks = n >= 8192 ? 32 : 1;  // parallelism for the few composition columns
  const size_t n_otr = 2 * (size_t)W * chunks, n_ocp = 2 * (size_t)Cc * chunks;
  C->oodv.ensure((n_otr + n_ocp) * sizeof(fe));
  fe* dood = C->oodv.f();
  if (Cc > 16) throw std::runtime_error("internal: more than 16 composition columns");
  {
    KScope k(C, KF_MISC);
    OodArgs a{};
    a.coef = C->coef.f(); a.col_stride = n; a.elem_stride = 1; a.n = n;
    a.pw1 = pw + 2 * n; a.pw2 = pw + 3 * n; a.ncols = W; a.chunks = chunks; a.use_off = 0;
    launch_ood(a, dood, s);
    OodArgs b{};
    b.coef = C->ce.f(); b.col_stride = 0; b.elem_stride = ce / n; b.n = n;
    b.pw1 = pw + 2 * n; b.pw2 = pw + 3 * n; b.ncols = (uint32_t)Cc; b.chunks = chunks; b.use_off = 1;
    for (int j = 0; j < Cc; j++) b.off[j] = bitrev_u((uint32_t)j, loge);
    launch_ood(b, dood + n_otr, s);
  }
  std::vector<fe> cmult(Cc);
  for (int j = 0; j < Cc; j++) cmult[j] = fe_mul(fe_pow64(inv3, (uint64_t)j * n), inv_ce);
  // chunk sums and the composition scaling on the device, so only the 2 (W + C) frame values
  // cross PCIe (a small copy: no SDMA start-up latency in the transcript's critical path)
  C->oodf.ensure(2 * ((size_t)W + Cc) * sizeof(fe));
  fe* dframe = C->oodf.f();
  launch_ood_frame(dood, dood + n_otr, W, (uint32_t)Cc, chunks, cmult.data(), dframe, s);
  check_launch("OOD evaluation");
  const size_t nfr = 2 * ((size_t)W + Cc);
  C->h_ood.ensure(nfr * sizeof(fe));
  const fe* frame = C->h_ood.at<fe>();
  HIPCHECK(hipMemcpyAsync(C->h_ood.p, dframe, nfr * sizeof(fe), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipEventRecord(C->hev, s));
  // the DEEP denominators depend on z only: the device computes them while the host hashes the
  // frame into the transcript
  C->xinv.ensure(std::max(ce, N) * sizeof(fe));
  {
    KScope k(C, KF_DEEP);
    launch_deep_denoms(roots, Ntab, N, z, zg, C->xinv.f(), s);
  }
  check_launch("DEEP denominators");
  HT("ood_enqueued");
  HIPCHECK(hipEventSynchronize(C->hev));
  // frame = t(z) [W] | H(z) [Cc] | t(zg) [W] | H(zg) [Cc]: the order hashed (agg/fs.rs:152-164)
  std::vector<fe> tz(frame, frame + W), hz(frame + W, frame + W + Cc);
  std::vector<fe> tzg(frame + W + Cc, frame + 2 * W + Cc), hzg(frame + 2 * W + Cc, frame + nfr);
  coin.reseed(H.hash_elements(frame, nfr));
  T.mark(5);

  // ---- 5. DEEP composition coefficients (W trace, then C constraint) and evaluations: drawn,
  // converted and dotted with the frame on the device
  HT("ood_hashed");
  launch_draws(coin.seed, coin.counter, W + Cc, C->draws.f(), s);
  check_launch("DEEP coefficient draws");
  coin.counter += W + Cc;
  launch_deep_coeffs(C->draws.f(), W, (uint32_t)Cc, dframe, dD, s);
  check_launch("DEEP coefficients");
  HT("gam");
  DeepParams dp{};
  dp.N = N; dp.W = W; dp.C = Cc; dp.z = z; dp.zg = zg;
  C->deep.ensure(N * sizeof(fe));
  {
    KScope k(C, KF_DEEP);
    launch_deep(C->lde.f(), C->clde.f(), roots, Ntab, dp, dD, C->xinv.f(), C->deep.f(), s, split);
  }
  check_launch("DEEP composition");
  T.mark(6);

  // ---- 6. FRI (FriProver::build_layers, folding 2, remainder degree rem_deg)
  const size_t rem_max = (size_t)(o.fri_remainder_max_degree + 1) * B;
  int nl = 0;
  for (size_t d = N; d > rem_max; d /= 2) nl++;
  std::vector<size_t> ev_off(nl + 1), tr_off(nl);
  size_t ev_tot = 0, tr_tot = 0;
  for (int d = 0; d <= nl; d++) {
    ev_off[d] = ev_tot;
    if (d >= 1) ev_tot += N >> d;
    if (d < nl) { tr_off[d] = tr_tot; tr_tot += N >> d; }  // tree over Nd/2 leaves: 2*(Nd/2) nodes
  }
  C->fri_ev.ensure((ev_tot + 1) * sizeof(fe));
  C->fri_tree.ensure((tr_tot + 1) * sizeof(fe));
  auto layer_ev = [&](int d) -> fe* { return d == 0 ? C->deep.f() : C->fri_ev.f() + ev_off[d]; };
  // the layer transcript (reseed with the layer root, draw alpha) runs on the device, so the
  // whole layer chain is queued without a host round trip
  std::vector<fe> fri_roots(nl);
  C->fri_coin.ensure((2 + (size_t)nl) * sizeof(fe));
  fe* d_coin = C->fri_coin.f();
  htx[TX_FRI_SEED] = coin.seed;
  HIPCHECK(hipMemcpyAsync(d_coin, htx + TX_FRI_SEED, sizeof(fe), hipMemcpyHostToDevice, s));
  for (int d = 0; d < nl; d++) {
    size_t Nd = N >> d, h = Nd / 2;
    fe* tr = C->fri_tree.f() + tr_off[d];
    {
      KScope k(C, KF_FRI);
      launch_fri_leaves(layer_ev(d), Nd, tr + h, s);
    }
    {
      KScope k(C, KF_MERKLE);
      launch_merkle(tr, h, s, d_coin, d_coin + 2 + d, 2);  // + the layer's reseed and alpha
    }
    KScope k(C, KF_FRI);
    launch_fri_fold(layer_ev(d), Nd, d_coin + 1, iroots, Ntab, layer_ev(d + 1), s);
  }
  check_launch("FRI layers");
  HT("fri_enqueued");
  // FRI remainder, its commitment and the reseed, grinding, the query seed and the query draws
  // all follow the layer chain on the device; the host reads the results back once
  const size_t Nr = N >> nl;
  const uint32_t rlen = o.fri_remainder_max_degree + 1;
  {
    const fe w = root_of_unity(ilog2(Nr)), wi = fe_inv(w), inv_nr = fe_inv(fe{Nr, 0});
    fe wk[16], sk[16];
    for (uint32_t k = 0; k < rlen; k++) {
      wk[k] = fe_pow64(wi, k);
      sk[k] = fe_mul(inv_nr, fe_pow64(inv3, k));
    }
    KScope k(C, KF_FRI);
    launch_fri_remainder(layer_ev(nl), (uint32_t)Nr, rlen, wk, sk, d_coin, tx + 4, s);
  }
  check_launch("FRI remainder");
  T.mark(7);

  // ---- 7. grinding: smallest nonce >= 1 (winterfell without `concurrent`)
  HT("grind_start");
  uint64_t nonce = 0;
  C->best.ensure(8);
  unsigned long long* hbest = (unsigned long long*)(htx + 40);
  // Ascending windows of nonces; the answer is the minimum of the first window that holds a
  // solution.  Four windows (2^g, 2^g, 2^(g+1), 2^(g+2) tries) are queued per read-back, and a
  // window's kernel returns at once when an earlier one has already found a solution (grind
  // kernels check *best first), so the search costs the windows it needs plus a few empty
  // launches, and one read-back settles it with probability 1 - e^-8.  A window of 2^16 tries is
  // one permutation's latency on the chip (~0.45 ms); the expected cost is (1 + e^-1 + 2 e^-2 +
  // 4 e^-4) windows = 1.7 instead of the 2.6 of one 2^(g+1) window first and doubling after it.
  // grinding factor 0: the first candidate, nonce 1.
  uint32_t batch = 1u << std::min<uint32_t>(std::max<uint32_t>(o.grinding_factor, 14), 22);
  // test-only: ZKL_TEST_GRIND_FIRST=<tries> shrinks the first window, so a test reaches the host
  // continuation below (a path real proofs take with probability e^-8) and checks its nonce
  // (read per proof because a test process sets it per test; announced once per process)
  if (const char* e = getenv("ZKL_TEST_GRIND_FIRST")) {
    batch = (uint32_t)std::max(1L, std::min(atol(e), 1L << 22));
    static std::once_flag said;
    std::call_once(said, [&] { fprintf(stderr, "zkl_hip: test hook ZKL_TEST_GRIND_FIRST=%s active\n", e); });
  }
  uint64_t base = 1;
  auto queue_windows = [&](const fe* d_seed, fe h_seed) {
    *hbest = o.grinding_factor == 0 ? 1ull : ~0ull;
    HIPCHECK(hipMemcpyAsync(C->best.p, hbest, 8, hipMemcpyHostToDevice, s));
    if (o.grinding_factor == 0) return;
    KScope k(C, KF_GRIND);
    for (int w = 0; w < 4; w++) {
      launch_grind(h_seed, base, batch, o.grinding_factor, (unsigned long long*)C->best.p, s, d_seed);
      base += batch;
      if (w >= 1) batch = std::min<uint32_t>(batch * 2, 1u << 22);
    }
  };
  queue_windows(d_coin, fe_zero());
  launch_query_seed(d_coin, (const unsigned long long*)C->best.p, s);
  launch_draws(fe_zero(), 0, o.num_queries, C->draws.f(), s, d_coin + 1);
  check_launch("grinding and query draws");
  // one read-back: layer coins / roots, remainder + commitment, nonce, query draws
  if (2 + (size_t)nl > TX_CS_MAX || o.num_queries > TX_QD_MAX) throw std::runtime_error("internal: transcript staging");
  HIPCHECK(hipMemcpyAsync(htx + TX_CS, d_coin, (2 + (size_t)nl) * sizeof(fe), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipMemcpyAsync(htx + 4, tx + 4, (rlen + 1) * sizeof(fe), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipMemcpyAsync(hbest, C->best.p, 8, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipMemcpyAsync(htx + TX_QD, C->draws.p, o.num_queries * sizeof(fe), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  std::vector<fe> cs(htx + TX_CS, htx + TX_CS + 2 + nl), qd(htx + TX_QD, htx + TX_QD + o.num_queries);
  for (int d = 0; d < nl; d++) fri_roots[d] = cs[2 + d];
  std::vector<fe> rem(htx + 4, htx + 4 + rlen);
  const fe rem_commit = htx[4 + rlen];
  coin.seed = cs[0];  // after the remainder reseed
  coin.counter = 0;
  HT("rem");
  if (*hbest != ~0ull) {
    nonce = *hbest;
  } else {  // none in the first four windows (probability e^-8): continue from the host
    while (nonce == 0) {
      queue_windows(nullptr, coin.seed);
      check_launch("grinding");
      HIPCHECK(hipMemcpyAsync(hbest, C->best.p, 8, hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
      if (*hbest != ~0ull) nonce = *hbest;
    }
    launch_draws(H.merge_with_int(coin.seed, nonce), 0, o.num_queries, C->draws.f(), s);
    check_launch("query draws");
    HIPCHECK(hipMemcpyAsync(htx + TX_QD, C->draws.p, o.num_queries * sizeof(fe), hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    qd.assign(htx + TX_QD, htx + TX_QD + o.num_queries);
  }
  T.mark(8);

  // ---- 8. query positions: draw_integers(q, N, nonce), sort, dedup
  HT("q_start");
  HT("q_drawn");
  std::vector<size_t> pos;
  for (auto& v : qd) pos.push_back((size_t)(v.lo & (N - 1)));
  std::sort(pos.begin(), pos.end());
  pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
  const size_t nq = pos.size();

  HT("q_sorted");
  // gather plan: trace rows, comp rows, trace/comp tree nodes, FRI values + tree nodes.  Host
  // work between two device round trips (the GPU idles through it): written into per-context
  // scratch that keeps its capacity, no allocation in the steady state.
  // upper bound of the address count: rows, two tree plans, per FRI layer two values and a plan
  // per position (a plan has at most depth + 2 entries per position)
  const size_t na_max = nq * ((size_t)W + Cc) + 2 * nq * ((size_t)logN + 2) + (size_t)nl * nq * ((size_t)logN + 4);
  C->h_addr.ensure(na_max * 8);
  uint64_t* const abase = C->h_addr.at<uint64_t>();
  uint64_t* ap = abase;
  for (size_t k = 0; k < nq; k++) {
    const fe* rp = C->lde.f() + lde_pos(pos[k], N, split);
    for (uint32_t c = 0; c < W; c++) *ap++ = (uint64_t)(uintptr_t)(rp + (size_t)c * N);
  }
  for (size_t k = 0; k < nq; k++)
    for (int j = 0; j < Cc; j++) *ap++ = (uint64_t)(uintptr_t)(C->clde.f() + (size_t)j * N + pos[k]);
  // every section checks its room before it writes (the bound above is an estimate of the plans)
  auto room = [&](size_t k) {
    if ((size_t)(ap - abase) + k > na_max) throw std::runtime_error("internal: gather plan bound");
  };
  auto append_nodes = [&](const fe* tree, const Plan& plan) {
    room(plan.node.size());
    for (uint64_t ix : plan.node) *ap++ = (uint64_t)(uintptr_t)(tree + ix);
  };
  Plan& tplan = C->tplan_s;
  batch_plan_into(N, pos.data(), nq, tplan);
  append_nodes(C->tree.f(), tplan);
  append_nodes(C->ctree.f(), tplan);
  std::vector<std::vector<size_t>>& fpos = C->fpos_s;
  std::vector<Plan>& fplan = C->fplan_s;
  if (fpos.size() < (size_t)nl) fpos.resize(nl);
  if (fplan.size() < (size_t)nl) fplan.resize(nl);
  {
    size_t dsz = N;
    for (int d = 0; d < nl; d++) {
      const size_t h = dsz / 2;
      const std::vector<size_t>& p = d ? fpos[d - 1] : pos;
      std::vector<size_t>& f = fpos[d];
      f.clear();
      // fold positions, first occurrence kept (FriProver::build_proof order); a 512-slot open
      // addressing set instead of a linear search per position (nq <= 256)
      uint64_t seen_key[512];
      uint8_t seen[512] = {0};
      for (size_t x : p) {
        const size_t y = x & (h - 1);
        size_t k = (size_t)(((uint64_t)y * 0x9E3779B97F4A7C15ull) >> 55);
        while (seen[k] && seen_key[k] != y) k = (k + 1) & 511;
        if (!seen[k]) {
          seen[k] = 1;
          seen_key[k] = y;
          f.push_back(y);
        }
      }
      room(2 * f.size());
      for (size_t y : f) { *ap++ = (uint64_t)(uintptr_t)(layer_ev(d) + y); *ap++ = (uint64_t)(uintptr_t)(layer_ev(d) + y + h); }
      batch_plan_into(h, f.data(), f.size(), fplan[d]);
      append_nodes(C->fri_tree.f() + tr_off[d], fplan[d]);
      dsz = h;
    }
  }
  HT("q_planned");
  const size_t na_g = (size_t)(ap - abase);
  C->gaddr.ensure((na_g + na_g / 4) * 8);
  C->gout.ensure((na_g + na_g / 4) * sizeof(fe));
  C->h_gv.ensure(na_g * sizeof(fe));
  HIPCHECK(hipMemcpyAsync(C->gaddr.p, C->h_addr.p, na_g * 8, hipMemcpyHostToDevice, s));
  launch_gather((const uint64_t*)C->gaddr.p, na_g, C->gout.f(), s);
  check_launch("query gather");
  HIPCHECK(hipMemcpyAsync(C->h_gv.p, C->gout.p, na_g * sizeof(fe), hipMemcpyDeviceToHost, s));
  // the proof's device work ends here: its closing stage events go in before the wait, so
  // T.finish() finds them complete instead of queueing a record behind it and waiting again
  T.mark(9);
  T.mark(10);
  HIPCHECK(hipStreamSynchronize(s));
  HT("q_gathered");
  const fe* gv = C->h_gv.at<fe>();
  size_t gi = 0;

  // ---- 9. Proof::to_bytes  [WF-recall layout, DESIGN.md §Proof bytes]
  Bytes P;
  P.v.swap(C->proof_s);
  P.v.clear();
  P.v.reserve(na_g * 32 + 4096);
  P.u8((uint8_t)W); P.u8(0); P.u8(0); P.u8((uint8_t)logn); P.u8(0); P.u8(0);  // TraceInfo
  P.u8(16); P.felem(fe{P_LO, P_HI});                                           // modulus bytes
  P.u8((uint8_t)o.num_queries); P.u8((uint8_t)o.blowup_factor); P.u8((uint8_t)o.grinding_factor);
  P.u8((uint8_t)o.field_extension); P.u8((uint8_t)o.fri_folding_factor); P.u8((uint8_t)o.fri_remainder_max_degree);
  P.u8((uint8_t)o.batching_constraints); P.u8((uint8_t)o.batching_deep);
  P.u8((uint8_t)o.num_partitions); P.u8((uint8_t)o.hash_rate);
  P.u8((uint8_t)nq);
  {
    Bytes cm;
    cm.digest(troot); cm.digest(croot);
    for (auto& r : fri_roots) cm.digest(r);
    cm.digest(rem_commit);
    P.vec(cm);
  }
  // BatchMerkleProof bytes of a plan whose node values start at gv[g]: [depth][lists] then per
  // list [len][len digests]; written with its vint length prefix (Vec<u8> of the proof)
  auto mp_len = [](const Plan& plan) {
    size_t n = 2 + plan.len.size();
    for (uint32_t l : plan.len) n += 32 * (size_t)l;
    return n;
  };
  auto emit_multiproof = [&](const Plan& plan, int depth, size_t g) {
    const size_t len = mp_len(plan);
    P.usize(len);
    const size_t o = P.v.size();
    P.v.resize(o + len);
    uint8_t* w = P.v.data() + o;
    *w++ = (uint8_t)depth;
    *w++ = (uint8_t)plan.len.size();
    for (uint32_t l : plan.len) {
      *w++ = (uint8_t)l;
      for (uint32_t k = 0; k < l; k++, w += 32) {  // digest: the 16 value bytes + 16 zero bytes
        memcpy(w, gv + g++, 16);
        memset(w + 16, 0, 16);
      }
    }
  };
  const size_t g_rows = 0, g_crows = nq * W, g_tnodes = nq * ((size_t)W + Cc), g_cnodes = g_tnodes + tplan.node.size();
  P.usize(1);
  P.usize(nq * W * sizeof(fe));  // felem = the 16 LE bytes of the canonical value
  P.raw(gv + g_rows, nq * W * sizeof(fe));
  emit_multiproof(tplan, logN, g_tnodes);
  P.usize(nq * Cc * sizeof(fe));
  P.raw(gv + g_crows, nq * Cc * sizeof(fe));
  emit_multiproof(tplan, logN, g_cnodes);
  gi = g_cnodes + tplan.node.size();
  {
    Bytes ts, es;
    for (auto& v : tz) ts.felem(v);
    for (auto& v : tzg) ts.felem(v);
    for (auto& v : hz) es.felem(v);
    for (auto& v : hzg) es.felem(v);
    P.vec(ts); P.vec(es);
  }
  P.usize((uint64_t)nl);
  for (int d = 0; d < nl; d++) {
    const size_t nv = 2 * fpos[d].size();
    P.usize(nv * sizeof(fe));
    P.raw(gv + gi, nv * sizeof(fe));
    gi += nv;
    emit_multiproof(fplan[d], ilog2((N >> d) / 2), gi);
    gi += fplan[d].node.size();
  }
  {
    Bytes rv;
    for (auto& v : rem) rv.felem(v);
    P.vec(rv);
  }
  P.u8(0);  // FriProof num_partitions (log2 of 1)
  P.u64(nonce);
  if (gi != na_g) throw std::runtime_error("internal: gather plan mismatch");
  HT("serialised");
  T.finish();
  HT("stage_events");
  resolve_kernel_times(C);
  C->proof_s.swap(P.v);
  HT("returned");
  C->host_ms[2] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call0).count();
  {
    float gpu_ms = 0;
    HIPCHECK(hipEventElapsedTime(&gpu_ms, T.ev[0], T.ev[ZKL_NUM_STAGES]));
    C->host_ms[1] = C->host_ms[2] - C->host_ms[0] - gpu_ms;  // host time not overlapped by the stream
  }
}

int run_guarded(zkl_ctx* ctx, const std::function<void()>& f) {
  try {
    f();
    return ZKL_OK;
  } catch (const InvalidArg& e) {
    set_err(ctx, e.what());
    return ZKL_E_INVALID;
  } catch (const std::invalid_argument& e) {
    set_err(ctx, e.what());
    return ZKL_E_INVALID;
  } catch (const DeviceError& e) {
    set_err(ctx, e.what());
    return ZKL_E_DEVICE;
  } catch (const std::bad_alloc&) {
    set_err(ctx, "host allocation failed");
    return ZKL_E_OOM;
  } catch (const std::exception& e) {
    set_err(ctx, e.what());
    return ZKL_E_INTERNAL;
  }
}

}  // namespace

// context-free ABI entry points of other translation units (agg.cpp) report through the same
// thread-local last-error string
int zkl::guarded_call(const std::function<void()>& f) { return run_guarded(nullptr, f); }

// ====================================================================== C ABI
extern "C" {

int zkl_hip_abi_version(void) { return ZKL_ABI_VERSION; }

const char* zkl_hip_build_config(void) {
  static const std::string cfg = std::string(poseidon_build_config()) + ";" + kernels_build_config();
  return cfg.c_str();
}

int zkl_hip_init(int device, zkl_ctx** out) {
  if (!out) return ZKL_E_INVALID;
  *out = nullptr;
  return run_guarded(nullptr, [&] {
    int cnt = 0;
    HIPCHECK(hipGetDeviceCount(&cnt));
    if (device < 0 || device >= cnt) throw InvalidArg("no such HIP device");
    HIPCHECK(hipSetDevice(device));
    auto* c = new zkl_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete c; throw DeviceError(hipGetErrorString(e)); }
    *out = c;
  });
}

// Process-level settings are the embedding application's decision, so zkl_hip_init changes
// nothing outside the library; this call applies them on request (include/zkl_hip.h).
int zkl_hip_process_tuning(uint32_t flags, uint32_t* applied) {
  if (applied) *applied = 0;
  if (flags & ~(uint32_t)(ZKL_TUNE_SPIN | ZKL_TUNE_MALLOC)) return ZKL_E_INVALID;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  uint32_t ok = 0;
  if (flags & ZKL_TUNE_SPIN) {
    // The transcript's host round trips wait on short device tails; a blocking (interrupt) wait
    // there was seen to wake 20-30 ms late on some boxes.  Spin-waiting costs one host core per
    // waiting context.  The flag is per device and only takes effect before the device's primary
    // context exists: every visible device gets it, and it counts as applied only if all took it.
    int cnt = 0, cur = 0;
    bool all = hipGetDeviceCount(&cnt) == hipSuccess && cnt > 0 && hipGetDevice(&cur) == hipSuccess;
    for (int d = 0; all && d < cnt; d++)
      all = hipSetDevice(d) == hipSuccess && hipSetDeviceFlags(hipDeviceScheduleSpin) == hipSuccess;
    if (cnt > 0) (void)hipSetDevice(cur);
    (void)hipGetLastError();
    if (all) ok |= ZKL_TUNE_SPIN;
  }
  if (flags & ZKL_TUNE_MALLOC) {
    // Host memory handed back to the kernel (munmap, heap trim) while a proof runs was followed
    // by 10-30 ms of idle GPU in ~1 proof of 3 in round 4 (profiles/r04/stalls.md).
    // glibc returns memory on free() of blocks above its (dynamic) mmap threshold and when the
    // free heap top exceeds the trim threshold; with these settings the process keeps what it
    // allocated: blocks below 32 MiB come from the heap, the heap grows in 64 MiB steps and is not
    // trimmed until 2 GiB of its top are free.
    if (mallopt(M_MMAP_THRESHOLD, 32 << 20) == 1 && mallopt(M_TOP_PAD, 64 << 20) == 1 &&
        mallopt(M_TRIM_THRESHOLD, 0x7fffffff) == 1)
      ok |= ZKL_TUNE_MALLOC;
  }
  if (applied) *applied = ok;
  return ok == flags ? ZKL_OK : ZKL_E_DEVICE;
}

int zkl_hip_trace_buffer(zkl_ctx* c, uint32_t slot, size_t bytes, zkl_f128** out) {
  if (!c || !out || !bytes || slot >= ZKL_TRACE_BUFFERS) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  *out = nullptr;
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    HBuf& b = c->tbuf[slot];
    if (bytes > b.bytes) {  // exact size: one segment shape is the common case
      HIPCHECK(b.release());
      pin_alloc(&b.p, bytes);
      b.bytes = bytes;
    }
    *out = (zkl_f128*)b.p;
  });
}

int zkl_hip_pinned_bytes(uint64_t* current, uint64_t* peak) {
  if (current) *current = g_pin_cur.load();
  if (peak) *peak = g_pin_peak.load();
  return ZKL_OK;
}

void zkl_hip_destroy(zkl_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamDestroy(c->stream);
  if (c->stage_ev_ready)
    for (auto& e : c->stage_ev) (void)hipEventDestroy(e);
  if (c->up) {
    (void)hipStreamSynchronize(c->up);
    (void)hipStreamDestroy(c->up);
    for (void* p : c->up_slot) (void)pin_free(p, c->up_slot_bytes);
    for (hipEvent_t e : c->up_ev) (void)hipEventDestroy(e);
  }
  if (c->aux) {
    (void)hipStreamSynchronize(c->aux);
    (void)hipStreamDestroy(c->aux);
    (void)hipEventDestroy(c->aux_ev);
    (void)hipEventDestroy(c->hev);
  }
  delete c;
}

const char* zkl_hip_last_error(const zkl_ctx* c) { return c ? c->err.c_str() : g_global_err; }

void zkl_hip_free(uint8_t* p) { free(p); }

static int finish_proof(std::vector<uint8_t>& v, uint8_t** out, size_t* len) {
  uint8_t* b = (uint8_t*)malloc(v.size());
  if (!b) return ZKL_E_OOM;
  memcpy(b, v.data(), v.size());
  *out = b;
  *len = v.size();
  return ZKL_OK;
}

int zkl_hip_prove_segment(zkl_ctx* c, const zkl_f128* trace, uint32_t width, uint32_t n, const zkl_air_public_inputs* pi,
                          const zkl_proof_options* o, uint8_t** proof, size_t* len) {
  if (!c || !trace || !pi || !o || !proof || !len) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  c->proof_s.clear();
  int rc = run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    prove_impl(c, trace, true, width, n, *pi, *o);
  });
  return rc ? rc : finish_proof(c->proof_s, proof, len);
}

int zkl_hip_prove_segment_device(zkl_ctx* c, const void* d_trace, uint32_t width, uint32_t n,
                                 const zkl_air_public_inputs* pi, const zkl_proof_options* o, uint8_t** proof,
                                 size_t* len) {
  if (!c || !d_trace || !pi || !o || !proof || !len) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  c->proof_s.clear();
  int rc = run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    prove_impl(c, d_trace, false, width, n, *pi, *o);
  });
  return rc ? rc : finish_proof(c->proof_s, proof, len);
}

// copy of the context's last proof into caller memory (no allocation); caller holds c->mu
static int copy_last_proof(zkl_ctx* c, uint8_t* buf, size_t cap, size_t* len) {
  *len = c->proof_s.size();
  if (c->proof_s.empty()) {
    c->err = "no proof on this context (the last prove call failed or none was made)";
    return ZKL_E_INVALID;
  }
  if (!buf) return ZKL_OK;  // size query
  if (cap < c->proof_s.size()) {
    c->err = "proof buffer too small: " + std::to_string(c->proof_s.size()) + " bytes needed, " +
             std::to_string(cap) + " given (zkl_hip_last_proof still returns it)";
    return ZKL_E_INVALID;
  }
  memcpy(buf, c->proof_s.data(), c->proof_s.size());
  return ZKL_OK;
}

int zkl_hip_last_proof(zkl_ctx* c, uint8_t* buf, size_t cap, size_t* len) {
  if (!c || !len) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  return copy_last_proof(c, buf, cap, len);
}

int zkl_hip_prove_segment_device_into(zkl_ctx* c, const void* d_trace, uint32_t width, uint32_t n,
                                      const zkl_air_public_inputs* pi, const zkl_proof_options* o, uint8_t* buf,
                                      size_t cap, size_t* len) {
  if (!c || !d_trace || !pi || !o || !len) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  c->proof_s.clear();
  int rc = run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    prove_impl(c, d_trace, false, width, n, *pi, *o);
  });
  return rc ? rc : copy_last_proof(c, buf, cap, len);
}

int zkl_hip_check_request(uint32_t width, uint32_t n_rows, const zkl_air_public_inputs* pi,
                          const zkl_proof_options* o) {
  if (!pi || !o) return ZKL_E_INVALID;
  return run_guarded(nullptr, [&] {
    validate_request(width, n_rows, *pi, *o);
    AirInstance air;
    std::string e = build_air(*pi, width, n_rows, air);
    if (e.empty() && o->blowup_factor < (uint32_t)air.ce_blowup) e = "blowup factor below constraint-evaluation blowup";
    if (!e.empty()) throw InvalidArg(e);
  });
}

int zkl_verify_segment(const uint8_t* proof, size_t len, const zkl_air_public_inputs* pi,
                       const zkl_proof_options* opts) {
  if (!proof || !pi || !opts) return ZKL_E_INVALID;
  return run_guarded(nullptr, [&] {
    const std::string e = verify_segment(proof, len, *pi, *opts, nullptr);
    if (!e.empty()) throw InvalidArg(e);
  });
}

int zkl_hip_host_times(const zkl_ctx* c, double* out_ms, int max_n) {
  if (!c || !out_ms) return ZKL_E_INVALID;
  const double v[4] = {c->host_ms[0], c->host_ms[1], c->host_ms[2], c->up_ms};
  const int k = std::min(max_n, 4);
  for (int i = 0; i < k; i++) out_ms[i] = v[i];
  return k;
}

int zkl_hip_stage_times(const zkl_ctx* c, double* out, int max_n) {
  if (!c || !out) return 0;
  int k = std::min(max_n, ZKL_NUM_STAGES);
  for (int i = 0; i < k; i++) out[i] = c->stage_ms[i];
  return k;
}

int zkl_hip_kernel_times(const zkl_ctx* c, double* out, int* launches, int max_n, const char** names) {
  if (names) *names = kFamilyNames;
  if (!c) return 0;
  int k = std::min(max_n, ZKL_NUM_KFAMILIES);
  for (int i = 0; i < k; i++) {
    if (out) out[i] = c->kfam_ms[i];
    if (launches) launches[i] = c->kfam_n[i];
  }
  return k;
}

int zkl_hip_set_kernel_timing(zkl_ctx* c, int mode) {
  if (!c || mode < 0 || mode > 2) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  c->ktiming = mode;
  return 0;
}

int zkl_step_proof_encode(const zkl_air_public_inputs* pi, const zkl_step_info* info, const uint8_t* inner,
                          size_t inner_len, uint8_t** out, size_t* out_len) {
  if (!pi || !info || !inner || !out || !out_len) return ZKL_E_INVALID;
  std::vector<uint8_t> v;
  int rc = run_guarded(nullptr, [&] { v = step_encode(*pi, *info, inner, inner_len); });
  if (rc) return rc;
  return finish_proof(v, out, out_len);
}

int zkl_children_root(const uint8_t suite_id[32], const uint8_t* digests, const uint8_t* root_traces, uint32_t n,
                      uint8_t root_out[32]) {
  if (!suite_id || !root_out || (n && (!digests || !root_traces))) return ZKL_E_INVALID;
  return run_guarded(nullptr, [&] { children_root(suite_id, digests, root_traces, n, root_out); });
}

int zkl_step_proof_digest(const uint8_t* step, size_t len, uint8_t digest_out[32], uint8_t root_trace_out[32]) {
  if (!step) return ZKL_E_INVALID;
  return run_guarded(nullptr, [&] { step_digest(step, len, digest_out, root_trace_out); });
}

int zkl_hip_device_count(int* count) {
  if (!count) return ZKL_E_INVALID;
  return run_guarded(nullptr, [&] { HIPCHECK(hipGetDeviceCount(count)); });
}

int zkl_hip_device_alloc(zkl_ctx* c, size_t bytes, void** d) {
  if (!c || !d) return ZKL_E_INVALID;
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    hipError_t e = hipMalloc(d, bytes);
    if (e == hipErrorOutOfMemory) throw std::bad_alloc();
    HIPCHECK(e);
  });
}

int zkl_hip_device_free(zkl_ctx* c, void* d) {
  if (!c) return ZKL_E_INVALID;
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    HIPCHECK(hipFree(d));
  });
}

int zkl_hip_memcpy(zkl_ctx* c, void* dst, const void* src, size_t bytes, int kind) {
  if (!c || kind < 1 || kind > 3) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    HIPCHECK(hipMemcpyAsync(dst, src, bytes, k, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
  });
}

int zkl_hip_synchronize(zkl_ctx* c) {
  if (!c) return ZKL_E_INVALID;
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    HIPCHECK(hipStreamSynchronize(c->stream));
    HIPCHECK(hipDeviceSynchronize());
  });
}

void zkl_select_partitions(uint32_t w, uint32_t len, uint32_t* parts, uint32_t* rate) {
  if (rate) *rate = w <= 32 ? 8 : 16;
  if (parts) *parts = len >= (1u << 20) ? 16 : len >= (1u << 18) ? 8 : len >= (1u << 16) ? 4 : len >= (1u << 14) ? 2 : 1;
}

int zkl_hip_hash_rows(zkl_ctx* c, const void* d_m, uint32_t nc, uint32_t nr, uint32_t np, uint32_t rate, void* d_out) {
  if (!c || !d_m || !d_out || nc == 0 || np < 1 || np > 16 || rate < 1 || rate > 256) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    upload_hasher(c->stream);
    c->parts.ensure((size_t)std::max<uint32_t>(np, 1) * nr * sizeof(fe) + 16);
    launch_hash_rows((const fe*)d_m, nc, nr, np, rate, c->parts.f(), (fe*)d_out, c->stream);
    check_launch("stage entry point");
    HIPCHECK(hipStreamSynchronize(c->stream));
  });
}

int zkl_hip_set_ntt_mode(int mode) {
  if (mode < 0 || mode > 1) return ZKL_E_INVALID;
  if (g_proofs_in_flight.load() != 0) {  // every pass of a proof must see one kernel form
    set_err(nullptr, "the NTT mode cannot change while a proof is in flight");
    return ZKL_E_INVALID;
  }
  set_ntt_lazy(mode != 0);
  return 0;
}

int zkl_hip_set_row_digest_rule(int rule) {
  if (rule < 0 || rule > 1) return ZKL_E_INVALID;
  if (g_proofs_in_flight.load() != 0) {
    set_err(nullptr, "the row-digest rule cannot change while a proof is in flight");
    return ZKL_E_INVALID;
  }
  set_row_digest_rule(rule);
  return 0;
}

int zkl_hip_row_digest_rule(void) { return row_digest_rule(); }

int zkl_hip_set_hash_policy(int engine, uint32_t pm_min_items) {
  if (engine < 0 || engine > 1) return ZKL_E_INVALID;
  set_hash_policy(engine, pm_min_items);
  return 0;
}

int zkl_hip_poseidon_permute(zkl_ctx* c, void* d_states, uint32_t n_states, int engine) {
  if (!c || !d_states || engine < 0 || engine > 2) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    upload_hasher(c->stream);
    launch_permute((fe*)d_states, n_states, engine, c->stream);
    check_launch("stage entry point");
    HIPCHECK(hipStreamSynchronize(c->stream));
  });
}

int zkl_hip_merkle_tree(zkl_ctx* c, const void* d_leaves, uint32_t n, void* d_nodes) {
  if (!c || n < 2 || (n & (n - 1))) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    upload_hasher(c->stream);
    HIPCHECK(hipMemcpyAsync((fe*)d_nodes + n, d_leaves, (size_t)n * sizeof(fe), hipMemcpyDeviceToDevice, c->stream));
    HIPCHECK(hipMemsetAsync(d_nodes, 0, sizeof(fe), c->stream));
    launch_merkle((fe*)d_nodes, n, c->stream);
    check_launch("stage entry point");
    HIPCHECK(hipStreamSynchronize(c->stream));
  });
}

int zkl_hip_ntt(zkl_ctx* c, void* d_data, uint32_t nc, uint32_t n, int dif, int inverse) {
  if (!c || !d_data || n < 2 || (n & (n - 1))) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    ensure_tables(c, c->tab_n ? c->tab_n : n, std::max<size_t>(n, c->tab_N));
    const MontTab t = mont_tab(inverse ? c->miroots.p : c->mroots.p, c->tab_N);
    launch_ntt_stages((fe*)d_data, nc, n, dif != 0, 0, ilog2(n) - 1, t, c->tab_N, c->stream);
    check_launch("stage entry point");
    HIPCHECK(hipStreamSynchronize(c->stream));
  });
}

int zkl_hip_lde(zkl_ctx* c, const void* d_values, uint32_t nc, uint32_t n, uint32_t blowup, void* d_coeffs,
                void* d_lde) {
  if (!c || n < 2 || (n & (n - 1)) || blowup < 1 || (blowup & (blowup - 1))) return ZKL_E_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  return run_guarded(c, [&] {
    HIPCHECK(hipSetDevice(c->device));
    size_t N = (size_t)n * blowup;
    ensure_tables(c, n, N);
    hipStream_t s = c->stream;
    fe* coef = (fe*)d_coeffs;
    HIPCHECK(hipMemcpyAsync(coef, d_values, (size_t)nc * n * sizeof(fe), hipMemcpyDeviceToDevice, s));
    launch_ntt_stages(coef, nc, n, true, 0, ilog2(n) - 1, mont_tab(c->miroots.p, c->tab_N), c->tab_N, s);
    launch_scale_bitrev(coef, nc, n, c->opow_n.f(), s);
    launch_lde_from_coeffs(coef, nc, n, N, mont_tab(c->mroots.p, c->tab_N), c->tab_N, (fe*)d_lde, s);
    check_launch("stage entry point");
    // return natural-order coefficients: scale n*c (bitrev) by 1/n and un-permute on host side is
    // not needed by callers; convert in place to natural order here
    std::vector<fe> h((size_t)nc * n), r((size_t)nc * n);
    HIPCHECK(hipMemcpyAsync(h.data(), coef, h.size() * sizeof(fe), hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    // coef[bitrev(k)] = c_k * 3^k
    const fe inv3 = fe_inv(fe{3, 0});
    int logn = ilog2(n);
    std::vector<fe> i3k(n);
    i3k[0] = fe_one();
    for (uint32_t k = 1; k < n; k++) i3k[k] = fe_mul(i3k[k - 1], inv3);
    for (uint32_t col = 0; col < nc; col++)
      for (uint32_t j = 0; j < n; j++) {
        const uint32_t k = bitrev_u(j, logn);
        r[(size_t)col * n + k] = fe_mul(h[(size_t)col * n + j], i3k[k]);
      }
    HIPCHECK(hipMemcpyAsync(coef, r.data(), r.size() * sizeof(fe), hipMemcpyHostToDevice, s));
    HIPCHECK(hipStreamSynchronize(s));
  });
}

}  // extern "C"
