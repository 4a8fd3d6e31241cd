// zkl_hip.hpp — C++17 host mirror of the reference's prover interface for the segment-proof
// path, over the C ABI of zkl_hip.h (header-only; link libzkl_hip.so).
//
// The reference is Rust (zk-lisp-proof-winterfell) and cannot be compiled here, so this header
// restates the part of its API a caller of this path uses, with the same names, argument
// meaning and error behaviour, for C++ hosts and for tests that read like the reference's:
//
//   zkl::ProofOptions            winterfell::ProofOptions::new(q, blowup, grind, None, 2, 1,
//                                Linear, Linear) (prove.rs:963-972) + with_partitions
//                                (prove.rs:1121)
//   zkl::select_partitions_for_trace   utils.rs:394-409
//   zkl::TraceTable              winterfell::TraceTable<BaseElement>, column-major
//   zkl::AirPublicInputs         crate::AirPublicInputs (lib.rs:75-95), flattened
//   zkl::ZkProver                ZkProver::new / prove (prove.rs:105-257): one segment proof,
//                                Proof::to_bytes out (the call at prove.rs:1142)
//   zkl::verify_proof            verify_proof (prove.rs:802-941), one segment
//   zkl::StepProof               proof::step::StepProof::to_bytes / digest (step.rs:79-151,
//                                digest.rs:16-68), step_meta_for (prove.rs:1103-1174),
//                                children_root (agg/child.rs:853-895)
//   zkl::WinterfellBackend       RecursionBackend::prove / verify (lib.rs:295-372): the
//                                aggregation proof and its ZKLRC1 artifact
//   zkl::Error                   prove::Error (prove.rs:51-60): Backend(String) for prover and
//                                device failures, RecursionInvalid for a batch the aggregation
//                                rejects
//   zkl::Program                 build_trace + build_segment_trace_with_state (vm/trace/mod.rs:
//                                279-365) for one segment at a time, without the full trace
//                                (zkl_program_new / zkl_build_segment_trace)
//   zkl::process_tuning          the opt-in process-wide settings (zkl_hip_process_tuning)
//
// Nothing here runs on the GPU by itself: every call goes through libzkl_hip.so.
#ifndef ZKL_HIP_HPP
#define ZKL_HIP_HPP

#include <array>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "zkl_hip.h"

namespace zkl {

using BaseElement = zkl_f128;  // canonical f128, {lo, hi}
using Digest = std::array<uint8_t, 32>;

// prove::Error (prove.rs:51-60)
class Error : public std::runtime_error {
 public:
  enum class Kind { Backend, RecursionInvalid };
  Error(Kind k, int code, const std::string& msg)
      : std::runtime_error(std::string(k == Kind::Backend ? "backend error: " : "recursion invalid input: ") + msg),
        kind_(k), code_(code) {}
  Kind kind() const { return kind_; }
  int code() const { return code_; }  // ZKL_E_*

 private:
  Kind kind_;
  int code_;
};

namespace detail {
inline std::string last_error(const zkl_ctx* ctx) {
  const char* m = zkl_hip_last_error(ctx);
  return m ? std::string(m) : std::string("unknown error");
}
inline void check(int rc, const zkl_ctx* ctx = nullptr, Error::Kind k = Error::Kind::Backend) {
  if (rc != ZKL_OK) throw Error(k, rc, last_error(ctx));
}
// takes ownership of a library buffer (zkl_hip_free)
inline std::vector<uint8_t> take(uint8_t* p, size_t n) {
  std::vector<uint8_t> v(p, p + n);
  zkl_hip_free(p);
  return v;
}
}  // namespace detail

// utils::select_partitions_for_trace (utils.rs:394-409): (num_partitions, hash_rate)
inline std::pair<uint32_t, uint32_t> select_partitions_for_trace(uint32_t trace_width, uint32_t trace_length) {
  uint32_t parts = 0, rate = 0;
  zkl_select_partitions(trace_width, trace_length, &parts, &rate);
  return {parts, rate};
}

// winterfell::ProofOptions as prove_program builds it (prove.rs:963-972): FieldExtension::None,
// FRI folding 2, remainder max degree 1, Linear batching; partitions via with_partitions.
class ProofOptions {
 public:
  ProofOptions(uint32_t num_queries, uint32_t blowup_factor, uint32_t grinding_factor) {
    std::memset(&o_, 0, sizeof o_);
    o_.num_queries = num_queries;
    o_.blowup_factor = blowup_factor;
    o_.grinding_factor = grinding_factor;
    o_.field_extension = 1;  // None
    o_.fri_folding_factor = 2;
    o_.fri_remainder_max_degree = 1;
    o_.batching_constraints = 0;  // Linear
    o_.batching_deep = 0;
    o_.num_partitions = 1;
    o_.hash_rate = 1;
  }
  // ProofOptions::with_partitions(num_partitions, hash_rate)
  ProofOptions with_partitions(uint32_t num_partitions, uint32_t hash_rate) const {
    ProofOptions p = *this;
    p.o_.num_partitions = num_partitions;
    p.o_.hash_rate = hash_rate;
    return p;
  }
  // the options prove_segment uses for a width x length trace (prove.rs:1115-1121)
  ProofOptions for_trace(uint32_t width, uint32_t length) const {
    const auto pr = select_partitions_for_trace(width, length);
    return with_partitions(pr.first, pr.second);
  }
  uint32_t num_queries() const { return o_.num_queries; }
  uint32_t blowup_factor() const { return o_.blowup_factor; }
  uint32_t grinding_factor() const { return o_.grinding_factor; }
  uint32_t num_partitions() const { return o_.num_partitions; }
  uint32_t hash_rate() const { return o_.hash_rate; }
  const zkl_proof_options& raw() const { return o_; }

 private:
  zkl_proof_options o_;
};

// crate::AirPublicInputs (lib.rs:75-95) in the C ABI's flattened form
struct AirPublicInputs : zkl_air_public_inputs {
  AirPublicInputs() { std::memset(static_cast<zkl_air_public_inputs*>(this), 0, sizeof(zkl_air_public_inputs)); }
  explicit AirPublicInputs(const zkl_air_public_inputs& p) : zkl_air_public_inputs(p) {}
};

// winterfell::TraceTable<BaseElement>: width columns of `length` rows, column-major
class TraceTable {
 public:
  TraceTable(uint32_t width, uint32_t length) : w_(width), n_(length), d_((size_t)width * length, BaseElement{0, 0}) {}
  uint32_t width() const { return w_; }
  uint32_t length() const { return n_; }
  BaseElement get(uint32_t col, uint32_t row) const { return d_[(size_t)col * n_ + row]; }
  void set(uint32_t col, uint32_t row, BaseElement v) { d_[(size_t)col * n_ + row] = v; }
  BaseElement* data() { return d_.data(); }
  const BaseElement* data() const { return d_.data(); }

 private:
  uint32_t w_, n_;
  std::vector<BaseElement> d_;
};

// One device context (streams, buffers, tables); the reference's rayon pool calls prove_segment
// from several threads: use one Device per thread and device (calls on one Device serialise).
class Device {
 public:
  explicit Device(int device = 0) { detail::check(zkl_hip_init(device, &ctx_)); }
  ~Device() { if (ctx_) zkl_hip_destroy(ctx_); }
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;
  Device(Device&& o) noexcept : ctx_(o.ctx_) { o.ctx_ = nullptr; }
  zkl_ctx* ctx() const { return ctx_; }
  // pinned host trace buffer `slot` (0 / 1) of this device context, at least `bytes`: fill it (e.g.
  // Program::build_segment_into) and prove it with ZkProver::prove_host -- no staging copy
  BaseElement* trace_buffer(uint32_t slot, size_t bytes) {
    zkl_f128* p = nullptr;
    detail::check(zkl_hip_trace_buffer(ctx_, slot, bytes, &p), ctx_);
    return p;
  }
  static int count() {
    int n = 0;
    detail::check(zkl_hip_device_count(&n));
    return n;
  }

 private:
  zkl_ctx* ctx_ = nullptr;
};

// winterfell::Proof as bytes (Proof::to_bytes / from_bytes is the boundary, prove.rs:1142-1144)
struct Proof {
  std::vector<uint8_t> bytes;
  const std::vector<uint8_t>& to_bytes() const { return bytes; }
};

// The request checks prove runs before any device work (options bounds, trace shape, public
// inputs); throws Error::Backend with the prover's message.  Needs no device.
inline void check_request(uint32_t width, uint32_t length, const AirPublicInputs& pi, const ProofOptions& opts) {
  detail::check(zkl_hip_check_request(width, length, &pi, &opts.raw()));
}

// ZkProver (prove.rs:105-257): ZkProver::new(options, pub_inputs, rom_acc) + prove(trace).  The
// rom_acc the reference passes separately travels in AirPublicInputs::rom_acc here.
class ZkProver {
 public:
  ZkProver(ProofOptions options, AirPublicInputs pub_inputs, Device& device)
      : opts_(std::move(options)), pi_(pub_inputs), dev_(&device) {}
  // prove(trace) -> Proof (the call at prove.rs:1142), trace in host memory
  Proof prove(const TraceTable& trace) const {
    uint8_t* out = nullptr;
    size_t len = 0;
    detail::check(zkl_hip_prove_segment(dev_->ctx(), trace.data(), trace.width(), trace.length(), &pi_, &opts_.raw(),
                                        &out, &len),
                  dev_->ctx());
    return Proof{detail::take(out, len)};
  }
  // same with a host trace given as a pointer (e.g. one of the Device's pinned trace buffers)
  Proof prove_host(const BaseElement* trace, uint32_t width, uint32_t length) const {
    uint8_t* out = nullptr;
    size_t len = 0;
    detail::check(zkl_hip_prove_segment(dev_->ctx(), trace, width, length, &pi_, &opts_.raw(), &out, &len),
                  dev_->ctx());
    return Proof{detail::take(out, len)};
  }
  // same with the trace already resident in HBM (device pointer on this Device)
  Proof prove_device(const void* d_trace, uint32_t width, uint32_t length) const {
    uint8_t* out = nullptr;
    size_t len = 0;
    detail::check(zkl_hip_prove_segment_device(dev_->ctx(), d_trace, width, length, &pi_, &opts_.raw(), &out, &len),
                  dev_->ctx());
    return Proof{detail::take(out, len)};
  }
  // same, the bytes written into `out` (resized; its capacity is kept across calls, so a
  // caller proving many segments allocates once): zkl_hip_prove_segment_device_into
  void prove_device_into(const void* d_trace, uint32_t width, uint32_t length, std::vector<uint8_t>& out) const {
    out.resize(out.capacity());
    size_t len = 0;
    const int rc = zkl_hip_prove_segment_device_into(dev_->ctx(), d_trace, width, length, &pi_, &opts_.raw(),
                                                     out.data(), out.size(), &len);
    if (len > out.size()) {  // too small (or empty: a size query): the bytes stay on the context
      out.resize(len);
      detail::check(zkl_hip_last_proof(dev_->ctx(), out.data(), out.size(), &len), dev_->ctx());
    } else {
      detail::check(rc, dev_->ctx());
    }
    out.resize(len);
  }
  const ProofOptions& options() const { return opts_; }

 private:
  ProofOptions opts_;
  AirPublicInputs pi_;
  Device* dev_;
};

// The opt-in process-wide settings (ZKL_TUNE_SPIN | ZKL_TUNE_MALLOC, zkl_hip.h): returns the flags
// that took effect; the spin flag only before the first Device of the process
inline uint32_t process_tuning(uint32_t flags) {
  uint32_t applied = 0;
  (void)zkl_hip_process_tuning(flags, &applied);
  return applied;
}

// A compiled program (builder::Op list) run once, then traced segment by segment
// (prove.rs:1057-1134's input side without the full trace): the segment's trace in its own
// layout, its AirPublicInputs and the VM state hashes at its first and last rows.
class Program {
 public:
  Program(const std::vector<zkl_op>& ops, const Digest& program_id, const Digest& commitment,
          const std::vector<uint64_t>& secret_args = {}, const std::vector<zkl_vm_arg>& main_args = {}) {
    detail::check(zkl_program_new(ops.data(), (uint32_t)ops.size(), program_id.data(), commitment.data(),
                                  secret_args.empty() ? nullptr : secret_args.data(), (uint32_t)secret_args.size(),
                                  main_args.empty() ? nullptr : main_args.data(), (uint32_t)main_args.size(), nullptr,
                                  &p_, &width_, &rows_));
  }
  ~Program() { zkl_program_free(p_); }
  Program(const Program&) = delete;
  Program& operator=(const Program&) = delete;
  uint32_t full_width() const { return width_; }
  uint32_t rows() const { return rows_; }  // 32 * next_pow2(ops)
  uint32_t segment_width(uint32_t r_start, uint32_t r_end) const {
    uint32_t w = 0;
    detail::check(zkl_build_segment_trace(p_, r_start, r_end, nullptr, nullptr, &w, nullptr, nullptr));
    return w;
  }
  struct Segment {
    AirPublicInputs pi;
    uint32_t width = 0;
    Digest state_in{}, state_out{};
  };
  // writes rows [r_start, r_end) into `out` (segment_width x (r_end - r_start), column-major)
  Segment build_segment_into(uint32_t r_start, uint32_t r_end, BaseElement* out) const {
    Segment s;
    detail::check(zkl_build_segment_trace(p_, r_start, r_end, out, &s.pi, &s.width, s.state_in.data(),
                                          s.state_out.data()));
    return s;
  }
  // build_segment_trace_with_state (mod.rs:279-310): (trace, segment info)
  std::pair<TraceTable, Segment> build_segment_trace_with_state(uint32_t r_start, uint32_t r_end) const {
    TraceTable t(segment_width(r_start, r_end), r_end - r_start);
    Segment s = build_segment_into(r_start, r_end, t.data());
    return {std::move(t), s};
  }

 private:
  zkl_program* p_ = nullptr;
  uint32_t width_ = 0, rows_ = 0;
};

// WinterfellSegmentPlanner::plan_segments (segment_planner.rs:93-276): [(r_start, r_end)]
inline std::vector<std::pair<uint32_t, uint32_t>> plan_segments(uint32_t n_ops, uint32_t max_rows) {
  uint32_t k = 0;
  detail::check(zkl_plan_segments(n_ops, max_rows, nullptr, nullptr, 0, &k));
  std::vector<uint32_t> a(k), b(k);
  detail::check(zkl_plan_segments(n_ops, max_rows, a.data(), b.data(), k, &k));
  std::vector<std::pair<uint32_t, uint32_t>> out;
  for (uint32_t i = 0; i < k; i++) out.emplace_back(a[i], b[i]);
  return out;
}

// verify_proof (prove.rs:802-941) for one segment proof; throws Error::Backend naming the first
// failing check
inline void verify_proof(const Proof& proof, const AirPublicInputs& pi, const ProofOptions& opts) {
  detail::check(zkl_verify_segment(proof.bytes.data(), proof.bytes.size(), &pi, &opts.raw()));
}

// zl1 step metadata as prove_segment fills it (prove.rs:1103-1174): suite = program_id
// (prove.rs:985), the boundary bytes fe_to_bytes_fold of the AIR public inputs' pc_init, RAM
// grand products and ROM lanes (SegmentBoundaryBytes, prove.rs:1112), the segment position and
// the VM state hashes of the trace builder.  Typed main args (pi.rs VmArg) go in meta.main_args.
inline zkl_step_info step_meta_for(const AirPublicInputs& pi, uint32_t index, uint32_t total, const Digest& state_in,
                                   const Digest& state_out, uint32_t lambda_bits = 128) {
  zkl_step_info m;
  std::memset(&m, 0, sizeof m);
  std::memcpy(m.suite_id, pi.program_id, 32);
  m.lambda_bits = lambda_bits;
  m.segment_index = index;
  m.segments_total = total;
  auto fold = [](const BaseElement& v, uint8_t out[32]) {  // 16 LE bytes of the value, 16 zero
    for (int i = 0; i < 8; i++) out[i] = (uint8_t)(v.lo >> (8 * i));
    for (int i = 0; i < 8; i++) out[8 + i] = (uint8_t)(v.hi >> (8 * i));
  };
  fold(pi.pc_init, m.pc_init);
  std::memcpy(m.state_in_hash, state_in.data(), 32);
  std::memcpy(m.state_out_hash, state_out.data(), 32);
  fold(pi.ram_gp_unsorted_in, m.ram_gp_unsorted_in);
  fold(pi.ram_gp_unsorted_out, m.ram_gp_unsorted_out);
  fold(pi.ram_gp_sorted_in, m.ram_gp_sorted_in);
  fold(pi.ram_gp_sorted_out, m.ram_gp_sorted_out);
  for (int i = 0; i < 3; i++) {
    fold(pi.rom_s_in[i], m.rom_s_in[i]);
    fold(pi.rom_s_out[i], m.rom_s_out[i]);
  }
  return m;
}

// zl1 step proof (proof/step.rs, proof/format.rs, proof/digest.rs)
struct StepProof {
  std::vector<uint8_t> bytes;  // ZKLSTP1 encoding (StepProof::to_bytes)
  // prove_segment's wrapping of an inner proof (prove.rs:1144-1170)
  static StepProof from_inner(const AirPublicInputs& pi, const zkl_step_info& meta, const Proof& inner) {
    uint8_t* out = nullptr;
    size_t len = 0;
    detail::check(zkl_step_proof_encode(&pi, &meta, inner.bytes.data(), inner.bytes.size(), &out, &len));
    return StepProof{detail::take(out, len)};
  }
  // StepProof::from_bytes validation + (step digest, zl1 root_trace)
  std::pair<Digest, Digest> digest() const {
    Digest d{}, r{};
    detail::check(zkl_step_proof_digest(bytes.data(), bytes.size(), d.data(), r.data()));
    return {d, r};
  }
};

// agg::child::children_root_from_compact (agg/child.rs:853-895)
inline Digest children_root(const Digest& suite_id, const std::vector<Digest>& digests, const std::vector<Digest>& roots) {
  if (digests.size() != roots.size()) throw Error(Error::Kind::RecursionInvalid, ZKL_E_INVALID, "children count mismatch");
  std::vector<uint8_t> d, r;
  for (const auto& x : digests) d.insert(d.end(), x.begin(), x.end());
  for (const auto& x : roots) r.insert(r.end(), x.begin(), x.end());
  Digest out{};
  detail::check(zkl_children_root(suite_id.data(), d.data(), r.data(), (uint32_t)digests.size(), out.data()));
  return out;
}

// zk_lisp_proof::ProverOptions as the aggregation reads it (zk-lisp-proof/src/lib.rs:40-66)
struct ProverOptions {
  uint32_t queries = 64, blowup = 16, grind = 16, min_security_bits = 128;
};

// RecursionBackend for the HIP backend (lib.rs:295-372): prove = build_public + prove_agg_proof
// + RecursionArtifactCodec::encode, verify = decode + verify_agg_proof
struct WinterfellBackend {
  struct Artifact {
    std::vector<uint8_t> bytes;  // ZKLRC1 (proof.bin)
    Digest recursion_digest;
  };
  static Artifact prove(const std::vector<StepProof>& steps, const ProverOptions& opts,
                        uint32_t trace_mode = ZKL_AGG_TRACE_VALID) {
    std::vector<const uint8_t*> ptrs;
    std::vector<size_t> lens;
    for (const auto& s : steps) {
      ptrs.push_back(s.bytes.data());
      lens.push_back(s.bytes.size());
    }
    zkl_agg_options o{opts.queries, opts.blowup, opts.grind, opts.min_security_bits, trace_mode};
    uint8_t* out = nullptr;
    size_t len = 0;
    Artifact a{};
    const int rc = zkl_agg_prove(ptrs.data(), lens.data(), (uint32_t)steps.size(), &o, &out, &len,
                                 a.recursion_digest.data());
    detail::check(rc, nullptr, rc == ZKL_E_INVALID ? Error::Kind::RecursionInvalid : Error::Kind::Backend);
    a.bytes = detail::take(out, len);
    return a;
  }
  static void verify(const std::vector<uint8_t>& artifact, uint32_t min_security_bits) {
    const int rc = zkl_agg_verify(artifact.data(), artifact.size(), min_security_bits);
    detail::check(rc, nullptr, rc == ZKL_E_INVALID ? Error::Kind::RecursionInvalid : Error::Kind::Backend);
  }
};

}  // namespace zkl

#endif  // ZKL_HIP_HPP
