// Tests of the C++ host mirror (include/zkl_hip.hpp), written the way the reference's Rust
// tests use its API (ZkProver::new(..).prove(trace), verify_proof, StepProof, RecursionBackend).
//   host_api_test cpu              checks that need no device
//   host_api_test gpu <proof.bin>  proves a 2^8-row synthetic segment on device 0, verifies it,
//                                  wraps it as a zl1 step, aggregates it and verifies the
//                                  artifact; writes the segment proof bytes for the pytest
//                                  caller to compare with the CPU oracle
// Prints "ok ..." and exits 0 on success; any failure exits 1 with the reason.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "zkl_hip.hpp"

namespace {

int g_fail = 0;
#define EXPECT(c)                                                        \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail = 1;                                                        \
    }                                                                    \
  } while (0)

// the synthetic VM segment generator (workload generator of the C ABI) as a TraceTable
struct Segment {
  zkl::TraceTable trace;
  zkl::AirPublicInputs pi;
};
Segment synth_segment(uint64_t seed, uint32_t log_n) {
  uint32_t w = 0;
  zkl::detail::check(zkl_synth_vm_segment(seed, log_n, nullptr, nullptr, &w));
  Segment s{zkl::TraceTable(w, 1u << log_n), zkl::AirPublicInputs()};
  zkl::detail::check(zkl_synth_vm_segment(seed, log_n, s.trace.data(), &s.pi, &w));
  return s;
}

template <class F>
bool throws_backend(F&& f, const char* needle) {
  try {
    f();
  } catch (const zkl::Error& e) {
    if (e.kind() != zkl::Error::Kind::Backend) return false;
    if (std::string(e.what()).find("backend error: ") != 0) return false;
    return !needle || std::string(e.what()).find(needle) != std::string::npos;
  }
  return false;
}

int run_cpu() {
  // utils::select_partitions_for_trace (utils.rs:394-409)
  EXPECT(zkl::select_partitions_for_trace(204, 1u << 12) == std::make_pair(1u, 16u));
  EXPECT(zkl::select_partitions_for_trace(204, 1u << 16) == std::make_pair(4u, 16u));
  EXPECT(zkl::select_partitions_for_trace(204, 1u << 20) == std::make_pair(16u, 16u));
  EXPECT(zkl::select_partitions_for_trace(31, 16) == std::make_pair(1u, 8u));
  // ProofOptions as prove_program builds them (prove.rs:963-972) + with_partitions
  const zkl::ProofOptions o = zkl::ProofOptions(64, 16, 16).for_trace(204, 1u << 16);
  EXPECT(o.num_queries() == 64 && o.blowup_factor() == 16 && o.grinding_factor() == 16);
  EXPECT(o.num_partitions() == 4 && o.hash_rate() == 16);
  EXPECT(o.raw().field_extension == 1 && o.raw().fri_folding_factor == 2 && o.raw().fri_remainder_max_degree == 1);
  // a generated segment passes the request checks; bad options fail them like ProofOptions::new
  Segment s = synth_segment(0x5EED0001, 6);
  const uint32_t w = s.trace.width(), n = s.trace.length();
  EXPECT(w == 204 && n == 64);
  const zkl::ProofOptions ok = zkl::ProofOptions(8, 16, 0).for_trace(w, n);
  zkl::check_request(w, n, s.pi, ok);
  EXPECT(throws_backend([&] { zkl::check_request(w, n, s.pi, zkl::ProofOptions(8, 16, 33).for_trace(w, n)); }, "grinding"));
  EXPECT(throws_backend([&] { zkl::check_request(w, n, s.pi, zkl::ProofOptions(8, 256, 0).for_trace(w, n)); }, nullptr));
  EXPECT(throws_backend([&] { zkl::check_request(w, n, s.pi, zkl::ProofOptions(0, 16, 0).for_trace(w, n)); }, nullptr));
  EXPECT(throws_backend([&] { zkl::check_request(w + 1, n, s.pi, ok); }, nullptr));
  // TraceTable is column-major: (col, row) at data[col * length + row]
  EXPECT(s.trace.get(3, 5).lo == s.trace.data()[3 * n + 5].lo);
  // a step proof cannot wrap bytes that are not a proof (the encoder reads the inner proof's
  // trace info, as StepProof::to_bytes does), and garbage is not a step proof
  zkl_step_info meta{};
  std::memcpy(meta.suite_id, s.pi.program_id, 32);
  meta.lambda_bits = 128;
  meta.segments_total = 1;
  EXPECT(throws_backend([&] { (void)zkl::StepProof::from_inner(s.pi, meta, zkl::Proof{{1, 2, 3}}); }, "truncated"));
  EXPECT(throws_backend([&] { (void)zkl::StepProof{{'Z', 'K', 'L'}}.digest(); }, nullptr));
  // a program traced segment by segment (Program) equals the full trace cut by the planner:
  // Const/Add ops over 96 levels -> 128 levels, two segments of 2048 rows
  {
    std::vector<zkl_op> ops;
    for (int i = 0; i < 95; i++) {
      zkl_op a{};
      a.kind = i % 2 ? ZKL_OP_ADD : ZKL_OP_CONST;
      a.dst = (uint8_t)(i % 8);
      a.a = (uint8_t)((i + 1) % 8);
      a.b = (uint8_t)((i + 3) % 8);
      a.imm = 1000u + (uint64_t)i;
      ops.push_back(a);
    }
    zkl_op end{};
    end.kind = ZKL_OP_END;
    ops.push_back(end);
    zkl::Digest pid{};
    pid[0] = 7;
    const zkl::Program prog(ops, pid, pid);
    EXPECT(prog.full_width() == 204 && prog.rows() == 4096);
    const auto plan = zkl::plan_segments((uint32_t)ops.size(), 2048);
    EXPECT(plan.size() == 2 && plan[1].first == 2048);
    std::vector<zkl_f128> full((size_t)prog.full_width() * prog.rows());
    zkl_air_public_inputs fpi{};
    uint32_t fw = 0, fn = 0;
    zkl::detail::check(zkl_build_trace(ops.data(), (uint32_t)ops.size(), pid.data(), pid.data(), nullptr, 0, nullptr, 0,
                                       nullptr, full.data(), &fpi, &fw, &fn));
    for (const auto& seg : plan) {
      const auto got = prog.build_segment_trace_with_state(seg.first, seg.second);
      std::vector<zkl_f128> want((size_t)got.first.width() * got.first.length());
      zkl_air_public_inputs wpi{};
      uint32_t ww = 0;
      zkl::Digest win{}, wout{};
      zkl::detail::check(zkl_slice_segment(full.data(), fw, fn, ops.data(), (uint32_t)ops.size(), &fpi, seg.first,
                                           seg.second, want.data(), &wpi, &ww, win.data(), wout.data()));
      EXPECT(ww == got.first.width() && std::memcmp(want.data(), got.first.data(), want.size() * 16) == 0);
      EXPECT(std::memcmp(&wpi, static_cast<const zkl_air_public_inputs*>(&got.second.pi), sizeof wpi) == 0);
      EXPECT(win == got.second.state_in && wout == got.second.state_out);
    }
    EXPECT(throws_backend([&] { (void)prog.segment_width(16, 48); }, nullptr));
  }
  // no device here: the context fails with Error::Backend, not a crash
  int devs = 0;
  if (zkl_hip_device_count(&devs) != ZKL_OK || devs == 0) EXPECT(throws_backend([] { zkl::Device d(0); }, nullptr));
  if (g_fail) return 1;
  std::printf("ok cpu\n");
  return 0;
}

int run_gpu(const char* out_path) {
  Segment s = synth_segment(0x5EED0001, 8);
  const uint32_t w = s.trace.width(), n = s.trace.length();
  const zkl::ProofOptions opts = zkl::ProofOptions(32, 16, 8).for_trace(w, n);
  zkl::Device dev(0);
  const zkl::ZkProver prover(opts, s.pi, dev);  // ZkProver::new(options, pub_inputs, rom_acc)
  const zkl::Proof proof = prover.prove(s.trace);
  // the same trace from the device's pinned trace buffer (no staging copy) gives the same bytes
  zkl::BaseElement* tb = dev.trace_buffer(1, (size_t)w * n * sizeof(zkl::BaseElement));
  std::memcpy(tb, s.trace.data(), (size_t)w * n * sizeof(zkl::BaseElement));
  EXPECT(prover.prove_host(tb, w, n).bytes == proof.bytes);
  // the trace resident in HBM: prove_device, and prove_device_into with an empty vector (the
  // too-small path through zkl_hip_last_proof) and again with the capacity it kept
  {
    void* d = nullptr;
    const size_t bytes = (size_t)w * n * sizeof(zkl::BaseElement);
    EXPECT(zkl_hip_device_alloc(dev.ctx(), bytes, &d) == ZKL_OK);
    EXPECT(zkl_hip_memcpy(dev.ctx(), d, s.trace.data(), bytes, 1) == ZKL_OK);
    EXPECT(prover.prove_device(d, w, n).bytes == proof.bytes);
    std::vector<uint8_t> out;
    prover.prove_device_into(d, w, n, out);
    EXPECT(out == proof.bytes);
    const size_t cap = out.capacity();
    prover.prove_device_into(d, w, n, out);
    EXPECT(out == proof.bytes && out.capacity() == cap);
    EXPECT(zkl_hip_device_free(dev.ctx(), d) == ZKL_OK);
  }
  zkl::verify_proof(proof, s.pi, opts);
  // a corrupted proof is rejected by the verifier with Error::Backend
  zkl::Proof bad = proof;
  bad.bytes[bad.bytes.size() / 2] ^= 1;
  EXPECT(throws_backend([&] { zkl::verify_proof(bad, s.pi, opts); }, nullptr));
  // zl1 step + aggregation of the one-segment program (RecursionBackend::prove / verify)
  zkl::Digest s_in{}, s_out{};
  s_out[0] = 1;
  const zkl_step_info meta = zkl::step_meta_for(s.pi, 0, 1, s_in, s_out);
  const zkl::StepProof step = zkl::StepProof::from_inner(s.pi, meta, proof);
  const auto dr = step.digest();
  zkl::Digest suite{};
  std::memcpy(suite.data(), s.pi.program_id, 32);
  const zkl::Digest root = zkl::children_root(suite, {dr.first}, {dr.second});
  zkl::ProverOptions po;
  po.grind = 8;
  const auto art = zkl::WinterfellBackend::prove({step}, po);
  zkl::WinterfellBackend::verify(art.bytes, 128);
  FILE* f = std::fopen(out_path, "wb");
  if (!f || std::fwrite(proof.bytes.data(), 1, proof.bytes.size(), f) != proof.bytes.size()) {
    std::fprintf(stderr, "cannot write %s\n", out_path);
    return 1;
  }
  std::fclose(f);
  if (g_fail) return 1;
  std::printf("ok gpu proof %zu bytes, artifact %zu bytes, children root %02x%02x..\n", proof.bytes.size(),
              art.bytes.size(), root[0], root[1]);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  try {
    if (mode == "cpu") return run_cpu();
    if (mode == "gpu" && argc > 2) return run_gpu(argv[2]);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "FAILED: %s\n", e.what());
    return 1;
  }
  std::fprintf(stderr, "usage: host_api_test cpu | gpu <proof.bin>\n");
  return 2;
}
