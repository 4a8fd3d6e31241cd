// zl1 step proof around an inner segment proof: the ZKLSTP1 encoding of
// StepProof (zk-lisp-proof-winterfell/src/proof/step.rs:79-151), its decoder
// (step.rs:153-493), the zl1 commitment echo root_trace (proof/format.rs:214-238) and the
// step digest (proof/digest.rs:16-68).  Host-only byte work; the inner proof is the
// Proof::to_bytes image written by prover.cpp.
#include <string.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/zkl_hip.h"
#include "field.h"
#include "host_hash.h"
#include "proof_view.h"

namespace zkl {

namespace {

struct Out {
  std::vector<uint8_t> v;
  void raw(const void* p, size_t n) { v.insert(v.end(), (const uint8_t*)p, (const uint8_t*)p + n); }
  void u32(uint32_t x) { for (int i = 0; i < 4; i++) v.push_back((uint8_t)(x >> (8 * i))); }
  void u64(uint64_t x) { for (int i = 0; i < 8; i++) v.push_back((uint8_t)(x >> (8 * i))); }
  void u16(uint16_t x) { v.push_back((uint8_t)x); v.push_back((uint8_t)(x >> 8)); }
  void b32(const uint8_t* b) { raw(b, 32); }
  void fe_fold(fe x) {  // utils::fe_to_bytes_fold (utils.rs:375-381): 16 LE bytes + 16 zero
    u64(x.lo); u64(x.hi);
    for (int i = 0; i < 16; i++) v.push_back(0);
  }
};

struct In {
  const uint8_t* p;
  size_t n, off = 0;
  void need(size_t k, const char* what) {
    if (off + k > n) throw std::invalid_argument(std::string("step proof truncated before ") + what);
  }
  uint32_t u32(const char* what) {
    need(4, what);
    uint32_t x = 0;
    for (int i = 0; i < 4; i++) x |= (uint32_t)p[off + i] << (8 * i);
    off += 4;
    return x;
  }
  uint64_t u64(const char* what) {
    need(8, what);
    uint64_t x = 0;
    for (int i = 0; i < 8; i++) x |= (uint64_t)p[off + i] << (8 * i);
    off += 8;
    return x;
  }
  const uint8_t* take(size_t k, const char* what) {
    need(k, what);
    const uint8_t* r = p + off;
    off += k;
    return r;
  }
};

// Fields of the inner Proof::to_bytes image the wrapper reads: trace length (TraceInfo),
// blowup and queries (ProofOptions), and the Commitments digests (trace root, constraint
// root, FRI layer roots + remainder commitment), in prover.cpp's writer layout.
struct InnerView {
  uint32_t log_n = 0, blowup = 0, queries = 0;
  std::vector<const uint8_t*> digests;  // 32 bytes each
};

uint64_t read_usize(In& r) {  // winter-utils read_usize (vint64)
  const uint8_t first = *r.take(1, "inner proof commitments");
  if (first == 0) return r.u64("inner proof commitments");
  const int len = __builtin_ctz(first) + 1;
  r.off -= 1;
  const uint8_t* b = r.take((size_t)len, "inner proof commitments");
  uint64_t enc = 0;
  for (int i = 0; i < len; i++) enc |= (uint64_t)b[i] << (8 * i);
  return enc >> len;
}

InnerView view_inner(const uint8_t* p, size_t n) {
  In r{p, n};
  InnerView v;
  const uint8_t* ti = r.take(6, "inner proof trace info");
  if (ti[1] || ti[2]) throw std::invalid_argument("inner proof: auxiliary trace segments are not supported");
  v.log_n = ti[3];
  const uint8_t* fb = r.take(1, "inner proof field modulus");
  r.take(fb[0], "inner proof field modulus");
  const uint8_t* po = r.take(10, "inner proof options");
  v.queries = po[0];
  v.blowup = po[1];
  r.take(1, "inner proof num_unique_queries");
  const uint64_t clen = read_usize(r);
  if (clen % 32 || clen < 64) throw std::invalid_argument("invalid Winterfell commitments layout in zl1::Proof");
  const uint8_t* c = r.take((size_t)clen, "inner proof commitments");
  for (uint64_t k = 0; k < clen / 32; k++) v.digests.push_back(c + 32 * k);
  return v;
}

// BLAKE3("zkl/step/root_trace" | suite | trace roots | constraint root | FRI roots)
void root_trace(const uint8_t suite[32], const InnerView& v, uint8_t out[32]) {
  std::vector<uint8_t> m;
  const char* dom = "zkl/step/root_trace";
  m.insert(m.end(), dom, dom + 19);
  m.insert(m.end(), suite, suite + 32);
  for (const uint8_t* d : v.digests) m.insert(m.end(), d, d + 32);
  blake3_hash(m.data(), m.size(), out);
}

// poseidon_hash_two_lanes (poseidon/mod.rs:255-291): state [l, r, 0 x 8, dom0, dom1] under
// the suite of suite_id, 27 rounds of cube + MDS + rc, output lane 0
fe two_lanes(const PoseidonSuite& S, fe l, fe r) {
  fe st[12] = {l, r};
  for (int i = 2; i < 10; i++) st[i] = fe_zero();
  st[10] = S.dom[0];
  st[11] = S.dom[1];
  for (int rd = 0; rd < S.rounds; rd++) {
    fe c[12];
    for (int i = 0; i < 12; i++) c[i] = fe_mul(fe_mul(st[i], st[i]), st[i]);
    for (int i = 0; i < 12; i++) {
      fe acc = fe_zero();
      for (int k = 0; k < 12; k++) acc = fe_add(acc, fe_mul(S.mds[i][k], c[k]));
      st[i] = fe_add(acc, S.rc[rd][i]);
    }
  }
  return st[0];
}

size_t arg_slots(uint32_t tag) { return tag == 2 ? 2 : 1; }  // utils.rs:79-97

}  // namespace

std::vector<uint8_t> step_encode(const zkl_air_public_inputs& pi, const zkl_step_info& s, const uint8_t* inner,
                                 size_t inner_len) {
  if (s.n_main_args > ZKL_MAX_MAIN_SLOTS) throw std::invalid_argument("too many main_args");
  view_inner(inner, inner_len);  // the commitments must parse (format.rs:226-232)
  Out o;
  o.raw("ZKLSTP1", 7);
  o.u32(s.lambda_bits);
  o.b32(s.suite_id);
  o.b32(pi.program_id);
  o.b32(pi.program_commitment);
  o.b32(pi.merkle_root);
  o.u64(pi.feature_mask);
  o.u32(s.n_main_args);
  for (uint32_t i = 0; i < s.n_main_args; i++) {
    const zkl_vm_arg& a = s.main_args[i];
    if (a.tag > 2) throw std::invalid_argument("invalid VmArg tag");
    o.v.push_back((uint8_t)a.tag);
    o.raw(a.bytes, a.tag == 0 ? 8 : a.tag == 1 ? 16 : 32);
  }
  o.u32(pi.vm_usage_mask);
  o.u32(pi.ram_delta_clk_bits);
  for (int i = 0; i < 3; i++) o.fe_fold(fe{pi.rom_acc[i].lo, pi.rom_acc[i].hi});
  o.u32(s.segment_index);
  o.u32(s.segments_total);
  o.b32(s.pc_init);
  o.b32(s.state_in_hash);
  o.b32(s.state_out_hash);
  o.b32(s.ram_gp_unsorted_in);
  o.b32(s.ram_gp_unsorted_out);
  o.b32(s.ram_gp_sorted_in);
  o.b32(s.ram_gp_sorted_out);
  for (int i = 0; i < 3; i++) o.b32(s.rom_s_in[i]);
  for (int i = 0; i < 3; i++) o.b32(s.rom_s_out[i]);
  o.u32((uint32_t)inner_len);
  o.raw(inner, inner_len);
  return o.v;
}

StepDecoded decode_step(const uint8_t* p, size_t n) {
  In r{p, n};
  if (n < 7) throw std::invalid_argument("step proof too short to contain magic header");
  if (std::string((const char*)p, 7) != "ZKLSTP1") throw std::invalid_argument("invalid step proof magic tag");
  r.off = 7;
  StepDecoded D;
  D.lambda_bits = r.u32("lambda_bits");
  memcpy(D.suite, r.take(32, "suite_id bytes"), 32);
  memcpy(D.program_id, r.take(32, "program_id bytes"), 32);
  memcpy(D.program_commitment, r.take(32, "program_commitment bytes"), 32);
  memcpy(D.merkle_root, r.take(32, "merkle_root bytes"), 32);
  D.feature_mask = r.u64("feature_mask");
  const uint32_t nargs = r.u32("main_args length");
  size_t slots = 0;
  for (uint32_t i = 0; i < nargs; i++) {
    const uint8_t tag = *r.take(1, "VmArg tag");
    if (tag > 2) throw std::invalid_argument("invalid VmArg tag in step proof encoding");
    const size_t len = tag == 0 ? 8 : tag == 1 ? 16 : 32;
    zkl_vm_arg a{};
    a.tag = tag;
    memcpy(a.bytes, r.take(len, tag == 0 ? "VmArg::U64" : tag == 1 ? "VmArg::U128" : "VmArg::Bytes32"), len);
    D.main_args.push_back(a);
    slots += arg_slots(tag);
  }
  D.vm_usage_mask = r.u32("vm_usage_mask");
  D.ram_delta_clk_bits = r.u32("ram_delta_clk_bits");
  const uint8_t* ra = r.take(96, "rom_acc bytes");
  for (int i = 0; i < 3; i++) D.rom_acc[i] = be_from_le16(ra + 32 * i);  // fe_from_bytes_fold (utils.rs:386-390)
  D.segment_index = r.u32("segment_index");
  D.segments_total = r.u32("segments_total");
  memcpy(D.pc_init, r.take(32, "pc_init bytes"), 32);
  memcpy(D.bnd, r.take(32 * 12, "state_in_hash bytes"), 32 * 12);  // state in/out, ram gp x4, rom in/out x3
  const uint32_t inner_len = r.u32("inner proof length");
  D.inner = r.take(inner_len, "inner proof bytes");
  D.inner_len = inner_len;
  const InnerView v = view_inner(D.inner, D.inner_len);
  if (D.segments_total <= 1) { D.segment_index = 0; D.segments_total = 1; }  // new_single_segment (step.rs:413-432)
  root_trace(D.suite, v, D.root_trace);

  // StepMeta::from_env (step.rs:516-533): m, rho, q, o = 2, lambda, pi_len (5 + slots + 13
  // elements of AirPublicInputs::to_elements, lib.rs:116-160), v_units = m q
  D.m = 1u << v.log_n;
  D.rho = (uint16_t)v.blowup;
  D.q = (uint16_t)v.queries;
  D.o = 2;
  D.lambda = (uint16_t)(D.lambda_bits > 65535 ? 65535 : D.lambda_bits);
  D.pi_len = (uint32_t)(5 + slots + 13);
  D.v_units = (uint64_t)D.m * D.q;
  Out mb;
  mb.u32(D.m); mb.u16(D.rho); mb.u16(D.q); mb.u16(D.o); mb.u16(D.lambda); mb.u32(D.pi_len); mb.u64(D.v_units);
  Out pb;
  pb.b32(D.program_id);
  pb.b32(D.program_commitment);
  pb.u64(D.feature_mask);
  pb.u32(D.segment_index);
  pb.u32(D.segments_total);
  pb.b32(D.pc_init);
  pb.raw(D.bnd, 32 * 12);

  const PoseidonSuite S = derive_poseidon_suite(D.suite, 27);
  const fe suite_fe = ro_from_parts("zkl/step/digest/suite", {std::vector<uint8_t>(D.suite, D.suite + 32)});
  const fe h_meta = two_lanes(S, ro_from_parts("zkl/step/digest/meta", {mb.v}), fe_zero());
  const fe h_pi = two_lanes(S, ro_from_parts("zkl/step/digest/pi", {pb.v}), fe_zero());
  const fe h_roots = two_lanes(S, fold_bytes32(D.root_trace), fe_zero());
  const fe c0 = two_lanes(S, suite_fe, h_meta);
  const fe c1 = two_lanes(S, c0, h_pi);
  const fe ch = two_lanes(S, c1, h_roots);
  Out d;
  d.fe_fold(ch);
  memcpy(D.digest, d.v.data(), 32);
  return D;
}

void step_digest(const uint8_t* p, size_t n, uint8_t digest[32], uint8_t rt[32]) {
  const StepDecoded D = decode_step(p, n);
  if (rt) memcpy(rt, D.root_trace, 32);
  if (digest) memcpy(digest, D.digest, 32);
}

// agg::child::children_root_from_compact (agg/child.rs:853-895): leaf_i =
// two_lanes(fold(step_digest_i), fold(root_trace_i)) as 32 folded bytes, leaves sorted
// bytewise, then pairwise two_lanes levels (an odd tail pairs with itself); [0; 32] when empty.
void children_root(const uint8_t suite[32], const uint8_t* digests, const uint8_t* roots, size_t n, uint8_t out[32]) {
  for (int i = 0; i < 32; i++) out[i] = 0;
  if (n == 0) return;
  const PoseidonSuite S = derive_poseidon_suite(suite, 27);
  std::vector<std::vector<uint8_t>> items(n);
  for (size_t i = 0; i < n; i++) {
    const fe leaf = two_lanes(S, fold_bytes32(digests + 32 * i), fold_bytes32(roots + 32 * i));
    Out o;
    o.fe_fold(leaf);
    items[i] = o.v;
  }
  std::sort(items.begin(), items.end());  // lexicographic, as [u8; 32]::sort_unstable
  std::vector<fe> layer;
  for (auto& it : items) layer.push_back(fold_bytes32(it.data()));
  while (layer.size() > 1) {
    std::vector<fe> next;
    for (size_t i = 0; i < layer.size(); i += 2)
      next.push_back(two_lanes(S, layer[i], i + 1 < layer.size() ? layer[i + 1] : layer[i]));
    layer.swap(next);
  }
  Out o;
  o.fe_fold(layer[0]);
  for (int i = 0; i < 32; i++) out[i] = o.v[i];
}

}  // namespace zkl
