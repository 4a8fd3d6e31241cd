// Segment-proof verifier on the host: the checks of winter-verifier
// 0.13.1 for a ZkLispAir proof, which the reference runs as verify_proof (prove.rs:802-941)
// and, for the aggregation, re-runs piecewise over a step proof's transcript (agg/fs.rs:38-245,
// agg/child.rs:905-1023, agg/trace.rs:697-1260).  Order of checks:
//   context / options, commitments, transcript replay (agg/fs.rs:67-237), out-of-domain
//   constraint identity  H(z) = sum_j H_j(z) z^(j n)
//                             = sum_k alpha_k c_k(z) (z - g^(n-1)) / (z^n - 1)
//                               + sum_a beta_a (t_a(z) - v_a) / (z - g^(s_a)),
//   proof of work, query positions, trace / constraint Merkle openings (row digests under
//   the library's row-digest rule), DEEP values at x = 3 w_N^p (agg/trace.rs:1126-1218),
//   every FRI layer opening and fold (agg/trace.rs:697-955, positions agg/child.rs:1072-1100),
//   the remainder and its commitment.
// The transition constraints c_k(z) come from the same air_transition_sum the device
// evaluator uses (air_eval.h); everything else is independent of the prover's code.
#include <string.h>

#include <algorithm>
#include <stdexcept>
#include <thread>

#include "air_eval.h"
#include "air_host.h"
#include "host_hash.h"
#include "kernels.h"
#include "proof_view.h"

namespace zkl {

uint8_t Rd::u8() {
  if (off + 1 > len) { bad = true; return 0; }
  return p[off++];
}
uint64_t Rd::u64() {
  if (off + 8 > len) { bad = true; return 0; }
  uint64_t v;
  memcpy(&v, p + off, 8);
  off += 8;
  return v;
}
uint64_t Rd::usize() {
  if (off >= len) { bad = true; return 0; }
  const uint8_t b0 = p[off];
  if (b0 == 0) { off++; return u64(); }
  const int l = __builtin_ctz(b0) + 1;
  if (off + (size_t)l > len) { bad = true; return 0; }
  uint64_t enc = 0;
  memcpy(&enc, p + off, (size_t)l);
  off += (size_t)l;
  return enc >> l;
}
fe Rd::felem() {
  if (off + 16 > len) { bad = true; return fe_zero(); }
  fe v;
  memcpy(&v.lo, p + off, 8);
  memcpy(&v.hi, p + off + 8, 8);
  off += 16;
  if (v.hi > P_HI || (v.hi == P_HI && v.lo >= P_LO)) bad = true;
  return v;
}
fe Rd::digest() {
  const fe v = felem();
  if (off + 16 > len) { bad = true; return v; }
  for (int i = 0; i < 16; i++) bad |= p[off + (size_t)i] != 0;
  off += 16;
  return v;
}
Rd Rd::vec() {
  Rd s;
  const uint64_t l = usize();
  if (bad || off + l > len) { bad = true; s.bad = true; return s; }
  s.p = p + off;
  s.len = (size_t)l;
  off += (size_t)l;
  return s;
}

bool batch_merkle_root(Rd& r, size_t n_leaves, const std::vector<size_t>& idx, const std::vector<fe>& leaves,
                       fe* root) {
  const Hasher& H = hasher();
  size_t depth = 0;
  while (((size_t)1 << depth) < n_leaves) depth++;
  if (r.u8() != depth) return false;
  const size_t m = r.u8();
  std::vector<std::vector<fe>> lists(m);
  for (size_t k = 0; k < m && !r.bad; k++) {
    const size_t c = r.u8();
    for (size_t j = 0; j < c; j++) lists[k].push_back(r.digest());
  }
  if (r.bad) return false;
  // leaf pairs (even index of each requested leaf), in increasing order
  std::vector<size_t> norm;
  for (size_t i : idx) {
    const size_t b = i & ~(size_t)1;
    if (norm.empty() || norm.back() != b) norm.push_back(b);
  }
  if (norm.size() != m) return false;
  std::vector<size_t> used(m, 0), cur(m), nxt;
  std::vector<fe> cv(m), nv;
  auto pop = [&](size_t k, fe& out) {
    if (used[k] >= lists[k].size()) return false;
    out = lists[k][used[k]++];
    return true;
  };
  for (size_t k = 0; k < m; k++) {
    fe v[2];
    for (int t = 0; t < 2; t++) {
      const size_t j = norm[k] + (size_t)t;
      auto it = std::lower_bound(idx.begin(), idx.end(), j);
      if (it != idx.end() && *it == j) v[t] = leaves[(size_t)(it - idx.begin())];
      else if (!pop(k, v[t])) return false;
    }
    cv[k] = H.merge(v[0], v[1]);
    cur[k] = (norm[k] + n_leaves) >> 1;
  }
  size_t cn = m;
  for (size_t lvl = 1; lvl < depth; lvl++) {
    nxt.clear();
    nv.clear();
    for (size_t i = 0; i < cn; i++) {
      const size_t sib = cur[i] ^ 1;
      fe parent;
      if (i + 1 < cn && cur[i + 1] == sib) {
        parent = H.merge(cv[i], cv[i + 1]);
        i++;
      } else {
        fe s;
        if (!pop(i, s)) return false;
        parent = (cur[i] & 1) ? H.merge(s, cv[i]) : H.merge(cv[i], s);
      }
      nxt.push_back(sib >> 1);
      nv.push_back(parent);
    }
    cn = nxt.size();
    std::copy(nxt.begin(), nxt.end(), cur.begin());
    std::copy(nv.begin(), nv.end(), cv.begin());
  }
  if (cn != 1 || cur[0] != 1) return false;
  for (size_t k = 0; k < m; k++)
    if (used[k] != lists[k].size()) return false;  // every proof node consumed
  *root = cv[0];
  return true;
}

namespace {

struct VCoin {  // DefaultRandomCoin<PoseidonHasher> [WF-recall]
  fe seed;
  uint64_t counter = 0;
  void reseed(fe d) { seed = hasher().merge(seed, d); counter = 0; }
  fe draw() { return hasher().merge_with_int(seed, ++counter); }
};

size_t partition_size(uint32_t np, uint32_t rate, size_t ncols) {
  if (np <= 1) return ncols;
  const size_t a = (ncols + np - 1) / np;
  return std::max<size_t>(a, rate);
}

// row digest of commit_to_rows under a one-chunk rule (0: winterfell, 1: hash_row_poseidon of
// agg/child.rs:1025-1045)
fe row_digest_rule_n(const fe* row, size_t ncols, size_t psize, int rule) {
  const Hasher& H = hasher();
  if (psize == ncols) return H.hash_elements(row, ncols);
  std::vector<fe> d;
  for (size_t s = 0; s < ncols; s += psize) d.push_back(H.hash_elements(row + s, std::min(psize, ncols - s)));
  if (d.size() == 1 && rule == 1) return d[0];
  return H.merge_many(d.data(), d.size());
}
// ... under the library's rule (kernels.h row_digest_rule)
fe row_digest(const fe* row, size_t ncols, size_t psize) {
  return row_digest_rule_n(row, ncols, psize, row_digest_rule());
}

// the root a batch opening reproduces with hash_row_poseidon leaves (SegmentView::*_root_ref);
// `proof` is a copy of the opening's reader taken before it was consumed
fe reference_rule_root(Rd proof, size_t N, const std::vector<size_t>& pos, const std::vector<fe>& rows, size_t ncols,
                       size_t psize, const std::vector<fe>& leaves, fe committed) {
  std::vector<fe> l1(pos.size());
  bool same = true;
  for (size_t k = 0; k < pos.size(); k++) {
    l1[k] = row_digest_rule_n(&rows[k * ncols], ncols, psize, 1);
    same = same && fe_eq(l1[k], leaves[k]);
  }
  if (same) return committed;
  fe root{};
  if (!batch_merkle_root(proof, N, pos, l1, &root)) return committed;  // malformed: rejected by the caller
  return root;
}

int ilog2z(size_t n) { int k = 0; while (((size_t)1 << k) < n) k++; return k; }

fe transition_sum(const AirInstance& air, const std::vector<fe>& cur, const std::vector<fe>& nxt, const fe* per,
                  fe p_last, const fe* alphas) {
  auto c = [&](int i) { return cur[(size_t)i]; };
  auto x = [&](int i) { return nxt[(size_t)i]; };
  const bool pose = air.dev.pose_block != 0, rm = (air.dev.ram_block | air.dev.merkle_block) != 0;
  if (pose && rm) return air_transition_sum<true, true>(air.dev, c, x, per, p_last, alphas);
  if (pose) return air_transition_sum<true, false>(air.dev, c, x, per, p_last, alphas);
  if (rm) return air_transition_sum<false, true>(air.dev, c, x, per, p_last, alphas);
  return air_transition_sum<false, false>(air.dev, c, x, per, p_last, alphas);
}

}  // namespace

std::string check_proof_options(const zkl_proof_options& o) {
  const auto pow2 = [](uint32_t x) { return x && !(x & (x - 1)); };
  if (o.num_queries < 1 || o.num_queries > 255) return "number of queries must be in 1..255";
  if (!pow2(o.blowup_factor) || o.blowup_factor < 2 || o.blowup_factor > 128)
    return "blowup factor must be a power of two in 2..128";
  if (o.grinding_factor > 32) return "grinding factor must be at most 32";
  if (o.field_extension < 1 || o.field_extension > 3) return "unknown field extension";
  if (o.fri_folding_factor != 2) return "FRI folding factor must be 2";
  if (!pow2(o.fri_remainder_max_degree + 1) || o.fri_remainder_max_degree >= o.blowup_factor)
    return "FRI remainder degree must be 2^k - 1 below the blowup factor";
  if (o.num_partitions < 1 || o.num_partitions > 16) return "number of partitions must be in 1..16";
  if (o.hash_rate < 1 || o.hash_rate > 255) return "hash rate must be in 1..255";
  return "";
}

std::string verify_segment(const uint8_t* proof, size_t len, const zkl_air_public_inputs& pi,
                           const zkl_proof_options& opts, SegmentView* out) {
  return verify_segment_ex(proof, len, pi, &opts, out, true);
}

std::string verify_segment_ex(const uint8_t* proof, size_t len, const zkl_air_public_inputs& pi,
                              const zkl_proof_options* want_opts, SegmentView* out, bool check_ood) {
  SegmentView local;
  SegmentView& V = out ? *out : local;
  const Hasher& H = hasher();
  Rd r{proof, len, 0, false};

  // ---- Context (TraceInfo, field modulus, ProofOptions) + num_unique_queries
  const uint32_t W = r.u8();
  if (r.u8() != 0 || r.u8() != 0) return "trace info: auxiliary segments are not supported";
  const unsigned logn = r.u8();
  if (r.u8() != 0 || r.u8() != 0) return "trace info: trace metadata must be empty";
  if (r.u8() != 16) return "context: field element size must be 16";
  if (r.off + 16 > r.len) return "truncated context";
  {
    uint64_t m[2];
    memcpy(m, r.p + r.off, 16);
    if (m[0] != P_LO || m[1] != P_HI) return "field modulus in the context is not f128";
    r.off += 16;
  }
  zkl_proof_options po{};
  po.num_queries = r.u8(); po.blowup_factor = r.u8(); po.grinding_factor = r.u8();
  po.field_extension = r.u8(); po.fri_folding_factor = r.u8(); po.fri_remainder_max_degree = r.u8();
  po.batching_constraints = r.u8(); po.batching_deep = r.u8();
  po.num_partitions = r.u8(); po.hash_rate = r.u8();
  if (want_opts && memcmp(&po, want_opts, sizeof po) != 0)
    return "proof options in the proof differ from the expected options";
  const zkl_proof_options opts = po;
  const size_t nq_proof = r.u8();
  if (r.bad) return "truncated context";
  {
    const std::string e = check_proof_options(opts);  // options decoded from the proof (winterfell reads them so)
    if (!e.empty()) return "proof options: " + e;
  }
  if (logn < 5 || logn > 30) return "trace length out of range";
  if (opts.field_extension != 1 || opts.fri_folding_factor != 2) return "unsupported proof options";
  const size_t n = (size_t)1 << logn, N = n * opts.blowup_factor;
  AirInstance air;
  {
    const std::string e = build_air(pi, W, n, air, check_ood);
    if (!e.empty()) return "AIR construction failed: " + e;
  }
  const int C = air.num_comp_cols;
  const fe g = root_of_unity(logn), wN = root_of_unity(ilog2z(N));
  const size_t rem_max = (size_t)(opts.fri_remainder_max_degree + 1) * opts.blowup_factor;
  int nl = 0;
  for (size_t d = N; d > rem_max; d /= 2) nl++;
  V.width = W; V.n = n; V.lde = N; V.comp_cols = C; V.opts = opts;

  // ---- Commitments
  {
    Rd cm = r.vec();
    V.trace_root = cm.digest();
    V.constraint_root = cm.digest();
    V.fri_roots.resize(nl);
    for (int d = 0; d < nl; d++) V.fri_roots[d] = cm.digest();
    V.remainder_commit = cm.digest();
    if (!cm.done() || r.bad) return "malformed commitments";
  }

  // ---- transcript up to the out-of-domain point
  std::vector<fe> seed = context_elements(W, n, opts);
  {
    const std::vector<fe> pe = pi_elements(pi);
    seed.insert(seed.end(), pe.begin(), pe.end());
  }
  VCoin coin{H.hash_elements(seed.data(), seed.size()), 0};
  coin.reseed(V.trace_root);
  // composition coefficients: draw k = merge_with_int(seed, k), k = 1.. (alphas then betas).
  // They are independent, so the ~2.9e5 of a 2^16-row segment run on host threads.  The
  // replay without the out-of-domain identity needs none of them: a reseed follows, and
  // draws only advance the counter the reseed resets (agg/fs.rs:132-138 skips them too).
  std::vector<fe> alphas, betas;
  if (check_ood) {
    const size_t na = (size_t)air.n_tc, nb = air.assertions.size(), tot = na + nb;
    std::vector<fe> all(tot);
    const fe sd = coin.seed;
    const size_t nt = std::max<size_t>(1, std::min<size_t>(16, std::thread::hardware_concurrency()));
    const size_t chunk = (tot + nt - 1) / nt;
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt && t * chunk < tot; t++)
      th.emplace_back([&, t] {
        for (size_t k = t * chunk; k < std::min(tot, (t + 1) * chunk); k++) all[k] = H.merge_with_int(sd, k + 1);
      });
    for (auto& x : th) x.join();
    alphas.assign(all.begin(), all.begin() + (long)na);
    betas.assign(all.begin() + (long)na, all.end());
  }
  coin.reseed(V.constraint_root);
  V.z = coin.draw();
  const fe z = V.z, zg = fe_mul(z, g);

  // ---- queries / OOD sections
  if (r.usize() != 1) return "trace queries: exactly one main segment expected";
  Rd tq_v = r.vec(), tq_p = r.vec(), cq_v = r.vec(), cq_p = r.vec(), ood_ts = r.vec(), ood_es = r.vec();
  if (r.bad) return "malformed query / OOD sections";
  if (ood_ts.len != 2 * (size_t)W * 16 || ood_es.len != 2 * (size_t)C * 16) return "OOD frame has the wrong shape";
  V.ood_trace_z.resize(W); V.ood_trace_zg.resize(W); V.ood_comp_z.resize(C); V.ood_comp_zg.resize(C);
  for (auto& v : V.ood_trace_z) v = ood_ts.felem();
  for (auto& v : V.ood_trace_zg) v = ood_ts.felem();
  for (auto& v : V.ood_comp_z) v = ood_es.felem();
  for (auto& v : V.ood_comp_zg) v = ood_es.felem();
  if (ood_ts.bad || ood_es.bad) return "non-canonical OOD values";

  // ---- out-of-domain constraint identity
  if (check_ood) {
    std::vector<fe> per = periodic_at(n, z);
    const fe gl = fe_pow64(g, n - 1), zn = fe_pow64(z, n);
    const fe p_last = fe_mul(fe_mul(gl, fe_sub(zn, fe_one())), fe_inv(fe_mul(fe{n, 0}, fe_sub(z, gl))));
    fe t = transition_sum(air, V.ood_trace_z, V.ood_trace_zg, per.data(), p_last, alphas.data());
    t = fe_mul(fe_mul(t, fe_sub(z, gl)), fe_inv(fe_sub(zn, fe_one())));
    // boundary: groups of assertions at one step share the divisor (z - g^step); batch-inverted
    std::vector<fe> num, den;
    for (size_t a = 0; a < air.assertions.size();) {
      size_t e = a;
      fe s = fe_zero();
      for (; e < air.assertions.size() && air.assertions[e].step == air.assertions[a].step; e++)
        s = fe_add(s, fe_mul(betas[e], fe_sub(V.ood_trace_z[air.assertions[e].col], air.assertions[e].value)));
      num.push_back(s);
      den.push_back(fe_sub(z, fe_pow64(g, air.assertions[a].step)));
      a = e;
    }
    std::vector<fe> pre(den.size());
    fe acc = fe_one();
    for (size_t i = 0; i < den.size(); i++) { pre[i] = acc; acc = fe_mul(acc, den[i]); }
    fe inv = fe_inv(acc), b = fe_zero();
    for (size_t i = den.size(); i-- > 0;) {
      b = fe_add(b, fe_mul(num[i], fe_mul(inv, pre[i])));
      inv = fe_mul(inv, den[i]);
    }
    fe h = fe_zero(), zjn = fe_one();
    for (int j = 0; j < C; j++) { h = fe_add(h, fe_mul(V.ood_comp_z[j], zjn)); zjn = fe_mul(zjn, zn); }
    if (!fe_eq(fe_add(t, b), h)) return "out-of-domain constraint identity does not hold";
  }
  {
    std::vector<fe> oc;  // trace(z) | H(z) | trace(zg) | H(zg)  (agg/fs.rs:152-164)
    oc.insert(oc.end(), V.ood_trace_z.begin(), V.ood_trace_z.end());
    oc.insert(oc.end(), V.ood_comp_z.begin(), V.ood_comp_z.end());
    oc.insert(oc.end(), V.ood_trace_zg.begin(), V.ood_trace_zg.end());
    oc.insert(oc.end(), V.ood_comp_zg.begin(), V.ood_comp_zg.end());
    coin.reseed(H.hash_elements(oc.data(), oc.size()));
  }
  V.deep_coeffs.resize((size_t)W + C);
  for (auto& c : V.deep_coeffs) c = coin.draw();
  V.fri_alphas.resize(nl);
  for (int d = 0; d < nl; d++) { coin.reseed(V.fri_roots[d]); V.fri_alphas[d] = coin.draw(); }
  coin.reseed(V.remainder_commit);

  // ---- FRI proof sections, proof of work
  if ((int)r.usize() != nl) return "FRI layer count mismatch";
  std::vector<Rd> fl_v(nl), fl_p(nl);
  for (int d = 0; d < nl; d++) { fl_v[d] = r.vec(); fl_p[d] = r.vec(); }
  Rd remv = r.vec();
  if (r.u8() != 0) return "FRI remainder partitions must be 1";
  V.pow_nonce = r.u64();
  if (!r.done()) return "malformed FRI section or trailing bytes";
  {
    const fe h = H.merge_with_int(coin.seed, V.pow_nonce);
    const unsigned tz = h.lo ? (unsigned)__builtin_ctzll(h.lo) : 64u;
    if (tz < opts.grinding_factor) return "proof-of-work nonce does not meet the grinding factor";
  }

  // ---- query positions: draw_integers(q, N, nonce), sorted, de-duplicated
  coin.seed = H.merge_with_int(coin.seed, V.pow_nonce);
  coin.counter = 0;
  V.positions.clear();
  for (uint32_t k = 0; k < opts.num_queries; k++) V.positions.push_back((size_t)(coin.draw().lo & (N - 1)));
  std::sort(V.positions.begin(), V.positions.end());
  V.positions.erase(std::unique(V.positions.begin(), V.positions.end()), V.positions.end());
  const std::vector<size_t>& pos = V.positions;
  const size_t nq = pos.size();
  if (nq != nq_proof) return "num_unique_queries does not match the drawn positions";

  // ---- trace and constraint openings
  if (tq_v.len != nq * W * 16 || cq_v.len != nq * (size_t)C * 16) return "query value sections have the wrong size";
  V.trace_rows.resize(nq * W);
  V.comp_rows.resize(nq * (size_t)C);
  for (auto& v : V.trace_rows) v = tq_v.felem();
  for (auto& v : V.comp_rows) v = cq_v.felem();
  if (tq_v.bad || cq_v.bad) return "non-canonical query values";
  {
    std::vector<fe> leaves(nq);
    fe root;
    const Rd tq_p0 = tq_p, cq_p0 = cq_p;
    size_t ps = partition_size(opts.num_partitions, opts.hash_rate, W);
    for (size_t k = 0; k < nq; k++) leaves[k] = row_digest(&V.trace_rows[k * W], W, ps);
    if (!batch_merkle_root(tq_p, N, pos, leaves, &root) || !fe_eq(root, V.trace_root) || !tq_p.done())
      return "trace Merkle opening does not reproduce the trace commitment";
    V.trace_root_ref = reference_rule_root(tq_p0, N, pos, V.trace_rows, W, ps, leaves, V.trace_root);
    ps = partition_size(opts.num_partitions, opts.hash_rate, (size_t)C);
    for (size_t k = 0; k < nq; k++) leaves[k] = row_digest(&V.comp_rows[k * C], (size_t)C, ps);
    if (!batch_merkle_root(cq_p, N, pos, leaves, &root) || !fe_eq(root, V.constraint_root) || !cq_p.done())
      return "constraint Merkle opening does not reproduce the constraint commitment";
    V.constraint_root_ref = reference_rule_root(cq_p0, N, pos, V.comp_rows, (size_t)C, ps, leaves, V.constraint_root);
  }

  // ---- DEEP composition at the query positions
  std::vector<fe> evals(nq);
  {
    const std::vector<fe>& gam = V.deep_coeffs;
    fe sz = fe_zero(), szg = fe_zero();
    for (uint32_t c = 0; c < W; c++) {
      sz = fe_add(sz, fe_mul(gam[c], V.ood_trace_z[c]));
      szg = fe_add(szg, fe_mul(gam[c], V.ood_trace_zg[c]));
    }
    for (int j = 0; j < C; j++) {
      sz = fe_add(sz, fe_mul(gam[W + j], V.ood_comp_z[j]));
      szg = fe_add(szg, fe_mul(gam[W + j], V.ood_comp_zg[j]));
    }
    for (size_t k = 0; k < nq; k++) {
      const fe x = fe_mul(fe{3, 0}, fe_pow64(wN, pos[k]));
      fe s = fe_zero();
      for (uint32_t c = 0; c < W; c++) s = fe_add(s, fe_mul(gam[c], V.trace_rows[k * W + c]));
      for (int j = 0; j < C; j++) s = fe_add(s, fe_mul(gam[W + j], V.comp_rows[k * C + j]));
      evals[k] = fe_add(fe_mul(fe_sub(s, sz), fe_inv(fe_sub(x, z))), fe_mul(fe_sub(s, szg), fe_inv(fe_sub(x, zg))));
    }
  }

  // ---- FRI: layer openings, folds, remainder
  std::vector<size_t> fpos = pos;
  size_t Nd = N;
  const fe inv2 = fe_inv(fe{2, 0}), three{3, 0};
  V.fri_positions.assign(nl, {});
  V.fri_values.assign(nl, {});
  for (int d = 0; d < nl; d++) {
    const size_t h = Nd / 2;
    std::vector<size_t>& np = V.fri_positions[d];
    for (size_t p : fpos)
      if (std::find(np.begin(), np.end(), p % h) == np.end()) np.push_back(p % h);
    const size_t m = np.size();
    if (fl_v[d].len != m * 32) return "FRI layer values have the wrong size";
    std::vector<fe>& lv = V.fri_values[d];
    lv.resize(2 * m);
    for (auto& v : lv) v = fl_v[d].felem();
    if (fl_v[d].bad) return "non-canonical FRI layer values";
    for (size_t k = 0; k < fpos.size(); k++) {
      const size_t j = (size_t)(std::find(np.begin(), np.end(), fpos[k] % h) - np.begin());
      if (!fe_eq(lv[2 * j + (fpos[k] >= h ? 1 : 0)], evals[k])) return "FRI layer opening disagrees with the folded values";
    }
    {
      std::vector<size_t> sp(np);
      std::sort(sp.begin(), sp.end());
      std::vector<fe> sl(m);
      for (size_t k = 0; k < m; k++) {
        const size_t j = (size_t)(std::find(np.begin(), np.end(), sp[k]) - np.begin());
        sl[k] = H.hash_elements(&lv[2 * j], 2);
      }
      fe root;
      if (!batch_merkle_root(fl_p[d], h, sp, sl, &root) || !fe_eq(root, V.fri_roots[d]) || !fl_p[d].done())
        return "FRI layer Merkle opening does not reproduce the layer commitment";
    }
    // fold: (v0 + v1)/2 + alpha (v0 - v1) / (2 x0), x0 = 3 w_Nd^y
    const fe gd = root_of_unity(ilog2z(Nd));
    std::vector<fe> next(m);
    for (size_t j = 0; j < m; j++) {
      const fe v0 = lv[2 * j], v1 = lv[2 * j + 1];
      const fe x0 = fe_mul(three, fe_pow64(gd, np[j]));
      next[j] = fe_mul(fe_add(fe_add(v0, v1), fe_mul(V.fri_alphas[d], fe_mul(fe_sub(v0, v1), fe_inv(x0)))), inv2);
    }
    fpos = np;
    evals.swap(next);
    Nd = h;
  }
  const size_t rlen = opts.fri_remainder_max_degree + 1;
  if (remv.len != rlen * 16) return "FRI remainder has the wrong size";
  V.remainder.resize(rlen);
  for (auto& v : V.remainder) v = remv.felem();
  if (remv.bad) return "non-canonical remainder";
  if (!fe_eq(H.hash_elements(V.remainder.data(), rlen), V.remainder_commit)) return "remainder does not match its commitment";
  const fe gr = root_of_unity(ilog2z(Nd));
  for (size_t k = 0; k < fpos.size(); k++) {
    const fe x = fe_mul(three, fe_pow64(gr, fpos[k]));
    fe v = fe_zero(), xp = fe_one();
    for (size_t c = 0; c < rlen; c++) { v = fe_add(v, fe_mul(V.remainder[rlen - 1 - c], xp)); xp = fe_mul(xp, x); }
    if (!fe_eq(v, evals[k])) return "FRI remainder does not match the last layer";
  }
  return "";
}

}  // namespace zkl
