// Host pieces shared by the segment prover (prover.cpp) and the aggregation prover (agg.cpp):
// the Fiat-Shamir coin, the winter-utils byte writer and the MerkleTree::prove_batch index
// plan.  All three follow winterfell 0.13.1 [WF-recall]; the transcript order they serve is
// pinned by agg/fs.rs:67-237.
#pragma once
#include <string.h>

#include <algorithm>
#include <memory>
#include <stdexcept>
#include <vector>

#include "field.h"
#include "host_hash.h"

namespace zkl {

inline int ilog2(size_t n) { int k = 0; while (((size_t)1 << k) < n) k++; return k; }

// DefaultRandomCoin<PoseidonHasher>: draw = merge_with_int(seed, ++counter) (a Poseidon
// digest value is canonical, so the first try is always accepted)
struct Coin {
  fe seed;
  uint64_t counter = 0;
  void reseed(fe d) { seed = hasher().merge(seed, d); counter = 0; }
  fe draw() { return hasher().merge_with_int(seed, ++counter); }
};

// winter-utils ByteWriter
struct Bytes {
  std::vector<uint8_t> v;
  void u8(uint8_t x) { v.push_back(x); }
  void raw(const void* p, size_t n) {
    const size_t o = v.size();
    v.resize(o + n);
    memcpy(v.data() + o, p, n);
  }
  void u16(uint16_t x) { raw(&x, 2); }  // little-endian host (x86-64 / gfx950 hosts)
  void u32(uint32_t x) { raw(&x, 4); }
  void u64(uint64_t x) { raw(&x, 8); }
  void usize(uint64_t x) {  // winter-utils write_usize (vint64)
    int lz = x ? __builtin_clzll(x) : 64;
    int l = (lz > 0 ? lz - 1 : 0) / 7;
    int len = 9 - std::min(l, 8);
    if (len == 9) { u8(0); u64(x); return; }
    uint64_t enc = ((x << 1) | 1) << (len - 1);
    raw(&enc, (size_t)len);
  }
  void felem(fe x) {
    const uint64_t w[2] = {x.lo, x.hi};
    raw(w, 16);
  }
  void digest(fe x) {
    const uint64_t w[4] = {x.lo, x.hi, 0, 0};
    raw(w, 32);
  }
  void vec(const Bytes& b) { usize(b.v.size()); raw(b.v.data(), b.v.size()); }
};

// MerkleTree::prove_batch node-index plan: per normalized leaf pair, the tree-node indices
// whose digests go into the BatchMerkleProof (leaves are tree nodes n + i)
struct Plan {
  std::vector<uint64_t> node;  // the lists back to back
  std::vector<uint32_t> len;   // entries per list
};
// plan of idx[0..Q) into P (its vectors keep their capacity across calls: no allocation in the
// steady state).  Q <= 256 (ProofOptions' num_queries is a byte).
inline void batch_plan_into(size_t n_leaves, const size_t* idx, size_t Q, Plan& P) {
  if (Q > 256) throw std::invalid_argument("batch_plan: more than 256 query positions");
  const int depth = ilog2(n_leaves);
  // normalised leaf pairs (sorted, unique) and the requested leaves (sorted)
  size_t norm[256], req[256], cur[256], nxt[256];
  uint32_t cnt[256];
  for (size_t k = 0; k < Q; k++) { norm[k] = idx[k] & ~(size_t)1; req[k] = idx[k]; }
  std::sort(norm, norm + Q);
  const size_t L = (size_t)(std::unique(norm, norm + Q) - norm);
  std::sort(req, req + Q);
  // list k takes at most two leaves and one node per level: fixed-stride scratch, compacted
  const size_t stride = (size_t)depth + 2;
  P.node.resize(L * stride);
  uint64_t* tmp = P.node.data();
  size_t r = 0;  // req and norm are both ascending: one merge pass finds the requested leaves
  for (size_t k = 0; k < L; k++) {
    cnt[k] = 0;
    for (size_t j = norm[k]; j < norm[k] + 2; j++) {
      while (r < Q && req[r] < j) r++;
      if (!(r < Q && req[r] == j)) tmp[k * stride + cnt[k]++] = n_leaves + j;
    }
    cur[k] = (norm[k] + n_leaves) >> 1;
  }
  size_t nc = L;
  size_t *a = cur, *b = nxt;
  for (int lvl = 1; lvl < depth; lvl++) {
    size_t nn = 0;
    for (size_t i = 0; i < nc; i++) {
      const size_t sib = a[i] ^ 1;
      if (i + 1 < nc && a[i + 1] == sib) i++;
      else tmp[i * stride + cnt[i]++] = sib;
      b[nn++] = sib >> 1;
    }
    std::swap(a, b);
    nc = nn;
  }
  // compact the lists in place (list k starts at or after where it is moved to)
  P.len.assign(cnt, cnt + L);
  size_t o = 0;
  for (size_t k = 0; k < L; k++) {
    memmove(tmp + o, tmp + k * stride, cnt[k] * sizeof(uint64_t));
    o += cnt[k];
  }
  P.node.resize(o);
}
inline Plan batch_plan(size_t n_leaves, const std::vector<size_t>& idx) {
  Plan P;
  batch_plan_into(n_leaves, idx.data(), idx.size(), P);
  return P;
}

}  // namespace zkl
