// Host hashing for the prover.  BLAKE3 per the published spec (blake3 crate 1.8.2,
// Cargo.lock:110-113); Poseidon suite + PoseidonHasher per
// zk-lisp-proof-winterfell/src/poseidon/{mod.rs:56-217,421-440, hasher.rs:57-231}.
#include "host_hash.h"

#include <stdlib.h>
#include <string.h>

#include <array>
#include <mutex>

namespace zkl {

// ----------------------------------------------------------------- BLAKE3
namespace {
const uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                         0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
const int kPerm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
constexpr uint32_t kChunkStart = 1, kChunkEnd = 2, kParent = 4, kRoot = 8;

inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

struct Compressor {
  static void round(uint32_t v[16], const uint32_t m[16]) {
    auto g = [&](int a, int b, int c, int d, uint32_t x, uint32_t y) {
      v[a] += v[b] + x; v[d] = rotr32(v[d] ^ v[a], 16);
      v[c] += v[d];     v[b] = rotr32(v[b] ^ v[c], 12);
      v[a] += v[b] + y; v[d] = rotr32(v[d] ^ v[a], 8);
      v[c] += v[d];     v[b] = rotr32(v[b] ^ v[c], 7);
    };
    g(0, 4, 8, 12, m[0], m[1]); g(1, 5, 9, 13, m[2], m[3]);
    g(2, 6, 10, 14, m[4], m[5]); g(3, 7, 11, 15, m[6], m[7]);
    g(0, 5, 10, 15, m[8], m[9]); g(1, 6, 11, 12, m[10], m[11]);
    g(2, 7, 8, 13, m[12], m[13]); g(3, 4, 9, 14, m[14], m[15]);
  }
  static void run(const uint32_t cv[8], const uint32_t block[16], uint64_t ctr, uint32_t len,
                  uint32_t flags, uint32_t out[16]) {
    uint32_t v[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                      kIV[0], kIV[1], kIV[2], kIV[3], (uint32_t)ctr, (uint32_t)(ctr >> 32), len, flags};
    uint32_t m[16];
    memcpy(m, block, sizeof m);
    for (int r = 0; r < 7; r++) {
      round(v, m);
      uint32_t t[16];
      for (int i = 0; i < 16; i++) t[i] = m[kPerm[i]];
      memcpy(m, t, sizeof m);
    }
    for (int i = 0; i < 8; i++) { out[i] = v[i] ^ v[i + 8]; out[i + 8] = v[i + 8] ^ cv[i]; }
  }
};

struct Node {
  uint32_t cv[8], block[16];
  uint64_t ctr;
  uint32_t len, flags;
  void chaining(uint32_t out[8]) const {
    uint32_t o[16];
    Compressor::run(cv, block, ctr, len, flags, o);
    memcpy(out, o, 32);
  }
};

Node chunk_node(const uint8_t* p, size_t len, uint64_t idx) {
  uint32_t cv[8];
  memcpy(cv, kIV, sizeof cv);
  size_t blocks = len ? (len + 63) / 64 : 1;
  Node nd{};
  for (size_t b = 0; b < blocks; b++) {
    uint8_t buf[64] = {0};
    size_t bl = b + 1 < blocks ? 64 : len - 64 * b;
    memcpy(buf, p + 64 * b, bl);
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = buf[4 * i] | (buf[4 * i + 1] << 8) | (buf[4 * i + 2] << 16) | ((uint32_t)buf[4 * i + 3] << 24);
    uint32_t flags = (b == 0 ? kChunkStart : 0) | (b + 1 == blocks ? kChunkEnd : 0);
    if (b + 1 == blocks) {
      memcpy(nd.cv, cv, 32); memcpy(nd.block, w, 64);
      nd.ctr = idx; nd.len = (uint32_t)bl; nd.flags = flags;
    } else {
      uint32_t o[16];
      Compressor::run(cv, w, idx, 64, flags, o);
      memcpy(cv, o, 32);
    }
  }
  return nd;
}

Node parent_node(const uint32_t l[8], const uint32_t r[8]) {
  Node nd{};
  memcpy(nd.cv, kIV, 32);
  memcpy(nd.block, l, 32);
  memcpy(nd.block + 8, r, 32);
  nd.ctr = 0; nd.len = 64; nd.flags = kParent;
  return nd;
}
}  // namespace

void blake3_hash(const uint8_t* in, size_t len, uint8_t out[32]) {
  std::vector<std::array<uint32_t, 8>> stack;
  size_t chunks = len ? (len + 1023) / 1024 : 1;
  for (size_t c = 0; c + 1 < chunks; c++) {
    std::array<uint32_t, 8> cv;
    chunk_node(in + 1024 * c, 1024, c).chaining(cv.data());
    for (uint64_t tot = c + 1; (tot & 1) == 0; tot >>= 1) {
      Node p = parent_node(stack.back().data(), cv.data());
      stack.pop_back();
      p.chaining(cv.data());
    }
    stack.push_back(cv);
  }
  Node nd = chunk_node(in + 1024 * (chunks - 1), len - 1024 * (chunks - 1), chunks - 1);
  while (!stack.empty()) {
    uint32_t cv[8];
    nd.chaining(cv);
    nd = parent_node(stack.back().data(), cv);
    stack.pop_back();
  }
  uint32_t o[16];
  Compressor::run(nd.cv, nd.block, nd.ctr, nd.len, nd.flags | kRoot, o);
  for (int i = 0; i < 8; i++)
    for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(o[i] >> (8 * b));
}

// ----------------------------------------------------------------- field helpers
static fe le16_raw(const uint8_t b[16]) {
  fe v{0, 0};
  for (int i = 7; i >= 0; i--) v.lo = (v.lo << 8) | b[i];
  for (int i = 15; i >= 8; i--) v.hi = (v.hi << 8) | b[i];
  return v;
}
// n mod p for n < 2^128 (be_from_u128, utils.rs:47-63)
fe be_from_le16(const uint8_t b[16]) {
  fe v = le16_raw(b);
  if (v.hi == P_HI && v.lo >= P_LO) v = fe{v.lo - P_LO, 0};
  return v;
}
fe fold_bytes32(const uint8_t b[32]) { return fold_pair(be_from_le16(b), be_from_le16(b + 16)); }

fe ro_from_parts(const std::string& domain, const std::vector<std::vector<uint8_t>>& parts) {
  std::vector<uint8_t> buf(domain.begin(), domain.end());
  for (auto& p : parts) buf.insert(buf.end(), p.begin(), p.end());
  uint8_t h[32];
  blake3_hash(buf.data(), buf.size(), h);
  return be_from_le16(h);  // BE::from(lo) + BE::from(hi) * 2^64
}

static std::vector<uint8_t> u32le(uint32_t v) {
  return {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
}

static std::vector<fe> cauchy_points(const char* dom, const uint8_t sid[32], int n) {
  std::vector<fe> pts;
  std::vector<uint8_t> s(sid, sid + 32);
  uint32_t ctr = 0;
  while ((int)pts.size() < n) {
    fe c = ro_from_parts(dom, {s, {(uint8_t)pts.size()}, u32le(ctr)});
    bool bad = fe_is_zero(c);
    for (auto& q : pts) bad = bad || fe_eq(q, c);
    if (bad) ctr++;
    else pts.push_back(c);
  }
  return pts;
}

PoseidonSuite derive_poseidon_suite(const uint8_t sid[32], int rounds) {
  PoseidonSuite s{};
  std::vector<uint8_t> sv(sid, sid + 32);
  s.dom[0] = ro_from_parts("zkl/poseidon2/dom/c0", {sv});
  s.dom[1] = ro_from_parts("zkl/poseidon2/dom/c1", {sv});
  auto x = cauchy_points("zkl/poseidon2/mds/x", sid, 12);
  auto y = cauchy_points("zkl/poseidon2/mds/y", sid, 12);
  for (uint32_t adj = 0;; adj++) {  // poseidon/mod.rs:136-172
    bool ok = true;
    for (auto& a : x)
      for (auto& b : y) ok = ok && !fe_is_zero(fe_add(a, b));
    if (ok) break;
    for (int j = 0; j < 12; j++) {
      fe c = ro_from_parts("zkl/poseidon2/mds/y", {sv, {(uint8_t)j}, u32le(adj)});
      y[j] = fe_is_zero(c) ? fe_one() : c;
    }
  }
  for (int i = 0; i < 12; i++)
    for (int j = 0; j < 12; j++) s.mds[i][j] = fe_inv(fe_add(x[i], y[j]));
  s.rounds = rounds;
  for (int r = 0; r < rounds && r < 27; r++)
    for (int l = 0; l < 12; l++) s.rc[r][l] = ro_from_parts("zkl/poseidon2/rc", {sv, {(uint8_t)r}, {(uint8_t)l}});
  return s;
}

void derive_rom_constants(const uint8_t sid[32], fe rc[27][3], fe mds[3][3]) {
  std::vector<uint8_t> sv(sid, sid + 32);
  for (int r = 0; r < 27; r++)
    for (int l = 0; l < 3; l++) rc[r][l] = ro_from_parts("zkl/rom3/rc", {sv, {(uint8_t)r}, {(uint8_t)l}});
  auto x = cauchy_points("zkl/rom3/mds/x", sid, 3);
  auto y = cauchy_points("zkl/rom3/mds/y", sid, 3);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) mds[i][j] = fe_inv(fe_add(x[i], y[j]));
}

static void permute_with(const PoseidonSuite& s, fe st[12]) {
  for (int r = 0; r < s.rounds; r++) {
    fe c[12];
    for (int i = 0; i < 12; i++) c[i] = fe_cube(st[i]);
    for (int i = 0; i < 12; i++) {
      // lazy 256+4-bit accumulation, one reduction per lane
      u128 hi = 0, lo = 0;
      uint64_t ex = 0;
      for (int k = 0; k < 12; k++) {
        u128 ph, pl;
        host_mul_wide(s.mds[i][k], c[k], &ph, &pl);
        lo += pl;
        ph += (lo < pl);
        hi += ph;
        ex += (hi < ph);
      }
      fe t = host_reduce((u128)ex, hi);
      st[i] = fe_add(host_reduce(to128(t), lo), s.rc[r][i]);
    }
  }
}

void program_field_commitment(const uint8_t b32[32], fe out[2]) {
  PoseidonSuite s = derive_poseidon_suite(b32, 27);
  fe st[12] = {};
  st[0] = be_from_le16(b32);
  st[1] = be_from_le16(b32 + 16);
  st[10] = s.dom[0];
  st[11] = s.dom[1];
  permute_with(s, st);
  out[0] = st[0];
  out[1] = st[1];
}

fe domain_fe(const char* domain) {
  uint8_t d[32] = {0};
  size_t l = strlen(domain);
  memcpy(d, domain, l < 32 ? l : 32);
  return fold_bytes32(d);
}

Hasher::Hasher() {
  uint8_t zero[32] = {0};
  suite = derive_poseidon_suite(zero, 27);
  dom_bytes = domain_fe("zkl/winter/hash/bytes");
  dom_merge = domain_fe("zkl/winter/hash/merge");
  dom_many = domain_fe("zkl/winter/hash/merge_many");
  dom_int = domain_fe("zkl/winter/hash/merge_with_int");
  dom_elems = domain_fe("winter/hash/elements");
  // the vector permutation is used only after it reproduces the scalar one on a few states
  const char* env = getenv("ZKL_HOST_IFMA");  // ZKL_HOST_IFMA=0: the scalar permutation (A/B)
  if (ifma_available() && !(env && !strcmp(env, "0"))) {
    IfmaSuite* v = ifma_new();
    ifma_prepare(suite, *v);
    bool same = true;
    for (uint64_t t = 0; t < 4 && same; t++) {
      fe a[12], b[12];
      for (int i = 0; i < 12; i++) a[i] = b[i] = fe{0x9E3779B97F4A7C15ull * (t * 12 + i + 1), t ? ~(uint64_t)i >> t : 0};
      for (int i = 0; i < 12; i++)
        if (a[i].hi == P_HI && a[i].lo >= P_LO) a[i] = b[i] = fe{a[i].lo, 0};
      permute_with(suite, a);
      ifma_permute(*v, b);
      for (int i = 0; i < 12; i++) same = same && a[i].lo == b[i].lo && a[i].hi == b[i].hi;
    }
    if (same) ifma = v;
    else ifma_delete(v);
  }
}

void Hasher::permute(fe st[12]) const {
  if (ifma) ifma_permute(*ifma, st);
  else permute_with(suite, st);
}

fe Hasher::sponge(fe dom_fe, const fe* m, size_t n) const {
  fe st[12] = {};
  st[10] = suite.dom[0];
  st[11] = suite.dom[1];
  st[0] = dom_fe;
  int lane = 1;
  for (size_t i = 0; i < n; i++) {
    st[lane] = fe_add(st[lane], m[i]);
    if (++lane == 10) { permute(st); lane = 0; }
  }
  if (lane) permute(st);
  return st[0];
}
fe Hasher::merge(fe a, fe b) const { fe m[2] = {a, b}; return sponge(dom_merge, m, 2); }
fe Hasher::merge_many(const fe* d, size_t n) const { return n ? sponge(dom_many, d, n) : fe_zero(); }
fe Hasher::merge_with_int(fe s, uint64_t v) const { fe m[2] = {s, fe{v, 0}}; return sponge(dom_int, m, 2); }
fe Hasher::hash_elements(const fe* e, size_t n) const {
  std::vector<fe> m((n + 1) / 2);
  for (size_t j = 0; j < m.size(); j++) m[j] = fold_pair(e[2 * j], 2 * j + 1 < n ? e[2 * j + 1] : fe_zero());
  return sponge(dom_elems, m.data(), m.size());
}

const Hasher& hasher() {
  static Hasher* h = nullptr;
  static std::once_flag once;
  std::call_once(once, [] { h = new Hasher(); });
  return *h;
}

}  // namespace zkl
