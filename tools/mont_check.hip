// Host-side check of the device Montgomery helpers in kernels.hip (REDC, mont_mul,
// mont_cube) against u128 reference arithmetic.  Build: tools/mont_check.sh
#include "../zk-lisp_amd/csrc/kernels.hip"
#include <cstdio>
#include <random>
using namespace zkl;
static fe from26(const uint32_t l[5]) {  // value may exceed p: reduce via u128 mod
  unsigned __int128 v = 0;
  // value < 2^130: accumulate as (hi part) carefully
  unsigned __int128 lo = (unsigned __int128)l[0] + ((unsigned __int128)l[1] << 26) + ((unsigned __int128)l[2] << 52) +
                         ((unsigned __int128)l[3] << 78);
  unsigned __int128 top = (unsigned __int128)l[4];  // * 2^104
  unsigned __int128 P = ((unsigned __int128)P_HI << 64) | P_LO;
  // top * 2^104 mod p
  unsigned __int128 t = top << 24;  // top*2^24 < 2^50
  // (t * 2^80) mod p computed by repeated doubling
  for (int i = 0; i < 80; i++) { t = (t >= P - t) ? t - (P - t) : t + t; }
  lo %= P;
  v = (lo >= P - t) ? lo - (P - t) : lo + t;
  return fe{(uint64_t)v, (uint64_t)(v >> 64)};
}
int main() {
  std::mt19937_64 rng(7);
  fe R = fe_pow64(fe{2, 0}, 156), Rinv = fe_inv(R);
  int bad = 0;
  for (int it = 0; it < 200000; it++) {
    fe a{rng(), rng() >> (it % 3)}, b{rng(), rng() >> (it % 5)};
    if (a.hi == P_HI && a.lo >= P_LO) a.hi--;
    if (b.hi == P_HI && b.lo >= P_LO) b.hi--;
    uint32_t la[5], lb[5], lo[5], lc[5];
    to26(a, la); to26(b, lb);
    if (it & 1) { for (int j = 0; j < 5; j++) { la[j] += (uint32_t)(rng() & 0x3FFFFFF); } }  // lazy limbs < 2^27
    fe av = from26(la);
    mont_mul(la, lb, lo);
    fe got = from26(lo), want = fe_mul(fe_mul(av, b), Rinv);
    unsigned __int128 gv = ((unsigned __int128)0);
    (void)gv;
    bool lim = true;
    for (int j = 0; j < 4; j++) lim &= lo[j] < (1u << 26);
    lim &= lo[4] < (1u << 26);
    if (!fe_eq(got, want) || !lim) { if (bad++ < 5) printf("mul mismatch it=%d\n", it); }
    mont_cube(la, lc);
    fe wantc = fe_mul(fe_mul(fe_mul(av, av), av), fe_mul(Rinv, Rinv));
    if (!fe_eq(from26(lc), wantc)) { if (bad++ < 5) printf("cube mismatch it=%d\n", it); }
  }
  // 12-term accumulated products (MDS shape), max-size limbs
  for (int it = 0; it < 50000; it++) {
    uint64_t col[10] = {0};
    fe acc = fe_zero();
    for (int k = 0; k < 12; k++) {
      uint32_t x[5], y[5];
      for (int j = 0; j < 5; j++) { x[j] = (uint32_t)(rng() & 0x3FFFFFF); y[j] = (uint32_t)(rng() & 0x3FFFFFF); }
      x[4] &= 0x1FFFFFF; y[4] &= 0xFFFFFF;
      if (it == 0) { for (int j = 0; j < 5; j++) { x[j] = 0x3FFFFFF; } x[4] = 0x1FFFFFF; y[0]=y[1]=y[2]=y[3]=0x3FFFFFF; y[4]=0xFFFFFF; }
      mac5(x, y, col);
      acc = fe_add(acc, fe_mul(from26(x), from26(y)));
    }
    uint32_t o[5];
    redc(col, o);
    if (!fe_eq(from26(o), fe_mul(acc, Rinv))) { if (bad++ < 10) printf("mds mismatch it=%d\n", it); }
  }
  // mul_tw (NTT twiddle product): random twiddles, plus the operands seen on device where
  // the REDC result exceeds 2^128 (twiddle w_512^128)
  {
    fe g = root_of_unity(9);
    std::vector<fe> ws = {fe_pow64(g, 128), fe_pow64(g, 384), fe_pow64(g, 1)};
    for (int i = 0; i < 64; i++) ws.push_back(fe{rng(), rng() >> 1});
    std::vector<fe> as = {fe{0x618373d3c785bcbdull, 0x46ca9081269b2944ull}, fe{0x2b3a64ac8a8a20c7ull, 0x4d817dfe6e9ca187ull},
                          fe{0xda9b84022150b7b7ull, 0x6617b8dd37180ea2ull}, fe{0x2018d63f9d60e4ddull, 0x67958cd2ead8edc8ull},
                          fe{0, 0}, fe{1, 0}, fe{P_LO - 1, P_HI}};
    for (int i = 0; i < 20000; i++) as.push_back(fe{rng(), rng() >> 1});
    for (const fe& w : ws) {
      uint32_t l[5];
      limbs26(fe_mul(w, R), l);
      uint4 l4 = make_uint4(l[0], l[1], l[2], l[3]);
      uint32_t l1 = l[4];
      MontTab t{&l4, &l1};
      for (const fe& a : as)
        if (!fe_eq(mul_tw(a, t, 0), fe_mul(a, w))) { if (bad++ < 10) printf("mul_tw mismatch\n"); }
    }
  }
  // R' = 2^130 helpers of the matrix-core permutation: cubes of values < 2^129 (normalised
  // limbs, the round invariant) stay < 2^129; cubes of sums of two such values (< 2^130, a
  // state element after absorbing a message) stay < 2^131; extreme limb patterns included
  {
    const fe R1 = fe_pow64(fe{2, 0}, 130), R1inv = fe_inv(R1);
    auto val_bits_ok = [](const uint32_t l[5], int bits) {  // normalised limbs, value < 2^bits
      for (int j = 0; j < 4; j++)
        if (l[j] >= (1u << 26)) return false;
      return l[4] < (1u << (bits - 104));
    };
    for (int it = 0; it < 200000; it++) {
      uint32_t a[5], c[5];
      const int mode = it % 4;
      for (int j = 0; j < 5; j++) a[j] = (uint32_t)(rng() & 0x3FFFFFF);
      a[4] &= 0x1FFFFFF;  // < 2^129
      if (mode == 1) { for (int j = 0; j < 4; j++) a[j] = 0x3FFFFFF; a[4] = 0x1FFFFFF; }
      if (mode >= 2) {  // sum of two normalised values < 2^129: limbs < 2^27, value < 2^130
        for (int j = 0; j < 5; j++) a[j] += (uint32_t)(rng() & 0x3FFFFFF) & (j == 4 ? 0x1FFFFFFu : 0x3FFFFFFu);
        if (mode == 3) { for (int j = 0; j < 4; j++) a[j] = 0x7FFFFFE; a[4] = 0x3FFFFFE; }
      }
      const fe av = from26(a);
      mont_cube130(a, c);
      const fe want = fe_mul(fe_mul(fe_mul(av, av), av), fe_mul(R1inv, R1inv));
      const bool bound = val_bits_ok(c, mode >= 2 ? 131 : 129);
      if (!fe_eq(from26(c), want) || !bound) { if (bad++ < 10) printf("cube130 mismatch it=%d mode=%d\n", it, mode); }
      uint64_t col[10] = {a[0], a[1], a[2], a[3], a[4], 0, 0, 0, 0, 0};
      uint32_t o[5];
      redc130(col, o);  // from_mont130: < p + 2
      if (!fe_eq(from26(o), fe_mul(av, R1inv)) || !val_bits_ok(o, 129)) { if (bad++ < 10) printf("redc130 exit mismatch it=%d\n", it); }
    }
  }
  printf(bad ? "FAIL %d\n" : "OK\n", bad);
  return bad != 0;
}
