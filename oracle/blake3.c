/*
 * ORACLE — test infrastructure only.
 *
 * BLAKE3 (hash mode, 32-byte output), restating the published BLAKE3 spec that
 * the `blake3` crate 1.8.2 implements (third-party, not vendored; Cargo.lock:110-113).
 * Used by the reference for program_id (zk-lisp-compiler/src/lib.rs:239-245) and for
 * Poseidon constant derivation ro_from_slices (poseidon/mod.rs:421-440).
 * Pinned by the spec's known answers (tests/test_oracle_blake3.py).
 */
#include <stdint.h>
#include <string.h>
#include "oracle.h"

static const uint32_t IV[8] = {0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
                               0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19};
static const uint8_t PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void g(uint32_t *s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
  s[a] = s[a] + s[b] + mx; s[d] = rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];      s[b] = rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + my; s[d] = rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];      s[b] = rotr(s[b] ^ s[c], 7);
}

static void compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter,
                     uint32_t block_len, uint32_t flags, uint32_t out[16]) {
  uint32_t s[16], m[16], t[16];
  for (int i = 0; i < 8; i++) s[i] = cv[i];
  for (int i = 0; i < 4; i++) s[8 + i] = IV[i];
  s[12] = (uint32_t)counter; s[13] = (uint32_t)(counter >> 32);
  s[14] = block_len; s[15] = flags;
  memcpy(m, block, 64);
  for (int r = 0; r < 7; r++) {
    g(s, 0, 4, 8, 12, m[0], m[1]);  g(s, 1, 5, 9, 13, m[2], m[3]);
    g(s, 2, 6, 10, 14, m[4], m[5]); g(s, 3, 7, 11, 15, m[6], m[7]);
    g(s, 0, 5, 10, 15, m[8], m[9]); g(s, 1, 6, 11, 12, m[10], m[11]);
    g(s, 2, 7, 8, 13, m[12], m[13]); g(s, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) { for (int i = 0; i < 16; i++) t[i] = m[PERM[i]]; memcpy(m, t, 64); }
  }
  for (int i = 0; i < 8; i++) { out[i] = s[i] ^ s[i + 8]; out[i + 8] = s[i + 8] ^ cv[i]; }
}

static void load_block(const uint8_t *p, size_t len, uint32_t w[16]) {
  uint8_t b[64] = {0};
  memcpy(b, p, len);
  for (int i = 0; i < 16; i++)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
}

/* "output" of a node before the root decision: cv + block + counter + len + flags */
typedef struct { uint32_t cv[8]; uint32_t block[16]; uint64_t counter; uint32_t len, flags; } node_out;

static void chunk_output(const uint8_t *chunk, size_t len, uint64_t counter, node_out *o) {
  uint32_t cv[8];
  memcpy(cv, IV, 32);
  size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
  for (size_t b = 0; b < nblocks; b++) {
    size_t bl = (b + 1 < nblocks) ? 64 : len - 64 * b;
    uint32_t w[16];
    load_block(chunk + 64 * b, bl, w);
    uint32_t flags = (b == 0 ? CHUNK_START : 0) | (b + 1 == nblocks ? CHUNK_END : 0);
    if (b + 1 == nblocks) {
      memcpy(o->cv, cv, 32); memcpy(o->block, w, 64);
      o->counter = counter; o->len = (uint32_t)bl; o->flags = flags;
      return;
    }
    uint32_t out[16];
    compress(cv, w, counter, 64, flags, out);
    memcpy(cv, out, 32);
  }
}

static void node_cv(const node_out *o, uint32_t cv[8]) {
  uint32_t out[16];
  compress(o->cv, o->block, o->counter, o->len, o->flags, out);
  memcpy(cv, out, 32);
}

static void parent_output(const uint32_t l[8], const uint32_t r[8], node_out *o) {
  memcpy(o->cv, IV, 32);
  memcpy(o->block, l, 32); memcpy(o->block + 8, r, 32);
  o->counter = 0; o->len = 64; o->flags = PARENT;
}

void orc_blake3(const uint8_t *in, size_t len, uint8_t out32[32]) {
  /* incremental stack algorithm of the BLAKE3 reference implementation */
  uint32_t stack[64][8];
  int sp = 0;
  size_t nchunks = len == 0 ? 1 : (len + 1023) / 1024;
  node_out o;
  for (size_t c = 0; c + 1 < nchunks; c++) {
    chunk_output(in + 1024 * c, 1024, c, &o);
    uint32_t cv[8];
    node_cv(&o, cv);
    uint64_t total = c + 1;
    while ((total & 1) == 0) {
      node_out p;
      parent_output(stack[--sp], cv, &p);
      node_cv(&p, cv);
      total >>= 1;
    }
    memcpy(stack[sp++], cv, 32);
  }
  size_t last = nchunks - 1;
  chunk_output(in + 1024 * last, len - 1024 * last, last, &o);
  while (sp > 0) {
    uint32_t cv[8];
    node_cv(&o, cv);
    parent_output(stack[--sp], cv, &o);
  }
  uint32_t res[16];
  compress(o.cv, o.block, o.counter, o.len, o.flags | ROOT, res);
  for (int i = 0; i < 8; i++) {
    out32[4 * i] = (uint8_t)res[i]; out32[4 * i + 1] = (uint8_t)(res[i] >> 8);
    out32[4 * i + 2] = (uint8_t)(res[i] >> 16); out32[4 * i + 3] = (uint8_t)(res[i] >> 24);
  }
}

/* streaming helper over several parts (ro_from_slices hashes domain || parts) */
void orc_blake3_parts(const uint8_t *const *parts, const size_t *lens, int nparts, uint8_t out32[32]) {
  size_t tot = 0;
  for (int i = 0; i < nparts; i++) tot += lens[i];
  uint8_t buf[4096];
  uint8_t *b = buf;
  uint8_t *heap = 0;
  if (tot > sizeof buf) { heap = (uint8_t *)malloc(tot); b = heap; }
  size_t off = 0;
  for (int i = 0; i < nparts; i++) { memcpy(b + off, parts[i], lens[i]); off += lens[i]; }
  orc_blake3(b, tot, out32);
  if (heap) free(heap);
}
