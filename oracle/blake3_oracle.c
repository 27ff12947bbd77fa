/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see rs_oracle.c header for the rules).
 *
 * Portable single-threaded restatement of BLAKE3 (the `blake3` 1.8.2 crate,
 * /root/reference/Cargo.lock:136-145, called via src/utils.rs:22-28
 * blake3_hash_bytes) from the published BLAKE3 specification: 1 KiB chunks,
 * 64-byte blocks, 7-round compression, binary tree with left-full subtrees.
 * Pinned by the reference's doctest KAT src/utils.rs:17-18
 * (blake3("blockframe") = c41e3ccb...8fb7) and the specification's
 * empty-input vector, see tests/test_oracle.py.
 *
 * Also restates src/merkle_tree/mod.rs:77-100 (build_tree): parents hash the
 * ASCII concatenation of the two lowercase-hex child digests; an odd node is
 * paired with itself.
 */
#include "oracle.h"

#include <stdio.h>
#include <string.h>

static const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                               0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static inline void g(uint32_t *s, int a, int b, int c, int d, uint32_t x, uint32_t y) {
  s[a] = s[a] + s[b] + x;
  s[d] = rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + y;
  s[d] = rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 7);
}

static void compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter,
                     uint32_t block_len, uint32_t flags, uint32_t out[16]) {
  uint32_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                    IV[0], IV[1], IV[2], IV[3], (uint32_t)counter, (uint32_t)(counter >> 32),
                    block_len, flags};
  uint32_t m[16], t[16];
  memcpy(m, block, sizeof m);
  for (int r = 0; r < 7; ++r) {
    g(s, 0, 4, 8, 12, m[0], m[1]);
    g(s, 1, 5, 9, 13, m[2], m[3]);
    g(s, 2, 6, 10, 14, m[4], m[5]);
    g(s, 3, 7, 11, 15, m[6], m[7]);
    g(s, 0, 5, 10, 15, m[8], m[9]);
    g(s, 1, 6, 11, 12, m[10], m[11]);
    g(s, 2, 7, 8, 13, m[12], m[13]);
    g(s, 3, 4, 9, 14, m[14], m[15]);
    for (int i = 0; i < 16; ++i) t[i] = m[PERM[i]];
    memcpy(m, t, sizeof m);
  }
  for (int i = 0; i < 8; ++i) {
    out[i] = s[i] ^ s[i + 8];
    out[i + 8] = s[i + 8] ^ cv[i];
  }
}

static void words_le(const uint8_t *p, size_t n, uint32_t w[16]) {
  uint8_t buf[64] = {0};
  if (n) memcpy(buf, p, n); /* p is NULL for the empty message */
  for (int i = 0; i < 16; ++i)
    w[i] = (uint32_t)buf[4 * i] | (uint32_t)buf[4 * i + 1] << 8 | (uint32_t)buf[4 * i + 2] << 16 |
           (uint32_t)buf[4 * i + 3] << 24;
}

/* The pending "output" of the last node: compressing it with ROOT gives the digest. */
typedef struct {
  uint32_t cv[8];
  uint32_t block[16];
  uint64_t counter;
  uint32_t block_len, flags;
} node_out;

static void out_cv(const node_out *o, uint32_t cv[8]) {
  uint32_t t[16];
  compress(o->cv, o->block, o->counter, o->block_len, o->flags, t);
  memcpy(cv, t, 32);
}

/* Process one chunk (<= 1024 bytes); returns its (non-root) output node. */
static node_out chunk_node(const uint8_t *p, size_t n, uint64_t chunk_index) {
  uint32_t cv[8];
  memcpy(cv, IV, sizeof cv);
  size_t nblocks = n == 0 ? 1 : (n + 63) / 64;
  node_out o;
  for (size_t b = 0; b < nblocks; ++b) {
    size_t len = (b + 1 < nblocks) ? 64 : n - b * 64;
    uint32_t w[16];
    words_le(p + b * 64, len, w);
    uint32_t flags = (b == 0 ? CHUNK_START : 0) | (b + 1 == nblocks ? CHUNK_END : 0);
    if (b + 1 < nblocks) {
      uint32_t t[16];
      compress(cv, w, chunk_index, 64, flags, t);
      memcpy(cv, t, 32);
    } else {
      memcpy(o.cv, cv, 32);
      memcpy(o.block, w, 64);
      o.counter = chunk_index;
      o.block_len = (uint32_t)len;
      o.flags = flags;
    }
  }
  return o;
}

static node_out parent_node(const uint32_t l[8], const uint32_t r[8]) {
  node_out o;
  memcpy(o.cv, IV, 32);
  memcpy(o.block, l, 32);
  memcpy(o.block + 8, r, 32);
  o.counter = 0;
  o.block_len = 64;
  o.flags = PARENT;
  return o;
}

void oracle_blake3(const uint8_t *data, size_t len, uint8_t digest[32]) {
  uint32_t stack[64][8];
  int depth = 0;
  size_t nchunks = len == 0 ? 1 : (len + 1023) / 1024;
  node_out last;
  for (size_t c = 0; c < nchunks; ++c) {
    size_t off = c * 1024, n = (len - off) < 1024 ? (len - off) : 1024;
    node_out o = chunk_node(data + off, n, c);
    if (c + 1 == nchunks) {
      last = o;
      break;
    }
    uint32_t cv[8];
    out_cv(&o, cv);
    /* merge completed subtrees: chunk count after this one = c + 1 */
    uint64_t total = c + 1;
    while ((total & 1) == 0) {
      node_out p = parent_node(stack[--depth], cv);
      out_cv(&p, cv);
      total >>= 1;
    }
    memcpy(stack[depth++], cv, 32);
  }
  while (depth > 0) {
    uint32_t cv[8];
    out_cv(&last, cv);
    last = parent_node(stack[--depth], cv);
  }
  uint32_t t[16];
  compress(last.cv, last.block, last.counter, last.block_len, last.flags | ROOT, t);
  for (int i = 0; i < 8; ++i) {
    digest[4 * i] = (uint8_t)t[i];
    digest[4 * i + 1] = (uint8_t)(t[i] >> 8);
    digest[4 * i + 2] = (uint8_t)(t[i] >> 16);
    digest[4 * i + 3] = (uint8_t)(t[i] >> 24);
  }
}

void oracle_blake3_hex(const uint8_t *data, size_t len, char hex[65]) {
  uint8_t d[32];
  oracle_blake3(data, len, d);
  for (int i = 0; i < 32; ++i) snprintf(hex + 2 * i, 3, "%02x", d[i]);
  hex[64] = 0;
}

/* src/merkle_tree/mod.rs:77-100 over n lowercase-hex leaves (64 chars each,
 * packed back to back in `leaves`).  Writes the root hex into `root`. */
int oracle_merkle_root_hex(const char *leaves, size_t n, char root[65]) {
  if (n == 0) return -1;
  char level[256][65];
  if (n > 256) return -1;
  for (size_t i = 0; i < n; ++i) {
    memcpy(level[i], leaves + 64 * i, 64);
    level[i][64] = 0;
  }
  while (n > 1) {
    size_t m = 0;
    for (size_t i = 0; i < n; i += 2) {
      char cat[128];
      memcpy(cat, level[i], 64);
      memcpy(cat + 64, (i + 1 < n) ? level[i + 1] : level[i], 64);
      oracle_blake3_hex((const uint8_t *)cat, 128, level[m++]);
    }
    n = m;
  }
  memcpy(root, level[0], 65);
  return 0;
}
