/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Nothing under blockframe-rs_amd/ links, loads or calls this file.  Only
 * tests/, __graft_entry__.smoke() (as the checker) and bench.py's cpu_baseline
 * leg may load liboracle.so.
 *
 * What it is: a plain-C restatement of the Reed-Solomon codec the reference
 * calls, reed-solomon-simd 3.1.0 (crates.io, checksum
 * cffef0520d30fbd4151fb20e262947ae47fb0ab276a744a19b6398438105a072, pinned at
 * /root/reference/Cargo.lock:1596-1605, declared at Cargo.toml:18).  The crate
 * is NOT vendored in /root/reference and there is no Rust toolchain here, so
 * it cannot be built (oracle/_ref is empty by necessity).
 * Its published algorithm (Leopard-RS "ff16": GF(2^16) in Cantor basis,
 * Lin-Chung-Han additive FFT) is restated from SURVEY.md Appendix A.
 *
 * Reference call sites this oracle stands in for:
 *   encode  src/chunker/generate.rs:37-49   (RS(1,3), generate_parity_segmented)
 *           src/chunker/generate.rs:84-96   (RS(k,3), generate_parity)
 *   decode  src/filestore/recovery.rs:58-68 (recover_segment_rs13)
 *           src/filestore/recovery.rs:152-170 (recover_segment_rs30_3)
 *           src/filestore/health.rs:514-528, 613-623, 733-752 (repairs)
 *
 * Pinning (see tests/test_oracle.py): the reference's own tests pin no parity
 * bytes, so parity is pinned against the independent
 * known-answer vector of SURVEY Appendix A.7 (k=30, shard_bytes=128) and the
 * derived constants of Appendix A.6 (G_30, Gamma); RS(1,3) == replication is
 * pinned by src/filestore/README.md:178.
 *
 * Two engines over the same algorithm:
 *   - ENGINE_SCALAR : per-symbol nibble tables (the crate's NoSimd engine shape);
 *                     this is the checker.
 *   - ENGINE_AVX2   : 32-byte PSHUFB nibble tables (the crate's Avx2 engine
 *                     shape); used only as the CPU baseline in bench.py and
 *                     cross-checked against ENGINE_SCALAR in tests.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#define GF_BITS 16
#define GF_ORDER 65536u
#define GF_MODULUS 65535u
#define GF_POLY 0x1002Du

/* SURVEY A.2 */
static const uint16_t CANTOR_BASIS[GF_BITS] = {
    0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

static uint16_t g_exp[GF_ORDER];
static uint16_t g_log[GF_ORDER];
static uint16_t g_skew[GF_ORDER];      /* 65535 used entries */
static uint16_t g_log_walsh[GF_ORDER];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static inline uint16_t add_mod(uint16_t x, uint16_t y) {
  uint32_t s = (uint32_t)x + (uint32_t)y;
  return (uint16_t)(s + (s >> GF_BITS));
}
static inline uint16_t sub_mod(uint16_t x, uint16_t y) {
  uint32_t d = (uint32_t)x - (uint32_t)y; /* wrapping */
  return (uint16_t)(d + (d >> GF_BITS));
}
/* x * exp(log_m); SURVEY A.2 */
static inline uint16_t gf_mul(uint16_t x, uint16_t log_m) {
  return x == 0 ? 0 : g_exp[add_mod(g_log[x], log_m)];
}

/* Walsh-Hadamard transform mod 65535, radix-4 passes, truncated input (A.2). */
static void fwht(uint16_t *d, size_t trunc) {
  for (size_t dist = 1, dist4 = 4; dist4 <= GF_ORDER; dist = dist4, dist4 <<= 2) {
    for (size_t r = 0; r < trunc; r += dist4) {
      for (size_t i = r; i < r + dist; ++i) {
        uint16_t a0 = d[i], a1 = d[i + dist], a2 = d[i + 2 * dist], a3 = d[i + 3 * dist];
        uint16_t s0 = add_mod(a0, a1), d0 = sub_mod(a0, a1);
        uint16_t s1 = add_mod(a2, a3), d1 = sub_mod(a2, a3);
        d[i] = add_mod(s0, s1);
        d[i + dist] = add_mod(d0, d1);
        d[i + 2 * dist] = sub_mod(s0, s1);
        d[i + 3 * dist] = sub_mod(d0, d1);
      }
    }
  }
}

static void init_tables(void) {
  /* LFSR pass: g_exp temporarily holds discrete logs (polynomial basis). */
  uint32_t state = 1;
  for (uint32_t i = 0; i < GF_MODULUS; ++i) {
    g_exp[state] = (uint16_t)i;
    state <<= 1;
    if (state >= GF_ORDER) state ^= GF_POLY;
  }
  g_exp[0] = GF_MODULUS;
  /* Cantor basis: g_log[j] = polynomial-basis value of Cantor element j. */
  g_log[0] = 0;
  for (unsigned i = 0; i < GF_BITS; ++i) {
    uint32_t w = 1u << i;
    for (uint32_t j = 0; j < w; ++j) g_log[j + w] = g_log[j] ^ CANTOR_BASIS[i];
  }
  for (uint32_t i = 0; i < GF_ORDER; ++i) g_log[i] = g_exp[g_log[i]];
  for (uint32_t i = 0; i < GF_ORDER; ++i) g_exp[g_log[i]] = (uint16_t)i;
  g_exp[GF_MODULUS] = g_exp[0];

  /* skew factors (A.2) */
  uint16_t temp[GF_BITS - 1];
  for (unsigned i = 1; i < GF_BITS; ++i) temp[i - 1] = (uint16_t)(1u << i);
  for (unsigned m = 0; m < GF_BITS - 1; ++m) {
    size_t step = (size_t)1 << (m + 1);
    g_skew[((size_t)1 << m) - 1] = 0;
    for (unsigned i = m; i < GF_BITS - 1; ++i) {
      size_t s = (size_t)1 << (i + 1);
      for (size_t j = ((size_t)1 << m) - 1; j < s; j += step) g_skew[j + s] = g_skew[j] ^ temp[i];
    }
    temp[m] = (uint16_t)(GF_MODULUS - g_log[gf_mul(temp[m], g_log[temp[m] ^ 1])]);
    for (unsigned i = m + 1; i < GF_BITS - 1; ++i)
      temp[i] = gf_mul(temp[i], add_mod(g_log[temp[i] ^ 1], temp[m]));
  }
  for (uint32_t i = 0; i < GF_MODULUS; ++i) g_skew[i] = g_log[g_skew[i]];

  memcpy(g_log_walsh, g_log, sizeof g_log);
  g_log_walsh[0] = 0;
  fwht(g_log_walsh, GF_ORDER);
}

static void ensure_tables(void) { pthread_once(&g_once, init_tables); }

/* ------------------------------------------------------------------------ */
/* Shard work area: `count` shards of `chunks` 64-byte chunks each.          */
/* Chunk layout (A.1): bytes [0,32) = low bytes of 32 symbols, [32,64) high. */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint8_t *base;
  size_t chunks;  /* 64-byte chunks per shard */
  size_t count;
  int engine;
} work_t;

static inline uint8_t *W(const work_t *w, size_t i) { return w->base + i * w->chunks * 64; }

#if defined(__x86_64__)
__attribute__((target("avx2"))) static void xor_avx2(uint8_t *x, const uint8_t *y, size_t n) {
  for (size_t b = 0; b < n; b += 32) {
    __m256i a = _mm256_loadu_si256((const __m256i *)(x + b));
    __m256i c = _mm256_loadu_si256((const __m256i *)(y + b));
    _mm256_storeu_si256((__m256i *)(x + b), _mm256_xor_si256(a, c));
  }
}
#endif

static void xor_into(const work_t *w, uint8_t *x, const uint8_t *y) {
  size_t n = w->chunks * 64;
#if defined(__x86_64__)
  if (w->engine == ORACLE_ENGINE_AVX2) {
    xor_avx2(x, y, n);
    return;
  }
#endif
  for (size_t b = 0; b < n; ++b) x[b] ^= y[b];
}

/* Nibble product tables for multiplication by exp(log_m):
 * lut[q][v] = (v << 4q) * exp(log_m) as a 16-bit Cantor-basis value. */
static void build_lut(uint16_t lut[4][16], uint16_t log_m) {
  for (int q = 0; q < 4; ++q)
    for (int v = 0; v < 16; ++v) lut[q][v] = gf_mul((uint16_t)(v << (4 * q)), log_m);
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) static void mul_chunks_avx2(uint8_t *x, const uint8_t *y,
                                                            size_t chunks, uint16_t log_m,
                                                            int add) {
  uint16_t lut[4][16];
  build_lut(lut, log_m);
  uint8_t tl[4][16], th[4][16];
  for (int q = 0; q < 4; ++q)
    for (int v = 0; v < 16; ++v) {
      tl[q][v] = (uint8_t)lut[q][v];
      th[q][v] = (uint8_t)(lut[q][v] >> 8);
    }
  __m256i TL[4], TH[4];
  for (int q = 0; q < 4; ++q) {
    TL[q] = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)tl[q]));
    TH[q] = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)th[q]));
  }
  const __m256i mask = _mm256_set1_epi8(0x0F);
  for (size_t c = 0; c < chunks; ++c) {
    const uint8_t *yc = y + c * 64;
    uint8_t *xc = x + c * 64;
    __m256i lo = _mm256_loadu_si256((const __m256i *)yc);
    __m256i hi = _mm256_loadu_si256((const __m256i *)(yc + 32));
    __m256i l0 = _mm256_and_si256(lo, mask), l1 = _mm256_and_si256(_mm256_srli_epi64(lo, 4), mask);
    __m256i h0 = _mm256_and_si256(hi, mask), h1 = _mm256_and_si256(_mm256_srli_epi64(hi, 4), mask);
    __m256i pl = _mm256_xor_si256(
        _mm256_xor_si256(_mm256_shuffle_epi8(TL[0], l0), _mm256_shuffle_epi8(TL[1], l1)),
        _mm256_xor_si256(_mm256_shuffle_epi8(TL[2], h0), _mm256_shuffle_epi8(TL[3], h1)));
    __m256i ph = _mm256_xor_si256(
        _mm256_xor_si256(_mm256_shuffle_epi8(TH[0], l0), _mm256_shuffle_epi8(TH[1], l1)),
        _mm256_xor_si256(_mm256_shuffle_epi8(TH[2], h0), _mm256_shuffle_epi8(TH[3], h1)));
    if (add) {
      pl = _mm256_xor_si256(pl, _mm256_loadu_si256((const __m256i *)xc));
      ph = _mm256_xor_si256(ph, _mm256_loadu_si256((const __m256i *)(xc + 32)));
    }
    _mm256_storeu_si256((__m256i *)xc, pl);
    _mm256_storeu_si256((__m256i *)(xc + 32), ph);
  }
}
#endif

/* add != 0: x ^= y * exp(log_m)  (engine mul_add);  add == 0: x = y * exp(log_m). */
static void mul_chunks(const work_t *w, uint8_t *x, const uint8_t *y, uint16_t log_m, int add) {
#if defined(__x86_64__)
  if (w->engine == ORACLE_ENGINE_AVX2) {
    mul_chunks_avx2(x, y, w->chunks, log_m, add);
    return;
  }
#endif
  uint16_t lut[4][16];
  build_lut(lut, log_m);
  for (size_t c = 0; c < w->chunks; ++c) {
    const uint8_t *yc = y + c * 64;
    uint8_t *xc = x + c * 64;
    for (int s = 0; s < 32; ++s) {
      uint8_t lo = yc[s], hi = yc[32 + s];
      uint16_t p = lut[0][lo & 15] ^ lut[1][lo >> 4] ^ lut[2][hi & 15] ^ lut[3][hi >> 4];
      if (add) {
        xc[s] ^= (uint8_t)p;
        xc[32 + s] ^= (uint8_t)(p >> 8);
      } else {
        xc[s] = (uint8_t)p;
        xc[32 + s] = (uint8_t)(p >> 8);
      }
    }
  }
}

/* Inverse FFT on shards [pos, pos+size), radix-2 statement of A.3.
 * Input positions >= trunc are zero, so skipped groups stay zero. */
static void ifft(const work_t *w, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
  for (size_t dist = 1; dist < size; dist <<= 1) {
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      uint16_t lm = g_skew[r + dist + skew_delta - 1];
      for (size_t i = r; i < r + dist; ++i) {
        uint8_t *x = W(w, pos + i), *y = W(w, pos + i + dist);
        xor_into(w, y, x);
        if (lm != GF_MODULUS) mul_chunks(w, x, y, lm, 1);
      }
    }
  }
}

/* Forward FFT; only outputs < trunc are meaningful. */
static void fft(const work_t *w, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
  for (size_t dist = size >> 1; dist > 0; dist >>= 1) {
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      uint16_t lm = g_skew[r + dist + skew_delta - 1];
      for (size_t i = r; i < r + dist; ++i) {
        uint8_t *x = W(w, pos + i), *y = W(w, pos + i + dist);
        if (lm != GF_MODULUS) mul_chunks(w, x, y, lm, 1);
        xor_into(w, y, x);
      }
    }
  }
}

static void formal_derivative(const work_t *w, size_t n) {
  for (size_t i = 1; i < n; ++i) {
    size_t width = i & (~i + 1);
    for (size_t j = 0; j < width; ++j) xor_into(w, W(w, i - width + j), W(w, i + j));
  }
}

/* erasures[i] <- log of the error-locator value (A.3 eval_poly). */
static void eval_poly(uint16_t *e, size_t trunc) {
  fwht(e, trunc);
  for (uint32_t i = 0; i < GF_ORDER; ++i) {
    uint32_t p = (uint32_t)e[i] * (uint32_t)g_log_walsh[i];
    e[i] = add_mod((uint16_t)p, (uint16_t)(p >> GF_BITS));
  }
  fwht(e, GF_ORDER);
}

static size_t next_pow2(size_t x) {
  size_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

/* DefaultRate selection (A.4, SURVEY risk r2 for k in {3,4}). */
int oracle_use_high_rate(uint32_t k, uint32_t m) {
  size_t kp = next_pow2(k), mp = next_pow2(m);
  if (kp < mp) return 0;
  if (kp > mp) return 1;
  return k <= m;
}

int oracle_supported(uint32_t k, uint32_t m) {
  if (k == 0 || m == 0 || k > GF_ORDER || m > GF_ORDER) return 0;
  size_t kp = next_pow2(k), mp = next_pow2(m);
  size_t smaller = kp < mp ? kp : mp;
  size_t larger = k > m ? k : m;
  return smaller + larger <= GF_ORDER;
}

/* Copy a user shard into the 64-byte chunk layout (A.1 incl. tail rule). */
static void shard_in(uint8_t *dst, size_t chunks, const uint8_t *src, size_t nbytes) {
  size_t whole = nbytes / 64, tail = nbytes % 64;
  memcpy(dst, src, whole * 64);
  memset(dst + whole * 64, 0, (chunks - whole) * 64);
  if (tail) {
    memcpy(dst + whole * 64, src + whole * 64, tail / 2);
    memcpy(dst + whole * 64 + 32, src + whole * 64 + tail / 2, tail / 2);
  }
}
static void shard_out(uint8_t *dst, size_t nbytes, const uint8_t *src) {
  size_t whole = nbytes / 64, tail = nbytes % 64;
  memcpy(dst, src, whole * 64);
  if (tail) {
    memcpy(dst + whole * 64, src + whole * 64, tail / 2);
    memcpy(dst + whole * 64 + tail / 2, src + whole * 64 + 32, tail / 2);
  }
}

static int check_args(uint32_t k, uint32_t m, size_t shard_bytes) {
  if (shard_bytes == 0 || (shard_bytes & 1)) return ORACLE_E_INVALID_SHARD_SIZE;
  if (!oracle_supported(k, m)) return ORACLE_E_UNSUPPORTED_SHARD_COUNT;
  return 0;
}

static int work_alloc(work_t *w, size_t count, size_t shard_bytes, int engine) {
  w->chunks = (shard_bytes + 63) / 64;
  w->count = count;
  w->engine = engine;
  w->base = (uint8_t *)calloc(count * w->chunks, 64);
  return w->base ? 0 : ORACLE_E_NOMEM;
}

/* HighRate encode (A.4): recovery j = work[j] after the chunked IFFTs + FFT. */
static void encode_high(const work_t *w, uint32_t k, uint32_t m) {
  size_t c = next_pow2(m);
  size_t first = k < c ? k : c;
  ifft(w, 0, c, first, c);
  if (k > c) {
    size_t p = c;
    for (; p + c <= k; p += c) {
      ifft(w, p, c, c, p + c);
      for (size_t i = 0; i < c; ++i) xor_into(w, W(w, i), W(w, p + i));
    }
    size_t last = k % c;
    if (last) {
      ifft(w, p, c, last, p + c);
      for (size_t i = 0; i < c; ++i) xor_into(w, W(w, i), W(w, p + i));
    }
  }
  fft(w, 0, c, m, 0);
}

/* LowRate encode (A.4): originals at positions [0,k), recovery at [c, c+m). */
static void encode_low(const work_t *w, uint32_t k, uint32_t m) {
  size_t c = next_pow2(k);
  ifft(w, 0, c, k, 0);
  for (size_t p = c; p < m; p += c)
    for (size_t i = 0; i < c; ++i) memcpy(W(w, p + i), W(w, i), w->chunks * 64);
  size_t p = 0;
  for (; p + c <= m; p += c) fft(w, p, c, c, p + c);
  size_t last = m % c;
  if (last) fft(w, p, c, last, p + c);
}

/* rate < 0: DefaultRate (oracle_use_high_rate); 0: LowRate; 1: HighRate.  The
 * forced rates exist only to write the RS(3,3)/RS(4,3) fixtures of risk r2
 * under both rates (tests/golden/make_golden.py). */
static int pick_rate(int rate, uint32_t k, uint32_t m) {
  return rate < 0 ? oracle_use_high_rate(k, m) : rate != 0;
}

int oracle_encode_rate(int engine, int rate, uint32_t k, uint32_t m, size_t shard_bytes,
                       const uint8_t *const *originals, uint8_t *const *recovery) {
  int rc = check_args(k, m, shard_bytes);
  if (rc) return rc;
  ensure_tables();
  int high = pick_rate(rate, k, m);
  size_t count;
  if (high) {
    size_t c = next_pow2(m);
    count = (k + c - 1) / c * c;
  } else {
    size_t c = next_pow2(k);
    size_t rc_ = (m + c - 1) / c * c;
    count = rc_ > c ? rc_ : c;
  }
  work_t w;
  if (work_alloc(&w, count, shard_bytes, engine)) return ORACLE_E_NOMEM;
  for (uint32_t i = 0; i < k; ++i) shard_in(W(&w, i), w.chunks, originals[i], shard_bytes);
  if (high)
    encode_high(&w, k, m);
  else
    encode_low(&w, k, m);
  for (uint32_t j = 0; j < m; ++j) shard_out(recovery[j], shard_bytes, W(&w, j));
  free(w.base);
  return 0;
}

int oracle_encode_engine(int engine, uint32_t k, uint32_t m, size_t shard_bytes,
                         const uint8_t *const *originals, uint8_t *const *recovery) {
  return oracle_encode_rate(engine, -1, k, m, shard_bytes, originals, recovery);
}

int oracle_encode(uint32_t k, uint32_t m, size_t shard_bytes, const uint8_t *const *originals,
                  uint8_t *const *recovery) {
  return oracle_encode_engine(ORACLE_ENGINE_SCALAR, k, m, shard_bytes, originals, recovery);
}

/* Decode (A.4).  originals[i]/recovery[j] == NULL marks a missing shard.
 * restored[i] is written only for missing originals.  Mirrors the crate's
 * ReedSolomonDecoder: all received shards take part. */
int oracle_decode_rate(int engine, int rate, uint32_t k, uint32_t m, size_t shard_bytes,
                       const uint8_t *const *originals, const uint8_t *const *recovery,
                       uint8_t *const *restored) {
  int rc = check_args(k, m, shard_bytes);
  if (rc) return rc;
  ensure_tables();
  uint32_t orig_recv = 0, rec_recv = 0;
  for (uint32_t i = 0; i < k; ++i) orig_recv += originals[i] != NULL;
  for (uint32_t j = 0; j < m; ++j) rec_recv += recovery[j] != NULL;
  if (orig_recv == k) return 0; /* nothing to restore */
  if (orig_recv + rec_recv < k) return ORACLE_E_NOT_ENOUGH_SHARDS;

  int high = pick_rate(rate, k, m);
  uint16_t *E = (uint16_t *)calloc(GF_ORDER, sizeof(uint16_t));
  if (!E) return ORACLE_E_NOMEM;
  work_t w;
  size_t n;
  if (high) {
    size_t c = next_pow2(m), end = c + k;
    n = next_pow2(end);
    if (work_alloc(&w, n, shard_bytes, engine)) {
      free(E);
      return ORACLE_E_NOMEM;
    }
    for (uint32_t j = 0; j < m; ++j)
      if (!recovery[j]) E[j] = 1;
    for (size_t j = m; j < c; ++j) E[j] = 1;
    for (uint32_t i = 0; i < k; ++i)
      if (!originals[i]) E[c + i] = 1;
    eval_poly(E, end);
    uint8_t *tmp = (uint8_t *)malloc(w.chunks * 64);
    for (uint32_t j = 0; j < m; ++j)
      if (recovery[j]) {
        shard_in(tmp, w.chunks, recovery[j], shard_bytes);
        mul_chunks(&w, W(&w, j), tmp, E[j], 0);
      }
    for (uint32_t i = 0; i < k; ++i)
      if (originals[i]) {
        shard_in(tmp, w.chunks, originals[i], shard_bytes);
        mul_chunks(&w, W(&w, c + i), tmp, E[c + i], 0);
      }
    free(tmp);
    ifft(&w, 0, n, end, 0);
    formal_derivative(&w, n);
    fft(&w, 0, n, end, 0);
    for (uint32_t i = 0; i < k; ++i)
      if (!originals[i]) {
        mul_chunks(&w, W(&w, c + i), W(&w, c + i), (uint16_t)(GF_MODULUS - E[c + i]), 0);
        shard_out(restored[i], shard_bytes, W(&w, c + i));
      }
  } else {
    size_t c = next_pow2(k), rend = c + m;
    n = next_pow2(rend);
    if (work_alloc(&w, n, shard_bytes, engine)) {
      free(E);
      return ORACLE_E_NOMEM;
    }
    /* originals' zero padding [k, c) is a known zero of the codeword (encode_low
     * zero-fills it before the IFFT), so it is not an erasure: marking it
     * would cost c-k of the m erasures the code corrects */
    for (uint32_t i = 0; i < k; ++i)
      if (!originals[i]) E[i] = 1;
    for (uint32_t j = 0; j < m; ++j)
      if (!recovery[j]) E[c + j] = 1;
    for (size_t i = rend; i < GF_ORDER; ++i) E[i] = 1;
    eval_poly(E, GF_ORDER);
    uint8_t *tmp = (uint8_t *)malloc(w.chunks * 64);
    for (uint32_t i = 0; i < k; ++i)
      if (originals[i]) {
        shard_in(tmp, w.chunks, originals[i], shard_bytes);
        mul_chunks(&w, W(&w, i), tmp, E[i], 0);
      }
    for (uint32_t j = 0; j < m; ++j)
      if (recovery[j]) {
        shard_in(tmp, w.chunks, recovery[j], shard_bytes);
        mul_chunks(&w, W(&w, c + j), tmp, E[c + j], 0);
      }
    free(tmp);
    ifft(&w, 0, n, rend, 0);
    formal_derivative(&w, n);
    fft(&w, 0, n, k, 0);
    for (uint32_t i = 0; i < k; ++i)
      if (!originals[i]) {
        mul_chunks(&w, W(&w, i), W(&w, i), (uint16_t)(GF_MODULUS - E[i]), 0);
        shard_out(restored[i], shard_bytes, W(&w, i));
      }
  }
  free(w.base);
  free(E);
  return 0;
}

int oracle_decode_engine(int engine, uint32_t k, uint32_t m, size_t shard_bytes,
                         const uint8_t *const *originals, const uint8_t *const *recovery,
                         uint8_t *const *restored) {
  return oracle_decode_rate(engine, -1, k, m, shard_bytes, originals, recovery, restored);
}

int oracle_decode(uint32_t k, uint32_t m, size_t shard_bytes, const uint8_t *const *originals,
                  const uint8_t *const *recovery, uint8_t *const *restored) {
  return oracle_decode_engine(ORACLE_ENGINE_SCALAR, k, m, shard_bytes, originals, recovery,
                              restored);
}

int oracle_have_avx2(void) {
#if defined(__x86_64__)
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2");
#else
  return 0;
#endif
}

/* Field helpers exposed for tests (A.5/A.6 constant checks). */
uint16_t oracle_gf_exp(uint16_t i) {
  ensure_tables();
  return g_exp[i];
}
uint16_t oracle_gf_log(uint16_t x) {
  ensure_tables();
  return g_log[x];
}
uint16_t oracle_gf_mul(uint16_t a, uint16_t b) {
  ensure_tables();
  if (a == 0 || b == 0) return 0;
  return gf_mul(a, g_log[b]);
}
uint16_t oracle_skew(uint32_t i) {
  ensure_tables();
  return g_skew[i];
}

/* ------------------------------------------------------------------------ */
/* Multi-threaded batch driver for the CPU baseline: one RS block per task,  */
/* mirroring rayon's into_par_iter over blocks (src/chunker/commit.rs:391).  */
/* ------------------------------------------------------------------------ */
typedef struct {
  int engine, decode;
  uint32_t nblocks, m;
  const uint32_t *k;
  size_t shard_bytes;
  const uint8_t *const *const *orig;  /* per block: k pointers (NULL = erased) */
  const uint8_t *const *const *rec;   /* per block: m pointers */
  uint8_t *const *const *out;         /* per block: m (encode) or k (decode) pointers */
  int next;
  int err;
  pthread_mutex_t mu;
  int copies; /* 1: the reference wrappers' copies around every call (see oracle_batch2) */
} batch_t;

/* One block with the copies BlockFrame's wrappers make around the crate call:
 * every input is copied first (generate.rs:75-82 pads each segment with
 * to_vec; the decoder wrappers take owned Vecs), the codec writes into its own
 * buffers, and the results are copied out (recovery_iter().to_vec(),
 * generate.rs:95-96; restored_original(..).to_vec(), recovery.rs:167-169). */
static int block_with_copies(const batch_t *b, uint32_t i) {
  const uint32_t k = b->k[i], m = b->m, nout = b->decode ? k : m;
  const size_t n = b->shard_bytes;
  const uint8_t **in = (const uint8_t **)calloc(k + m, sizeof(void *));
  uint8_t **out = (uint8_t **)calloc(nout, sizeof(void *));
  int rc = 0;
  for (uint32_t x = 0; x < k + m && !rc; ++x) {
    const uint8_t *src = x < k ? b->orig[i][x] : (b->decode ? b->rec[i][x - k] : NULL);
    if (!src) continue;
    uint8_t *c = (uint8_t *)malloc(n);
    if (!c) rc = -100;
    else memcpy(c, src, n);
    in[x] = c;
  }
  for (uint32_t x = 0; x < nout && !rc; ++x)
    if (b->out[i][x]) {
      out[x] = (uint8_t *)malloc(n);
      if (!out[x]) rc = -100;
    }
  if (!rc)
    rc = b->decode ? oracle_decode_engine(b->engine, k, m, n, in, in + k, out)
                   : oracle_encode_engine(b->engine, k, m, n, in, out);
  for (uint32_t x = 0; x < nout; ++x)
    if (out[x]) {
      if (!rc) memcpy(b->out[i][x], out[x], n);
      free(out[x]);
    }
  for (uint32_t x = 0; x < k + m; ++x) free((void *)in[x]);
  free(in);
  free(out);
  return rc;
}

static void *batch_worker(void *arg) {
  batch_t *b = (batch_t *)arg;
  for (;;) {
    pthread_mutex_lock(&b->mu);
    int i = b->next++;
    pthread_mutex_unlock(&b->mu);
    if (i >= (int)b->nblocks) break;
    int rc = b->copies ? block_with_copies(b, (uint32_t)i)
           : b->decode ? oracle_decode_engine(b->engine, b->k[i], b->m, b->shard_bytes, b->orig[i],
                                              b->rec[i], b->out[i])
                       : oracle_encode_engine(b->engine, b->k[i], b->m, b->shard_bytes, b->orig[i],
                                              b->out[i]);
    if (rc) {
      pthread_mutex_lock(&b->mu);
      b->err = rc;
      pthread_mutex_unlock(&b->mu);
    }
  }
  return NULL;
}

int oracle_batch2(int engine, int decode, int threads, uint32_t nblocks, const uint32_t *k,
                  uint32_t m, size_t shard_bytes, const uint8_t *const *const *orig,
                  const uint8_t *const *const *rec, uint8_t *const *const *out, int copies) {
  ensure_tables();
  batch_t b = {engine, decode, nblocks, m, k, shard_bytes, orig, rec, out, 0, 0,
               PTHREAD_MUTEX_INITIALIZER, copies};
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, batch_worker, &b);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  return b.err;
}

int oracle_batch(int engine, int decode, int threads, uint32_t nblocks, const uint32_t *k,
                 uint32_t m, size_t shard_bytes, const uint8_t *const *const *orig,
                 const uint8_t *const *const *rec, uint8_t *const *const *out) {
  return oracle_batch2(engine, decode, threads, nblocks, k, m, shard_bytes, orig, rec, out, 0);
}
