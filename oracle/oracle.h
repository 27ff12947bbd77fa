/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement of reed-solomon-simd
 * 3.1.0 and BLAKE3 used as the checker for the HIP path (tests/, smoke())
 * and as the CPU baseline (bench.py cpu_baseline).  The product
 * (blockframe-rs_amd/, include/bfrs.h) never includes or links this.
 */
#ifndef BLOCKFRAME_ORACLE_H
#define BLOCKFRAME_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ORACLE_ENGINE_SCALAR = 0,
  ORACLE_ENGINE_AVX2 = 1,
};

enum {
  ORACLE_OK = 0,
  ORACLE_E_INVALID_SHARD_SIZE = -1,
  ORACLE_E_UNSUPPORTED_SHARD_COUNT = -2,
  ORACLE_E_NOT_ENOUGH_SHARDS = -3,
  ORACLE_E_NOMEM = -4,
};

int oracle_use_high_rate(uint32_t k, uint32_t m);
int oracle_supported(uint32_t k, uint32_t m);
int oracle_have_avx2(void);

int oracle_encode(uint32_t k, uint32_t m, size_t shard_bytes, const uint8_t *const *originals,
                  uint8_t *const *recovery);
int oracle_decode(uint32_t k, uint32_t m, size_t shard_bytes, const uint8_t *const *originals,
                  const uint8_t *const *recovery, uint8_t *const *restored);
int oracle_encode_engine(int engine, uint32_t k, uint32_t m, size_t shard_bytes,
                         const uint8_t *const *originals, uint8_t *const *recovery);
int oracle_decode_engine(int engine, uint32_t k, uint32_t m, size_t shard_bytes,
                         const uint8_t *const *originals, const uint8_t *const *recovery,
                         uint8_t *const *restored);
/* rate: -1 DefaultRate, 0 LowRate, 1 HighRate (risk r2 fixtures only) */
int oracle_encode_rate(int engine, int rate, uint32_t k, uint32_t m, size_t shard_bytes,
                       const uint8_t *const *originals, uint8_t *const *recovery);
int oracle_decode_rate(int engine, int rate, uint32_t k, uint32_t m, size_t shard_bytes,
                       const uint8_t *const *originals, const uint8_t *const *recovery,
                       uint8_t *const *restored);
int oracle_batch(int engine, int decode, int threads, uint32_t nblocks, const uint32_t *k,
                 uint32_t m, size_t shard_bytes, const uint8_t *const *const *orig,
                 const uint8_t *const *const *rec, uint8_t *const *const *out);
/* copies = 1: each block also pays the reference wrappers' copies (bench.py) */
int oracle_batch2(int engine, int decode, int threads, uint32_t nblocks, const uint32_t *k,
                  uint32_t m, size_t shard_bytes, const uint8_t *const *const *orig,
                  const uint8_t *const *const *rec, uint8_t *const *const *out, int copies);

uint16_t oracle_gf_exp(uint16_t i);
uint16_t oracle_gf_log(uint16_t x);
uint16_t oracle_gf_mul(uint16_t a, uint16_t b);
uint16_t oracle_skew(uint32_t i);

void oracle_blake3(const uint8_t *data, size_t len, uint8_t digest[32]);
void oracle_blake3_hex(const uint8_t *data, size_t len, char hex[65]);
int oracle_merkle_root_hex(const char *leaves, size_t n, char root[65]);

#ifdef __cplusplus
}
#endif
#endif
