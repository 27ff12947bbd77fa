/* tsan_oracle.c — ThreadSanitizer driver for the oracle's threaded paths
 * (test infrastructure: oracle/Makefile `sanitize`, tests/test_sanitize.py).
 *
 * 1. oracle_batch2 over many small blocks on 8 worker threads, encode and
 *    decode, with and without the reference-wrapper copies (bench.py's
 *    cpu_baseline runs exactly these), results checked against one thread;
 * 2. independent threads calling oracle_encode / oracle_blake3 at once from a
 *    cold start (the pthread_once table init races with the first callers).
 * Exit 0 = every result equal; TSan reports go to stderr (and exit 66). */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

enum { NB = 24, M = 3, N = 64 * 40 + 64 };

static uint64_t sm_state = 0x7A5A;
static uint8_t next_byte(void) {
  uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint8_t)(z ^ (z >> 31));
}

static void *cold_caller(void *arg) {
  const int id = (int)(intptr_t)arg;
  uint8_t *d[5], *r[3];
  for (int i = 0; i < 5; ++i) {
    d[i] = malloc(N);
    for (int j = 0; j < N; ++j) d[i][j] = (uint8_t)(i * 31 + j + id);
  }
  for (int j = 0; j < 3; ++j) r[j] = malloc(N);
  int rc = oracle_encode(5, 3, N, (const uint8_t *const *)d, r);
  uint8_t dig[32];
  oracle_blake3(d[0], N, dig);
  for (int i = 0; i < 5; ++i) free(d[i]);
  for (int j = 0; j < 3; ++j) free(r[j]);
  return (void *)(intptr_t)rc;
}

int main(void) {
  /* 2. cold start: first use of the tables from 6 threads at once */
  pthread_t th[6];
  for (int t = 0; t < 6; ++t) pthread_create(&th[t], NULL, cold_caller, (void *)(intptr_t)t);
  for (int t = 0; t < 6; ++t) {
    void *rc;
    pthread_join(th[t], &rc);
    if (rc) {
      fprintf(stderr, "cold caller %d failed: %d\n", t, (int)(intptr_t)rc);
      return 1;
    }
  }

  /* 1. batches */
  uint32_t k[NB];
  uint8_t *data[NB][30], *par1[NB][M], *par8[NB][M], *rest[NB][30];
  const uint8_t *orig[NB][30], *rec[NB][M], *dec_in[NB][30];
  uint8_t *const *outp1[NB], *const *outp8[NB], *const *restp[NB];
  const uint8_t *const *origp[NB], *const *recp[NB], *const *decp[NB];
  for (int b = 0; b < NB; ++b) {
    k[b] = 1 + (uint32_t)(b * 7) % 30;
    for (uint32_t i = 0; i < k[b]; ++i) {
      data[b][i] = malloc(N);
      for (int j = 0; j < N; ++j) data[b][i][j] = next_byte();
      orig[b][i] = data[b][i];
      rest[b][i] = NULL;
      dec_in[b][i] = data[b][i];
    }
    for (int j = 0; j < M; ++j) {
      par1[b][j] = malloc(N);
      par8[b][j] = malloc(N);
      rec[b][j] = par1[b][j];
    }
    /* erase up to 3 originals */
    for (uint32_t e = 0; e < k[b] && e < 3; ++e) {
      const uint32_t i = (uint32_t)(b + 5 * e) % k[b];
      if (!dec_in[b][i]) continue;
      dec_in[b][i] = NULL;
      rest[b][i] = malloc(N);
    }
    outp1[b] = par1[b];
    outp8[b] = par8[b];
    restp[b] = rest[b];
    origp[b] = orig[b];
    recp[b] = rec[b];
    decp[b] = dec_in[b];
  }
  for (int copies = 0; copies < 2; ++copies) {
    if (oracle_batch2(ORACLE_ENGINE_SCALAR, 0, 1, NB, k, M, N, origp, NULL, outp1, copies) ||
        oracle_batch2(ORACLE_ENGINE_SCALAR, 0, 8, NB, k, M, N, origp, NULL, outp8, copies)) {
      fprintf(stderr, "encode batch failed\n");
      return 1;
    }
    for (int b = 0; b < NB; ++b)
      for (int j = 0; j < M; ++j)
        if (memcmp(par1[b][j], par8[b][j], N)) {
          fprintf(stderr, "threaded encode differs: block %d parity %d\n", b, j);
          return 1;
        }
    if (oracle_batch2(ORACLE_ENGINE_SCALAR, 1, 8, NB, k, M, N, decp, recp, restp, copies)) {
      fprintf(stderr, "decode batch failed\n");
      return 1;
    }
    for (int b = 0; b < NB; ++b)
      for (uint32_t i = 0; i < k[b]; ++i)
        if (rest[b][i] && memcmp(rest[b][i], data[b][i], N)) {
          fprintf(stderr, "threaded decode differs: block %d shard %u\n", b, i);
          return 1;
        }
  }
  printf("tsan_oracle ok: %d blocks, 8 threads, encode + decode, with and without copies\n", NB);
  return 0;
}
