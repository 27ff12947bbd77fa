/*
 * bfrs.h — C-ABI of the MI355X-native Reed-Solomon path for BlockFrame.
 *
 * This library replaces the bottom box of the reference's hot path: the
 * third-party crate reed-solomon-simd 3.1.0 (Cargo.toml:18) that BlockFrame
 * calls from src/chunker/generate.rs, src/filestore/recovery.rs and
 * src/filestore/health.rs.  Output is bit-exact with that crate's algorithm
 * (GF(2^16) Leopard/LCH code, 64-byte lo/hi shard layout).
 *
 * Plain C types only: pointers, sizes, opaque handles.  No torch, no HIP
 * types in signatures (a HIP stream is passed as `void *`).
 *
 * Error convention: every entry point returns 0 on success or a negative
 * BFRS_E_* code; it never aborts on bad input (the reference builds with
 * panic = "abort", Cargo.toml:79).  bfrs_last_error() returns the message of
 * the calling thread's last failure, using the reference's own strings where
 * the reference has them (src/filestore/recovery.rs:48,55,124,128,132,138).
 *
 * Threading: one context per device may be shared by all threads, which is
 * how rayon's one-encoder-per-block use (src/chunker/commit.rs:391-466) maps
 * onto it.  Encoder/decoder objects and the batch calls may run concurrently
 * on one context: each codec object owns a pooled slot (device rows, pinned
 * rows, a HIP stream), the plan cache
 * and the slot pool are locked, the
 * host-batch pipeline and the BLAKE3 work area are serialised.  A single
 * encoder or decoder object is used by one thread at a time (as the crate's
 * &mut self API implies).  A context keeps at most BFRS_CODEC_SLOTS idle codec
 * slots (environment, read by bfrs_open; default 2): set it to the number of
 * worker threads to keep their pinned + device rows across blocks.  The
 * archive calls (commit, repair, health check) and an open archive handle are
 * serialised inside the library; a handle may be read from several threads.
 * Distinct contexts are independent.
 *
 * Lifetimes: an encoder or decoder may be freed before or after bfrs_close of
 * its context (it shares the context's slot pool); every other call on it
 * needs the context open.  An archive handle should be closed before its
 * context; if it is not, bfrs_close detaches it (joins its prefetch threads
 * and drops what it holds of the context), later bfrs_archive_read calls on
 * it fail with BFRS_E_INVALID_ARGUMENT and bfrs_archive_close still frees it.
 * No library thread outlives bfrs_close.  bfrs_close must not run while
 * another thread is inside a call on the same context or one of its handles.
 *
 * Environment: libbfrs.so reads exactly these six knobs (tests/test_abi.py
 * checks the BFRS_* strings in the binary against this list).  The knobs of
 * concluded A/B studies (pipeline depth, slab width, stream layout, prefault
 * modes, ...) exist only in the measurement build
 * libbfrs_ab.so (csrc/knobs.hpp).
 *   BFRS_CODEC_SLOTS    idle codec slots a context keeps (read by bfrs_open;
 *                       default 2; 0 = none)
 *   BFRS_CODEC_STAGING  "pinned" (default: add_*_shard copies into a pinned
 *                       row on several threads and queues its H2D) or
 *                       "direct" (one DMA straight from the caller's buffer);
 *                       either way the buffer is free on return (bfrs_open)
 *   BFRS_PLAN_CACHE     coefficient plans a context caches (bfrs_open;
 *                       default 4096, at least 1)
 *   BFRS_PREFETCH_DEPTH archive read handles: segments loaded ahead of the
 *                       reader (default 16, at most half the cache; read by
 *                       bfrs_archive_open)
 *   BFRS_HOST_COPY_BUDGET  helper threads of all concurrent host copies
 *                       together (default: the process's CPU share - 1, the
 *                       cgroup quota; read once per process), split evenly
 *                       between the calls in flight
 *   BFRS_KERNEL_VARIANT unset or 76 (default kernel); 75 / 73 force the looped
 *                       subfield / general kernels; anything else fails
 *                       bfrs_open with BFRS_E_INVALID_ARGUMENT (the A/B
 *                       variants exist only in the measurement build)
 */
#ifndef BFRS_H
#define BFRS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BFRS_ABI_VERSION 1

/* Error codes.  -1..-10 mirror reed_solomon_simd::Error (3.x). */
enum {
  BFRS_OK = 0,
  BFRS_E_DIFFERENT_SHARD_SIZE = -1,
  BFRS_E_DUPLICATE_ORIGINAL_SHARD_INDEX = -2,
  BFRS_E_DUPLICATE_RECOVERY_SHARD_INDEX = -3,
  BFRS_E_INVALID_ORIGINAL_SHARD_INDEX = -4,
  BFRS_E_INVALID_RECOVERY_SHARD_INDEX = -5,
  BFRS_E_INVALID_SHARD_SIZE = -6,
  BFRS_E_NOT_ENOUGH_SHARDS = -7,
  BFRS_E_TOO_FEW_ORIGINAL_SHARDS = -8,
  BFRS_E_TOO_MANY_ORIGINAL_SHARDS = -9,
  BFRS_E_UNSUPPORTED_SHARD_COUNT = -10,
  /* BlockFrame wrapper errors (src/chunker/generate.rs, src/filestore/recovery.rs) */
  BFRS_E_WRAPPER = -20,          /* message in bfrs_last_error(), reference wording */
  /* Boundary / device errors */
  BFRS_E_INVALID_ARGUMENT = -30, /* NULL handle/pointer, misaligned device pointer */
  BFRS_E_HIP = -31,              /* HIP runtime failure; message has hipGetErrorString */
  BFRS_E_NO_DEVICE = -32,        /* no usable gfx950 device / device id out of range */
  BFRS_E_NOMEM = -33,
  BFRS_E_NOT_RESTORED = -34,     /* restored_original(i): index was not restored (None) */
  BFRS_E_NOT_FOUND = -35,        /* bfrs_store_find: no archived file of that name */
};

typedef struct bfrs_ctx bfrs_ctx;
typedef struct bfrs_encoder bfrs_encoder;
typedef struct bfrs_decoder bfrs_decoder;

/* ---- context --------------------------------------------------------- */
int bfrs_abi_version(void);
const char *bfrs_strerror(int code);
const char *bfrs_last_error(void);
int bfrs_device_count(void);
/* Opens a context on HIP device `device` (>= 0).  Fails with BFRS_E_NO_DEVICE
 * if the device is absent — there is no CPU fallback. */
int bfrs_open(int device, bfrs_ctx **out);
void bfrs_close(bfrs_ctx *ctx);
/* Blocks until all work the context queued has finished. */
int bfrs_synchronize(bfrs_ctx *ctx);
/* Recommended byte distance between consecutive shards of one allocation
 * (HBM layout hint, no reference counterpart).  Shards of >= 1 MiB placed a
 * power of two apart alias onto the same HBM channels when the kernel reads
 * one column of all of them together; a pitch = 12 KiB (mod 64 KiB) spreads
 * them (measured 0.8-5% faster).  Smaller shards: rounded up to 256 B. */
size_t bfrs_shard_pitch(size_t shard_bytes);

/* ---- codec rules (pure host logic) ------------------------------------ */
/* 1 = HighRate, 0 = LowRate (reed-solomon-simd DefaultRate), <0 = unsupported. */
int bfrs_use_high_rate(size_t original_count, size_t recovery_count);
/* Encode/decode coefficient of output `out_index` w.r.t. input `in_index`
 * (GF(2^16), Cantor basis) — exposed for tests and INTEGRATION.md. */
int bfrs_encode_coefficient(size_t original_count, size_t recovery_count, size_t recovery_index,
                            size_t original_index, uint16_t *coef_out);
/* Decode coefficient matrix for an erasure pattern (host logic only).
 * orig_present[k], rec_present[m] are 0/1.  Rows = missing originals
 * ascending; cols = present recovery ascending, then present originals
 * ascending.  Writes rows*cols values row-major if cap allows. */
int bfrs_plan_decode(size_t original_count, size_t recovery_count, const uint8_t *orig_present,
                     const uint8_t *rec_present, uint16_t *coef_out, size_t cap, size_t *rows,
                     size_t *cols);

/* ---- streaming API: mirrors reed_solomon_simd::ReedSolomonEncoder ----- */
/* replaces ReedSolomonEncoder::new (generate.rs:37,84) */
int bfrs_encoder_new(bfrs_ctx *ctx, size_t original_count, size_t recovery_count,
                     size_t shard_bytes, bfrs_encoder **out);
/* replaces add_original_shard (generate.rs:41,44,88); host memory, copied to
 * the device before the call returns (the caller may reuse the buffer). */
int bfrs_encoder_add_original_shard(bfrs_encoder *enc, const uint8_t *shard, size_t len);
/* replaces encode() (generate.rs:47,92) */
int bfrs_encoder_encode(bfrs_encoder *enc);
/* replaces EncoderResult::recovery_iter() (generate.rs:48,96): pointer valid
 * until the next call on this encoder. */
int bfrs_encoder_recovery(bfrs_encoder *enc, size_t index, const uint8_t **data, size_t *len);
void bfrs_encoder_free(bfrs_encoder *enc);

/* ---- streaming API: mirrors reed_solomon_simd::ReedSolomonDecoder ----- */
/* replaces ReedSolomonDecoder::new (recovery.rs:58,152; health.rs:514,613,733) */
int bfrs_decoder_new(bfrs_ctx *ctx, size_t original_count, size_t recovery_count,
                     size_t shard_bytes, bfrs_decoder **out);
/* replaces add_original_shard(index, shard) (recovery.rs:157; health.rs:737) */
int bfrs_decoder_add_original_shard(bfrs_decoder *dec, size_t index, const uint8_t *shard,
                                    size_t len);
/* replaces add_recovery_shard(index, shard) (recovery.rs:61-63,162-164; health.rs:742) */
int bfrs_decoder_add_recovery_shard(bfrs_decoder *dec, size_t index, const uint8_t *shard,
                                    size_t len);
/* replaces decode() (recovery.rs:65,166; health.rs:746) */
int bfrs_decoder_decode(bfrs_decoder *dec);
/* replaces DecoderResult::restored_original(index) (recovery.rs:66-69,167-169):
 * BFRS_E_NOT_RESTORED plays the role of Option::None.  The first call for an
 * index copies that shard to host memory; the pointer is valid until the next
 * add/decode call on this decoder. */
int bfrs_decoder_restored_original(bfrs_decoder *dec, size_t index, const uint8_t **data,
                                   size_t *len);
void bfrs_decoder_free(bfrs_decoder *dec);

/* ---- one-shot host-memory API (host buffers in, host buffers out) ----- */
/* k originals -> m recovery shards; every buffer shard_bytes long, caller-owned. */
int bfrs_encode(bfrs_ctx *ctx, size_t original_count, size_t recovery_count, size_t shard_bytes,
                const uint8_t *const *originals, uint8_t *const *recovery_out);
/* originals[i] == NULL: erased; recovery[j] == NULL: missing.  restored_out[i]
 * is written only where originals[i] == NULL. */
int bfrs_decode(bfrs_ctx *ctx, size_t original_count, size_t recovery_count, size_t shard_bytes,
                const uint8_t *const *originals, const uint8_t *const *recovery,
                uint8_t *const *restored_out);

/* Host-memory batch API (the reference's path starts and ends in host memory:
 * mmap'd files, fs::read).  Same shapes as the device batch API below but
 * every pointer is host memory; shards are streamed through HBM in 64-byte
 * aligned column slabs over several HIP streams so host->device copies,
 * kernels and device->host copies overlap.  Pinned (page-locked) host
 * buffers reach PCIe rate; pageable ones work but go through the runtime's
 * staging.  Blocks until the outputs are in host memory. */
int bfrs_encode_host_batch(bfrs_ctx *ctx, size_t nblocks, const uint32_t *original_counts,
                           size_t recovery_count, size_t shard_bytes,
                           const uint8_t *const *originals, uint8_t *const *recovery_out);
int bfrs_decode_host_batch(bfrs_ctx *ctx, size_t nblocks, const uint32_t *original_counts,
                           size_t recovery_count, size_t shard_bytes,
                           const uint8_t *const *originals, const uint8_t *const *recovery,
                           uint8_t *const *restored_out);

/* The same host-memory batch spread over several contexts from ONE process
 * (BlockFrame is one process: rayon over blocks, src/chunker/commit.rs:391-393;
 * BASELINE configs[3], a 10 GiB archive over 1/2/4/8 GPUs).  ctxs[d] is
 * normally one context per device; context d streams the 64-byte-aligned
 * column stripe d of every shard (the tail chunk in the last stripe) through
 * its own device on a host thread of its own, so any block list balances
 * exactly and no bytes move between devices (the code acts per 64-byte
 * chunk).  Same arguments and results as bfrs_encode_host_batch /
 * bfrs_decode_host_batch; an error names the stripe and device. */
int bfrs_encode_host_batch_multi(bfrs_ctx *const *ctxs, size_t n_ctx, size_t nblocks,
                                 const uint32_t *original_counts, size_t recovery_count,
                                 size_t shard_bytes, const uint8_t *const *originals,
                                 uint8_t *const *recovery_out);
int bfrs_decode_host_batch_multi(bfrs_ctx *const *ctxs, size_t n_ctx, size_t nblocks,
                                 const uint32_t *original_counts, size_t recovery_count,
                                 size_t shard_bytes, const uint8_t *const *originals,
                                 const uint8_t *const *recovery, uint8_t *const *restored_out);

/* ---- device-resident batch API (pointers are device memory) ----------- */
/* Encodes nblocks independent RS blocks in one launch.  Block b has
 * original_counts[b] originals, all blocks share recovery_count and
 * shard_bytes.  d_originals holds sum(original_counts) pointers, block by
 * block; d_recovery holds nblocks*recovery_count pointers.  Pointer arrays
 * are host arrays of device addresses; shard pointers must be 16-byte
 * aligned.  Work is queued on `hip_stream` (a hipStream_t; NULL = HIP's
 * default stream, as in every HIP API) and ordered after earlier work on it. */
int bfrs_encode_batch_dev(bfrs_ctx *ctx, size_t nblocks, const uint32_t *original_counts,
                          size_t recovery_count, size_t shard_bytes,
                          const uint8_t *const *d_originals, uint8_t *const *d_recovery,
                          void *hip_stream);
/* Same shape; NULL entries mark erased originals / missing recovery shards.
 * d_restored holds sum(original_counts) pointers; written where erased. */
int bfrs_decode_batch_dev(bfrs_ctx *ctx, size_t nblocks, const uint32_t *original_counts,
                          size_t recovery_count, size_t shard_bytes,
                          const uint8_t *const *d_originals, const uint8_t *const *d_recovery,
                          uint8_t *const *d_restored, void *hip_stream);

/* ---- BlockFrame wrappers (C++ restatement of the reference functions) -- */
/* Chunker::generate_parity (src/chunker/generate.rs:59-104): pads every
 * segment to the longest one, RS(data_shards, parity_shards) encode.
 * parity_out[p] must hold max(seg_lens) bytes; *parity_len receives it. */
int bfrs_generate_parity(bfrs_ctx *ctx, const uint8_t *const *segments, const size_t *seg_lens,
                         size_t n_segments, size_t data_shards, size_t parity_shards,
                         uint8_t *const *parity_out, size_t *parity_len);
/* Chunker::generate_parity_segmented (generate.rs:26-57): RS(1,3) of the
 * data padded to a multiple of 64.  parity_out[0..3] hold ceil64(len) bytes. */
int bfrs_generate_parity_segmented(bfrs_ctx *ctx, const uint8_t *segment, size_t len,
                                   uint8_t *const *parity_out, size_t *parity_len);
/* recover_segment_rs13 (src/filestore/recovery.rs:43-79).  expected_size ==
 * SIZE_MAX means None.  out must hold the parity length. */
int bfrs_recover_segment_rs13(bfrs_ctx *ctx, const uint8_t *const *parity,
                              const size_t *parity_lens, size_t n_parity, size_t expected_size,
                              uint8_t *out, size_t *out_len);
/* recover_segment_rs30_3 (recovery.rs:118-173): segments[30] with NULL for
 * None, block_parity[3], target index.  out must hold the shard size (its
 * contents are unspecified after an error) and must not overlap any segment
 * or parity buffer (BFRS_E_INVALID_ARGUMENT): it is first-touched while they
 * are staged. */
int bfrs_recover_segment_rs30_3(bfrs_ctx *ctx, const uint8_t *const *segments,
                                const size_t *seg_lens, size_t n_slots,
                                const uint8_t *const *block_parity, const size_t *parity_lens,
                                size_t n_parity, size_t target_index, uint8_t *out,
                                size_t *out_len);

/* ---- Integrity helpers (host) -------------------------------------------- */
/* blake3_hash_bytes (src/utils.rs:22-28): lowercase hex digest + NUL into
 * out65.  threads > 1 hashes independent chunk subtrees in parallel. */
int bfrs_blake3_hex(const uint8_t *data, size_t len, int threads, char *out65);
/* BLAKE3 of n device-resident messages on the GPU (blake3_kernels.hip).
 * d_msgs[i] must be 16-byte aligned (NULL allowed when lens[i] == 0).
 * digests_out: host, n * 32 bytes.  cvs_out (may be NULL): host, n * 32
 * bytes, each message's subtree chaining value, for bfrs_blake3_combine.
 * chunk_offsets (may be NULL = all 0): message i's first BLAKE3 chunk
 * counter.  A part of a larger message hashed at its chunk offset yields the
 * CV of its node in that message's tree (digests_out is then meaningless);
 * at offset 0 it yields the part's own digest.
 * Work is queued on hip_stream (NULL = HIP default) and waited for. */
int bfrs_blake3_batch_dev(bfrs_ctx *ctx, size_t n, const uint8_t *const *d_msgs,
                          const size_t *lens, const uint64_t *chunk_offsets, uint8_t *digests_out,
                          uint8_t *cvs_out, void *hip_stream);
/* Digest of a whole message from the CVs of its n >= 2 consecutive parts,
 * where every part but the last has the same power-of-two number of KiB (the
 * file hash of commit.rs:478 from per-segment CVs of 32 MiB segments). */
int bfrs_blake3_combine(const uint8_t *cvs, size_t n, char *out65);
/* MerkleTree::from_hashes(..).get_root (src/merkle_tree/mod.rs:56-100):
 * `leaves` is n concatenated 64-char hex digests (no separators). */
int bfrs_merkle_root_hex(const char *leaves, size_t n, char *out65);

/* ManifestFile::new + validate (src/merkle_tree/manifest.rs:47-88): parses
 * manifest.json text (BFRS_E_WRAPPER + message on a parse error), sets
 * *valid, and writes the canonical serialisation this library writes (the
 * reference's serde_json layout: compact, keys sorted) into canonical/cap;
 * *needed = its length + 1. */
int bfrs_manifest_check(const char *text, size_t len, int *valid, char *canonical, size_t cap,
                        size_t *needed);

/* ---- Archive pipeline (host, arithmetic on the GPU) ----------------------- */
/* Chunker::commit (src/chunker/commit.rs:593-613): writes
 * {archive_root}/{basename}_{blake3}/ with the reference's layout and
 * manifest.json.  tier 0 picks the tier by size like commit (:596-608);
 * 1/2/3 call commit_tiny (:25) / commit_segmented (:124) / commit_blocked
 * (:314) directly.  segment_size 0 = 32 MiB (src/utils.rs:68).  The archive
 * directory is written to out_dir (NUL-terminated, truncated to out_cap). */
int bfrs_commit(bfrs_ctx *ctx, const char *file_path, const char *archive_root,
                size_t segment_size, int tier, char *out_dir, size_t out_cap);
/* bfrs_commit over several contexts (normally one per device) from one
 * process: a tier-3 file's blocks are dealt round-robin (block b to context
 * b % n_ctx, rayon's independent blocks, commit.rs:391-393), each context
 * runs the commit pipeline of its blocks on a host thread of its own (fill,
 * H2D, encode, device BLAKE3, D2H, file writes).  The archive -- every file
 * and the manifest except time_of_creation -- is byte-identical to
 * bfrs_commit's.  Tiers 1/2 (one RS(1,3) stream, <= 1 GB) run on ctxs[0]. */
int bfrs_commit_multi(bfrs_ctx *const *ctxs, size_t n_ctx, const char *file_path,
                      const char *archive_root, size_t segment_size, int tier, char *out_dir,
                      size_t out_cap);

typedef struct {
  uint64_t blocks_checked;      /* tier 3: blocks; tiers 1/2: segments */
  uint64_t segments_checked;
  uint64_t segments_repaired;   /* missing or BLAKE3-mismatched, restored + written */
  uint64_t parity_repaired;     /* tier 3: parity shards re-encoded + written */
  uint64_t unrecoverable_blocks;
} bfrs_repair_report;
/* FileStore::repair (src/filestore/health.rs:470-495 -> repair_tiny :497,
 * repair_segment :542, repair_blocked :642), with the intended semantics:
 * every missing or corrupt segment of a block is restored by one RS(k,3)
 * decode and written to its own in-block index; corrupt parity is
 * re-encoded.  Blocks with more damage than valid parity are counted, not
 * errors. */
int bfrs_repair(bfrs_ctx *ctx, const char *archive_dir, bfrs_repair_report *report);
/* bfrs_repair over several contexts (normally one per device) from one
 * process: a tier-3 archive's blocks are dealt round-robin (block b to context
 * b % n_ctx, repair_blocked's independent blocks, health.rs:642-765), each
 * context verifying, decoding and writing its blocks on a host thread of its
 * own; the report is the sum.  Tiers 1/2 run on ctxs[0]. */
int bfrs_repair_multi(bfrs_ctx *const *ctxs, size_t n_ctx, const char *archive_dir,
                      bfrs_repair_report *report);

/* FileStore::health_check (src/filestore/health.rs:111-438), intended
 * semantics: every shard is hashed against the manifest (tier 3: device
 * BLAKE3), so corrupt counts like missing; each block (tier 3) or segment
 * (tiers 1/2) is Healthy (all shards valid), Degraded (data valid, some
 * parity not), Recoverable (damaged data <= valid parity) or Unrecoverable.
 * Writes a JSON report with HealthReport's fields (src/filestore/models.rs:
 * 67-82: status, recoverable, missing_data, missing_parity, corrupt_segments,
 * details) plus corrupt_parity and per-unit counts; *needed = length + 1. */
int bfrs_health_check(bfrs_ctx *ctx, const char *archive_dir, char *json_out, size_t cap,
                      size_t *needed);

/* Archive discovery (FileStore, src/filestore/mod.rs:81-154, health.rs:45-74).
 * Every entry of store_root is an archive directory {name}_{hash} whose
 * manifest.json must parse (as FileStore::all_files/get_all; an unreadable
 * one fails the call).  Entries are visited in name order.
 * bfrs_store_list: JSON array of {"file_name", "file_data": {"hash", "path"
 * (the manifest path)}, "dir"} (models.rs File).
 * bfrs_store_find: the archive directory of the first file named file_name;
 * BFRS_E_NOT_FOUND with "File '<name>' not found" otherwise (mod.rs:150-153).
 * bfrs_batch_health_check: BatchHealthReport (models.rs:84-92) as JSON:
 * total_files, healthy, degraded, recoverable, unrecoverable and reports =
 * [[file_name, <bfrs_health_check report>], ...].
 * Output convention as bfrs_health_check: *needed = length + 1. */
int bfrs_store_list(const char *store_root, char *json_out, size_t cap, size_t *needed);
int bfrs_store_find(const char *store_root, const char *file_name, char *dir_out, size_t cap,
                    size_t *needed);
int bfrs_batch_health_check(bfrs_ctx *ctx, const char *store_root, char *json_out, size_t cap,
                            size_t *needed);

/* Read-path core of the FUSE mount (src/mount/filesystem_unix.rs:176-305,
 * src/mount/cache.rs): offset->segment mapping, LRU segment cache,
 * BLAKE3 verification on every miss and GPU reconstruction of a corrupt or
 * missing segment (tier 3: RS(k,3) block decode). */
typedef struct bfrs_archive bfrs_archive;
typedef struct {
  uint64_t hits, misses;
  uint64_t verified;            /* segments loaded that hashed clean (GPU BLAKE3) */
  uint64_t recoveries;          /* decode calls */
  uint64_t recovered_segments;  /* segments restored by those calls */
  uint64_t bytes_served;
  uint64_t prefetched;          /* segments loaded + verified ahead of the reader */
} bfrs_archive_stats;
/* Memory: cached segments live in pinned buffers drawn from a pool the
 * context keeps per segment size and shares between its handles (about
 * cache_segments + 8 buffers per handle open at the same time).  When a
 * handle closes, idle buffers beyond 2 GiB per segment size are unpinned, and
 * the pools no open handle uses keep at most 2 GiB of idle buffers together
 * (the least recently released pools go first); the rest stay for the next
 * handle until bfrs_close.  The tier-3 block reconstructions of all handles
 * of a context share ONE block arena (33 HBM segment slots, 22 pinned),
 * reserved by the first tier-3 handle's prefetch thread and kept until
 * bfrs_close.  Each handle has one HBM segment buffer per verification lane
 * (prefetch workers + 1), freed by bfrs_archive_close. */
int bfrs_archive_open(bfrs_ctx *ctx, const char *archive_dir, size_t cache_segments,
                      int write_back, bfrs_archive **out);
int bfrs_archive_size(bfrs_archive *a, uint64_t *size);
/* The mount's getattr / read geometry of an archive directory (host only, no
 * context): the manifest's size, tier and segment size
 * (src/mount/filesystem_unix.rs:153-174 get_file_attr, :428-434 read), with
 * the derived segment and block counts.  The manifest is validated first
 * (tier 1..3, size <= 2^50, 0 < segment_size <= 2^36 for tiers 2/3, one
 * manifest entry per segment / block of the right shape); a damaged or
 * hostile manifest fails with BFRS_E_WRAPPER, never a crash. */
typedef struct {
  uint64_t size, segment_size, segments, blocks;
  int32_t tier, reserved;
} bfrs_archive_attr;
int bfrs_archive_stat(const char *archive_dir, bfrs_archive_attr *out);
/* Reads up to len bytes at offset (clamped at EOF; *nread = bytes copied). */
int bfrs_archive_read(bfrs_archive *a, uint64_t offset, size_t len, uint8_t *out, size_t *nread);
int bfrs_archive_stats_get(bfrs_archive *a, bfrs_archive_stats *out);
void bfrs_archive_close(bfrs_archive *a);

#ifdef __cplusplus
}
#endif
#endif /* BFRS_H */
