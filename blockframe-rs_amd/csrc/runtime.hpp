// runtime.hpp — internal C++ runtime behind include/bfrs.h.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <new>
#include <stdexcept>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bfrs.h"
#include "host_copy.hpp"
#include "kernels.hpp"
#include "plan.hpp"

namespace bfrs {

// Shard pitch for multi-shard allocations (bfrs_shard_pitch):
// >= 1 MiB shards get a pitch = 12 KiB (mod 64 KiB) so that one column of
// many shards does not alias onto the same HBM channels.
inline size_t shard_pitch(size_t shard_bytes) {
  size_t p = (shard_bytes + 255) / 256 * 256;
  if (shard_bytes < (size_t(1) << 20)) return p;
  p = (p + 4095) / 4096 * 4096;
  return p + (12288 + 65536 - p % 65536) % 65536;
}

// Makes `dev` current for a scope and restores the caller's device after it:
// the last codec object of a pool may be freed on any thread (a GC running
// in a worker bound to another GPU), which must not be left switched to this
// pool's device.
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Pinned host memory of the staging buffers (archive segment pools and block
// arenas): anonymous mmap, 2 MiB aligned, MADV_HUGEPAGE, populated, then
// hipHostRegister (portable).  hipHostMalloc pinned 5.3-7.0 GB/s on the
// boxes -- faulting in 4 KiB pages is most of its cost -- against 22.6 GB/s
// this way, whose register step alone runs ~390 GB/s (tools/pin_probe.py,
// profiles/r06/pin/), so a first commit or read on a context waits a quarter
// as long for its staging.  Falls back to hipHostMalloc when
// any step fails.  pinned_free frees by what pinned_alloc did (it records each mapping's length).
void *pinned_alloc(size_t bytes);
void pinned_free(void *p, size_t bytes);

// Thread-local error reporting (bfrs_last_error).
int set_error(int code, const std::string &msg);
int hip_error(hipError_t e, const char *what);

// Every int-returning C entry point runs inside BFRS_API_BEGIN/END: a C++
// exception (allocation failure, malformed input reaching an .at()) becomes
// an error code and never crosses the C-ABI (bfrs.h: never aborts).
#define BFRS_API_BEGIN try {
#define BFRS_API_END                                                             \
  }                                                                              \
  catch (const std::bad_alloc &) {                                               \
    return bfrs::set_error(BFRS_E_NOMEM, "host memory allocation failed");       \
  }                                                                              \
  catch (const std::exception &ex_) {                                            \
    return bfrs::set_error(BFRS_E_WRAPPER, std::string("internal error: ") + ex_.what()); \
  }                                                                              \
  catch (...) {                                                                  \
    return bfrs::set_error(BFRS_E_WRAPPER, "internal error");                    \
  }

#define HIP_TRY(expr)                                   \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return bfrs::hip_error(e_, #expr); \
  } while (0)

// One kernel pass of a plan: outputs [r0, r1) x inputs [c0, c1) with its
// nibble tables resident on the device.
struct PlanPass {
  uint32_t r0, r1, c0, c1;
  uint32_t phase;  // input-group index; phase > 0 accumulates
  const uint2 *d_table = nullptr;
  // every coefficient lies in the GF(2^8) subfield (values < 256):
  // the products of a symbol's low byte then have a zero high byte, so the
  // kernel reads those table entries as 4 bytes and skips their high XORs
  bool subfield = false;
};

// A coefficient plan for one (k, m, erasure pattern), tables on device.
struct Plan {
  CoefMatrix coef;
  std::vector<PlanPass> passes;
  uint32_t n_phases = 0;
  void *d_tables = nullptr;  // one allocation for all pass tables
  uint64_t last_use = 0;     // plan-cache LRU tick (under Context::mu)
  ~Plan();
};
using PlanRef = std::shared_ptr<const Plan>;

// One RS block in a batch: device addresses of its pass inputs/outputs.  The
// plan reference keeps its device tables alive while the batch is queued
// (the cache evicts only plans nobody holds, after a device synchronize).
struct BlockIO {
  PlanRef plan;
  std::vector<const uint8_t *> in;  // plan.coef.cols device pointers
  std::vector<uint8_t *> out;       // plan.coef.rows device pointers
};

// Device + pinned-host shard slots of the streaming codec objects
// (bfrs_encoder / bfrs_decoder), each with its own stream so objects on
// different threads overlap.  Cached per context (CodecPool), so an encoder
// per block -- BlockFrame's pattern, generate.rs:84 -- allocates and pins
// nothing after the first few blocks.
struct CodecSlot {
  void *d = nullptr;     // nshards x stride bytes of HBM
  uint8_t *h = nullptr;  // nshards x stride bytes of pinned host memory
  size_t stride = 0, nshards = 0;
  hipStream_t stream = nullptr;  // the pool's stream this slot's kernels run on (or its own)
  bool own_stream = false;       // BFRS_CODEC_STREAMS=0: one stream per slot
  int stream_idx = -1;           // index into CodecPool::streams while acquired
  // the last H2D, kernel and D2H this slot queued (each on its own stream)
  hipEvent_t ev_h2d = nullptr, ev_k = nullptr, ev_d2h = nullptr;
  // second stream of the slab-pipelined wrapper encode (encoder_encode_slabs):
  // kernels and D2H of slab s run on it while slab s + 1's H2D runs on
  // `stream`; created on first use
  hipStream_t aux = nullptr;
  // Waits for this slot's work queued so far (not for later work of other
  // slots sharing a stream).
  int sync();
  ~CodecSlot();
};

// How add_*_shard moves a caller's shard to the device (BFRS_CODEC_STAGING):
//   kPinned: memcpy into the slot's pinned row on up to 8 threads, then an
//            async H2D, so copying shard i+1 overlaps the DMA of shard i
//            (default);
//   kDirect: hipMemcpyAsync straight from the caller's pageable buffer, then
//            a stream sync.  Equal on buffers HIP has seen before, but the
//            runtime locks a new buffer's pages on first use, and BlockFrame
//            hands over new mmap'd segments for every block: measured 27-51 ms
//            against 26-28 ms for kPinned per 32 MiB RS(30,3) block in the
//            bench process.
// Either way the caller's buffer is free again when add returns.
enum class Staging { kDirect, kPinned };

// The slot cache of one context.  Shared (shared_ptr) by the context and by
// every live codec object, so an object freed after bfrs_close still returns
// or frees its slot safely; the pool goes away with the last of them.
//
// Streams (round 4): by default every slot has a stream
// of its own and runs its copies and kernel on it (rounds 2-3).
// BFRS_CODEC_STREAMS=n > 0 instead shares n streams created with the
// context (an acquired slot takes the one with the fewest live slots), and
// BFRS_CODEC_COPIES=stream sends every object's H2D / D2H through two FIFO
// copy streams with the kernels waiting on per-slot events.  Measured in the
// bench process over two boxes, neither option was consistently faster than
// one stream per slot, so they stay options.
struct CodecPool {
  int device = 0;
  Staging staging = Staging::kPinned;
  std::mutex mu;
  std::vector<std::unique_ptr<CodecSlot>> free;
  size_t cached = 2;  // BFRS_CODEC_SLOTS: idle slots kept (0 = none)
  std::vector<hipStream_t> streams;  // shared codec streams (empty: one per slot)
  std::vector<int> users;            // live slots per shared stream
  // BFRS_CODEC_COPIES=stream (default): every object's H2D copies go through
  // one stream and its D2H copies through another, in FIFO order, and the
  // kernels wait on events; =slot: copies on the object's own kernel stream
  hipStream_t h2d = nullptr, d2h = nullptr;
  int init_streams(size_t n, bool copy_streams);
  int acquire(size_t nshards, size_t shard_bytes, std::unique_ptr<CodecSlot> *out);
  void release(std::unique_ptr<CodecSlot> slot);
  ~CodecPool();
};

struct Context {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;  // guards the plan cache (shared by every thread using the context)
  std::map<std::string, std::shared_ptr<Plan>> plans;
  uint64_t plan_tick = 0;
  size_t max_plans = 4096;  // BFRS_PLAN_CACHE overrides at bfrs_open (tests)

  // Host-path pipeline: slots of device slab buffers, one stream each.
  // pipe_mu serialises run_host: archive prefetch threads, repair and the
  // owner's host-batch calls may share one context.
  // pipe_slots (default 3; BFRS_PIPE_SLOTS = 2..kPipeSlotsMax, A/B knob):
  // 5-6 slots ran the pinned host batches ~1.5% faster, but 3 is the depth
  // every long soak ran with
  static constexpr int kPipeSlotsMax = 6;
  int pipe_slots = 3;
  std::mutex pipe_mu;
  hipStream_t pipe_stream[kPipeSlotsMax] = {};
  void *pipe_buf = nullptr;
  size_t pipe_cap = 0;  // bytes per slot

  // Pinned-host + device staging arenas of the archive pipeline
  // (gpu_block.hpp StagingCache, type-erased here), kept across calls:
  // pinning a GiB per commit or repair cost more than the work itself.
  std::shared_ptr<void> staging;
  std::mutex staging_init;

  // Read handles open on this context (bfrs_archive_open).  bfrs_close
  // detaches them first (detach_archives): their prefetch threads are joined
  // and they drop everything of the context, so a handle closed after its
  // context -- a drop order the caller may not control -- touches nothing
  // freed, and no thread of the library outlives the context.
  std::mutex handles_mu;
  std::vector<bfrs_archive *> handles;

  // BLAKE3 (hash_gpu.cpp): device work area + pinned descriptor/result area,
  // guarded by hash_mu (callers on several threads may share a context).
  std::mutex hash_mu;
  void *d_hash = nullptr;
  size_t d_hash_cap = 0;
  void *h_hash = nullptr;
  size_t h_hash_cap = 0;

  // Codec-object slot cache: at most codec_pool->cached idle slots are kept
  // (BFRS_CODEC_SLOTS, default 2), which bounds a context's idle pinned +
  // HBM footprint to 2 x (k + m) x shard_bytes each; slots beyond that are
  // freed on release.  Any number of objects may be alive at once.
  std::shared_ptr<CodecPool> codec_pool = std::make_shared<CodecPool>();

  ~Context();
  int init(int dev);
  // BLAKE3 of n device messages; digests (and subtree CVs if cvs != NULL)
  // land in host memory, n * 32 bytes each.  chunk_offsets (may be NULL)
  // shifts each message's chunk counters (its position in an enclosing
  // message, for CVs).  Synchronises `stream`.
  int blake3_dev(size_t n, const uint8_t *const *d_msgs, const size_t *lens,
                 const uint64_t *chunk_offsets, uint8_t *digests, uint8_t *cvs,
                 hipStream_t stream);
  int get_encode_plan(size_t k, size_t m, PlanRef *out);
  int get_decode_plan(size_t k, size_t m, const std::vector<uint8_t> &orig_present,
                      const std::vector<uint8_t> &rec_present, PlanRef *out);
  // Queue the passes of all blocks (same shard_bytes) on `stream`.  Shards
  // longer than kMaxWindowBytes run as column windows (the kernels address a
  // shard with 32-bit lane offsets).
  static constexpr size_t kMaxWindowBytes = size_t(1) << 31;
  int run_blocks(const std::vector<BlockIO> &blocks, size_t shard_bytes, hipStream_t stream);
  int run_window(const std::vector<BlockIO> &blocks, size_t shard_bytes, hipStream_t stream);
  // Streams host-memory blocks through HBM (see bfrs_encode_host_batch).
  // orig/rec/out are per-block host pointer lists (decode: NULL = missing).
  int run_host(bool decode, size_t nblocks, const uint32_t *ks, size_t m, size_t shard_bytes,
               const uint8_t *const *orig, const uint8_t *const *rec, uint8_t *const *out);
};

// Argument validation shared by every entry point (crate's Error variants).
int check_shape(size_t k, size_t m, size_t shard_bytes);

// Batch entry points with an explicit stream (the C-ABI wrappers pass the
// caller's stream, NULL meaning HIP's default stream; the host-memory API and
// the streaming objects pass the context's own stream).
int encode_batch_on(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                    size_t shard_bytes, const uint8_t *const *d_orig, uint8_t *const *d_rec,
                    hipStream_t s);
int decode_batch_on(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                    size_t shard_bytes, const uint8_t *const *d_orig, const uint8_t *const *d_rec,
                    uint8_t *const *d_restored, hipStream_t s);

}  // namespace bfrs

struct bfrs_ctx {
  bfrs::Context impl;
};

namespace bfrs {
// bfrs_close's first step (archive.cpp): stop and detach every read handle
// still open on the context.
void detach_archives(bfrs_ctx *ctx);
// Pointer and shape checks of the host-memory batch API (one block list).
int check_host_batch(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                     size_t shard_bytes, bool decode, const uint8_t *const *orig,
                     const uint8_t *const *rec, uint8_t *const *out);
// Wrapper fast paths (blockframe.cpp): the owned Vec outputs of
// generate_parity / recover_segment_rs30_3 (generate.rs:95-96,
// recovery.rs:166-170) are filled by D2H straight into the caller's buffers.
// encode into m host buffers of shard_bytes each (object left encoded)
int encoder_encode_to_host(bfrs_encoder *e, uint8_t *const *outs);
// generate_parity's whole block at once, for a fresh encoder: column slabs of
// all k segments staged and DMA'd slab by slab, each slab's kernel and D2H
// overlapping the next slab's copies, the outputs copied out slab by slab.
// lens[i] < shard_bytes: zero padding (generate.rs:75-82).  Same results and
// object state as k adds + encoder_encode_to_host.
int encoder_encode_slabs(bfrs_encoder *e, const uint8_t *const *segs, const size_t *lens,
                         uint8_t *const *outs);
// restored original `index` of a decoded decoder into a host buffer
int decoder_restored_to_host(bfrs_decoder *d, size_t index, uint8_t *out);
// recover_segment_rs30_3's whole decode at once, for a fresh decoder: segs[k]
// (NULL = missing, segs[target] among them), all m parity shards, every
// length shard_bytes; slab-pipelined like encoder_encode_slabs, only the
// target leaves the device.  Object state as after the adds + decode +
// restored_original(target).
int decoder_restore_slabs(bfrs_decoder *d, const uint8_t *const *segs, const uint8_t *const *par,
                          size_t target, uint8_t *out);
}  // namespace bfrs
