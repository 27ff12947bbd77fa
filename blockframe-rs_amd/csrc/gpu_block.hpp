// gpu_block.hpp — one tier-3 RS block staged through pinned host memory into
// HBM, verified with the device BLAKE3, decoded / re-encoded in place.
//
// The reference reads a block's shards into Vec<u8>s, hashes each on the CPU
// and calls reed-solomon-simd (health.rs:642-765, recovery.rs:118-173).  Here
// a block of k segments + 3 parity shards occupies k+3 equal slots of an
// Arena: the files are read straight into pinned slots (each shard's H2D
// queued as its read ends), every shard is hashed in one device BLAKE3 call, the decode
// writes restored segments over their own (erased) device slots, and the
// restored bytes are re-hashed on the device before anything reaches disk.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "archive_io.hpp"
#include "knobs.hpp"
#include "runtime.hpp"

namespace bfrs {

// Pinned host slots and device slots of equal size (grow-only); `parts`
// picks which of the two an arena holds (a regrow keeps what it had).
enum : unsigned { kArenaHost = 1, kArenaDevice = 2, kArenaBoth = 3 };
struct Arena {
  size_t slot = 0, nslots = 0;
  uint8_t *h = nullptr, *d = nullptr;
  Arena() = default;
  Arena(const Arena &) = delete;
  Arena &operator=(const Arena &) = delete;
  ~Arena();
  int reserve(size_t slot_bytes, size_t n, unsigned parts = kArenaBoth);
  uint8_t *hs(size_t i) const { return h + i * slot; }
  uint8_t *ds(size_t i) const { return d + i * slot; }
};

// Pipeline timeline, measurement build only (BFRS_TRACE): [what, unit,
// start us, duration us] events, one line on stderr at the end.  `on` is
// false in libbfrs.so (one branch per event).
struct PipeTrace {
  const bool on = BFRS_AB_KNOB("BFRS_TRACE") != nullptr;
  const std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  std::mutex mu;
  std::vector<std::string> ev;
  long long now_us() const {
    return (long long)std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::steady_clock::now() - t0)
        .count();
  }
  void event(const char *what, size_t unit, long long start) {
    if (!on) return;
    const long long end = now_us();
    std::lock_guard<std::mutex> l(mu);
    ev.push_back(std::string("[\"") + what + "\"," + std::to_string(unit) + "," +
                 std::to_string(start) + "," + std::to_string(end - start) + "]");
  }
  void print(const char *name, int threads) {
    if (!on) return;
    std::string line = std::string(name) + " {\"thr\":" + std::to_string(threads) + ",\"events_us\":[";
    for (size_t i = 0; i < ev.size(); ++i) line += (i ? "," : "") + ev[i];
    line += "],\"total_us\":" + std::to_string(now_us()) + "}\n";
    std::fputs(line.c_str(), stderr);
  }
};

// A tier-3 block's staging: HBM slots for the whole block (k segments + 3
// parity) and the pinned memory the block passes through — a ring the shard
// files are read (or copied) into on their way to HBM, two slots per staging
// thread, and kOutSlots slots for what comes back (restored segments,
// re-encoded parity).  The ring's H2D copies run on its own stream; ring_ev[r]
// marks slot r's last copy.  Pinned: (2 x kRingThreads + kOutSlots) slots,
// not the whole block.
constexpr size_t kRingThreads = 8;
constexpr size_t kOutSlots = 2 * kParity;
struct BlockArena {
  Arena dev, ring, out;
  hipStream_t h2d = nullptr;
  std::vector<hipEvent_t> ring_ev;
  hipEvent_t done = nullptr;  // load_block's end-of-block marker
  BlockArena() = default;
  BlockArena(const BlockArena &) = delete;
  BlockArena &operator=(const BlockArena &) = delete;
  ~BlockArena();
  int reserve(size_t slot_bytes);  // all of it, on the context's device
  // the ring (at least `slots` slots), its stream and events only
  int reserve_ring(size_t slot_bytes, size_t slots = 2 * kRingThreads);
};

// Device BLAKE3 -> lowercase hex digests (on `stream`, default the context's;
// synchronises it).  The context's hash_mu is held throughout, so callers
// synchronise their own copies first rather than make it wait behind them.
int gpu_hash_hex(bfrs_ctx *ctx, const std::vector<const uint8_t *> &d_msgs,
                 const std::vector<size_t> &lens, std::vector<std::string> *hex,
                 const uint64_t *chunk_offsets = nullptr, std::vector<uint8_t> *cvs = nullptr,
                 hipStream_t stream = nullptr);

// The context's staging arenas (Context::staging): archive calls on one
// context take `mu` for their duration.  The RS(1,3) tiers' commit uses
// a[0..1] as device round buffers, blk's ring to fill them and a[2..3] as
// pinned parity buffers.  Tier 3: repair and
// health check use `blk`; the commit uses blk.dev and blk2 as its two device
// block buffers, blk's ring to fill them, blk.out slots [0,3) / [3,6) as the
// pinned parity of the blocks being written, and `filled[i]` to mark a
// block's last H2D.  Arenas grow and are never shrunk.
struct StagingCache {
  std::mutex mu;
  Arena a[4];
  BlockArena blk;
  Arena blk2;  // also repair's and the health check's second block buffer
  hipEvent_t filled[2] = {nullptr, nullptr};
  int commit_events();  // under mu, on the context's device
  StagingCache() = default;
  StagingCache(const StagingCache &) = delete;
  StagingCache &operator=(const StagingCache &) = delete;
  ~StagingCache();
  // Pinned segment buffers of the read handles (archive.cpp PinnedPool,
  // type-erased, keyed by buffer size), shared by every handle of the
  // context: pinning a 32 MiB buffer costs about as much as reading and
  // verifying the segment it holds.  Pools no open handle uses keep at most
  // kIdlePinnedCap idle bytes together (archive.cpp release_pool).
  // pools_mu only; pool_tick orders the pools by their last release.
  std::mutex pools_mu;
  std::map<size_t, std::shared_ptr<void>> seg_pools;
  uint64_t pool_tick = 0;
  // The read handles' tier-3 block reconstructions: ONE arena per context
  // (~1.1 GiB HBM + 22 pinned slots at 32 MiB segments), reserved by the
  // first tier-3 handle's prefetch worker and shared by every handle, one
  // reconstruction at a time (read_mu).  A handle per open file no longer
  // costs an arena each.
  std::mutex read_mu;
  BlockArena read_blk;
};
StagingCache &staging(bfrs_ctx *ctx);

// State of tier-3 block b in an Arena: slots [0, k) segments, [k, k+3) parity.
struct BlockState {
  size_t b = 0, k = 0, shard = 0;
  Arena *dev = nullptr;                // the HBM slots holding the block
  std::vector<uint8_t> readable;       // shard files read whole (load_block_reads)
  std::vector<size_t> lens;            // unpadded segment lengths
  std::vector<uint8_t> seg_ok, par_ok;  // present and matching the manifest
  // where restore_block / reencode_parity left host copies: segment index ->
  // bytes (lens[s]), parity p -> bytes (shard)
  std::vector<std::pair<size_t, const uint8_t *>> restored;
  const uint8_t *parity_host[kParity] = {};
  size_t damaged_segments() const;
  size_t valid_parity() const;
};

// Reads block b's files through the arena's ring (segments zero-padded to
// the shard size) into its HBM slots and verifies every shard against the
// manifest with the device BLAKE3.  Each shard's H2D is queued as soon as
// its file is read, so the copies overlap the other reads.
int load_block(bfrs_ctx *ctx, const Geometry &g, size_t b, BlockArena &a, BlockState *st,
               PipeTrace *pt = nullptr);
// load_block in two phases, so a caller can read block b+1 while block b is
// verified and restored: load_block_reads reads the files through the ring
// into `dev` (a.dev or a second device arena of k + 3 slots) and records
// `done` on the ring's stream after the last H2D; load_block_verify waits
// for `done` and hashes.  Between the two, st->dev must stay untouched.
int load_block_reads(bfrs_ctx *ctx, const Geometry &g, size_t b, BlockArena &a, Arena &dev,
                     hipEvent_t done, BlockState *st, PipeTrace *pt = nullptr);
int load_block_verify(bfrs_ctx *ctx, const Geometry &g, BlockState *st, hipEvent_t done,
                      PipeTrace *pt = nullptr);
// RS(k,3)-decodes every damaged segment into its own device slot, re-verifies
// the restored bytes on the device and copies them to host memory: to
// host_out[s] where given (pinned, >= lens[s] bytes), else to the arena's out
// slots; st.restored lists where each one landed.  Returns the number
// restored, BFRS_E_NOT_ENOUGH_SHARDS if the block has more damage than valid
// parity, or another error.
int restore_block(bfrs_ctx *ctx, const Geometry &g, BlockArena &a, BlockState &st,
                  const std::vector<uint8_t *> *host_out = nullptr);
// Re-encodes the 3 parity shards from the (whole) data on the device,
// verifies them against the manifest and copies them to the arena's out
// slots [kParity, 2 kParity) (st.parity_host).
int reencode_parity(bfrs_ctx *ctx, const Geometry &g, BlockArena &a, BlockState &st);

}  // namespace bfrs
