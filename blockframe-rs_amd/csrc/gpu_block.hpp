// gpu_block.hpp — one tier-3 RS block staged through pinned host memory into
// HBM, verified with the device BLAKE3, decoded / re-encoded in place.
//
// The reference reads a block's shards into Vec<u8>s, hashes each on the CPU
// and calls reed-solomon-simd (health.rs:642-765, recovery.rs:118-173).  Here
// a block of k segments + 3 parity shards occupies k+3 equal slots of an
// Arena: the files are read straight into pinned slots (one H2D copy of the
// whole block), every shard is hashed in one device BLAKE3 call, the decode
// writes restored segments over their own (erased) device slots, and the
// restored bytes are re-hashed on the device before anything reaches disk.
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "archive_io.hpp"
#include "runtime.hpp"

namespace bfrs {

// Pinned host slots and device slots of equal size (grow-only).
struct Arena {
  size_t slot = 0, nslots = 0;
  uint8_t *h = nullptr, *d = nullptr;
  Arena() = default;
  Arena(const Arena &) = delete;
  Arena &operator=(const Arena &) = delete;
  ~Arena();
  int reserve(size_t slot_bytes, size_t n);
  uint8_t *hs(size_t i) const { return h + i * slot; }
  uint8_t *ds(size_t i) const { return d + i * slot; }
};

// Device BLAKE3 -> lowercase hex digests (on `stream`, default the context's;
// synchronises it).  The context's hash_mu is held throughout, so callers
// synchronise their own copies first rather than make it wait behind them.
int gpu_hash_hex(bfrs_ctx *ctx, const std::vector<const uint8_t *> &d_msgs,
                 const std::vector<size_t> &lens, std::vector<std::string> *hex,
                 const uint64_t *chunk_offsets = nullptr, std::vector<uint8_t> *cvs = nullptr,
                 hipStream_t stream = nullptr);

// The context's staging arenas (Context::staging): archive calls on one
// context take `mu` for their duration and use a[0..1] as block arenas and
// a[2..3] as parity buffers.  Arenas grow and are never shrunk.
struct StagingCache {
  std::mutex mu;
  Arena a[4];
  // Pinned segment buffers of the read handles (archive.cpp PinnedPool,
  // type-erased, keyed by buffer size), shared by every handle of the
  // context and kept until bfrs_close: pinning a 32 MiB buffer costs about
  // as much as reading and verifying the segment it holds.  pools_mu only.
  std::mutex pools_mu;
  std::map<size_t, std::shared_ptr<void>> seg_pools;
};
StagingCache &staging(bfrs_ctx *ctx);

// State of tier-3 block b in an Arena: slots [0, k) segments, [k, k+3) parity.
struct BlockState {
  size_t b = 0, k = 0, shard = 0;
  std::vector<size_t> lens;            // unpadded segment lengths
  std::vector<uint8_t> seg_ok, par_ok;  // present and matching the manifest
  size_t damaged_segments() const;
  size_t valid_parity() const;
};

// Reads block b's files into the arena's pinned slots (segments zero-padded
// to the shard size), copies the block to HBM and verifies every shard
// against the manifest with the device BLAKE3.  Each shard's H2D copy is
// queued as soon as its file is read, so the copies overlap the other reads.
int load_block(bfrs_ctx *ctx, const Geometry &g, size_t b, Arena &a, BlockState *st);
// RS(k,3)-decodes every damaged segment into its own device slot, re-verifies
// the restored bytes on the device and copies them to the pinned slots, or,
// where host_out[s] is given (pinned, >= lens[s] bytes), straight there.
// Returns the number restored, BFRS_E_NOT_ENOUGH_SHARDS if the block has more
// damage than valid parity, or another error.
int restore_block(bfrs_ctx *ctx, const Geometry &g, Arena &a, BlockState &st,
                  const std::vector<uint8_t *> *host_out = nullptr);
// Re-encodes the 3 parity shards from the (whole) data on the device,
// verifies them against the manifest and copies them to the pinned slots.
int reencode_parity(bfrs_ctx *ctx, const Geometry &g, Arena &a, BlockState &st);

}  // namespace bfrs
