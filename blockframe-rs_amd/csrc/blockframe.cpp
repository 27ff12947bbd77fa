// blockframe.cpp — C++ restatement of the BlockFrame functions that sit on the
// RS codec, rewired onto the HIP path.  Same argument meaning, same checks in
// the same order, same error wording as the reference:
//   Chunker::generate_parity            src/chunker/generate.rs:59-104
//   Chunker::generate_parity_segmented  src/chunker/generate.rs:26-57
//   recover_segment_rs13                src/filestore/recovery.rs:43-79
//   recover_segment_rs30_3              src/filestore/recovery.rs:118-173
// The reference's println! calls inside the hot path (generate.rs:51-54,
// 98-101) are deliberately not reproduced.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <thread>

#include "runtime.hpp"
#include "knobs.hpp"

using namespace bfrs;

namespace {

int wrapper_error(const std::string &msg) { return set_error(BFRS_E_WRAPPER, msg); }

// First-touch of the caller's output buffer on a helper thread while the
// input shards stream to the device (recover_segment_rs30_3: one 32 MiB
// shard).  The reference's outputs are fresh Vecs (recovery.rs:167-169), and
// faulting fresh pages inside a D2H runs at a fraction of the link rate; done
// here the faults overlap the PCIe-bound H2D.  The bytes written are
// overwritten by the D2H.  (generate_parity's three outputs take the pinned
// rows + threaded copy-out instead: codec_objects.cpp)
class Prefault {
 public:
  Prefault(uint8_t *const *bufs, size_t n, size_t len) {
    auto touch = [bufs, n, len] {
      for (size_t j = 0; j < n; ++j) prefault_range(bufs[j], len);
    };
    try {
      th_ = std::thread(touch);
    } catch (...) {  // no thread: the D2H faults the pages itself
    }
  }
  void join() {
    if (th_.joinable()) th_.join();
  }
  ~Prefault() { join(); }

 private:
  std::thread th_;
};

// [a, a + na) and [b, b + nb) share a byte.
bool overlaps(const uint8_t *a, size_t na, const uint8_t *b, size_t nb) {
  if (!a || !b || !na || !nb) return false;
  const auto x = reinterpret_cast<uintptr_t>(a), y = reinterpret_cast<uintptr_t>(b);
  return x < y + nb && y < x + na;
}

// The slab-pipelined generate_parity (encoder_encode_slabs): pinned staging,
// shards of >= 16 MiB (at least two ~8 MiB slabs); BFRS_WRAPPER_SLABS=0
// turns it off (A/B).
bool slab_wrapper_ok(bfrs_ctx *ctx, const uint8_t *const *segs, size_t n, size_t shard,
                     bool allow_missing = false) {
  static const bool on = [] {
    const char *e = BFRS_AB_KNOB("BFRS_WRAPPER_SLABS");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  if (!on || shard < (size_t(16) << 20) || ctx->impl.codec_pool->staging != Staging::kPinned)
    return false;
  for (size_t i = 0; i < n; ++i)
    if (!segs[i] && !allow_missing) return false;
  return true;
}

// RAII holders for the streaming objects.
struct Enc {
  bfrs_encoder *p = nullptr;
  ~Enc() { bfrs_encoder_free(p); }
};
struct Dec {
  bfrs_decoder *p = nullptr;
  ~Dec() { bfrs_decoder_free(p); }
};

}  // namespace

extern "C" {

int bfrs_generate_parity(bfrs_ctx *ctx, const uint8_t *const *segments, const size_t *seg_lens,
                         size_t n_segments, size_t data_shards, size_t parity_shards,
                         uint8_t *const *parity_out, size_t *parity_len) {
  BFRS_API_BEGIN
  if (!ctx || (n_segments && (!segments || !seg_lens)) || !parity_len)
    return set_error(BFRS_E_INVALID_ARGUMENT, "generate_parity: NULL argument");
  // generate.rs:66-72 — max chunk size, error on empty input
  if (n_segments == 0) return wrapper_error("No chunks provided");
  size_t max_len = 0;
  for (size_t i = 0; i < n_segments; ++i) max_len = std::max(max_len, seg_lens[i]);
  *parity_len = max_len;
  // generate.rs:84 — ReedSolomonEncoder::new(data_shards, parity_shards, max)
  Enc enc;
  int rc = bfrs_encoder_new(ctx, data_shards, parity_shards, max_len, &enc.p);
  if (rc) return rc;
  if (!parity_out) return set_error(BFRS_E_INVALID_ARGUMENT, "generate_parity: parity_out NULL");
  for (size_t j = 0; j < parity_shards; ++j)
    if (!parity_out[j]) return set_error(BFRS_E_INVALID_ARGUMENT, "parity buffer is NULL");
  // A whole block of pageable segments (BlockFrame's case): slab-pipelined,
  // so each column slab's kernel and D2H run while the next slab's segments
  // are copied and DMA'd.  A segment count other than
  // data_shards takes the adds below, which report the crate's errors.
  if (n_segments == data_shards && slab_wrapper_ok(ctx, segments, n_segments, max_len))
    return encoder_encode_slabs(enc.p, segments, seg_lens, parity_out);
  // generate.rs:75-82 + 87-89 — zero-pad each segment to max_len and add it
  const auto t_add = std::chrono::steady_clock::now();
  std::vector<uint8_t> padded;
  for (size_t i = 0; i < n_segments; ++i) {
    const uint8_t *src = segments[i];
    if (seg_lens[i] < max_len) {
      padded.assign(max_len, 0);
      if (seg_lens[i]) std::memcpy(padded.data(), segments[i], seg_lens[i]);
      src = padded.data();
    }
    if ((rc = bfrs_encoder_add_original_shard(enc.p, src, max_len))) return rc;
  }
  if (BFRS_AB_KNOB("BFRS_TRACE"))  // measurement aid (tools/crate_probe.py)
    std::fprintf(stderr, "bfrs trace: generate_parity adds %.3f ms\n",
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_add)
                     .count());
  // generate.rs:92 + 95-96: encode; the recovery shards come back into the
  // slot's pinned rows and are copied out on several threads, which is also
  // where a fresh Vec's pages fault in (the reference's to_vec copies)
  return encoder_encode_to_host(enc.p, parity_out);
  BFRS_API_END
}

int bfrs_generate_parity_segmented(bfrs_ctx *ctx, const uint8_t *segment, size_t len,
                                   uint8_t *const *parity_out, size_t *parity_len) {
  BFRS_API_BEGIN
  if (!ctx || (len && !segment) || !parity_len)
    return set_error(BFRS_E_INVALID_ARGUMENT, "generate_parity_segmented: NULL argument");
  // generate.rs:31-37 — RS(1,3) over the data padded to a multiple of 64
  const size_t padded = (len + 63) / 64 * 64;
  *parity_len = padded;
  Enc enc;
  int rc = bfrs_encoder_new(ctx, 1, 3, padded, &enc.p);
  if (rc) return rc;
  if (!parity_out) return set_error(BFRS_E_INVALID_ARGUMENT, "parity_out is NULL");
  if (len < padded) {  // generate.rs:39-42
    std::vector<uint8_t> buf(padded, 0);
    std::memcpy(buf.data(), segment, len);
    rc = bfrs_encoder_add_original_shard(enc.p, buf.data(), padded);
  } else {
    rc = bfrs_encoder_add_original_shard(enc.p, segment, padded);
  }
  if (rc) return rc;
  for (size_t j = 0; j < 3; ++j)
    if (!parity_out[j]) return set_error(BFRS_E_INVALID_ARGUMENT, "parity buffer is NULL");
  return encoder_encode_to_host(enc.p, parity_out);
  BFRS_API_END
}

int bfrs_recover_segment_rs13(bfrs_ctx *ctx, const uint8_t *const *parity,
                              const size_t *parity_lens, size_t n_parity, size_t expected_size,
                              uint8_t *out, size_t *out_len) {
  BFRS_API_BEGIN
  if (!ctx || !out_len || (n_parity && (!parity || !parity_lens)))
    return set_error(BFRS_E_INVALID_ARGUMENT, "recover_segment_rs13: NULL argument");
  if (n_parity != 3) return wrapper_error("Exactly 3 parity shards required for RS(1,3)");
  const size_t shard_size = parity_lens[0];
  for (size_t j = 0; j < 3; ++j)
    if (parity_lens[j] != shard_size) return wrapper_error("All parity shards must be the same size");
  Dec dec;
  int rc = bfrs_decoder_new(ctx, 1, 3, shard_size, &dec.p);
  if (rc) return rc;
  for (size_t j = 0; j < 3; ++j)
    if ((rc = bfrs_decoder_add_recovery_shard(dec.p, j, parity[j], shard_size))) return rc;
  if ((rc = bfrs_decoder_decode(dec.p))) return rc;
  const uint8_t *data;
  size_t len;
  if (bfrs_decoder_restored_original(dec.p, 0, &data, &len))
    return wrapper_error("Recovery failed");
  // recovery.rs:71-76 — truncate to Some(expected_size) if shorter
  if (expected_size != SIZE_MAX && len > expected_size) len = expected_size;
  if (!out) return set_error(BFRS_E_INVALID_ARGUMENT, "out is NULL");
  host_copy(out, data, len);
  *out_len = len;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_recover_segment_rs30_3(bfrs_ctx *ctx, const uint8_t *const *segments,
                                const size_t *seg_lens, size_t n_slots,
                                const uint8_t *const *block_parity, const size_t *parity_lens,
                                size_t n_parity, size_t target_index, uint8_t *out,
                                size_t *out_len) {
  BFRS_API_BEGIN
  if (!ctx || !out_len || (n_slots && (!segments || !seg_lens)) ||
      (n_parity && (!block_parity || !parity_lens)))
    return set_error(BFRS_E_INVALID_ARGUMENT, "recover_segment_rs30_3: NULL argument");
  // recovery.rs:123-133
  if (n_slots != 30) return wrapper_error("Exactly 30 segment slots required for RS(30,3)");
  if (n_parity != 3) return wrapper_error("Exactly 3 block parity shards required for RS(30,3)");
  if (target_index >= 30) return wrapper_error("Target index must be 0-29");
  // recovery.rs:136-143
  size_t missing = 0;
  for (size_t i = 0; i < 30; ++i) missing += segments[i] == nullptr;
  if (missing > 3) {
    std::ostringstream os;
    os << "Too many missing segments: " << missing << " (max 3 for RS(30,3))";
    return wrapper_error(os.str());
  }
  // recovery.rs:146-150 — shard size from the first present segment, else parity
  size_t shard_size = parity_lens[0];
  for (size_t i = 0; i < 30; ++i)
    if (segments[i]) {
      shard_size = seg_lens[i];
      break;
    }
  Dec dec;
  int rc = bfrs_decoder_new(ctx, 30, 3, shard_size, &dec.p);
  if (rc) return rc;
  if (!out) return set_error(BFRS_E_INVALID_ARGUMENT, "out is NULL");
  // out is first-touched (zeroed) by a helper thread while the inputs are
  // still being staged, so it must not share bytes with any of them (the
  // reference's output is a fresh Vec; include/bfrs.h states the rule)
  for (size_t i = 0; i < 30; ++i)
    if (overlaps(out, shard_size, segments[i], segments[i] ? seg_lens[i] : 0))
      return set_error(BFRS_E_INVALID_ARGUMENT, "recover_segment_rs30_3: out overlaps a segment");
  for (size_t j = 0; j < 3; ++j)
    if (overlaps(out, shard_size, block_parity[j], parity_lens[j]))
      return set_error(BFRS_E_INVALID_ARGUMENT,
                       "recover_segment_rs30_3: out overlaps a parity shard");
  // Pageable inputs of one size, the target erased, all parity present (the
  // reference's case): slab-pipelined, each slab's decode and the target's
  // D2H overlapping the next slab's copies.  Anything else takes the adds,
  // which report the crate's errors.
  {
    bool slabs = !segments[target_index] && missing >= 1 &&
                 slab_wrapper_ok(ctx, segments, 30, shard_size, true);
    for (size_t i = 0; slabs && i < 30; ++i)
      if (segments[i] && seg_lens[i] != shard_size) slabs = false;
    for (size_t j = 0; slabs && j < 3; ++j)
      if (!block_parity[j] || parity_lens[j] != shard_size) slabs = false;
    if (slabs) {
      if ((rc = decoder_restore_slabs(dec.p, segments, block_parity, target_index, out))) return rc;
      *out_len = shard_size;
      return BFRS_OK;
    }
  }
  uint8_t *const outs[1] = {out};
  Prefault pf(outs, 1, shard_size);
  for (size_t i = 0; i < 30; ++i)
    if (segments[i] && (rc = bfrs_decoder_add_original_shard(dec.p, i, segments[i], seg_lens[i])))
      return rc;
  for (size_t j = 0; j < 3; ++j)
    if ((rc = bfrs_decoder_add_recovery_shard(dec.p, j, block_parity[j], parity_lens[j])))
      return rc;
  if ((rc = bfrs_decoder_decode(dec.p))) return rc;
  pf.join();
  // recovery.rs:166-170: only the target leaves the device, straight into out
  if (decoder_restored_to_host(dec.p, target_index, out))
    return wrapper_error("Failed to restore target segment");
  *out_len = shard_size;
  return BFRS_OK;
  BFRS_API_END
}

}  // extern "C"
