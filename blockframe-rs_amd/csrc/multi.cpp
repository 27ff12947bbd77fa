// multi.cpp — one process driving several devices (BASELINE configs[3]'s
// 10 GiB archive over 1/2/4/8 GPUs, from host memory).
//
// BlockFrame is one Rust process whose rayon workers take independent blocks
// (src/chunker/commit.rs:391-393).  The host-memory batch calls here spread one
// batch over several contexts -- normally one per device -- each context
// streaming its share through its own HBM, streams and pinned path on a host
// thread of its own.  No bytes move between devices: the code acts per
// 64-byte chunk, so device d takes the 64-byte-aligned column
// stripe d of every shard (bfrs/parallel.py::stripe_ranges), which balances
// any block list exactly.
#include <algorithm>
#include <thread>
#include <vector>

#include "runtime.hpp"

using namespace bfrs;

namespace {

// [start, end) of stripe g of n over a shard, 64-byte aligned; the tail chunk
// (shard_bytes % 64) goes to the last stripe (parallel.py::stripe_ranges).
void stripe_range(size_t shard_bytes, size_t n, size_t g, size_t *start, size_t *end) {
  const size_t chunks = shard_bytes / 64;
  *start = chunks * g / n * 64;
  *end = g + 1 == n ? shard_bytes : chunks * (g + 1) / n * 64;
}

struct Share {
  bfrs_ctx *ctx = nullptr;
  size_t lo = 0, width = 0;
  std::vector<const uint8_t *> orig, rec;
  std::vector<uint8_t *> out;
  int rc = BFRS_OK;
  std::string err;
};

int run_multi(bool decode, bfrs_ctx *const *ctxs, size_t n_ctx, size_t nblocks,
              const uint32_t *ks, size_t m, size_t shard_bytes, const uint8_t *const *orig,
              const uint8_t *const *rec, uint8_t *const *out) {
  if (!ctxs || n_ctx == 0) return set_error(BFRS_E_INVALID_ARGUMENT, "multi batch: no contexts");
  for (size_t d = 0; d < n_ctx; ++d)
    if (!ctxs[d]) return set_error(BFRS_E_INVALID_ARGUMENT, "multi batch: NULL context");
  int rc = check_host_batch(ctxs[0], nblocks, ks, m, shard_bytes, decode, orig, rec, out);
  if (rc || nblocks == 0) return rc;
  size_t n_orig = 0;
  for (size_t b = 0; b < nblocks; ++b) n_orig += ks[b];
  const size_t n_out = decode ? n_orig : nblocks * m;
  // shares: the stripes with at least one whole chunk (a shard narrower than
  // n_ctx chunks leaves the last contexts idle)
  std::vector<Share> shares;
  for (size_t d = 0; d < n_ctx; ++d) {
    Share s;
    size_t end;
    stripe_range(shard_bytes, n_ctx, d, &s.lo, &end);
    s.width = end - s.lo;
    if (!s.width) continue;
    s.ctx = ctxs[d];
    auto at = [&](const uint8_t *p) { return p ? p + s.lo : nullptr; };
    for (size_t i = 0; i < n_orig; ++i) s.orig.push_back(at(orig[i]));
    if (decode)
      for (size_t j = 0; j < nblocks * m; ++j) s.rec.push_back(at(rec[j]));
    for (size_t i = 0; i < n_out; ++i) s.out.push_back(out[i] ? out[i] + s.lo : nullptr);
    shares.push_back(std::move(s));
  }
  auto work = [&](Share &s) {
    Context &c = s.ctx->impl;
    if (hipSetDevice(c.device) != hipSuccess) {
      s.rc = set_error(BFRS_E_HIP, "multi batch: hipSetDevice failed");
    } else {
      try {
        s.rc = c.run_host(decode, nblocks, ks, m, s.width, s.orig.data(),
                          decode ? s.rec.data() : nullptr, s.out.data());
      } catch (const std::bad_alloc &) {
        s.rc = set_error(BFRS_E_NOMEM, "host memory allocation failed");
      } catch (const std::exception &e) {
        s.rc = set_error(BFRS_E_WRAPPER, std::string("internal error: ") + e.what());
      }
    }
    if (s.rc) s.err = bfrs_last_error();  // thread-local: carried back to the caller
  };
  // one host thread per further context; share 0 runs on the calling thread.
  // A thread that cannot be started leaves its share to the caller, after.
  std::vector<std::thread> th;
  std::vector<Share *> inline_shares;
  for (size_t i = 1; i < shares.size(); ++i) {
    try {
      th.emplace_back(work, std::ref(shares[i]));
    } catch (...) {
      inline_shares.push_back(&shares[i]);
    }
  }
  int prev = -1;
  (void)hipGetDevice(&prev);
  work(shares[0]);
  for (Share *s : inline_shares) work(*s);
  for (auto &t : th) t.join();
  if (prev >= 0) (void)hipSetDevice(prev);
  for (size_t i = 0; i < shares.size(); ++i)
    if (shares[i].rc)
      return set_error(shares[i].rc, "stripe " + std::to_string(i) + " (device " +
                                         std::to_string(shares[i].ctx->impl.device) +
                                         "): " + shares[i].err);
  return BFRS_OK;
}

}  // namespace

extern "C" {

int bfrs_encode_host_batch_multi(bfrs_ctx *const *ctxs, size_t n_ctx, size_t nblocks,
                                 const uint32_t *original_counts, size_t recovery_count,
                                 size_t shard_bytes, const uint8_t *const *originals,
                                 uint8_t *const *recovery_out) {
  BFRS_API_BEGIN
  return run_multi(false, ctxs, n_ctx, nblocks, original_counts, recovery_count, shard_bytes,
                   originals, nullptr, recovery_out);
  BFRS_API_END
}

int bfrs_decode_host_batch_multi(bfrs_ctx *const *ctxs, size_t n_ctx, size_t nblocks,
                                 const uint32_t *original_counts, size_t recovery_count,
                                 size_t shard_bytes, const uint8_t *const *originals,
                                 const uint8_t *const *recovery, uint8_t *const *restored_out) {
  BFRS_API_BEGIN
  return run_multi(true, ctxs, n_ctx, nblocks, original_counts, recovery_count, shard_bytes,
                   originals, recovery, restored_out);
  BFRS_API_END
}

}  // extern "C"
