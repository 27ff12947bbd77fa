// gpu_block.cpp — see gpu_block.hpp.
#include "gpu_block.hpp"

#include "blake3.hpp"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <sstream>

namespace bfrs {

Arena::~Arena() {
  pinned_free(h, slot * nslots);
  if (d) (void)hipFree(d);
}

int Arena::reserve(size_t slot_bytes, size_t n, unsigned parts) {
  slot_bytes = std::max<size_t>(256, shard_pitch(slot_bytes));
  n = std::max<size_t>(1, n);
  const bool have = (!(parts & kArenaHost) || h) && (!(parts & kArenaDevice) || d);
  if (have && slot_bytes <= slot && n <= nslots) return BFRS_OK;
  parts |= (h ? kArenaHost : 0u) | (d ? kArenaDevice : 0u);
  if (h || d) HIP_TRY(hipDeviceSynchronize());
  if (h) {
    pinned_free(h, slot * nslots);
    h = nullptr;
  }
  if (d) {
    HIP_TRY(hipFree(d));
    d = nullptr;
  }
  slot = std::max(slot, slot_bytes);
  nslots = std::max(nslots, n);
  if (parts & kArenaHost) {
    h = static_cast<uint8_t *>(pinned_alloc(slot * nslots));
    if (!h) return set_error(BFRS_E_NOMEM, "pinned staging arena allocation failed");
  }
  if (parts & kArenaDevice) HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d), slot * nslots));
  return BFRS_OK;
}

int BlockArena::reserve(size_t slot_bytes) {
  int rc = dev.reserve(slot_bytes, kBlockSegments + kParity, kArenaDevice);
  if (!rc) rc = out.reserve(slot_bytes, kOutSlots, kArenaHost);
  return rc ? rc : reserve_ring(slot_bytes);
}

int BlockArena::reserve_ring(size_t slot_bytes, size_t slots) {
  int rc = ring.reserve(slot_bytes, slots, kArenaHost);
  if (rc) return rc;
  if (!h2d) HIP_TRY(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
  while (ring_ev.size() < ring.nslots) {
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ring_ev.push_back(e);
  }
  return BFRS_OK;
}

BlockArena::~BlockArena() {
  if (h2d) (void)hipStreamSynchronize(h2d);
  for (hipEvent_t e : ring_ev) (void)hipEventDestroy(e);
  if (done) (void)hipEventDestroy(done);
  if (h2d) (void)hipStreamDestroy(h2d);
}

int StagingCache::commit_events() {
  for (auto &e : filled)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return BFRS_OK;
}

StagingCache::~StagingCache() {
  for (hipEvent_t e : filled)
    if (e) (void)hipEventDestroy(e);
}

StagingCache &staging(bfrs_ctx *ctx) {
  Context &c = ctx->impl;
  std::lock_guard<std::mutex> l(c.staging_init);
  if (!c.staging) c.staging = std::make_shared<StagingCache>();
  return *static_cast<StagingCache *>(c.staging.get());
}

int gpu_hash_hex(bfrs_ctx *ctx, const std::vector<const uint8_t *> &d_msgs,
                 const std::vector<size_t> &lens, std::vector<std::string> *hex,
                 const uint64_t *chunk_offsets, std::vector<uint8_t> *cvs, hipStream_t stream) {
  const size_t n = d_msgs.size();
  std::vector<uint8_t> dig(n * 32);
  if (cvs) cvs->assign(n * 32, 0);
  int rc = ctx->impl.blake3_dev(n, d_msgs.data(), lens.data(), chunk_offsets, dig.data(),
                                cvs ? cvs->data() : nullptr, stream ? stream : ctx->impl.stream);
  if (rc) return rc;
  hex->resize(n);
  for (size_t i = 0; i < n; ++i) (*hex)[i] = to_hex(dig.data() + 32 * i, 32);
  return BFRS_OK;
}

size_t BlockState::damaged_segments() const {
  size_t n = 0;
  for (uint8_t v : seg_ok) n += !v;
  return n;
}

size_t BlockState::valid_parity() const {
  size_t n = 0;
  for (uint8_t v : par_ok) n += v;
  return n;
}

int load_block_reads(bfrs_ctx *ctx, const Geometry &g, size_t b, BlockArena &a, Arena &dev,
                     hipEvent_t done, BlockState *st, PipeTrace *pt) {
  const bool tr = pt && pt->on;
  const long long t0 = tr ? pt->now_us() : 0;
  auto it = g.mf.blocks.find(int64_t(b));
  if (it == g.mf.blocks.end()) return set_error(BFRS_E_WRAPPER, "manifest has no block " + std::to_string(b));
  const BlockHashes &bh = it->second;
  st->b = b;
  st->k = bh.segments.size();
  st->shard = g.block_shard(b);
  st->dev = &dev;
  st->restored.clear();
  for (auto &p : st->parity_host) p = nullptr;
  const size_t k = st->k, shard = st->shard;
  st->lens.resize(k);
  for (size_t s = 0; s < k; ++s) st->lens[s] = g.seg_len(b * kBlockSegments + s);
  Context &c = ctx->impl;
  // the arena's HBM must be on this context's device: the caller may be a
  // read handle's prefetch thread or an API thread bound to another GPU
  HIP_TRY(hipSetDevice(c.device));
  int rc = a.reserve(shard);
  if (!rc) rc = dev.reserve(shard, kBlockSegments + kParity, kArenaDevice);
  if (rc) return rc;
  // thread w reads shards w, w + nthr, ... into its two ring slots in turn;
  // each shard's H2D goes as soon as its read ends
  const size_t n = k + kParity;
  const size_t nthr = std::min<size_t>(kRingThreads, size_t(std::max(1, hw_threads())));
  std::vector<uint8_t> &readable = st->readable;
  readable.assign(n, 0);
  std::atomic<int> hip_rc{int(hipSuccess)};
  auto hip_ok = [&](hipError_t e) {
    int ok = int(hipSuccess);
    if (e != hipSuccess) hip_rc.compare_exchange_strong(ok, int(e));
    return e == hipSuccess;
  };
  parallel_for(nthr, int(nthr), [&](size_t w) {
    if (!hip_ok(hipSetDevice(c.device))) return;
    size_t turn = 0;
    for (size_t i = w; i < n && hip_rc.load() == int(hipSuccess); i += nthr, ++turn) {
      const size_t r = 2 * w + (turn & 1);
      if (!hip_ok(hipEventSynchronize(a.ring_ev[r]))) return;  // slot r's last copy is done
      uint8_t *h = a.ring.hs(r);
      if (i < k) {
        const long long got = read_file_into(t3_seg(g.dir, b, i), h, a.ring.slot);
        readable[i] = got == (long long)st->lens[i];
        if (readable[i] && st->lens[i] < shard)  // generate.rs:75-82 zero padding
          std::memset(h + st->lens[i], 0, shard - st->lens[i]);
      } else {
        readable[i] = read_file_into(t3_par(g.dir, b, i - k), h, a.ring.slot) == (long long)shard;
      }
      if (!readable[i]) continue;  // excluded from the hash and the decode: no copy
      if (!hip_ok(hipMemcpyAsync(dev.ds(i), h, shard, hipMemcpyHostToDevice, a.h2d))) return;
      if (!hip_ok(hipEventRecord(a.ring_ev[r], a.h2d))) return;
    }
  });
  if (hip_rc.load() == int(hipSuccess)) hip_ok(hipEventRecord(done, a.h2d));
  if (tr) pt->event("read", b, t0);
  if (hip_rc.load() != int(hipSuccess)) {
    (void)hipStreamSynchronize(a.h2d);  // nothing may still be reading the ring
    return hip_error(hipError_t(hip_rc.load()), "block shard H2D through the ring");
  }
  return BFRS_OK;
}

int load_block_verify(bfrs_ctx *ctx, const Geometry &g, BlockState *st, hipEvent_t done,
                      PipeTrace *pt) {
  const bool tr = pt && pt->on;
  const long long t1 = tr ? pt->now_us() : 0;
  // the block's copies land before the hash takes hash_mu
  HIP_TRY(hipEventSynchronize(done));
  if (tr) pt->event("h2d_tail", st->b, t1);
  const long long t2 = tr ? pt->now_us() : 0;
  const BlockHashes &bh = g.mf.blocks.at(int64_t(st->b));
  const size_t k = st->k, n = k + kParity;
  std::vector<const uint8_t *> msgs;
  std::vector<size_t> lens, idx;
  for (size_t i = 0; i < n; ++i)
    if (st->readable[i]) {
      msgs.push_back(st->dev->ds(i));
      lens.push_back(i < k ? st->lens[i] : st->shard);
      idx.push_back(i);
    }
  std::vector<std::string> hex;
  int rc = gpu_hash_hex(ctx, msgs, lens, &hex);
  if (rc) return rc;
  if (tr) pt->event("hash", st->b, t2);
  st->seg_ok.assign(k, 0);
  st->par_ok.assign(kParity, 0);
  for (size_t j = 0; j < idx.size(); ++j) {
    const size_t i = idx[j];
    if (i < k)
      st->seg_ok[i] = hex[j] == bh.segments[i];
    else
      st->par_ok[i - k] = hex[j] == bh.parity[i - k];
  }
  return BFRS_OK;
}

int load_block(bfrs_ctx *ctx, const Geometry &g, size_t b, BlockArena &a, BlockState *st,
               PipeTrace *pt) {
  if (!a.done) {
    HIP_TRY(hipSetDevice(ctx->impl.device));
    HIP_TRY(hipEventCreateWithFlags(&a.done, hipEventDisableTiming));
  }
  int rc = load_block_reads(ctx, g, b, a, a.dev, a.done, st, pt);
  return rc ? rc : load_block_verify(ctx, g, st, a.done, pt);
}

int restore_block(bfrs_ctx *ctx, const Geometry &g, BlockArena &a, BlockState &st,
                  const std::vector<uint8_t *> *host_out) {
  const size_t k = st.k, erased = st.damaged_segments(), present = st.valid_parity();
  st.restored.clear();
  if (erased == 0) return 0;
  if (erased > present) {
    std::ostringstream os;
    os << "block " << st.b << ": " << erased << " damaged segments but only " << present
       << " valid parity shards - unrecoverable";
    return set_error(BFRS_E_NOT_ENOUGH_SHARDS, os.str());
  }
  std::vector<const uint8_t *> orig(k), rec(kParity);
  std::vector<uint8_t *> out(k);
  for (size_t s = 0; s < k; ++s) {
    orig[s] = st.seg_ok[s] ? st.dev->ds(s) : nullptr;
    out[s] = st.dev->ds(s);  // written only where erased: the restored segment lands in its own slot
  }
  for (size_t p = 0; p < kParity; ++p) rec[p] = st.par_ok[p] ? st.dev->ds(k + p) : nullptr;
  Context &c = ctx->impl;
  const uint32_t kk = uint32_t(k);
  int rc = decode_batch_on(ctx, 1, &kk, kParity, st.shard, orig.data(), rec.data(), out.data(),
                           c.stream);
  if (rc) return rc;
  // src/merkle_tree re-verify of the reconstructed bytes, on the device
  std::vector<const uint8_t *> msgs;
  std::vector<size_t> lens, idx;
  for (size_t s = 0; s < k; ++s)
    if (!st.seg_ok[s]) {
      msgs.push_back(st.dev->ds(s));
      lens.push_back(st.lens[s]);
      idx.push_back(s);
    }
  std::vector<std::string> hex;
  if ((rc = gpu_hash_hex(ctx, msgs, lens, &hex))) return rc;
  const BlockHashes &bh = g.mf.blocks.at(int64_t(st.b));
  for (size_t j = 0; j < idx.size(); ++j)
    if (hex[j] != bh.segments[idx[j]]) {
      std::ostringstream os;
      os << "block " << st.b << " segment " << idx[j] << ": restored bytes fail the manifest hash";
      return set_error(BFRS_E_WRAPPER, os.str());
    }
  // erased <= kParity, so the out slots [0, kParity) hold every one of them
  for (size_t j = 0; j < idx.size(); ++j) {
    const size_t s = idx[j];
    uint8_t *dst = host_out && (*host_out)[s] ? (*host_out)[s] : a.out.hs(j);
    HIP_TRY(hipMemcpyAsync(dst, st.dev->ds(s), st.lens[s], hipMemcpyDeviceToHost, c.stream));
    st.restored.emplace_back(s, dst);
  }
  HIP_TRY(hipStreamSynchronize(c.stream));
  for (size_t s : idx) st.seg_ok[s] = 1;
  return int(idx.size());
}

int reencode_parity(bfrs_ctx *ctx, const Geometry &g, BlockArena &a, BlockState &st) {
  const size_t k = st.k;
  if (st.damaged_segments()) return set_error(BFRS_E_WRAPPER, "re-encode needs whole data");
  std::vector<const uint8_t *> orig(k);
  std::vector<uint8_t *> rec(kParity);
  for (size_t s = 0; s < k; ++s) orig[s] = st.dev->ds(s);
  for (size_t p = 0; p < kParity; ++p) rec[p] = st.dev->ds(k + p);
  Context &c = ctx->impl;
  const uint32_t kk = uint32_t(k);
  int rc = encode_batch_on(ctx, 1, &kk, kParity, st.shard, orig.data(), rec.data(), c.stream);
  if (rc) return rc;
  std::vector<const uint8_t *> msgs(rec.begin(), rec.end());
  std::vector<size_t> lens(kParity, st.shard);
  std::vector<std::string> hex;
  if ((rc = gpu_hash_hex(ctx, msgs, lens, &hex))) return rc;
  const BlockHashes &bh = g.mf.blocks.at(int64_t(st.b));
  for (size_t p = 0; p < kParity; ++p)
    if (hex[p] != bh.parity[p])
      return set_error(BFRS_E_WRAPPER, "re-encoded parity fails the manifest hash");
  for (size_t p = 0; p < kParity; ++p) {
    HIP_TRY(hipMemcpyAsync(a.out.hs(kParity + p), st.dev->ds(k + p), st.shard,
                           hipMemcpyDeviceToHost, c.stream));
    st.parity_host[p] = a.out.hs(kParity + p);
  }
  HIP_TRY(hipStreamSynchronize(c.stream));
  for (size_t p = 0; p < kParity; ++p) st.par_ok[p] = 1;
  return BFRS_OK;
}

}  // namespace bfrs
