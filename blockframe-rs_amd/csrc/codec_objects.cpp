// codec_objects.cpp — bfrs_encoder / bfrs_decoder: the stateful surface of
// reed_solomon_simd::ReedSolomonEncoder / ReedSolomonDecoder (3.x) as the
// reference uses it (src/chunker/generate.rs:37-49,84-96;
// src/filestore/recovery.rs:58-69,152-170; src/filestore/health.rs:733-752).
//
// Each object holds a CodecSlot from its context's pool (runtime.hpp): k + m
// shard rows of HBM, the same rows of pinned host memory, and a stream of its
// own.  add_*_shard takes the caller's bytes before it returns (the crate
// likewise copies each added shard into its work area, so the caller may
// reuse its buffer at once): by default a threaded memcpy into the slot's
// pinned row and an async H2D that overlaps the next shard's copy
// (Staging::kPinned); BFRS_CODEC_STAGING=direct DMAs straight from the
// caller's buffer instead.  encode() queues the HIP pass and the D2H of the recovery
// shards into pinned rows; decode() runs the pass and restored_original(i)
// fetches row i on first use (BlockFrame asks for one target,
// recovery.rs:166-170).  Results stay valid until the next call on the
// object.  Objects are used by one thread at a time; objects of one context
// may live on different threads.  An object holds its context's slot pool
// (shared), so it may be freed after bfrs_close; every other call needs the
// context open.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <sstream>
#include <thread>

#include "runtime.hpp"
#include "knobs.hpp"

using namespace bfrs;

namespace {

// Helper threads per output buffer that fault it in (BFRS_PREFAULT_PARTS,
// 1-8; 0 or unset: the call's default).  A/B knob.
size_t prefault_parts(size_t dflt) {
  static const long v = [] {
    const char *e = BFRS_AB_KNOB("BFRS_PREFAULT_PARTS");
    return e ? std::strtol(e, nullptr, 10) : 0L;
  }();
  return v >= 1 && v <= 8 ? size_t(v) : dflt;
}

// BFRS_PREFAULT_OUTPUTS (default 1): fault the wrapper's fresh output
// buffers in while the device works (encoder_encode_to_host).
bool prefault_outputs() {
  static const bool on = [] {
    const char *e = BFRS_AB_KNOB("BFRS_PREFAULT_OUTPUTS");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

int shard_size_error(size_t expected, size_t got) {
  std::ostringstream os;
  os << "different shard size: expected " << expected << " bytes, got " << got << " bytes";
  return set_error(BFRS_E_DIFFERENT_SHARD_SIZE, os.str());
}

struct CodecObject {
  bfrs_ctx *ctx;
  std::shared_ptr<CodecPool> pool;
  size_t k, m, shard_bytes;
  std::unique_ptr<CodecSlot> slot;
  uint8_t *d_row(size_t i) const { return static_cast<uint8_t *>(slot->d) + i * slot->stride; }
  uint8_t *h_row(size_t i) const { return slot->h + i * slot->stride; }
  int acquire(bfrs_ctx *c, size_t k_, size_t m_, size_t bytes) {
    ctx = c;
    pool = c->impl.codec_pool;
    k = k_;
    m = m_;
    shard_bytes = bytes;
    return pool->acquire(k + m, shard_bytes, &slot);
  }
  // Copy streams (runtime.hpp CodecPool): H2D and D2H of every object of the
  // context in FIFO order on two streams, or on the object's kernel stream.
  hipStream_t h2d() const { return pool->h2d ? pool->h2d : slot->stream; }
  hipStream_t d2h() const { return pool->d2h ? pool->d2h : slot->stream; }
  // Stage a host shard into device row i; the caller's buffer is free again
  // on return.
  int stage(size_t i, const uint8_t *src, size_t len) {
    HIP_TRY(hipSetDevice(pool->device));
    if (pool->staging == Staging::kPinned) {
      // the row's previous H2D (an earlier round on this object) is done:
      // rows are reused only after encode()/decode() synchronised the slot
      host_copy(h_row(i), src, len);
      HIP_TRY(hipMemcpyAsync(d_row(i), h_row(i), len, hipMemcpyHostToDevice, h2d()));
      HIP_TRY(hipEventRecord(slot->ev_h2d, h2d()));
    } else {
      HIP_TRY(hipMemcpyAsync(d_row(i), src, len, hipMemcpyHostToDevice, h2d()));
      HIP_TRY(hipEventRecord(slot->ev_h2d, h2d()));
      HIP_TRY(hipEventSynchronize(slot->ev_h2d));
    }
    return BFRS_OK;
  }
  // The kernel stream waits for this object's staged rows (the copy stream's
  // later work, other objects' copies, is not waited for).
  int kernel_after_h2d() {
    if (h2d() != slot->stream) HIP_TRY(hipStreamWaitEvent(slot->stream, slot->ev_h2d, 0));
    return BFRS_OK;
  }
  // After the kernel: mark it, and let the D2H stream wait for it.
  int d2h_after_kernel() {
    HIP_TRY(hipEventRecord(slot->ev_k, slot->stream));
    if (d2h() != slot->stream) HIP_TRY(hipStreamWaitEvent(d2h(), slot->ev_k, 0));
    return BFRS_OK;
  }
  ~CodecObject() {
    if (slot) pool->release(std::move(slot));
  }
};

}  // namespace

struct bfrs_encoder : CodecObject {
  size_t received = 0;
  bool encoded = false;
  bool fetched_to_pinned = false;  // the pinned rows k.. hold the recovery shards
};

struct bfrs_decoder : CodecObject {
  std::vector<uint8_t> orig_present, rec_present;
  std::vector<uint8_t> restored;  // 1 = device row i holds a restored original
  std::vector<uint8_t> fetched;   // 1 = its pinned row holds it too
  bool decoded = false;
};

extern "C" {

int bfrs_encoder_new(bfrs_ctx *ctx, size_t k, size_t m, size_t shard_bytes, bfrs_encoder **out) {
  BFRS_API_BEGIN
  if (!ctx || !out) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_encoder_new: NULL argument");
  *out = nullptr;
  int rc = check_shape(k, m, shard_bytes);
  if (rc) return rc;
  auto *e = new (std::nothrow) bfrs_encoder;
  if (!e) return set_error(BFRS_E_NOMEM, "encoder allocation failed");
  if ((rc = e->acquire(ctx, k, m, shard_bytes))) {
    delete e;
    return rc;
  }
  *out = e;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_encoder_add_original_shard(bfrs_encoder *e, const uint8_t *shard, size_t len) {
  BFRS_API_BEGIN
  if (!e || !shard) return set_error(BFRS_E_INVALID_ARGUMENT, "add_original_shard: NULL argument");
  if (e->encoded) {  // the crate resets an encoder once its result is released
    e->encoded = false;
    e->received = 0;
  }
  if (e->received >= e->k) {
    std::ostringstream os;
    os << "too many original shards: got more than original_count (" << e->k << ") shards";
    return set_error(BFRS_E_TOO_MANY_ORIGINAL_SHARDS, os.str());
  }
  if (len != e->shard_bytes) return shard_size_error(e->shard_bytes, len);
  int rc = e->stage(e->received, shard, len);
  if (rc) return rc;
  ++e->received;
  return BFRS_OK;
  BFRS_API_END
}

}  // extern "C"

namespace {
// Queue the encode pass of a fully staged encoder on its slot stream.
int encoder_run(bfrs_encoder *e) {
  if (e->received < e->k || e->encoded) {
    std::ostringstream os;
    os << "too few original shards: got " << (e->encoded ? 0 : e->received)
       << " shards while original_count is " << e->k;
    return set_error(BFRS_E_TOO_FEW_ORIGINAL_SHARDS, os.str());
  }
  std::vector<const uint8_t *> din(e->k);
  std::vector<uint8_t *> dout(e->m);
  for (size_t i = 0; i < e->k; ++i) din[i] = e->d_row(i);
  for (size_t j = 0; j < e->m; ++j) dout[j] = e->d_row(e->k + j);
  const uint32_t kk = uint32_t(e->k);
  int rc = e->kernel_after_h2d();
  if (rc) return rc;
  if ((rc = encode_batch_on(e->ctx, 1, &kk, e->m, e->shard_bytes, din.data(), dout.data(),
                            e->slot->stream)))
    return rc;
  return e->d2h_after_kernel();
}
}  // namespace

int bfrs::encoder_encode_to_host(bfrs_encoder *e, uint8_t *const *outs) {
  // D2H into the pinned rows, then host_copy (up to 8 threads per shard) into
  // the caller's buffers.  A D2H straight into a fresh pageable buffer faults
  // its pages inside the copy at a fraction of the link rate, and touching
  // them on a helper thread during the H2D of the inputs contended with the
  // pageable H2D (bench crate_api).  Shard j's copy-out
  // overlaps the D2H of shard j + 1.
  int rc = encoder_run(e);
  if (rc) return rc;
  hipStream_t st = e->d2h();
  std::vector<hipEvent_t> done(e->m, nullptr);
  struct Events {
    std::vector<hipEvent_t> &v;
    ~Events() {
      for (hipEvent_t x : v)
        if (x) (void)hipEventDestroy(x);
    }
  } guard{done};
  // Fresh output buffers (the reference's to_vec, generate.rs:95-96) take
  // their page faults here, one helper thread per output, while the H2D
  // tail, the kernel and the first D2H run: the caller's thread would only
  // wait in that window.  (Touching them during the adds competed with the
  // staging copies for host memory bandwidth)  Each output's
  // thread is joined before its copy-out, and on every exit path.
  struct Touch {
    std::vector<std::thread> t;
    ~Touch() {
      for (auto &x : t)
        if (x.joinable()) x.join();
    }
  } touch;
  if (prefault_outputs()) {
    const size_t n = e->shard_bytes;
    for (size_t j = 0; j < e->m; ++j) {
      uint8_t *p = outs[j];
      try {
        touch.t.emplace_back([p, n] { prefault_range(p, n); });
      } catch (...) {  // no thread: the copy-out faults the pages itself
        break;
      }
    }
  }
  for (size_t j = 0; j < e->m; ++j) {
    HIP_TRY(hipMemcpyAsync(e->h_row(e->k + j), e->d_row(e->k + j), e->shard_bytes,
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventCreateWithFlags(&done[j], hipEventDisableTiming));
    HIP_TRY(hipEventRecord(done[j], st));
  }
  HIP_TRY(hipEventRecord(e->slot->ev_d2h, st));
  using clk = std::chrono::steady_clock;
  double wait_ms = 0, copy_ms = 0;
  for (size_t j = 0; j < e->m; ++j) {
    const auto t0 = clk::now();
    HIP_TRY(hipEventSynchronize(done[j]));
    if (j < touch.t.size()) touch.t[j].join();
    const auto t1 = clk::now();
    host_copy(outs[j], e->h_row(e->k + j), e->shard_bytes);
    wait_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    copy_ms += std::chrono::duration<double, std::milli>(clk::now() - t1).count();
  }
  if (BFRS_AB_KNOB("BFRS_TRACE"))  // measurement aid (tools/crate_probe.py)
    std::fprintf(stderr, "bfrs trace: encode_to_host wait %.3f ms, copy-out %.3f ms\n", wait_ms,
                 copy_ms);
  // the pinned rows hold the recovery shards too, as after encode()
  e->encoded = true;
  e->fetched_to_pinned = true;
  return BFRS_OK;
}

namespace {
// First-touch of fresh output buffers (the reference's to_vec / fresh Vec
// outputs) on `parts` helper threads per buffer, joined by join() or on
// destruction (every exit path).
struct TouchThreads {
  std::vector<std::thread> t;
  void start(uint8_t *const *bufs, size_t nbuf, size_t len, size_t parts) {
    const size_t per = (len + parts - 1) / parts;
    for (size_t b = 0; b < nbuf; ++b)
      for (size_t q = 0; q < parts; ++q) {
        const size_t lo = q * per, hi = std::min(len, lo + per);
        if (lo >= hi) continue;
        uint8_t *p = bufs[b];
        auto f = [p, lo, hi] { prefault_range(p + lo, hi - lo); };
        try {
          t.emplace_back(f);
        } catch (...) {
          f();
        }
      }
  }
  void join() {
    for (auto &x : t)
      if (x.joinable()) x.join();
    t.clear();
  }
  ~TouchThreads() { join(); }
};


// Column slabs of ~8 MiB of 64-byte chunks; the last slab takes the tail.
std::vector<size_t> slab_offsets(size_t S) {
  const size_t chunks = S / 64;
  const size_t nslab = std::max<size_t>(1, std::min<size_t>(8, S >> 23));
  std::vector<size_t> off(nslab + 1);
  for (size_t q = 0; q < nslab; ++q) off[q] = chunks * q / nslab * 64;
  off[nslab] = S;
  return off;
}

// done() of the slab copies: the H2D of a slab's rows, queued by the copy
// threads that filled them (the stream is thread-safe).  Jobs (row i, or
// rows[i]) come in groups of kRowGroup; the thread that completes a group
// queues it, and consecutive slot rows of a group go as one 2-D copy (the
// slot's rows are `stride` apart on both sides).  One 2-D copy of many rows
// moves more per second than as many 1-D copies while the previous slab's
// D2H runs beside it (tools/copy2d_probe.py: 55.3 vs 52.5 GB/s for 30 rows);
// groups keep the DMA starting while later rows are still being copied.
struct SlabH2D {
  static constexpr size_t kRowGroup = 8;
  const CodecObject *obj;
  hipStream_t st;
  size_t off, len, njobs;
  std::vector<size_t> rows;  // empty: job i is row i
  size_t group;              // jobs per group (1: every row its own copy)
  std::unique_ptr<std::atomic<int>[]> left;  // jobs of each group still copying
  std::atomic<int> err_{0};
  hipError_t err = hipSuccess;
  SlabH2D(const CodecObject *o, hipStream_t s, size_t of, size_t ln, size_t n,
          std::vector<size_t> r)
      : obj(o), st(s), off(of), len(ln), njobs(n), rows(std::move(r)), group(row_group()) {
    const size_t ng = (njobs + group - 1) / group;
    left.reset(new std::atomic<int>[ng]);
    for (size_t g = 0; g < ng; ++g) left[g] = int(std::min(group, njobs - g * group));
  }
  static size_t row_group() {
    const char *e = BFRS_AB_KNOB("BFRS_SLAB_ROW_GROUP");  // A/B: 1 = one copy per row
    const long v = e && *e ? std::strtol(e, nullptr, 10) : long(kRowGroup);
    return size_t(std::clamp(v, 1L, 64L));
  }
  size_t row(size_t i) const { return rows.empty() ? i : rows[i]; }
  void fail(hipError_t e) {
    int expect = 0;
    if (e != hipSuccess && err_.compare_exchange_strong(expect, 1)) err = e;
  }
  static void row_done(void *p, size_t i) {
    auto *h = static_cast<SlabH2D *>(p);
    const size_t g = i / h->group;
    if (h->left[g].fetch_sub(1, std::memory_order_acq_rel) != 1) return;  // not the last
    // a host_copy helper thread: make the pool's device current on it, so
    // the copy never depends on which device the thread last used
    hipError_t e = hipSetDevice(h->obj->pool->device);
    const size_t a = g * h->group, b = std::min(h->njobs, a + h->group);
    const size_t pitch = h->obj->slot->stride;
    for (size_t j = a; j < b && e == hipSuccess;) {
      size_t t = j + 1;  // consecutive slot rows: one 2-D copy
      while (t < b && h->row(t) == h->row(t - 1) + 1) ++t;
      const size_t r = h->row(j);
      e = t - j == 1
              ? hipMemcpyAsync(h->obj->d_row(r) + h->off, h->obj->h_row(r) + h->off, h->len,
                               hipMemcpyHostToDevice, h->st)
              : hipMemcpy2DAsync(h->obj->d_row(r) + h->off, pitch, h->obj->h_row(r) + h->off,
                                 pitch, h->len, t - j, hipMemcpyHostToDevice, h->st);
      j = t;
    }
    h->fail(e);
  }
};

// Every exit of a slab wrapper, an error included: the slot's events cover
// all the work it queued on both streams, so release() and the slot's next
// user wait for it (an early return used to leave slab copies and
// kernels in flight behind events of an earlier call).
struct SlabFence {
  CodecSlot &sl;
  hipStream_t st, ax;
  ~SlabFence() {
    (void)hipEventRecord(sl.ev_h2d, st);
    (void)hipEventRecord(sl.ev_d2h, ax);
  }
};

// Measurement build only (knobs.hpp): BFRS_FAIL_SLAB=q fails a slab wrapper
// after it queued slab q, read on every call (tests/test_gpu_parity.py: a
// failed call leaves its slot safe to reuse).
int injected_slab_failure(size_t q) {
  const char *e = BFRS_AB_KNOB("BFRS_FAIL_SLAB");
  if (e && *e && std::strtol(e, nullptr, 10) == long(q))
    return set_error(BFRS_E_HIP, "injected slab failure (BFRS_FAIL_SLAB)");
  return BFRS_OK;
}

struct EventList {
  std::vector<hipEvent_t> v;
  ~EventList() {
    for (hipEvent_t x : v)
      if (x) (void)hipEventDestroy(x);
  }
  int add(hipStream_t st, hipEvent_t *out) {
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    v.push_back(e);
    HIP_TRY(hipEventRecord(e, st));
    *out = e;
    return BFRS_OK;
  }
};
}  // namespace

int bfrs::encoder_encode_slabs(bfrs_encoder *e, const uint8_t *const *segs, const size_t *lens,
                               uint8_t *const *outs) {
  const size_t S = e->shard_bytes, k = e->k, m = e->m;
  if (e->received != 0 || e->encoded)
    return set_error(BFRS_E_INVALID_ARGUMENT, "encode_slabs: encoder already in use");
  HIP_TRY(hipSetDevice(e->pool->device));
  CodecSlot &sl = *e->slot;
  if (!sl.aux) HIP_TRY(hipStreamCreateWithFlags(&sl.aux, hipStreamNonBlocking));
  hipStream_t st = sl.stream, ax = sl.aux;
  SlabFence fence{sl, st, ax};
  const std::vector<size_t> off = slab_offsets(S);
  const size_t nslab = off.size() - 1;
  EventList ev;
  std::vector<hipEvent_t> done(nslab);
  const uint32_t kk = uint32_t(k);
  std::vector<const uint8_t *> din(k);
  std::vector<uint8_t *> dout(m);
  std::vector<CopyJob> jobs(k);
  TouchThreads touch;
  for (size_t q = 0; q < nslab; ++q) {
    const size_t o = off[q], len = off[q + 1] - o;
    // slab q of every segment into the pinned rows on the copy threads, each
    // row's H2D queued by the thread that copied it
    for (size_t i = 0; i < k; ++i) {
      const size_t avail = lens[i] > o ? std::min(len, lens[i] - o) : 0;
      jobs[i] = CopyJob{e->h_row(i) + o, avail ? segs[i] + o : nullptr, avail, len - avail};
      din[i] = e->d_row(i) + o;
    }
    SlabH2D h2d{e, st, o, len, k, {}};
    host_copy_batch(jobs.data(), k, &SlabH2D::row_done, &h2d);
    if (h2d.err) return hip_error(h2d.err, "slab H2D");
    hipEvent_t staged;
    if (int rc = ev.add(st, &staged)) return rc;
    HIP_TRY(hipStreamWaitEvent(ax, staged, 0));
    for (size_t j = 0; j < m; ++j) dout[j] = e->d_row(k + j) + o;
    int rc = encode_batch_on(e->ctx, 1, &kk, m, len, din.data(), dout.data(), ax);
    if (rc) return rc;
    for (size_t j = 0; j < m; ++j)
      HIP_TRY(hipMemcpyAsync(e->h_row(k + j) + o, e->d_row(k + j) + o, len,
                             hipMemcpyDeviceToHost, ax));
    if ((rc = ev.add(ax, &done[q]))) return rc;
    if ((rc = injected_slab_failure(q))) return rc;
  }
  // the caller's fresh outputs fault in while the last slabs transfer, 4
  // threads per output (from the start of the call, beside the input copies,
  // they cost more: r04n; 1 thread per output: r04v)
  if (prefault_outputs()) touch.start(outs, m, S, prefault_parts(4));
  touch.join();
  for (size_t q = 0; q < nslab; ++q) {
    HIP_TRY(hipEventSynchronize(done[q]));
    for (size_t j = 0; j < m; ++j)
      host_copy(outs[j] + off[q], e->h_row(k + j) + off[q], off[q + 1] - off[q]);
  }
  e->received = k;
  e->encoded = true;
  e->fetched_to_pinned = true;
  return BFRS_OK;
}

extern "C" {

int bfrs_encoder_encode(bfrs_encoder *e) {
  BFRS_API_BEGIN
  if (!e) return set_error(BFRS_E_INVALID_ARGUMENT, "encode: NULL encoder");
  int rc = encoder_run(e);
  if (rc) return rc;
  hipStream_t st = e->d2h();
  for (size_t j = 0; j < e->m; ++j)
    HIP_TRY(hipMemcpyAsync(e->h_row(e->k + j), e->d_row(e->k + j), e->shard_bytes,
                           hipMemcpyDeviceToHost, st));
  HIP_TRY(hipEventRecord(e->slot->ev_d2h, st));
  if ((rc = e->slot->sync())) return rc;
  e->encoded = true;
  e->fetched_to_pinned = true;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_encoder_recovery(bfrs_encoder *e, size_t index, const uint8_t **data, size_t *len) {
  BFRS_API_BEGIN
  if (!e || !data || !len) return set_error(BFRS_E_INVALID_ARGUMENT, "recovery: NULL argument");
  if (!e->encoded || !e->fetched_to_pinned || index >= e->m) {
    std::ostringstream os;
    os << "invalid recovery shard index: " << index << " >= recovery_count " << e->m;
    return set_error(BFRS_E_INVALID_RECOVERY_SHARD_INDEX, os.str());
  }
  *data = e->h_row(e->k + index);
  *len = e->shard_bytes;
  return BFRS_OK;
  BFRS_API_END
}

void bfrs_encoder_free(bfrs_encoder *e) { delete e; }

int bfrs_decoder_new(bfrs_ctx *ctx, size_t k, size_t m, size_t shard_bytes, bfrs_decoder **out) {
  BFRS_API_BEGIN
  if (!ctx || !out) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_decoder_new: NULL argument");
  *out = nullptr;
  int rc = check_shape(k, m, shard_bytes);
  if (rc) return rc;
  auto *d = new (std::nothrow) bfrs_decoder;
  if (!d) return set_error(BFRS_E_NOMEM, "decoder allocation failed");
  d->orig_present.assign(k, 0);
  d->rec_present.assign(m, 0);
  if ((rc = d->acquire(ctx, k, m, shard_bytes))) {
    delete d;
    return rc;
  }
  *out = d;
  return BFRS_OK;
  BFRS_API_END
}

static void decoder_reset_if_done(bfrs_decoder *d) {
  if (d->decoded) {
    d->decoded = false;
    d->restored.clear();
    d->fetched.clear();
    std::fill(d->orig_present.begin(), d->orig_present.end(), 0);
    std::fill(d->rec_present.begin(), d->rec_present.end(), 0);
  }
}

int bfrs_decoder_add_original_shard(bfrs_decoder *d, size_t index, const uint8_t *shard,
                                    size_t len) {
  BFRS_API_BEGIN
  if (!d || !shard) return set_error(BFRS_E_INVALID_ARGUMENT, "add_original_shard: NULL argument");
  decoder_reset_if_done(d);
  if (index >= d->k) {
    std::ostringstream os;
    os << "invalid original shard index: " << index << " >= original_count " << d->k;
    return set_error(BFRS_E_INVALID_ORIGINAL_SHARD_INDEX, os.str());
  }
  if (d->orig_present[index]) {
    std::ostringstream os;
    os << "duplicate original shard index: " << index;
    return set_error(BFRS_E_DUPLICATE_ORIGINAL_SHARD_INDEX, os.str());
  }
  if (len != d->shard_bytes) return shard_size_error(d->shard_bytes, len);
  int rc = d->stage(index, shard, len);
  if (rc) return rc;
  d->orig_present[index] = 1;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_decoder_add_recovery_shard(bfrs_decoder *d, size_t index, const uint8_t *shard,
                                    size_t len) {
  BFRS_API_BEGIN
  if (!d || !shard) return set_error(BFRS_E_INVALID_ARGUMENT, "add_recovery_shard: NULL argument");
  decoder_reset_if_done(d);
  if (index >= d->m) {
    std::ostringstream os;
    os << "invalid recovery shard index: " << index << " >= recovery_count " << d->m;
    return set_error(BFRS_E_INVALID_RECOVERY_SHARD_INDEX, os.str());
  }
  if (d->rec_present[index]) {
    std::ostringstream os;
    os << "duplicate recovery shard index: " << index;
    return set_error(BFRS_E_DUPLICATE_RECOVERY_SHARD_INDEX, os.str());
  }
  if (len != d->shard_bytes) return shard_size_error(d->shard_bytes, len);
  int rc = d->stage(d->k + index, shard, len);
  if (rc) return rc;
  d->rec_present[index] = 1;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_decoder_decode(bfrs_decoder *d) {
  BFRS_API_BEGIN
  if (!d) return set_error(BFRS_E_INVALID_ARGUMENT, "decode: NULL decoder");
  size_t orig_recv = 0, rec_recv = 0;
  for (uint8_t b : d->orig_present) orig_recv += b;
  for (uint8_t b : d->rec_present) rec_recv += b;
  if (orig_recv + rec_recv < d->k) {
    std::ostringstream os;
    os << "not enough shards: " << orig_recv << " original + " << rec_recv << " recovery < "
       << d->k << " original_count";
    return set_error(BFRS_E_NOT_ENOUGH_SHARDS, os.str());
  }
  d->restored.assign(d->k, 0);
  d->fetched.assign(d->k, 0);
  d->decoded = true;
  hipStream_t st = d->slot->stream;
  if (orig_recv == d->k) {  // nothing to restore; the staged copies still have to land
    return d->slot->sync();
  }
  // Restored shards are written over the erased originals' own rows.
  std::vector<const uint8_t *> dorig(d->k), drec(d->m);
  std::vector<uint8_t *> drest(d->k, nullptr);
  for (size_t i = 0; i < d->k; ++i) {
    if (d->orig_present[i])
      dorig[i] = d->d_row(i);
    else
      drest[i] = d->d_row(i);
  }
  for (size_t j = 0; j < d->m; ++j)
    if (d->rec_present[j]) drec[j] = d->d_row(d->k + j);
  const uint32_t kk = uint32_t(d->k);
  int rc = d->kernel_after_h2d();
  if (rc) return rc;
  if ((rc = decode_batch_on(d->ctx, 1, &kk, d->m, d->shard_bytes, dorig.data(), drec.data(),
                            drest.data(), st)))
    return rc;
  if ((rc = d->d2h_after_kernel())) return rc;
  if ((rc = d->slot->sync())) return rc;
  for (size_t i = 0; i < d->k; ++i) d->restored[i] = !d->orig_present[i];
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_decoder_restored_original(bfrs_decoder *d, size_t index, const uint8_t **data,
                                   size_t *len) {
  BFRS_API_BEGIN
  if (!d || !data || !len)
    return set_error(BFRS_E_INVALID_ARGUMENT, "restored_original: NULL argument");
  *data = nullptr;
  *len = 0;
  if (!d->decoded || index >= d->restored.size() || !d->restored[index])
    return set_error(BFRS_E_NOT_RESTORED, "original shard was not restored");
  if (!d->fetched[index]) {  // D2H of this row on first use
    HIP_TRY(hipSetDevice(d->pool->device));
    HIP_TRY(hipMemcpyAsync(d->h_row(index), d->d_row(index), d->shard_bytes, hipMemcpyDeviceToHost,
                           d->d2h()));
    HIP_TRY(hipEventRecord(d->slot->ev_d2h, d->d2h()));
    int rc = d->slot->sync();
    if (rc) return rc;
    d->fetched[index] = 1;
  }
  *data = d->h_row(index);
  *len = d->shard_bytes;
  return BFRS_OK;
  BFRS_API_END
}

void bfrs_decoder_free(bfrs_decoder *d) { delete d; }

}  // extern "C"

int bfrs::decoder_restored_to_host(bfrs_decoder *d, size_t index, uint8_t *out) {
  if (!d->decoded || index >= d->restored.size() || !d->restored[index])
    return set_error(BFRS_E_NOT_RESTORED, "original shard was not restored");
  if (d->pool->staging == Staging::kPinned || d->fetched[index]) {  // via the pinned row
    const uint8_t *data;
    size_t len;
    int rc = bfrs_decoder_restored_original(d, index, &data, &len);
    if (rc) return rc;
    host_copy(out, data, len);
    return BFRS_OK;
  }
  HIP_TRY(hipSetDevice(d->pool->device));
  HIP_TRY(hipMemcpyAsync(out, d->d_row(index), d->shard_bytes, hipMemcpyDeviceToHost, d->d2h()));
  HIP_TRY(hipEventRecord(d->slot->ev_d2h, d->d2h()));
  return d->slot->sync();
}

int bfrs::decoder_restore_slabs(bfrs_decoder *d, const uint8_t *const *segs,
                                const uint8_t *const *par, size_t target, uint8_t *out) {
  const size_t S = d->shard_bytes, k = d->k, m = d->m;
  if (d->decoded || std::count(d->orig_present.begin(), d->orig_present.end(), 1) ||
      std::count(d->rec_present.begin(), d->rec_present.end(), 1))
    return set_error(BFRS_E_INVALID_ARGUMENT, "restore_slabs: decoder already in use");
  HIP_TRY(hipSetDevice(d->pool->device));
  CodecSlot &sl = *d->slot;
  if (!sl.aux) HIP_TRY(hipStreamCreateWithFlags(&sl.aux, hipStreamNonBlocking));
  hipStream_t st = sl.stream, ax = sl.aux;
  SlabFence fence{sl, st, ax};
  for (size_t i = 0; i < k; ++i) d->orig_present[i] = segs[i] != nullptr;
  for (size_t j = 0; j < m; ++j) d->rec_present[j] = par[j] != nullptr;
  const std::vector<size_t> off = slab_offsets(S);
  const size_t nslab = off.size() - 1;
  EventList ev;
  std::vector<hipEvent_t> done(nslab);
  const uint32_t kk = uint32_t(k);
  std::vector<const uint8_t *> dorig(k), drec(m);
  std::vector<uint8_t *> drest(k);
  uint8_t *const outs[1] = {out};
  TouchThreads touch;
  for (size_t q = 0; q < nslab; ++q) {
    const size_t o = off[q], len = off[q + 1] - o;
    std::vector<CopyJob> jobs;
    std::vector<size_t> rows;
    for (size_t r = 0; r < k + m; ++r) {
      const uint8_t *src = r < k ? segs[r] : par[r - k];
      if (!src) continue;
      jobs.push_back(CopyJob{d->h_row(r) + o, src + o, len, 0});
      rows.push_back(r);
    }
    SlabH2D h2d{d, st, o, len, jobs.size(), rows};
    host_copy_batch(jobs.data(), jobs.size(), &SlabH2D::row_done, &h2d);
    if (h2d.err) return hip_error(h2d.err, "slab H2D");
    for (size_t i = 0; i < k; ++i) {
      dorig[i] = segs[i] ? d->d_row(i) + o : nullptr;
      drest[i] = segs[i] ? nullptr : d->d_row(i) + o;
    }
    for (size_t j = 0; j < m; ++j) drec[j] = par[j] ? d->d_row(k + j) + o : nullptr;
    hipEvent_t staged;
    if (int rc = ev.add(st, &staged)) return rc;
    HIP_TRY(hipStreamWaitEvent(ax, staged, 0));
    int rc = decode_batch_on(d->ctx, 1, &kk, m, len, dorig.data(), drec.data(), drest.data(), ax);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(d->h_row(target) + o, d->d_row(target) + o, len, hipMemcpyDeviceToHost,
                           ax));
    if ((rc = ev.add(ax, &done[q]))) return rc;
    if ((rc = injected_slab_failure(q))) return rc;
  }
  if (prefault_outputs()) touch.start(outs, 1, S, prefault_parts(4));
  touch.join();
  for (size_t q = 0; q < nslab; ++q) {
    HIP_TRY(hipEventSynchronize(done[q]));
    host_copy(out + off[q], d->h_row(target) + off[q], off[q + 1] - off[q]);
  }
  d->decoded = true;
  d->restored.assign(k, 0);
  d->fetched.assign(k, 0);
  for (size_t i = 0; i < k; ++i) d->restored[i] = !d->orig_present[i];
  d->fetched[target] = 1;  // its pinned row holds the whole shard
  return BFRS_OK;
}
