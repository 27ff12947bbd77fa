// runtime.cpp — context, plan cache, pass scheduling and the codec C-ABI.
//
// Mirrors the reed-solomon-simd 3.1.0 surface the reference uses
// (ReedSolomonEncoder/Decoder) on top of the HIP kernels.
// There is no CPU compute path: without a HIP device every codec entry point
// fails with BFRS_E_NO_DEVICE.
#include "runtime.hpp"

#include <sys/mman.h>
#include "knobs.hpp"

#include <algorithm>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <sstream>

namespace bfrs {

namespace {
thread_local std::string g_last_error;

// Device-path limits (the crate allows up to 65535; the matrix form here is
// sized for BlockFrame's RS(<=30, 3) and moderate generalisations).
constexpr size_t kMaxOriginal = 1024;
constexpr size_t kMaxRecovery = 1024;

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// One slab's piece of each row of a host batch: `len` bytes from src to dst.
struct RowCopy {
  uint8_t *dst;
  const uint8_t *src;
};

// The HIP allocation holding host pointer p, if it is pinned host memory
// that the device sees at the same address (hipHostMalloc'd, as a pinned
// tensor's storage), so its range is in host addresses; false for pageable
// memory and for registered memory mapped elsewhere.
bool pinned_range(const void *p, uintptr_t *lo, uintptr_t *hi) {
  auto dp = reinterpret_cast<hipDeviceptr_t>(const_cast<void *>(p));
  unsigned type = 0;
  void *hostp = nullptr, *devp = nullptr, *start = nullptr;
  size_t size = 0;
  if (hipPointerGetAttribute(&type, HIP_POINTER_ATTRIBUTE_MEMORY_TYPE, dp) != hipSuccess ||
      type != unsigned(hipMemoryTypeHost) ||
      hipPointerGetAttribute(&hostp, HIP_POINTER_ATTRIBUTE_HOST_POINTER, dp) != hipSuccess ||
      hipPointerGetAttribute(&devp, HIP_POINTER_ATTRIBUTE_DEVICE_POINTER, dp) != hipSuccess ||
      hostp != p || devp != p ||
      hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, dp) != hipSuccess ||
      hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, dp) != hipSuccess ||
      !start || !size) {
    (void)hipGetLastError();  // a pageable pointer is not an error here
    return false;
  }
  *lo = reinterpret_cast<uintptr_t>(start);
  *hi = *lo + size;
  return *lo <= reinterpret_cast<uintptr_t>(p) && reinterpret_cast<uintptr_t>(p) < *hi;
}

// Queues the row copies on `st`.  Consecutive rows whose source and
// destination both advance by one constant pitch (>= len) go as ONE
// hipMemcpy2DAsync when the host side of the whole run lies inside one
// pinned allocation: the rows of a pinned tensor into the pipeline's device
// rows `stride` apart.  With the D2H of the previous slab running beside it,
// one 2-D copy of 30 rows moved 55.3 GB/s against 52.5 GB/s for 30 separate
// copies (tools/copy2d_probe.py, profiles/r05/copy2d_r05.json; DESIGN.md
// §7).  Pageable rows, and rows of different allocations, stay one copy each.
int copy_rows(const std::vector<RowCopy> &rows, size_t len, hipMemcpyKind kind, hipStream_t st) {
  auto at = [](const void *p) { return reinterpret_cast<uintptr_t>(p); };
  auto host = [&](const RowCopy &r) {
    return kind == hipMemcpyHostToDevice ? at(r.src) : at(r.dst);
  };
  size_t i = 0;
  while (i < rows.size()) {
    size_t j = i + 1;  // end of the run starting at row i
    intptr_t dp = 0, sp = 0;
    uintptr_t lo = 0, hi = 0;
    if (j < rows.size()) {
      dp = intptr_t(at(rows[j].dst) - at(rows[i].dst));
      sp = intptr_t(at(rows[j].src) - at(rows[i].src));
      // a run: constant pitches, the host side inside row i's pinned allocation
      if (dp >= intptr_t(len) && sp >= intptr_t(len) &&
          pinned_range(reinterpret_cast<const void *>(host(rows[i])), &lo, &hi) &&
          host(rows[i]) >= lo) {
        while (j < rows.size() && intptr_t(at(rows[j].dst) - at(rows[j - 1].dst)) == dp &&
               intptr_t(at(rows[j].src) - at(rows[j - 1].src)) == sp && host(rows[j]) + len <= hi)
          ++j;
      }
    }
    if (j - i == 1) {
      HIP_TRY(hipMemcpyAsync(rows[i].dst, rows[i].src, len, kind, st));
    } else {
      HIP_TRY(hipMemcpy2DAsync(rows[i].dst, size_t(dp), rows[i].src, size_t(sp), len, j - i, kind,
                               st));
    }
    i = j;
  }
  return BFRS_OK;
}
}  // namespace

namespace {
constexpr size_t kHugePage = size_t(2) << 20;
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
// the measurement build can force hipHostMalloc for a same-box A/B
bool pin_by_register() {
  const char *e = BFRS_AB_KNOB("BFRS_PIN_MODE");
  return !(e && std::strcmp(e, "malloc") == 0);
}
// The registered mappings and their mapped lengths: a large buffer may still
// be hipHostMalloc'd (the registration failed, or the A/B malloc mode), so
// pinned_free goes by what pinned_alloc did, not by the size it is handed.
// Never destroyed: a caller's own static destructor may free staging after
// this library's statics are gone (__cxa_finalize order across DSOs).
struct Registry {
  std::mutex mu;
  std::unordered_map<void *, size_t> len;
};
Registry &registry() {
  static Registry *r = new Registry;
  return *r;
}
}  // namespace

// below this, hipHostMalloc (a huge-page mapping would round a small buffer
// up to 2 MiB; the codec slots of small shapes come and go often)
constexpr size_t kRegisterMin = size_t(4) << 20;

void *pinned_alloc(size_t bytes) {
  if (bytes == 0) return nullptr;
  const size_t len = round_up(bytes, kHugePage);
  if (bytes >= kRegisterMin && pin_by_register()) {
    // over-allocate by one huge page and trim, so the range is 2 MiB aligned
    void *raw = mmap(nullptr, len + kHugePage, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS,
                     -1, 0);
    if (raw != MAP_FAILED) {
      const uintptr_t r = reinterpret_cast<uintptr_t>(raw);
      const uintptr_t a = round_up(r, kHugePage);
      if (a > r) munmap(raw, a - r);
      if (r + kHugePage > a) munmap(reinterpret_cast<void *>(a + len), r + kHugePage - a);
      void *p = reinterpret_cast<void *>(a);
      (void)madvise(p, len, MADV_HUGEPAGE);
      // not inherited by a fork()ed child (the bench's subprocesses, a
      // caller's workers): the parent's registered pages never turn
      // copy-on-write under the GPU's mapping, as with RDMA registrations
      (void)madvise(p, len, MADV_DONTFORK);
      if (madvise(p, len, MADV_POPULATE_WRITE) != 0) std::memset(p, 0, len);  // first touch
      if (hipHostRegister(p, len, hipHostRegisterPortable) == hipSuccess) {
        Registry &reg = registry();
        std::lock_guard<std::mutex> g(reg.mu);
        reg.len[p] = len;
        return p;
      }
      (void)hipGetLastError();
      munmap(p, len);
    }
  }
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void pinned_free(void *p, size_t) {
  if (!p) return;
  // a registered mapping, or else hipHostMalloc'd (small, or the fallback)
  size_t mapped = 0;
  {
    Registry &reg = registry();
    std::lock_guard<std::mutex> g(reg.mu);
    auto it = reg.len.find(p);
    if (it != reg.len.end()) {
      mapped = it->second;
      reg.len.erase(it);
    }
  }
  if (mapped) {
    if (hipHostUnregister(p) != hipSuccess) (void)hipGetLastError();
    munmap(p, mapped);
    return;
  }
  (void)hipHostFree(p);
}

int set_error(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

int hip_error(hipError_t e, const char *what) {
  std::ostringstream os;
  os << what << ": " << hipGetErrorString(e);
  return set_error(BFRS_E_HIP, os.str());
}


int check_shape(size_t k, size_t m, size_t shard_bytes) {
  if (shard_bytes == 0 || (shard_bytes & 1)) {
    std::ostringstream os;
    os << "invalid shard size: " << shard_bytes << " bytes (must non-zero and multiple of 2)";
    return set_error(BFRS_E_INVALID_SHARD_SIZE, os.str());
  }
  Rate rate;
  if (!choose_rate(k, m, &rate) || k > kMaxOriginal || m > kMaxRecovery) {
    std::ostringstream os;
    os << "unsupported shard count: " << k << " original shards with " << m
       << " recovery shards";
    return set_error(BFRS_E_UNSUPPORTED_SHARD_COUNT, os.str());
  }
  return BFRS_OK;
}

Plan::~Plan() {
  if (d_tables) (void)hipFree(d_tables);
}

static int upload_plan(Plan *p) {
  const CoefMatrix &c = p->coef;
  std::vector<uint32_t> all, t;
  std::vector<size_t> offs;
  for (size_t r0 = 0; r0 < c.rows; r0 += kMaxPassOutputs) {
    const size_t r1 = std::min(c.rows, r0 + kMaxPassOutputs);
    for (size_t c0 = 0; c0 < c.cols; c0 += kMaxPassInputs) {
      const size_t c1 = std::min(c.cols, c0 + kMaxPassInputs);
      build_tables(c, r0, r1, c0, c1, &t);
      // The kernel consumes inputs in pairs: pad odd passes with one input
      // whose table is all zeros (it reads a duplicate pointer, adds nothing).
      if ((c1 - c0) & 1) t.resize(t.size() + 128, 0);
      offs.push_back(all.size());
      all.insert(all.end(), t.begin(), t.end());
      PlanPass pp;
      pp.subfield = true;
      for (size_t r = r0; r < r1 && pp.subfield; ++r)
        for (size_t cc = c0; cc < c1; ++cc)
          if (c.at(r, cc) >= 256) {
            pp.subfield = false;
            break;
          }
      pp.r0 = uint32_t(r0);
      pp.r1 = uint32_t(r1);
      pp.c0 = uint32_t(c0);
      pp.c1 = uint32_t(c1);
      pp.phase = uint32_t(c0 / kMaxPassInputs);
      p->passes.push_back(pp);
      p->n_phases = std::max(p->n_phases, pp.phase + 1);
    }
  }
  if (all.empty()) return BFRS_OK;
  HIP_TRY(hipMalloc(&p->d_tables, all.size() * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(p->d_tables, all.data(), all.size() * sizeof(uint32_t),
                    hipMemcpyHostToDevice));
  for (size_t i = 0; i < p->passes.size(); ++i)
    p->passes[i].d_table =
        reinterpret_cast<const uint2 *>(static_cast<uint32_t *>(p->d_tables) + offs[i]);
  return BFRS_OK;
}

int CodecSlot::sync() {
  // an event never recorded counts as complete
  for (hipEvent_t e : {ev_h2d, ev_k, ev_d2h})
    if (e) HIP_TRY(hipEventSynchronize(e));
  return BFRS_OK;
}

CodecSlot::~CodecSlot() {
  (void)sync();
  for (hipEvent_t e : {ev_h2d, ev_k, ev_d2h})
    if (e) (void)hipEventDestroy(e);
  if (stream && own_stream) {
    (void)hipStreamSynchronize(stream);
    (void)hipStreamDestroy(stream);
  }
  if (aux) {
    (void)hipStreamSynchronize(aux);
    (void)hipStreamDestroy(aux);
  }
  if (d) (void)hipFree(d);
  pinned_free(h, stride * nshards);
}

int CodecPool::init_streams(size_t n, bool copy_streams) {
  if (copy_streams) {
    HIP_TRY(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));
  }
  for (size_t i = 0; i < n; ++i) {
    hipStream_t st;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    streams.push_back(st);
    users.push_back(0);
  }
  return BFRS_OK;
}

int CodecPool::acquire(size_t nshards, size_t shard_bytes, std::unique_ptr<CodecSlot> *out) {
  const size_t stride = (shard_bytes + 255) / 256 * 256;
  std::unique_ptr<CodecSlot> s;
  {
    std::lock_guard<std::mutex> g(mu);
    for (size_t i = 0; i < free.size(); ++i)
      if (free[i]->stride >= stride && free[i]->nshards >= nshards &&
          free[i]->stride * free[i]->nshards <= 2 * stride * nshards) {
        s = std::move(free[i]);
        free.erase(free.begin() + long(i));
        break;
      }
  }
  if (!s) {
    s = std::make_unique<CodecSlot>();
    s->stride = stride;
    s->nshards = nshards;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_h2d, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_k, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_d2h, hipEventDisableTiming));
    if (streams.empty()) {
      HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
      s->own_stream = true;
    }
    HIP_TRY(hipMalloc(&s->d, stride * nshards));
    s->h = static_cast<uint8_t *>(pinned_alloc(stride * nshards));
    if (!s->h) return set_error(BFRS_E_NOMEM, "pinned codec slot allocation failed");
  }
  if (!streams.empty()) {  // the shared stream with the fewest live slots
    std::lock_guard<std::mutex> g(mu);
    size_t best = 0;
    for (size_t i = 1; i < streams.size(); ++i)
      if (users[i] < users[best]) best = i;
    ++users[best];
    s->stream = streams[best];
    s->stream_idx = int(best);
  }
  *out = std::move(s);
  return BFRS_OK;
}

void CodecPool::release(std::unique_ptr<CodecSlot> slot) {
  if (!slot) return;
  DeviceScope scope(device);  // a slot dropped below is freed on its own device
  (void)slot->sync();
  // and whatever else the slot's own streams still hold (the slab wrappers'
  // second stream): the next user must find the rows idle
  if (slot->aux) (void)hipStreamSynchronize(slot->aux);
  if (slot->own_stream && slot->stream) (void)hipStreamSynchronize(slot->stream);
  std::unique_ptr<CodecSlot> drop;  // freed after the lock is released
  {
    std::lock_guard<std::mutex> g(mu);
    if (slot->stream_idx >= 0) {  // give the shared stream back
      --users[size_t(slot->stream_idx)];
      slot->stream_idx = -1;
    }
    if (free.size() < cached) {
      free.push_back(std::move(slot));
      return;
    }
    if (!free.empty()) {  // full: keep the larger of the smallest idle slot and this one
      size_t small = 0;
      for (size_t i = 1; i < free.size(); ++i)
        if (free[i]->stride * free[i]->nshards < free[small]->stride * free[small]->nshards)
          small = i;
      if (free[small]->stride * free[small]->nshards < slot->stride * slot->nshards)
        std::swap(free[small], slot);
    }
    drop = std::move(slot);
  }
}

CodecPool::~CodecPool() {
  DeviceScope scope(device);
  free.clear();
  for (hipStream_t st : streams) {
    (void)hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
  }
  for (hipStream_t st : {h2d, d2h})
    if (st) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
    }
}

Context::~Context() {
  DeviceScope scope(device);
  if (stream) (void)hipStreamSynchronize(stream);
  codec_pool.reset();  // idle slots go now; live codec objects keep the pool
  staging.reset();  // archive staging arenas (pinned + device)
  plans.clear();
  for (auto &ps : pipe_stream)
    if (ps) {
      (void)hipStreamSynchronize(ps);
      (void)hipStreamDestroy(ps);
    }
  if (pipe_buf) (void)hipFree(pipe_buf);
  if (d_hash) (void)hipFree(d_hash);
  if (h_hash) (void)hipHostFree(h_hash);
  if (stream) (void)hipStreamDestroy(stream);
}

int Context::init(int dev) {
  // a kernel this build does not carry is refused before anything else
  // (the A/B variants and probes exist only in libbfrs_ab.so)
  if (kernel_variant() < 0)
    return set_error(BFRS_E_INVALID_ARGUMENT,
                     std::string("BFRS_KERNEL_VARIANT=") + std::getenv("BFRS_KERNEL_VARIANT") +
#ifdef BFRS_AB_VARIANTS
                         " is not a known kernel variant (probes need BFRS_ALLOW_PROBE=1)"
#else
                         " is not built into this library (product kernels: 76, 75, "
                         "73; A/B variants: make ab -> libbfrs_ab.so)"
#endif
    );
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    return set_error(BFRS_E_NO_DEVICE, "no HIP device available (no CPU fallback)");
  if (dev < 0 || dev >= n) return set_error(BFRS_E_NO_DEVICE, "HIP device id out of range");
  device = dev;
  if (const char *e = std::getenv("BFRS_PLAN_CACHE")) max_plans = std::max(1, atoi(e));
  if (const char *e = BFRS_AB_KNOB("BFRS_PIPE_SLOTS"))
    pipe_slots = std::min(kPipeSlotsMax, std::max(2, atoi(e)));
  codec_pool->device = dev;
  if (const char *e = std::getenv("BFRS_CODEC_SLOTS")) {
    char *end = nullptr;
    const long v = std::strtol(e, &end, 10);
    codec_pool->cached = (end != e && v > 0) ? size_t(std::min<long>(v, 1024)) : 0;
  }
  if (const char *e = std::getenv("BFRS_CODEC_STAGING")) {
    if (std::strcmp(e, "direct") == 0)
      codec_pool->staging = Staging::kDirect;
    else if (std::strcmp(e, "pinned") != 0 && *e)
      return set_error(BFRS_E_INVALID_ARGUMENT,
                       std::string("BFRS_CODEC_STAGING=") + e + ": expected direct or pinned");
  }
  // defaults: one stream per slot, copies on it (rounds 2-3); the shared
  // stream set and the FIFO copy streams are kept as options: neither was
  // consistently faster in the bench process
  size_t codec_streams = 0;
  if (const char *e = BFRS_AB_KNOB("BFRS_CODEC_STREAMS")) {
    char *end = nullptr;
    const long v = std::strtol(e, &end, 10);
    if (end == e || v < 0 || v > 64)
      return set_error(BFRS_E_INVALID_ARGUMENT,
                       std::string("BFRS_CODEC_STREAMS=") + e + ": expected 0..64");
    codec_streams = size_t(v);
  }
  bool copy_streams = false;
  if (const char *e = BFRS_AB_KNOB("BFRS_CODEC_COPIES")) {
    if (std::strcmp(e, "stream") == 0)
      copy_streams = true;
    else if (std::strcmp(e, "slot") != 0 && *e)
      return set_error(BFRS_E_INVALID_ARGUMENT,
                       std::string("BFRS_CODEC_COPIES=") + e + ": expected stream or slot");
  }
  HIP_TRY(hipSetDevice(dev));
  // the codec streams first: created before any copy, consecutively
  if (int rc = codec_pool->init_streams(codec_streams, copy_streams)) return rc;
  HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  for (int i = 0; i < pipe_slots; ++i)
    HIP_TRY(hipStreamCreateWithFlags(&pipe_stream[i], hipStreamNonBlocking));
  return BFRS_OK;
}

int Context::run_host(bool decode, size_t nblocks, const uint32_t *ks, size_t m,
                      size_t shard_bytes, const uint8_t *const *orig, const uint8_t *const *rec,
                      uint8_t *const *out) {
  std::lock_guard<std::mutex> pipe_lock(pipe_mu);
  // Slab width: whole 64-byte chunks, ~8 MiB of columns per shard (env
  // BFRS_SLAB_BYTES overrides), the shard's tail chunk rides in the last slab.
  size_t slab = 8u << 20;
  if (const char *e = BFRS_AB_KNOB("BFRS_SLAB_BYTES")) slab = std::max<size_t>(64, atoll(e));
  slab = std::max<size_t>(64, slab / 64 * 64);
  if (slab >= shard_bytes) slab = shard_bytes;
  size_t kmax = 0;
  for (size_t b = 0; b < nblocks; ++b) kmax = std::max<size_t>(kmax, ks[b]);
  // slab + 64 covers a last slab that carries the tail chunk; stride 256-aligned
  const size_t stride = round_up(slab + 64, 256);
  const size_t need = stride * (kmax + m);
  if (need > pipe_cap) {
    for (int i = 0; i < pipe_slots; ++i) HIP_TRY(hipStreamSynchronize(pipe_stream[i]));
    if (pipe_buf) HIP_TRY(hipFree(pipe_buf));
    pipe_buf = nullptr;
    pipe_cap = 0;
    HIP_TRY(hipMalloc(&pipe_buf, need * pipe_slots));
    pipe_cap = need;
  }
  int slot = 0;
  size_t oi = 0;
  std::vector<RowCopy> h2d, d2h;
  for (size_t b = 0; b < nblocks; ++b) {
    const size_t k = ks[b];
    const uint8_t *const *bo = orig + oi;
    const uint8_t *const *br = decode ? rec + b * m : nullptr;
    uint8_t *const *bout = decode ? out + oi : out + b * m;
    oi += k;
    for (size_t off = 0; off < shard_bytes;) {
      size_t len = std::min(slab, shard_bytes - off);
      if (shard_bytes - (off + len) < 64) len = shard_bytes - off;  // fold the tail in
      hipStream_t st = pipe_stream[slot];
      uint8_t *base = static_cast<uint8_t *>(pipe_buf) + size_t(slot) * pipe_cap;
      std::vector<const uint8_t *> din(k, nullptr), drec(m, nullptr);
      std::vector<uint8_t *> dout(decode ? k : m, nullptr);
      h2d.clear();
      for (size_t i = 0; i < k; ++i) {
        if (!bo[i]) {
          if (decode) dout[i] = base + i * stride;
          continue;
        }
        din[i] = base + i * stride;
        h2d.push_back({base + i * stride, bo[i] + off});
      }
      for (size_t j = 0; j < m; ++j) {
        uint8_t *d = base + (kmax + j) * stride;
        if (decode) {
          if (!br[j]) continue;
          drec[j] = d;
          h2d.push_back({d, br[j] + off});
        } else {
          dout[j] = d;
        }
      }
      if (int rc = copy_rows(h2d, len, hipMemcpyHostToDevice, st)) return rc;
      uint32_t kk = uint32_t(k);
      bfrs_ctx *self = reinterpret_cast<bfrs_ctx *>(this);
      int rc = decode ? decode_batch_on(self, 1, &kk, m, len, din.data(), drec.data(),
                                        dout.data(), st)
                      : encode_batch_on(self, 1, &kk, m, len, din.data(), dout.data(), st);
      if (rc) return rc;
      d2h.clear();
      for (size_t t = 0; t < dout.size(); ++t)
        if (dout[t]) d2h.push_back({bout[t] + off, dout[t]});
      if ((rc = copy_rows(d2h, len, hipMemcpyDeviceToHost, st))) return rc;
      slot = (slot + 1) % pipe_slots;
      off += len;
    }
  }
  for (int i = 0; i < pipe_slots; ++i) HIP_TRY(hipStreamSynchronize(pipe_stream[i]));
  return BFRS_OK;
}

namespace {
// Cache lookup / insert under Context::mu.  When the cache is full, the
// least recently used half of the plans nobody else holds is dropped, after a
// device synchronize: a plan's tables may still be read by queued kernels of
// an earlier call even when no BlockIO holds it any more.
template <typename Make>
int cached_plan(Context &c, const std::string &key, Make make, PlanRef *out) {
  std::lock_guard<std::mutex> g(c.mu);
  auto it = c.plans.find(key);
  if (it == c.plans.end()) {
    if (c.plans.size() >= c.max_plans) {
      std::vector<std::pair<uint64_t, std::string>> idle;
      for (auto &kv : c.plans)
        if (kv.second.use_count() == 1) idle.emplace_back(kv.second->last_use, kv.first);
      if (!idle.empty()) {
        HIP_TRY(hipDeviceSynchronize());
        std::sort(idle.begin(), idle.end());
        const size_t drop = std::max<size_t>(1, idle.size() / 2);
        for (size_t i = 0; i < drop; ++i) c.plans.erase(idle[i].second);
      }
    }
    auto p = std::make_shared<Plan>();
    p->coef = make();
    int rc = upload_plan(p.get());
    if (rc) return rc;
    it = c.plans.emplace(key, std::move(p)).first;
  }
  it->second->last_use = ++c.plan_tick;
  *out = it->second;
  return BFRS_OK;
}
}  // namespace

int Context::get_encode_plan(size_t k, size_t m, PlanRef *out) {
  return cached_plan(*this, "E" + std::to_string(k) + "," + std::to_string(m),
                     [&] { return plan_encode(k, m); }, out);
}

int Context::get_decode_plan(size_t k, size_t m, const std::vector<uint8_t> &orig_present,
                             const std::vector<uint8_t> &rec_present, PlanRef *out) {
  std::string key = "D" + std::to_string(k) + "," + std::to_string(m) + ":";
  for (uint8_t b : orig_present) key.push_back(b ? '1' : '0');
  key.push_back('/');
  for (uint8_t b : rec_present) key.push_back(b ? '1' : '0');
  return cached_plan(*this, key, [&] { return plan_decode(k, m, orig_present, rec_present); }, out);
}

int Context::run_blocks(const std::vector<BlockIO> &blocks, size_t shard_bytes, hipStream_t s) {
  if (shard_bytes <= kMaxWindowBytes) return run_window(blocks, shard_bytes, s);
  // column windows of kMaxWindowBytes (a multiple of 64: the crate's chunk
  // layout is per 64-byte chunk, so a window is a valid shard of its own);
  // the last window keeps the tail chunk
  std::vector<BlockIO> w = blocks;
  for (size_t off = 0; off < shard_bytes;) {
    size_t len = std::min(kMaxWindowBytes, shard_bytes - off);
    if (shard_bytes - (off + len) < 64) len = shard_bytes - off;
    for (size_t b = 0; b < blocks.size(); ++b) {
      for (size_t i = 0; i < blocks[b].in.size(); ++i) w[b].in[i] = blocks[b].in[i] + off;
      for (size_t i = 0; i < blocks[b].out.size(); ++i) w[b].out[i] = blocks[b].out[i] + off;
    }
    int rc = run_window(w, len, s);
    if (rc) return rc;
    off += len;
  }
  return BFRS_OK;
}

int Context::run_window(const std::vector<BlockIO> &blocks, size_t shard_bytes,
                        hipStream_t s) {
  const uint64_t full_chunks = shard_bytes / 64;
  const uint32_t tail = uint32_t(shard_bytes % 64);
  uint32_t max_phase = 0;
  for (const BlockIO &b : blocks) max_phase = std::max(max_phase, b.plan->n_phases);

  struct Item {
    const BlockIO *b;
    const PlanPass *p;
  };
  // Pointer slots a pass needs: inputs padded to even, +3 prefetch slots
  // (the kernels read up to 3 inputs past the end; duplicates of the last
  // input, served from cache, never consumed), outputs.
  constexpr uint32_t kPrefetchPad = 3;
  auto ptr_need = [](const PlanPass &p) {
    return ((p.c1 - p.c0 + 1) & ~1u) + kPrefetchPad + (p.r1 - p.r0);
  };

  for (uint32_t phase = 0; phase < max_phase; ++phase) {
    std::vector<Item> items;
    for (const BlockIO &b : blocks)
      for (const PlanPass &p : b.plan->passes)
        if (p.phase == phase) items.push_back({&b, &p});

    // Launches of up to kMaxLaunchPasses passes / kMaxLaunchPtrs pointers.
    for (size_t first = 0; first < items.size();) {
      size_t last = first, nptr = 0;
      while (last < items.size() && last - first < kMaxLaunchPasses &&
             nptr + ptr_need(*items[last].p) <= kMaxLaunchPtrs)
        nptr += ptr_need(*items[last++].p);
      if (last == first)
        return set_error(BFRS_E_INVALID_ARGUMENT, "pass exceeds one launch's pointer capacity");

      // Tile size of this launch (8 KiB; the A/B build's LDS-DMA variants
      // take wider tiles when every pass has an unrolled size).
      bool unrolled_sizes = true;
      for (size_t it = first; it < last; ++it) {
        const PlanPass &p = *items[it].p;
        const uint32_t n_pad = (p.c1 - p.c0 + 1) & ~1u;
        unrolled_sizes = unrolled_sizes && p.subfield && (n_pad == 30 || n_pad == 20 || n_pad == 8);
      }
      uint32_t tb = 0, n_tiles = 0, tpw = 1;
      for (;;) {
        tb = tile_bytes(unrolled_sizes);
        n_tiles = uint32_t((full_chunks * 64 + tb - 1) / tb);
        // Workgroup sizing: one tile per workgroup unless the grid is huge.
        const uint64_t total_tiles = uint64_t(n_tiles) * (last - first);
        tpw = uint32_t(std::max<uint64_t>(1, total_tiles / 65536));
        if (const char *e = BFRS_AB_KNOB("BFRS_TILES_PER_WG")) tpw = std::max(1, atoi(e));
        // the wide tiles exist only for one tile per workgroup: otherwise
        // the launch falls back to 8 KiB tiles, so size the grid for them
        if (tpw == 1 || !unrolled_sizes || tb == tile_bytes(false)) break;
        unrolled_sizes = false;
      }
      const uint32_t wgs_per_pass = (n_tiles + tpw - 1) / tpw;

      KernArgs ka{};
      ka.n_passes = uint32_t(last - first);
      ka.tiles_per_wg = tpw;
      uint32_t pi = 0, wg = 0, max_in = 0;
      bool subfield = true;
      for (size_t it = first; it < last; ++it) {
        const BlockIO &b = *items[it].b;
        const PlanPass &p = *items[it].p;
        PassDesc &d = ka.passes[it - first];
        const uint32_t n_real = p.c1 - p.c0, n_pad = (n_real + 1) & ~1u;
        d.in = pi;
        for (uint32_t c = p.c0; c < p.c1; ++c) ka.ptrs[pi++] = reinterpret_cast<uint64_t>(b.in[c]);
        const uint64_t lastp = reinterpret_cast<uint64_t>(b.in[p.c1 - 1]);
        for (uint32_t c = n_real; c < n_pad + kPrefetchPad; ++c) ka.ptrs[pi++] = lastp;
        d.out = pi;
        for (uint32_t r = p.r0; r < p.r1; ++r) ka.ptrs[pi++] = reinterpret_cast<uint64_t>(b.out[r]);
        d.table = reinterpret_cast<uint64_t>(p.d_table);
        subfield = subfield && p.subfield;
        d.n_in = n_pad;
        d.n_out = p.r1 - p.r0;
        d.wg_begin = wg;
        d.n_tiles = n_tiles;
        d.full_chunks = full_chunks;
        d.tail_bytes = tail;
        d.accumulate = phase > 0;
        d.rotate = n_real == n_pad;
        d.n_real = n_real;
        wg += wgs_per_pass;
        max_in = std::max(max_in, n_pad);
      }
      if (n_tiles) {
        if (kernel_variant() < 0)
          return set_error(BFRS_E_INVALID_ARGUMENT, "BFRS_KERNEL_VARIANT names a kernel this "
                                                    "library does not carry");
        HIP_TRY(launch_gf_apply(ka, wg, max_in, subfield, unrolled_sizes, s));
      }
      if (tail) HIP_TRY(launch_gf_tail(ka, s));
      first = last;
    }
  }
  return BFRS_OK;
}

}  // namespace bfrs

using namespace bfrs;

extern char **environ;

namespace {
// knobs of earlier rounds (BFRS_PREFETCH_WORKERS, the codec
// stream and copy layouts, ...) now live only in the measurement build, and
// libbfrs.so ignores them.  A deployment that still sets one is told so once
// per process on stderr instead of silently getting the default.  The scan
// goes by prefix so that no other knob name is written into the binary
// (tests/test_abi.py: the product names exactly the six of include/bfrs.h).
void warn_ignored_knobs() {
#ifndef BFRS_AB_VARIANTS
  static std::once_flag once;
  std::call_once(once, [] {
    static const char *const known[] = {"CODEC_SLOTS", "CODEC_STAGING", "HOST_COPY_BUDGET",
                                        "KERNEL_VARIANT", "PLAN_CACHE", "PREFETCH_DEPTH",
                                        "LIB" /* the Python binding's library choice */};
    const char prefix[] = {'B', 'F', 'R', 'S', '_'};
    for (char **e = environ; e && *e; ++e) {
      if (std::strncmp(*e, prefix, sizeof prefix) != 0) continue;
      const char *name = *e + sizeof prefix;
      const char *eq = std::strchr(name, '=');
      const size_t n = eq ? size_t(eq - name) : std::strlen(name);
      bool ok = false;
      for (const char *k : known) ok = ok || (std::strlen(k) == n && std::strncmp(k, name, n) == 0);
      if (!ok)
        std::fprintf(stderr,
                     "libbfrs: ignoring environment variable %.*s%.*s (not a knob of this "
                     "library; include/bfrs.h lists the six it reads)\n",
                     int(sizeof prefix), prefix, int(n), name);
    }
  });
#endif
}
}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

int bfrs_abi_version(void) { return BFRS_ABI_VERSION; }

const char *bfrs_strerror(int code) {
  switch (code) {
    case BFRS_OK: return "ok";
    case BFRS_E_DIFFERENT_SHARD_SIZE: return "different shard size";
    case BFRS_E_DUPLICATE_ORIGINAL_SHARD_INDEX: return "duplicate original shard index";
    case BFRS_E_DUPLICATE_RECOVERY_SHARD_INDEX: return "duplicate recovery shard index";
    case BFRS_E_INVALID_ORIGINAL_SHARD_INDEX: return "invalid original shard index";
    case BFRS_E_INVALID_RECOVERY_SHARD_INDEX: return "invalid recovery shard index";
    case BFRS_E_INVALID_SHARD_SIZE: return "invalid shard size";
    case BFRS_E_NOT_ENOUGH_SHARDS: return "not enough shards";
    case BFRS_E_TOO_FEW_ORIGINAL_SHARDS: return "too few original shards";
    case BFRS_E_TOO_MANY_ORIGINAL_SHARDS: return "too many original shards";
    case BFRS_E_UNSUPPORTED_SHARD_COUNT: return "unsupported shard count";
    case BFRS_E_WRAPPER: return "blockframe wrapper error";
    case BFRS_E_INVALID_ARGUMENT: return "invalid argument";
    case BFRS_E_HIP: return "HIP runtime error";
    case BFRS_E_NO_DEVICE: return "no HIP device";
    case BFRS_E_NOMEM: return "out of memory";
    case BFRS_E_NOT_RESTORED: return "original shard was not restored";
    case BFRS_E_NOT_FOUND: return "not found";
    default: return "unknown error";
  }
}

const char *bfrs_last_error(void) { return g_last_error.c_str(); }

size_t bfrs_shard_pitch(size_t shard_bytes) { return bfrs::shard_pitch(shard_bytes); }

int bfrs_device_count(void) {
  BFRS_API_BEGIN
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
  BFRS_API_END
}

int bfrs_open(int device, bfrs_ctx **out) {
  BFRS_API_BEGIN
  warn_ignored_knobs();
  if (!out) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_open: out is NULL");
  *out = nullptr;
  auto *c = new (std::nothrow) bfrs_ctx;
  if (!c) return set_error(BFRS_E_NOMEM, "bfrs_open: allocation failed");
  int rc = c->impl.init(device);
  if (rc) {
    delete c;
    return rc;
  }
  *out = c;
  return BFRS_OK;
  BFRS_API_END
}

void bfrs_close(bfrs_ctx *ctx) {
  if (!ctx) return;
  detach_archives(ctx);  // no prefetch thread of an open handle outlives the context
  delete ctx;
}

int bfrs_synchronize(bfrs_ctx *ctx) {
  BFRS_API_BEGIN
  if (!ctx) return set_error(BFRS_E_INVALID_ARGUMENT, "NULL context");
  HIP_TRY(hipSetDevice(ctx->impl.device));
  HIP_TRY(hipStreamSynchronize(ctx->impl.stream));
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_use_high_rate(size_t k, size_t m) {
  BFRS_API_BEGIN
  Rate r;
  if (!choose_rate(k, m, &r)) return BFRS_E_UNSUPPORTED_SHARD_COUNT;
  return r == Rate::kHigh ? 1 : 0;
  BFRS_API_END
}

int bfrs_encode_coefficient(size_t k, size_t m, size_t j, size_t i, uint16_t *coef_out) {
  BFRS_API_BEGIN
  if (!coef_out) return set_error(BFRS_E_INVALID_ARGUMENT, "coef_out is NULL");
  int rc = check_shape(k, m, 2);
  if (rc) return rc;
  if (j >= m || i >= k) return set_error(BFRS_E_INVALID_ARGUMENT, "index out of range");
  CoefMatrix c = plan_encode(k, m);
  *coef_out = c.at(j, i);
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_plan_decode(size_t k, size_t m, const uint8_t *orig_present, const uint8_t *rec_present,
                     uint16_t *coef_out, size_t cap, size_t *rows, size_t *cols) {
  BFRS_API_BEGIN
  if (!orig_present || !rec_present || !rows || !cols)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_plan_decode: NULL argument");
  int rc = check_shape(k, m, 2);
  if (rc) return rc;
  std::vector<uint8_t> op(orig_present, orig_present + k), rp(rec_present, rec_present + m);
  size_t orecv = 0, rrecv = 0;
  for (uint8_t b : op) orecv += b != 0;
  for (uint8_t b : rp) rrecv += b != 0;
  if (orecv + rrecv < k) return set_error(BFRS_E_NOT_ENOUGH_SHARDS, "not enough shards");
  if (orecv == k) {
    *rows = 0;
    *cols = 0;
    return BFRS_OK;
  }
  CoefMatrix c = plan_decode(k, m, op, rp);
  *rows = c.rows;
  *cols = c.cols;
  if (coef_out && cap >= c.c.size()) std::copy(c.c.begin(), c.c.end(), coef_out);
  return BFRS_OK;
  BFRS_API_END
}

// ---- batch (device-resident) ------------------------------------------------
int check_dev_ptr(const void *p, const char *what) {
  if (!p) return set_error(BFRS_E_INVALID_ARGUMENT, std::string(what) + " is NULL");
  if (reinterpret_cast<uintptr_t>(p) & 15)
    return set_error(BFRS_E_INVALID_ARGUMENT, std::string(what) + " is not 16-byte aligned");
  return BFRS_OK;
}

int bfrs_encode_batch_dev(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                          size_t shard_bytes, const uint8_t *const *d_orig,
                          uint8_t *const *d_rec, void *hip_stream) {
  BFRS_API_BEGIN
  return encode_batch_on(ctx, nblocks, ks, m, shard_bytes, d_orig, d_rec,
                         static_cast<hipStream_t>(hip_stream));
  BFRS_API_END
}

int bfrs_decode_batch_dev(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                          size_t shard_bytes, const uint8_t *const *d_orig,
                          const uint8_t *const *d_rec, uint8_t *const *d_restored,
                          void *hip_stream) {
  BFRS_API_BEGIN
  return decode_batch_on(ctx, nblocks, ks, m, shard_bytes, d_orig, d_rec, d_restored,
                         static_cast<hipStream_t>(hip_stream));
  BFRS_API_END
}

}  // extern "C"

namespace bfrs {

int encode_batch_on(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                    size_t shard_bytes, const uint8_t *const *d_orig, uint8_t *const *d_rec,
                    hipStream_t s) {
  if (!ctx || (nblocks && (!ks || !d_orig || !d_rec)))
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_encode_batch_dev: NULL argument");
  Context &c = ctx->impl;
  HIP_TRY(hipSetDevice(c.device));
  std::vector<BlockIO> blocks(nblocks);
  size_t oi = 0;
  for (size_t b = 0; b < nblocks; ++b) {
    int rc = check_shape(ks[b], m, shard_bytes);
    if (rc) return rc;
    rc = c.get_encode_plan(ks[b], m, &blocks[b].plan);
    if (rc) return rc;
    blocks[b].in.resize(ks[b]);
    for (uint32_t i = 0; i < ks[b]; ++i) {
      if ((rc = check_dev_ptr(d_orig[oi], "original shard pointer"))) return rc;
      blocks[b].in[i] = d_orig[oi++];
    }
    blocks[b].out.resize(m);
    for (size_t j = 0; j < m; ++j) {
      if ((rc = check_dev_ptr(d_rec[b * m + j], "recovery shard pointer"))) return rc;
      blocks[b].out[j] = d_rec[b * m + j];
    }
  }
  return c.run_blocks(blocks, shard_bytes, s);
}

int decode_batch_on(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                    size_t shard_bytes, const uint8_t *const *d_orig, const uint8_t *const *d_rec,
                    uint8_t *const *d_restored, hipStream_t s) {
  if (!ctx || (nblocks && (!ks || !d_orig || !d_rec || !d_restored)))
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_decode_batch_dev: NULL argument");
  Context &c = ctx->impl;
  HIP_TRY(hipSetDevice(c.device));
  std::vector<BlockIO> blocks;
  blocks.reserve(nblocks);
  size_t oi = 0;
  for (size_t b = 0; b < nblocks; ++b) {
    const size_t k = ks[b];
    int rc = check_shape(k, m, shard_bytes);
    if (rc) return rc;
    std::vector<uint8_t> op(k), rp(m);
    size_t orig_recv = 0, rec_recv = 0;
    for (size_t i = 0; i < k; ++i) orig_recv += (op[i] = d_orig[oi + i] != nullptr);
    for (size_t j = 0; j < m; ++j) rec_recv += (rp[j] = d_rec[b * m + j] != nullptr);
    if (orig_recv + rec_recv < k) {
      std::ostringstream os;
      os << "not enough shards: " << orig_recv << " original + " << rec_recv << " recovery < "
         << k << " original_count";
      return set_error(BFRS_E_NOT_ENOUGH_SHARDS, os.str());
    }
    if (orig_recv == k) {  // nothing to restore (crate returns an empty result)
      oi += k;
      continue;
    }
    BlockIO io;
    if ((rc = c.get_decode_plan(k, m, op, rp, &io.plan))) return rc;
    for (size_t j = 0; j < m; ++j)
      if (rp[j]) {
        if ((rc = check_dev_ptr(d_rec[b * m + j], "recovery shard pointer"))) return rc;
        io.in.push_back(d_rec[b * m + j]);
      }
    for (size_t i = 0; i < k; ++i)
      if (op[i]) {
        if ((rc = check_dev_ptr(d_orig[oi + i], "original shard pointer"))) return rc;
        io.in.push_back(d_orig[oi + i]);
      } else {
        if ((rc = check_dev_ptr(d_restored[oi + i], "restored shard pointer"))) return rc;
        io.out.push_back(d_restored[oi + i]);
      }
    oi += k;
    blocks.push_back(std::move(io));
  }
  return c.run_blocks(blocks, shard_bytes, s);
}

}  // namespace bfrs

// ---- host-memory API: pipelined through HBM ----------------------------------
int bfrs::check_host_batch(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                           size_t shard_bytes, bool decode, const uint8_t *const *orig,
                           const uint8_t *const *rec, uint8_t *const *out) {
  if (!ctx || (nblocks && (!ks || !orig || !out || (decode && !rec))))
    return set_error(BFRS_E_INVALID_ARGUMENT, "host batch: NULL argument");
  size_t oi = 0;
  for (size_t b = 0; b < nblocks; ++b) {
    int rc = check_shape(ks[b], m, shard_bytes);
    if (rc) return rc;
    size_t orecv = 0, rrecv = 0;
    for (size_t i = 0; i < ks[b]; ++i) {
      orecv += orig[oi + i] != nullptr;
      if (!decode && !orig[oi + i]) return set_error(BFRS_E_INVALID_ARGUMENT, "original is NULL");
      if (decode && !orig[oi + i] && !out[oi + i])
        return set_error(BFRS_E_INVALID_ARGUMENT, "restored buffer for erased shard is NULL");
    }
    if (decode) {
      for (size_t j = 0; j < m; ++j) rrecv += rec[b * m + j] != nullptr;
      if (orecv + rrecv < ks[b]) {
        std::ostringstream os;
        os << "not enough shards: " << orecv << " original + " << rrecv << " recovery < "
           << ks[b] << " original_count";
        return set_error(BFRS_E_NOT_ENOUGH_SHARDS, os.str());
      }
    } else {
      for (size_t j = 0; j < m; ++j)
        if (!out[b * m + j]) return set_error(BFRS_E_INVALID_ARGUMENT, "recovery buffer is NULL");
    }
    oi += ks[b];
  }
  return BFRS_OK;
}

extern "C" {

int bfrs_encode_host_batch(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                           size_t shard_bytes, const uint8_t *const *orig,
                           uint8_t *const *rec_out) {
  BFRS_API_BEGIN
  int rc = check_host_batch(ctx, nblocks, ks, m, shard_bytes, false, orig, nullptr, rec_out);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(ctx->impl.device));
  return ctx->impl.run_host(false, nblocks, ks, m, shard_bytes, orig, nullptr, rec_out);
  BFRS_API_END
}

int bfrs_decode_host_batch(bfrs_ctx *ctx, size_t nblocks, const uint32_t *ks, size_t m,
                           size_t shard_bytes, const uint8_t *const *orig,
                           const uint8_t *const *rec, uint8_t *const *restored_out) {
  BFRS_API_BEGIN
  int rc = check_host_batch(ctx, nblocks, ks, m, shard_bytes, true, orig, rec, restored_out);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(ctx->impl.device));
  return ctx->impl.run_host(true, nblocks, ks, m, shard_bytes, orig, rec, restored_out);
  BFRS_API_END
}

int bfrs_encode(bfrs_ctx *ctx, size_t k, size_t m, size_t shard_bytes,
                const uint8_t *const *originals, uint8_t *const *recovery_out) {
  BFRS_API_BEGIN
  if (!ctx || !originals || !recovery_out)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_encode: NULL argument");
  int rc = check_shape(k, m, shard_bytes);
  if (rc) return rc;
  const uint32_t kk = uint32_t(k);
  return bfrs_encode_host_batch(ctx, 1, &kk, m, shard_bytes, originals, recovery_out);
  BFRS_API_END
}

int bfrs_decode(bfrs_ctx *ctx, size_t k, size_t m, size_t shard_bytes,
                const uint8_t *const *originals, const uint8_t *const *recovery,
                uint8_t *const *restored_out) {
  BFRS_API_BEGIN
  if (!ctx || !originals || !recovery || !restored_out)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_decode: NULL argument");
  int rc = check_shape(k, m, shard_bytes);
  if (rc) return rc;
  const uint32_t kk = uint32_t(k);
  return bfrs_decode_host_batch(ctx, 1, &kk, m, shard_bytes, originals, recovery, restored_out);
  BFRS_API_END
}

}  // extern "C"
