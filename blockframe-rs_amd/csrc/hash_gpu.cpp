// hash_gpu.cpp — host side of the device BLAKE3 (blake3_kernels.hip):
// splits messages into 256 KiB groups, plans the CV reduction levels, and
// exposes bfrs_blake3_batch_dev / bfrs_blake3_combine.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "blake3.hpp"
#include "hash_kernels.hpp"
#include "runtime.hpp"

namespace bfrs {

namespace {
size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
// Narrow tree levels by quads (the product); the measurement build also
// takes BFRS_B3_QUADS=0, read per call (same-process A/B, tools/b3_levels_ab.py).
bool quads() {
#ifdef BFRS_AB_VARIANTS
  const char *e = std::getenv("BFRS_B3_QUADS");
  if (e && std::strcmp(e, "0") == 0) return false;
#endif
  return true;
}
}  // namespace

int Context::blake3_dev(size_t n, const uint8_t *const *d_msgs, const size_t *lens,
                        const uint64_t *chunk_offsets, uint8_t *digests, uint8_t *cvs,
                        hipStream_t s) {
  if (n == 0) return BFRS_OK;
  if (!d_msgs || !lens || !digests)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_blake3_batch_dev: NULL argument");
  if (n > (1u << 30)) return set_error(BFRS_E_INVALID_ARGUMENT, "too many messages");
  // the work areas below are per context; archive handles call this from
  // their prefetch threads while the owner may hash on the same context
  std::lock_guard<std::mutex> hash_lock(hash_mu);
  HIP_TRY(hipSetDevice(device));

  // kernel-1 workgroups: messages in order, groups of a message contiguous;
  // one descriptor per message (the kernel finds its message by group index)
  std::vector<HashMsg> msgs(n);
  std::vector<uint32_t> g_first(n), g_count(n);
  size_t n_groups = 0;
  for (size_t i = 0; i < n; ++i) {
    if (lens[i] && !d_msgs[i])
      return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_blake3_batch_dev: NULL message");
    if (reinterpret_cast<uintptr_t>(d_msgs[i]) % 16)
      return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_blake3_batch_dev: message not 16-byte aligned");
    const size_t ng = lens[i] == 0 ? 1 : (lens[i] + kGroupBytes - 1) / kGroupBytes;
    if (n_groups + ng > (size_t(1) << 31))
      return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_blake3_batch_dev: batch too large");
    g_first[i] = uint32_t(n_groups);
    g_count[i] = uint32_t(ng);
    msgs[i] = HashMsg{reinterpret_cast<uint64_t>(d_msgs[i]), chunk_offsets ? chunk_offsets[i] : 0,
                      uint64_t(lens[i]), uint32_t(n_groups), uint32_t(ng)};
    n_groups += ng;
  }
  // reduction levels: level L's nodes of message i are cur[off[i], off[i]+cnt[i]).
  // Kernel 1 leaves a multi-group message's level-kGroupLevels nodes
  // (256 >> levels per full group, ceil(chunks / 2^levels) for its last
  // one) at group index * (256 >> levels).
  std::vector<std::vector<HashReduce>> levels;
  std::vector<uint32_t> cnt(n), off(n);
  const uint32_t glv = kGroupLevels, group_out = kGroupChunks >> glv;
  const bool q = quads();
  for (size_t i = 0; i < n; ++i) {
    if (g_count[i] == 1) {  // finalised by kernel 1
      cnt[i] = 1;
      continue;
    }
    const size_t last = lens[i] - size_t(g_count[i] - 1) * kGroupBytes;
    const uint32_t last_nodes =
        uint32_t(((last + kChunkBytes - 1) / kChunkBytes + (1u << glv) - 1) >> glv);
    off[i] = g_first[i] * group_out;
    cnt[i] = (g_count[i] - 1) * group_out + last_nodes;
  }
  for (;;) {
    std::vector<HashReduce> jobs;
    uint32_t next = 0;
    bool more = false;
    for (size_t i = 0; i < n; ++i) {
      if (cnt[i] <= 1) continue;  // finished (or finalised by kernel 1)
      if (cnt[i] <= kReduceFanIn) {
        jobs.push_back({off[i], cnt[i], 0, 1, uint32_t(i), {0, 0, 0}});
        cnt[i] = 0;
        continue;
      }
      const uint32_t runs = (cnt[i] + kReduceFanIn - 1) / kReduceFanIn;
      for (uint32_t r = 0; r < runs; ++r) {
        const uint32_t nn = cnt[i] - r * kReduceFanIn < kReduceFanIn ? cnt[i] - r * kReduceFanIn
                                                                      : kReduceFanIn;
        jobs.push_back({off[i] + r * kReduceFanIn, nn, next + r, 0, uint32_t(i), {0, 0, 0}});
      }
      off[i] = next;
      cnt[i] = runs;
      next += runs;
      more = true;
    }
    if (jobs.empty()) break;
    levels.push_back(std::move(jobs));
    if (!more) break;
  }

  // device layout: msgs | jobs (all levels) | cvA | cvB | msg_cvs | digests
  size_t njobs = 0;
  for (auto &l : levels) njobs += l.size();
  const size_t b_groups = align_up(n * sizeof(HashMsg), 256);
  const size_t b_jobs = align_up(njobs * sizeof(HashReduce) + 16, 256);
  // cvA holds kernel 1's level-2 nodes (and later levels in place); cvB the
  // first reduce level's outputs, <= one per kReduceFanIn nodes per message
  const size_t b_cv = align_up(n_groups * group_out * 32, 256);
  const size_t b_cv1 = align_up((n_groups * group_out / kReduceFanIn + n + 1) * 32, 256);
  const size_t b_out = align_up(n * 32, 256);
  const size_t need = b_groups + b_jobs + b_cv + b_cv1 + 2 * b_out;
  const size_t h_need = b_groups + b_jobs + 2 * b_out;
  // Work areas grow rarely: at least 32 MiB / 1 MiB (a 4 GiB batch of
  // 32 MiB messages needs ~17 MiB) and doubling, because a regrow waits for
  // the whole device (a commit's next block is in flight on another stream)
  constexpr size_t kDevFloor = size_t(32) << 20, kHostFloor = size_t(1) << 20;
  if (need > d_hash_cap) {
    const size_t cap = std::max({need, kDevFloor, 2 * d_hash_cap});
    if (d_hash) {
      HIP_TRY(hipDeviceSynchronize());
      HIP_TRY(hipFree(d_hash));
      d_hash = nullptr;
      d_hash_cap = 0;
    }
    HIP_TRY(hipMalloc(&d_hash, cap));
    d_hash_cap = cap;
  }
  if (h_need > h_hash_cap) {
    const size_t cap = std::max({h_need, kHostFloor, 2 * h_hash_cap});
    if (h_hash) {
      HIP_TRY(hipDeviceSynchronize());
      HIP_TRY(hipHostFree(h_hash));
      h_hash = nullptr;
      h_hash_cap = 0;
    }
    HIP_TRY(hipHostMalloc(&h_hash, cap, hipHostMallocDefault));
    h_hash_cap = cap;
  }
  uint8_t *d = static_cast<uint8_t *>(d_hash);
  uint8_t *h = static_cast<uint8_t *>(h_hash);
  auto *d_hmsgs = reinterpret_cast<HashMsg *>(d);
  auto *d_jobs = reinterpret_cast<HashReduce *>(d + b_groups);
  auto *d_cv0 = reinterpret_cast<uint32_t *>(d + b_groups + b_jobs);
  auto *d_cv1 = reinterpret_cast<uint32_t *>(d + b_groups + b_jobs + b_cv);
  auto *d_msg_cvs = reinterpret_cast<uint32_t *>(d + b_groups + b_jobs + b_cv + b_cv1);
  auto *d_digests = reinterpret_cast<uint32_t *>(d + b_groups + b_jobs + b_cv + b_cv1 + b_out);
  // descriptors through pinned memory (one async copy)
  std::memcpy(h, msgs.data(), n * sizeof(HashMsg));
  size_t jo = 0;
  for (auto &l : levels) {
    std::memcpy(h + b_groups + jo * sizeof(HashReduce), l.data(), l.size() * sizeof(HashReduce));
    jo += l.size();
  }
  HIP_TRY(hipMemcpyAsync(d, h, b_groups + b_jobs, hipMemcpyHostToDevice, s));
  HIP_TRY(launch_blake3_groups(d_hmsgs, uint32_t(n), uint32_t(n_groups), glv, d_cv0, d_msg_cvs,
                               d_digests, s));
  uint32_t *cur = d_cv0, *nxt = d_cv1;
  jo = 0;
  for (auto &l : levels) {
    HIP_TRY(launch_blake3_reduce(d_jobs + jo, uint32_t(l.size()), q, cur, nxt, d_msg_cvs, d_digests,
                                 s));
    jo += l.size();
    std::swap(cur, nxt);
  }
  uint8_t *h_digests = h + b_groups + b_jobs;
  uint8_t *h_cvs = h_digests + b_out;
  HIP_TRY(hipMemcpyAsync(h_digests, d_digests, n * 32, hipMemcpyDeviceToHost, s));
  if (cvs) HIP_TRY(hipMemcpyAsync(h_cvs, d_msg_cvs, n * 32, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  std::memcpy(digests, h_digests, n * 32);
  if (cvs) std::memcpy(cvs, h_cvs, n * 32);
  return BFRS_OK;
}

}  // namespace bfrs

extern "C" {

int bfrs_blake3_batch_dev(bfrs_ctx *ctx, size_t n, const uint8_t *const *d_msgs, const size_t *lens,
                          const uint64_t *chunk_offsets, uint8_t *digests_out, uint8_t *cvs_out,
                          void *hip_stream) {
  BFRS_API_BEGIN
  if (!ctx) return bfrs::set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_blake3_batch_dev: NULL context");
  return ctx->impl.blake3_dev(n, d_msgs, lens, chunk_offsets, digests_out, cvs_out,
                              static_cast<hipStream_t>(hip_stream));
  BFRS_API_END
}

int bfrs_blake3_combine(const uint8_t *cvs, size_t n, char *out65) {
  BFRS_API_BEGIN
  if (!cvs || !out65 || n < 2)
    return bfrs::set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_blake3_combine: need >= 2 CVs");
  const std::string h = bfrs::blake3_combine_cvs_hex(cvs, n);
  std::memcpy(out65, h.c_str(), 65);
  return BFRS_OK;
  BFRS_API_END
}

}  // extern "C"
