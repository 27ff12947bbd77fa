// host_copy.cpp — multi-threaded host memcpy (pageable <-> pinned staging).
// Host-only (no HIP): also linked into the ThreadSanitizer driver
// (tools/tsan_host.cpp, make host-tsan).
#include "host_copy.hpp"
#include "knobs.hpp"

#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace bfrs {

namespace {

long env_long(const char *name, long dflt) {
  const char *e = std::getenv(name);
  return e && *e ? std::strtol(e, nullptr, 10) : dflt;
}

long ab_long(const char *value, long dflt) {  // a BFRS_AB_KNOB's value (knobs.hpp)
  return value && *value ? std::strtol(value, nullptr, 10) : dflt;
}

// CPUs this process may use: the affinity mask, capped by a cgroup-v2 CPU
// quota (the GPU boxes show 256 CPUs with a quota of 16).
long cpu_share() {
  cpu_set_t set;
  long n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 8;
  if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char quota[32] = {};
    long period = 0;
    if (std::fscanf(f, "%31s %ld", quota, &period) == 2 && std::strcmp(quota, "max") != 0 &&
        period > 0)
      n = std::min(n, std::max(1L, (std::strtol(quota, nullptr, 10) + period - 1) / period));
    std::fclose(f);
  }
  return std::max(1L, n);
}

// At most 8 threads per call (BFRS_HOST_COPY_THREADS, 1..8: measurement
// build only).
size_t max_parts() {
  static const size_t v = size_t(std::clamp(ab_long(BFRS_AB_KNOB("BFRS_HOST_COPY_THREADS"), 8), 1L, 8L));
  return v;
}

// Threads of all concurrent calls together stay within the process's CPU
// share (BFRS_HOST_COPY_BUDGET overrides the helper count, share - 1), split
// evenly between the calls in flight: rayon runs one generate_parity per
// block on every worker (commit.rs:391-466), and 5 blocks x 8 threads on a
// 16-CPU quota ran 5-15% slower than 5 x 4 (tools/rayon_probe.py, DESIGN.md
// §7c), while a block alone wants all 8.  The calling thread always copies
// its own part, so a call never waits for the budget.
std::atomic<long> g_helpers{0}, g_calls{0};
long helper_budget() {
  static const long v = std::max(0L, env_long("BFRS_HOST_COPY_BUDGET", cpu_share() - 1));
  return v;
}

// Reserve up to `want` helpers for a call while `calls` calls are in flight;
// returns how many were granted.
long reserve_helpers(long want, long calls) {
  const long budget = helper_budget();
  want = std::min(want, std::max(0L, (budget + 1) / std::max(1L, calls) - 1));
  long cur = g_helpers.load(std::memory_order_relaxed);
  while (want > 0) {
    const long take = std::min(want, budget - cur);
    if (take <= 0) return 0;
    if (g_helpers.compare_exchange_weak(cur, cur + take, std::memory_order_relaxed)) return take;
  }
  return 0;
}

}  // namespace

// Host copy into pinned memory: up to 8 threads of >= 4 MiB for large shards
// (one core copies ~10-20 GB/s from pageable memory; the PCIe link takes
// ~50 GB/s).  A thread that fails to start (thread quota) leaves its part to
// this thread; the started ones are always joined, so nothing terminates.
void host_copy(uint8_t *dst, const uint8_t *src, size_t n) {
  constexpr size_t kPart = 4u << 20, kMaxParts = 8;
  const size_t want = std::min<size_t>(max_parts(), n / kPart);
  if (want < 2) {
    std::memcpy(dst, src, n);
    return;
  }
  struct InFlight {  // this call counts toward the even split until it returns
    long calls = g_calls.fetch_add(1, std::memory_order_relaxed) + 1;
    ~InFlight() { g_calls.fetch_sub(1, std::memory_order_relaxed); }
  } in_flight;
  const long helpers = reserve_helpers(long(want) - 1, in_flight.calls);
  const size_t parts = size_t(helpers) + 1;
  if (parts < 2) {
    std::memcpy(dst, src, n);
    return;
  }
  // ceil(n / parts) rounded up to 64 B, so that the parts cover all n bytes
  const size_t per = ((n + parts - 1) / parts + 63) / 64 * 64;
  std::thread th[kMaxParts];
  bool started[kMaxParts] = {};
  for (size_t t = 1; t < parts; ++t) {
    const size_t a = std::min(n, t * per), b = std::min(n, a + per);
    try {
      th[t] = std::thread([=] { std::memcpy(dst + a, src + a, b - a); });
      started[t] = true;
    } catch (...) {  // std::system_error: copy this part here instead
      std::memcpy(dst + a, src + a, b - a);
    }
  }
  std::memcpy(dst, src, std::min(n, per));
  for (size_t t = 1; t < parts; ++t)
    if (started[t]) th[t].join();
  g_helpers.fetch_sub(helpers, std::memory_order_relaxed);
}

void prefault_range(uint8_t *p, size_t n) {
  if (!p || !n) return;
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
  static const uintptr_t page = uintptr_t(sysconf(_SC_PAGESIZE) > 0 ? sysconf(_SC_PAGESIZE) : 4096);
  static std::atomic<bool> populate_ok{[] {  // BFRS_PREFAULT_POPULATE=0: always touch (A/B)
    const char *e = BFRS_AB_KNOB("BFRS_PREFAULT_POPULATE");
    return !(e && e[0] == '0');
  }()};
  const uintptr_t a = reinterpret_cast<uintptr_t>(p), e = a + n;
  const uintptr_t lo = (a + page - 1) / page * page, hi = e / page * page;
  volatile uint8_t *q = p;
  if (hi > lo && populate_ok.load(std::memory_order_relaxed)) {
    if (madvise(reinterpret_cast<void *>(lo), hi - lo, MADV_POPULATE_WRITE) == 0) {
      q[0] = 0;  // the partial pages at either end
      q[n - 1] = 0;
      return;
    }
    // EINVAL: a kernel without MADV_POPULATE_WRITE, so touch from now on.
    // Anything else (EINTR, EAGAIN, or EFAULT / ENOMEM on an unusual mapping
    // of this caller) falls back for this call only.
    if (errno == EINVAL) populate_ok.store(false, std::memory_order_relaxed);
  }
  for (size_t o = 0; o < n; o += 4096) q[o] = 0;
  q[n - 1] = 0;
}

void host_copy_batch(const CopyJob *jobs, size_t count, void (*done)(void *, size_t), void *arg) {
  if (count == 0) return;
  size_t bytes = 0;
  for (size_t i = 0; i < count; ++i) bytes += jobs[i].n + jobs[i].pad;
  struct InFlight {
    long calls = g_calls.fetch_add(1, std::memory_order_relaxed) + 1;
    ~InFlight() { g_calls.fetch_sub(1, std::memory_order_relaxed); }
  } in_flight;
  constexpr size_t kPart = 4u << 20, kMaxParts = 8;
  const size_t want = std::min<size_t>({max_parts(), count, std::max<size_t>(1, bytes / kPart)});
  const long helpers = want > 1 ? reserve_helpers(long(want) - 1, in_flight.calls) : 0;
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < count;) {
      const CopyJob &j = jobs[i];
      if (j.n) std::memcpy(j.dst, j.src, j.n);
      if (j.pad) std::memset(j.dst + j.n, 0, j.pad);
      if (done) done(arg, i);
    }
  };
  std::thread th[kMaxParts];
  bool started[kMaxParts] = {};
  for (long t = 0; t < helpers && size_t(t) < kMaxParts; ++t) {
    try {
      th[t] = std::thread(work);
      started[t] = true;
    } catch (...) {  // no thread: the others take its jobs
    }
  }
  work();
  for (size_t t = 0; t < kMaxParts; ++t)
    if (started[t]) th[t].join();
  g_helpers.fetch_sub(helpers, std::memory_order_relaxed);
}

}  // namespace bfrs
