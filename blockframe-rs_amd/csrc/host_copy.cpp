// host_copy.cpp — multi-threaded host memcpy (pageable <-> pinned staging).
// Host-only (no HIP): also linked into the ThreadSanitizer driver
// (tools/tsan_host.cpp, make host-tsan).
#include "host_copy.hpp"

#include <algorithm>
#include <cstring>
#include <thread>

namespace bfrs {

// Host copy into pinned memory: up to 8 threads of >= 4 MiB for large shards
// (one core copies ~10-20 GB/s from pageable memory; the PCIe link takes
// ~50 GB/s).  A thread that fails to start (thread quota) leaves its part to
// this thread; the started ones are always joined, so nothing terminates.
void host_copy(uint8_t *dst, const uint8_t *src, size_t n) {
  constexpr size_t kPart = 4u << 20, kMaxParts = 8;
  const size_t parts = std::min<size_t>(kMaxParts, n / kPart);
  if (parts < 2) {
    std::memcpy(dst, src, n);
    return;
  }
  const size_t per = (n / parts + 63) / 64 * 64;
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
}

}  // namespace bfrs
