// tsan_host.cpp — ThreadSanitizer driver for libbfrs.so's threaded host code
// (test infrastructure: make -C blockframe-rs_amd/csrc host-tsan,
// tests/test_sanitize.py).
//
// 1. bfrs::blake3_hash with 1..16 threads on sizes around the tree's
//    boundaries (1 KiB chunks, power-of-two subtrees): the subtree threads
//    must give the single-thread digest;
// 2. bfrs::host_copy (up to 8 copy threads, within the process-wide helper
//    budget) called from 4 threads at once, as codec objects on several rayon
//    workers do (codec_objects.cpp); sizes whose parts end in a remainder,
//    canaries past the end (tests/test_sanitize.py also runs it with
//    BFRS_HOST_COPY_BUDGET=3, so the part counts vary between callers);
// 3. both at once.
// Exit 0 = every result equal; TSan reports go to stderr (exit 66).
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "blake3.hpp"
#include "host_copy.hpp"

namespace {

std::vector<uint8_t> bytes(size_t n, uint64_t seed) {
  std::vector<uint8_t> v(n);
  uint64_t x = seed;
  for (size_t i = 0; i < n; ++i) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    v[i] = uint8_t(z ^ (z >> 31));
  }
  return v;
}

bool hash_checks() {
  const size_t sizes[] = {0, 1, 1023, 1024, 1025, 4096, 65536 - 1, 65536 + 1,
                          (1u << 20) + 7, (3u << 20) + 1024 * 5 + 3, 5u << 20};
  for (size_t n : sizes) {
    const std::vector<uint8_t> d = bytes(n, n + 1);
    const std::string want = bfrs::blake3_hex(d.data(), n, 1);
    for (int t : {2, 3, 4, 7, 8, 16})
      if (bfrs::blake3_hex(d.data(), n, t) != want) {
        std::fprintf(stderr, "blake3 %zu bytes, %d threads: digest differs\n", n, t);
        return false;
      }
  }
  return true;
}

bool copy_checks() {
  // (12 MiB + 2) and (32 MiB + 2) split into 3 and 8 parts of a 64-B multiple
  // plus a remainder: the round-2/3 part size dropped those last bytes
  const size_t sizes[] = {100, (4u << 20) - 1, 8u << 20, (12u << 20) + 2, (17u << 20) + 17,
                          (24u << 20) + 6, (32u << 20) + 2};
  constexpr size_t kCanary = 64;
  bool ok = true;
  std::vector<std::thread> th;
  std::vector<int> good(4, 0);
  for (int w = 0; w < 4; ++w)
    th.emplace_back([&, w] {
      int g = 1;
      for (size_t n : sizes) {
        const std::vector<uint8_t> src = bytes(n, 77 + w);
        std::vector<uint8_t> dst(n + kCanary, 0xA5);
        bfrs::host_copy(dst.data(), src.data(), n);
        g &= std::memcmp(dst.data(), src.data(), n) == 0;
        for (size_t i = n; i < n + kCanary; ++i) g &= dst[i] == 0xA5;  // nothing past n
      }
      good[w] = g;
    });
  for (auto &t : th) t.join();
  for (int g : good) ok = ok && g;
  if (!ok) std::fprintf(stderr, "host_copy result differs\n");
  return ok;
}

}  // namespace

int main() {
  if (!hash_checks() || !copy_checks()) return 1;
  bool a = false, b = false;
  std::thread t1([&] { a = hash_checks(); });
  std::thread t2([&] { b = copy_checks(); });
  t1.join();
  t2.join();
  if (!a || !b) return 1;
  std::printf("tsan_host ok: threaded BLAKE3 and host_copy, alone and concurrent\n");
  return 0;
}
