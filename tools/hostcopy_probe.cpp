// hostcopy_probe.cpp — what bounds the crate-shaped path (bfrs_generate_parity
// with pageable caller buffers)?  Times, for 30 x 32 MiB shards:
//   copy_T<n>      pageable -> pinned memcpy over n threads (host_copy's shape,
//                  fresh threads per shard)
//   h2d_pinned     hipMemcpyAsync pinned -> device
//   h2d_pageable   hipMemcpyAsync straight from the pageable buffer
//   h2d_register   hipHostRegister + H2D + hipHostUnregister per shard
//   pipe_T<n>      copy_T<n> of shard i+1 overlapped with the H2D of shard i
// One JSON line per measurement (GB/s, best of 3).  No kernels.
// Build: hipcc -O2 -std=c++17 tools/hostcopy_probe.cpp -o tools/hostcopy_probe -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

static constexpr size_t kShard = 32u << 20, kN = 30;

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(uint8_t *dst, const uint8_t *src, size_t n, int nt) {
  if (nt <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  const size_t per = (n / nt + 63) / 64 * 64;
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) {
    const size_t a = t * per, b = std::min(n, a + per);
    if (a < b) th.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
  }
  std::memcpy(dst, src, std::min(n, per));
  for (auto &x : th) x.join();
}

static void report(const char *what, double secs) {
  std::printf("{\"probe\": \"%s\", \"GBps\": %.2f, \"ms\": %.2f}\n", what,
              double(kN * kShard) / secs / 1e9, secs * 1e3);
  std::fflush(stdout);
}

static double best3(const std::function<void()> &f) {
  double b = 1e30;
  for (int r = 0; r < 3; ++r) {
    const double t0 = now();
    f();
    b = std::min(b, now() - t0);
  }
  return b;
}

int main() {
  std::vector<uint8_t *> src(kN);
  for (auto &p : src) {
    p = static_cast<uint8_t *>(std::aligned_alloc(4096, kShard));
    for (size_t i = 0; i < kShard; i += 8) *reinterpret_cast<uint64_t *>(p + i) = i * 0x9E3779B97F4A7C15ull;
  }
  uint8_t *pinned = nullptr, *dev = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void **>(&pinned), kN * kShard, hipHostMallocDefault));
  CHECK(hipMalloc(&dev, kN * kShard));
  std::memset(pinned, 0, kN * kShard);
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

  for (int nt : {1, 2, 4, 8, 16}) {
    char name[32];
    std::snprintf(name, sizeof name, "copy_T%d", nt);
    report(name, best3([&] {
             for (size_t i = 0; i < kN; ++i) par_copy(pinned + i * kShard, src[i], kShard, nt);
           }));
  }
  report("h2d_pinned", best3([&] {
           for (size_t i = 0; i < kN; ++i)
             CHECK(hipMemcpyAsync(dev + i * kShard, pinned + i * kShard, kShard, hipMemcpyHostToDevice, st));
           CHECK(hipStreamSynchronize(st));
         }));
  report("h2d_pageable", best3([&] {
           for (size_t i = 0; i < kN; ++i)
             CHECK(hipMemcpyAsync(dev + i * kShard, src[i], kShard, hipMemcpyHostToDevice, st));
           CHECK(hipStreamSynchronize(st));
         }));
  report("h2d_register", best3([&] {
           for (size_t i = 0; i < kN; ++i) {
             CHECK(hipHostRegister(src[i], kShard, hipHostRegisterDefault));
             CHECK(hipMemcpyAsync(dev + i * kShard, src[i], kShard, hipMemcpyHostToDevice, st));
             CHECK(hipStreamSynchronize(st));
             CHECK(hipHostUnregister(src[i]));
           }
         }));
  for (int nt : {4, 8, 16}) {
    char name[32];
    std::snprintf(name, sizeof name, "pipe_T%d", nt);
    report(name, best3([&] {
             for (size_t i = 0; i < kN; ++i) {
               par_copy(pinned + i * kShard, src[i], kShard, nt);
               CHECK(hipMemcpyAsync(dev + i * kShard, pinned + i * kShard, kShard,
                                    hipMemcpyHostToDevice, st));
             }
             CHECK(hipStreamSynchronize(st));
           }));
  }
  CHECK(hipStreamDestroy(st));
  CHECK(hipFree(dev));
  CHECK(hipHostFree(pinned));
  for (auto p : src) std::free(p);
  return 0;
}
