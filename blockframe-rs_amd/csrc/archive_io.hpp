// archive_io.hpp — file helpers, on-disk layout and manifest geometry shared
// by commit, repair and the read path:
//
//   {root}/{name}_{blake3}/manifest.json
//   tier 1: data.dat, parity_{0,1,2}.dat                               (commit.rs:25-118)
//   tier 2: segments/segment_{i}.dat, parity/segment_{i}_parity_{p}.dat (commit.rs:124-309)
//   tier 3: blocks/block_{b}/segments/segment_{s}.dat,
//           blocks/block_{b}/parity/block_parity_{p}.dat               (commit.rs:314-536)
#pragma once

#include <cstddef>
#include <cstdint>
#include <exception>
#include <functional>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "manifest.hpp"

namespace bfrs {

constexpr size_t kBlockSegments = 30;  // commit.rs:359,402
constexpr size_t kParity = 3;
// Geometry limits a manifest must respect (load_geometry): 2^50 B files
// (1 PiB) and 2^36 B segments (64 GiB; BlockFrame writes 32 MiB, utils.rs:68).
constexpr uint64_t kMaxFileBytes = uint64_t(1) << 50;
constexpr uint64_t kMaxSegmentBytes = uint64_t(1) << 36;

int io_error(const std::string &what);  // BFRS_E_WRAPPER + strerror(errno)
int hw_threads();                        // host worker threads (<= 16)
// f(i) for i in [0, n) on up to `threads` threads (fewer if a thread cannot
// be started).  Every thread is joined before it returns; the first exception
// thrown by f is rethrown then.
void parallel_for(size_t n, int threads, const std::function<void(size_t)> &f);

// A task on a thread of its own (the commit pipelines' block filler and shard
// writers), joined on every exit path, an exception included: declare it
// after everything the task refers to.  When no thread can be started the
// task runs inside start().  An exception thrown by the task is kept and
// rethrown by join().
class BgTask {
 public:
  BgTask() = default;
  BgTask(const BgTask &) = delete;
  BgTask &operator=(const BgTask &) = delete;
  ~BgTask() {
    if (t_.joinable()) t_.join();
  }
  template <class F>
  void start(F f) {
    join();
    auto body = [this, f] {
      try {
        f();
      } catch (...) {
        err_ = std::current_exception();
      }
    };
    try {
      t_ = std::thread(body);
    } catch (const std::system_error &) {
      body();
    }
  }
  void join() {
    if (t_.joinable()) t_.join();
    if (err_) {
      std::exception_ptr e = err_;
      err_ = nullptr;
      std::rethrow_exception(e);
    }
  }

 private:
  std::thread t_;
  std::exception_ptr err_;
};

bool mkdirs(const std::string &path);
bool rmtree(const std::string &path);
bool write_file(const std::string &path, const uint8_t *data, size_t n);
bool read_file(const std::string &path, std::vector<uint8_t> *out);
// Whole file into dst[0, cap).  Returns its size, or -1 if it is missing,
// unreadable or longer than cap.  threads > 1: parallel preads (>= 4 MiB each).
long long read_file_into(const std::string &path, uint8_t *dst, size_t cap, int threads = 1);

std::string t3_seg(const std::string &dir, size_t b, size_t s);
std::string t3_par(const std::string &dir, size_t b, size_t p);
std::string t2_seg(const std::string &dir, size_t i);
std::string t2_par(const std::string &dir, size_t i, size_t p);

// manifest.json + derived segment geometry of one archive directory.
struct Geometry {
  Manifest mf;
  std::string dir;
  uint64_t S = 0;   // segment size (tier 1: the file size)
  size_t nseg = 0;  // data segments in the file
  size_t seg_len(size_t g) const {
    const uint64_t size = uint64_t(mf.size);
    return g * S >= size ? 0 : size_t(size - g * S < S ? size - g * S : S);
  }
  // tier 3: segments in block b and its padded shard size (longest segment)
  size_t block_k(size_t b) const;
  size_t block_shard(size_t b) const { return seg_len(b * kBlockSegments); }
};
int load_geometry(const std::string &dir, Geometry *g);

}  // namespace bfrs
