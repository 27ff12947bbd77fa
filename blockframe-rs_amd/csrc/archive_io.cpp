// archive_io.cpp — see archive_io.hpp.
#include "archive_io.hpp"

#include <fcntl.h>
#include <ftw.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstring>
#include <sstream>
#include <thread>

#include <mutex>

#include "runtime.hpp"

namespace bfrs {

int io_error(const std::string &what) {
  return set_error(BFRS_E_WRAPPER, what + ": " + std::strerror(errno));
}

int hw_threads() {
  const unsigned n = std::thread::hardware_concurrency();
  return int(std::max(1u, std::min(16u, n ? n : 4u)));
}

void parallel_for(size_t n, int threads, const std::function<void(size_t)> &f) {
  if (n == 0) return;
  std::atomic<size_t> next{0};
  std::mutex err_mu;
  std::exception_ptr err;
  auto worker = [&] {
    try {
      for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    } catch (...) {
      next = n;  // the other workers stop after their current item
      std::lock_guard<std::mutex> g(err_mu);
      if (!err) err = std::current_exception();
    }
  };
  std::vector<std::thread> ts;
  const int t = int(std::min<size_t>(n, size_t(std::max(1, threads))));
  try {
    ts.reserve(size_t(t));
    for (int k = 1; k < t; ++k) ts.emplace_back(worker);
  } catch (...) {  // no more threads (quota, memory): the started ones and this one do it all
  }
  worker();
  for (auto &th : ts) th.join();
  if (err) std::rethrow_exception(err);
}

bool mkdirs(const std::string &path) {
  std::string cur;
  std::stringstream ss(path);
  std::string part;
  if (!path.empty() && path[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
  }
  return true;
}

namespace {
int rm_cb(const char *p, const struct stat *, int, struct FTW *) { return remove(p); }
}  // namespace

bool rmtree(const std::string &p) { return nftw(p.c_str(), rm_cb, 32, FTW_DEPTH | FTW_PHYS) == 0; }

bool write_file(const std::string &path, const uint8_t *data, size_t n) {
  const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return false;
  size_t done = 0;
  while (done < n) {
    const ssize_t w = write(fd, data + done, n - done);
    if (w <= 0) {
      close(fd);
      return false;
    }
    done += size_t(w);
  }
  return close(fd) == 0;
}

bool read_file(const std::string &path, std::vector<uint8_t> *out) {
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return false;
  }
  out->resize(size_t(st.st_size));
  size_t done = 0;
  while (done < out->size()) {
    const ssize_t r = read(fd, out->data() + done, out->size() - done);
    if (r <= 0) {
      close(fd);
      return false;
    }
    done += size_t(r);
  }
  close(fd);
  return true;
}

long long read_file_into(const std::string &path, uint8_t *dst, size_t cap, int threads) {
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) return -1;
  struct stat st;
  if (fstat(fd, &st) != 0 || size_t(st.st_size) > cap) {
    close(fd);
    return -1;
  }
  const size_t n = size_t(st.st_size);
  // large files: parallel preads of >= 4 MiB pieces (page-cache copies are
  // per-thread bandwidth bound)
  const size_t pieces = threads > 1 ? std::min<size_t>(size_t(threads), n >> 22) : 1;
  std::atomic<bool> ok{true};
  auto piece = [&](size_t i) {
    const size_t lo = n * i / std::max<size_t>(pieces, 1), hi = n * (i + 1) / std::max<size_t>(pieces, 1);
    size_t done = lo;
    while (done < hi) {
      const ssize_t r = pread(fd, dst + done, hi - done, off_t(done));
      if (r <= 0) {
        ok = false;
        return;
      }
      done += size_t(r);
    }
  };
  if (pieces <= 1)
    piece(0);
  else
    parallel_for(pieces, int(pieces), piece);
  close(fd);
  return ok ? (long long)n : -1;
}

std::string t3_seg(const std::string &dir, size_t b, size_t s) {
  return dir + "/blocks/block_" + std::to_string(b) + "/segments/segment_" + std::to_string(s) +
         ".dat";
}
std::string t3_par(const std::string &dir, size_t b, size_t p) {
  return dir + "/blocks/block_" + std::to_string(b) + "/parity/block_parity_" + std::to_string(p) +
         ".dat";
}
std::string t2_seg(const std::string &dir, size_t i) {
  return dir + "/segments/segment_" + std::to_string(i) + ".dat";
}
std::string t2_par(const std::string &dir, size_t i, size_t p) {
  return dir + "/parity/segment_" + std::to_string(i) + "_parity_" + std::to_string(p) + ".dat";
}

size_t Geometry::block_k(size_t b) const {
  auto it = mf.blocks.find(int64_t(b));
  return it == mf.blocks.end() ? 0 : it->second.segments.size();
}

int load_geometry(const std::string &dir, Geometry *g) {
  std::vector<uint8_t> text;
  if (!read_file(dir + "/manifest.json", &text)) return io_error("read manifest " + dir);
  std::string err;
  if (!Manifest::from_json(std::string(text.begin(), text.end()), &g->mf, &err))
    return set_error(BFRS_E_WRAPPER, err);
  g->dir = dir;
  // Bounds before any arithmetic: a manifest is read from disk and may be
  // damaged or hostile (tests/malformed_manifests).  The reference's serde
  // types are i32 tier / usize sizes (manifest.rs:12-53); these limits only
  // refuse shapes no commit writes.
  const Manifest &mf = g->mf;
  if (mf.tier < 1 || mf.tier > 3) return set_error(BFRS_E_WRAPPER, "manifest: tier must be 1, 2 or 3");
  if (mf.size < 0) return set_error(BFRS_E_WRAPPER, "manifest: negative size");
  if (uint64_t(mf.size) > kMaxFileBytes) return set_error(BFRS_E_WRAPPER, "manifest: size too large");
  if (mf.tier != 1 && (mf.segment_size == 0 || mf.segment_size > kMaxSegmentBytes))
    return set_error(BFRS_E_WRAPPER, mf.segment_size == 0 ? "manifest: segment_size is 0"
                                                          : "manifest: segment_size too large");
  g->S = mf.tier == 1 ? uint64_t(std::max<int64_t>(mf.size, 1)) : mf.segment_size;
  g->nseg = mf.tier == 1 ? 1 : size_t((uint64_t(mf.size) + g->S - 1) / g->S);
  if (mf.tier == 2) {  // one entry per segment, keys 0..n-1 (commit.rs:124-309)
    if (mf.segments.size() != g->nseg) return set_error(BFRS_E_WRAPPER, "manifest: segment count");
    for (size_t i = 0; i < g->nseg; ++i) {
      auto it = mf.segments.find(int64_t(i));
      if (it == mf.segments.end() || it->second.parity.size() != kParity)
        return set_error(BFRS_E_WRAPPER, "manifest: segment " + std::to_string(i) + " shape");
    }
  }
  if (mf.tier == 3) {  // blocks must cover the segments in order (commit.rs:359-402)
    const size_t nblocks = (g->nseg + kBlockSegments - 1) / kBlockSegments;
    if (mf.blocks.size() != nblocks) return set_error(BFRS_E_WRAPPER, "manifest: block count");
    for (size_t b = 0; b < nblocks; ++b) {
      auto it = mf.blocks.find(int64_t(b));
      const size_t want = std::min(kBlockSegments, g->nseg - b * kBlockSegments);
      if (it == mf.blocks.end() || it->second.segments.size() != want ||
          it->second.parity.size() != kParity)
        return set_error(BFRS_E_WRAPPER, "manifest: block " + std::to_string(b) + " shape");
    }
  }
  return BFRS_OK;
}

}  // namespace bfrs
