// archive.cpp — BlockFrame's host pipeline around the RS codec, restated in
// C++ over the HIP path: commit (tiers 1-3), repair, and the read-path core
// that the FUSE mount uses.  On-disk layout and manifest are the reference's
// (SURVEY.md Appendix B):
//
//   {root}/{name}_{blake3}/manifest.json
//   tier 1: data.dat, parity_{0,1,2}.dat                          (commit.rs:25-118)
//   tier 2: segments/segment_{i}.dat, parity/segment_{i}_parity_{p}.dat (commit.rs:124-309)
//   tier 3: blocks/block_{b}/segments/segment_{s}.dat,
//           blocks/block_{b}/parity/block_parity_{p}.dat          (commit.rs:314-536)
//
// Repair and read follow the reference's *intended* semantics, not its bugs
// (SURVEY §0.5): every missing or corrupt (BLAKE3 mismatch) segment of a
// tier-3 block is restored with one RS(k,3) decode of that block and written
// back to its in-block index; reads map offsets with `%`, not `&`
// (filesystem_unix.rs:216), and tier-3 recovery decodes RS(30,3), not RS(1,3)
// (:112-113).
#include <dirent.h>
#include <fcntl.h>
#include <ftw.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstring>
#include <functional>
#include <list>
#include <memory>
#include <mutex>
#include <sstream>
#include <thread>
#include <unordered_map>

#include "blake3.hpp"
#include "manifest.hpp"
#include "runtime.hpp"

using namespace bfrs;

namespace {

constexpr uint64_t kTier1Limit = 25000000;    // commit.rs:596
constexpr uint64_t kTier2Limit = 1000000000;  // commit.rs:597
constexpr size_t kBlockSegments = 30;         // commit.rs:359,402
constexpr size_t kParity = 3;
constexpr size_t kDefaultSegment = 32u << 20;  // utils.rs:68 on any real host

int io_error(const std::string &what) {
  return set_error(BFRS_E_WRAPPER, what + ": " + std::strerror(errno));
}

int hw_threads() {
  const unsigned n = std::thread::hardware_concurrency();
  return int(std::max(1u, std::min(16u, n ? n : 4u)));
}

// Runs f(i) for i in [0, n) on up to `threads` threads.
void parallel_for(size_t n, int threads, const std::function<void(size_t)> &f) {
  if (n == 0) return;
  std::atomic<size_t> next{0};
  auto worker = [&] {
    for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
  };
  std::vector<std::thread> ts;
  const int t = int(std::min<size_t>(n, size_t(std::max(1, threads))));
  for (int k = 1; k < t; ++k) ts.emplace_back(worker);
  worker();
  for (auto &th : ts) th.join();
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

int rm_cb(const char *p, const struct stat *, int, struct FTW *) { return remove(p); }
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

// Whole file into `out`; false if absent/unreadable.
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

std::string basename_of(const std::string &p) {
  const size_t s = p.find_last_of('/');
  return s == std::string::npos ? p : p.substr(s + 1);
}

struct Mapped {
  int fd = -1;
  const uint8_t *p = nullptr;
  size_t n = 0;
  ~Mapped() {
    if (p && n) munmap(const_cast<uint8_t *>(p), n);
    if (fd >= 0) close(fd);
  }
};

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

// RS(k,3) encode of `blocks` (each a list of k host shards of shard_bytes) on the GPU.
int gpu_encode(bfrs_ctx *ctx, const std::vector<std::vector<const uint8_t *>> &blocks,
               size_t shard_bytes, std::vector<std::vector<std::vector<uint8_t>>> *parity) {
  std::vector<uint32_t> ks;
  std::vector<const uint8_t *> in;
  std::vector<uint8_t *> out;
  parity->assign(blocks.size(), {});
  for (size_t b = 0; b < blocks.size(); ++b) {
    ks.push_back(uint32_t(blocks[b].size()));
    in.insert(in.end(), blocks[b].begin(), blocks[b].end());
    (*parity)[b].assign(kParity, std::vector<uint8_t>(shard_bytes));
    for (auto &p : (*parity)[b]) out.push_back(p.data());
  }
  return bfrs_encode_host_batch(ctx, blocks.size(), ks.data(), kParity, shard_bytes, in.data(),
                                out.data());
}

struct Commit {
  bfrs_ctx *ctx;
  std::string root, name, path;
  size_t S;
  Mapped m;
  int threads = hw_threads();

  int tier1(std::string *out_dir);
  int tier2(std::string *out_dir);
  int tier3(std::string *out_dir);
  int finish(const std::string &computing, const std::string &file_hash, Manifest &mf,
             std::string *out_dir);
};

int Commit::finish(const std::string &computing, const std::string &file_hash, Manifest &mf,
                   std::string *out_dir) {
  const std::string final_dir = root + "/" + name + "_" + file_hash;
  if (computing != final_dir) {
    struct stat st;
    if (stat(final_dir.c_str(), &st) == 0 && !rmtree(final_dir))  // duplicate commit overwrites
      return io_error("remove existing " + final_dir);
    if (rename(computing.c_str(), final_dir.c_str()) != 0) return io_error("rename " + computing);
  }
  mf.original_hash = file_hash;
  mf.name = name;
  mf.size = int64_t(m.n);
  mf.time_of_creation = utc_now_string();
  const std::string js = mf.to_json();
  if (!write_file(final_dir + "/manifest.json", reinterpret_cast<const uint8_t *>(js.data()),
                  js.size()))
    return io_error("write manifest");
  *out_dir = final_dir;
  return BFRS_OK;
}

// commit_tiny (commit.rs:25-118): RS(1,3) of the 64-padded file.
int Commit::tier1(std::string *out_dir) {
  const size_t padded = (m.n + 63) / 64 * 64;
  std::vector<uint8_t> buf(padded, 0);
  std::memcpy(buf.data(), m.p, m.n);
  std::vector<std::vector<std::vector<uint8_t>>> par;
  int rc = gpu_encode(ctx, {{buf.data()}}, padded, &par);
  if (rc) return rc;
  const std::string file_hash = blake3_hex(m.p, m.n, threads);
  const std::string dir = root + "/" + name + "_" + file_hash;
  if (!mkdirs(dir)) return io_error("mkdir " + dir);
  if (!write_file(dir + "/data.dat", m.p, m.n)) return io_error("write data.dat");
  Manifest mf;
  mf.tier = 1;
  mf.data_shards = 6;  // commit.rs:98 (sic)
  mf.parity_shards = 3;
  mf.segment_size = padded;
  std::vector<std::string> leaves{file_hash};
  for (size_t p = 0; p < kParity; ++p) {
    if (!write_file(dir + "/parity_" + std::to_string(p) + ".dat", par[0][p].data(), padded))
      return io_error("write parity");
    leaves.push_back(blake3_hex(par[0][p].data(), padded));
  }
  for (size_t i = 0; i < leaves.size(); ++i) mf.leaves[int64_t(i)] = leaves[i];
  mf.root = merkle_root_hex(leaves);
  return finish(dir, file_hash, mf, out_dir);
}

// commit_segmented (commit.rs:124-309): per-segment RS(1,3).
int Commit::tier2(std::string *out_dir) {
  const std::string dir = root + "/" + name + "_computing";
  if (!mkdirs(dir + "/segments") || !mkdirs(dir + "/parity")) return io_error("mkdir " + dir);
  const size_t nseg = (m.n + S - 1) / S;
  Manifest mf;
  mf.tier = 2;
  mf.data_shards = 6;  // commit.rs:294 (sic)
  mf.parity_shards = 3;
  mf.segment_size = S;
  std::vector<std::string> seg_roots(nseg);
  // full segments in one GPU batch, the (padded) tail segment on its own
  const size_t full = m.n / S;
  for (size_t first = 0; first < nseg;) {
    const size_t len = std::min(S, m.n - first * S);
    const size_t padded = (len + 63) / 64 * 64;
    const size_t count = len == S ? std::min<size_t>(full - first, 64) : 1;
    std::vector<std::vector<uint8_t>> pads;
    std::vector<std::vector<const uint8_t *>> blocks;
    for (size_t i = 0; i < count; ++i) {
      const uint8_t *src = m.p + (first + i) * S;
      if (padded != len) {
        pads.emplace_back(padded, 0);
        std::memcpy(pads.back().data(), src, len);
        src = pads.back().data();
      }
      blocks.push_back({src});
    }
    std::vector<std::vector<std::vector<uint8_t>>> par;
    int rc = gpu_encode(ctx, blocks, padded, &par);
    if (rc) return rc;
    std::vector<SegmentHashes> hs(count);
    std::atomic<bool> ok{true};
    parallel_for(count * 4, threads, [&](size_t t) {
      const size_t i = t / 4, what = t % 4;
      const size_t seg = first + i;
      if (what == 0) {
        const uint8_t *src = m.p + seg * S;
        if (!write_file(t2_seg(dir, seg), src, len)) ok = false;
        hs[i].data = blake3_hex(src, len);
      } else {
        const auto &p = par[i][what - 1];
        if (!write_file(t2_par(dir, seg, what - 1), p.data(), p.size())) ok = false;
      }
    });
    if (!ok) return io_error("write tier-2 shards");
    for (size_t i = 0; i < count; ++i) {
      for (size_t p = 0; p < kParity; ++p)
        hs[i].parity.push_back(blake3_hex(par[i][p].data(), par[i][p].size()));
      std::vector<std::string> leaves{hs[i].data};
      leaves.insert(leaves.end(), hs[i].parity.begin(), hs[i].parity.end());
      seg_roots[first + i] = merkle_root_hex(leaves);
      mf.segments[int64_t(first + i)] = hs[i];
    }
    first += count;
  }
  mf.root = merkle_root_hex(seg_roots);
  return finish(dir, blake3_hex(m.p, m.n, threads), mf, out_dir);
}

// commit_blocked (commit.rs:314-536): blocks of <= 30 segments, RS(k,3) each,
// block Merkle over segment+parity hashes, root over block roots.
int Commit::tier3(std::string *out_dir) {
  const std::string dir = root + "/" + name + "_computing";
  const size_t nseg = (m.n + S - 1) / S;
  const size_t nblocks = (nseg + kBlockSegments - 1) / kBlockSegments;
  for (size_t b = 0; b < nblocks; ++b)
    if (!mkdirs(dir + "/blocks/block_" + std::to_string(b) + "/segments") ||
        !mkdirs(dir + "/blocks/block_" + std::to_string(b) + "/parity"))
      return io_error("mkdir " + dir);
  Manifest mf;
  mf.tier = 3;
  mf.data_shards = 30;
  mf.parity_shards = 3;
  mf.segment_size = S;
  std::vector<std::string> block_roots(nblocks);
  // GPU batches of up to 8 full blocks (bounded host parity memory).
  for (size_t b0 = 0; b0 < nblocks;) {
    std::vector<std::vector<const uint8_t *>> blocks;
    std::vector<uint8_t> tail_pad;
    size_t shard_bytes = 0;
    size_t b1 = b0;
    for (; b1 < nblocks && b1 - b0 < 8; ++b1) {
      const size_t s0 = b1 * kBlockSegments, s1 = std::min(nseg, s0 + kBlockSegments);
      const size_t blk_max = std::min(S, m.n - s0 * S);  // first segment is the longest
      if (b1 > b0 && blk_max != shard_bytes) break;      // one shard size per batch
      shard_bytes = blk_max;
      std::vector<const uint8_t *> segs;
      for (size_t s = s0; s < s1; ++s) {
        const size_t len = std::min(S, m.n - s * S);
        if (len < shard_bytes) {  // generate.rs:75-82: zero-pad to the block's max length
          tail_pad.assign(shard_bytes, 0);
          std::memcpy(tail_pad.data(), m.p + s * S, len);
          segs.push_back(tail_pad.data());
        } else {
          segs.push_back(m.p + s * S);
        }
      }
      blocks.push_back(segs);
    }
    std::vector<std::vector<std::vector<uint8_t>>> par;
    int rc = gpu_encode(ctx, blocks, shard_bytes, &par);
    if (rc) return rc;
    // segment + parity files and hashes, in parallel
    for (size_t b = b0; b < b1; ++b) {
      const size_t s0 = b * kBlockSegments, s1 = std::min(nseg, s0 + kBlockSegments);
      BlockHashes bh;
      bh.segments.resize(s1 - s0);
      bh.parity.resize(kParity);
      std::atomic<bool> ok{true};
      const auto &bp = par[b - b0];
      parallel_for((s1 - s0) + kParity, threads, [&](size_t t) {
        if (t < s1 - s0) {
          const size_t s = s0 + t, len = std::min(S, m.n - s * S);
          if (!write_file(t3_seg(dir, b, t), m.p + s * S, len)) ok = false;
          bh.segments[t] = blake3_hex(m.p + s * S, len);
        } else {
          const size_t p = t - (s1 - s0);
          if (!write_file(t3_par(dir, b, p), bp[p].data(), bp[p].size())) ok = false;
          bh.parity[p] = blake3_hex(bp[p].data(), bp[p].size());
        }
      });
      if (!ok) return io_error("write tier-3 shards");
      std::vector<std::string> leaves = bh.segments;
      leaves.insert(leaves.end(), bh.parity.begin(), bh.parity.end());
      block_roots[b] = merkle_root_hex(leaves);
      mf.blocks[int64_t(b)] = bh;
    }
    b0 = b1;
  }
  mf.root = merkle_root_hex(block_roots);
  return finish(dir, blake3_hex(m.p, m.n, threads), mf, out_dir);
}

// ---------------------------------------------------------------------------
// Archive geometry shared by repair and read.
struct Geometry {
  Manifest mf;
  std::string dir;
  uint64_t S = 0;
  size_t nseg = 0;
  size_t seg_len(size_t g) const { return size_t(std::min<uint64_t>(S, uint64_t(mf.size) - g * S)); }
};

int load_geometry(const std::string &dir, Geometry *g) {
  std::vector<uint8_t> text;
  if (!read_file(dir + "/manifest.json", &text)) return io_error("read manifest " + dir);
  std::string err;
  if (!Manifest::from_json(std::string(text.begin(), text.end()), &g->mf, &err))
    return set_error(BFRS_E_WRAPPER, err);
  g->dir = dir;
  g->S = g->mf.tier == 1 ? uint64_t(std::max<int64_t>(g->mf.size, 1)) : g->mf.segment_size;
  if (g->S == 0) return set_error(BFRS_E_WRAPPER, "manifest: segment_size is 0");
  g->nseg = g->mf.tier == 1 ? 1 : size_t((uint64_t(g->mf.size) + g->S - 1) / g->S);
  return BFRS_OK;
}

// Verified bytes of one stored shard (false = missing or hash mismatch).
// threads > 1 splits the hash over chunk subtrees (callers already running in
// a parallel_for pass 1).
bool load_verified(const std::string &path, const std::string &want_hex, std::vector<uint8_t> *out,
                   int threads = 1) {
  if (!read_file(path, out)) return false;
  return blake3_hex(out->data(), out->size(), threads) == want_hex;
}

// Tier-3 block recovery: restores every missing/corrupt segment of block b.
// present[s]/data[s] in, restored data out (unpadded lengths).  Returns the
// number of restored segments, or <0 (error) / BFRS_E_NOT_ENOUGH_SHARDS.
int recover_block(bfrs_ctx *ctx, const Geometry &g, size_t b,
                  std::vector<std::vector<uint8_t>> &data, std::vector<uint8_t> &ok,
                  int *parity_bad) {
  const BlockHashes &bh = g.mf.blocks.at(int64_t(b));
  const size_t k = bh.segments.size();
  const size_t g0 = b * kBlockSegments;
  const size_t shard = g.seg_len(g0);  // the block's longest segment = padded shard size
  std::vector<std::vector<uint8_t>> par(kParity);
  std::vector<uint8_t> par_ok(kParity, 0);
  int nbad = 0;
  parallel_for(std::min(kParity, bh.parity.size()), int(kParity), [&](size_t p) {
    par_ok[p] = load_verified(t3_par(g.dir, b, p), bh.parity[p], &par[p], hw_threads() / 3) &&
                par[p].size() == shard;
  });
  for (size_t p = 0; p < kParity; ++p) nbad += !par_ok[p];
  if (parity_bad) *parity_bad = nbad;
  size_t erased = 0;
  for (size_t s = 0; s < k; ++s) erased += !ok[s];
  if (erased == 0) return 0;
  size_t present = 0;
  for (uint8_t v : par_ok) present += v;
  if (erased > present) {
    std::ostringstream os;
    os << "block " << b << ": " << erased << " damaged segments but only " << present
       << " valid parity shards - unrecoverable";
    return set_error(BFRS_E_NOT_ENOUGH_SHARDS, os.str());
  }
  std::vector<std::vector<uint8_t>> padded(k);
  std::vector<const uint8_t *> orig(k, nullptr), rec(kParity, nullptr);
  std::vector<uint8_t *> out(k, nullptr);
  for (size_t s = 0; s < k; ++s) {
    if (ok[s]) {
      if (data[s].size() < shard) {
        padded[s].assign(shard, 0);
        std::memcpy(padded[s].data(), data[s].data(), data[s].size());
        orig[s] = padded[s].data();
      } else {
        orig[s] = data[s].data();
      }
    } else {
      padded[s].assign(shard, 0);
      out[s] = padded[s].data();
    }
  }
  for (size_t p = 0; p < kParity; ++p)
    if (par_ok[p]) rec[p] = par[p].data();
  const uint32_t kk = uint32_t(k);
  int rc = bfrs_decode_host_batch(ctx, 1, &kk, kParity, shard, orig.data(), rec.data(), out.data());
  if (rc) return rc;
  std::vector<size_t> todo;
  for (size_t s = 0; s < k; ++s)
    if (!ok[s]) todo.push_back(s);
  std::vector<uint8_t> good(todo.size(), 0);
  parallel_for(todo.size(), int(todo.size()), [&](size_t i) {
    const size_t s = todo[i], len = g.seg_len(g0 + s);
    padded[s].resize(len);
    data[s] = std::move(padded[s]);
    // src/merkle_tree re-verify of the reconstructed bytes
    good[i] = blake3_hex(data[s].data(), len, hw_threads() / int(todo.size())) == bh.segments[s];
  });
  for (size_t i = 0; i < todo.size(); ++i) {
    if (!good[i]) {
      std::ostringstream os;
      os << "block " << b << " segment " << todo[i] << ": restored bytes fail the manifest hash";
      return set_error(BFRS_E_WRAPPER, os.str());
    }
    ok[todo[i]] = 1;
  }
  return int(todo.size());
}

// RS(1,3) recovery (tiers 1/2): decode from the valid parity shards.
int recover_rs13(bfrs_ctx *ctx, const std::vector<std::string> &paths,
                 const std::vector<std::string> &hashes, size_t expected, const std::string &want,
                 std::vector<uint8_t> *out) {
  std::vector<std::vector<uint8_t>> par(kParity);
  std::vector<const uint8_t *> rec(kParity, nullptr);
  size_t shard = 0;
  for (size_t p = 0; p < kParity; ++p)
    if (load_verified(paths[p], hashes[p], &par[p])) {
      rec[p] = par[p].data();
      shard = par[p].size();
    }
  if (!shard) return set_error(BFRS_E_NOT_ENOUGH_SHARDS, "no valid parity shard");
  std::vector<uint8_t> restored(shard);
  const uint8_t *orig[1] = {nullptr};
  uint8_t *outp[1] = {restored.data()};
  const uint32_t k1 = 1;
  int rc = bfrs_decode_host_batch(ctx, 1, &k1, kParity, shard, orig, rec.data(), outp);
  if (rc) return rc;
  restored.resize(std::min(expected, shard));
  if (blake3_hex(restored.data(), restored.size()) != want)
    return set_error(BFRS_E_WRAPPER, "restored bytes fail the manifest hash");
  *out = std::move(restored);
  return BFRS_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// Archive read handle (src/mount/filesystem_unix.rs:176-305 + cache.rs)
struct bfrs_archive {
  bfrs_ctx *ctx;
  Geometry g;
  size_t cap;
  bool write_back;
  std::mutex mu;
  std::list<size_t> lru;
  std::unordered_map<size_t, std::pair<std::shared_ptr<std::vector<uint8_t>>,
                                       std::list<size_t>::iterator>>
      cache;
  bfrs_archive_stats st{};

  void put(size_t g_idx, std::shared_ptr<std::vector<uint8_t>> v) {
    auto it = cache.find(g_idx);
    if (it != cache.end()) {
      lru.erase(it->second.second);
      cache.erase(it);
    }
    lru.push_front(g_idx);
    cache[g_idx] = {std::move(v), lru.begin()};
    while (cache.size() > cap) {
      cache.erase(lru.back());
      lru.pop_back();
    }
  }
  int segment(size_t gi, std::shared_ptr<std::vector<uint8_t>> *out);
};

int bfrs_archive::segment(size_t gi, std::shared_ptr<std::vector<uint8_t>> *out) {
  auto it = cache.find(gi);
  if (it != cache.end()) {
    lru.splice(lru.begin(), lru, it->second.second);
    ++st.hits;
    *out = it->second.first;
    return BFRS_OK;
  }
  ++st.misses;
  const Manifest &mf = g.mf;
  auto v = std::make_shared<std::vector<uint8_t>>();
  if (mf.tier == 3) {
    const size_t b = gi / kBlockSegments, s = gi % kBlockSegments;
    auto bit = mf.blocks.find(int64_t(b));
    if (bit == mf.blocks.end() || s >= bit->second.segments.size())
      return set_error(BFRS_E_WRAPPER, "manifest has no hash for segment " + std::to_string(gi));
    if (load_verified(t3_seg(g.dir, b, s), bit->second.segments[s], v.get(), hw_threads())) {
      ++st.verified;
      put(gi, v);
      *out = v;
      return BFRS_OK;
    }
    // hash mismatch or missing: restore the whole block in one GPU decode
    const size_t k = bit->second.segments.size();
    std::vector<std::vector<uint8_t>> data(k);
    std::vector<uint8_t> ok(k, 0);
    parallel_for(k, hw_threads(), [&](size_t t) {
      auto c = cache.find(b * kBlockSegments + t);  // read-only lookups under a.mu
      if (c != cache.end()) {
        data[t] = *c->second.first;
        ok[t] = 1;
      } else if (t != s) {
        ok[t] = load_verified(t3_seg(g.dir, b, t), bit->second.segments[t], &data[t]);
      }
    });
    std::vector<uint8_t> was_ok = ok;
    int rc = recover_block(ctx, g, b, data, ok, nullptr);
    if (rc < 0) return rc;
    ++st.recoveries;
    for (size_t t = 0; t < k; ++t) {
      if (was_ok[t]) continue;
      ++st.recovered_segments;
      if (write_back && !write_file(t3_seg(g.dir, b, t), data[t].data(), data[t].size()))
        return io_error("write back segment");
      if (t != s) put(b * kBlockSegments + t, std::make_shared<std::vector<uint8_t>>(data[t]));
    }
    *v = std::move(data[s]);
  } else if (mf.tier == 2) {
    auto sit = mf.segments.find(int64_t(gi));
    if (sit == mf.segments.end()) return set_error(BFRS_E_WRAPPER, "manifest has no segment");
    if (load_verified(t2_seg(g.dir, gi), sit->second.data, v.get(), hw_threads())) {
      ++st.verified;
    } else {
      std::vector<std::string> paths;
      for (size_t p = 0; p < kParity; ++p) paths.push_back(t2_par(g.dir, gi, p));
      int rc = recover_rs13(ctx, paths, sit->second.parity, g.seg_len(gi), sit->second.data, v.get());
      if (rc) return rc;
      ++st.recoveries;
      ++st.recovered_segments;
      if (write_back && !write_file(t2_seg(g.dir, gi), v->data(), v->size()))
        return io_error("write back segment");
    }
  } else {
    if (mf.leaves.size() < 4) return set_error(BFRS_E_WRAPPER, "tier-1 manifest needs 4 leaves");
    if (load_verified(g.dir + "/data.dat", mf.leaves.at(0), v.get(), hw_threads())) {
      ++st.verified;
    } else {
      std::vector<std::string> paths, hashes;
      for (size_t p = 0; p < kParity; ++p) {
        paths.push_back(g.dir + "/parity_" + std::to_string(p) + ".dat");
        hashes.push_back(mf.leaves.at(int64_t(p + 1)));
      }
      int rc = recover_rs13(ctx, paths, hashes, size_t(mf.size), mf.leaves.at(0), v.get());
      if (rc) return rc;
      ++st.recoveries;
      ++st.recovered_segments;
      if (write_back && !write_file(g.dir + "/data.dat", v->data(), v->size()))
        return io_error("write back data.dat");
    }
  }
  put(gi, v);
  *out = v;
  return BFRS_OK;
}

extern "C" {

int bfrs_blake3_hex(const uint8_t *data, size_t len, int threads, char *out65) {
  if ((!data && len) || !out65) return set_error(BFRS_E_INVALID_ARGUMENT, "blake3: NULL argument");
  const std::string h = blake3_hex(data, len, threads);
  std::memcpy(out65, h.c_str(), 65);
  return BFRS_OK;
}

int bfrs_merkle_root_hex(const char *leaves, size_t n, char *out65) {
  if (!leaves || !out65 || n == 0) return set_error(BFRS_E_INVALID_ARGUMENT, "merkle: bad argument");
  std::vector<std::string> v;
  for (size_t i = 0; i < n; ++i) v.emplace_back(leaves + 64 * i, 64);
  const std::string r = merkle_root_hex(v);
  std::memcpy(out65, r.c_str(), 65);
  return BFRS_OK;
}

int bfrs_manifest_check(const char *text, size_t len, int *valid, char *canonical, size_t cap,
                        size_t *needed) {
  if (!text || !valid) return set_error(BFRS_E_INVALID_ARGUMENT, "manifest_check: NULL argument");
  Manifest mf;
  std::string err;
  if (!Manifest::from_json(std::string(text, len), &mf, &err)) return set_error(BFRS_E_WRAPPER, err);
  auto hex64 = [](const std::string &h) {
    return h.size() == 64 && std::all_of(h.begin(), h.end(), [](char c) { return std::isxdigit(uint8_t(c)); });
  };
  // ManifestFile::validate (src/merkle_tree/manifest.rs:55-88)
  bool ok = hex64(mf.root) && !(mf.leaves.empty() && mf.segments.empty() && mf.blocks.empty());
  int64_t expect = 0;
  for (const auto &kv : mf.leaves) ok = ok && hex64(kv.second) && kv.first == expect++;
  *valid = ok ? 1 : 0;
  const std::string js = mf.to_json();
  if (needed) *needed = js.size() + 1;
  if (canonical && cap) {
    const size_t n = std::min(cap - 1, js.size());
    std::memcpy(canonical, js.data(), n);
    canonical[n] = 0;
  }
  return BFRS_OK;
}

int bfrs_commit(bfrs_ctx *ctx, const char *file_path, const char *archive_root,
                size_t segment_size, int tier, char *out_dir, size_t out_cap) {
  if (!ctx || !file_path || !archive_root)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_commit: NULL argument");
  Commit c{ctx, archive_root, basename_of(file_path), file_path,
           segment_size ? segment_size : kDefaultSegment};
  c.m.fd = open(file_path, O_RDONLY);
  if (c.m.fd < 0) return io_error(std::string("open ") + file_path);
  struct stat st;
  if (fstat(c.m.fd, &st) != 0) return io_error("stat");
  c.m.n = size_t(st.st_size);
  if (c.m.n == 0) return set_error(BFRS_E_WRAPPER, "empty file");  // commit.rs:599
  void *p = mmap(nullptr, c.m.n, PROT_READ, MAP_PRIVATE, c.m.fd, 0);
  if (p == MAP_FAILED) return io_error("mmap");
  c.m.p = static_cast<const uint8_t *>(p);
  if (!mkdirs(c.root)) return io_error("mkdir " + c.root);
  if (tier < 0 || tier > 3) return set_error(BFRS_E_INVALID_ARGUMENT, "tier must be 0..3");
  if (tier == 0) tier = c.m.n <= kTier1Limit ? 1 : c.m.n <= kTier2Limit ? 2 : 3;
  std::string dir;
  int rc = tier == 1 ? c.tier1(&dir) : tier == 2 ? c.tier2(&dir) : c.tier3(&dir);
  if (rc) return rc;
  if (out_dir && out_cap) {
    std::strncpy(out_dir, dir.c_str(), out_cap - 1);
    out_dir[out_cap - 1] = 0;
  }
  return BFRS_OK;
}

int bfrs_repair(bfrs_ctx *ctx, const char *archive_dir, bfrs_repair_report *report) {
  if (!ctx || !archive_dir || !report)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_repair: NULL argument");
  *report = bfrs_repair_report{};
  Geometry g;
  int rc = load_geometry(archive_dir, &g);
  if (rc) return rc;
  const Manifest &mf = g.mf;
  if (mf.tier == 3) {
    for (const auto &kv : mf.blocks) {
      const size_t b = size_t(kv.first), k = kv.second.segments.size();
      ++report->blocks_checked;
      std::vector<std::vector<uint8_t>> data(k);
      std::vector<uint8_t> ok(k, 0);
      parallel_for(k, hw_threads(), [&](size_t s) {
        ok[s] = load_verified(t3_seg(g.dir, b, s), kv.second.segments[s], &data[s]);
      });
      report->segments_checked += k;
      std::vector<uint8_t> was_ok = ok;
      int parity_bad = 0;
      const int restored = recover_block(ctx, g, b, data, ok, &parity_bad);
      if (restored < 0) {
        if (restored != BFRS_E_NOT_ENOUGH_SHARDS) return restored;
        ++report->unrecoverable_blocks;
        continue;
      }
      for (size_t s = 0; s < k; ++s)
        if (!was_ok[s]) {
          if (!write_file(t3_seg(g.dir, b, s), data[s].data(), data[s].size()))
            return io_error("write restored segment");
          ++report->segments_repaired;
        }
      if (parity_bad) {  // data is whole now: re-encode and rewrite the parity
        const size_t shard = g.seg_len(b * kBlockSegments);
        std::vector<std::vector<uint8_t>> padded(k);
        std::vector<const uint8_t *> segs(k);
        for (size_t s = 0; s < k; ++s) {
          if (data[s].size() < shard) {
            padded[s].assign(shard, 0);
            std::memcpy(padded[s].data(), data[s].data(), data[s].size());
            segs[s] = padded[s].data();
          } else {
            segs[s] = data[s].data();
          }
        }
        std::vector<std::vector<std::vector<uint8_t>>> par;
        if ((rc = gpu_encode(ctx, {segs}, shard, &par))) return rc;
        for (size_t p = 0; p < kParity; ++p) {
          if (blake3_hex(par[0][p].data(), shard) != kv.second.parity[p])
            return set_error(BFRS_E_WRAPPER, "re-encoded parity fails the manifest hash");
          if (!write_file(t3_par(g.dir, b, p), par[0][p].data(), shard))
            return io_error("write parity");
        }
        report->parity_repaired += uint64_t(parity_bad);
      }
    }
    return BFRS_OK;
  }
  // tiers 1/2: per-segment RS(1,3)
  bfrs_archive a{ctx, g, 1, true};
  for (size_t i = 0; i < g.nseg; ++i) {
    std::shared_ptr<std::vector<uint8_t>> v;
    ++report->segments_checked;
    const uint64_t before = a.st.recovered_segments;
    rc = a.segment(i, &v);
    if (rc == BFRS_E_NOT_ENOUGH_SHARDS) {
      ++report->unrecoverable_blocks;
      continue;
    }
    if (rc) return rc;
    report->segments_repaired += a.st.recovered_segments - before;
  }
  report->blocks_checked = g.nseg;
  return BFRS_OK;
}

int bfrs_archive_open(bfrs_ctx *ctx, const char *archive_dir, size_t cache_segments,
                      int write_back, bfrs_archive **out) {
  if (!ctx || !archive_dir || !out)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_archive_open: NULL argument");
  *out = nullptr;
  auto *a = new (std::nothrow) bfrs_archive{ctx, {}, std::max<size_t>(1, cache_segments),
                                            write_back != 0};
  if (!a) return set_error(BFRS_E_NOMEM, "archive allocation failed");
  int rc = load_geometry(archive_dir, &a->g);
  if (rc) {
    delete a;
    return rc;
  }
  *out = a;
  return BFRS_OK;
}

int bfrs_archive_size(bfrs_archive *a, uint64_t *size) {
  if (!a || !size) return set_error(BFRS_E_INVALID_ARGUMENT, "NULL argument");
  *size = uint64_t(a->g.mf.size);
  return BFRS_OK;
}

int bfrs_archive_read(bfrs_archive *a, uint64_t offset, size_t len, uint8_t *out, size_t *nread) {
  if (!a || (!out && len) || !nread) return set_error(BFRS_E_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> g(a->mu);
  *nread = 0;
  const uint64_t size = uint64_t(a->g.mf.size);
  if (offset >= size) return BFRS_OK;
  len = size_t(std::min<uint64_t>(len, size - offset));
  const uint64_t S = a->g.S;
  while (*nread < len) {
    const uint64_t pos = offset + *nread;
    const size_t gi = size_t(pos / S);
    const size_t in_seg = size_t(pos % S);  // filesystem_unix.rs:216 uses '&' (bug)
    std::shared_ptr<std::vector<uint8_t>> seg;
    int rc = a->segment(gi, &seg);
    if (rc) return rc;
    if (in_seg >= seg->size()) return set_error(BFRS_E_WRAPPER, "segment shorter than manifest size");
    const size_t n = std::min(len - *nread, seg->size() - in_seg);
    std::memcpy(out + *nread, seg->data() + in_seg, n);
    *nread += n;
  }
  a->st.bytes_served += *nread;
  return BFRS_OK;
}

int bfrs_archive_stats_get(bfrs_archive *a, bfrs_archive_stats *out) {
  if (!a || !out) return set_error(BFRS_E_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> g(a->mu);
  *out = a->st;
  return BFRS_OK;
}

void bfrs_archive_close(bfrs_archive *a) { delete a; }

}  // extern "C"
