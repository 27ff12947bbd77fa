// archive.cpp — BlockFrame's host pipeline around the RS codec: commit
// (tiers 1-3), repair, and the read-path core of the FUSE mount, with the RS
// arithmetic and (tier 3) the BLAKE3 verification on the GPU.  Layout and
// manifest: archive_io.hpp.
//
// Repair and read follow the reference's *intended* semantics, not its bugs
// (SURVEY §0.5): every missing or corrupt (BLAKE3 mismatch) segment of a
// tier-3 block is restored with one RS(k,3) decode of that block and written
// back to its in-block index; reads map offsets with `%`, not `&`
// (filesystem_unix.rs:216), and tier-3 recovery decodes RS(k,3), not RS(1,3)
// (:112-113).
#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cctype>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <list>
#include <memory>
#include <mutex>
#include <sstream>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "archive_io.hpp"
#include "knobs.hpp"
#include "blake3.hpp"
#include "gpu_block.hpp"
#include "manifest.hpp"
#include "runtime.hpp"

using namespace bfrs;

namespace {

constexpr uint64_t kTier1Limit = 25000000;     // commit.rs:596
constexpr uint64_t kTier2Limit = 1000000000;   // commit.rs:597
constexpr size_t kDefaultSegment = 32u << 20;  // utils.rs:68 on any real host

std::string basename_of(const std::string &p) {
  const size_t s = p.find_last_of('/');
  return s == std::string::npos ? p : p.substr(s + 1);
}

bool pow2_kib(uint64_t s) { return s >= 1024 && s % 1024 == 0 && ((s / 1024) & (s / 1024 - 1)) == 0; }

struct Mapped {
  int fd = -1;
  const uint8_t *p = nullptr;
  size_t n = 0;
  ~Mapped() {
    if (p && n) munmap(const_cast<uint8_t *>(p), n);
    if (fd >= 0) close(fd);
  }
};

struct Commit {
  bfrs_ctx *ctx;
  std::string root, name;
  size_t S;
  std::vector<bfrs_ctx *> ctxs;  // tier 3: blocks dealt over these (ctxs[0] == ctx)
  Mapped m;
  int threads = hw_threads();

  int tier1(std::string *out_dir);
  int tier2(std::string *out_dir);
  int tier3(std::string *out_dir);
  int rs13_segments(size_t nseg, bool cv_hash, std::vector<uint8_t> *seg_cvs,
                    std::vector<struct Rs13Hashes> *hashes,
                    const std::function<bool(size_t, size_t, const uint8_t *const *, size_t)> &write);
  int finish(const std::string &computing, const std::string &file_hash, Manifest &mf,
             std::string *out_dir);
};

int Commit::finish(const std::string &computing, const std::string &file_hash, Manifest &mf,
                   std::string *out_dir) {
  const std::string final_dir = root + "/" + name + "_" + file_hash;
  if (computing != final_dir) {  // commit.rs:266,487
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

// RS(1,3) segments on the GPU (tiers 1 and 2): segment j = file bytes
// [j*S, j*S + len_j), zero-padded to 64 (generate.rs:26-57).  Rounds of up to
// kRound segments with one padded size share an arena: host threads copy
// them from the mmap into pinned slots (4 per segment: data + 3 parity), one
// H2D copy each, one batched encode, device BLAKE3 of data (unpadded) and
// parity, optionally the CV pass at file chunk offsets, D2H of the parity;
// `write` (called on a writer thread) stores the files.  Two arenas and two
// parity buffers alternate so filling, the GPU and writing overlap.
struct Rs13Hashes {
  std::string data;
  std::string parity[3];
};
// writes file `file` of segment `seg`: 0 = the data, 1 + p = parity copy p
using Rs13Writer =
    std::function<bool(size_t seg, size_t file, const uint8_t *const par[3], size_t shard)>;

int Commit::rs13_segments(size_t nseg, bool cv_hash, std::vector<uint8_t> *seg_cvs,
                          std::vector<Rs13Hashes> *hashes, const Rs13Writer &write) {
  constexpr size_t kRound = 4;
  auto seg_len = [&](size_t j) { return std::min(S, m.n - j * S); };
  auto padded = [&](size_t j) { return (seg_len(j) + 63) / 64 * 64; };
  // rounds: consecutive segments with the same padded size, <= kRound each
  std::vector<std::pair<size_t, size_t>> rounds;  // [first, count)
  for (size_t j = 0; j < nseg;) {
    size_t c = 1;
    while (j + c < nseg && c < kRound && padded(j + c) == padded(j)) ++c;
    rounds.push_back({j, c});
    j += c;
  }
  hashes->assign(nseg, {});
  if (cv_hash) seg_cvs->assign(nseg * 32, 0);
  const size_t slot = (std::min(S, m.n) + 63) / 64 * 64;
  PipeTrace pt;
  StagingCache &sc = staging(ctx);
  std::lock_guard<std::mutex> staging_lock(sc.mu);
  // device round buffers (4 slots per segment: data + 3 parity), filled
  // through the pinned ring of sc.blk like the tier-3 commit; only the
  // rounds' parity (3 slots per segment, two rounds) is pinned besides
  Arena *arena = sc.a, *pbuf = sc.a + 2;
  BlockArena &ba = sc.blk;
  Context &c = ctx->impl;
  if (hipSetDevice(c.device) != hipSuccess) return set_error(BFRS_E_HIP, "commit: hipSetDevice");
  const long long t_res = pt.on ? pt.now_us() : 0;
  const size_t nfill = std::min({kRingThreads, size_t(std::max(1, threads)), std::min(kRound, nseg)});
  int rc = ba.reserve_ring(slot, 2 * nfill);
  if (!rc) rc = sc.commit_events();
  for (int i = 0; i < 2 && !rc; ++i) {
    rc = arena[i].reserve(slot, 4 * std::min(kRound, nseg), kArenaDevice);
    if (!rc) rc = pbuf[i].reserve(slot, 3 * std::min(kRound, nseg), kArenaHost);
  }
  if (rc) return rc;
  pt.event("reserve", 0, t_res);
  // round r's segments -> arena[r % 2] (slots 4j); sc.filled[r % 2] marks
  // the last H2D.  arena[r % 2] was last read by round r - 2's GPU work,
  // finished before round r - 1's began; a ring slot is rewritten once its
  // H2D is done.
  auto fill = [&](size_t r) -> int {
    const long long t0 = pt.on ? pt.now_us() : 0;
    const size_t first = rounds[r].first, cnt = rounds[r].second;
    Arena &a = arena[r % 2];
    std::atomic<int> hip_rc{int(hipSuccess)};
    auto hip_ok = [&](hipError_t e) {
      int ok = int(hipSuccess);
      if (e != hipSuccess) hip_rc.compare_exchange_strong(ok, int(e));
      return e == hipSuccess;
    };
    parallel_for(nfill, int(nfill), [&](size_t w) {
      if (!hip_ok(hipSetDevice(c.device))) return;
      size_t turn = 0;
      for (size_t j = w; j < cnt && hip_rc.load() == int(hipSuccess); j += nfill, ++turn) {
        const size_t rs = 2 * w + (turn & 1);
        if (!hip_ok(hipEventSynchronize(ba.ring_ev[rs]))) return;
        const size_t len = seg_len(first + j), pad = padded(first + j);
        uint8_t *h = ba.ring.hs(rs);
        std::memcpy(h, m.p + (first + j) * S, len);
        if (pad > len) std::memset(h + len, 0, pad - len);  // generate.rs:34-46
        if (!hip_ok(hipMemcpyAsync(a.ds(4 * j), h, pad, hipMemcpyHostToDevice, ba.h2d))) return;
        if (!hip_ok(hipEventRecord(ba.ring_ev[rs], ba.h2d))) return;
      }
    });
    if (hip_rc.load() == int(hipSuccess)) hip_ok(hipEventRecord(sc.filled[r % 2], ba.h2d));
    pt.event("fill", r, t0);
    return hip_rc.load() == int(hipSuccess)
               ? BFRS_OK
               : hip_error(hipError_t(hip_rc.load()), "commit: segment H2D through the ring");
  };
  std::atomic<bool> write_ok{true};
  auto write_round = [&](size_t r) {
    const size_t first = rounds[r].first, cnt = rounds[r].second;
    const Arena &pb = pbuf[r % 2];
    const long long t0 = pt.on ? pt.now_us() : 0;
    parallel_for(cnt * (1 + kParity), threads, [&](size_t item) {  // one file per item
      const size_t j = item / (1 + kParity), file = item % (1 + kParity);
      const uint8_t *par[3] = {pb.hs(3 * j), pb.hs(3 * j + 1), pb.hs(3 * j + 2)};
      if (!write(first + j, file, par, padded(first + j))) write_ok = false;
    });
    pt.event("write", r, t0);
  };
  // `wait_writer` is the writer of round r - 2, which still owns pbuf[r % 2]
  auto gpu_round = [&](size_t r, BgTask &wait_writer) -> int {
    const size_t first = rounds[r].first, cnt = rounds[r].second;
    const size_t shard = padded(first);
    Arena &a = arena[r % 2];
    const long long t0 = pt.on ? pt.now_us() : 0;
    if (hipStreamWaitEvent(c.stream, sc.filled[r % 2], 0) != hipSuccess)
      return set_error(BFRS_E_HIP, "commit: wait for the round's H2D failed");
    std::vector<uint32_t> ks(cnt, 1);
    std::vector<const uint8_t *> orig(cnt);
    std::vector<uint8_t *> rec(3 * cnt);
    for (size_t j = 0; j < cnt; ++j) {
      orig[j] = a.ds(4 * j);
      for (size_t p = 0; p < kParity; ++p) rec[3 * j + p] = a.ds(4 * j + 1 + p);
    }
    int rc = encode_batch_on(ctx, cnt, ks.data(), kParity, shard, orig.data(), rec.data(), c.stream);
    if (rc) return rc;
    std::vector<const uint8_t *> msgs;
    std::vector<size_t> lens;
    for (size_t j = 0; j < cnt; ++j) {
      msgs.push_back(a.ds(4 * j));
      lens.push_back(seg_len(first + j));
      for (size_t p = 0; p < kParity; ++p) {
        msgs.push_back(a.ds(4 * j + 1 + p));
        lens.push_back(shard);
      }
    }
    std::vector<std::string> hex;
    if ((rc = gpu_hash_hex(ctx, msgs, lens, &hex))) return rc;
    for (size_t j = 0; j < cnt; ++j) {
      Rs13Hashes &h = (*hashes)[first + j];
      h.data = hex[4 * j];
      for (size_t p = 0; p < kParity; ++p) h.parity[p] = hex[4 * j + 1 + p];
    }
    if (cv_hash) {  // the segments as nodes of the file's BLAKE3 tree
      std::vector<const uint8_t *> sm;
      std::vector<size_t> sl;
      std::vector<uint64_t> offs;
      for (size_t j = 0; j < cnt; ++j) {
        sm.push_back(a.ds(4 * j));
        sl.push_back(seg_len(first + j));
        offs.push_back(uint64_t(first + j) * (S / 1024));
      }
      std::vector<std::string> unused;
      std::vector<uint8_t> cvs;
      if ((rc = gpu_hash_hex(ctx, sm, sl, &unused, offs.data(), &cvs))) return rc;
      std::memcpy(seg_cvs->data() + first * 32, cvs.data(), cnt * 32);
    }
    pt.event("h2d_encode_hash", r, t0);
    const long long t1 = pt.on ? pt.now_us() : 0;
    wait_writer.join();
    pt.event("wait_writer", r, t1);
    const long long t2 = pt.on ? pt.now_us() : 0;
    Arena &pb = pbuf[r % 2];
    for (size_t j = 0; j < cnt; ++j)
      for (size_t p = 0; p < kParity; ++p)
        if (hipMemcpyAsync(pb.hs(3 * j + p), a.ds(4 * j + 1 + p), shard, hipMemcpyDeviceToHost,
                           c.stream) != hipSuccess)
          return set_error(BFRS_E_HIP, "commit: D2H copy failed");
    if (hipStreamSynchronize(c.stream) != hipSuccess)
      return set_error(BFRS_E_HIP, "commit: stream synchronize failed");
    pt.event("d2h", r, t2);
    return BFRS_OK;
  };
  rc = fill(0);
  {
    BgTask writer[2];  // after the lambdas: joined first on every exit path
    for (size_t r = 0; r < rounds.size() && rc == BFRS_OK; ++r) {
      int fill_rc = BFRS_OK;
      std::string fill_err;
      {
        BgTask filler;
        if (r + 1 < rounds.size())
          filler.start([&fill, &fill_rc, &fill_err, r] {
            fill_rc = fill(r + 1);
            if (fill_rc) fill_err = bfrs_last_error();  // thread-local: carried back
          });
        rc = gpu_round(r, writer[r % 2]);
        filler.join();
      }
      if (rc == BFRS_OK && fill_rc) rc = set_error(fill_rc, fill_err);
      if (rc == BFRS_OK) writer[r % 2].start([&write_round, r] { write_round(r); });
    }
    for (auto &w : writer) w.join();
  }
  // nothing of this call may still be copying into the ring or the rounds
  if (hipStreamSynchronize(ba.h2d) != hipSuccess && rc == BFRS_OK)
    rc = set_error(BFRS_E_HIP, "commit: ring stream synchronize failed");
  pt.print("bfrs_rs13_trace", threads);
  if (rc) return rc;
  return write_ok ? BFRS_OK : io_error("write RS(1,3) shards");
}

// commit_tiny (commit.rs:25-118): RS(1,3) of the 64-padded file; the file
// digest is the data shard's (unpadded) device BLAKE3.
int Commit::tier1(std::string *out_dir) {
  S = m.n;  // one segment: the whole file
  std::vector<Rs13Hashes> hs;
  std::string dir;
  // the directory name needs the file hash, which the GPU pass produces: hash
  // and encode into memory first (the writer runs after the pass completes)
  std::vector<std::vector<uint8_t>> par(kParity);
  // called for files 1-3 on the writer's threads at once: each touches only
  // its own parity copy (no shared write)
  auto keep = [&](size_t, size_t file, const uint8_t *const p[3], size_t sh) {
    if (file == 0) return true;  // the data is written from the mapping below
    par[file - 1].assign(p[file - 1], p[file - 1] + sh);
    return true;
  };
  int rc = rs13_segments(1, false, nullptr, &hs, keep);
  if (rc) return rc;
  const size_t shard = par[0].size();  // the 64-padded file (generate.rs:34-46)
  const std::string file_hash = hs[0].data;
  dir = root + "/" + name + "_" + file_hash;
  if (!mkdirs(dir)) return io_error("mkdir " + dir);
  std::atomic<bool> ok{true};
  parallel_for(1 + kParity, 1 + kParity, [&](size_t f) {  // the four files side by side
    const bool w = f == 0 ? write_file(dir + "/data.dat", m.p, m.n)
                          : write_file(dir + "/parity_" + std::to_string(f - 1) + ".dat",
                                       par[f - 1].data(), shard);
    if (!w) ok = false;
  });
  if (!ok) return io_error("write tier-1 shards");
  Manifest mf;
  mf.tier = 1;
  mf.data_shards = 6;  // commit.rs:98 (sic)
  mf.parity_shards = 3;
  mf.segment_size = shard;
  std::vector<std::string> leaves{file_hash, hs[0].parity[0], hs[0].parity[1], hs[0].parity[2]};
  for (size_t i = 0; i < leaves.size(); ++i) mf.leaves[int64_t(i)] = leaves[i];
  mf.root = merkle_root_hex(leaves);
  return finish(dir, file_hash, mf, out_dir);
}

// commit_segmented (commit.rs:124-309): per-segment RS(1,3), all on the GPU.
int Commit::tier2(std::string *out_dir) {
  const std::string dir = root + "/" + name + "_computing";
  if (!mkdirs(dir + "/segments") || !mkdirs(dir + "/parity")) return io_error("mkdir " + dir);
  const size_t nseg = (m.n + S - 1) / S;
  const bool cv_hash = pow2_kib(S) && nseg >= 2;
  std::vector<Rs13Hashes> hs;
  std::vector<uint8_t> seg_cvs;
  auto write = [&](size_t j, size_t file, const uint8_t *const par[3], size_t shard) {
    if (file == 0) return write_file(t2_seg(dir, j), m.p + j * S, std::min(S, m.n - j * S));
    return write_file(t2_par(dir, j, file - 1), par[file - 1], shard);
  };
  int rc = rs13_segments(nseg, cv_hash, &seg_cvs, &hs, write);
  if (rc) return rc;
  Manifest mf;
  mf.tier = 2;
  mf.data_shards = 6;  // commit.rs:294 (sic)
  mf.parity_shards = 3;
  mf.segment_size = S;
  std::vector<std::string> seg_roots(nseg);
  for (size_t j = 0; j < nseg; ++j) {
    SegmentHashes sh;
    sh.data = hs[j].data;
    sh.parity.assign(hs[j].parity, hs[j].parity + kParity);
    std::vector<std::string> leaves{sh.data};
    leaves.insert(leaves.end(), sh.parity.begin(), sh.parity.end());
    seg_roots[j] = merkle_root_hex(leaves);
    mf.segments[int64_t(j)] = sh;
  }
  mf.root = merkle_root_hex(seg_roots);
  const std::string file_hash = cv_hash ? blake3_combine_cvs_hex(seg_cvs.data(), nseg)
                                        : nseg == 1 ? hs[0].data : blake3_hex(m.p, m.n, threads);
  return finish(dir, file_hash, mf, out_dir);
}

// commit_blocked (commit.rs:314-536), GPU-pipelined.  Per block of k <= 30
// segments: host threads copy the segments from the mmap into a pinned
// arena (zero-padding a short last segment, generate.rs:75-82), one H2D
// copy, RS(k,3) encode, device BLAKE3 of all k+3 shards (commit.rs:429,451)
// plus a second pass at file chunk offsets for the whole-file hash
// (commit.rs:478, combined from the segment CVs), D2H of the parity.  Two
// arenas alternate: the next block is filled while the GPU works, and the
// previous block's files are written by a writer thread.
int Commit::tier3(std::string *out_dir) {
  const std::string dir = root + "/" + name + "_computing";
  const size_t nseg = (m.n + S - 1) / S;
  const size_t nblocks = (nseg + kBlockSegments - 1) / kBlockSegments;
  // A block's shard size is its first segment's length (generate.rs:66-72);
  // the crate rejects an odd one (ReedSolomonEncoder::new, generate.rs:84,
  // called at commit.rs:440-441): a file whose last block is one odd-length
  // segment fails here, before anything is written.
  for (size_t b = 0; b < nblocks; ++b) {
    const size_t shard = std::min(S, m.n - b * kBlockSegments * S);
    if (shard & 1) {
      std::ostringstream os;
      os << "invalid shard size: " << shard << " bytes (block " << b
         << "; must be non-zero and a multiple of 2)";
      return set_error(BFRS_E_INVALID_SHARD_SIZE, os.str());
    }
  }
  for (size_t b = 0; b < nblocks; ++b)
    if (!mkdirs(dir + "/blocks/block_" + std::to_string(b) + "/segments") ||
        !mkdirs(dir + "/blocks/block_" + std::to_string(b) + "/parity"))
      return io_error("mkdir " + dir);
  Manifest mf;
  mf.tier = 3;
  mf.data_shards = 30;
  mf.parity_shards = 3;
  mf.segment_size = S;
  const bool cv_hash = pow2_kib(S) && nseg >= 2;
  std::vector<uint8_t> seg_cvs(cv_hash ? nseg * 32 : 0);
  std::vector<std::string> block_roots(nblocks);
  std::vector<BlockHashes> block_hashes(nblocks);
  auto geom = [&](size_t b, size_t *s0, size_t *k, size_t *shard) {
    *s0 = b * kBlockSegments;
    *k = std::min(kBlockSegments, nseg - *s0);
    *shard = std::min(S, m.n - *s0 * S);  // the block's first segment is its longest
  };
  std::atomic<bool> write_ok{true};
  std::atomic<bool> stop{false};  // a failed context stops the others before their next block
  PipeTrace pt;
  const bool trace = pt.on;
  auto now_us = [&] { return pt.now_us(); };
  auto event = [&](const char *what, size_t b, long long t0) { pt.event(what, b, t0); };
  // The pipeline of one context over its blocks `mine` (in file order): its
  // own staging arenas, stream, filler and writers; `thr` host threads for
  // the copies.  Every result lands in a per-block slot (seg_cvs ranges,
  // block_roots, block_hashes), so several pipelines run side by side.
  auto pipeline = [&](bfrs_ctx *cx, const std::vector<size_t> &mine, int thr) -> int {
    Context &c = cx->impl;
    if (hipSetDevice(c.device) != hipSuccess) return set_error(BFRS_E_HIP, "commit: hipSetDevice");
    StagingCache &sc = staging(cx);
    std::lock_guard<std::mutex> staging_lock(sc.mu);
    // Segments reach HBM through a ring of pinned slots: filler thread w
    // copies segments w, w + nfill, ... of a block from the mmap into its two
    // slots in turn and queues each one's H2D on the ring's stream, so copies
    // and DMA overlap and only 2 x nfill segments (not two whole blocks) are
    // pinned.
    const size_t nfill = std::min<size_t>(kRingThreads, size_t(std::max(1, thr)));
    BlockArena &ba = sc.blk;
    // what block 0's fill needs first (the ring and one device block); the
    // second device block and the pinned parity slots are reserved beside
    // that fill (a context's first commit spent ~1/3 of its time reserving
    // before any segment moved)
    int rc = ba.reserve_ring(S);
    if (!rc) rc = ba.dev.reserve(S, kBlockSegments + kParity, kArenaDevice);
    if (!rc) rc = sc.commit_events();
    if (rc) return rc;
    int late_rc = BFRS_OK;
    std::string late_err;
    BgTask late;
    late.start([&] {
      late_rc = hipSetDevice(c.device) == hipSuccess
                    ? sc.blk2.reserve(S, kBlockSegments + kParity, kArenaDevice)
                    : set_error(BFRS_E_HIP, "commit: hipSetDevice");
      if (!late_rc) late_rc = ba.out.reserve(S, kOutSlots, kArenaHost);
      if (late_rc) late_err = bfrs_last_error();  // thread-local: carried back
    });
    Arena *blk[2] = {&ba.dev, &sc.blk2};
    // the pinned parity of the block being written: out slots [3 (i % 2), +3)
    auto pbuf = [&](size_t i, size_t p) { return ba.out.hs(kParity * (i % 2) + p); };
    // block i's segments -> blk[i % 2]; sc.filled[i % 2] marks the last H2D.
    // blk[i % 2] was last read by block i - 2's GPU work, finished before
    // block i - 1's began; a ring slot is rewritten once its H2D is done.
    auto fill = [&](size_t i) -> int {
      const long long t0 = trace ? now_us() : 0;
      size_t s0, k, shard;
      geom(mine[i], &s0, &k, &shard);
      Arena &a = *blk[i % 2];
      std::atomic<int> hip_rc{int(hipSuccess)};
      auto hip_ok = [&](hipError_t e) {
        int ok = int(hipSuccess);
        if (e != hipSuccess) hip_rc.compare_exchange_strong(ok, int(e));
        return e == hipSuccess;
      };
      parallel_for(nfill, int(nfill), [&](size_t w) {
        if (!hip_ok(hipSetDevice(c.device))) return;
        size_t turn = 0;
        for (size_t s = w; s < k && hip_rc.load() == int(hipSuccess); s += nfill, ++turn) {
          const size_t r = 2 * w + (turn & 1);
          if (!hip_ok(hipEventSynchronize(ba.ring_ev[r]))) return;
          const size_t len = std::min(S, m.n - (s0 + s) * S);
          uint8_t *h = ba.ring.hs(r);
          std::memcpy(h, m.p + (s0 + s) * S, len);
          if (len < shard) std::memset(h + len, 0, shard - len);  // generate.rs:75-82
          if (!hip_ok(hipMemcpyAsync(a.ds(s), h, shard, hipMemcpyHostToDevice, ba.h2d))) return;
          if (!hip_ok(hipEventRecord(ba.ring_ev[r], ba.h2d))) return;
        }
      });
      if (hip_rc.load() == int(hipSuccess)) hip_ok(hipEventRecord(sc.filled[i % 2], ba.h2d));
      event("fill", mine[i], t0);
      return hip_rc.load() == int(hipSuccess)
                 ? BFRS_OK
                 : hip_error(hipError_t(hip_rc.load()), "commit: segment H2D through the ring");
    };
    auto write_block = [&](size_t i) {  // segments from the mmap, parity from pbuf
      const size_t b = mine[i];
      size_t s0, k, shard;
      geom(b, &s0, &k, &shard);
      const long long t0 = trace ? now_us() : 0;
      parallel_for(k + kParity, thr, [&](size_t j) {
        bool ok;
        if (j < k)
          ok = write_file(t3_seg(dir, b, j), m.p + (s0 + j) * S, std::min(S, m.n - (s0 + j) * S));
        else
          ok = write_file(t3_par(dir, b, j - k), pbuf(i, j - k), shard);
        if (!ok) write_ok = false;
      });
      event("write", b, t0);
    };
    // one block on the GPU: encode, hashes, D2H parity into pbuf[i % 2].
    // `wait_writer` is the writer of block i - 2, which still owns pbuf[i % 2]
    auto gpu_block = [&](size_t i, BgTask &wait_writer) -> int {
      const size_t b = mine[i];
      size_t s0, k, shard;
      geom(b, &s0, &k, &shard);
      Arena &a = *blk[i % 2];
      const long long t1 = trace ? now_us() : 0;
      if (hipStreamWaitEvent(c.stream, sc.filled[i % 2], 0) != hipSuccess)
        return set_error(BFRS_E_HIP, "commit: wait for the block's H2D failed");
      std::vector<const uint8_t *> orig(k);
      std::vector<uint8_t *> rec(kParity);
      for (size_t s = 0; s < k; ++s) orig[s] = a.ds(s);
      for (size_t p = 0; p < kParity; ++p) rec[p] = a.ds(k + p);
      const uint32_t kk = uint32_t(k);
      int rc = encode_batch_on(cx, 1, &kk, kParity, shard, orig.data(), rec.data(), c.stream);
      if (rc) return rc;
      // the block's H2D and encode land before the hash takes hash_mu
      if (hipStreamSynchronize(c.stream) != hipSuccess)
        return set_error(BFRS_E_HIP, "commit: stream synchronize failed");
      event("h2d_encode", b, t1);
      const long long t2 = trace ? now_us() : 0;
      std::vector<const uint8_t *> msgs;
      std::vector<size_t> lens;
      for (size_t s = 0; s < k; ++s) {
        msgs.push_back(a.ds(s));
        lens.push_back(std::min(S, m.n - (s0 + s) * S));
      }
      for (size_t p = 0; p < kParity; ++p) {
        msgs.push_back(a.ds(k + p));
        lens.push_back(shard);
      }
      std::vector<std::string> hex;
      if ((rc = gpu_hash_hex(cx, msgs, lens, &hex))) return rc;
      if (cv_hash) {  // the segments as nodes of the file's BLAKE3 tree
        std::vector<const uint8_t *> sm(msgs.begin(), msgs.begin() + k);
        std::vector<size_t> sl(lens.begin(), lens.begin() + k);
        std::vector<uint64_t> offs(k);
        for (size_t s = 0; s < k; ++s) offs[s] = uint64_t(s0 + s) * (S / 1024);
        std::vector<std::string> unused;
        std::vector<uint8_t> cvs;
        if ((rc = gpu_hash_hex(cx, sm, sl, &unused, offs.data(), &cvs))) return rc;
        std::memcpy(seg_cvs.data() + s0 * 32, cvs.data(), k * 32);
      }
      event("hash", b, t2);
      const long long t3 = trace ? now_us() : 0;
      wait_writer.join();
      event("wait_writer", b, t3);
      const long long t4 = trace ? now_us() : 0;
      for (size_t p = 0; p < kParity; ++p)
        if (hipMemcpyAsync(pbuf(i, p), a.ds(k + p), shard, hipMemcpyDeviceToHost, c.stream) !=
            hipSuccess)
          return set_error(BFRS_E_HIP, "commit: D2H copy failed");
      if (hipStreamSynchronize(c.stream) != hipSuccess)
        return set_error(BFRS_E_HIP, "commit: stream synchronize failed");
      event("d2h", b, t4);
      BlockHashes &bh = block_hashes[b];
      bh.segments.assign(hex.begin(), hex.begin() + k);
      bh.parity.assign(hex.begin() + k, hex.end());
      std::vector<std::string> leaves = bh.segments;
      leaves.insert(leaves.end(), bh.parity.begin(), bh.parity.end());
      block_roots[b] = merkle_root_hex(leaves);
      return BFRS_OK;
    };
    if (mine.empty()) {
      late.join();
      return late_rc ? set_error(late_rc, late_err) : rc;
    }
    rc = fill(0);
    late.join();  // blk2 and the parity slots are first used below
    if (rc == BFRS_OK && late_rc) rc = set_error(late_rc, late_err);
    {
      BgTask writer[2];  // after the lambdas: joined first on every exit path
      for (size_t i = 0; i < mine.size() && rc == BFRS_OK; ++i) {
        if (stop.load(std::memory_order_relaxed)) break;  // another context failed
        int fill_rc = BFRS_OK;
        std::string fill_err;
        {
          BgTask filler;
          if (i + 1 < mine.size())
            filler.start([&fill, &fill_rc, &fill_err, i] {
              fill_rc = fill(i + 1);
              if (fill_rc) fill_err = bfrs_last_error();  // thread-local: carried back
            });
          rc = gpu_block(i, writer[i % 2]);
          filler.join();
        }
        if (rc == BFRS_OK && fill_rc) rc = set_error(fill_rc, fill_err);
        if (rc == BFRS_OK) writer[i % 2].start([&write_block, i] { write_block(i); });
      }
      for (auto &w : writer) w.join();
    }
    // nothing of this call may still be copying into the ring or the blocks
    if (hipStreamSynchronize(ba.h2d) != hipSuccess && rc == BFRS_OK)
      rc = set_error(BFRS_E_HIP, "commit: ring stream synchronize failed");
    return rc;
  };
  // blocks dealt round-robin over the contexts (block b to context b % n)
  const size_t n = std::max<size_t>(1, std::min(ctxs.size(), nblocks));
  std::vector<std::vector<size_t>> mine(n);
  for (size_t b = 0; b < nblocks; ++b) mine[b % n].push_back(b);
  const int thr = std::max(2, threads / int(n));
  std::vector<int> rcs(n, BFRS_OK);
  std::vector<std::string> errs(n);
  auto run = [&](size_t d) {
    try {
      rcs[d] = pipeline(ctxs[d], mine[d], n == 1 ? threads : thr);
    } catch (const std::bad_alloc &) {
      rcs[d] = set_error(BFRS_E_NOMEM, "host memory allocation failed");
    } catch (const std::exception &e) {
      rcs[d] = set_error(BFRS_E_WRAPPER, std::string("internal error: ") + e.what());
    }
    if (rcs[d]) {
      errs[d] = bfrs_last_error();  // thread-local: carried back below
      stop = true;
    }
  };
  {
    std::vector<BgTask> others(n - 1);  // joined on every exit path
    for (size_t d = 1; d < n; ++d) others[d - 1].start([&run, d] { run(d); });
    run(0);
    for (auto &t : others) t.join();
  }
  pt.print("bfrs_commit_trace", threads);
  for (size_t d = 0; d < n; ++d)
    if (rcs[d]) return set_error(rcs[d], n == 1 ? errs[d] : "context " + std::to_string(d) + ": " + errs[d]);
  if (!write_ok) return io_error("write tier-3 shards");
  for (size_t b = 0; b < nblocks; ++b) mf.blocks[int64_t(b)] = std::move(block_hashes[b]);
  mf.root = merkle_root_hex(block_roots);
  const std::string file_hash = cv_hash ? blake3_combine_cvs_hex(seg_cvs.data(), nseg)
                                        : nseg == 1 ? mf.blocks[0].segments[0]
                                                    : blake3_hex(m.p, m.n, threads);
  return finish(dir, file_hash, mf, out_dir);
}

// ---------------------------------------------------------------------------
// Verified bytes of one stored shard, CPU hash on the host threads (tiers
// 1/2: files of up to a segment; the digest does not depend on the threads).
bool load_verified(const std::string &path, const std::string &want_hex, std::vector<uint8_t> *out,
                   int threads = hw_threads()) {
  if (!read_file(path, out)) return false;
  return blake3_hex(out->data(), out->size(), threads) == want_hex;
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
  if (blake3_hex(restored.data(), restored.size(), hw_threads()) != want)
    return set_error(BFRS_E_WRAPPER, "restored bytes fail the manifest hash");
  *out = std::move(restored);
  return BFRS_OK;
}

// Fixed-size pinned buffers backing the read cache (pinned so a segment
// goes to HBM for verification without a staging copy).
struct PinnedPool {
  size_t slot;
  std::mutex mu;
  std::vector<uint8_t *> free_, all_;
  explicit PinnedPool(size_t s) : slot(std::max<size_t>(256, (s + 255) / 256 * 256)) {}
  ~PinnedPool() {
    for (uint8_t *p : all_) pinned_free(p, slot);
  }
  uint8_t *get() {
    {
      std::lock_guard<std::mutex> g(mu);
      if (!free_.empty()) {
        uint8_t *p = free_.back();
        free_.pop_back();
        return p;
      }
    }
    void *p = pinned_alloc(slot);
    if (!p) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    all_.push_back(static_cast<uint8_t *>(p));
    return static_cast<uint8_t *>(p);
  }
  void put(uint8_t *p) {
    std::lock_guard<std::mutex> g(mu);
    free_.push_back(p);
  }
  size_t idle_bytes() {
    std::lock_guard<std::mutex> g(mu);
    return free_.size() * slot;
  }
  size_t size() {
    std::lock_guard<std::mutex> g(mu);
    return all_.size();
  }
  // pins one more buffer into the idle list (a handle's pre-pinning thread)
  bool grow() {
    void *p = pinned_alloc(slot);
    if (!p) return false;
    std::lock_guard<std::mutex> g(mu);
    all_.push_back(static_cast<uint8_t *>(p));
    free_.push_back(static_cast<uint8_t *>(p));
    return true;
  }
  uint64_t last_release = 0;  // StagingCache::pool_tick at the last release (pools_mu)
  // unpins idle buffers beyond `keep` (a handle closing: what a long-lived
  // context retains is bounded, not the largest cache it ever served)
  void trim(size_t keep) {
    std::vector<uint8_t *> drop;
    {
      std::lock_guard<std::mutex> g(mu);
      while (free_.size() > keep) {
        drop.push_back(free_.back());
        free_.pop_back();
        all_.erase(std::find(all_.begin(), all_.end(), drop.back()));
      }
    }
    for (uint8_t *p : drop) pinned_free(p, slot);
  }
};
// idle pinned segment buffers a context keeps per segment size: 2 GiB, >= 8
inline size_t pool_keep(size_t slot) { return std::max<size_t>(8, (size_t(2) << 30) / slot); }
// idle pinned bytes a context keeps over every pool no open handle uses
constexpr size_t kIdlePinnedCap = size_t(2) << 30;
// the measurement build may lower it (BFRS_IDLE_PIN_CAP, bytes) so a test can
// drive the eviction with small files (tests/test_gpu_archive.py)
size_t idle_pinned_cap() {
  if (const char *e = BFRS_AB_KNOB("BFRS_IDLE_PIN_CAP")) return size_t(std::strtoull(e, nullptr, 10));
  return kIdlePinnedCap;
}

// A read handle lets go of its pool (closing or detached).  The pool keeps at
// most pool_keep idle buffers; then, over the pools of the context that no
// other handle holds, the least recently released are unpinned and dropped
// until their idle buffers fit kIdlePinnedCap.  (before, every
// distinct segment size -- each tier-1 file size -- kept a pool until
// bfrs_close, so a long-lived mount context grew pinned memory without limit.)
void release_pool(bfrs_ctx *ctx, std::shared_ptr<PinnedPool> pool) {
  if (!pool) return;
  pool->trim(pool_keep(pool->slot));
  StagingCache &sc = staging(ctx);
  std::vector<std::shared_ptr<void>> drop;  // unpinned after the lock is released
  {
    std::lock_guard<std::mutex> l(sc.pools_mu);
    pool->last_release = ++sc.pool_tick;
    pool.reset();
    struct Idle {
      size_t key;
      uint64_t tick;
      size_t bytes;
    };
    std::vector<Idle> idle;
    size_t total = 0;
    for (auto &e : sc.seg_pools) {
      if (e.second.use_count() > 1) continue;  // an open handle holds it
      auto *pp = static_cast<PinnedPool *>(e.second.get());
      const size_t bytes = pp->idle_bytes();
      idle.push_back({e.first, pp->last_release, bytes});
      total += bytes;
    }
    std::sort(idle.begin(), idle.end(), [](const Idle &a, const Idle &b) { return a.tick < b.tick; });
    for (const Idle &i : idle) {
      if (total <= idle_pinned_cap()) break;
      auto it = sc.seg_pools.find(i.key);
      drop.push_back(std::move(it->second));
      sc.seg_pools.erase(it);
      total -= i.bytes;
    }
  }
}

// The context's pool for buffers of `bytes` (StagingCache::seg_pools).
std::shared_ptr<PinnedPool> segment_pool(bfrs_ctx *ctx, size_t bytes) {
  StagingCache &sc = staging(ctx);
  auto pool = std::make_shared<PinnedPool>(bytes);
  std::lock_guard<std::mutex> l(sc.pools_mu);
  std::shared_ptr<void> &slot = sc.seg_pools[pool->slot];
  if (slot) return std::static_pointer_cast<PinnedPool>(slot);
  slot = pool;
  return pool;
}

// A clean segment's verification lane: one HBM segment buffer and a stream
// of its own, so prefetch workers verify segments side by side and beside a
// block reconstruction (which uses the context's read arena and stream);
// only the hash itself is serialised (the context's hash_mu).
struct CleanLane {
  std::mutex mu;
  uint8_t *d = nullptr;
  size_t cap = 0;
  hipStream_t st = nullptr;
  CleanLane() = default;
  CleanLane(const CleanLane &) = delete;
  CleanLane &operator=(const CleanLane &) = delete;
  ~CleanLane() {
    if (st) (void)hipStreamDestroy(st);
    if (d) (void)hipFree(d);
  }
  int ready(size_t bytes) {  // under mu, on the context's device
    if (!st) HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    if (d && cap >= bytes) return BFRS_OK;
    if (d) {
      HIP_TRY(hipFree(d));
      d = nullptr;
    }
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d), bytes));
    cap = bytes;
    return BFRS_OK;
  }
};

struct Seg {
  uint8_t *p = nullptr;
  size_t n = 0;
  std::shared_ptr<PinnedPool> pool;
  Seg(std::shared_ptr<PinnedPool> pl, uint8_t *buf, size_t len) : p(buf), n(len), pool(std::move(pl)) {}
  ~Seg() {
    if (p) pool->put(p);
  }
};
using SegPtr = std::shared_ptr<Seg>;

// Read-path timeline, measurement build only (BFRS_TRACE): what the reader
// waits for and how long loads and block reconstructions take, one line on
// stderr when the handle closes.  Off (one branch) in libbfrs.so.
struct ReadTrace {
  bool on = false;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  std::mutex mu;
  std::vector<std::string> events;
  std::atomic<long long> reader_wait_ns{0}, reader_miss_ns{0}, gpu_lock_wait_ns{0},
      clean_read_ns{0}, clean_gpu_ns{0}, rec_load_ns{0}, rec_restore_ns{0}, rec_copy_ns{0};
  std::atomic<long long> reader_waits{0}, cleans{0};
  long long ns() const {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
        .count();
  }
  void event(const char *what, size_t gi, long long start, long long end) {
    if (!on) return;
    std::lock_guard<std::mutex> l(mu);
    std::ostringstream os;
    os << "[\"" << what << "\"," << gi << "," << start / 1000 << "," << (end - start) / 1000 << "]";
    events.push_back(os.str());
  }
  void print() {
    if (!on) return;
    std::ostringstream os;
    os << "bfrs_read_trace {\"reader_waits\":" << reader_waits << ",\"reader_wait_ms\":"
       << reader_wait_ns / 1e6 << ",\"reader_miss_ms\":" << reader_miss_ns / 1e6
       << ",\"cleans\":" << cleans << ",\"clean_read_ms\":" << clean_read_ns / 1e6
       << ",\"clean_gpu_ms\":" << clean_gpu_ns / 1e6 << ",\"gpu_lock_wait_ms\":"
       << gpu_lock_wait_ns / 1e6 << ",\"rec_load_ms\":" << rec_load_ns / 1e6
       << ",\"rec_restore_ms\":" << rec_restore_ns / 1e6 << ",\"rec_copy_ms\":"
       << rec_copy_ns / 1e6 << ",\"events_us\":[";
    for (size_t i = 0; i < events.size(); ++i) os << (i ? "," : "") << events[i];
    os << "]}\n";
    std::fputs(os.str().c_str(), stderr);
  }
};

}  // namespace

// ---------------------------------------------------------------------------
// Archive read handle (src/mount/filesystem_unix.rs:176-305 + cache.rs).
// Segments are cached in pinned buffers (LRU); a miss reads the file,
// verifies it on the GPU and, if it is missing or corrupt, reconstructs it
// (tier 3: RS(k,3) decode of its block on the GPU, device re-verify).  When
// reads move to a new segment, the next prefetch_depth segments are queued
// for prefetch_workers threads that load and verify them (reconstructing a
// damaged one with its block), so sequential reads
// overlap file reads, PCIe and hashing with serving (the file read of one
// segment overlaps the GPU verify of another).
struct bfrs_archive {
  bfrs_ctx *ctx = nullptr;
  Geometry g;
  size_t cap = 1;
  bool write_back = false;
  bool prefetch = true;
  std::shared_ptr<PinnedPool> pool;

  std::mutex mu;  // cache, stats, prefetch state
  std::condition_variable cv;
  std::list<size_t> lru;
  std::unordered_map<size_t, std::pair<SegPtr, std::list<size_t>::iterator>> cache;
  bfrs_archive_stats st{};
  // segments queued ahead of the reader and the threads that load them
  // (BFRS_PREFETCH_DEPTH / BFRS_PREFETCH_WORKERS override at open)
  size_t prefetch_depth = 16, prefetch_workers = 2;
  std::deque<size_t> wantq;               // queued, not started
  // segments being loaded (by a prefetch worker or a reader); everyone else
  // waits on cv for them instead of loading them again
  std::unordered_set<size_t> inflight;
  long long last_gi = -1;
  bool stop = false;
  std::vector<std::thread> workers;
  // Pre-pinning at open: reserves the context's read
  // arena (tier 3) and pins the pool up to what this handle's cache and
  // prefetch will hold, beside the first reads instead of inside them.
  std::atomic<bool> stop_pin{false};
  BgTask pinner;

  std::mutex gpu_mu;  // tier 1/2 reconstructions, one at a time (tier 3: StagingCache::read_mu)
  std::vector<std::unique_ptr<CleanLane>> lanes;  // clean-segment verification
  ReadTrace trace;

  bfrs_archive() { add_lanes(1); }
  void add_lanes(size_t n) {
    for (size_t i = 0; i < n; ++i) lanes.emplace_back(new CleanLane);
  }
  // a free lane, else the lane for gi (blocking); lanes are never resized
  // once prefetch workers run
  std::unique_lock<std::mutex> take_lane(size_t gi, CleanLane **out) {
    for (auto &ln : lanes) {
      std::unique_lock<std::mutex> l(ln->mu, std::try_to_lock);
      if (l.owns_lock()) {
        *out = ln.get();
        return l;
      }
    }
    *out = lanes[gi % lanes.size()].get();
    return std::unique_lock<std::mutex>((*out)->mu);
  }

  void stop_workers() {
    stop_pin = true;
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto &w : workers)
      if (w.joinable()) w.join();
    workers.clear();
    try {
      pinner.join();
    } catch (...) {  // the pre-pinning is best effort
    }
  }
  void prepin();
  // bfrs_close of the context (under its handles_mu): joins the prefetch
  // threads and lets go of everything of the context; later reads fail with
  // an error and bfrs_archive_close frees only the handle.
  void detach() {
    stop_workers();
    {
      DeviceScope scope(ctx->impl.device);
      lanes.clear();  // their HBM and streams
    }
    std::lock_guard<std::mutex> l(mu);
    cache.clear();
    lru.clear();
    release_pool(ctx, std::move(pool));
    ctx = nullptr;
  }
  ~bfrs_archive() {
    stop_workers();
    cache.clear();
    if (ctx) {
      {
        std::lock_guard<std::mutex> l(ctx->impl.handles_mu);
        auto &h = ctx->impl.handles;
        h.erase(std::remove(h.begin(), h.end(), this), h.end());
      }
      release_pool(ctx, std::move(pool));
    }
    trace.print();
  }

  SegPtr lookup(size_t gi) {  // under mu
    auto it = cache.find(gi);
    if (it == cache.end()) return nullptr;
    lru.splice(lru.begin(), lru, it->second.second);
    return it->second.first;
  }
  void put(size_t gi, SegPtr v) {  // under mu
    auto it = cache.find(gi);
    if (it != cache.end()) {
      lru.erase(it->second.second);
      cache.erase(it);
    }
    lru.push_front(gi);
    cache[gi] = {std::move(v), lru.begin()};
    while (cache.size() > cap) {
      cache.erase(lru.back());
      lru.pop_back();
    }
  }
  std::string expected_hash(size_t gi) const;
  std::string seg_path(size_t gi) const;
  int load_clean(size_t gi, SegPtr *out, bool *ok);  // no locks held
  // device BLAKE3 of `len` pinned bytes on a free verification lane
  int lane_hash(const uint8_t *buf, size_t len, size_t key, std::string *hex);
  // *ok = the file at `path` hashes to want_hex (device BLAKE3; tiers 1/2's
  // parity copies, up to one pool buffer long)
  int verify_file(const std::string &path, const std::string &want_hex, bool *ok);
  int recover(size_t gi, SegPtr *out);              // no locks held
  // Verify segment gi (and reconstruct it if damaged) with mu released,
  // holding gi in `inflight` so that other readers wait for it.  Every exit,
  // an exception included, re-locks, drops gi from inflight and wakes the
  // waiters; an exception becomes an error code here (a prefetch thread has
  // nobody to catch it).  *verified: the file was clean; *restored: rebuilt.
  int load_inflight(std::unique_lock<std::mutex> &l, size_t gi, SegPtr *seg, bool *verified,
                    bool *restored);
  void prefetch_loop(size_t worker);
};

int bfrs_archive::load_inflight(std::unique_lock<std::mutex> &l, size_t gi, SegPtr *seg,
                                bool *verified, bool *restored) {
  inflight.insert(gi);
  struct Done {
    bfrs_archive *a;
    std::unique_lock<std::mutex> &l;
    size_t gi;
    ~Done() {
      if (!l.owns_lock()) l.lock();
      a->inflight.erase(gi);
      a->cv.notify_all();
    }
  } done{this, l, gi};
  *verified = *restored = false;
  l.unlock();
  int rc;
  try {
    rc = load_clean(gi, seg, verified);
    if (rc == BFRS_OK && !*verified) {
      rc = recover(gi, seg);
      *restored = rc == BFRS_OK;
    }
  } catch (const std::bad_alloc &) {
    rc = set_error(BFRS_E_NOMEM, "host memory allocation failed");
  } catch (const std::exception &ex) {
    rc = set_error(BFRS_E_WRAPPER, std::string("internal error: ") + ex.what());
  } catch (...) {
    rc = set_error(BFRS_E_WRAPPER, "internal error");
  }
  l.lock();
  return rc;
}

std::string bfrs_archive::expected_hash(size_t gi) const {
  const Manifest &mf = g.mf;
  if (mf.tier == 3) return mf.blocks.at(int64_t(gi / kBlockSegments)).segments[gi % kBlockSegments];
  if (mf.tier == 2) return mf.segments.at(int64_t(gi)).data;
  return mf.leaves.at(0);
}

std::string bfrs_archive::seg_path(size_t gi) const {
  if (g.mf.tier == 3) return t3_seg(g.dir, gi / kBlockSegments, gi % kBlockSegments);
  if (g.mf.tier == 2) return t2_seg(g.dir, gi);
  return g.dir + "/data.dat";
}

// Reads segment gi into a pinned buffer and verifies it with the device
// BLAKE3; *ok = false if it is missing, short or fails the manifest hash.
int bfrs_archive::load_clean(size_t gi, SegPtr *out, bool *ok) {
  *ok = false;
  const size_t len = g.seg_len(gi);
  uint8_t *buf = pool->get();
  if (!buf) return set_error(BFRS_E_NOMEM, "pinned segment buffer allocation failed");
  auto seg = std::make_shared<Seg>(pool, buf, len);
  const long long t_read = trace.on ? trace.ns() : 0;
  if (read_file_into(seg_path(gi), buf, pool->slot, 8) != (long long)len) return BFRS_OK;
  const long long t_gpu = trace.on ? trace.ns() : 0;
  struct Done {  // trace only
    bfrs_archive *a;
    size_t gi;
    long long t_read, t_gpu;
    ~Done() {
      if (!a->trace.on) return;
      const long long t_end = a->trace.ns();
      a->trace.clean_read_ns += t_gpu - t_read;
      a->trace.clean_gpu_ns += t_end - t_gpu;
      ++a->trace.cleans;
      a->trace.event("clean", gi, t_read, t_end);
    }
  } done{this, gi, t_read, t_gpu};
  std::string hex;
  int rc = lane_hash(buf, len, gi, &hex);
  if (rc) return rc;
  if (hex == expected_hash(gi)) {
    *ok = true;
    *out = std::move(seg);
  }
  return BFRS_OK;
}

int bfrs_archive::lane_hash(const uint8_t *buf, size_t len, size_t key, std::string *hex) {
  CleanLane *ln = nullptr;
  std::unique_lock<std::mutex> lane_lock = take_lane(key, &ln);
  Context &c = ctx->impl;
  HIP_TRY(hipSetDevice(c.device));  // before the lane's HBM: a prefetch thread starts on device 0
  int rc = ln->ready(pool->slot);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(ln->d, buf, len, hipMemcpyHostToDevice, ln->st));
  HIP_TRY(hipStreamSynchronize(ln->st));  // before the hash takes hash_mu
  std::vector<std::string> h;
  if ((rc = gpu_hash_hex(ctx, {ln->d}, {len}, &h, nullptr, nullptr, ln->st))) return rc;
  *hex = h[0];
  return BFRS_OK;
}

int bfrs_archive::verify_file(const std::string &path, const std::string &want_hex, bool *ok) {
  *ok = false;
  uint8_t *buf = pool->get();
  if (!buf) return set_error(BFRS_E_NOMEM, "pinned segment buffer allocation failed");
  Seg hold(pool, buf, 0);  // back to the pool on every exit
  const long long n = read_file_into(path, buf, pool->slot, 8);
  if (n < 0) return BFRS_OK;  // missing, unreadable or longer than any shard here
  std::string hex;
  int rc = lane_hash(buf, size_t(n), 0, &hex);
  if (rc) return rc;
  *ok = hex == want_hex;
  return BFRS_OK;
}

// Reconstructs segment gi (and, tier 3, every other damaged segment of its
// block, which is cached too).
int bfrs_archive::recover(size_t gi, SegPtr *out) {
  const Manifest &mf = g.mf;
  if (mf.tier == 3) {
    std::vector<std::pair<size_t, SegPtr>> restored;
    {
      StagingCache &sc = staging(ctx);
      BlockArena &arena = sc.read_blk;
      const long long t_lock = trace.on ? trace.ns() : 0;
      std::lock_guard<std::mutex> lg(sc.read_mu);
      const long long t_gpu = trace.on ? trace.ns() : 0;
      if (trace.on) trace.gpu_lock_wait_ns += t_gpu - t_lock;
      {  // another thread's reconstruction of this block may have restored it meanwhile
        std::lock_guard<std::mutex> l(mu);
        if (SegPtr c = lookup(gi)) {
          *out = c;
          return BFRS_OK;
        }
      }
      const size_t b = gi / kBlockSegments;
      BlockState bs;
      int rc = load_block(ctx, g, b, arena, &bs);
      if (rc) return rc;
      const long long t_loaded = trace.on ? trace.ns() : 0;
      const std::vector<uint8_t> was_ok = bs.seg_ok;
      // the restored segments go from HBM straight into their cache buffers
      std::vector<uint8_t *> dst(bs.k, nullptr);
      for (size_t s = 0; s < bs.k; ++s) {
        const bool need = !was_ok[s] || b * kBlockSegments + s == gi;
        if (!need) continue;
        uint8_t *buf = pool->get();
        if (!buf) return set_error(BFRS_E_NOMEM, "pinned segment buffer allocation failed");
        // owned by a Seg before anything can fail, so every path returns it to the pool
        restored.emplace_back(b * kBlockSegments + s, std::make_shared<Seg>(pool, buf, bs.lens[s]));
        dst[s] = buf;
      }
      rc = restore_block(ctx, g, arena, bs, &dst);
      if (rc < 0) return rc;
      const long long t_restored = trace.on ? trace.ns() : 0;
      for (auto &r : restored) {
        const size_t s = r.first - b * kBlockSegments;
        if (was_ok[s]) {  // the target itself was clean (another reader's view was stale)
          HIP_TRY(hipMemcpy(r.second->p, arena.dev.ds(s), bs.lens[s], hipMemcpyDeviceToHost));
        } else if (write_back && !write_file(t3_seg(g.dir, b, s), r.second->p, bs.lens[s])) {
          return io_error("write back segment");
        }
      }
      if (trace.on) {
        const long long t_end = trace.ns();
        trace.rec_load_ns += t_loaded - t_gpu;
        trace.rec_restore_ns += t_restored - t_loaded;
        trace.rec_copy_ns += t_end - t_restored;
        trace.event("recover", gi, t_gpu, t_end);
      }
      std::lock_guard<std::mutex> l(mu);
      ++st.recoveries;
      for (size_t s = 0; s < bs.k; ++s) st.recovered_segments += !was_ok[s];
      for (auto &r : restored)
        if (r.first != gi) put(r.first, r.second);
    }
    for (auto &r : restored)
      if (r.first == gi) *out = r.second;
    return *out ? BFRS_OK : set_error(BFRS_E_WRAPPER, "segment not restored");
  }
  std::vector<uint8_t> v;
  int rc;
  if (mf.tier == 2) {
    const auto &sh = mf.segments.at(int64_t(gi));
    std::vector<std::string> paths;
    for (size_t p = 0; p < kParity; ++p) paths.push_back(t2_par(g.dir, gi, p));
    std::lock_guard<std::mutex> lg(gpu_mu);
    rc = recover_rs13(ctx, paths, sh.parity, g.seg_len(gi), sh.data, &v);
  } else {
    if (mf.leaves.size() < 4) return set_error(BFRS_E_WRAPPER, "tier-1 manifest needs 4 leaves");
    std::vector<std::string> paths, hashes;
    for (size_t p = 0; p < kParity; ++p) {
      paths.push_back(g.dir + "/parity_" + std::to_string(p) + ".dat");
      hashes.push_back(mf.leaves.at(int64_t(p + 1)));
    }
    std::lock_guard<std::mutex> lg(gpu_mu);
    rc = recover_rs13(ctx, paths, hashes, size_t(mf.size), mf.leaves.at(0), &v);
  }
  if (rc) return rc;
  if (write_back && !write_file(seg_path(gi), v.data(), v.size())) return io_error("write back segment");
  uint8_t *buf = pool->get();
  if (!buf) return set_error(BFRS_E_NOMEM, "pinned segment buffer allocation failed");
  auto seg = std::make_shared<Seg>(pool, buf, v.size());
  std::memcpy(buf, v.data(), v.size());
  *out = std::move(seg);
  std::lock_guard<std::mutex> l(mu);
  ++st.recoveries;
  ++st.recovered_segments;
  return BFRS_OK;
}

void bfrs_archive::prepin() {
  if (hipSetDevice(ctx->impl.device) != hipSuccess) return;
  if (g.mf.tier == 3) {
    // the context's read arena (~1.1 GiB HBM + 22 pinned slots at 32 MiB
    // segments), reserved here -- once per context, by its first tier-3
    // handle -- rather than when the first damaged block is found and the
    // reader is about to need it; a failure is left to that reconstruction
    StagingCache &sc = staging(ctx);
    std::lock_guard<std::mutex> lg(sc.read_mu);
    (void)sc.read_blk.reserve(pool->slot);
  }
  // then the segment pool, up to the buffers this handle's cache, prefetch
  // and readers hold at once (a pool another handle filled is left as is);
  // pinning runs ~22 GB/s (pinned_alloc), ahead of a ~15 GB/s reader
  const size_t want = std::min(g.nseg, cap + prefetch_workers + 2);
  while (!stop_pin && pool->size() < want)
    if (!pool->grow()) return;
}

void bfrs_archive::prefetch_loop(size_t) {
  std::unique_lock<std::mutex> l(mu);
  for (;;) {
    cv.wait(l, [&] { return stop || !wantq.empty(); });
    if (stop) return;
    const size_t gi = wantq.front();
    wantq.pop_front();
    if (cache.count(gi) || inflight.count(gi)) continue;
    // damaged: reconstructed (with its block's siblings) ahead of the reader;
    // a failure is left to the reader, which loads the segment itself
    SegPtr seg;
    bool ok = false, restored = false;
    const int rc = load_inflight(l, gi, &seg, &ok, &restored);
    if (rc == BFRS_OK && (ok || restored)) {
      put(gi, seg);
      st.verified += ok;
      ++st.prefetched;
    }
  }
}

extern "C" {

int bfrs_blake3_hex(const uint8_t *data, size_t len, int threads, char *out65) {
  BFRS_API_BEGIN
  if ((!data && len) || !out65) return set_error(BFRS_E_INVALID_ARGUMENT, "blake3: NULL argument");
  const std::string h = blake3_hex(data, len, threads);
  std::memcpy(out65, h.c_str(), 65);
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_merkle_root_hex(const char *leaves, size_t n, char *out65) {
  BFRS_API_BEGIN
  if (!leaves || !out65 || n == 0) return set_error(BFRS_E_INVALID_ARGUMENT, "merkle: bad argument");
  std::vector<std::string> v;
  for (size_t i = 0; i < n; ++i) v.emplace_back(leaves + 64 * i, 64);
  const std::string r = merkle_root_hex(v);
  std::memcpy(out65, r.c_str(), 65);
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_manifest_check(const char *text, size_t len, int *valid, char *canonical, size_t cap,
                        size_t *needed) {
  BFRS_API_BEGIN
  if (!text || !valid) return set_error(BFRS_E_INVALID_ARGUMENT, "manifest_check: NULL argument");
  Manifest mf;
  std::string err;
  if (!Manifest::from_json(std::string(text, len), &mf, &err)) return set_error(BFRS_E_WRAPPER, err);
  auto hex64 = [](const std::string &h) {
    return h.size() == 64 &&
           std::all_of(h.begin(), h.end(), [](char c) { return std::isxdigit(uint8_t(c)) != 0; });
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
  BFRS_API_END
}

}  // extern "C"

namespace {
int commit_impl(const std::vector<bfrs_ctx *> &ctxs, const char *file_path,
                const char *archive_root, size_t segment_size, int tier, char *out_dir,
                size_t out_cap) {
  if (ctxs.empty() || !file_path || !archive_root)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_commit: NULL argument");
  for (bfrs_ctx *c : ctxs)
    if (!c) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_commit: NULL context");
  Commit c{ctxs[0], archive_root, basename_of(file_path),
           segment_size ? segment_size : kDefaultSegment, ctxs};
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
  if (rc) {  // no half-written archive: drop this call's work directory
    const std::string computing = c.root + "/" + c.name + "_computing";
    struct stat cs;
    if (tier != 1 && stat(computing.c_str(), &cs) == 0) (void)rmtree(computing);
    return rc;
  }
  if (out_dir && out_cap) {
    std::strncpy(out_dir, dir.c_str(), out_cap - 1);
    out_dir[out_cap - 1] = 0;
  }
  return BFRS_OK;
}
}  // namespace

extern "C" {

int bfrs_commit(bfrs_ctx *ctx, const char *file_path, const char *archive_root,
                size_t segment_size, int tier, char *out_dir, size_t out_cap) {
  BFRS_API_BEGIN
  return commit_impl({ctx}, file_path, archive_root, segment_size, tier, out_dir, out_cap);
  BFRS_API_END
}

int bfrs_commit_multi(bfrs_ctx *const *ctxs, size_t n_ctx, const char *file_path,
                      const char *archive_root, size_t segment_size, int tier, char *out_dir,
                      size_t out_cap) {
  BFRS_API_BEGIN
  if (!ctxs || n_ctx == 0) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_commit_multi: no contexts");
  return commit_impl(std::vector<bfrs_ctx *>(ctxs, ctxs + n_ctx), file_path, archive_root,
                     segment_size, tier, out_dir, out_cap);
  BFRS_API_END
}

}  // extern "C"

namespace {
// Runs body(block state) over the tier-3 blocks `blocks` in order, reading
// block i + 1 through the ring into the other device buffer (sc.blk.dev /
// sc.blk2) while block i is verified and handled.  Under sc.mu, on the
// context's device.  `stop` (may be NULL) ends the loop before a block.
template <class Body>
int for_each_block(bfrs_ctx *ctx, const Geometry &g, StagingCache &sc,
                   const std::vector<size_t> &blocks, PipeTrace &pt,
                   const std::atomic<bool> *stop, Body body) {
  if (blocks.empty()) return BFRS_OK;
  BlockArena &a = sc.blk;
  // sized for the largest block up front: the reader thread must not regrow
  // buffers the verify and the body are using
  size_t shard = 0;
  for (size_t b : blocks) shard = std::max(shard, g.block_shard(b));
  int rc = a.reserve(shard);
  if (!rc) rc = sc.blk2.reserve(shard, kBlockSegments + kParity, kArenaDevice);
  if (!rc) rc = sc.commit_events();  // the two end-of-block markers
  if (rc) return rc;
  Arena *dev[2] = {&a.dev, &sc.blk2};
  BlockState st[2];
  struct RingSync {  // on every exit nothing of this call still copies into the buffers
    BlockArena &a;
    ~RingSync() {
      if (a.h2d) (void)hipStreamSynchronize(a.h2d);
    }
  } ring_sync{a};
  auto reads = [&](size_t i) {
    return load_block_reads(ctx, g, blocks[i], a, *dev[i % 2], sc.filled[i % 2], &st[i % 2], &pt);
  };
  if ((rc = reads(0))) return rc;
  for (size_t i = 0; i < blocks.size(); ++i) {
    if (stop && stop->load(std::memory_order_relaxed)) break;
    int next_rc = BFRS_OK;
    std::string next_err;
    {
      BgTask reader;
      if (i + 1 < blocks.size())
        reader.start([&, i] {
          next_rc = reads(i + 1);
          if (next_rc) next_err = bfrs_last_error();  // thread-local: carried back
        });
      rc = load_block_verify(ctx, g, &st[i % 2], sc.filled[i % 2], &pt);
      if (!rc) rc = body(st[i % 2]);
      reader.join();
    }
    if (rc) return rc;
    if (next_rc) return set_error(next_rc, next_err);
  }
  return BFRS_OK;
}

// repair_blocked (health.rs:642-765), intended semantics, over the blocks
// `mine` of a tier-3 archive on one context; counts land in *rep.
// `stop`: set when another context's repair failed (repair_tier3); the
// loop ends before its next block, so a failing call writes no more files
// than the blocks already in progress.
int repair_blocks(bfrs_ctx *ctx, const Geometry &g, const std::vector<size_t> &mine,
                  bfrs_repair_report *rep, const std::atomic<bool> *stop = nullptr) {
  if (hipSetDevice(ctx->impl.device) != hipSuccess)
    return set_error(BFRS_E_HIP, "repair: hipSetDevice failed");
  StagingCache &sc = staging(ctx);
  std::lock_guard<std::mutex> staging_lock(sc.mu);
  BlockArena &a = sc.blk;
  PipeTrace pt;
  struct Print {  // the timeline on every exit (measurement build)
    PipeTrace &pt;
    ~Print() { pt.print("bfrs_repair_trace", hw_threads()); }
  } print{pt};
  // a block's restored segments are written (from the arena's out slots
  // [0, 3)) while the next block loads; joined before the next restore
  // reuses those slots, and on every exit path
  std::atomic<bool> write_ok{true};
  std::atomic<size_t> written{0};
  BgTask writer;
  auto finish_writes = [&]() -> int {
    writer.join();
    return write_ok ? BFRS_OK : io_error("write restored segment");
  };
  int rc = for_each_block(ctx, g, sc, mine, pt, stop, [&](BlockState &bs) -> int {
    const size_t b = bs.b;
    const long long t0 = pt.on ? pt.now_us() : 0;
    ++rep->blocks_checked;
    rep->segments_checked += bs.k;
    const size_t parity_bad = kParity - bs.valid_parity();
    int rc = finish_writes();
    if (rc) return rc;
    const int restored = restore_block(ctx, g, a, bs);
    if (restored == BFRS_E_NOT_ENOUGH_SHARDS) {
      ++rep->unrecoverable_blocks;
      return BFRS_OK;
    }
    if (restored < 0) return restored;
    pt.event("restore", b, t0);
    // exactly the segments that were damaged, one file per thread
    writer.start([&, b, files = bs.restored, lens = bs.lens] {
      const long long t1 = pt.on ? pt.now_us() : 0;
      parallel_for(files.size(), int(files.size()), [&](size_t j) {
        const size_t s = files[j].first;
        if (write_file(t3_seg(g.dir, b, s), files[j].second, lens[s]))
          ++written;
        else
          write_ok = false;
      });
      pt.event("write", b, t1);
    });
    if (parity_bad) {
      const std::vector<uint8_t> par_was = bs.par_ok;
      if ((rc = reencode_parity(ctx, g, a, bs))) return rc;
      for (size_t p = 0; p < kParity; ++p)
        if (!par_was[p] && !write_file(t3_par(g.dir, b, p), bs.parity_host[p], bs.shard))
          return io_error("write parity");
      rep->parity_repaired += parity_bad;
    }
    return BFRS_OK;
  });
  const int wrc = finish_writes();
  rep->segments_repaired += written;
  return rc ? rc : wrc;
}

// Tier-3 blocks dealt round-robin over the contexts (block b to context
// b % n), each context on a host thread of its own; reports summed.
int repair_tier3(const std::vector<bfrs_ctx *> &ctxs, const Geometry &g, bfrs_repair_report *report) {
  std::vector<size_t> blocks;
  for (const auto &kv : g.mf.blocks) blocks.push_back(size_t(kv.first));
  const size_t n = std::max<size_t>(1, std::min(ctxs.size(), blocks.size()));
  std::vector<std::vector<size_t>> mine(n);
  for (size_t i = 0; i < blocks.size(); ++i) mine[i % n].push_back(blocks[i]);
  std::vector<bfrs_repair_report> reps(n, bfrs_repair_report{});
  std::vector<int> rcs(n, BFRS_OK);
  std::vector<std::string> errs(n);
  std::atomic<bool> stop{false};  // a failed context stops the others' next block
  auto run = [&](size_t d) {
    try {
      rcs[d] = repair_blocks(ctxs[d], g, mine[d], &reps[d], &stop);
    } catch (const std::bad_alloc &) {
      rcs[d] = set_error(BFRS_E_NOMEM, "host memory allocation failed");
    } catch (const std::exception &e) {
      rcs[d] = set_error(BFRS_E_WRAPPER, std::string("internal error: ") + e.what());
    }
    if (rcs[d]) {
      errs[d] = bfrs_last_error();
      stop = true;
    }
  };
  {
    std::vector<BgTask> others(n - 1);  // joined on every exit path
    for (size_t d = 1; d < n; ++d) others[d - 1].start([&run, d] { run(d); });
    run(0);
    for (auto &t : others) t.join();
  }
  for (const auto &r : reps) {
    report->blocks_checked += r.blocks_checked;
    report->segments_checked += r.segments_checked;
    report->segments_repaired += r.segments_repaired;
    report->parity_repaired += r.parity_repaired;
    report->unrecoverable_blocks += r.unrecoverable_blocks;
  }
  for (size_t d = 0; d < n; ++d)
    if (rcs[d]) return set_error(rcs[d], n == 1 ? errs[d] : "context " + std::to_string(d) + ": " + errs[d]);
  return BFRS_OK;
}

int repair_impl(const std::vector<bfrs_ctx *> &ctxs, const char *archive_dir,
                bfrs_repair_report *report) {
  if (ctxs.empty() || !archive_dir || !report)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_repair: NULL argument");
  for (bfrs_ctx *c : ctxs)
    if (!c) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_repair: NULL context");
  bfrs_ctx *ctx = ctxs[0];
  *report = bfrs_repair_report{};
  Geometry g;
  int rc = load_geometry(archive_dir, &g);
  if (rc) return rc;
  if (g.mf.tier == 3) return repair_tier3(ctxs, g, report);
  // tiers 1/2 (repair_tiny :497, repair_segment :542): per-segment RS(1,3).
  // The reference restores only the data; with the intended semantics, as
  // for tier 3, a damaged parity copy is re-encoded from the verified data
  // (RS(1,3) through the codec) and checked against the manifest too.
  bfrs_archive a;
  a.ctx = ctx;
  a.g = g;
  a.write_back = true;
  a.pool = segment_pool(ctx, g.S);
  for (size_t i = 0; i < g.nseg; ++i) {
    ++report->segments_checked;
    ++report->blocks_checked;
    SegPtr v;
    bool ok = false;
    if ((rc = a.load_clean(i, &v, &ok))) return rc;
    if (!ok) {
      rc = a.recover(i, &v);
      if (rc == BFRS_E_NOT_ENOUGH_SHARDS) {
        ++report->unrecoverable_blocks;
        continue;
      }
      if (rc) return rc;
      ++report->segments_repaired;
    }
    std::vector<std::string> ppath, phash;
    for (size_t p = 0; p < kParity; ++p) {
      ppath.push_back(g.mf.tier == 2 ? t2_par(g.dir, i, p)
                                     : g.dir + "/parity_" + std::to_string(p) + ".dat");
      phash.push_back(g.mf.tier == 2 ? g.mf.segments.at(int64_t(i)).parity[p]
                                     : g.mf.leaves.at(int64_t(p + 1)));
    }
    std::vector<size_t> bad;
    for (size_t p = 0; p < kParity; ++p) {  // device BLAKE3 on the lanes, as the data
      bool valid = false;
      if ((rc = a.verify_file(ppath[p], phash[p], &valid))) return rc;
      if (!valid) bad.push_back(p);
    }
    if (bad.empty()) continue;
    const size_t shard = (v->n + 63) / 64 * 64;  // generate.rs:34: padded to 64
    std::vector<uint8_t> padded(shard, 0);
    std::memcpy(padded.data(), v->p, v->n);
    std::vector<std::vector<uint8_t>> par(kParity, std::vector<uint8_t>(shard));
    const uint8_t *orig[1] = {padded.data()};
    uint8_t *outp[kParity];
    for (size_t p = 0; p < kParity; ++p) outp[p] = par[p].data();
    const uint32_t k1 = 1;
    if ((rc = bfrs_encode_host_batch(ctx, 1, &k1, kParity, shard, orig, outp))) return rc;
    for (size_t p : bad) {
      if (blake3_hex(par[p].data(), shard, hw_threads()) != phash[p])
        return set_error(BFRS_E_WRAPPER, "re-encoded parity fails the manifest hash");
      if (!write_file(ppath[p], par[p].data(), shard)) return io_error("write parity");
      ++report->parity_repaired;
    }
  }
  return BFRS_OK;
}
}  // namespace

extern "C" {

int bfrs_repair(bfrs_ctx *ctx, const char *archive_dir, bfrs_repair_report *report) {
  BFRS_API_BEGIN
  return repair_impl({ctx}, archive_dir, report);
  BFRS_API_END
}

int bfrs_repair_multi(bfrs_ctx *const *ctxs, size_t n_ctx, const char *archive_dir,
                      bfrs_repair_report *report) {
  BFRS_API_BEGIN
  if (!ctxs || n_ctx == 0) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_repair_multi: no contexts");
  return repair_impl(std::vector<bfrs_ctx *>(ctxs, ctxs + n_ctx), archive_dir, report);
  BFRS_API_END
}

// FileStore::health_check (src/filestore/health.rs:111-438) with intended
// semantics: every shard is verified against the manifest hash (tier 3 on the
// GPU), so corruption counts like absence, and a block whose data is whole
// but whose parity is not is Degraded (the reference tier-3 check only tests
// existence, :363-411).  Report: JSON with HealthReport's fields
// (src/filestore/models.rs:67-82) plus per-tier counts.
}  // extern "C"

namespace {
int health_report(bfrs_ctx *ctx, const char *archive_dir, Json *out) {
  Geometry g;
  int rc = load_geometry(archive_dir, &g);
  if (rc) return rc;
  enum { kHealthy, kDegraded, kRecoverable, kUnrecoverable };
  Json missing_data = Json::arr(), missing_parity = Json::arr(), corrupt_segments = Json::arr(),
       corrupt_parity = Json::arr();
  size_t units = 0, healthy = 0, degraded = 0, recoverable = 0, unrecoverable = 0;
  auto exists = [](const std::string &p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0;
  };
  auto classify = [&](size_t damaged, size_t par_ok) {
    ++units;
    if (damaged == 0 && par_ok == kParity) ++healthy;
    else if (damaged == 0) ++degraded;
    else if (damaged <= par_ok) ++recoverable;
    else ++unrecoverable;
  };
  if (g.mf.tier == 3) {
    HIP_TRY(hipSetDevice(ctx->impl.device));
    StagingCache &sc = staging(ctx);
    std::lock_guard<std::mutex> staging_lock(sc.mu);
    PipeTrace pt;
    struct Print {  // the timeline on every exit (measurement build)
      PipeTrace &pt;
      ~Print() { pt.print("bfrs_health_trace", hw_threads()); }
    } print{pt};
    std::vector<size_t> blocks;
    for (const auto &kv : g.mf.blocks) blocks.push_back(size_t(kv.first));
    rc = for_each_block(ctx, g, sc, blocks, pt, nullptr, [&](BlockState &bs) -> int {
      const size_t b = bs.b;
      const std::string bn = "block_" + std::to_string(b);
      for (size_t s = 0; s < bs.k; ++s)
        if (!bs.seg_ok[s]) {
          const std::string n = bn + "/segment_" + std::to_string(s) + ".dat";
          (exists(t3_seg(g.dir, b, s)) ? corrupt_segments : missing_data).a.push_back(Json::str(n));
        }
      for (size_t p = 0; p < kParity; ++p)
        if (!bs.par_ok[p]) {
          const std::string n = bn + "/block_parity_" + std::to_string(p) + ".dat";
          (exists(t3_par(g.dir, b, p)) ? corrupt_parity : missing_parity).a.push_back(Json::str(n));
        }
      classify(bs.damaged_segments(), bs.valid_parity());
      return BFRS_OK;
    });
    if (rc) return rc;
  } else {
    bfrs_archive ar;
    ar.ctx = ctx;
    ar.g = g;
    ar.pool = segment_pool(ctx, g.S);
    for (size_t i = 0; i < g.nseg; ++i) {
      SegPtr v;
      bool ok = false;
      if ((rc = ar.load_clean(i, &v, &ok))) return rc;
      const std::string dn = g.mf.tier == 1 ? "data.dat" : "segment_" + std::to_string(i) + ".dat";
      if (!ok) (exists(ar.seg_path(i)) ? corrupt_segments : missing_data).a.push_back(Json::str(dn));
      size_t par_ok = 0;
      for (size_t p = 0; p < kParity; ++p) {
        const std::string path = g.mf.tier == 1 ? g.dir + "/parity_" + std::to_string(p) + ".dat"
                                                : t2_par(g.dir, i, p);
        const std::string want = g.mf.tier == 1 ? g.mf.leaves.count(int64_t(p + 1)) ? g.mf.leaves.at(int64_t(p + 1)) : ""
                                                : g.mf.segments.at(int64_t(i)).parity.at(p);
        bool valid = false;
        if ((rc = ar.verify_file(path, want, &valid))) return rc;
        if (valid) {
          ++par_ok;
        } else {
          const std::string pn = g.mf.tier == 1 ? "parity_" + std::to_string(p) + ".dat"
                                                : "segment_" + std::to_string(i) + "_parity_" + std::to_string(p) + ".dat";
          (exists(path) ? corrupt_parity : missing_parity).a.push_back(Json::str(pn));
        }
      }
      classify(ok ? 0 : 1, par_ok);
    }
  }
  const int status = healthy == units ? kHealthy
                     : unrecoverable ? kUnrecoverable
                     : recoverable   ? kRecoverable
                                     : kDegraded;
  static const char *kNames[] = {"Healthy", "Degraded", "Recoverable", "Unrecoverable"};
  Json r = Json::obj();
  r["status"] = Json::str(kNames[status]);
  Json rec;
  rec.kind = Json::kBool;
  rec.b = status != kUnrecoverable;
  r["recoverable"] = rec;
  r["missing_data"] = missing_data;
  r["missing_parity"] = missing_parity;
  r["corrupt_segments"] = corrupt_segments;
  r["corrupt_parity"] = corrupt_parity;
  r["tier"] = Json::num(g.mf.tier);
  r["units"] = Json::num(int64_t(units));
  r["healthy"] = Json::num(int64_t(healthy));
  r["degraded"] = Json::num(int64_t(degraded));
  r["recoverable_units"] = Json::num(int64_t(recoverable));
  r["unrecoverable_units"] = Json::num(int64_t(unrecoverable));
  std::ostringstream det;
  det << healthy << "/" << units << (g.mf.tier == 3 ? " blocks" : " segments") << " healthy, "
      << degraded << " degraded, " << recoverable << " recoverable, " << unrecoverable
      << " unrecoverable";
  r["details"] = Json::str(det.str());
  *out = std::move(r);
  return BFRS_OK;
}

// JSON text into a caller buffer: *needed = length + 1, truncated copy.
void put_json(const Json &j, char *json_out, size_t cap, size_t *needed) {
  const std::string js = j.dump();
  if (needed) *needed = js.size() + 1;
  if (json_out && cap) {
    const size_t n = std::min(cap - 1, js.size());
    std::memcpy(json_out, js.data(), n);
    json_out[n] = 0;
  }
}

// FileStore::all_files + get_all (src/filestore/mod.rs:81-112): every entry of
// the store root is taken as an archive directory whose manifest.json must
// parse (the reference fails the whole listing otherwise).  read_dir order is
// unspecified there; here entries are sorted by name.
struct StoreFile {
  std::string name, hash, manifest_path, dir;
};
int store_files(const char *root, std::vector<StoreFile> *out) {
  DIR *d = opendir(root);
  if (!d) return io_error(std::string("read_dir ") + root);
  std::vector<std::string> entries;
  while (const dirent *e = readdir(d)) {
    const std::string n = e->d_name;
    if (n != "." && n != "..") entries.push_back(n);
  }
  closedir(d);
  std::sort(entries.begin(), entries.end());
  for (const std::string &n : entries) {
    StoreFile f;
    f.dir = std::string(root) + "/" + n;
    f.manifest_path = f.dir + "/manifest.json";
    std::vector<uint8_t> text;
    if (!read_file(f.manifest_path, &text)) return io_error("read manifest " + f.manifest_path);
    Manifest mf;
    std::string err;
    if (!Manifest::from_json(std::string(text.begin(), text.end()), &mf, &err))
      return set_error(BFRS_E_WRAPPER, f.manifest_path + ": " + err);
    f.name = mf.name;
    f.hash = mf.original_hash;
    out->push_back(std::move(f));
  }
  return BFRS_OK;
}

Json file_json(const StoreFile &f) {
  Json j = Json::obj(), data = Json::obj();
  j["file_name"] = Json::str(f.name);
  data["hash"] = Json::str(f.hash);
  data["path"] = Json::str(f.manifest_path);
  j["file_data"] = data;
  j["dir"] = Json::str(f.dir);
  return j;
}
}  // namespace

extern "C" {

int bfrs_health_check(bfrs_ctx *ctx, const char *archive_dir, char *json_out, size_t cap,
                      size_t *needed) {
  BFRS_API_BEGIN
  if (!ctx || !archive_dir) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_health_check: NULL argument");
  Json r;
  int rc = health_report(ctx, archive_dir, &r);
  if (rc) return rc;
  put_json(r, json_out, cap, needed);
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_store_list(const char *store_root, char *json_out, size_t cap, size_t *needed) {
  BFRS_API_BEGIN
  if (!store_root) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_store_list: NULL argument");
  std::vector<StoreFile> files;
  int rc = store_files(store_root, &files);
  if (rc) return rc;
  Json a = Json::arr();
  for (const StoreFile &f : files) a.a.push_back(file_json(f));
  put_json(a, json_out, cap, needed);
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_store_find(const char *store_root, const char *file_name, char *dir_out, size_t cap,
                    size_t *needed) {
  BFRS_API_BEGIN
  if (!store_root || !file_name)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_store_find: NULL argument");
  std::vector<StoreFile> files;
  int rc = store_files(store_root, &files);
  if (rc) return rc;
  for (const StoreFile &f : files)
    if (f.name == file_name) {  // first match, as FileStore::find (mod.rs:137-146)
      if (needed) *needed = f.dir.size() + 1;
      if (dir_out && cap) {
        const size_t n = std::min(cap - 1, f.dir.size());
        std::memcpy(dir_out, f.dir.data(), n);
        dir_out[n] = 0;
      }
      return BFRS_OK;
    }
  return set_error(BFRS_E_NOT_FOUND, std::string("File '") + file_name + "' not found");  // mod.rs:150-153
  BFRS_API_END
}

int bfrs_batch_health_check(bfrs_ctx *ctx, const char *store_root, char *json_out, size_t cap,
                            size_t *needed) {
  BFRS_API_BEGIN
  if (!ctx || !store_root)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_batch_health_check: NULL argument");
  std::vector<StoreFile> files;
  int rc = store_files(store_root, &files);
  if (rc) return rc;
  int64_t counts[4] = {0, 0, 0, 0};
  static const char *kNames[] = {"Healthy", "Degraded", "Recoverable", "Unrecoverable"};
  Json reports = Json::arr();
  for (const StoreFile &f : files) {
    Json r;
    if ((rc = health_report(ctx, f.dir.c_str(), &r))) return rc;  // `?` in health.rs:53
    const Json *st = r.get("status");
    for (int i = 0; i < 4; ++i)
      if (st && st->s == kNames[i]) ++counts[i];
    Json pair = Json::arr();  // (String, HealthReport) serialises as a 2-array
    pair.a.push_back(Json::str(f.name));
    pair.a.push_back(std::move(r));
    reports.a.push_back(std::move(pair));
  }
  Json b = Json::obj();
  b["total_files"] = Json::num(int64_t(files.size()));
  b["healthy"] = Json::num(counts[0]);
  b["degraded"] = Json::num(counts[1]);
  b["recoverable"] = Json::num(counts[2]);
  b["unrecoverable"] = Json::num(counts[3]);
  b["reports"] = std::move(reports);
  put_json(b, json_out, cap, needed);
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_archive_open(bfrs_ctx *ctx, const char *archive_dir, size_t cache_segments,
                      int write_back, bfrs_archive **out) {
  BFRS_API_BEGIN
  if (!ctx || !archive_dir || !out)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_archive_open: NULL argument");
  *out = nullptr;
  std::unique_ptr<bfrs_archive> a(new (std::nothrow) bfrs_archive);
  if (!a) return set_error(BFRS_E_NOMEM, "archive allocation failed");
  a->ctx = ctx;
  a->cap = std::max<size_t>(1, cache_segments);
  a->write_back = write_back != 0;
  int rc = load_geometry(archive_dir, &a->g);
  if (rc) return rc;
  a->pool = segment_pool(ctx, a->g.S);
  a->trace.on = BFRS_AB_KNOB("BFRS_TRACE") != nullptr;
  if (const char *e = std::getenv("BFRS_PREFETCH_DEPTH"))
    a->prefetch_depth = size_t(std::clamp(std::strtol(e, nullptr, 10), 1L, 256L));
  if (const char *e = BFRS_AB_KNOB("BFRS_PREFETCH_WORKERS"))
    a->prefetch_workers = size_t(std::clamp(std::strtol(e, nullptr, 10), 1L, 16L));
  a->prefetch = a->g.nseg > 1;
  if (a->prefetch) a->add_lanes(a->prefetch_workers);  // one per worker + the reader's
  {
    std::lock_guard<std::mutex> l(ctx->impl.handles_mu);
    ctx->impl.handles.push_back(a.get());  // from here on the destructor unregisters it
  }
  if (a->prefetch) {
    try {
      for (size_t w = 0; w < a->prefetch_workers; ++w)
        a->workers.emplace_back(&bfrs_archive::prefetch_loop, a.get(), w);
    } catch (const std::system_error &) {  // no thread: fewer prefetch workers, or none
    }
    a->prefetch = !a->workers.empty();
    if (a->prefetch) {
      bfrs_archive *h = a.get();
      try {
        h->pinner.start([h] { h->prepin(); });
      } catch (...) {  // start() runs the task inline if no thread can be made
      }
    }
  }
  *out = a.release();
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_archive_size(bfrs_archive *a, uint64_t *size) {
  BFRS_API_BEGIN
  if (!a || !size) return set_error(BFRS_E_INVALID_ARGUMENT, "NULL argument");
  *size = uint64_t(a->g.mf.size);
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_archive_stat(const char *archive_dir, bfrs_archive_attr *out) {
  BFRS_API_BEGIN
  if (!archive_dir || !out) return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_archive_stat: NULL argument");
  Geometry g;
  int rc = load_geometry(archive_dir, &g);
  if (rc) return rc;
  *out = bfrs_archive_attr{};
  out->size = uint64_t(g.mf.size);
  out->segment_size = g.mf.tier == 1 ? g.mf.segment_size : g.S;
  out->segments = g.nseg;
  out->blocks = g.mf.tier == 3 ? (g.nseg + kBlockSegments - 1) / kBlockSegments : 0;
  out->tier = g.mf.tier;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_archive_read(bfrs_archive *a, uint64_t offset, size_t len, uint8_t *out, size_t *nread) {
  BFRS_API_BEGIN
  if (!a || (!out && len) || !nread) return set_error(BFRS_E_INVALID_ARGUMENT, "NULL argument");
  *nread = 0;
  if (!a->ctx)
    return set_error(BFRS_E_INVALID_ARGUMENT, "bfrs_archive_read: the handle's context was closed");
  const uint64_t size = uint64_t(a->g.mf.size);
  if (offset >= size) return BFRS_OK;
  len = size_t(std::min<uint64_t>(len, size - offset));
  const uint64_t S = a->g.S;
  std::unique_lock<std::mutex> l(a->mu);
  while (*nread < len) {
    const uint64_t pos = offset + *nread;
    const size_t gi = size_t(pos / S);
    const size_t in_seg = size_t(pos % S);  // filesystem_unix.rs:216 uses '&' (bug)
    SegPtr seg = a->lookup(gi);
    if (seg) {
      ++a->st.hits;
    } else if (a->inflight.count(gi)) {  // a prefetch worker or another reader is loading it
      const long long t = a->trace.on ? a->trace.ns() : 0;
      a->cv.wait(l, [&] { return !a->inflight.count(gi); });
      if (a->trace.on) {
        const long long e = a->trace.ns();
        a->trace.reader_wait_ns += e - t;
        ++a->trace.reader_waits;
        a->trace.event("reader_wait", gi, t, e);
      }
      continue;
    } else {
      ++a->st.misses;
      // queued but not started: load it here instead
      a->wantq.erase(std::remove(a->wantq.begin(), a->wantq.end(), gi), a->wantq.end());
      bool ok = false, restored = false;
      const long long t = a->trace.on ? a->trace.ns() : 0;
      const int rc = a->load_inflight(l, gi, &seg, &ok, &restored);
      if (a->trace.on) {
        const long long e = a->trace.ns();
        a->trace.reader_miss_ns += e - t;
        a->trace.event("reader_miss", gi, t, e);
      }
      if (rc) return rc;
      if (ok) ++a->st.verified;
      a->put(gi, seg);
    }
    if (a->prefetch && (long long)gi != a->last_gi) {  // moved to a new segment
      a->last_gi = (long long)gi;
      // the next segments, at most half the cache so they are not evicted unread
      const size_t depth = std::min(a->prefetch_depth, std::max<size_t>(1, a->cap / 2));
      bool queued = false;
      for (size_t nx = gi + 1; nx <= gi + depth && nx < a->g.nseg; ++nx)
        if (!a->cache.count(nx) && !a->inflight.count(nx) &&
            std::find(a->wantq.begin(), a->wantq.end(), nx) == a->wantq.end()) {
          a->wantq.push_back(nx);
          queued = true;
        }
      if (queued) a->cv.notify_all();
    }
    if (in_seg >= seg->n) return set_error(BFRS_E_WRAPPER, "segment shorter than manifest size");
    const size_t n = std::min(len - *nread, seg->n - in_seg);
    // the copy runs unlocked (seg keeps the buffer alive): a reader that held
    // mu through its copies starved the prefetch workers of it
    l.unlock();
    std::memcpy(out + *nread, seg->p + in_seg, n);
    l.lock();
    *nread += n;
  }
  a->st.bytes_served += *nread;
  return BFRS_OK;
  BFRS_API_END
}

int bfrs_archive_stats_get(bfrs_archive *a, bfrs_archive_stats *out) {
  BFRS_API_BEGIN
  if (!a || !out) return set_error(BFRS_E_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> g(a->mu);
  *out = a->st;
  return BFRS_OK;
  BFRS_API_END
}

void bfrs_archive_close(bfrs_archive *a) { delete a; }

}  // extern "C"

namespace bfrs {
void detach_archives(bfrs_ctx *ctx) {
  {
    std::lock_guard<std::mutex> l(ctx->impl.handles_mu);
    for (bfrs_archive *a : ctx->impl.handles) a->detach();
    ctx->impl.handles.clear();
  }
  // measurement build (BFRS_TRACE): the context's segment pools as bfrs_close
  // finds them, one stderr line (tests check the idle cap with it)
  if (BFRS_AB_KNOB("BFRS_TRACE") && ctx->impl.staging) {
    StagingCache &sc = staging(ctx);
    std::lock_guard<std::mutex> l(sc.pools_mu);
    std::ostringstream os;
    size_t idle = 0;
    os << "bfrs_pools {\"pools\":" << sc.seg_pools.size() << ",\"slots\":[";
    bool first = true;
    for (auto &e : sc.seg_pools) {
      auto *pp = static_cast<PinnedPool *>(e.second.get());
      idle += pp->idle_bytes();
      os << (first ? "" : ",") << pp->slot;
      first = false;
    }
    os << "],\"idle_bytes\":" << idle << ",\"idle_cap\":" << idle_pinned_cap() << "}\n";
    std::fputs(os.str().c_str(), stderr);
  }
}
}  // namespace bfrs
