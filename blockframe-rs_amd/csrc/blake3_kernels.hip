// blake3_kernels.hip — BLAKE3 of device-resident messages on gfx950.
//
// BlockFrame hashes every segment and parity shard with BLAKE3 at commit
// (src/chunker/commit.rs:429,451), the whole file (:478), and every segment
// again on each FUSE cache miss (src/mount/filesystem_unix.rs:238-246).  The
// reference does this on the CPU (blake3 1.8.2, src/utils.rs:22-28); here the
// shards are already in HBM for the RS kernels, so they are hashed there.
//
// Tree shape.  BLAKE3 splits a message into 1 KiB chunks and builds a
// left-complete binary tree (left subtree = largest power of two < n chunks).
// That tree is exactly what level-wise pairing gives when an odd last node is
// carried up unchanged, and pairing stays aligned inside any power-of-two
// aligned run of nodes.  So:
//   kernel 1 (blake3_group_kernel): one 256-lane workgroup per 256 KiB group;
//     lane t compresses chunk t (16 blocks, message words in VGPRs), then the
//     group's 256 chaining values are paired down in LDS to one CV.  A group
//     that is the whole message finalises it (ROOT on its last compression).
//   kernel 2 (blake3_reduce_kernel): pairs up to 1024 aligned CVs of one
//     message in LDS; the last job of a message finalises it.
// The final parent is compressed twice: with ROOT -> the message digest, and
// without -> the message's subtree CV, which is a node of any enclosing tree
// whose chunks it aligns with (a 32 MiB segment is level 15 of the file's
// tree), so the whole-file hash follows from the segment CVs.
//
// Roofline: compute.  One 64-byte block costs 7 rounds x 8 G functions x ~12
// VALU ops (v_add3, v_xor, v_alignbit rotates) ~ 690 ops, i.e. ~10.8 VALU ops
// per byte; no MFMA (32-bit add/xor/rotate has no matrix form).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hash_kernels.hpp"

namespace bfrs {
namespace {

enum : uint32_t { kStart = 1, kEnd = 2, kParent = 4, kRoot = 8 };

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

#define B3_G(a, b, c, d, x, y) \
  a = a + b + (x);             \
  d = rotr(d ^ a, 16);         \
  c = c + d;                   \
  b = rotr(b ^ c, 12);         \
  a = a + b + (y);             \
  d = rotr(d ^ a, 8);          \
  c = c + d;                   \
  b = rotr(b ^ c, 7);

// 7 rounds over state v with message m; m is permuted in registers between
// rounds (fully unrolled: the permutation is register renaming).
__device__ __forceinline__ void rounds(uint32_t v[16], uint32_t m[16]) {
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    B3_G(v[0], v[4], v[8], v[12], m[0], m[1]);
    B3_G(v[1], v[5], v[9], v[13], m[2], m[3]);
    B3_G(v[2], v[6], v[10], v[14], m[4], m[5]);
    B3_G(v[3], v[7], v[11], v[15], m[6], m[7]);
    B3_G(v[0], v[5], v[10], v[15], m[8], m[9]);
    B3_G(v[1], v[6], v[11], v[12], m[10], m[11]);
    B3_G(v[2], v[7], v[8], v[13], m[12], m[13]);
    B3_G(v[3], v[4], v[9], v[14], m[14], m[15]);
    if (r < 6) {
      const uint32_t t0 = m[2], t1 = m[6], t2 = m[3], t3 = m[10], t4 = m[7], t5 = m[0],
                     t6 = m[4], t7 = m[13], t8 = m[1], t9 = m[11], t10 = m[12], t11 = m[5],
                     t12 = m[9], t13 = m[14], t14 = m[15], t15 = m[8];
      m[0] = t0; m[1] = t1; m[2] = t2; m[3] = t3; m[4] = t4; m[5] = t5; m[6] = t6; m[7] = t7;
      m[8] = t8; m[9] = t9; m[10] = t10; m[11] = t11; m[12] = t12; m[13] = t13; m[14] = t14;
      m[15] = t15;
    }
  }
}

__device__ __forceinline__ void init_state(uint32_t v[16], const uint32_t cv[8], uint64_t counter,
                                           uint32_t len, uint32_t flags) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = cv[i];
  v[8] = 0x6A09E667u;
  v[9] = 0xBB67AE85u;
  v[10] = 0x3C6EF372u;
  v[11] = 0xA54FF53Au;
  v[12] = uint32_t(counter);
  v[13] = uint32_t(counter >> 32);
  v[14] = len;
  v[15] = flags;
}

// Chaining value (first 8 output words) of one compression; m is clobbered.
__device__ __forceinline__ void compress_cv(uint32_t cv[8], uint32_t m[16], uint64_t counter,
                                            uint32_t len, uint32_t flags) {
  uint32_t v[16];
  init_state(v, cv, counter, len, flags);
  rounds(v, m);
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = v[i] ^ v[i + 8];
}

__device__ __forceinline__ void set_iv(uint32_t cv[8]) {
  cv[0] = 0x6A09E667u; cv[1] = 0xBB67AE85u; cv[2] = 0x3C6EF372u; cv[3] = 0xA54FF53Au;
  cv[4] = 0x510E527Fu; cv[5] = 0x9B05688Cu; cv[6] = 0x1F83D9ABu; cv[7] = 0x5BE0CD19u;
}

// Final node: writes the non-root CV and the ROOT digest words.
__device__ __forceinline__ void finalize(const uint32_t cv_in[8], const uint32_t m_in[16],
                                         uint64_t counter, uint32_t len, uint32_t flags,
                                         uint32_t *msg_cv, uint32_t *digest) {
  uint32_t cv[8], m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = cv_in[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = m_in[i];
  compress_cv(cv, m, counter, len, flags);
#pragma unroll
  for (int i = 0; i < 8; ++i) msg_cv[i] = cv[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = cv_in[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = m_in[i];
  compress_cv(cv, m, counter, len, flags | kRoot);
#pragma unroll
  for (int i = 0; i < 8; ++i) digest[i] = cv[i];
}

// 64-byte block at p (little-endian words); bytes at or past `len` read as 0
// and are never touched.
__device__ __forceinline__ void load_block(const uint8_t *p, uint32_t len, uint32_t m[16]) {
  if (len == 64) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 w = q[i];
      m[4 * i] = w.x;
      m[4 * i + 1] = w.y;
      m[4 * i + 2] = w.z;
      m[4 * i + 3] = w.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint32_t w = 0;
      for (uint32_t b = 0; b < 4; ++b)
        if (4 * i + b < len) w |= uint32_t(p[4 * i + b]) << (8 * b);
      m[i] = w;
    }
  }
}

// Parent of two CVs held in LDS rows a, b -> (non-final) CV in r.
__device__ __forceinline__ void parent_cv(const uint32_t *a, const uint32_t *b, uint32_t r[8]) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = a[i];
    m[8 + i] = b[i];
  }
  set_iv(r);
  compress_cv(r, m, 0, 64, kParent);
}

__device__ __forceinline__ void parent_final(const uint32_t *a, const uint32_t *b, uint32_t *msg_cv,
                                             uint32_t *digest) {
  uint32_t m[16], iv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = a[i];
    m[8 + i] = b[i];
  }
  set_iv(iv);
  finalize(iv, m, 0, 64, kParent, msg_cv, digest);
}

constexpr int kRow = 9;  // LDS row stride in words (odd: spreads a row's reads over banks)

// ---- Quad-cooperative parent compression (the tree's narrow levels).
// A lone wave compressing alone is latency-bound: ~700 dependent VALU ops per
// compression, ~2.4 us each on the box, and the upper tree
// levels are a chain of such compressions.  Here the four lanes of a quad
// share one compression: lane q holds column q of the 4x4 state (v[q],
// v[4+q], v[8+q], v[12+q]) and applies G to it; for the diagonal step rows
// b, c, d rotate by 1, 2, 3 lanes inside the quad (DPP quad_perm), and back.
// ~4x fewer dependent ops per compression; the message words come from the
// children's LDS rows at lane-dependent offsets (left row, right row = left
// + kRow), per round through the permuted schedule below.
struct QuadSched {
  // off[r][k] byte q: LDS word offset (from the left child's row) of the
  // message word lane q uses in round r: k = 0, 1 column step (words 2q,
  // 2q+1 of the round's message), k = 2, 3 diagonal step (8+2q, 9+2q)
  uint32_t off[7][4];
};
constexpr QuadSched make_quad_sched() {
  constexpr uint8_t P[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
  QuadSched s{};
  uint8_t S[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};  // round r: word at i
  for (int r = 0; r < 7; ++r) {
    for (uint32_t q = 0; q < 4; ++q) {
      const uint8_t pos[4] = {uint8_t(2 * q), uint8_t(2 * q + 1), uint8_t(8 + 2 * q),
                              uint8_t(9 + 2 * q)};
      for (int k = 0; k < 4; ++k) {
        const uint32_t w = S[pos[k]];
        s.off[r][k] |= (w + (w >> 3) * (kRow - 8)) << (8 * q);  // words 8-15: the right row
      }
    }
    uint8_t T[16] = {};
    for (int i = 0; i < 16; ++i) T[i] = S[P[i]];
    for (int i = 0; i < 16; ++i) S[i] = T[i];
  }
  return s;
}
constexpr QuadSched kQuadSched = make_quad_sched();

// DPP quad_perm controls: lane i of each quad reads lane p_i
constexpr int kQuadRot1 = 1 | (2 << 2) | (3 << 4) | (0 << 6);  // [1,2,3,0]
constexpr int kQuadRot2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);  // [2,3,0,1]
constexpr int kQuadRot3 = 3 | (0 << 2) | (1 << 4) | (2 << 6);  // [3,0,1,2]

template <int kCtrl>
__device__ __forceinline__ uint32_t quad_perm(uint32_t x) {
  return uint32_t(__builtin_amdgcn_mov_dpp(int(x), kCtrl, 0xF, 0xF, true));
}

// Parent of the two children whose rows start at `left` (right = left +
// kRow) with `flags`, computed by the whole quad (all four lanes active, q =
// lane & 3); lane q returns output words q (lo) and 4 + q (hi).
__device__ __forceinline__ void parent_quad(const uint32_t *left, uint32_t q, uint32_t flags,
                                            uint32_t &lo, uint32_t &hi) {
  const uint32_t iv_a = q == 0 ? 0x6A09E667u : q == 1 ? 0xBB67AE85u : q == 2 ? 0x3C6EF372u : 0xA54FF53Au;
  const uint32_t iv_b = q == 0 ? 0x510E527Fu : q == 1 ? 0x9B05688Cu : q == 2 ? 0x1F83D9ABu : 0x5BE0CD19u;
  uint32_t a = iv_a, b = iv_b, c = iv_a;
  uint32_t d = q == 2 ? 64u : q == 3 ? flags : 0u;  // counter lo, counter hi, block len, flags
  const uint32_t sh = 8 * q;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const uint32_t x0 = left[__builtin_amdgcn_ubfe(kQuadSched.off[r][0], sh, 8)];
    const uint32_t y0 = left[__builtin_amdgcn_ubfe(kQuadSched.off[r][1], sh, 8)];
    const uint32_t x1 = left[__builtin_amdgcn_ubfe(kQuadSched.off[r][2], sh, 8)];
    const uint32_t y1 = left[__builtin_amdgcn_ubfe(kQuadSched.off[r][3], sh, 8)];
    B3_G(a, b, c, d, x0, y0);  // column step
    b = quad_perm<kQuadRot1>(b);
    c = quad_perm<kQuadRot2>(c);
    d = quad_perm<kQuadRot3>(d);
    B3_G(a, b, c, d, x1, y1);  // diagonal step
    b = quad_perm<kQuadRot3>(b);
    c = quad_perm<kQuadRot2>(c);
    d = quad_perm<kQuadRot1>(d);
  }
  lo = a ^ c;
  hi = b ^ d;
}

// One tree level of up to 64 parents by quads (quad i: parent i); an odd
// last node is carried up unchanged.  Whole quads are active or not, so the
// DPP reads inside a quad see only active lanes.
__device__ __forceinline__ void level_by_quads(const uint32_t *src, uint32_t *dst, uint32_t n,
                                               uint32_t t) {
  const uint32_t i = t >> 2, q = t & 3, half = (n + 1) / 2;
  if (i < half) {
    uint32_t lo, hi;
    if (2 * i + 1 < n) {
      parent_quad(src + 2 * i * kRow, q, kParent, lo, hi);
    } else {
      lo = src[2 * i * kRow + q];
      hi = src[2 * i * kRow + 4 + q];
    }
    dst[i * kRow + q] = lo;
    dst[i * kRow + 4 + q] = hi;
  }
}

// Pairs n <= 2 * 256 * per_lane nodes down to one in LDS (ping-pong buffers).
// If `final_msg`, the top pair is finalised into msg_cv/digest instead.
// Levels of at most kQuadMax parents run by quads (latency), wider ones one
// parent per lane (throughput); kQuadMax = 0: lanes only.
template <int kPerLane, uint32_t kQuadMax>
__device__ __forceinline__ void pair_down(uint32_t *buf0, uint32_t *buf1, uint32_t n, bool final_msg,
                                          uint32_t *out_cv, uint32_t *msg_cv, uint32_t *digest) {
  static_assert(kQuadMax <= 64, "a quad level covers at most 64 parents");
  uint32_t *src = buf0, *dst = buf1;
  const uint32_t t = threadIdx.x;
  while (n > 1) {
    const uint32_t half = (n + 1) / 2;
    if (n == 2 && final_msg) {
      if (kQuadMax > 0) {  // quad 0: the subtree CV, quad 1: the ROOT digest
        if (t < 8) {
          uint32_t lo, hi;
          parent_quad(src, t & 3, t < 4 ? kParent : kParent | kRoot, lo, hi);
          uint32_t *o = t < 4 ? msg_cv : digest;
          o[t & 3] = lo;
          o[4 + (t & 3)] = hi;
        }
      } else if (t == 0) {
        parent_final(src, src + kRow, msg_cv, digest);
      }
      return;
    }
    if (half <= kQuadMax) {
      level_by_quads(src, dst, n, t);
      __syncthreads();
      uint32_t *tmp = src;
      src = dst;
      dst = tmp;
      n = half;
      continue;
    }
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) {
      const uint32_t i = t + 256 * j;
      if (i < half) {
        uint32_t r[8];
        if (2 * i + 1 < n) {
          parent_cv(src + 2 * i * kRow, src + (2 * i + 1) * kRow, r);
        } else {
#pragma unroll
          for (int w = 0; w < 8; ++w) r[w] = src[2 * i * kRow + w];
        }
#pragma unroll
        for (int w = 0; w < 8; ++w) dst[i * kRow + w] = r[w];
      }
    }
    __syncthreads();
    uint32_t *tmp = src;
    src = dst;
    dst = tmp;
    n = half;
  }
  if (t == 0 && out_cv) {
#pragma unroll
    for (int w = 0; w < 8; ++w) out_cv[w] = src[w];
  }
}

// Workgroup w's group: the message whose group range holds w (binary search
// over first_group, uniform across the workgroup), then its offset in it.
struct Group {
  uint64_t addr, chunk0;
  uint32_t nbytes, msg, single;
};
__device__ __forceinline__ Group find_group(const HashMsg *__restrict__ msgs, uint32_t n_msgs,
                                            uint32_t w) {
  uint32_t lo = 0, hi = n_msgs - 1;  // the last message with first_group <= w
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) / 2;
    if (msgs[mid].first_group <= w) lo = mid;
    else hi = mid - 1;
  }
  const HashMsg m = msgs[lo];
  const uint32_t g = w - m.first_group;
  const uint64_t off = uint64_t(g) * kGroupBytes;
  const uint64_t rem = m.nbytes - off;
  Group r;
  r.addr = m.addr + off;
  r.chunk0 = m.chunk0 + uint64_t(g) * kGroupChunks;
  r.nbytes = uint32_t(m.nbytes == 0 ? 0 : (rem < kGroupBytes ? rem : kGroupBytes));
  r.msg = lo;
  r.single = m.groups == 1;
  return r;
}

// kQuadMax: levels of at most that many parents by quads.  Kernel 1 is
// throughput-bound and launched with 0: quads at its level 3 (32 parents)
// would save ~0.4% of its issue slots, but the quad code pushed the kernel
// past its 64-VGPR cap (17 spilled registers), DESIGN.md §7b.
template <uint32_t kLevels, uint32_t kQuadMax>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void blake3_group_kernel(
    const HashMsg *__restrict__ msgs, uint32_t n_msgs, uint32_t *__restrict__ group_cvs,
    uint32_t *__restrict__ msg_cvs, uint32_t *__restrict__ digests) {
  __shared__ uint32_t lds[2][256 * kRow];
  const Group g = find_group(msgs, n_msgs, blockIdx.x);
  const uint32_t t = threadIdx.x;
  const uint32_t nchunks = g.nbytes == 0 ? 1 : (g.nbytes + kChunkBytes - 1) / kChunkBytes;
  uint32_t cv[8];
  set_iv(cv);
  if (t < nchunks) {
    const uint32_t off = t * kChunkBytes;
    const uint32_t clen = g.nbytes - off < kChunkBytes ? g.nbytes - off : kChunkBytes;
    const uint32_t nblocks = clen == 0 ? 1 : (clen + 63) / 64;
    const uint8_t *p = reinterpret_cast<const uint8_t *>(g.addr) + off;
    const uint64_t counter = g.chunk0 + t;
    for (uint32_t b = 0; b + 1 < nblocks; ++b) {
      uint32_t m[16];
      load_block(p + 64 * b, 64, m);
      compress_cv(cv, m, counter, 64, b == 0 ? kStart : 0);
    }
    const uint32_t last = nblocks - 1, blen = clen - 64 * last;
    uint32_t m[16];
    load_block(p + 64 * last, blen, m);
    const uint32_t flags = (last == 0 ? kStart : 0) | kEnd;
    if (g.single && nchunks == 1) {  // one-chunk message: this block is the root
      finalize(cv, m, counter, blen, flags, msg_cvs + 8 * g.msg, digests + 8 * g.msg);
      return;  // whole workgroup takes this branch (nchunks is uniform)
    }
    compress_cv(cv, m, counter, blen, flags);
  }
  if (nchunks == 1 && g.single) return;
#pragma unroll
  for (int w = 0; w < 8; ++w) lds[0][t * kRow + w] = cv[w];
  __syncthreads();
  if (g.single) {  // the whole message: pair down to the root here
    pair_down<1, kQuadMax>(lds[0], lds[1], nchunks, true, nullptr, msg_cvs + 8 * g.msg,
                           digests + 8 * g.msg);
    return;
  }
  // kLevels levels (256 -> 256 >> kLevels nodes); an odd last node is carried up
  uint32_t n = nchunks, *src = lds[0], *dst = lds[1];
#pragma unroll
  for (uint32_t lv = 0; lv < kLevels; ++lv) {
    const uint32_t half = (n + 1) / 2;
    if (half <= kQuadMax) {
      level_by_quads(src, dst, n, t);
    } else if (t < half) {
      uint32_t r[8];
      if (2 * t + 1 < n) {
        parent_cv(src + 2 * t * kRow, src + (2 * t + 1) * kRow, r);
      } else {
#pragma unroll
        for (int w = 0; w < 8; ++w) r[w] = src[2 * t * kRow + w];
      }
#pragma unroll
      for (int w = 0; w < 8; ++w) dst[t * kRow + w] = r[w];
    }
    __syncthreads();
    uint32_t *tmp = src;
    src = dst;
    dst = tmp;
    n = half;
  }
  if (t < n) {
    uint32_t *o = group_cvs + 8 * (size_t(blockIdx.x) * (kGroupChunks >> kLevels) + t);
#pragma unroll
    for (int w = 0; w < 8; ++w) o[w] = src[t * kRow + w];
  }
}

// Latency-bound (a chain of levels per job): every level of <= 64 parents by quads.
template <uint32_t kQuadMax>
__global__ __launch_bounds__(256) void blake3_reduce_kernel(const HashReduce *__restrict__ jobs,
                                                            const uint32_t *__restrict__ in_cvs,
                                                            uint32_t *__restrict__ out_cvs,
                                                            uint32_t *__restrict__ msg_cvs,
                                                            uint32_t *__restrict__ digests) {
  __shared__ uint32_t lds[2][kReduceFanIn * kRow];
  const HashReduce j = jobs[blockIdx.x];
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < j.n; i += 256)
#pragma unroll
    for (int w = 0; w < 8; ++w) lds[0][i * kRow + w] = in_cvs[8 * (j.first + i) + w];
  __syncthreads();
  pair_down<kReduceFanIn / 512, kQuadMax>(lds[0], lds[1], j.n, j.final != 0,
                                j.final ? nullptr : out_cvs + 8 * j.out, msg_cvs + 8 * j.msg,
                                digests + 8 * j.msg);
}

}  // namespace

hipError_t launch_blake3_groups(const HashMsg *d_msgs, uint32_t n_msgs, uint32_t n_groups,
                                uint32_t levels, uint32_t *d_group_cvs, uint32_t *d_msg_cvs,
                                uint32_t *d_digests, hipStream_t stream) {
  if (n_groups == 0 || n_msgs == 0) return hipSuccess;
  if (levels != 3) return hipErrorInvalidValue;
  hipLaunchKernelGGL((blake3_group_kernel<3, 0>), dim3(n_groups), dim3(256), 0, stream, d_msgs,
                     n_msgs, d_group_cvs, d_msg_cvs, d_digests);
  return hipGetLastError();
}

hipError_t launch_blake3_reduce(const HashReduce *d_jobs, uint32_t n_jobs, bool quads,
                                const uint32_t *d_in, uint32_t *d_out, uint32_t *d_msg_cvs,
                                uint32_t *d_digests, hipStream_t stream) {
  if (n_jobs == 0) return hipSuccess;
#ifdef BFRS_AB_VARIANTS
  if (!quads) {
    hipLaunchKernelGGL((blake3_reduce_kernel<0>), dim3(n_jobs), dim3(256), 0, stream, d_jobs, d_in,
                       d_out, d_msg_cvs, d_digests);
    return hipGetLastError();
  }
#else
  if (!quads) return hipErrorInvalidValue;
#endif
  hipLaunchKernelGGL((blake3_reduce_kernel<64>), dim3(n_jobs), dim3(256), 0, stream, d_jobs, d_in,
                     d_out, d_msg_cvs, d_digests);
  return hipGetLastError();
}

}  // namespace bfrs
