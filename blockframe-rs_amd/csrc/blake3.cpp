// blake3.cpp — see blake3.hpp.
#include "blake3.hpp"

#include <algorithm>
#include <array>
#include <cstring>
#include <thread>

namespace bfrs {
namespace {

constexpr std::array<uint32_t, 8> kIV = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                         0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
constexpr size_t kChunkLen = 1024;
constexpr size_t kBlockLen = 64;
enum : uint32_t { kChunkStart = 1, kChunkEnd = 2, kParent = 4, kRoot = 8 };

using Words8 = std::array<uint32_t, 8>;

inline uint32_t rotr32(uint32_t x, unsigned n) { return (x >> n) | (x << (32 - n)); }

struct State {
  uint32_t v[16];
  void quarter(int a, int b, int c, int d, uint32_t mx, uint32_t my) {
    v[a] += v[b] + mx;
    v[d] = rotr32(v[d] ^ v[a], 16);
    v[c] += v[d];
    v[b] = rotr32(v[b] ^ v[c], 12);
    v[a] += v[b] + my;
    v[d] = rotr32(v[d] ^ v[a], 8);
    v[c] += v[d];
    v[b] = rotr32(v[b] ^ v[c], 7);
  }
};

// Message word schedule per round (the spec's permutation applied r times).
struct Schedule {
  uint8_t s[7][16];
  Schedule() {
    static const uint8_t perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
    for (int i = 0; i < 16; ++i) s[0][i] = uint8_t(i);
    for (int r = 1; r < 7; ++r)
      for (int i = 0; i < 16; ++i) s[r][i] = s[r - 1][perm[i]];
  }
};
const Schedule kSched;

// Full 16-word compression output.
void compress(const Words8 &cv, const uint32_t m[16], uint64_t counter, uint32_t len,
              uint32_t flags, uint32_t out[16]) {
  State st;
  for (int i = 0; i < 8; ++i) st.v[i] = cv[i];
  for (int i = 0; i < 4; ++i) st.v[8 + i] = kIV[i];
  st.v[12] = uint32_t(counter);
  st.v[13] = uint32_t(counter >> 32);
  st.v[14] = len;
  st.v[15] = flags;
  for (int r = 0; r < 7; ++r) {
    const uint8_t *s = kSched.s[r];
    st.quarter(0, 4, 8, 12, m[s[0]], m[s[1]]);
    st.quarter(1, 5, 9, 13, m[s[2]], m[s[3]]);
    st.quarter(2, 6, 10, 14, m[s[4]], m[s[5]]);
    st.quarter(3, 7, 11, 15, m[s[6]], m[s[7]]);
    st.quarter(0, 5, 10, 15, m[s[8]], m[s[9]]);
    st.quarter(1, 6, 11, 12, m[s[10]], m[s[11]]);
    st.quarter(2, 7, 8, 13, m[s[12]], m[s[13]]);
    st.quarter(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; ++i) {
    out[i] = st.v[i] ^ st.v[i + 8];
    out[i + 8] = st.v[i + 8] ^ cv[i];
  }
}

void load_block(const uint8_t *p, size_t n, uint32_t m[16]) {
  uint8_t buf[kBlockLen];
  if (n < kBlockLen) {
    std::memset(buf, 0, sizeof buf);
    if (n) std::memcpy(buf, p, n);  // p is NULL for the empty message
    p = buf;
  }
  for (int i = 0; i < 16; ++i)
    m[i] = uint32_t(p[4 * i]) | uint32_t(p[4 * i + 1]) << 8 | uint32_t(p[4 * i + 2]) << 16 |
           uint32_t(p[4 * i + 3]) << 24;
}

// A node whose final compression is pending (it may become the root).
struct Pending {
  Words8 cv;
  uint32_t m[16];
  uint64_t counter;
  uint32_t len, flags;
  Words8 chaining() const {
    uint32_t o[16];
    compress(cv, m, counter, len, flags, o);
    Words8 r;
    std::copy(o, o + 8, r.begin());
    return r;
  }
};

Pending chunk_node(const uint8_t *p, size_t n, uint64_t index) {
  Words8 cv = kIV;
  const size_t blocks = n == 0 ? 1 : (n + kBlockLen - 1) / kBlockLen;
  Pending last{};
  for (size_t b = 0; b < blocks; ++b) {
    const size_t len = b + 1 < blocks ? kBlockLen : n - b * kBlockLen;
    uint32_t m[16];
    load_block(p + b * kBlockLen, len, m);
    const uint32_t flags = (b == 0 ? kChunkStart : 0) | (b + 1 == blocks ? kChunkEnd : 0);
    if (b + 1 < blocks) {
      uint32_t o[16];
      compress(cv, m, index, kBlockLen, flags, o);
      std::copy(o, o + 8, cv.begin());
    } else {
      last.cv = cv;
      std::copy(m, m + 16, last.m);
      last.counter = index;
      last.len = uint32_t(len);
      last.flags = flags;
    }
  }
  return last;
}

Pending parent_node(const Words8 &l, const Words8 &r) {
  Pending p{};
  p.cv = kIV;
  std::copy(l.begin(), l.end(), p.m);
  std::copy(r.begin(), r.end(), p.m + 8);
  p.counter = 0;
  p.len = kBlockLen;
  p.flags = kParent;
  return p;
}

// Largest power of two strictly less than n (n >= 2).
size_t left_len(size_t n) {
  size_t p = 1;
  while (p * 2 < n) p *= 2;
  return p;
}

// Pending node for chunks [first, first+n) of the input (global chunk indices).
Pending subtree(const uint8_t *data, size_t len, size_t first, size_t n, int threads) {
  if (n == 1) {
    const size_t off = first * kChunkLen;
    return chunk_node(data + off, std::min(kChunkLen, len - off), first);
  }
  const size_t l = left_len(n);
  Words8 lcv, rcv;
  std::thread t;
  if (threads > 1 && n >= 64) {
    try {
      t = std::thread([&] { lcv = subtree(data, len, first, l, threads / 2).chaining(); });
    } catch (...) {  // no thread (quota): this subtree runs on the calling thread
    }
  }
  if (t.joinable()) {
    // the left half's thread is joined on every path, an exception included
    struct Join {
      std::thread &t;
      ~Join() { t.join(); }
    } join{t};
    rcv = subtree(data, len, first + l, n - l, threads - threads / 2).chaining();
  } else {
    lcv = subtree(data, len, first, l, 1).chaining();
    rcv = subtree(data, len, first + l, n - l, 1).chaining();
  }
  return parent_node(lcv, rcv);
}

}  // namespace

void blake3_hash(const uint8_t *data, size_t len, uint8_t out[32], int threads) {
  const size_t chunks = len == 0 ? 1 : (len + kChunkLen - 1) / kChunkLen;
  Pending root = subtree(data, len, 0, chunks, std::max(1, threads));
  uint32_t o[16];
  compress(root.cv, root.m, root.counter, root.len, root.flags | kRoot, o);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = uint8_t(o[i]);
    out[4 * i + 1] = uint8_t(o[i] >> 8);
    out[4 * i + 2] = uint8_t(o[i] >> 16);
    out[4 * i + 3] = uint8_t(o[i] >> 24);
  }
}

std::string blake3_combine_cvs_hex(const uint8_t *cvs, size_t n) {
  std::vector<Words8> level(n);
  for (size_t i = 0; i < n; ++i)
    for (int w = 0; w < 8; ++w)
      level[i][w] = uint32_t(cvs[32 * i + 4 * w]) | uint32_t(cvs[32 * i + 4 * w + 1]) << 8 |
                    uint32_t(cvs[32 * i + 4 * w + 2]) << 16 | uint32_t(cvs[32 * i + 4 * w + 3]) << 24;
  // level-wise pairing, odd last node carried: BLAKE3's left-complete tree
  while (level.size() > 2) {
    std::vector<Words8> next;
    for (size_t i = 0; i + 1 < level.size(); i += 2)
      next.push_back(parent_node(level[i], level[i + 1]).chaining());
    if (level.size() % 2) next.push_back(level.back());
    level.swap(next);
  }
  Pending root = parent_node(level[0], level[1]);
  uint32_t o[16];
  compress(root.cv, root.m, root.counter, root.len, root.flags | kRoot, o);
  uint8_t d[32];
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 4; ++b) d[4 * i + b] = uint8_t(o[i] >> (8 * b));
  return to_hex(d, 32);
}

std::string to_hex(const uint8_t *d, size_t n) {
  static const char *digits = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = digits[d[i] >> 4];
    s[2 * i + 1] = digits[d[i] & 15];
  }
  return s;
}

std::string blake3_hex(const uint8_t *data, size_t len, int threads) {
  uint8_t d[32];
  blake3_hash(data, len, d, threads);
  return to_hex(d, 32);
}

std::string merkle_root_hex(const std::vector<std::string> &leaves) {
  if (leaves.empty()) return std::string();
  std::vector<std::string> level = leaves;
  while (level.size() > 1) {
    std::vector<std::string> next;
    next.reserve((level.size() + 1) / 2);
    for (size_t i = 0; i < level.size(); i += 2) {
      const std::string &l = level[i];
      const std::string &r = i + 1 < level.size() ? level[i + 1] : level[i];
      const std::string cat = l + r;
      next.push_back(blake3_hex(reinterpret_cast<const uint8_t *>(cat.data()), cat.size()));
    }
    level.swap(next);
  }
  return level[0];
}

}  // namespace bfrs
