// plan.cpp — GF(2^16) field and coefficient planner (see plan.hpp).
//
// The transform sequence restates reed-solomon-simd 3.1.0's HighRate/LowRate
// encoder and decoder on probe matrices instead
// of shard bytes.  Rows are code positions, columns are probes.
#include "plan.hpp"

#include "kernels.hpp"

#include <algorithm>
#include <array>

namespace bfrs {
namespace {

constexpr uint32_t kOrder = 1u << 16;
constexpr uint16_t kModulus = 0xFFFF;  // also "log of zero"

// Leopard/crate Cantor basis (beta_0 = 1, beta_i^2 + beta_i = beta_{i-1}).
constexpr std::array<uint16_t, 16> kCantor = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E,
                                              0x914C, 0x4012, 0x6C98, 0x10D8, 0x6A72, 0xB900,
                                              0xFDB8, 0xFB34, 0xFF38, 0x991E};

inline uint16_t log_add(uint32_t a, uint32_t b) {
  uint32_t s = a + b;
  return uint16_t(s + (s >> 16));
}

size_t pow2_at_least(size_t x) {
  size_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

Gf16::Gf16() : exp_(kOrder), log_(kOrder), skew_(kOrder) {
  // Polynomial-basis discrete log via the LFSR x^(i) mod 0x1002D.
  std::vector<uint16_t> plog(kOrder);
  uint32_t v = 1;
  for (uint32_t i = 0; i < kModulus; ++i) {
    plog[v] = uint16_t(i);
    v <<= 1;
    if (v & kOrder) v ^= 0x1002D;
  }
  plog[0] = kModulus;
  // Cantor element j -> polynomial-basis value, then to its log.
  std::vector<uint16_t> cantor_to_poly(kOrder, 0);
  for (uint32_t j = 1; j < kOrder; ++j) {
    uint32_t low = j & (j - 1);          // j without its lowest set bit
    unsigned bit = __builtin_ctz(j);
    cantor_to_poly[j] = cantor_to_poly[low] ^ kCantor[bit];
  }
  for (uint32_t j = 0; j < kOrder; ++j) log_[j] = plog[cantor_to_poly[j]];
  for (uint32_t j = 0; j < kOrder; ++j) exp_[log_[j]] = uint16_t(j);
  exp_[kModulus] = exp_[0];

  // Skew factors of the LCH basis (crate's initialize_skew).
  std::array<uint16_t, 15> t{};
  for (unsigned i = 1; i < 16; ++i) t[i - 1] = uint16_t(1u << i);
  for (unsigned m = 0; m < 15; ++m) {
    const size_t step = size_t(1) << (m + 1);
    skew_[(size_t(1) << m) - 1] = 0;
    for (unsigned i = m; i < 15; ++i) {
      const size_t s = size_t(1) << (i + 1);
      for (size_t j = (size_t(1) << m) - 1; j < s; j += step) skew_[j + s] = skew_[j] ^ t[i];
    }
    t[m] = uint16_t(kModulus - log_[mul_log(t[m], log_[t[m] ^ 1])]);
    for (unsigned i = m + 1; i < 15; ++i) t[i] = mul_log(t[i], log_add(log_[t[i] ^ 1], t[m]));
  }
  for (size_t i = 0; i < kModulus; ++i) skew_[i] = log_[skew_[i]];
}

const Gf16 &Gf16::get() {
  static const Gf16 f;
  return f;
}

bool choose_rate(size_t k, size_t m, Rate *rate) {
  if (k == 0 || m == 0 || k > kOrder || m > kOrder) return false;
  const size_t kp = pow2_at_least(k), mp = pow2_at_least(m);
  if (std::min(kp, mp) + std::max(k, m) > kOrder) return false;
  bool high = kp > mp || (kp == mp && k <= m);
  *rate = high ? Rate::kHigh : Rate::kLow;
  return true;
}

namespace {

// Probe matrix: `rows` code positions x `cols` probe columns.
struct Probe {
  size_t rows, cols;
  std::vector<uint16_t> v;
  Probe(size_t r, size_t c) : rows(r), cols(c), v(r * c, 0) {}
  uint16_t *row(size_t r) { return v.data() + r * cols; }
};

void row_xor(Probe &p, size_t dst, size_t src) {
  uint16_t *d = p.row(dst);
  const uint16_t *s = p.row(src);
  for (size_t c = 0; c < p.cols; ++c) d[c] ^= s[c];
}

// dst ^= src * exp(lm)
void row_muladd(Probe &p, size_t dst, size_t src, uint16_t lm) {
  const Gf16 &f = Gf16::get();
  uint16_t *d = p.row(dst);
  const uint16_t *s = p.row(src);
  for (size_t c = 0; c < p.cols; ++c) d[c] ^= f.mul_log(s[c], lm);
}

void row_scale(Probe &p, size_t r, uint16_t lm) {
  const Gf16 &f = Gf16::get();
  uint16_t *d = p.row(r);
  for (size_t c = 0; c < p.cols; ++c) d[c] = f.mul_log(d[c], lm);
}

// LCH inverse FFT over positions [pos, pos+size); inputs >= trunc are zero.
void ifft(Probe &p, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
  const Gf16 &f = Gf16::get();
  for (size_t dist = 1; dist < size; dist <<= 1)
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      const uint16_t lm = f.skew(r + dist + skew_delta - 1);
      for (size_t i = r; i < r + dist; ++i) {
        row_xor(p, pos + i + dist, pos + i);
        if (lm != kModulus) row_muladd(p, pos + i, pos + i + dist, lm);
      }
    }
}

// LCH forward FFT; outputs < trunc are exact.
void fft(Probe &p, size_t pos, size_t size, size_t trunc, size_t skew_delta) {
  const Gf16 &f = Gf16::get();
  for (size_t dist = size >> 1; dist; dist >>= 1)
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      const uint16_t lm = f.skew(r + dist + skew_delta - 1);
      for (size_t i = r; i < r + dist; ++i) {
        if (lm != kModulus) row_muladd(p, pos + i, pos + i + dist, lm);
        row_xor(p, pos + i + dist, pos + i);
      }
    }
}

void formal_derivative(Probe &p, size_t n) {
  for (size_t i = 1; i < n; ++i) {
    const size_t w = i & (~i + 1);
    for (size_t j = 0; j < w; ++j) row_xor(p, i - w + j, i + j);
  }
}

// Log of the erasure-locator value at every position < n:
//   loc[p] = sum_{e in erased, e != p} log(w_p + w_e)  (mod 65535).
// The crate evaluates the same sums with a Walsh-Hadamard convolution over all
// 65536 positions.  Erased positions outside [0, n) (LowRate marks every
// position past the recovery block) multiply the locator by one common
// non-zero constant on [0, n), which the final division cancels exactly, so
// they are dropped here.
std::vector<uint16_t> erasure_locator(const std::vector<uint8_t> &erased, size_t n) {
  const Gf16 &f = Gf16::get();
  std::vector<uint16_t> loc(n);
  for (size_t pos = 0; pos < n; ++pos) {
    uint64_t s = 0;
    for (size_t e = 0; e < n; ++e)
      if (erased[e] && e != pos) s += f.log(uint16_t(pos ^ e));
    loc[pos] = uint16_t(s % kModulus);
  }
  return loc;
}

}  // namespace

CoefMatrix plan_encode(size_t k, size_t m) {
  Rate rate;
  CoefMatrix out;
  if (!choose_rate(k, m, &rate)) return out;
  out.rows = m;
  out.cols = k;
  out.c.assign(m * k, 0);
  if (rate == Rate::kHigh) {
    // Originals sit at code positions c+i; recovery at [0, c).
    const size_t c = pow2_at_least(m);
    const size_t rows = (k + c - 1) / c * c;
    Probe p(rows, k);
    for (size_t i = 0; i < k; ++i) p.row(i)[i] = 1;
    ifft(p, 0, c, std::min(k, c), c);
    size_t pos = c;
    for (; pos + c <= k; pos += c) {
      ifft(p, pos, c, c, pos + c);
      for (size_t i = 0; i < c; ++i) row_xor(p, i, pos + i);
    }
    if (k > c && k % c) {
      ifft(p, pos, c, k % c, pos + c);
      for (size_t i = 0; i < c; ++i) row_xor(p, i, pos + i);
    }
    fft(p, 0, c, m, 0);
    for (size_t j = 0; j < m; ++j) std::copy(p.row(j), p.row(j) + k, out.c.begin() + j * k);
  } else {
    // Originals at positions [0, k); recovery chunks at c, 2c, ...
    const size_t c = pow2_at_least(k);
    const size_t rows = std::max(c, (m + c - 1) / c * c);
    Probe p(rows, k);
    for (size_t i = 0; i < k; ++i) p.row(i)[i] = 1;
    ifft(p, 0, c, k, 0);
    for (size_t pos = c; pos < m; pos += c)
      std::copy(p.row(0), p.row(0) + c * k, p.row(pos));
    size_t pos = 0;
    for (; pos + c <= m; pos += c) fft(p, pos, c, c, pos + c);
    if (m % c) fft(p, pos, c, m % c, pos + c);
    for (size_t j = 0; j < m; ++j) std::copy(p.row(j), p.row(j) + k, out.c.begin() + j * k);
  }
  return out;
}

CoefMatrix plan_decode(size_t k, size_t m, const std::vector<uint8_t> &orig_present,
                       const std::vector<uint8_t> &rec_present) {
  Rate rate;
  CoefMatrix out;
  if (!choose_rate(k, m, &rate)) return out;
  const Gf16 &f = Gf16::get();

  // Input columns: present recovery then present originals; output rows:
  // missing originals.
  std::vector<size_t> col_of_rec(m, SIZE_MAX), col_of_orig(k, SIZE_MAX), missing;
  size_t cols = 0;
  for (size_t j = 0; j < m; ++j)
    if (rec_present[j]) col_of_rec[j] = cols++;
  for (size_t i = 0; i < k; ++i) {
    if (orig_present[i])
      col_of_orig[i] = cols++;
    else
      missing.push_back(i);
  }
  out.rows = missing.size();
  out.cols = cols;
  out.c.assign(out.rows * cols, 0);

  size_t orig_base, rec_base, end, n, fft_trunc;
  std::vector<uint8_t> erased;
  if (rate == Rate::kHigh) {
    const size_t c = pow2_at_least(m);
    rec_base = 0;
    orig_base = c;
    end = c + k;
    n = pow2_at_least(end);
    fft_trunc = end;
    erased.assign(n, 0);
    for (size_t j = 0; j < m; ++j) erased[j] = !rec_present[j];
    for (size_t j = m; j < c; ++j) erased[j] = 1;
    for (size_t i = 0; i < k; ++i) erased[c + i] = !orig_present[i];
  } else {
    const size_t c = pow2_at_least(k);
    orig_base = 0;
    rec_base = c;
    end = c + m;
    n = pow2_at_least(end);
    fft_trunc = k;
    erased.assign(n, 0);
    // [k, c) holds the encoder's zero padding: a known zero, not an erasure
    // (its product with the locator is zero either way, but an erased pad
    // would spend c-k of the m correctable erasures)
    for (size_t i = 0; i < k; ++i) erased[i] = !orig_present[i];
    for (size_t j = 0; j < m; ++j) erased[c + j] = !rec_present[j];
    for (size_t i = end; i < n; ++i) erased[i] = 1;
  }
  const std::vector<uint16_t> loc = erasure_locator(erased, n);

  Probe p(n, cols);
  for (size_t j = 0; j < m; ++j)
    if (rec_present[j]) p.row(rec_base + j)[col_of_rec[j]] = f.exp(loc[rec_base + j]);
  for (size_t i = 0; i < k; ++i)
    if (orig_present[i]) p.row(orig_base + i)[col_of_orig[i]] = f.exp(loc[orig_base + i]);
  ifft(p, 0, n, end, 0);
  formal_derivative(p, n);
  fft(p, 0, n, fft_trunc, 0);
  for (size_t t = 0; t < missing.size(); ++t) {
    const size_t pos = orig_base + missing[t];
    row_scale(p, pos, uint16_t(kModulus - loc[pos]));
    std::copy(p.row(pos), p.row(pos) + cols, out.c.begin() + t * cols);
  }
  return out;
}

void build_tables(const CoefMatrix &m, size_t r0, size_t r1, size_t c0, size_t c1,
                  std::vector<uint32_t> *out) {
  const Gf16 &f = Gf16::get();
  out->assign((c1 - c0) * 64 * 2, 0);
  for (size_t in = c0; in < c1; ++in) {
    uint32_t *t = out->data() + (in - c0) * 128;
    for (size_t r = r0; r < r1; ++r) {
      const uint16_t coef = m.at(r, in);
      const unsigned shift = 8 * unsigned(r - r0);
      for (unsigned q = 0; q < 4; ++q)
        for (unsigned v = 0; v < 16; ++v) {
          const uint16_t prod = f.mul(uint16_t(v << (4 * q)), coef);
          uint32_t *e = t + tab_idx(q, v) * 2;
          e[0] |= uint32_t(prod & 0xFF) << shift;
          e[1] |= uint32_t(prod >> 8) << shift;
        }
    }
  }
}

}  // namespace bfrs
