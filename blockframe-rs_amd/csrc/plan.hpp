// plan.hpp — host-side coefficient planner for the MI355X RS path.
//
// reed-solomon-simd 3.1.0 (the crate behind src/chunker/generate.rs:84-96 and
// src/filestore/recovery.rs:152-170) computes recovery shards with a GF(2^16)
// additive FFT (Leopard "ff16", Cantor basis).  Every step of that transform
// is GF(2^16)-linear, so for a given (k, m, erasure pattern) each output shard
// is a fixed linear combination of the input shards, symbol by symbol.  The
// planner runs the crate's transform once over *probe* vectors (one column per
// input shard, identity on input) to obtain that coefficient matrix; the GPU
// then applies the matrix to every symbol of every shard in one HBM pass
// (rs_kernels.hip).  The matrix is the crate's own map, so outputs are
// bit-exact, including its choice of which received shards a decode uses.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace bfrs {

// GF(2^16) with the crate's representation: elements are Cantor-basis bit
// vectors (addition = XOR), logs modulo 65535 with 65535 marking zero.
class Gf16 {
 public:
  static const Gf16 &get();
  uint16_t exp(uint32_t l) const { return exp_[l]; }
  uint16_t log(uint16_t x) const { return log_[x]; }
  uint16_t skew(size_t i) const { return skew_[i]; }
  // x * exp(log_m)
  uint16_t mul_log(uint16_t x, uint16_t log_m) const {
    if (x == 0) return 0;
    uint32_t s = uint32_t(log_[x]) + log_m;
    return exp_[(s + (s >> 16)) & 0xFFFF];
  }
  uint16_t mul(uint16_t a, uint16_t b) const { return b == 0 ? 0 : mul_log(a, log_[b]); }

 private:
  Gf16();
  std::vector<uint16_t> exp_, log_, skew_;
};

enum class Rate { kHigh, kLow };

// DefaultRate choice; returns false if (k, m) is unsupported by the crate.
bool choose_rate(size_t k, size_t m, Rate *rate);

// Coefficient matrix: rows = outputs, cols = inputs, row-major.
struct CoefMatrix {
  size_t rows = 0, cols = 0;
  std::vector<uint16_t> c;
  uint16_t at(size_t r, size_t col) const { return c[r * cols + col]; }
};

// Encode: rows = recovery j (m), cols = original i (k).
CoefMatrix plan_encode(size_t k, size_t m);

// Decode: inputs are the present shards in the order
//   [present recovery j ascending] ++ [present original i ascending];
// outputs are the missing originals, ascending.  `orig_present` has k
// entries, `rec_present` m entries.  Caller guarantees at least one original
// is missing and enough shards are present.
CoefMatrix plan_decode(size_t k, size_t m, const std::vector<uint8_t> &orig_present,
                       const std::vector<uint8_t> &rec_present);

// Kernel nibble tables for one pass of <= 4 outputs over inputs [c0, c1):
// entry [in][q][v] (q = lo-low, lo-high, hi-low, hi-high nibble of the input
// symbol, v its value) packs, for output t, byte t of the low dword = low
// byte of coef(t,in)*(v<<4q) and byte t of the high dword = its high byte.
// Layout: uint32 pairs, (c1-c0) * 64 entries.
void build_tables(const CoefMatrix &m, size_t r0, size_t r1, size_t c0, size_t c1,
                  std::vector<uint32_t> *out);

}  // namespace bfrs
