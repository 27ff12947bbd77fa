// rs_kernels.hip — gfx950 kernels for the BlockFrame Reed-Solomon path.
//
// Replaces the arithmetic of reed-solomon-simd's encode()/decode() (called at
// src/chunker/generate.rs:92 and src/filestore/recovery.rs:166) with one HBM
// pass per RS block: every output shard is sum_i coef(t,i) * input_i over
// GF(2^16), coefficients from plan.cpp.
//
// Data layout (crate's): a shard is a run of 64-byte chunks; chunk
// c holds 32 symbols, low bytes at [64c, 64c+32), high bytes at [64c+32, 64c+64).
// Work unit: one lane owns a 32-byte *half-chunk* = 16 symbols: 16 low bytes at
// 64c + 16h and the matching 16 high bytes at 64c + 32 + 16h (h = half).  A
// 256-lane workgroup tile covers 8 KiB of columns of every shard of a block.
//
// Arithmetic: multiplication of a 16-bit symbol by a constant is GF(2)-linear,
// so coef*x = T0[x&15] ^ T1[(x>>4)&15] ^ T2[(x>>8)&15] ^ T3[x>>12] with 16-entry
// nibble tables.  One table entry packs the products for up to 4 outputs:
// low dword = the 4 outputs' low bytes, high dword = their high bytes.  A
// 16-entry x 8-byte table spans 32 LDS banks, so a ds_read_b64 with
// arbitrary nibbles per lane is bank-conflict free.  Per symbol and input: 4
// LDS lookups + XORs, independent of the number of outputs (<= 4).
#include "kernels.hpp"

namespace bfrs {
namespace {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }

// acc_lo[s] / acc_hi[s]: packed low/high output bytes of symbol s (byte t = output t).
__device__ __forceinline__ void mac_input(const uint4 &L, const uint4 &H, const uint2 *__restrict__ T,
                                          uint32_t (&acc_lo)[16], uint32_t (&acc_hi)[16]) {
  const uint32_t l[4] = {L.x, L.y, L.z, L.w};
  const uint32_t h[4] = {H.x, H.y, H.z, H.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int s = d * 4 + b;
      const uint32_t lb = (l[d] >> (8 * b)) & 0xFF;
      const uint32_t hb = (h[d] >> (8 * b)) & 0xFF;
      const uint2 e0 = T[lb & 15];
      const uint2 e1 = T[16 + (lb >> 4)];
      const uint2 e2 = T[32 + (hb & 15)];
      const uint2 e3 = T[48 + (hb >> 4)];
      acc_lo[s] = xor3(acc_lo[s], e0.x, e1.x) ^ xor3(e2.x, e3.x, 0);
      acc_hi[s] = xor3(acc_hi[s], e0.y, e1.y) ^ xor3(e2.y, e3.y, 0);
    }
  }
}

// Byte t of acc[4d..4d+3] -> dword d of output t (4x4 byte transpose).
__device__ __forceinline__ uint32_t gather_byte(const uint32_t (&acc)[16], int d, int t) {
  const uint32_t sh = 8u * t;
  return ((acc[4 * d + 0] >> sh) & 0xFF) | (((acc[4 * d + 1] >> sh) & 0xFF) << 8) |
         (((acc[4 * d + 2] >> sh) & 0xFF) << 16) | (((acc[4 * d + 3] >> sh) & 0xFF) << 24);
}

__device__ __forceinline__ uint4 load16(const uint8_t *p) {
  return *reinterpret_cast<const uint4 *>(p);
}

__global__ __launch_bounds__(256) void gf_apply_kernel(const PassDesc *__restrict__ passes,
                                                       uint32_t n_passes, uint32_t tiles_per_wg) {
  extern __shared__ __attribute__((aligned(16))) uint2 lds_table[];

  // Locate this workgroup's pass (wave-uniform binary search over wg_begin).
  const uint32_t wg = blockIdx.x;
  uint32_t lo = 0, hi = n_passes;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (passes[mid].wg_begin <= wg)
      lo = mid;
    else
      hi = mid;
  }
  const PassDesc &P = passes[lo];
  const uint32_t n_in = P.n_in, n_out = P.n_out;

  for (uint32_t e = threadIdx.x; e < n_in * 64; e += blockDim.x) lds_table[e] = P.table[e];
  __syncthreads();

  const uint64_t full_hc = P.full_chunks * 2;
  const uint32_t t_begin = (wg - P.wg_begin) * tiles_per_wg;
  const uint32_t t_end = min(t_begin + tiles_per_wg, P.n_tiles);

  for (uint32_t tile = t_begin; tile < t_end; ++tile) {
    const uint64_t hc = uint64_t(tile) * kTileHalfChunks + threadIdx.x;
    if (hc >= full_hc) break;
    const uint64_t off = (hc >> 1) * 64 + (hc & 1) * 16;

    uint32_t acc_lo[16], acc_hi[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) acc_lo[s] = acc_hi[s] = 0;

    // Software pipeline: loads of input i+1 are in flight while input i computes.
    uint4 L = load16(P.in[0] + off), H = load16(P.in[0] + off + 32);
    for (uint32_t i = 0; i < n_in; ++i) {
      uint4 Ln = L, Hn = H;
      if (i + 1 < n_in) {
        const uint8_t *src = P.in[i + 1];
        Ln = load16(src + off);
        Hn = load16(src + off + 32);
      }
      mac_input(L, H, lds_table + i * 64, acc_lo, acc_hi);
      L = Ln;
      H = Hn;
    }

    for (uint32_t t = 0; t < n_out; ++t) {
      uint4 ol = make_uint4(gather_byte(acc_lo, 0, t), gather_byte(acc_lo, 1, t),
                            gather_byte(acc_lo, 2, t), gather_byte(acc_lo, 3, t));
      uint4 oh = make_uint4(gather_byte(acc_hi, 0, t), gather_byte(acc_hi, 1, t),
                            gather_byte(acc_hi, 2, t), gather_byte(acc_hi, 3, t));
      uint8_t *dst = P.out[t] + off;
      if (P.accumulate) {
        const uint4 pl = load16(dst), ph = load16(dst + 32);
        ol.x ^= pl.x; ol.y ^= pl.y; ol.z ^= pl.z; ol.w ^= pl.w;
        oh.x ^= ph.x; oh.y ^= ph.y; oh.z ^= ph.z; oh.w ^= ph.w;
      }
      *reinterpret_cast<uint4 *>(dst) = ol;
      *reinterpret_cast<uint4 *>(dst + 32) = oh;
    }
  }
}

// Tail chunk (shard_bytes % 64 = tb != 0): tb/2 symbols, low bytes at
// [base, base+tb/2), high bytes at [base+tb/2, base+tb) — the crate's tail rule.
// One workgroup per pass, one lane per symbol; rare and tiny.
__global__ __launch_bounds__(64) void gf_tail_kernel(const PassDesc *__restrict__ passes) {
  const PassDesc &P = passes[blockIdx.x];
  const uint32_t half = P.tail_bytes / 2;
  const uint32_t s = threadIdx.x;
  if (P.tail_bytes == 0 || s >= half) return;
  const uint64_t base = P.full_chunks * 64;
  uint32_t acc_lo = 0, acc_hi = 0;
  for (uint32_t i = 0; i < P.n_in; ++i) {
    const uint32_t lb = P.in[i][base + s], hb = P.in[i][base + half + s];
    const uint2 *T = P.table + i * 64;
    const uint2 e0 = T[lb & 15], e1 = T[16 + (lb >> 4)], e2 = T[32 + (hb & 15)],
                e3 = T[48 + (hb >> 4)];
    acc_lo ^= e0.x ^ e1.x ^ e2.x ^ e3.x;
    acc_hi ^= e0.y ^ e1.y ^ e2.y ^ e3.y;
  }
  for (uint32_t t = 0; t < P.n_out; ++t) {
    uint8_t *dst = P.out[t] + base;
    uint8_t vl = uint8_t(acc_lo >> (8 * t)), vh = uint8_t(acc_hi >> (8 * t));
    if (P.accumulate) {
      vl ^= dst[s];
      vh ^= dst[half + s];
    }
    dst[s] = vl;
    dst[half + s] = vh;
  }
}

}  // namespace

hipError_t launch_gf_apply(const PassDesc *d_passes, uint32_t n_passes, uint32_t n_wgs,
                           uint32_t tiles_per_wg, uint32_t max_in, hipStream_t stream) {
  if (n_wgs == 0) return hipSuccess;
  const size_t lds = size_t(max_in) * 64 * sizeof(uint2);
  hipLaunchKernelGGL(gf_apply_kernel, dim3(n_wgs), dim3(256), lds, stream, d_passes, n_passes,
                     tiles_per_wg);
  return hipGetLastError();
}

hipError_t launch_gf_tail(const PassDesc *d_passes, uint32_t n_passes, hipStream_t stream) {
  if (n_passes == 0) return hipSuccess;
  hipLaunchKernelGGL(gf_tail_kernel, dim3(n_passes), dim3(64), 0, stream, d_passes);
  return hipGetLastError();
}

}  // namespace bfrs
