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
// nibble tables.  One 8-byte table entry packs the products for up to 4
// outputs: low dword = the outputs' low bytes, high dword = their high bytes.
// A 16-entry x 8-byte table spans 32 LDS banks, so a ds_read_b64 with any
// nibble per lane is bank-conflict free.  Per symbol and input: 4 LDS lookups
// and ~10 VALU, independent of the number of outputs (<= 4).
//
// LDS table layout per input i (512 B): entry tab_idx(q, v) (kernels.hpp) at
// i*512 + nib_hi*256 + byte_hi*128 + v*8, q = 2*byte_hi + nib_hi (low/high
// nibble of the symbol's low/high byte).  Address of a lookup: byte 0 =
// byte_hi*128 + 8*v, bytes 1-2 = 2i + nib_hi.  Byte 0 for four symbols at once
// comes from one shift+mask(+or) of the data dword (nibble*8 per byte, bit 7 =
// byte_hi); one v_perm_b32 splices byte b of it under the wave-uniform
// 2i + nib_hi -> 1 VALU/lookup.  The two bytes' tables for one nibble half sit
// in disjoint banks, so lanes holding different bytes of their symbols (the
// contiguous layout) look up conflict-free.
#include "kernels.hpp"

#include <algorithm>

namespace bfrs {
namespace {

#define AS_GLOBAL __attribute__((address_space(1)))
#define AS_LDS __attribute__((address_space(3)))
#define AS_CONST __attribute__((address_space(4)))

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// LDS read at an absolute LDS byte address (the dynamic LDS table starts at 0:
// the kernel declares no static LDS).
__device__ __forceinline__ uint2 lds_entry(const char *, uint32_t byte_addr) {
  const uint64_t v = *(const AS_LDS uint64_t *)(uintptr_t)byte_addr;
  return make_uint2(uint32_t(v), uint32_t(v >> 32));
}

// Variant 0: straightforward indexing (kept for A/B).
__device__ __forceinline__ void mac_input_v0(const uint4 &L, const uint4 &H, const uint2 *T,
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
      const uint2 e0 = T[tab_idx(0, lb & 15)], e1 = T[tab_idx(1, lb >> 4)],
                  e2 = T[tab_idx(2, hb & 15)], e3 = T[tab_idx(3, hb >> 4)];
      acc_lo[s] ^= e0.x ^ e1.x ^ e2.x ^ e3.x;
      acc_hi[s] ^= e0.y ^ e1.y ^ e2.y ^ e3.y;
    }
  }
}

// Variant 1: v_perm addressing + 3-input XOR.  L/H: the two byte registers of
// 16 symbols; flag_l/flag_h: 0x80808080 for the register holding high bytes,
// 0 for low bytes; base_even = 2i, base_odd = 2i + 1.
__device__ __forceinline__ void mac_input_v1(const uint4 &L, const uint4 &H, uint32_t flag_l,
                                             uint32_t flag_h, uint32_t base_even,
                                             uint32_t base_odd, uint32_t (&acc_lo)[16],
                                             uint32_t (&acc_hi)[16]) {
  const uint32_t l[4] = {L.x, L.y, L.z, L.w};
  const uint32_t h[4] = {H.x, H.y, H.z, H.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t ll = ((l[d] << 3) & 0x78787878u) | flag_l;
    const uint32_t lh = ((l[d] >> 1) & 0x78787878u) | flag_l;
    const uint32_t hl = ((h[d] << 3) & 0x78787878u) | flag_h;
    const uint32_t hh = ((h[d] >> 1) & 0x78787878u) | flag_h;
    uint2 e[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      // selector: byte0 <- byte b of the nibble word, byte1..2 <- base, byte3 <- 0
      const uint32_t sel = 0x0C050400u | uint32_t(b);
      e[b][0] = lds_entry(nullptr, __builtin_amdgcn_perm(base_even, ll, sel));
      e[b][1] = lds_entry(nullptr, __builtin_amdgcn_perm(base_odd, lh, sel));
      e[b][2] = lds_entry(nullptr, __builtin_amdgcn_perm(base_even, hl, sel));
      e[b][3] = lds_entry(nullptr, __builtin_amdgcn_perm(base_odd, hh, sel));
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int s = d * 4 + b;
      acc_lo[s] = xor3(xor3(acc_lo[s], e[b][0].x, e[b][1].x), e[b][2].x, e[b][3].x);
      acc_hi[s] = xor3(xor3(acc_hi[s], e[b][0].y, e[b][1].y), e[b][2].y, e[b][3].y);
    }
  }
}

// Variant 9 (measurement only, NOT a codec): same memory traffic, no tables.
// The XORs are asm so the compiler cannot fold "0 ^ load" into a register
// copy of a load that is still in flight (tools/inflight_check.py).
__device__ __forceinline__ void mac_input_stream(const uint4 &L, const uint4 &H,
                                                 uint32_t (&acc_lo)[16], uint32_t (&acc_hi)[16]) {
  const uint32_t l[4] = {L.x, L.y, L.z, L.w};
  const uint32_t h[4] = {H.x, H.y, H.z, H.w};
#pragma unroll
  for (int d = 0; d < 4; ++d)
    asm volatile("v_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %3"
                 : "+v"(acc_lo[4 * d]), "+v"(acc_hi[4 * d])
                 : "v"(l[d]), "v"(h[d]));
}

// Byte t of acc[4d..4d+3] -> dword d of output t (4x4 byte transpose).
__device__ __forceinline__ uint32_t gather_byte(const uint32_t (&acc)[16], int d, int t) {
  const uint32_t sh = 8u * t;
  return ((acc[4 * d + 0] >> sh) & 0xFF) | (((acc[4 * d + 1] >> sh) & 0xFF) << 8) |
         (((acc[4 * d + 2] >> sh) & 0xFF) << 16) | (((acc[4 * d + 3] >> sh) & 0xFF) << 24);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 load16(uint64_t a) {
  const u32x4 v = *(const AS_GLOBAL u32x4 *)(uintptr_t)a;
  return make_uint4(v.x, v.y, v.z, v.w);
}


__device__ __forceinline__ void store16_nt(uint64_t a, const u32x4 &v) {
  __builtin_nontemporal_store(v, (AS_GLOBAL u32x4 *)(uintptr_t)a);
}

// Inline-asm streaming loads (see the pipeline comment in gf_apply_kernel).
// saddr form: 64-bit wave-uniform shard base in SGPRs + 32-bit lane offset.
// LPOL 1: non-temporal (streaming) cache policy on the loads.
template <int LPOL = 0>
__device__ __forceinline__ void gload_half_chunk(u32x4 &L, u32x4 &H, uint64_t base,
                                                 uint32_t voff) {
  if constexpr (LPOL == 1)
    asm volatile(
        "global_load_dwordx4 %0, %2, %3 nt\n\t"
        "global_load_dwordx4 %1, %2, %3 offset:32 nt"
        : "=&v"(L), "=&v"(H)
        : "v"(voff), "s"(base)
        : "memory");
  else
    asm volatile(
        "global_load_dwordx4 %0, %2, %3\n\t"
        "global_load_dwordx4 %1, %2, %3 offset:32"
        : "=&v"(L), "=&v"(H)
        : "v"(voff), "s"(base)
        : "memory");
}

__device__ __forceinline__ void store16(uint64_t a, const u32x4 &v) {
  *(AS_GLOBAL u32x4 *)(uintptr_t)a = v;
}
// Wait until at most N vector-memory ops are outstanding; L/H are in/out
// operands so no consumer can be scheduled above the wait.
template <int N>
__device__ __forceinline__ void vm_wait(u32x4 &L, u32x4 &H) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(L), "+v"(H) : "n"(N) : "memory");
}

template <int VARIANT>
__device__ __forceinline__ void mac_input(const u32x4 &Lv, const u32x4 &Hv, uint32_t i,
                                          uint32_t (&acc_lo)[16], uint32_t (&acc_hi)[16]) {
  const uint4 L = make_uint4(Lv.x, Lv.y, Lv.z, Lv.w), H = make_uint4(Hv.x, Hv.y, Hv.z, Hv.w);
  extern __shared__ __attribute__((aligned(16))) uint2 lds_table[];
  if constexpr (VARIANT == 0) {
    mac_input_v0(L, H, lds_table + i * 64, acc_lo, acc_hi);
  } else if constexpr (VARIANT == 9) {
    mac_input_stream(L, H, acc_lo, acc_hi);
  } else {  // 1, 3, 4
    mac_input_v1(L, H, 0u, 0x80808080u, 2 * i, 2 * i + 1, acc_lo, acc_hi);
  }
}

// VARIANT 1: default; 3 / 4: variant 1 compiled for >= 7 / 8 waves per SIMD.
// XCD-aware remap (speed only, never correctness): hardware deals workgroups
// round-robin over 8 XCDs; remap so XCD x works through a contiguous range of
// the grid.  Bijective for any grid size.
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7, q = b >> 3;
  const uint32_t per = n >> 3, rem = n & 7;
  // XCDs < rem own per+1 workgroups, the rest per
  const uint32_t start = x * per + min(x, rem);
  return start + q;
}

template <int VARIANT>
__global__ __launch_bounds__(256, VARIANT == 3 ? 7 : (VARIANT == 4 ? 8 : 1)) void gf_apply_kernel(
    const KernArgs args) {
  extern __shared__ __attribute__((aligned(16))) uint2 lds_table[];
  // Descriptors live in the kernarg segment: wave-uniform scalar loads.
  const PassDesc *passes = args.passes;
  const uint32_t n_passes = args.n_passes, tiles_per_wg = args.tiles_per_wg;

  // Locate this workgroup's pass (wave-uniform binary search over wg_begin).
  const uint32_t wg = VARIANT == 7 ? xcd_swizzle(blockIdx.x, gridDim.x) : blockIdx.x;
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
  const uint64_t *in = args.ptrs + P.in;

  // Table -> LDS: all loads issued before any store (n_in <= 64: <= 8 x 16 B per lane).
  {
    const AS_GLOBAL u32x4 *tab = (const AS_GLOBAL u32x4 *)(uintptr_t)P.table;
    u32x4 *dst = reinterpret_cast<u32x4 *>(lds_table);
    const uint32_t n16 = n_in * 32;
    u32x4 v[kMaxPassInputs * 32 / 256];
#pragma unroll
    for (int r = 0; r < int(kMaxPassInputs * 32 / 256); ++r) {
      const uint32_t e = threadIdx.x + 256u * r;
      v[r] = e < n16 ? tab[e] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int r = 0; r < int(kMaxPassInputs * 32 / 256); ++r) {
      const uint32_t e = threadIdx.x + 256u * r;
      if (e < n16) dst[e] = v[r];
    }
  }
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

    // Ping-pong software pipeline: input r' loads while input r computes.
    // Loads are inline asm with explicit vmcnt waits (hipcc otherwise sinks
    // prefetches next to their uses).  Each wave starts at a different input
    // (wave-uniform rotation) so concurrently running waves stream from
    // different shards; past the last input the prefetch re-reads the input
    // just loaded (a cache hit), so no guard is needed.  Passes with a
    // zero-table pad input (odd counts) keep rotation 0 so the pad's
    // duplicate pointer stays adjacent to its original.
    const uint32_t voff = uint32_t(off);
    const uint32_t wave_id = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t r = P.rotate ? (tile * 4 + wave_id) % n_in : 0;
    u32x4 La, Ha, Lb, Hb;
    gload_half_chunk(La, Ha, in[r], voff);
    for (uint32_t i = 0; i < n_in; i += 2) {
      const uint32_t r1 = r + 1 == n_in ? 0 : r + 1;
      gload_half_chunk(Lb, Hb, in[r1], voff);
      vm_wait<2>(La, Ha);
      mac_input<VARIANT>(La, Ha, r, acc_lo, acc_hi);
      const uint32_t r2 = i + 2 < n_in ? (r1 + 1 == n_in ? 0 : r1 + 1) : r1;
      gload_half_chunk(La, Ha, in[r2], voff);
      vm_wait<2>(Lb, Hb);
      mac_input<VARIANT>(Lb, Hb, r1, acc_lo, acc_hi);
      r = r2;
    }
    vm_wait<0>(La, Ha);  // drain the final (unused) prefetch

    const uint64_t *outp = args.ptrs + P.out;
    const bool accumulate = P.accumulate != 0;
    for (uint32_t t = 0; t < n_out; ++t) {
      uint4 ol = make_uint4(gather_byte(acc_lo, 0, t), gather_byte(acc_lo, 1, t),
                            gather_byte(acc_lo, 2, t), gather_byte(acc_lo, 3, t));
      uint4 oh = make_uint4(gather_byte(acc_hi, 0, t), gather_byte(acc_hi, 1, t),
                            gather_byte(acc_hi, 2, t), gather_byte(acc_hi, 3, t));
      const uint64_t dst = outp[t] + off;
      if (accumulate) {
        const uint4 pl = load16(dst), ph = load16(dst + 32);
        ol.x ^= pl.x; ol.y ^= pl.y; ol.z ^= pl.z; ol.w ^= pl.w;
        oh.x ^= ph.x; oh.y ^= ph.y; oh.z ^= ph.z; oh.w ^= ph.w;
      }
      store16_nt(dst, u32x4{ol.x, ol.y, ol.z, ol.w});
      store16_nt(dst + 32, u32x4{oh.x, oh.y, oh.z, oh.w});
    }
  }
}

// ---------------------------------------------------------------------------
// Variants 5 / 6: variant 1 with an NB-buffer ring (NB-1 inputs in flight per
// wave instead of 1).  The loop body is unrolled NB times with a uniform exit
// after every input, so no input padding is needed; past the last input the
// prefetch re-reads the last processed input (a cache hit, never consumed).
// ---------------------------------------------------------------------------
// Stages this workgroup's pass tables in LDS; returns the pass.
__device__ __forceinline__ const PassDesc &enter_pass(const KernArgs &args, uint32_t wg) {
  extern __shared__ __attribute__((aligned(16))) uint2 lds_table[];
  const PassDesc *passes = args.passes;
  uint32_t lo = 0, hi = args.n_passes;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (passes[mid].wg_begin <= wg)
      lo = mid;
    else
      hi = mid;
  }
  const PassDesc &P = passes[lo];
  const uint32_t n_in = P.n_in;
  const AS_GLOBAL u32x4 *tab = (const AS_GLOBAL u32x4 *)(uintptr_t)P.table;
  u32x4 *dst = reinterpret_cast<u32x4 *>(lds_table);
  const uint32_t n16 = n_in * 32;
  u32x4 v[kMaxPassInputs * 32 / 256];
#pragma unroll
  for (int r = 0; r < int(kMaxPassInputs * 32 / 256); ++r) {
    const uint32_t e = threadIdx.x + 256u * r;
    v[r] = e < n16 ? tab[e] : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int r = 0; r < int(kMaxPassInputs * 32 / 256); ++r) {
    const uint32_t e = threadIdx.x + 256u * r;
    if (e < n16) dst[e] = v[r];
  }
  __syncthreads();
  return P;
}

template <int SPOL>
__device__ __forceinline__ void store16_pol(uint64_t a, const u32x4 &v) {
  if constexpr (SPOL == 1)
    store16_nt(a, v);
  else
    store16(a, v);
}

// The 4-buffer input ring shared by both lane layouts: 3 inputs in flight per
// wave; n_in is even (host pads), uniform exits every 2 inputs keep the
// register allocation flat; past the last input the prefetch re-reads the
// last processed input (a cache hit, never consumed).
template <typename Load, typename Mac>
__device__ __forceinline__ void input_ring(uint32_t n_in, const Load &load, const Mac &mac) {
  u32x4 LA, HA, LB, HB, LC, HC, LD, HD;
  load(LA, HA, 0);
  load(LB, HB, 1);
  load(LC, HC, 2);
  for (uint32_t i = 0;; i += 4) {
    load(LD, HD, i + 3);
    vm_wait<6>(LA, HA);
    mac(LA, HA, i);
    load(LA, HA, i + 4);
    vm_wait<6>(LB, HB);
    mac(LB, HB, i + 1);
    if (i + 2 >= n_in) break;
    load(LB, HB, i + 5);
    vm_wait<6>(LC, HC);
    mac(LC, HC, i + 2);
    load(LC, HC, i + 6);
    vm_wait<6>(LD, HD);
    mac(LD, HD, i + 3);
    if (i + 4 >= n_in) break;
  }
  vm_wait<0>(LA, HA);
}

// LAYOUT 0 (v5): lane = one 32-byte half-chunk, 16 B at +0 (low bytes) and
// 16 B at +32 (high bytes): every 128-B line is touched by two instructions.
// Accumulates lane `lane` (0..255) of `tile`; false if the lane's half-chunk
// is past the last full chunk.  `off` = the half-chunk's shard byte offset.
template <int LPOL, int ROT = 0, bool PROBE = false>
__device__ __forceinline__ bool ring_acc_halfchunk(const KernArgs &args, const PassDesc &P,
                                                   uint32_t tile, uint32_t wave_id, uint32_t lane,
                                                   uint32_t (&acc_lo)[16], uint32_t (&acc_hi)[16],
                                                   uint32_t &off) {
  const uint32_t n_in = P.n_in;
  const uint64_t *in = args.ptrs + P.in;
  const uint64_t hc = uint64_t(tile) * kTileHalfChunks + lane;
  if (hc >= P.full_chunks * 2) return false;
  off = uint32_t((hc >> 1) * 64 + (hc & 1) * 16);
  const uint32_t voff = off;
#pragma unroll
  for (int s = 0; s < 16; ++s) acc_lo[s] = acc_hi[s] = 0;
  // input index of step x (x >= n_in: repeat the last input -> cache hit)
  // ROT 0: every wave of a tile starts at its own input; 1: the whole
  // workgroup starts at one input (tiles rotated); 2: no rotation.
  // ROT 3/4/5: groups of 2/4/8 consecutive tiles share a rotation.
  const uint32_t rot = !P.rotate || ROT == 2 ? 0
                       : ROT == 1           ? (tile * 4) % n_in
                       : ROT >= 3           ? ((tile >> (ROT - 2)) * 4) % n_in
                                            : (tile * 4 + wave_id) % n_in;
  auto idx = [&](uint32_t x) -> uint32_t {
    if (x >= n_in) x = n_in - 1;
    const uint32_t y = rot + x;
    return y >= n_in ? y - n_in : y;
  };
  input_ring(
      n_in, [&](u32x4 &L, u32x4 &H, uint32_t x) { gload_half_chunk<LPOL>(L, H, in[idx(x)], voff); },
      [&](const u32x4 &Lv, const u32x4 &Hv, uint32_t x) {
        const uint32_t r = idx(x);
        if constexpr (PROBE)  // traffic-only probe (measurement, NOT a codec)
          mac_input_stream(make_uint4(Lv.x, Lv.y, Lv.z, Lv.w), make_uint4(Hv.x, Hv.y, Hv.z, Hv.w),
                           acc_lo, acc_hi);
        else
          mac_input_v1(make_uint4(Lv.x, Lv.y, Lv.z, Lv.w), make_uint4(Hv.x, Hv.y, Hv.z, Hv.w),
                       0u, 0x80808080u, 2 * r, 2 * r + 1, acc_lo, acc_hi);
      });
  return true;
}

template <int LPOL, int SPOL, int ROT = 0, bool PROBE = false>
__device__ __forceinline__ void ring_tile_halfchunk(const KernArgs &args, const PassDesc &P,
                                                    uint32_t tile, uint32_t wave_id) {
  uint32_t acc_lo[16], acc_hi[16], off;
  if (!ring_acc_halfchunk<LPOL, ROT, PROBE>(args, P, tile, wave_id, threadIdx.x, acc_lo, acc_hi, off)) return;
  const uint32_t n_out = P.n_out;
  const uint64_t *outp = args.ptrs + P.out;
  const bool accumulate = P.accumulate != 0;
  for (uint32_t t = 0; t < n_out; ++t) {
    uint4 ol = make_uint4(gather_byte(acc_lo, 0, t), gather_byte(acc_lo, 1, t),
                          gather_byte(acc_lo, 2, t), gather_byte(acc_lo, 3, t));
    uint4 oh = make_uint4(gather_byte(acc_hi, 0, t), gather_byte(acc_hi, 1, t),
                          gather_byte(acc_hi, 2, t), gather_byte(acc_hi, 3, t));
    const uint64_t dst = outp[t] + off;
    if (accumulate) {
      const uint4 pl = load16(dst), ph = load16(dst + 32);
      ol.x ^= pl.x; ol.y ^= pl.y; ol.z ^= pl.z; ol.w ^= pl.w;
      oh.x ^= ph.x; oh.y ^= ph.y; oh.z ^= ph.z; oh.w ^= ph.w;
    }
    store16_pol<SPOL>(dst, u32x4{ol.x, ol.y, ol.z, ol.w});
    store16_pol<SPOL>(dst + 32, u32x4{oh.x, oh.y, oh.z, oh.w});
  }
}

// Two 16-B loads per input at per-lane offsets vx, vy (contiguous layout).
template <int LPOL>
__device__ __forceinline__ void gload_pair(u32x4 &X, u32x4 &Y, uint64_t base, uint32_t vx,
                                           uint32_t vy) {
  if constexpr (LPOL == 1)
    asm volatile(
        "global_load_dwordx4 %0, %2, %4 nt\n\t"
        "global_load_dwordx4 %1, %3, %4 nt"
        : "=&v"(X), "=&v"(Y)
        : "v"(vx), "v"(vy), "s"(base)
        : "memory");
  else
    asm volatile(
        "global_load_dwordx4 %0, %2, %4\n\t"
        "global_load_dwordx4 %1, %3, %4"
        : "=&v"(X), "=&v"(Y)
        : "v"(vx), "v"(vy), "s"(base)
        : "memory");
}

// Value of lane l^2 (DPP quad_perm [2,3,0,1]).
__device__ __forceinline__ u32x4 quad_swap2(const u32x4 &v) {
  u32x4 r;
  r.x = uint32_t(__builtin_amdgcn_update_dpp(0, int(v.x), 0x4E, 0xF, 0xF, false));
  r.y = uint32_t(__builtin_amdgcn_update_dpp(0, int(v.y), 0x4E, 0xF, 0xF, false));
  r.z = uint32_t(__builtin_amdgcn_update_dpp(0, int(v.z), 0x4E, 0xF, 0xF, false));
  r.w = uint32_t(__builtin_amdgcn_update_dpp(0, int(v.w), 0x4E, 0xF, 0xF, false));
  return r;
}

// LAYOUT 1: contiguous lines.  A wave's 2 KiB column span is read as two
// 1 KiB runs, lane l taking 16 B at +16l of each (whole 128-B lines per
// instruction).  Lane l = 4*c4 + p then holds part p of chunk c4 (first run)
// and of chunk 16+c4 (second run); parts 0/1 are low bytes, 2/3 high bytes
// of 16 symbols.  Lanes p < 2 load the first run into X, lanes p >= 2 the
// second, so one DPP quad swap of Y (lanes l <-> l^2) hands every lane the
// other byte of its own 16 symbols: p < 2 owns chunk c4 (X = low, R = high),
// p >= 2 owns chunk 16+c4 (X = high, R = low) and just flips the byte_hi bit
// of its table addresses (tab_idx layout: no bank conflicts between them).  Stores mirror it: a lane writes one of its output
// halves at vx and swaps the other to its partner, which writes it at vy.
// Needs all 64 lanes (DPP): only for waves whose span is all full chunks.
template <int LPOL, int SPOL>
__device__ __forceinline__ void ring_tile_contig(const KernArgs &args, const PassDesc &P,
                                                 uint32_t tile, uint32_t wave_id) {
  const uint32_t n_in = P.n_in, n_out = P.n_out;
  const uint64_t *in = args.ptrs + P.in;
  const uint32_t lane = threadIdx.x & 63, p = lane & 3;
  const bool lowp = p < 2;
  const uint32_t span = tile * (kTileHalfChunks * 32) + wave_id * 2048;
  const uint32_t vx = span + (lowp ? 0u : 1024u) + 16 * lane;
  const uint32_t vy = span + (lowp ? 1024u : 0u) + 16 * lane;
  // X holds low bytes (p < 2) or high bytes (p >= 2); R the other byte
  const uint32_t flag_x = lowp ? 0u : 0x80808080u, flag_r = flag_x ^ 0x80808080u;
  uint32_t acc_lo[16], acc_hi[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) acc_lo[s] = acc_hi[s] = 0;
  const uint32_t rot = P.rotate ? (tile * 4 + wave_id) % n_in : 0;
  auto idx = [&](uint32_t x) -> uint32_t {
    if (x >= n_in) x = n_in - 1;
    const uint32_t y = rot + x;
    return y >= n_in ? y - n_in : y;
  };
  input_ring(
      n_in, [&](u32x4 &X, u32x4 &Y, uint32_t x) { gload_pair<LPOL>(X, Y, in[idx(x)], vx, vy); },
      [&](const u32x4 &X, const u32x4 &Y, uint32_t x) {
        const uint32_t r = idx(x);
        const u32x4 R = quad_swap2(Y);
        mac_input_v1(make_uint4(X.x, X.y, X.z, X.w), make_uint4(R.x, R.y, R.z, R.w), flag_x,
                     flag_r, 2 * r, 2 * r + 1, acc_lo, acc_hi);
      });
  const uint64_t *outp = args.ptrs + P.out;
  const bool accumulate = P.accumulate != 0;
  for (uint32_t t = 0; t < n_out; ++t) {
    const u32x4 ol = {gather_byte(acc_lo, 0, t), gather_byte(acc_lo, 1, t),
                      gather_byte(acc_lo, 2, t), gather_byte(acc_lo, 3, t)};
    const u32x4 oh = {gather_byte(acc_hi, 0, t), gather_byte(acc_hi, 1, t),
                      gather_byte(acc_hi, 2, t), gather_byte(acc_hi, 3, t)};
    u32x4 own = lowp ? ol : oh;
    u32x4 other = quad_swap2(lowp ? oh : ol);
    const uint64_t base = outp[t];
    if (accumulate) {
      const uint4 a = load16(base + vx), b = load16(base + vy);
      own ^= u32x4{a.x, a.y, a.z, a.w};
      other ^= u32x4{b.x, b.y, b.z, b.w};
    }
    store16_pol<SPOL>(base + vx, own);
    store16_pol<SPOL>(base + vy, other);
  }
}

// Variants 5 / 10-15: the ring kernel.  LAYOUT 0 = half-chunk lanes (v5),
// LAYOUT 1 = contiguous lines + DPP (falls back to LAYOUT 0 for a wave whose
// span crosses the last full chunk).
template <int NB, int LPOL = 0, int SPOL = 1, int LAYOUT = 0, int MINW = 1, int ROT = 0,
          bool PROBE = false>
__global__ __launch_bounds__(256, MINW) void gf_apply_ring_kernel(const KernArgs args) {
  static_assert(NB == 3, "4-buffer ring");
  const uint32_t wg = blockIdx.x;
  const PassDesc &P = enter_pass(args, wg);
  const uint32_t t_begin = (wg - P.wg_begin) * args.tiles_per_wg;
  const uint32_t t_end = min(t_begin + args.tiles_per_wg, P.n_tiles);
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint32_t tile = t_begin; tile < t_end; ++tile) {
    if constexpr (LAYOUT == 1) {
      const uint64_t span_end = uint64_t(tile) * (kTileHalfChunks * 32) + (wave_id + 1) * 2048;
      if (span_end <= P.full_chunks * 64) {
        ring_tile_contig<LPOL, SPOL>(args, P, tile, wave_id);
        continue;
      }
    }
    ring_tile_halfchunk<LPOL, SPOL, ROT, PROBE>(args, P, tile, wave_id);
  }
}

// ---------------------------------------------------------------------------
// Phased variants (17+): persistent grid, one workgroup per CU, NW waves.
// The host cuts every pass into "super-tiles" of T consecutive 8 KiB tiles
// (PassDesc::wg_begin counts super-tiles, tiles_per_wg = T); workgroup b
// walks super-tiles b, b+G, b+2G, ...  Per super-tile: NW/4 groups of 4 waves
// compute the T tiles (same lanes, ring and arithmetic as v5) into an LDS
// image of the outputs in shard byte order, then the whole workgroup writes
// the image out as one contiguous T x 8 KiB run per output shard.
// Why: with 30 read streams in flight, the parity writes cost far more than
// their bytes when every wave stores its own 2 KiB pieces as it finishes
// (membench5/6: ~1.6 TB/s marginal); bunching a CU's writes into one burst of
// long contiguous runs per phase recovered ~7% in the traffic-only probe
// (membench6 "ph_*").  Output-major burst order: each output's T x 8 KiB run
// is written by consecutive lanes, whole lines per instruction.
// LDS: [0, n_in*512) pass tables (absolute addresses, as in v5), image at
// args.lds_image_off: [o][j][512 x 16 B].
// ---------------------------------------------------------------------------
template <int NW, int T, int SPOL>
__global__ __launch_bounds__(NW * 64) void gf_apply_phased_kernel(const KernArgs args,
                                                                 uint32_t n_virtual) {
  static_assert(NW % 4 == 0 && T % (NW / 4) == 0, "T tiles split evenly over NW/4 wave groups");
  extern __shared__ __attribute__((aligned(16))) uint2 lds_table[];
  u32x4 *img = reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds_table) + args.lds_image_off);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t grp = wave >> 2, w4 = wave & 3, lane = threadIdx.x & 255;
  uint32_t cur = ~0u;
  for (uint32_t v = blockIdx.x; v < n_virtual; v += gridDim.x) {
    uint32_t lo = 0, hi = args.n_passes;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (args.passes[mid].wg_begin <= v)
        lo = mid;
      else
        hi = mid;
    }
    const PassDesc &P = args.passes[lo];
    if (lo != cur) {  // stage this pass's tables (the image barrier below fenced the old ones)
      const AS_GLOBAL u32x4 *tab = (const AS_GLOBAL u32x4 *)(uintptr_t)P.table;
      u32x4 *dst = reinterpret_cast<u32x4 *>(lds_table);
      for (uint32_t e = threadIdx.x; e < P.n_in * 32; e += NW * 64) dst[e] = tab[e];
      __syncthreads();
      cur = lo;
    }
    const uint32_t n_out = P.n_out;
    const uint32_t t0 = (v - P.wg_begin) * T;
#pragma unroll 1
    for (uint32_t jj = 0; jj < T / (NW / 4); ++jj) {
      const uint32_t j = grp + jj * (NW / 4);
      const uint32_t tile = t0 + j;
      if (tile >= P.n_tiles) break;  // wave-uniform
      uint32_t acc_lo[16], acc_hi[16], off;
      if (!ring_acc_halfchunk<0>(args, P, tile, w4, lane, acc_lo, acc_hi, off)) continue;
      const uint32_t rel = (off & (kTileHalfChunks * 32 - 1)) >> 4;  // 16-B unit within the tile
      for (uint32_t t = 0; t < n_out; ++t) {
        u32x4 *d = img + (t * T + j) * 512 + rel;
        d[0] = u32x4{gather_byte(acc_lo, 0, t), gather_byte(acc_lo, 1, t),
                     gather_byte(acc_lo, 2, t), gather_byte(acc_lo, 3, t)};
        d[2] = u32x4{gather_byte(acc_hi, 0, t), gather_byte(acc_hi, 1, t),
                     gather_byte(acc_hi, 2, t), gather_byte(acc_hi, 3, t)};
      }
    }
    __syncthreads();  // image complete
    {
      const uint64_t *outp = args.ptrs + P.out;
      const uint64_t limit = P.full_chunks * 64;
      const uint64_t base = uint64_t(t0) * (kTileHalfChunks * 32);
      const bool accumulate = P.accumulate != 0;
      for (uint32_t e = threadIdx.x; e < n_out * T * 512; e += NW * 64) {
        const uint32_t o = e / (T * 512), rem = e - o * (T * 512);
        const uint64_t byte = base + uint64_t(rem) * 16;  // rem = j*512 + r: contiguous run
        if (byte >= limit) continue;
        u32x4 val = img[e];
        const uint64_t dst = outp[o] + byte;
        if (accumulate) {
          const uint4 pv = load16(dst);
          val ^= u32x4{pv.x, pv.y, pv.z, pv.w};
        }
        store16_pol<SPOL>(dst, val);
      }
    }
    __syncthreads();  // image consumed before the next super-tile overwrites it
  }
}

// ---------------------------------------------------------------------------
// Streamed variants (24-26): the phased layout (persistent grid, one
// workgroup per CU, super-tiles of T = NC/4 tiles, LDS output image written
// as one contiguous T x 8 KiB run per output) without the phased kernel's
// bubbles.  NC compute waves never store and never drain their input ring:
// it runs on across tiles, super-tiles and passes.  4 writer waves (one per
// SIMD) burst image n out while the compute waves read super-tile n+1.
// Two barriers per super-tile n, in every wave:
//   B1(n): the writers are done with image n-1 (the image is free);
//   B2(n): image n is complete (compute waves go on to n+1's arithmetic).
// Pass tables sit in two LDS slots of 16 KiB (n_in <= 32).  When the table
// changes between consecutive super-tiles n and n+1 of a workgroup (a new
// "run"), the writers store n+1's table into the other slot between B1(n)
// and B2(n): that slot's last reader finished before B1(n-1), and compute
// waves start n+1's arithmetic only after B2(n).  The table is prefetched
// into writer registers one super-tile earlier, so the barrier wait is short.
// LDS: [0, 32 KiB) table slots, [32 KiB, +n_out*T*8 KiB) image [o][j][512].
// Lookup addresses: perm base 2r + nib_hi + 64*slot -> slot*16 KiB + r*512.
// ---------------------------------------------------------------------------
constexpr uint32_t kSlotBytes = 16384;

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Next super-tile of this workgroup: pass and table-slot bookkeeping.
__device__ __forceinline__ bool stream_advance(const AS_CONST KernArgs *a, uint32_t n_virtual, uint32_t &v,
                                               uint32_t &p, uint32_t &slot) {
  const uint64_t tab = a->passes[p].table;
  v += gridDim.x;
  if (v >= n_virtual) return false;
  while (p + 1 < a->n_passes && a->passes[p + 1].wg_begin <= v) ++p;
  if (a->passes[p].table != tab) slot ^= 1;
  return true;
}

// Per-tile state of a compute group (wave-uniform).
struct TileDesc {
  uint32_t in;        // KernArgs::ptrs index of the pass inputs
  uint32_t n_in;      // ring steps: inputs rounded up to a multiple of 4
  uint32_t n_real;    // steps with arithmetic (the rest re-read the last input)
  uint32_t rot;       // first input of this wave (rotation)
  uint32_t slot;      // LDS table slot
  uint32_t tile_off;  // tile's first shard byte
  uint32_t max_off;   // last valid half-chunk offset (lanes past it re-read it)
  uint32_t valid;     // tile inside the pass (else a dummy, never written)
};

__device__ __forceinline__ TileDesc stream_tile(const AS_CONST KernArgs *a, uint32_t v, uint32_t p,
                                                uint32_t slot, uint32_t g, uint32_t w4,
                                                uint32_t T) {
  const AS_CONST PassDesc &P = a->passes[p];
  TileDesc d;
  uint32_t tile = (v - P.wg_begin) * T + g;
  d.valid = tile < P.n_tiles;
  if (!d.valid) tile = P.n_tiles - 1;
  d.in = uint32_t(P.in);
  d.n_in = (P.n_in + 3) & ~3u;  // pointer slots up to n_in + 3 hold the last input
  d.n_real = P.n_real;
  d.rot = P.rotate ? (tile * 4 + w4) % d.n_in : 0;
  d.slot = slot;
  d.tile_off = tile * (kTileHalfChunks * 32);
  d.max_off = uint32_t(P.full_chunks * 64 - 48);  // the last chunk's second half-chunk
  return d;
}

// Step x of the current tile; x >= n_in: step x - n_in of the next tile
// (past the last tile: the current tile's last step again, never consumed).
__device__ __forceinline__ void stream_load(const AS_CONST KernArgs *A, u32x4 &L, u32x4 &H,
                                            uint32_t x, const TileDesc cur, const TileDesc nxt,
                                            bool has_next, uint32_t lane_off) {
  const bool in_cur = x < cur.n_in;
  const bool use_cur = in_cur || !has_next;
  uint32_t y = in_cur ? x : (has_next ? x - cur.n_in : cur.n_in - 1);
  const uint32_t n_in = use_cur ? cur.n_in : nxt.n_in;
  const uint32_t rot = use_cur ? cur.rot : nxt.rot;
  const uint32_t in = use_cur ? cur.in : nxt.in;
  const uint32_t tile_off = use_cur ? cur.tile_off : nxt.tile_off;
  const uint32_t max_off = use_cur ? cur.max_off : nxt.max_off;
  if (y >= n_in) y = n_in - 1;
  uint32_t r = y + rot;
  if (r >= n_in) r -= n_in;
  const uint32_t voff = min(tile_off + lane_off, max_off);
  gload_half_chunk<0>(L, H, A->ptrs[in + r], voff);
}

template <bool PROBE>
__device__ __forceinline__ void stream_mac(const u32x4 &Lv, const u32x4 &Hv, uint32_t x,
                                           const TileDesc cur, uint32_t (&acc_lo)[16],
                                           uint32_t (&acc_hi)[16]) {
  if constexpr (PROBE) {
    // Traffic-only probe (measurement, NOT a codec).  The XORs are asm so the
    // compiler cannot fold "0 ^ load" into a register copy of a load that is
    // still in flight (tools/inflight_check.py).
#pragma unroll
    for (int d = 0; d < 4; ++d)
      asm volatile("v_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %3"
                   : "+v"(acc_lo[d]), "+v"(acc_hi[d])
                   : "v"(Lv[d]), "v"(Hv[d]));
    return;
  }
  uint32_t r = x + cur.rot;
  if (r >= cur.n_in) r -= cur.n_in;
  if (r >= cur.n_real) return;  // padding step (wave-uniform)
  const uint32_t b = 2 * r + 64 * cur.slot;
  mac_input_v1(make_uint4(Lv.x, Lv.y, Lv.z, Lv.w), make_uint4(Hv.x, Hv.y, Hv.z, Hv.w), 0u,
               0x80808080u, b, b + 1, acc_lo, acc_hi);
}

// The 4-buffer input ring of one tile, entered with steps 0..2 in flight in
// X0..X2; leaves the next tile's steps 0..2 in flight in X0..X2.  Every tile
// has a multiple of 4 steps, so a tile always starts on the same buffer: two
// ring entry points (buffer rotations) would make the compiler reconcile
// register assignments with copies of registers whose loads are still in
// flight (asm loads are invisible to it) -- a race.
template <bool PROBE>
__device__ __forceinline__ void stream_ring(const AS_CONST KernArgs *A, const TileDesc cur,
                                            const TileDesc nxt, bool has_next, uint32_t lane_off,
                                            u32x4 &L0, u32x4 &H0, u32x4 &L1, u32x4 &H1,
                                            u32x4 &L2, u32x4 &H2, u32x4 &L3, u32x4 &H3,
                                            uint32_t (&acc_lo)[16], uint32_t (&acc_hi)[16]) {
  const uint32_t n_in = cur.n_in;
  for (uint32_t i = 0;; i += 4) {
    stream_load(A, L3, H3, i + 3, cur, nxt, has_next, lane_off);
    vm_wait<6>(L0, H0);
    stream_mac<PROBE>(L0, H0, i, cur, acc_lo, acc_hi);
    stream_load(A, L0, H0, i + 4, cur, nxt, has_next, lane_off);
    vm_wait<6>(L1, H1);
    stream_mac<PROBE>(L1, H1, i + 1, cur, acc_lo, acc_hi);
    stream_load(A, L1, H1, i + 5, cur, nxt, has_next, lane_off);
    vm_wait<6>(L2, H2);
    stream_mac<PROBE>(L2, H2, i + 2, cur, acc_lo, acc_hi);
    stream_load(A, L2, H2, i + 6, cur, nxt, has_next, lane_off);
    vm_wait<6>(L3, H3);
    stream_mac<PROBE>(L3, H3, i + 3, cur, acc_lo, acc_hi);
    if (i + 4 >= n_in) break;
  }
}

template <int NC, int SPOL, bool PROBE = false>
__global__ __launch_bounds__((NC + 4) * 64) void gf_apply_stream_kernel(const KernArgs args,
                                                                       uint32_t n_virtual) {
  static_assert(NC % 4 == 0, "whole 4-wave groups");
  constexpr uint32_t T = NC / 4;
  // Descriptors are read through the kernarg segment pointer (scalar loads):
  // taking the address of the by-value parameter would copy 4 KiB to scratch.
  const AS_CONST KernArgs *A = (const AS_CONST KernArgs *)__builtin_amdgcn_kernarg_segment_ptr();
  extern __shared__ __attribute__((aligned(16))) uint2 lds_table[];
  u32x4 *img = reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds_table) + 2 * kSlotBytes);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t v0 = blockIdx.x;
  uint32_t p0 = 0;
  while (p0 + 1 < A->n_passes && A->passes[p0 + 1].wg_begin <= v0) ++p0;
  {  // first run's table -> slot 0 (every wave)
    const AS_CONST PassDesc &P = A->passes[p0];
    const AS_GLOBAL u32x4 *tab = (const AS_GLOBAL u32x4 *)(uintptr_t)P.table;
    u32x4 *dst = reinterpret_cast<u32x4 *>(lds_table);
    for (uint32_t e = threadIdx.x; e < P.n_in * 32; e += (NC + 4) * 64) dst[e] = tab[e];
  }
  lds_barrier();

  if (wave >= NC) {
    // ---------------- writer waves ----------------
    const uint32_t wl = threadIdx.x - NC * 64;  // 0..255
    uint32_t v = v0, p = p0, slot = 0;
    // successor state (n+1) and the table prefetched for it
    uint32_t vn = v, pn = p, slotn = slot;
    bool has_next = stream_advance(A, n_virtual, vn, pn, slotn);
    bool pending = has_next && slotn != slot;
    u32x4 pre[4];
    auto prefetch = [&](const AS_CONST PassDesc &Q) {
      const AS_GLOBAL u32x4 *tab = (const AS_GLOBAL u32x4 *)(uintptr_t)Q.table;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t e = wl + 256u * r;
        pre[r] = e < Q.n_in * 32 ? tab[e] : u32x4{0, 0, 0, 0};
      }
    };
    if (pending) prefetch(A->passes[pn]);
    for (;;) {
      asm volatile("s_barrier" ::: "memory");  // B1(n)
      if (pending) {
        u32x4 *dst = reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds_table) + slotn * kSlotBytes);
        const uint32_t n16 = A->passes[pn].n_in * 32;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t e = wl + 256u * r;
          if (e < n16) dst[e] = pre[r];
        }
      }
      lds_barrier();  // B2(n)
      // prefetch the table of n+2 if a new run starts there
      uint32_t vnn = vn, pnn = pn, slotnn = slotn;
      const bool has_nn = has_next && stream_advance(A, n_virtual, vnn, pnn, slotnn);
      const bool pending_nn = has_nn && slotnn != slotn;
      if (pending_nn) prefetch(A->passes[pnn]);
      {  // burst image n: output-major, each output's T x 8 KiB run contiguous
        const AS_CONST PassDesc &P = A->passes[p];
        const uint32_t n_out = P.n_out;
        const uint32_t t0 = (v - P.wg_begin) * T;
        const AS_CONST uint64_t *outp = A->ptrs + P.out;
        const uint64_t limit = P.full_chunks * 64;
        const uint64_t base = uint64_t(t0) * (kTileHalfChunks * 32);
        const bool accumulate = P.accumulate != 0;
        for (uint32_t e = wl; e < n_out * T * 512; e += 256) {
          const uint32_t o = e / (T * 512), rem = e - o * (T * 512);
          const uint64_t byte = base + uint64_t(rem) * 16;
          if (byte >= limit) continue;
          u32x4 val = img[e];
          const uint64_t dst = outp[o] + byte;
          if (accumulate) {
            const uint4 pv = load16(dst);
            val ^= u32x4{pv.x, pv.y, pv.z, pv.w};
          }
          store16_pol<SPOL>(dst, val);
        }
      }
      if (!has_next) break;
      v = vn; p = pn; slot = slotn;
      vn = vnn; pn = pnn; slotn = slotnn;
      has_next = has_nn;
      pending = pending_nn;
    }
    return;
  }

  // ---------------- compute waves ----------------
  // One tile per super-tile per 4-wave group.  The input ring of a tile
  // prefetches the first 3 inputs of the group's next tile, so it never
  // drains.
  const uint32_t g = wave >> 2, w4 = wave & 3, lane = threadIdx.x & 255;
  const uint32_t lane_off = (lane >> 1) * 64 + (lane & 1) * 16;
  TileDesc cur = stream_tile(A, v0, p0, 0, g, w4, T);
  uint32_t v = v0, p = p0, slot = 0;
  uint32_t vn = v, pn = p, slotn = slot;
  bool has_next = stream_advance(A, n_virtual, vn, pn, slotn);
  TileDesc nxt = has_next ? stream_tile(A, vn, pn, slotn, g, w4, T) : cur;
  uint32_t acc_lo[16], acc_hi[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) acc_lo[s] = acc_hi[s] = 0;
  u32x4 LA, HA, LB, HB, LC, HC, LD, HD;
  stream_load(A, LA, HA, 0, cur, nxt, has_next, lane_off);
  stream_load(A, LB, HB, 1, cur, nxt, has_next, lane_off);
  stream_load(A, LC, HC, 2, cur, nxt, has_next, lane_off);
  for (;;) {
    stream_ring<PROBE>(A, cur, nxt, has_next, lane_off, LA, HA, LB, HB, LC, HC, LD, HD, acc_lo, acc_hi);
    asm volatile("s_barrier" ::: "memory");  // B1(n): image free
    if (cur.valid) {
      const AS_CONST PassDesc &P = A->passes[p];
      if (cur.tile_off + lane_off < P.full_chunks * 64) {
        const uint32_t rel = lane_off >> 4;  // 16-B unit within the tile
        for (uint32_t t = 0; t < P.n_out; ++t) {
          u32x4 *d = img + (t * T + g) * 512 + rel;
          d[0] = u32x4{gather_byte(acc_lo, 0, t), gather_byte(acc_lo, 1, t),
                       gather_byte(acc_lo, 2, t), gather_byte(acc_lo, 3, t)};
          d[2] = u32x4{gather_byte(acc_hi, 0, t), gather_byte(acc_hi, 1, t),
                       gather_byte(acc_hi, 2, t), gather_byte(acc_hi, 3, t)};
        }
      }
    }
    lds_barrier();  // B2(n): image complete
#pragma unroll
    for (int s = 0; s < 16; ++s) acc_lo[s] = acc_hi[s] = 0;
    if (!has_next) break;
    cur = nxt;
    v = vn; p = pn; slot = slotn;
    has_next = stream_advance(A, n_virtual, vn, pn, slotn);
    if (has_next) nxt = stream_tile(A, vn, pn, slotn, g, w4, T);
  }
  vm_wait<0>(LA, HA);
}

// Tail chunk (shard_bytes % 64 = tb != 0): tb/2 symbols, low bytes at
// [base, base+tb/2), high bytes at [base+tb/2, base+tb) — the crate's tail rule.
// One workgroup per pass, one lane per symbol; rare and tiny.
__global__ __launch_bounds__(64) void gf_tail_kernel(const KernArgs args) {
  const PassDesc &P = args.passes[blockIdx.x];
  const uint32_t half = P.tail_bytes / 2;
  const uint32_t s = threadIdx.x;
  if (P.tail_bytes == 0 || s >= half) return;
  const uint64_t base = P.full_chunks * 64;
  uint32_t acc_lo = 0, acc_hi = 0;
  const uint64_t *in = args.ptrs + P.in;
  const uint64_t *outp = args.ptrs + P.out;
  for (uint32_t i = 0; i < P.n_in; ++i) {
    const uint8_t *src = (const uint8_t *)(uintptr_t)in[i];
    const uint32_t lb = src[base + s], hb = src[base + half + s];
    const uint2 *T = (const uint2 *)(uintptr_t)P.table + i * 64;
    const uint2 e0 = T[tab_idx(0, lb & 15)], e1 = T[tab_idx(1, lb >> 4)],
                e2 = T[tab_idx(2, hb & 15)], e3 = T[tab_idx(3, hb >> 4)];
    acc_lo ^= e0.x ^ e1.x ^ e2.x ^ e3.x;
    acc_hi ^= e0.y ^ e1.y ^ e2.y ^ e3.y;
  }
  for (uint32_t t = 0; t < P.n_out; ++t) {
    uint8_t *dst = (uint8_t *)(uintptr_t)outp[t] + base;
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

// Kernel variant selector for A/B measurement (tools/kbench.py).  Variant 9
// is a traffic-only probe and is refused unless BFRS_ALLOW_PROBE=1.
int kernel_variant() {
  const char *e = std::getenv("BFRS_KERNEL_VARIANT");
  int v = e ? atoi(e) : 41;
  if ((v == 9 || v == 27 || v == 44) && !std::getenv("BFRS_ALLOW_PROBE")) v = 1;
  return v;
}

// Variants: 41 (default) = 5 with one input rotation per group of 16
// consecutive tiles (the 16 workgroups read one shard's 128 KiB together);
// 36 / 38 / 39 / 40 / 42 = the same with groups of 1 / 2 / 4 / 8 / 32 tiles;
// 37 = no rotation; 43 = 41 built for >= 6 waves per SIMD; 44 = traffic-only
// probe of 41 (refused unless BFRS_ALLOW_PROBE=1); 5 = v1 arithmetic with a 4-buffer ring (3 inputs in flight per wave, each
// wave of a tile starting at its own input); 1 = ping-pong (1 in flight); 0 = naive indexing;
// 3/4 = occupancy-bounded builds of 1; 7 = 1 with
// an XCD-aware grid remap; 9 = traffic-only probe (refused unless
// BFRS_ALLOW_PROBE=1); 10/11/12 = 5 with nt loads / nt loads + plain stores /
// plain stores; 13/14/15 = contiguous-line layout (DPP quad swap) with nt
// loads + nt stores / plain loads + nt stores / nt loads + plain stores;
// 16 = contiguous-line layout with plain loads + plain stores; 28 = 5 built
// for >= 6 waves per SIMD (80 VGPRs).  Results of each: DESIGN.md §9.
uint32_t tile_bytes() { return kTileHalfChunks * 32; }

// Phased variants (waves x tiles per super-tile; grid = CUs x occupancy):
// 17 = 16 x 4, 21 = 4 x 1.  Streamed (writer-wave) variants, + 4 writer
// waves: 24 = 12 compute waves x 3 tiles; 27 = traffic-only probe of 24
// (refused unless BFRS_ALLOW_PROBE=1).  Results: DESIGN.md §9.
static uint32_t phased_T(int v) {
  switch (v) {
    case 17: return 4;
    case 21: return 1;
    case 24: case 27: return 3;
    default: return 0;
  }
}
uint32_t phased_tiles() { return phased_T(kernel_variant()); }

static int device_cus() {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

template <int NW, int T, int SPOL>
static hipError_t launch_phased(const KernArgs &args, uint32_t n_virtual, uint32_t max_in,
                                uint32_t max_out, hipStream_t stream) {
  KernArgs a = args;
  a.lds_image_off = max_in * 64 * sizeof(uint2);
  const size_t lds = a.lds_image_off + size_t(max_out) * T * kTileHalfChunks * 32;
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gf_apply_phased_kernel<NW, T, SPOL>,
                                                   NW * 64, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const uint32_t grid = std::min<uint32_t>(n_virtual, uint32_t(device_cus() * per_cu));
  hipLaunchKernelGGL((gf_apply_phased_kernel<NW, T, SPOL>), dim3(grid), dim3(NW * 64), lds, stream,
                     a, n_virtual);
  return hipGetLastError();
}

template <int NC, int SPOL, bool PROBE = false>
static hipError_t launch_stream(const KernArgs &args, uint32_t n_virtual, uint32_t max_in,
                                uint32_t max_out, hipStream_t stream) {
  constexpr uint32_t T = NC / 4;
  const size_t lds = 2 * kSlotBytes + size_t(max_out) * T * kTileHalfChunks * 32;
  if (max_in > kSlotBytes / 512 || lds > 160 * 1024) {
    // Outside the streamed layout (tables > one slot, image too large): the
    // ring kernel reads the same descriptors (tiles_per_wg = T, one
    // workgroup per super-tile).
    hipLaunchKernelGGL((gf_apply_ring_kernel<3>), dim3(n_virtual), dim3(256),
                       size_t(max_in) * 64 * sizeof(uint2), stream, args);
    return hipGetLastError();
  }
  const uint32_t grid = std::min<uint32_t>(n_virtual, uint32_t(device_cus()));
  hipLaunchKernelGGL((gf_apply_stream_kernel<NC, SPOL, PROBE>), dim3(grid), dim3((NC + 4) * 64), lds,
                     stream, args, n_virtual);
  return hipGetLastError();
}

hipError_t launch_gf_apply(const KernArgs &args, uint32_t n_wgs, uint32_t max_in,
                           hipStream_t stream) {
  if (n_wgs == 0) return hipSuccess;
  const size_t lds = size_t(max_in) * 64 * sizeof(uint2);
  const int variant = kernel_variant();
  if (phased_T(variant)) {
    uint32_t max_out = 0;
    for (uint32_t p = 0; p < args.n_passes; ++p) max_out = std::max(max_out, args.passes[p].n_out);
    switch (variant) {
      case 17: return launch_phased<16, 4, 1>(args, n_wgs, max_in, max_out, stream);
      case 21: return launch_phased<4, 1, 1>(args, n_wgs, max_in, max_out, stream);
      case 24: return launch_stream<12, 1>(args, n_wgs, max_in, max_out, stream);
      default: return launch_stream<12, 1, true>(args, n_wgs, max_in, max_out, stream);
    }
  }
  switch (variant) {
    case 0:
      hipLaunchKernelGGL(gf_apply_kernel<0>, dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 9:
      hipLaunchKernelGGL(gf_apply_kernel<9>, dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 1:
      hipLaunchKernelGGL(gf_apply_kernel<1>, dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 3:
      hipLaunchKernelGGL(gf_apply_kernel<3>, dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 4:
      hipLaunchKernelGGL(gf_apply_kernel<4>, dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 7:
      hipLaunchKernelGGL(gf_apply_kernel<7>, dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 10:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 11:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 1, 0>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 12:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 0>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 13:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 1, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 14:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 15:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 1, 0, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 16:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 0, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 36:  // v5, one rotation per workgroup (all 4 waves read one input)
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 38:  // 36 with one rotation per 2 / 4 / 8 consecutive tiles
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 1, 3>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 39:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 1, 4>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 40:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 1, 5>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 41:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 1, 6>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 42:
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 1, 7>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 44:  // traffic-only probe of 41 (refused unless BFRS_ALLOW_PROBE=1)
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 1, 6, true>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 43:  // 41 built for >= 6 waves per SIMD
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 6, 6>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 37:  // v5 without rotation
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 1, 2>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 28:  // v5 built for >= 6 waves per SIMD
      hipLaunchKernelGGL((gf_apply_ring_kernel<3, 0, 1, 0, 6>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    default:  // 5
      hipLaunchKernelGGL((gf_apply_ring_kernel<3>), dim3(n_wgs), dim3(256), lds, stream, args);
  }
  return hipGetLastError();
}

hipError_t launch_gf_tail(const KernArgs &args, hipStream_t stream) {
  if (args.n_passes == 0) return hipSuccess;
  hipLaunchKernelGGL(gf_tail_kernel, dim3(args.n_passes), dim3(64), 0, stream, args);
  return hipGetLastError();
}

}  // namespace bfrs
