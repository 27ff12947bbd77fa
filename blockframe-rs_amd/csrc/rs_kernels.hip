// rs_kernels.hip — gfx950 kernels for the BlockFrame Reed-Solomon path.
//
// Replaces the arithmetic of reed-solomon-simd's encode()/decode() (called at
// src/chunker/generate.rs:92 and src/filestore/recovery.rs:166) with one HBM
// pass per RS block: every output shard is sum_i coef(t,i) * input_i over
// GF(2^16), coefficients from plan.cpp.
//
// Data layout (crate's): a shard is a run of 64-byte chunks; chunk
// c holds 32 symbols, low bytes at [64c, 64c+32), high bytes at [64c+32, 64c+64).
// Work unit: a lane owns 16 symbols (16 low + 16 high bytes).  A 256-lane
// workgroup tile covers 8 KiB of columns of every shard of a block.  The
// default kernel (v76, gf_apply_unrolled_kernel) loads whole 1 KiB lines per
// instruction and regroups halves with v_permlane32_swap (ring_acc_ct); the
// round-1 kernels load a lane's two 16-B halves directly (ring_acc_halfchunk).
//
// Arithmetic: multiplication of a 16-bit symbol by a constant is GF(2)-linear,
// so coef*x = T0[x&15] ^ T1[(x>>4)&15] ^ T2[(x>>8)&15] ^ T3[x>>12] with 16-entry
// nibble tables.  One 8-byte table entry packs the products for up to 4
// outputs: low dword = the outputs' low bytes, high dword = their high bytes.
// A 16-entry x 8-byte table spans 32 LDS banks, so a ds_read_b64 with any
// nibble per lane is bank-conflict free.  Per symbol and input: 4 LDS lookups
// and, in v76 (GF(2^8)-subfield coefficients), 4 SDWA address ops + 3 XORs,
// independent of the number of outputs (<= 4).  DESIGN.md §4.
//
// LDS table layout per input i (512 B, tab_idx in kernels.hpp): high-nibble
// entries at i*512 + 16*v + 8*byte_hi, low-nibble entries at i*512 + 256 +
// 16*v + 8*byte_hi (q = 2*byte_hi + nib_hi: low/high nibble of the symbol's
// low/high byte).  Looped kernels: a lookup address is byte 0 = the offset
// within the 256-B half, bytes 1-2 = 2i + (low nibble).  Byte 0 for four
// symbols at once is one mask of the data dword for high nibbles (x & 0xF0,
// | 8 for the high byte: one v_bitop3) and a shift + mask for low nibbles
// ((x << 4) & 0xF0, | 8 for the high byte); one v_perm_b32 splices byte b of it
// under the wave-uniform 2i + (low nibble) -> 1 VALU per lookup.  The unrolled
// kernel (tile_unrolled) needs no mask: one SDWA op per lookup straight from
// the data byte, the input's table base in the ds_read immediate.
#include "kernels.hpp"

#include <algorithm>
#include <utility>

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

// GF multiply-accumulate of one input into 16 symbols: v_perm addressing +
// 3-input XOR.  L/H: the low-byte and high-byte registers of the lane's 16
// symbols; base_hi = 2i (high-nibble half of input i's table), base_lo =
// 2i + 1 (low-nibble half).
__device__ __forceinline__ void mac_input_v1(const uint4 &L, const uint4 &H, uint32_t base_hi,
                                             uint32_t base_lo, uint32_t (&acc_lo)[16],
                                             uint32_t (&acc_hi)[16]) {
  const uint32_t l[4] = {L.x, L.y, L.z, L.w};
  const uint32_t h[4] = {H.x, H.y, H.z, H.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    // address bytes of 4 symbols; (x & M) | F is one v_bitop3 (0xEA)
    const uint32_t ll = (l[d] << 4) & 0xF0F0F0F0u;                                    // 16*v
    const uint32_t lh = l[d] & 0xF0F0F0F0u;                                           // 16*v
    const uint32_t hl = __builtin_amdgcn_bitop3_b32(h[d] << 4, 0xF0F0F0F0u, 0x08080808u, 0xEA);
    const uint32_t hh = __builtin_amdgcn_bitop3_b32(h[d], 0xF0F0F0F0u, 0x08080808u, 0xEA);
    uint2 e[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      // selector: byte0 <- byte b of the nibble word, byte1..2 <- base, byte3 <- 0
      const uint32_t sel = 0x0C050400u | uint32_t(b);
      e[b][0] = lds_entry(nullptr, __builtin_amdgcn_perm(base_lo, ll, sel));
      e[b][1] = lds_entry(nullptr, __builtin_amdgcn_perm(base_hi, lh, sel));
      e[b][2] = lds_entry(nullptr, __builtin_amdgcn_perm(base_lo, hl, sel));
      e[b][3] = lds_entry(nullptr, __builtin_amdgcn_perm(base_hi, hh, sel));
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int s = d * 4 + b;
      acc_lo[s] = xor3(xor3(acc_lo[s], e[b][0].x, e[b][1].x), e[b][2].x, e[b][3].x);
      acc_hi[s] = xor3(xor3(acc_hi[s], e[b][0].y, e[b][1].y), e[b][2].y, e[b][3].y);
    }
  }
}

__device__ __forceinline__ uint32_t lds_entry32(uint32_t byte_addr) {
  return *(const AS_LDS uint32_t *)(uintptr_t)byte_addr;
}

// mac_input_v1 for passes whose coefficients all lie in the GF(2^8) subfield
// (every RS(k<=30, 3) encode and decode; PlanPass::subfield).  There the
// product of a symbol's low byte has a zero high byte (the high
// output byte depends on the high input bytes only), so the two low-byte
// lookups read only the 4-byte low half of their entries and the high
// accumulator takes one 3-input XOR per symbol instead of two: 3 XORs per
// symbol and input instead of 4 (-16 VALU per input and lane; the kernel is
// VALU-bound, profiles/r02/).  Same table layout and addresses.
__device__ __forceinline__ void mac_input_sub(const uint4 &L, const uint4 &H, uint32_t base_hi,
                                              uint32_t base_lo, uint32_t (&acc_lo)[16],
                                              uint32_t (&acc_hi)[16]) {
  const uint32_t l[4] = {L.x, L.y, L.z, L.w};
  const uint32_t h[4] = {H.x, H.y, H.z, H.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t ll = (l[d] << 4) & 0xF0F0F0F0u;
    const uint32_t lh = l[d] & 0xF0F0F0F0u;
    const uint32_t hl = __builtin_amdgcn_bitop3_b32(h[d] << 4, 0xF0F0F0F0u, 0x08080808u, 0xEA);
    const uint32_t hh = __builtin_amdgcn_bitop3_b32(h[d], 0xF0F0F0F0u, 0x08080808u, 0xEA);
    uint32_t a[4], b[4];
    uint2 e2[4], e3[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t sel = 0x0C050400u | uint32_t(k);
      a[k] = lds_entry32(__builtin_amdgcn_perm(base_lo, ll, sel));
      b[k] = lds_entry32(__builtin_amdgcn_perm(base_hi, lh, sel));
      e2[k] = lds_entry(nullptr, __builtin_amdgcn_perm(base_lo, hl, sel));
      e3[k] = lds_entry(nullptr, __builtin_amdgcn_perm(base_hi, hh, sel));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int s = d * 4 + k;
      acc_lo[s] = xor3(xor3(acc_lo[s], a[k], b[k]), e2[k].x, e3[k].x);
      acc_hi[s] = xor3(acc_hi[s], e2[k].y, e3[k].y);
    }
  }
}

#ifdef BFRS_AB_VARIANTS
// Traffic-only probe (measurement only, NOT a codec): same memory traffic, no tables.
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
#endif  // BFRS_AB_VARIANTS

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// In-place 4x4 byte transpose of every group acc[4d..4d+3]: afterwards
// acc[4d + t] holds byte t (output t) of the four symbols 4d..4d+3, i.e. the
// dword gather_byte(acc, d, t) builds.  8 v_perm per group instead of ~28
// shift/mask/or ops of the four gather_byte calls.
__device__ __forceinline__ void transpose_outputs(uint32_t (&acc)[16]) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint32_t *a = acc + 4 * d;
    const uint32_t x0 = __builtin_amdgcn_perm(a[1], a[0], 0x05010400u);  // a0.0 a1.0 a0.1 a1.1
    const uint32_t x1 = __builtin_amdgcn_perm(a[1], a[0], 0x07030602u);  // a0.2 a1.2 a0.3 a1.3
    const uint32_t y0 = __builtin_amdgcn_perm(a[3], a[2], 0x05010400u);
    const uint32_t y1 = __builtin_amdgcn_perm(a[3], a[2], 0x07030602u);
    a[0] = __builtin_amdgcn_perm(y0, x0, 0x05040100u);  // byte 0 of a0..a3
    a[1] = __builtin_amdgcn_perm(y0, x0, 0x07060302u);  // byte 1
    a[2] = __builtin_amdgcn_perm(y1, x1, 0x05040100u);  // byte 2
    a[3] = __builtin_amdgcn_perm(y1, x1, 0x07060302u);  // byte 3
  }
}

__device__ __forceinline__ uint4 load16(uint64_t a) {
  const u32x4 v = *(const AS_GLOBAL u32x4 *)(uintptr_t)a;
  return make_uint4(v.x, v.y, v.z, v.w);
}


__device__ __forceinline__ void store16_nt(uint64_t a, const u32x4 &v) {
  __builtin_nontemporal_store(v, (AS_GLOBAL u32x4 *)(uintptr_t)a);
}

// Inline-asm streaming loads, waited for by a separate vm_wait asm: hipcc
// otherwise sinks a prefetch next to its first use, which serialises the
// ring.  saddr form: 64-bit wave-uniform shard base in SGPRs +
// 32-bit lane offset.  The compiler does not know an asm output is written
// asynchronously, so no code may copy or spill a destination register before
// its wait (tools/inflight_check.py, tests/test_isa_hazards.py).
#ifdef BFRS_AB_VARIANTS  // round-1 half-chunk layout (A/B build only)
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

#endif  // BFRS_AB_VARIANTS

// Wait until at most N vector-memory ops are outstanding; L/H are in/out
// operands so no consumer can be scheduled above the wait.
template <int N>
__device__ __forceinline__ void vm_wait(u32x4 &L, u32x4 &H) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(L), "+v"(H) : "n"(N) : "memory");
}

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
    *(AS_GLOBAL u32x4 *)(uintptr_t)a = v;
}

// The 4-buffer input ring: 3 inputs in flight per wave; n_in is even (host pads), uniform exits every 2 inputs keep the
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

#ifdef BFRS_AB_VARIANTS  // round-1 half-chunk layout (A/B build only)
// Lane layout: lane = one 32-byte half-chunk, 16 B at +0 (low bytes) and
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
  // Input of step x (x >= n_in: repeat the last input -> cache hit).  Read
  // order ROT: 0 = every wave of a tile starts at its own input; 1 = the
  // whole workgroup starts at one input; 2 = no rotation; g >= 3 = groups of
  // 2^(g-2) consecutive tiles share one starting input, so their workgroups
  // (dealt over the XCDs together) stream one shard's contiguous columns at
  // the same time (6 = 16 tiles = 128 KiB, the default).
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
                       2 * r, 2 * r + 1, acc_lo, acc_hi);
      });
  return true;
}

#endif  // BFRS_AB_VARIANTS

// ---- contiguous-line layout (LAY 1, round 2) --------------------------------
// Every load / store instruction covers 1 KiB of contiguous columns (16 whole
// 64-byte chunks = 8 whole 128-B lines), so each HBM line is fetched by one
// instruction: the half-chunk layout above touches every line with two
// instructions (32 B of each chunk each), which costs 7% of the memory
// system's rate in the traffic-only probes and doubles the fetch with `nt`
// loads (tools/membench8.hip, profiles/r02/).  A wave covers 2 KiB = 32
// chunks per input: load A = chunks 0..15, load B = chunks 16..31.  Lanes
// 0-31 load the low halves (16 B each) of A's chunks, lanes 32-63 their high
// halves; same for B.  One v_permlane32_swap per dword (A's lanes 32-63 <->
// B's lanes 0-31) then gives every lane the low bytes (A) and high bytes (B)
// of its own 16 symbols -- exactly the half-chunk register contents, so the
// GF arithmetic (mac_input_v1) is unchanged.  Outputs are swapped back the
// same way before their contiguous stores.
template <int LPOL = 0>
__device__ __forceinline__ void gload_ct(u32x4 &A, u32x4 &B, uint64_t base, uint32_t offA,
                                         uint32_t offB) {
  if constexpr (LPOL == 1)
    asm volatile(
        "global_load_dwordx4 %0, %2, %4 nt\n\t"
        "global_load_dwordx4 %1, %3, %4 nt"
        : "=&v"(A), "=&v"(B)
        : "v"(offA), "v"(offB), "s"(base)
        : "memory");
  else
    asm volatile(
        "global_load_dwordx4 %0, %2, %4\n\t"
        "global_load_dwordx4 %1, %3, %4"
        : "=&v"(A), "=&v"(B)
        : "v"(offA), "v"(offB), "s"(base)
        : "memory");
}

// A's lanes 32-63 <-> B's lanes 0-31, dword by dword.
__device__ __forceinline__ void halves_swap(u32x4 &A, u32x4 &B) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const auto r = __builtin_amdgcn_permlane32_swap(A[d], B[d], false, false);
    A[d] = r[0];
    B[d] = r[1];
  }
}

// Lane offsets of the wave's two 1 KiB runs (chunk base wchunk0); a lane whose
// chunk is past the last full chunk reads chunk 0's bytes instead (never
// stored) so every lane takes part in the swaps.
struct CtLane {
  uint32_t offA, offB;
  uint32_t fb;  // an offset inside the shard's first chunk
  bool okA, okB;
};
__device__ __forceinline__ CtLane ct_lane(uint64_t wchunk0, uint64_t full_chunks) {
  const uint32_t l = threadIdx.x & 63;
  const uint32_t in_kib = ((l & 31) >> 1) * 64 + (l >> 5) * 32 + (l & 1) * 16;
  const uint64_t cA = wchunk0 + ((l & 31) >> 1), cB = cA + 16;
  CtLane r;
  r.okA = cA < full_chunks;
  r.okB = cB < full_chunks;
  const uint32_t fallback = (l >> 5) * 32 + (l & 1) * 16;
  r.fb = fallback;
  r.offA = r.okA ? uint32_t(wchunk0 * 64) + in_kib : fallback;
  r.offB = r.okB ? uint32_t(wchunk0 * 64) + 1024 + in_kib : fallback;
  return r;
}

// TAIL 1: the ring's loads past the last input (issued only to keep the
// vmcnt arithmetic constant, never consumed) read the last input's first
// chunk -- one hot 64-B line -- instead of re-reading 2 KiB of its columns,
// which with non-temporal loads costs real HBM traffic (2 of 30 inputs).
// SLOTS: the tables sit in read order (stage_tables_rotated), so step x uses
// slot x instead of input idx(x).
template <int LPOL, int ROT = 0, bool PROBE = false, int TAIL = 0, int SUB = 0, bool SLOTS = false>
__device__ __forceinline__ bool ring_acc_ct(const KernArgs &args, const PassDesc &P, uint32_t tile,
                                            uint32_t wave_id, uint32_t (&acc_lo)[16],
                                            uint32_t (&acc_hi)[16], CtLane &ln,
                                            uint32_t slots_rot = 0) {
  const uint32_t n_in = P.n_in;
  const uint64_t *in = args.ptrs + P.in;
  const uint64_t wchunk0 = (uint64_t(tile) * 4 + wave_id) * 32;
  if (wchunk0 >= P.full_chunks) return false;  // wave-uniform
  ln = ct_lane(wchunk0, P.full_chunks);
  const uint32_t offA = ln.offA, offB = ln.offB;
#pragma unroll
  for (int s = 0; s < 16; ++s) acc_lo[s] = acc_hi[s] = 0;
  // SLOTS: the caller staged the tables in its read order and passes it
  const uint32_t rot = SLOTS                ? slots_rot
                       : !P.rotate || ROT == 2 ? 0
                       : ROT == 1           ? (tile * 4) % n_in
                       : ROT >= 3           ? ((tile >> (ROT - 2)) * 4) % n_in
                                            : (tile * 4 + wave_id) % n_in;
  auto idx = [&](uint32_t x) -> uint32_t {
    if (x >= n_in) x = n_in - 1;
    const uint32_t y = rot + x;
    return y >= n_in ? y - n_in : y;
  };
  input_ring(
      n_in,
      [&](u32x4 &A, u32x4 &B, uint32_t x) {
        // branch-free (a branch here made the compiler spill in-flight ring
        // registers; tools/inflight_check.py): select the offsets only
        const bool past = TAIL && x >= n_in;
        gload_ct<LPOL>(A, B, in[idx(x)], past ? ln.fb : offA, past ? ln.fb : offB);
      },
      [&](const u32x4 &Av, const u32x4 &Bv, uint32_t x) {
        const uint32_t r = SLOTS ? x : idx(x);
        u32x4 L = Av, H = Bv;
        halves_swap(L, H);
#ifdef BFRS_AB_VARIANTS
        if constexpr (PROBE)  // traffic-only probe (measurement, NOT a codec)
          mac_input_stream(make_uint4(L.x, L.y, L.z, L.w), make_uint4(H.x, H.y, H.z, H.w), acc_lo,
                           acc_hi);
        else
#else
        static_assert(!PROBE, "traffic-only probes exist only in the A/B build");
#endif
        if constexpr (SUB)
          mac_input_sub(make_uint4(L.x, L.y, L.z, L.w), make_uint4(H.x, H.y, H.z, H.w), 2 * r,
                        2 * r + 1, acc_lo, acc_hi);
        else
          mac_input_v1(make_uint4(L.x, L.y, L.z, L.w), make_uint4(H.x, H.y, H.z, H.w), 2 * r,
                       2 * r + 1, acc_lo, acc_hi);
      });
  return true;
}

template <int LPOL, int SPOL, int ROT = 0, bool PROBE = false, int TAIL = 0, int SUB = 0,
          bool SLOTS = false>
__device__ __forceinline__ void ring_tile_ct(const KernArgs &args, const PassDesc &P, uint32_t tile,
                                             uint32_t wave_id, uint32_t slots_rot = 0) {
  uint32_t acc_lo[16], acc_hi[16];
  CtLane ln;
  if (!ring_acc_ct<LPOL, ROT, PROBE, TAIL, SUB, SLOTS>(args, P, tile, wave_id, acc_lo, acc_hi, ln,
                                                       slots_rot))
    return;
  const uint32_t n_out = P.n_out;
  const uint64_t *outp = args.ptrs + P.out;
  const bool accumulate = P.accumulate != 0;
  transpose_outputs(acc_lo);
  transpose_outputs(acc_hi);
#pragma unroll
  for (uint32_t t = 0; t < kMaxPassOutputs; ++t) {
    if (t >= n_out) break;
    u32x4 ol = {acc_lo[t], acc_lo[4 + t], acc_lo[8 + t], acc_lo[12 + t]};
    u32x4 oh = {acc_hi[t], acc_hi[4 + t], acc_hi[8 + t], acc_hi[12 + t]};
    halves_swap(ol, oh);  // back to the contiguous layout: ol -> run A, oh -> run B
    const uint64_t dst = outp[t];
    if (accumulate) {
      if (ln.okA) {
        const uint4 p = load16(dst + ln.offA);
        ol ^= u32x4{p.x, p.y, p.z, p.w};
      }
      if (ln.okB) {
        const uint4 p = load16(dst + ln.offB);
        oh ^= u32x4{p.x, p.y, p.z, p.w};
      }
    }
    if (ln.okA) store16_pol<SPOL>(dst + ln.offA, ol);
    if (ln.okB) store16_pol<SPOL>(dst + ln.offB, oh);
  }
}

#ifdef BFRS_AB_VARIANTS  // round-1 half-chunk layout (A/B build only)
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

#endif  // BFRS_AB_VARIANTS

// The ring kernel: workgroup wg owns tiles_per_wg consecutive 8 KiB tiles of
// one pass (one by default); ROT picks the read order (ring_acc_halfchunk).
// XG > 0: workgroup -> tile remap so that XG consecutive tiles (a read
// group) run on one XCD (hardware deals workgroups round-robin over the 8
// XCDs): within each full run of 8*XG workgroups, XCD x's q-th workgroup
// takes tile XG * (8 * (q / XG) + x) + q % XG.  Bijective; speed only.
template <uint32_t XG>
__device__ __forceinline__ uint32_t xcd_group_remap(uint32_t b, uint32_t n) {
  constexpr uint32_t run = 8 * XG;
  const uint32_t full = n / run * run;
  if (b >= full) return b;
  const uint32_t base = b / run * run, r = b - base, x = r & 7u, q = r >> 3;
  return base + XG * (8u * (q / XG) + x) + q % XG;
}

// LAY 0: half-chunk lanes (round 1); LAY 1: contiguous lines + lane-half
// swaps (ring_acc_ct).  LPOL 1: non-temporal loads (only sound with LAY 1,
// where every line is read by one instruction).
template <int ROT, bool PROBE = false, uint32_t XG = 0, int LAY = 0, int LPOL = 0, int TAIL = 0,
          int SUB = 0>
__global__ __launch_bounds__(256, 5) void gf_apply_ring_kernel(const KernArgs args) {
  uint32_t wg = blockIdx.x;
  if constexpr (XG > 0) wg = xcd_group_remap<XG>(blockIdx.x, gridDim.x);
  const PassDesc &P = enter_pass(args, wg);
  const uint32_t t_begin = (wg - P.wg_begin) * args.tiles_per_wg;
  const uint32_t t_end = min(t_begin + args.tiles_per_wg, P.n_tiles);
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint32_t tile = t_begin; tile < t_end; ++tile) {
#ifdef BFRS_AB_VARIANTS
    if constexpr (LAY == 0)
      ring_tile_halfchunk<0, 1, ROT, PROBE>(args, P, tile, wave_id);
    else
#else
    static_assert(LAY == 1, "the half-chunk layout exists only in the A/B build");
#endif
    ring_tile_ct<LPOL, 1, ROT, PROBE, TAIL, SUB>(args, P, tile, wave_id);
  }
}

// ---- fully unrolled path (v76) ------------------------------------------------
// For the pass sizes BlockFrame runs (n_in = 30: every full RS(30,3) block,
// encode or 3-erasure decode; 8 and 20: the last blocks of configs 2 and 4),
// the input loop is unrolled at compile time.  The table of the input consumed at step x then
// sits at a compile-time LDS offset (the workgroup stages its tables in its
// own rotated read order: slot x <- input (rot + x) mod n_in), so a lookup
// address is ONE SDWA op straight from the data byte -- no mask/shift prep,
// no v_perm splice -- with slot, half and byte in the ds_read immediate:
//   high nibble of byte k: v_and_b32_sdwa (byte k) & 0xF0        = 16*v
//   low nibble of byte k : v_lshlrev_b32_sdwa (byte k) << 4, BYTE_0 = 16*v
// Per symbol and input: 4 SDWA + 4 ds_read + 3 v_bitop3 (GF(2^8)-subfield
// passes only; the host selects this kernel when every pass is), 7 VALU vs
// ~9 of mac_input_sub.  The ring is the same 4-buffer, 3-in-flight ring with
// compile-time buffers and vmcnt.

// (byte K of x) & mask, mask = 0xF0 in an SGPR
template <int K>
__device__ __forceinline__ uint32_t sdwa_hi_nib16(uint32_t x, uint32_t mask) {
  uint32_t r;
  asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_%c3 src1_sel:DWORD"
      : "=v"(r)
      : "v"(x), "s"(mask), "i"(K));
  return r;
}
// ((byte K of x) << 4) & 0xFF
template <int K>
__device__ __forceinline__ uint32_t sdwa_lo_nib16(uint32_t x) {
  uint32_t r;
  asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_%c2"
      : "=v"(r)
      : "v"(x), "i"(K));
  return r;
}

template <int N>
__device__ __forceinline__ void vm_wait_n(u32x4 &A, u32x4 &B) {
  if constexpr (N <= 0) vm_wait<0>(A, B);
  else if constexpr (N == 2) vm_wait<2>(A, B);
  else if constexpr (N == 4) vm_wait<4>(A, B);
  else vm_wait<6>(A, B);
}

// 3-input XOR as a volatile asm: in the fully unrolled tile the compiler
// would otherwise reorder the accumulator chains across inputs and keep
// hundreds of lookup results live (3451 spilled VGPRs in the first build).
__device__ __forceinline__ uint32_t xor3_ordered(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// a ^ lo32(b) ^ lo32(c) where b, c are whole 8-byte LDS entries: naming the
// 64-bit values as (unprinted) operands keeps the compiler from narrowing
// their ds_read_b64 to ds_read_b32.  A wave64 ds_read_b32 runs at 128 B/clk,
// i.e. in 32-bank mode, where the stride-16 tables put nibbles v and v + 8 in
// one bank (2-way conflicts: SQ_LDS_BANK_CONFLICT = 32% of the cycles,
// profiles/r02/); a ds_read_b64 takes the same 2 cycles conflict free.
__device__ __forceinline__ uint32_t xor3_lo64(uint32_t a, uint64_t b, uint64_t c) {
  uint32_t r;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96 ; %4 %5"
               : "=v"(r)
               : "v"(a), "v"(uint32_t(b)), "v"(uint32_t(c)), "v"(b), "v"(c));
  return r;
}

// One input's 16 symbols (L = low bytes, H = high bytes) into the
// accumulators with the tables of slot SLOT (compile-time LDS offsets).
// B64: the low-byte lookups read whole 8-byte entries (conflict free);
// else 4-byte reads (32-bank mode: 2-way conflicts on the stride-16 tables).
template <uint32_t SLOT, bool B64>
__device__ __forceinline__ void mac_slot(const u32x4 &L, const u32x4 &H, uint32_t mask,
                                         uint32_t (&acc_lo)[16], uint32_t (&acc_hi)[16]) {
  const AS_LDS uint8_t *t = (const AS_LDS uint8_t *)(uintptr_t)(SLOT * 512u);
  const uint32_t l[4] = {L.x, L.y, L.z, L.w};
  const uint32_t h[4] = {H.x, H.y, H.z, H.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint64_t a[4], b[4];
    uint2 e2[4], e3[4];
#define BFRS_LOOKUPS(K)                                                                  \
  if constexpr (B64) {                                                                   \
    a[K] = *(const AS_LDS uint64_t *)(t + 256 + sdwa_lo_nib16<K>(l[d]));                 \
    b[K] = *(const AS_LDS uint64_t *)(t + sdwa_hi_nib16<K>(l[d], mask));                 \
  } else {                                                                               \
    a[K] = *(const AS_LDS uint32_t *)(t + 256 + sdwa_lo_nib16<K>(l[d]));                 \
    b[K] = *(const AS_LDS uint32_t *)(t + sdwa_hi_nib16<K>(l[d], mask));                 \
  }                                                                                      \
  {                                                                                      \
    const uint64_t v2 = *(const AS_LDS uint64_t *)(t + 256 + 8 + sdwa_lo_nib16<K>(h[d])); \
    const uint64_t v3 = *(const AS_LDS uint64_t *)(t + 8 + sdwa_hi_nib16<K>(h[d], mask)); \
    e2[K] = make_uint2(uint32_t(v2), uint32_t(v2 >> 32));                                \
    e3[K] = make_uint2(uint32_t(v3), uint32_t(v3 >> 32));                                \
  }
    // two symbols (8 lookups) per group, a scheduling barrier after each
    // group's XORs: letting the compiler hoist more lookups costs live VGPRs
    // and spills at the 96-VGPR (5 waves/SIMD) budget
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if (g == 0) {
        BFRS_LOOKUPS(0)
        BFRS_LOOKUPS(1)
      } else {
        BFRS_LOOKUPS(2)
        BFRS_LOOKUPS(3)
      }
#pragma unroll
      for (int k = 2 * g; k < 2 * g + 2; ++k) {
        const int s = d * 4 + k;
        const uint32_t lo2 = B64 ? xor3_lo64(acc_lo[s], a[k], b[k])
                                 : xor3_ordered(acc_lo[s], uint32_t(a[k]), uint32_t(b[k]));
        acc_lo[s] = xor3_ordered(lo2, e2[k].x, e3[k].x);
        acc_hi[s] = xor3_ordered(acc_hi[s], e2[k].y, e3[k].y);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#undef BFRS_LOOKUPS
  }
}

template <int N, int LPOL, bool B64, uint32_t C>
__device__ __forceinline__ void unrolled_step(const uint64_t *in, uint32_t rot, const CtLane &ln,
                                              uint32_t mask, u32x4 (&A)[N], u32x4 (&B)[N],
                                              uint32_t (&acc_lo)[16], uint32_t (&acc_hi)[16]) {
  constexpr int D = 3;  // inputs in flight ahead of the one consumed
  if constexpr (C < uint32_t(N)) {  // issue input C
    uint32_t src = rot + C;
    src = src >= uint32_t(N) ? src - N : src;
    gload_ct<LPOL>(A[C], B[C], in[src], ln.offA, ln.offB);
  }
  if constexpr (C >= uint32_t(D) && C - D < uint32_t(N)) {  // consume input C - D
    constexpr uint32_t c = C - D;
    constexpr int after = (N - 1 - int(c)) < D ? (N - 1 - int(c)) : D;
    vm_wait_n<2 * after>(A[c], B[c]);
    u32x4 L = A[c], H = B[c];
    halves_swap(L, H);
    mac_slot<c, B64>(L, H, mask, acc_lo, acc_hi);
  }
}

template <int N, int LPOL, bool B64, uint32_t... Cs>
__device__ __forceinline__ void unrolled_ring(const uint64_t *in, uint32_t rot, const CtLane &ln,
                                              uint32_t mask, u32x4 (&A)[N], u32x4 (&B)[N],
                                              uint32_t (&acc_lo)[16], uint32_t (&acc_hi)[16],
                                              std::integer_sequence<uint32_t, Cs...>) {
  (unrolled_step<N, LPOL, B64, Cs>(in, rot, ln, mask, A, B, acc_lo, acc_hi), ...);
}

template <int N, int LPOL, bool B64>
__device__ __forceinline__ void tile_unrolled(const KernArgs &args, const PassDesc &P,
                                              uint32_t tile, uint32_t wave_id, uint32_t rot) {
  const uint64_t wchunk0 = (uint64_t(tile) * 4 + wave_id) * 32;
  if (wchunk0 >= P.full_chunks) return;  // wave-uniform
  const CtLane ln = ct_lane(wchunk0, P.full_chunks);
  const uint64_t *in = args.ptrs + P.in;
  const uint32_t mask = __builtin_amdgcn_readfirstlane(0xF0u);
  uint32_t acc_lo[16], acc_hi[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) acc_lo[s] = acc_hi[s] = 0;
  u32x4 A[N], B[N];
  unrolled_ring<N, LPOL, B64>(in, rot, ln, mask, A, B, acc_lo, acc_hi,
                         std::make_integer_sequence<uint32_t, N + 3>{});
  const uint32_t n_out = P.n_out;
  const uint64_t *outp = args.ptrs + P.out;
  const bool accumulate = P.accumulate != 0;
  transpose_outputs(acc_lo);
  transpose_outputs(acc_hi);
#pragma unroll
  for (uint32_t t = 0; t < kMaxPassOutputs; ++t) {
    if (t >= n_out) break;
    u32x4 ol = {acc_lo[t], acc_lo[4 + t], acc_lo[8 + t], acc_lo[12 + t]};
    u32x4 oh = {acc_hi[t], acc_hi[4 + t], acc_hi[8 + t], acc_hi[12 + t]};
    halves_swap(ol, oh);
    const uint64_t dst = outp[t];
    if (accumulate) {
      if (ln.okA) {
        const uint4 p = load16(dst + ln.offA);
        ol ^= u32x4{p.x, p.y, p.z, p.w};
      }
      if (ln.okB) {
        const uint4 p = load16(dst + ln.offB);
        oh ^= u32x4{p.x, p.y, p.z, p.w};
      }
    }
    if (ln.okA) store16_nt(dst + ln.offA, ol);
    if (ln.okB) store16_nt(dst + ln.offB, oh);
  }
}

// Pass lookup (binary search over wg_begin) without staging.
__device__ __forceinline__ const PassDesc &find_pass(const KernArgs &args, uint32_t wg) {
  const PassDesc *passes = args.passes;
  uint32_t lo = 0, hi = args.n_passes;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (passes[mid].wg_begin <= wg)
      lo = mid;
    else
      hi = mid;
  }
  return passes[lo];
}

// Stages the pass tables in LDS in read order: slot x <- input (rot + x) mod n_in.
// NT: threads of the workgroup.
template <uint32_t NT = 256>
__device__ __forceinline__ void stage_tables_rotated(const PassDesc &P, uint32_t rot) {
  extern __shared__ __attribute__((aligned(16))) uint2 lds_table[];
  const uint32_t n_in = P.n_in;
  const AS_GLOBAL u32x4 *tab = (const AS_GLOBAL u32x4 *)(uintptr_t)P.table;
  u32x4 *dst = reinterpret_cast<u32x4 *>(lds_table);
  const uint32_t n16 = n_in * 32;  // 32 x 16 B per input
  u32x4 v[kMaxPassInputs * 32 / NT];
#pragma unroll
  for (int r = 0; r < int(kMaxPassInputs * 32 / NT); ++r) {
    const uint32_t e = threadIdx.x + NT * r;
    v[r] = e < n16 ? tab[e] : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int r = 0; r < int(kMaxPassInputs * 32 / NT); ++r) {
    const uint32_t e = threadIdx.x + NT * r;
    if (e < n16) {
      const uint32_t i = e >> 5;  // source input
      const uint32_t x = i >= rot ? i - rot : i + n_in - rot;  // its slot
      dst[x * 32 + (e & 31)] = v[r];
    }
  }
  __syncthreads();
}

// v76: unrolled SDWA-addressed path for n_in in {30, 20, 8}, the looped
// subfield path (slot-indexed tables) for any other pass of the launch.
// Host contract: every pass subfield, tiles_per_wg == 1.
// GL: log2 of the read group (consecutive tiles sharing one starting input,
// placed on one XCD); STEP: how far consecutive groups' starting inputs move.
template <bool B64, int GL = 6, int STEP = 4>
__global__ __launch_bounds__(256, 5) void gf_apply_unrolled_kernel(const KernArgs args) {
  const uint32_t wg = xcd_group_remap<(1u << GL)>(blockIdx.x, gridDim.x);
  const PassDesc &P = find_pass(args, wg);
  const uint32_t tile = wg - P.wg_begin;
  const uint32_t n_in = P.n_in;
  const uint32_t rot = P.rotate ? ((tile >> GL) * STEP) % n_in : 0;  // read order of v41/v58
  stage_tables_rotated(P, rot);
  if (tile >= P.n_tiles) return;
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (n_in == 30)
    tile_unrolled<30, 1, B64>(args, P, tile, wave_id, rot);
  else if (n_in == 8)
    tile_unrolled<8, 1, B64>(args, P, tile, wave_id, rot);
  else if (n_in == 20)  // config 4's last block, RS(20,3)
    tile_unrolled<20, 1, B64>(args, P, tile, wave_id, rot);
  else
    ring_tile_ct<1, 1, 6, false, 1, 1, true>(args, P, tile, wave_id, rot);
}

#ifdef BFRS_AB_VARIANTS
// ---- LDS-DMA input ring, 4 KiB per wave and input (v107-v109, round 6) -------
// Measurement build only.  The traffic probes put 4 KiB of
// columns per wave and input 3-4% ahead of v76's 2 KiB in both HBM placement
// modes (tools/membench8.hip `place`); register rings of 4 KiB (v92-v95, v105)
// lost that to their VGPR cost.  Here the inputs go HBM -> LDS with
// global_load_lds_dwordx4 (no VGPRs in flight): each wave streams its 4 KiB
// run of input c (four 1 KiB lines, lane l's 16 B to slot + 1 KiB * j + 16 l)
// into a private ring of D slots, D inputs ahead of the one it consumes.  The
// lane offsets are v76's contiguous-line offsets (every 128-B line fetched by
// one instruction), so a line's LDS image holds the low 32-B halves of its 16
// chunks in positions 0-31 and the high halves in 32-63: the lane's L / H are
// then one conflict-free ds_read_b128 each (two contiguous 512-B runs per
// instruction), which replaces the v_permlane32_swap of the loads.  A lane owns
// 32 symbols (two 2 KiB sub-runs), 64 accumulator VGPRs; the nibble-table
// arithmetic is v76's mac_slot, unchanged.  Workgroup = W waves; LDS = the
// tables (n_in x 512 B) + W x D x 4 KiB.

// Input run of one wave into its LDS slot: line j -> m0 = slot_j.  m0 is saved
// and restored (the compiler may hold a value there); s_nop 0 after each m0
// write (M0 -> LDS-DMA hazard).
__device__ __forceinline__ void dma_run4(uint64_t base, const uint32_t (&off)[4], uint32_t s0,
                                         uint32_t s1, uint32_t s2, uint32_t s3) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %6\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %5 nt\n\t"
      "s_mov_b32 m0, %7\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %5 nt\n\t"
      "s_mov_b32 m0, %8\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %3, %5 nt\n\t"
      "s_mov_b32 m0, %9\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %4, %5 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), "s"(base), "s"(s0), "s"(s1), "s"(s2),
        "s"(s3)
      : "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait_lds() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Step C of the ring: consume input C (its run landed once at most 4 * after
// DMAs of later inputs are outstanding), then refill its slot with input C + D.
template <int N, int D, uint32_t C>
__device__ __forceinline__ void lds_step(const uint64_t *in, uint32_t rot, const uint32_t (&off)[4],
                                         uint32_t ring, uint32_t lane_base, uint32_t mask,
                                         uint32_t (&lo0)[16], uint32_t (&hi0)[16],
                                         uint32_t (&lo1)[16], uint32_t (&hi1)[16]) {
  constexpr int after = (N - 1 - int(C)) < D - 1 ? (N - 1 - int(C)) : D - 1;
  // the refill's shard base (a scalar kernarg load) is issued before the wait,
  // which no memory access may cross, so its latency hides behind it
  uint64_t next = 0;
  if constexpr (C + D < uint32_t(N)) {
    uint32_t src = rot + C + D;
    src = src >= uint32_t(N) ? src - N : src;
    next = in[src];
  }
  vm_wait_lds<4 * after>();
  const uint32_t slot = ring + (C % D) * 4096u;
  const AS_LDS u32x4 *p = (const AS_LDS u32x4 *)(uintptr_t)(slot + lane_base);
  u32x4 L0 = p[0], H0 = p[32], L1 = p[128], H1 = p[160];  // +0, +512, +2048, +2560 B
  if constexpr (C + D < uint32_t(N)) {
    // the slot's bytes are in registers before its refill is issued
    asm volatile("" : "+v"(L0), "+v"(H0), "+v"(L1), "+v"(H1));
    dma_run4(next, off, slot, slot + 1024u, slot + 2048u, slot + 3072u);
  }
  mac_slot<C, true>(L0, H0, mask, lo0, hi0);
  mac_slot<C, true>(L1, H1, mask, lo1, hi1);
}

template <int N, int D, uint32_t... Cs>
__device__ __forceinline__ void lds_ring(const uint64_t *in, uint32_t rot, const uint32_t (&off)[4],
                                         uint32_t ring, uint32_t lane_base, uint32_t mask,
                                         uint32_t (&lo0)[16], uint32_t (&hi0)[16],
                                         uint32_t (&lo1)[16], uint32_t (&hi1)[16],
                                         std::integer_sequence<uint32_t, Cs...>) {
  (lds_step<N, D, Cs>(in, rot, off, ring, lane_base, mask, lo0, hi0, lo1, hi1), ...);
}

// Transpose, swap back to contiguous lines and store one 2 KiB sub-run's outputs.
__device__ __forceinline__ void store_subrun(const KernArgs &args, const PassDesc &P,
                                             const CtLane &ln, uint32_t (&acc_lo)[16],
                                             uint32_t (&acc_hi)[16]) {
  const uint32_t n_out = P.n_out;
  const uint64_t *outp = args.ptrs + P.out;
  const bool accumulate = P.accumulate != 0;
  transpose_outputs(acc_lo);
  transpose_outputs(acc_hi);
#pragma unroll
  for (uint32_t t = 0; t < kMaxPassOutputs; ++t) {
    if (t >= n_out) break;
    u32x4 ol = {acc_lo[t], acc_lo[4 + t], acc_lo[8 + t], acc_lo[12 + t]};
    u32x4 oh = {acc_hi[t], acc_hi[4 + t], acc_hi[8 + t], acc_hi[12 + t]};
    halves_swap(ol, oh);
    const uint64_t dst = outp[t];
    if (accumulate) {
      if (ln.okA) {
        const uint4 q = load16(dst + ln.offA);
        ol ^= u32x4{q.x, q.y, q.z, q.w};
      }
      if (ln.okB) {
        const uint4 q = load16(dst + ln.offB);
        oh ^= u32x4{q.x, q.y, q.z, q.w};
      }
    }
    if (ln.okA) store16_nt(dst + ln.offA, ol);
    if (ln.okB) store16_nt(dst + ln.offB, oh);
  }
}

template <int N, int W, int D>
__device__ __forceinline__ void tile_lds(const KernArgs &args, const PassDesc &P, uint32_t tile,
                                         uint32_t wave_id, uint32_t rot) {
  const uint64_t wc = (uint64_t(tile) * W + wave_id) * 64;  // the wave's first chunk
  if (wc >= P.full_chunks) return;                          // wave-uniform
  const uint32_t l = threadIdx.x & 63;
  const uint32_t in_kib = ((l & 31) >> 1) * 64 + (l >> 5) * 32 + (l & 1) * 16;
  const uint32_t fallback = (l >> 5) * 32 + (l & 1) * 16;  // inside chunk 0, never stored
  uint32_t off[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint64_t c = wc + 16 * j + ((l & 31) >> 1);
    off[j] = c < P.full_chunks ? uint32_t((wc + 16 * j) * 64) + in_kib : fallback;
  }
  const uint64_t *in = args.ptrs + P.in;
  const uint32_t mask = __builtin_amdgcn_readfirstlane(0xF0u);
  const uint32_t ring = uint32_t(N) * 512u + wave_id * uint32_t(D) * 4096u;
  const uint32_t lane_base = (l >> 5) * 1024 + (l & 31) * 16;
  uint32_t lo0[16], hi0[16], lo1[16], hi1[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) lo0[s] = hi0[s] = lo1[s] = hi1[s] = 0;
#pragma unroll
  for (int c = 0; c < D; ++c) {  // prologue: inputs 0 .. D-1
    uint32_t src = rot + c;
    src = src >= uint32_t(N) ? src - N : src;
    const uint32_t slot = ring + uint32_t(c) * 4096u;
    dma_run4(in[src], off, slot, slot + 1024u, slot + 2048u, slot + 3072u);
  }
  lds_ring<N, D>(in, rot, off, ring, lane_base, mask, lo0, hi0, lo1, hi1,
                 std::make_integer_sequence<uint32_t, N>{});
  store_subrun(args, P, ct_lane(wc, P.full_chunks), lo0, hi0);
  store_subrun(args, P, ct_lane(wc + 32, P.full_chunks), lo1, hi1);
}

// W waves per workgroup, D inputs in flight per wave, read groups of 2^GL
// tiles (512 KiB of columns) on one XCD.  Host contract: every pass subfield
// with n_in in {30, 20, 8}, tiles_per_wg == 1, tile = W x 4 KiB
// (launch_tile_bytes), LDS = max_in x 512 + W x D x 4 KiB.
template <int W, int D, int GL, int WAVES_PER_EU>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WAVES_PER_EU)))
void gf_apply_lds_kernel(
    const KernArgs args) {
  const uint32_t wg = xcd_group_remap<(1u << GL)>(blockIdx.x, gridDim.x);
  const PassDesc &P = find_pass(args, wg);
  const uint32_t tile = wg - P.wg_begin;
  const uint32_t n_in = P.n_in;
  const uint32_t rot = P.rotate ? ((tile >> GL) * 4) % n_in : 0;
  stage_tables_rotated<64 * W>(P, rot);
  if (tile >= P.n_tiles) return;
  const uint32_t wave_id = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (n_in == 30)
    tile_lds<30, W, D>(args, P, tile, wave_id, rot);
  else if (n_in == 8)
    tile_lds<8, W, D>(args, P, tile, wave_id, rot);
  else if (n_in == 20)
    tile_lds<20, W, D>(args, P, tile, wave_id, rot);
}
#endif  // BFRS_AB_VARIANTS

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

// Kernel selection.  The product library carries the default (76) and the
// two looped forms it falls back to: 75 (looped GF(2^8)-subfield ring) and 73
// (looped general GF(2^16) ring).  BFRS_KERNEL_VARIANT may force 75 or 73 (the
// parity suite runs them on BlockFrame's shapes); any other value is refused
// with an error, never run.  The round-1/2 A/B variants and the traffic-only
// probes (which write wrong bytes) exist only in the measurement build
// (make ab -> libbfrs_ab.so, -DBFRS_AB_VARIANTS; tools/kbench.py).
//   76: contiguous-line nt loads/stores with lane-half swaps; for GF(2^8)-
//       subfield launches (every RS(k<=30,3) encode/decode) the fully unrolled
//       SDWA-addressed kernel for n_in 30 / 20 / 8, read groups of 64
//       consecutive tiles (512 KiB of every shard's columns) on one XCD;
//       other launches run 75 or 73.
#ifdef BFRS_AB_VARIANTS
// A/B build only: 77 (76 with 4-byte low-byte lookups), 78-80 (read groups of
// 16 / 32 / 128 tiles), 81-83 (group start moving by 1 / 2 / 8 inputs), the
// round-2 steps 70 / 71, the round-1 kernels 58 / 41 / 36 / 37 / 40 / 42 / 5,
// and the traffic-only probes 44 / 72 / 74 (wrong output; also need
// BFRS_ALLOW_PROBE=1).  DESIGN.md §9 / §9b hold their results.
static bool variant_known(int v) {
  switch (v) {
    case 5: case 36: case 37: case 40: case 41: case 42: case 58: case 70: case 71:
    case 73: case 75: case 76: case 77: case 78: case 79: case 80: case 81: case 82: case 83:
    case 107: case 108: case 109:
      return true;
    case 44: case 72: case 74:
      return std::getenv("BFRS_ALLOW_PROBE") != nullptr;
    default:
      return false;
  }
}
#else
static bool variant_known(int v) { return v == 76 || v == 75 || v == 73; }
#endif

int kernel_variant() {
  const char *e = std::getenv("BFRS_KERNEL_VARIANT");
  if (!e || !*e) return 76;
  char *end = nullptr;
  const long v = std::strtol(e, &end, 10);
  if (*end != '\0' || v < 0 || v > 1000 || !variant_known(int(v))) return -1;
  return int(v);
}

bool ab_build() {
#ifdef BFRS_AB_VARIANTS
  return true;
#else
  return false;
#endif
}

#ifdef BFRS_AB_VARIANTS
// LDS-DMA variants: W waves x 4 KiB per tile
static uint32_t lds_variant_waves(int v) { return v == 107 ? 8 : (v == 108 || v == 109) ? 4 : 0; }
#endif

uint32_t tile_bytes(bool unrolled_sizes) {
#ifdef BFRS_AB_VARIANTS
  if (unrolled_sizes) {
    const int v = kernel_variant();
    if (lds_variant_waves(v)) return lds_variant_waves(v) * 4096u;
  }
#else
  (void)unrolled_sizes;
#endif
  return kTileHalfChunks * 32;
}

#ifdef BFRS_AB_VARIANTS
static hipError_t launch_gf_default(const KernArgs &args, uint32_t n_wgs, size_t lds, bool subfield,
                                    hipStream_t stream) {
  if (subfield && args.tiles_per_wg == 1)
    hipLaunchKernelGGL(gf_apply_unrolled_kernel<true>, dim3(n_wgs), dim3(256), lds, stream, args);
  else if (subfield)
    hipLaunchKernelGGL((gf_apply_ring_kernel<6, false, 16, 1, 1, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
  else
    hipLaunchKernelGGL((gf_apply_ring_kernel<6, false, 16, 1, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
  return hipGetLastError();
}
#endif

hipError_t launch_gf_apply(const KernArgs &args, uint32_t n_wgs, uint32_t max_in, bool subfield,
                           bool unrolled_sizes, hipStream_t stream) {
  if (n_wgs == 0) return hipSuccess;
  const size_t lds = size_t(max_in) * 64 * sizeof(uint2);
  const int v = kernel_variant();
  if (v < 0) return hipErrorInvalidValue;  // Context::init reports it by name
  const bool unrolled_ok = subfield && args.tiles_per_wg == 1;
#ifdef BFRS_AB_VARIANTS
  if (lds_variant_waves(v)) {
    // the grid was sized with tile_bytes(unrolled_sizes): wide tiles only
    // when every pass has an unrolled size, else v76's 8 KiB tiles
    if (!unrolled_sizes || !unrolled_ok) return launch_gf_default(args, n_wgs, lds, subfield, stream);
    if (v == 107)  // 8 waves, 2 inputs in flight: 2 WGs = 16 waves per CU
      hipLaunchKernelGGL((gf_apply_lds_kernel<8, 2, 4, 4>), dim3(n_wgs), dim3(512),
                         lds + 8 * 2 * 4096, stream, args);
    else if (v == 108)  // 4 waves, 2 in flight: 3 WGs = 12 waves per CU
      hipLaunchKernelGGL((gf_apply_lds_kernel<4, 2, 5, 3>), dim3(n_wgs), dim3(256),
                         lds + 4 * 2 * 4096, stream, args);
    else  // 109: 4 waves, 3 in flight: 2 WGs = 8 waves per CU
      hipLaunchKernelGGL((gf_apply_lds_kernel<4, 3, 5, 2>), dim3(n_wgs), dim3(256),
                         lds + 4 * 3 * 4096, stream, args);
    return hipGetLastError();
  }
#else
  (void)unrolled_sizes;
#endif
  switch (v) {
    case 76:  // unrolled SDWA-addressed kernel where the launch allows it, else 75 / 73
      if (unrolled_ok) {
        hipLaunchKernelGGL(gf_apply_unrolled_kernel<true>, dim3(n_wgs), dim3(256), lds, stream, args);
        break;
      }
      [[fallthrough]];
    case 75:  // looped ring, GF(2^8)-subfield arithmetic when every pass allows it
      if (subfield) {
        hipLaunchKernelGGL((gf_apply_ring_kernel<6, false, 16, 1, 1, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
        break;
      }
      [[fallthrough]];
    case 73:  // looped ring, general GF(2^16) arithmetic
      hipLaunchKernelGGL((gf_apply_ring_kernel<6, false, 16, 1, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
#ifdef BFRS_AB_VARIANTS
    case 5:
      hipLaunchKernelGGL((gf_apply_ring_kernel<0>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 36:
      hipLaunchKernelGGL((gf_apply_ring_kernel<1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 37:
      hipLaunchKernelGGL((gf_apply_ring_kernel<2>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 40:
      hipLaunchKernelGGL((gf_apply_ring_kernel<5>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 42:
      hipLaunchKernelGGL((gf_apply_ring_kernel<7>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 44:
      hipLaunchKernelGGL((gf_apply_ring_kernel<6, true, 16>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 41:
      hipLaunchKernelGGL((gf_apply_ring_kernel<6>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 58:  // 41 with each read group's 16 workgroups on one XCD
      hipLaunchKernelGGL((gf_apply_ring_kernel<6, false, 16>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 70:  // 58 with contiguous-line loads/stores (LAY 1)
      hipLaunchKernelGGL((gf_apply_ring_kernel<6, false, 16, 1, 0>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 71:  // 70 with non-temporal loads
      hipLaunchKernelGGL((gf_apply_ring_kernel<6, false, 16, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 72:  // traffic-only probe of 71
      hipLaunchKernelGGL((gf_apply_ring_kernel<6, true, 16, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 74:  // traffic-only probe of 73
      hipLaunchKernelGGL((gf_apply_ring_kernel<6, true, 16, 1, 1, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 77:  // 76 with 4-byte low-byte lookups
      if (!unrolled_ok) return launch_gf_default(args, n_wgs, lds, subfield, stream);
      hipLaunchKernelGGL(gf_apply_unrolled_kernel<false>, dim3(n_wgs), dim3(256), lds, stream, args);
      break;
    case 78: case 79: case 80: case 81: case 82: case 83:
      if (!unrolled_ok) return launch_gf_default(args, n_wgs, lds, subfield, stream);
      if (v == 78)  // read groups of 16 tiles (the round-1 grouping)
        hipLaunchKernelGGL((gf_apply_unrolled_kernel<true, 4, 4>), dim3(n_wgs), dim3(256), lds, stream, args);
      else if (v == 79)  // read groups of 32 tiles
        hipLaunchKernelGGL((gf_apply_unrolled_kernel<true, 5, 4>), dim3(n_wgs), dim3(256), lds, stream, args);
      else if (v == 80)  // read groups of 128 tiles
        hipLaunchKernelGGL((gf_apply_unrolled_kernel<true, 7, 4>), dim3(n_wgs), dim3(256), lds, stream, args);
      else if (v == 81)  // group start moving by 1 input
        hipLaunchKernelGGL((gf_apply_unrolled_kernel<true, 6, 1>), dim3(n_wgs), dim3(256), lds, stream, args);
      else if (v == 82)  // by 2 inputs
        hipLaunchKernelGGL((gf_apply_unrolled_kernel<true, 6, 2>), dim3(n_wgs), dim3(256), lds, stream, args);
      else  // by 8 inputs
        hipLaunchKernelGGL((gf_apply_unrolled_kernel<true, 6, 8>), dim3(n_wgs), dim3(256), lds, stream, args);
      break;
#endif
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_gf_tail(const KernArgs &args, hipStream_t stream) {
  if (args.n_passes == 0) return hipSuccess;
  hipLaunchKernelGGL(gf_tail_kernel, dim3(args.n_passes), dim3(64), 0, stream, args);
  return hipGetLastError();
}

}  // namespace bfrs
