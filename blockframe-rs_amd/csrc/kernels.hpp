// kernels.hpp — device-side pass descriptors and launchers (rs_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>

#include <cstdint>

namespace bfrs {

// Max inputs one pass reads; larger codes are split into accumulate passes.
constexpr uint32_t kMaxPassInputs = 64;
// Max outputs one pass writes (one byte lane of the packed table entry each).
constexpr uint32_t kMaxPassOutputs = 4;
// One workgroup tile = 256 lanes x one 32-byte half-chunk = 8 KiB of columns.
constexpr uint32_t kTileHalfChunks = 256;

// Nibble-table entry (8 B) index within one input's 64 entries (512 B); q =
// 2*byte_hi + nib_hi selects which nibble of which symbol byte is looked up.
// Entry v of (nibble half, byte) sits at 16*v + 8*byte_hi of its 256-B half:
//   high nibbles (q = 1, 3): bytes [0, 256), lookup offset (x & 0xF0) + 8*byte_hi
//     -- the nibble stays in place;
//   low nibbles (q = 0, 2): bytes [256, 512), offset ((x << 4) & 0xF0) + 8*byte_hi.
// Both offsets are one SDWA op from the raw data byte (v_and_b32_sdwa /
// v_lshlrev_b32_sdwa dst_sel:BYTE_0), the 8*byte_hi + half + input part an
// immediate of the ds_read (the unrolled kernel, rs_kernels.hip).  The 16
// entries of one (nibble half, byte) span 32 distinct LDS banks (a half-wave's
// 32 ds_read_b64 hit distinct banks or broadcast): conflict free.
constexpr uint32_t tab_idx(uint32_t q, uint32_t v) {
  return (q & 1) ? 2 * v + (q >> 1) : 32 + 2 * v + (q >> 1);
}

// One pass: out[t] (^)= sum_i coef(t,i) * in[i] for t < n_out, over the
// 64-byte-chunk symbol layout of reed-solomon-simd.
struct alignas(16) PassDesc {
  uint64_t in;               // index into KernArgs::ptrs of n_in (+1 prefetch) shard addresses
  uint64_t out;              // index into KernArgs::ptrs of n_out shard addresses
  uint64_t table;            // device address of n_in * 64 packed nibble products (uint2)
  uint32_t n_in, n_out;
  uint32_t wg_begin;         // first workgroup of this pass in the grid
  uint32_t n_tiles;          // tiles in this pass
  uint64_t full_chunks;      // whole 64-byte chunks per shard
  uint32_t tail_bytes;       // shard_bytes % 64 (tail chunk, crate tail layout)
  uint16_t accumulate;       // 1: XOR into existing outputs
  uint16_t rotate;           // 1: rotate the input order (even, unpadded passes)
  uint32_t n_real;           // inputs with a nonzero table (n_in - 1 for an odd count)
};

// Kernel-argument form: up to kMaxLaunchPasses passes and kMaxLaunchPtrs shard
// addresses travel in the dispatch packet's kernarg segment (< 4 KiB), so a
// launch needs no descriptor upload.  PassDesc::in / ::out are then indices
// into KernArgs::ptrs.
constexpr uint32_t kMaxLaunchPasses = 16;
constexpr uint32_t kMaxLaunchPtrs = 376;

struct alignas(16) KernArgs {
  uint32_t n_passes;
  uint32_t tiles_per_wg;
  uint32_t pad[2];
  PassDesc passes[kMaxLaunchPasses];
  uint64_t ptrs[kMaxLaunchPtrs];
};
static_assert(sizeof(KernArgs) <= 4096, "kernel arguments must fit 4 KiB");

// Column bytes one workgroup tile of a launch covers in the selected kernel
// variant.  unrolled_sizes: every pass of the launch is GF(2^8)-subfield with
// n_in in {30, 20, 8} (the A/B build's LDS-DMA variants tile wider there).
uint32_t tile_bytes(bool unrolled_sizes);
// The kernel BFRS_KERNEL_VARIANT selects (76 when unset), or -1 when this
// build does not carry that variant (the product library: 76, 75 and 73 only;
// the A/B variants live in libbfrs_ab.so, rs_kernels.hip).
int kernel_variant();
bool ab_build();

// subfield: every pass of the launch has GF(2^8)-subfield coefficients
// (PlanPass::subfield), so the subfield kernel form may run; unrolled_sizes as
// for tile_bytes (the grid was sized with tile_bytes(unrolled_sizes)).
hipError_t launch_gf_apply(const KernArgs &args, uint32_t n_wgs, uint32_t max_in, bool subfield,
                           bool unrolled_sizes, hipStream_t stream);
hipError_t launch_gf_tail(const KernArgs &args, hipStream_t stream);

}  // namespace bfrs
