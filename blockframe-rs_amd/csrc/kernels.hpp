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

// One pass: out[t] (^)= sum_i coef(t,i) * in[i] for t < n_out, over the
// 64-byte-chunk symbol layout of reed-solomon-simd.
struct alignas(16) PassDesc {
  uint64_t in;               // device address of n_in shard addresses (16-byte aligned)
  uint64_t out;              // device address of n_out shard addresses
  uint64_t table;            // device address of n_in * 64 packed nibble products (uint2)
  uint32_t n_in, n_out;
  uint32_t wg_begin;         // first workgroup of this pass in the grid
  uint32_t n_tiles;          // tiles in this pass
  uint64_t full_chunks;      // whole 64-byte chunks per shard
  uint32_t tail_bytes;       // shard_bytes % 64 (tail chunk, crate tail layout)
  uint32_t accumulate;       // 1: XOR into existing outputs
};

hipError_t launch_gf_apply(const PassDesc *d_passes, uint32_t n_passes, uint32_t n_wgs,
                           uint32_t tiles_per_wg, uint32_t max_in, hipStream_t stream);
hipError_t launch_gf_tail(const PassDesc *d_passes, uint32_t n_passes, hipStream_t stream);

}  // namespace bfrs
