// hash_kernels.hpp — BLAKE3 device kernels (blake3_kernels.hip) and launchers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace bfrs {

constexpr uint32_t kChunkBytes = 1024;                  // BLAKE3 chunk
constexpr uint32_t kGroupChunks = 256;                  // chunks per workgroup of kernel 1
constexpr uint32_t kGroupBytes = kChunkBytes * kGroupChunks;
constexpr uint32_t kReduceFanIn = 512;                  // CVs one kernel-2 workgroup pairs down
// Tree levels kernel 1 pairs inside a group of a multi-group message: 256
// chunk CVs -> 32 level-3 nodes (8 KiB subtrees), written out for kernel 2.
// Levels 1-2 use every active lane and level 3 half a wave (32 slots idle per
// group, 0.8% of the group's work); the upper levels of a group would use a
// fraction of a wave (16 -> 1 nodes: 5 wave-compressions for 31 parents), so
// they are left to kernel 2, whose first levels over 512 nodes use every
// lane.  Three levels rather than two also halve kernel 2's first-level jobs,
// which then fit the chip in one round.
constexpr uint32_t kGroupLevels = 3;
constexpr uint32_t kGroupOutMax = kGroupChunks >> 2;  // level-2 nodes per group (the most)

// One message of a kernel-1 launch.  Workgroup w belongs to the message m
// with first_group(m) <= w < first_group(m + 1) (found by a binary search in
// the kernel, so the host uploads one descriptor per message, not per group)
// and hashes <= 256 KiB of it starting at a 256 KiB aligned offset (so its
// chunks form an aligned subtree of the message).  A single-group message is
// finished in kernel 1; a group of a longer message writes its ceil(chunks /
// 2^levels) level-`levels` nodes to group_cvs[(kGroupChunks >> levels) * w].
struct alignas(16) HashMsg {
  uint64_t addr;         // device address of the message (16-byte aligned)
  uint64_t chunk0;       // BLAKE3 chunk counter of its first chunk
  uint64_t nbytes;       // message length
  uint32_t first_group;  // its first workgroup
  uint32_t groups;       // its workgroups (an empty message has one)
};

// One kernel-2 workgroup: CVs in_cvs[first, first + n) of message `msg`.
// final = 1: they are all of the message's nodes at this level -> digest.
// final = 0: an aligned run of kReduceFanIn nodes (or the tail) -> out_cvs[out].
struct alignas(16) HashReduce {
  uint32_t first, n, out, final;
  uint32_t msg, pad[3];
};

hipError_t launch_blake3_groups(const HashMsg *d_msgs, uint32_t n_msgs, uint32_t n_groups,
                                uint32_t levels, uint32_t *d_group_cvs, uint32_t *d_msg_cvs,
                                uint32_t *d_digests, hipStream_t stream);
// quads: kernel 2's levels of <= 64 parents by quad-cooperative compressions
// (the product); false (one parent per lane) exists in the measurement build
// alone.
hipError_t launch_blake3_reduce(const HashReduce *d_jobs, uint32_t n_jobs, bool quads,
                                const uint32_t *d_in, uint32_t *d_out, uint32_t *d_msg_cvs,
                                uint32_t *d_digests, hipStream_t stream);

}  // namespace bfrs
