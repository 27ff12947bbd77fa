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
// chunk CVs -> 64 level-2 nodes (4 KiB subtrees), written out for kernel 2.
// Those two levels use every active lane; the upper levels of a group use a
// fraction of a wave (128 -> 1 nodes: 9 wave-compressions for 255 parents),
// so they are left to kernel 2, whose first levels over 512 nodes use every
// lane too.
constexpr uint32_t kGroupLevels = 2;
constexpr uint32_t kGroupOut = kGroupChunks >> kGroupLevels;  // level-2 nodes per full group

// One kernel-1 workgroup: <= 256 KiB of one message, starting at a 256 KiB
// aligned offset (so its chunks form an aligned subtree of the message).  A
// single-group message is finished in kernel 1; a group of a longer message
// writes its ceil(chunks / 4) level-2 nodes to group_cvs[kGroupOut * index].
struct alignas(16) HashGroup {
  uint64_t addr;    // device address of the group's first byte (16-byte aligned)
  uint64_t chunk0;  // BLAKE3 chunk counter of its first chunk
  uint32_t nbytes;  // bytes in the group (0 only for an empty message)
  uint32_t msg;     // message index (digest / CV slot)
  uint32_t single;  // 1: the group is the whole message -> finalise in kernel 1
  uint32_t pad;
};

// One kernel-2 workgroup: CVs in_cvs[first, first + n) of message `msg`.
// final = 1: they are all of the message's nodes at this level -> digest.
// final = 0: an aligned run of kReduceFanIn nodes (or the tail) -> out_cvs[out].
struct alignas(16) HashReduce {
  uint32_t first, n, out, final;
  uint32_t msg, pad[3];
};

hipError_t launch_blake3_groups(const HashGroup *d_groups, uint32_t n_groups, uint32_t *d_group_cvs,
                                uint32_t *d_msg_cvs, uint32_t *d_digests, hipStream_t stream);
hipError_t launch_blake3_reduce(const HashReduce *d_jobs, uint32_t n_jobs, const uint32_t *d_in,
                                uint32_t *d_out, uint32_t *d_msg_cvs, uint32_t *d_digests,
                                hipStream_t stream);

}  // namespace bfrs
