// host_copy.hpp — see host_copy.cpp.
#pragma once

#include <cstddef>
#include <cstdint>

namespace bfrs {

// memcpy on up to 8 threads for large buffers (pageable <-> pinned staging).
// Never throws: a thread that cannot start leaves its part to the caller.
void host_copy(uint8_t *dst, const uint8_t *src, size_t n);

// First touch of a fresh output buffer the library is about to fill (the
// reference's to_vec / fresh Vec outputs): madvise(MADV_POPULATE_WRITE) of
// its whole pages (Linux 5.14+: the pages are allocated in one call, without
// a fault per page), falling back to writing one byte per page.  The bytes
// written are zeros; the caller's copy-out overwrites them.
void prefault_range(uint8_t *p, size_t n);

// Many copies at once (the slab-pipelined wrappers: one column slab of every
// shard): job i copies n[i] bytes and zero-fills pad[i] more after them;
// the calling thread and the helpers the shared budget grants (as host_copy)
// take jobs in order, and done(i) runs on the thread that finished job i.
// Never throws.
struct CopyJob {
  uint8_t *dst;
  const uint8_t *src;
  size_t n, pad;
};
void host_copy_batch(const CopyJob *jobs, size_t count, void (*done)(void *, size_t), void *arg);

}  // namespace bfrs
