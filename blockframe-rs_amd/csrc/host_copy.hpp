// host_copy.hpp — see host_copy.cpp.
#pragma once

#include <cstddef>
#include <cstdint>

namespace bfrs {

// memcpy on up to 8 threads for large buffers (pageable <-> pinned staging).
// Never throws: a thread that cannot start leaves its part to the caller.
void host_copy(uint8_t *dst, const uint8_t *src, size_t n);

}  // namespace bfrs
