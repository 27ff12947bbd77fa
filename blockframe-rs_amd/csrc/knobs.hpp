// knobs.hpp — the library's environment knobs.
//
// libbfrs.so reads exactly the six product knobs include/bfrs.h documents
// (BFRS_KERNEL_VARIANT, BFRS_CODEC_SLOTS, BFRS_CODEC_STAGING, BFRS_PLAN_CACHE,
// BFRS_PREFETCH_DEPTH, BFRS_HOST_COPY_BUDGET; tests/test_abi.py checks the
// BFRS_* strings in the binary against that list).  The knobs of concluded
// A/B studies (pipeline depth, slab width, stream layout, prefault modes,
// tiles per workgroup, BLAKE3 quad levels, the trace lines; DESIGN.md §7,
// §7c, §9b) are read only by the measurement build libbfrs_ab.so
// (-DBFRS_AB_VARIANTS).  In the product they compile to "unset", so the
// soak-proven default is the only configuration it can run.
#pragma once

#include <cstdlib>

#ifdef BFRS_AB_VARIANTS
#define BFRS_AB_KNOB(name) std::getenv(name)
#else
#define BFRS_AB_KNOB(name) static_cast<const char *>(nullptr)
#endif
