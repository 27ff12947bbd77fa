// blake3.hpp — BLAKE3 (unkeyed hash) for BlockFrame's integrity checks.
//
// The reference hashes with the `blake3` crate (1.8.2, Cargo.lock:136-145)
// through blake3_hash_bytes (src/utils.rs:22-28): segments and parity shards
// at commit (src/chunker/commit.rs:429,451), the whole file (:478), and on
// every FUSE cache miss (src/mount/filesystem_unix.rs:238-246).  This is a
// portable implementation of the BLAKE3 specification; large inputs are
// split into independent power-of-two chunk subtrees hashed on threads (the
// tree shape makes those subtrees independent), which is how the 32 MiB
// segment and multi-GiB file hashes stay off the critical path.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace bfrs {

// 32-byte digest of data[0..len).  threads <= 1: single-threaded.
void blake3_hash(const uint8_t *data, size_t len, uint8_t out[32], int threads = 1);
std::string blake3_hex(const uint8_t *data, size_t len, int threads = 1);
std::string to_hex(const uint8_t *d, size_t n);

// Digest of a message from the subtree chaining values of its consecutive
// parts (n >= 2): every part but the last holds the same power-of-two number
// of 1 KiB chunks, so each part is one node of the message's tree (e.g. the
// 32 MiB segments of a file).  CVs are 32 bytes each, little-endian words.
std::string blake3_combine_cvs_hex(const uint8_t *cvs, size_t n);

// src/merkle_tree/mod.rs:56-100 (from_hashes + build_tree): parents hash the
// ASCII concatenation of the two lowercase-hex children; an odd node pairs
// with itself.  Single leaf -> the leaf itself.
std::string merkle_root_hex(const std::vector<std::string> &leaves);

}  // namespace bfrs
