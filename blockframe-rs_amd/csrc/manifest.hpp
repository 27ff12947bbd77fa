// manifest.hpp — BlockFrame manifest.json (src/merkle_tree/manifest.rs:12-53,
// written by src/chunker/io.rs:126-202).
//
// The reference serialises with serde_json's json! macro, whose object map is
// a BTreeMap (no "preserve_order" feature, Cargo.toml:22): keys come out
// sorted, compact (to_string).  Json below keeps objects in std::map for the
// same ordering, so manifests written here have the reference's byte layout
// (only time_of_creation differs).
#pragma once

#include <cstdint>
#include <map>
#include <set>
#include <memory>
#include <string>
#include <vector>

namespace bfrs {

// JSON value.  Numbers keep serde_json's three classes: kInt (an integer that
// fits i64), kUInt (a non-negative integer above i64's range that fits u64)
// and kFloat (a fraction, an exponent, or an integer beyond u64; its text is
// kept in `s`), so a typed field refuses what serde would.  `dup`: the object
// had a repeated key (serde: "duplicate field" for a struct; a map keeps the
// last value).
struct Json {
  enum Kind { kNull, kBool, kInt, kUInt, kFloat, kString, kArray, kObject } kind = kNull;
  bool b = false;
  bool dup = false;
  // keys whose raw text held a backslash escape: serde_json reads an integer
  // map key with the number grammar on the raw bytes, so an escaped digit is no key
  std::set<std::string> escaped_keys;
  int64_t i = 0;
  uint64_t u = 0;
  std::string s;
  std::vector<Json> a;
  std::map<std::string, Json> o;

  static Json str(std::string v) {
    Json j;
    j.kind = kString;
    j.s = std::move(v);
    return j;
  }
  static Json num(int64_t v) {
    Json j;
    j.kind = kInt;
    j.i = v;
    return j;
  }
  static Json arr() {
    Json j;
    j.kind = kArray;
    return j;
  }
  static Json obj() {
    Json j;
    j.kind = kObject;
    return j;
  }
  Json &operator[](const std::string &k) { return o[k]; }
  const Json *get(const std::string &k) const {
    auto it = o.find(k);
    return it == o.end() ? nullptr : &it->second;
  }
  std::string dump() const;                       // compact, sorted keys
  // RFC 8259 JSON as serde_json::from_str takes it: valid UTF-8, no raw
  // control characters in strings, paired surrogate escapes, strict number
  // grammar, nesting depth <= 128 (serde_json's recursion limit).
  static bool parse(const std::string &text, Json *out, std::string *err);
};

// Typed view of the fields the RS path needs.
struct BlockHashes {
  std::vector<std::string> segments, parity;
};
struct SegmentHashes {
  std::string data;
  std::vector<std::string> parity;
};
struct Manifest {
  std::string original_hash, name, time_of_creation, root;
  std::string ec_type = "reed-solomon";  // io.rs:141 writes "reed-solomon"
  int64_t size = 0;
  int tier = 0;
  uint64_t segment_size = 0;
  int data_shards = 0, parity_shards = 0;
  std::map<int64_t, std::string> leaves;           // tier 1
  std::map<int64_t, SegmentHashes> segments;       // tier 2
  std::map<int64_t, BlockHashes> blocks;           // tier 3

  // tier 1 writes merkle_tree = {leaves, root} (MerkleTree::get_json,
  // src/merkle_tree/mod.rs:240-251); tiers 2/3 the full MerkleTreeStructure.
  std::string to_json() const;
  // ManifestFile::new (manifest.rs:47-53): serde's derive rules for the
  // structs at manifest.rs:6-45 -- every field required except the three
  // merkle_tree maps (#[serde(default)]), exact integer types (size i64,
  // tier u8, segment_size u64, shard counts i8, leaf keys i32, segment /
  // block keys usize), unknown fields ignored, duplicate struct fields an
  // error.  Never throws.
  static bool from_json(const std::string &text, Manifest *m, std::string *err);
};

// chrono's DateTime<Utc> Display, e.g. "2026-10-15 22:07:01.123456789 UTC".
std::string utc_now_string();

}  // namespace bfrs
