// manifest.cpp — see manifest.hpp.
#include "manifest.hpp"

#include <cctype>
#include <climits>
#include <cstdint>
#include <chrono>
#include <cstdio>
#include <ctime>

namespace bfrs {

namespace {

void dump_string(const std::string &s, std::string *out) {
  out->push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': *out += "\\\""; break;
      case '\\': *out += "\\\\"; break;
      case '\n': *out += "\\n"; break;
      case '\r': *out += "\\r"; break;
      case '\t': *out += "\\t"; break;
      case '\b': *out += "\\b"; break;
      case '\f': *out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          *out += buf;
        } else {
          out->push_back(char(c));
        }
    }
  }
  out->push_back('"');
}

void dump_to(const Json &j, std::string *out) {
  switch (j.kind) {
    case Json::kNull: *out += "null"; break;
    case Json::kBool: *out += j.b ? "true" : "false"; break;
    case Json::kInt: *out += std::to_string(j.i); break;
    case Json::kUInt: *out += std::to_string(j.u); break;
    case Json::kFloat: *out += j.s; break;
    case Json::kString: dump_string(j.s, out); break;
    case Json::kArray: {
      out->push_back('[');
      for (size_t n = 0; n < j.a.size(); ++n) {
        if (n) out->push_back(',');
        dump_to(j.a[n], out);
      }
      out->push_back(']');
      break;
    }
    case Json::kObject: {
      out->push_back('{');
      bool first = true;
      for (const auto &kv : j.o) {
        if (!first) out->push_back(',');
        first = false;
        dump_string(kv.first, out);
        out->push_back(':');
        dump_to(kv.second, out);
      }
      out->push_back('}');
      break;
    }
  }
}

// Length of the UTF-8 sequence at t[p..] (RFC 3629: no overlongs, no
// surrogates, <= U+10FFFF), 0 if invalid.
size_t utf8_len(const std::string &t, size_t p) {
  const auto c = [&](size_t k) { return static_cast<unsigned char>(t[p + k]); };
  const size_t left = t.size() - p;
  const unsigned char b0 = c(0);
  if (b0 < 0x80) return 1;
  auto cont = [&](size_t k) { return k < left && (c(k) & 0xC0) == 0x80; };
  if (b0 >= 0xC2 && b0 <= 0xDF) return cont(1) ? 2 : 0;
  if (b0 >= 0xE0 && b0 <= 0xEF) {
    if (!cont(1) || !cont(2)) return 0;
    if (b0 == 0xE0 && c(1) < 0xA0) return 0;  // overlong
    if (b0 == 0xED && c(1) >= 0xA0) return 0;  // surrogate
    return 3;
  }
  if (b0 >= 0xF0 && b0 <= 0xF4) {
    if (!cont(1) || !cont(2) || !cont(3)) return 0;
    if (b0 == 0xF0 && c(1) < 0x90) return 0;  // overlong
    if (b0 == 0xF4 && c(1) >= 0x90) return 0;  // > U+10FFFF
    return 4;
  }
  return 0;
}

struct Parser {
  static constexpr int kMaxDepth = 128;  // serde_json's recursion limit
  const std::string &t;
  size_t p = 0;
  std::string err;
  explicit Parser(const std::string &text) : t(text) {}
  void ws() {  // JSON whitespace only (RFC 8259: space, tab, LF, CR)
    while (p < t.size() && (t[p] == ' ' || t[p] == '\t' || t[p] == '\n' || t[p] == '\r')) ++p;
  }
  bool fail(const char *m) {
    if (err.empty()) err = std::string(m) + " at offset " + std::to_string(p);
    return false;
  }
  static void put_utf8(uint32_t cp, std::string *out) {
    if (cp < 0x80) {
      out->push_back(char(cp));
    } else if (cp < 0x800) {
      out->push_back(char(0xC0 | (cp >> 6)));
      out->push_back(char(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out->push_back(char(0xE0 | (cp >> 12)));
      out->push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(char(0x80 | (cp & 0x3F)));
    } else {
      out->push_back(char(0xF0 | (cp >> 18)));
      out->push_back(char(0x80 | ((cp >> 12) & 0x3F)));
      out->push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(char(0x80 | (cp & 0x3F)));
    }
  }
  bool hex4(uint32_t *v) {
    if (t.size() - p < 4) return fail("short \\u escape");
    *v = 0;
    for (int n = 0; n < 4; ++n) {
      const char c = t[p++];
      *v <<= 4;
      if (c >= '0' && c <= '9') *v |= uint32_t(c - '0');
      else if (c >= 'a' && c <= 'f') *v |= uint32_t(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') *v |= uint32_t(c - 'A' + 10);
      else return fail("bad hex digit");
    }
    return true;
  }
  bool string(std::string *out, bool *escaped = nullptr) {
    if (p >= t.size() || t[p] != '"') return fail("expected string");
    ++p;
    while (p < t.size() && t[p] != '"') {
      const unsigned char c = static_cast<unsigned char>(t[p]);
      if (c < 0x20) return fail("control character in string");
      if (c != '\\') {
        const size_t n = utf8_len(t, p);
        if (!n) return fail("invalid UTF-8");
        out->append(t, p, n);
        p += n;
        continue;
      }
      if (++p >= t.size()) return fail("bad escape");
      if (escaped) *escaped = true;
      switch (t[p++]) {
        case '"': out->push_back('"'); break;
        case '\\': out->push_back('\\'); break;
        case '/': out->push_back('/'); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return false;
          if (cp >= 0xDC00 && cp < 0xE000) return fail("lone trailing surrogate");
          if (cp >= 0xD800 && cp < 0xDC00) {  // must pair with \uDC00-\uDFFF
            if (t.size() - p < 6 || t[p] != '\\' || t[p + 1] != 'u')
              return fail("lone leading surrogate");
            p += 2;
            uint32_t lo;
            if (!hex4(&lo)) return false;
            if (lo < 0xDC00 || lo >= 0xE000) return fail("invalid surrogate pair");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(cp, out);
          break;
        }
        default: return fail("bad escape");
      }
    }
    if (p >= t.size()) return fail("unterminated string");
    ++p;
    return true;
  }
  static bool digit(char c) { return c >= '0' && c <= '9'; }
  // RFC 8259 number; integers are classified as serde_json does.
  bool number(Json *v) {
    const size_t s0 = p;
    const bool neg = t[p] == '-';
    if (neg) ++p;
    if (p >= t.size() || !digit(t[p])) return fail("invalid number");
    if (t[p] == '0') {
      ++p;
      if (p < t.size() && digit(t[p])) return fail("invalid number (leading zero)");
    } else {
      while (p < t.size() && digit(t[p])) ++p;
    }
    bool integer = true;
    if (p < t.size() && t[p] == '.') {
      integer = false;
      ++p;
      if (p >= t.size() || !digit(t[p])) return fail("invalid number");
      while (p < t.size() && digit(t[p])) ++p;
    }
    if (p < t.size() && (t[p] == 'e' || t[p] == 'E')) {
      integer = false;
      ++p;
      if (p < t.size() && (t[p] == '+' || t[p] == '-')) ++p;
      if (p >= t.size() || !digit(t[p])) return fail("invalid number");
      while (p < t.size() && digit(t[p])) ++p;
    }
    const std::string text = t.substr(s0, p - s0);
    if (integer) {
      // magnitude with overflow detection (no strtoll clamping)
      uint64_t mag = 0;
      bool fits = true;
      for (size_t k = neg ? 1 : 0; k < text.size(); ++k) {
        const uint64_t d = uint64_t(text[k] - '0');
        if (mag > (UINT64_MAX - d) / 10) {
          fits = false;
          break;
        }
        mag = mag * 10 + d;
      }
      if (fits && !neg && mag <= uint64_t(INT64_MAX)) {
        v->kind = Json::kInt;
        v->i = int64_t(mag);
        return true;
      }
      if (fits && !neg) {
        v->kind = Json::kUInt;
        v->u = mag;
        return true;
      }
      if (fits && neg && mag <= uint64_t(INT64_MAX) + 1) {
        v->kind = Json::kInt;
        v->i = mag == uint64_t(INT64_MAX) + 1 ? INT64_MIN : -int64_t(mag);
        return true;
      }
    }
    v->kind = Json::kFloat;  // serde_json: f64 (never a valid integer field)
    v->s = text;
    return true;
  }
  bool value(Json *v, int depth) {
    if (depth > kMaxDepth) return fail("recursion limit exceeded");
    ws();
    if (p >= t.size()) return fail("unexpected end");
    const char c = t[p];
    if (c == '{') {
      ++p;
      v->kind = Json::kObject;
      ws();
      if (p < t.size() && t[p] == '}') {
        ++p;
        return true;
      }
      for (;;) {
        ws();
        std::string k;
        bool esc = false;
        if (!string(&k, &esc)) return false;
        if (esc) v->escaped_keys.insert(k);
        ws();
        if (p >= t.size() || t[p] != ':') return fail("expected ':'");
        ++p;
        auto ins = v->o.emplace(k, Json());
        if (!ins.second) {  // repeated key: the last value wins, noted
          v->dup = true;
          ins.first->second = Json();
        }
        if (!value(&ins.first->second, depth + 1)) return false;
        ws();
        if (p < t.size() && t[p] == ',') {
          ++p;
          continue;
        }
        if (p < t.size() && t[p] == '}') {
          ++p;
          return true;
        }
        return fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p;
      v->kind = Json::kArray;
      ws();
      if (p < t.size() && t[p] == ']') {
        ++p;
        return true;
      }
      for (;;) {
        v->a.emplace_back();
        if (!value(&v->a.back(), depth + 1)) return false;
        ws();
        if (p < t.size() && t[p] == ',') {
          ++p;
          continue;
        }
        if (p < t.size() && t[p] == ']') {
          ++p;
          return true;
        }
        return fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      v->kind = Json::kString;
      return string(&v->s);
    }
    if (t.compare(p, 4, "true") == 0) {
      p += 4;
      v->kind = Json::kBool;
      v->b = true;
      return true;
    }
    if (t.compare(p, 5, "false") == 0) {
      p += 5;
      v->kind = Json::kBool;
      return true;
    }
    if (t.compare(p, 4, "null") == 0) {
      p += 4;
      return true;
    }
    if (c == '-' || digit(c)) return number(v);
    return fail("expected value");
  }
};

Json str_array(const std::vector<std::string> &v) {
  Json a = Json::arr();
  for (const auto &s : v) a.a.push_back(Json::str(s));
  return a;
}

}  // namespace

std::string Json::dump() const {
  std::string out;
  dump_to(*this, &out);
  return out;
}

bool Json::parse(const std::string &text, Json *out, std::string *err) {
  Parser ps(text);
  *out = Json();
  if (!ps.value(out, 0)) {
    if (err) *err = ps.err;
    return false;
  }
  ps.ws();
  if (ps.p != text.size()) {
    if (err) *err = "trailing characters";
    return false;
  }
  return true;
}

std::string Manifest::to_json() const {
  Json j = Json::obj();
  j["original_hash"] = Json::str(original_hash);
  j["name"] = Json::str(name);
  j["size"] = Json::num(size);
  j["time_of_creation"] = Json::str(time_of_creation);
  Json ec = Json::obj();
  ec["type"] = Json::str(ec_type);
  ec["data_shards"] = Json::num(data_shards);
  ec["parity_shards"] = Json::num(parity_shards);
  j["erasure_coding"] = ec;
  Json mt = Json::obj();
  Json lv = Json::obj();
  for (const auto &kv : leaves) lv[std::to_string(kv.first)] = Json::str(kv.second);
  mt["leaves"] = lv;
  mt["root"] = Json::str(root);
  if (tier != 1) {
    Json sg = Json::obj();
    for (const auto &kv : segments) {
      Json e = Json::obj();
      e["data"] = Json::str(kv.second.data);
      e["parity"] = str_array(kv.second.parity);
      sg[std::to_string(kv.first)] = e;
    }
    Json bl = Json::obj();
    for (const auto &kv : blocks) {
      Json e = Json::obj();
      e["segments"] = str_array(kv.second.segments);
      e["parity"] = str_array(kv.second.parity);
      bl[std::to_string(kv.first)] = e;
    }
    mt["segments"] = sg;
    mt["blocks"] = bl;
  }
  j["merkle_tree"] = mt;
  j["tier"] = Json::num(tier);
  j["segment_size"] = Json::num(int64_t(segment_size));
  return j.dump();
}

namespace {

// serde field readers: a missing field or a value of the wrong type / range
// is the error serde_json reports ("missing field", "invalid type",
// "invalid value").
struct Reader {
  std::string *err;
  bool fail(const std::string &m) {
    if (err) *err = "manifest: " + m;
    return false;
  }
  bool object(const Json *v, const char *name, bool check_dup = true) {
    if (!v) return fail(std::string("missing field '") + name + "'");
    if (v->kind != Json::kObject) return fail(std::string("invalid type for '") + name + "'");
    if (check_dup && v->dup) return fail(std::string("duplicate field in '") + name + "'");
    return true;
  }
  bool str(const Json &o, const char *name, std::string *out) {
    const Json *v = o.get(name);
    if (!v) return fail(std::string("missing field '") + name + "'");
    if (v->kind != Json::kString) return fail(std::string("invalid type for '") + name + "'");
    *out = v->s;
    return true;
  }
  // integer field within [lo, hi] (i64 range); kUInt only for u64 fields
  bool int_field(const Json &o, const char *name, int64_t lo, int64_t hi, int64_t *out) {
    const Json *v = o.get(name);
    if (!v) return fail(std::string("missing field '") + name + "'");
    if (v->kind != Json::kInt && v->kind != Json::kUInt)
      return fail(std::string("invalid type for '") + name + "': expected an integer");
    if (v->kind == Json::kUInt || v->i < lo || v->i > hi)
      return fail(std::string("invalid value for '") + name + "': out of range");
    *out = v->i;
    return true;
  }
  bool u64_field(const Json &o, const char *name, uint64_t *out) {
    const Json *v = o.get(name);
    if (!v) return fail(std::string("missing field '") + name + "'");
    if (v->kind == Json::kUInt) {
      *out = v->u;
      return true;
    }
    if (v->kind != Json::kInt) return fail(std::string("invalid type for '") + name + "': expected u64");
    if (v->i < 0) return fail(std::string("invalid value for '") + name + "': negative");
    *out = uint64_t(v->i);
    return true;
  }
  bool str_array(const Json *v, const char *name, std::vector<std::string> *out) {
    if (!v) return fail(std::string("missing field '") + name + "'");
    if (v->kind != Json::kArray) return fail(std::string("invalid type for '") + name + "'");
    for (const auto &e : v->a) {
      if (e.kind != Json::kString) return fail(std::string("invalid type in '") + name + "'");
      out->push_back(e.s);
    }
    return true;
  }
  // map key: decimal integer in [lo, hi].  serde_json 1.0.148 (MapKey::
  // deserialize_number) runs the JSON number grammar over the key's raw bytes
  // between the quotes, so it refuses a leading zero ("01"), a key written
  // with an escaped digit, and "-0" (which that grammar yields as the float -0.0, no
  // integer) -- each of which would otherwise alias another key
  bool key(const Json &map, const std::string &k, int64_t lo, int64_t hi, int64_t *out) {
    size_t i = !k.empty() && k[0] == '-' ? 1 : 0;
    bool ok = i < k.size() && k.size() - i <= 19 && !map.escaped_keys.count(k);
    if (ok && k[i] == '0' && k.size() - i > 1) ok = false;  // leading zero
    if (ok && i == 1 && k == "-0") ok = false;
    uint64_t mag = 0;
    for (; ok && i < k.size(); ++i) {
      if (k[i] < '0' || k[i] > '9') ok = false;
      else mag = mag * 10 + uint64_t(k[i] - '0');
    }
    const bool neg = !k.empty() && k[0] == '-';
    ok = ok && mag <= uint64_t(INT64_MAX);
    const int64_t v = neg ? -int64_t(mag) : int64_t(mag);
    if (!ok || v < lo || v > hi) return fail("map key '" + k + "' is not a valid integer key");
    *out = v;
    return true;
  }
};

}  // namespace

bool Manifest::from_json(const std::string &text, Manifest *m, std::string *err) {
  Json j;
  if (!Json::parse(text, &j, err)) return false;
  Reader r{err};
  if (!r.object(&j, "<root>")) return false;
  int64_t v;
  if (!r.str(j, "original_hash", &m->original_hash) || !r.str(j, "name", &m->name) ||
      !r.int_field(j, "size", INT64_MIN, INT64_MAX, &m->size) ||
      !r.str(j, "time_of_creation", &m->time_of_creation) ||
      !r.int_field(j, "tier", 0, 255, &v))  // u8
    return false;
  m->tier = int(v);
  if (!r.u64_field(j, "segment_size", &m->segment_size)) return false;
  const Json *ec = j.get("erasure_coding");
  if (!r.object(ec, "erasure_coding") || !r.int_field(*ec, "data_shards", -128, 127, &v))  // i8
    return false;
  m->data_shards = int(v);
  if (!r.int_field(*ec, "parity_shards", -128, 127, &v)) return false;
  m->parity_shards = int(v);
  if (!r.str(*ec, "type", &m->ec_type)) return false;
  const Json *mt = j.get("merkle_tree");
  if (!r.object(mt, "merkle_tree") || !r.str(*mt, "root", &m->root)) return false;
  int64_t id;
  if (const Json *lv = mt->get("leaves")) {  // HashMap<i32, String>, #[serde(default)]
    if (!r.object(lv, "leaves", false)) return false;
    for (const auto &kv : lv->o) {
      if (!r.key(*lv, kv.first, INT32_MIN, INT32_MAX, &id)) return false;
      if (kv.second.kind != Json::kString) return r.fail("invalid type in 'leaves'");
      m->leaves[id] = kv.second.s;
    }
  }
  if (const Json *sg = mt->get("segments")) {  // HashMap<usize, SegmentHashes>
    if (!r.object(sg, "segments", false)) return false;
    for (const auto &kv : sg->o) {
      if (!r.key(*sg, kv.first, 0, INT64_MAX, &id)) return false;
      SegmentHashes sh;
      if (!r.object(&kv.second, "segments entry") || !r.str(kv.second, "data", &sh.data) ||
          !r.str_array(kv.second.get("parity"), "parity", &sh.parity))
        return false;
      m->segments[id] = std::move(sh);
    }
  }
  if (const Json *bl = mt->get("blocks")) {  // HashMap<usize, BlockHashes>
    if (!r.object(bl, "blocks", false)) return false;
    for (const auto &kv : bl->o) {
      if (!r.key(*bl, kv.first, 0, INT64_MAX, &id)) return false;
      BlockHashes bh;
      if (!r.object(&kv.second, "blocks entry") ||
          !r.str_array(kv.second.get("segments"), "segments", &bh.segments) ||
          !r.str_array(kv.second.get("parity"), "parity", &bh.parity))
        return false;
      m->blocks[id] = std::move(bh);
    }
  }
  return true;
}

std::string utc_now_string() {
  const auto now = std::chrono::system_clock::now();
  const auto ns =
      std::chrono::duration_cast<std::chrono::nanoseconds>(now.time_since_epoch()).count();
  const std::time_t secs = std::time_t(ns / 1000000000);
  std::tm tm{};
  gmtime_r(&secs, &tm);
  char buf[64];
  std::snprintf(buf, sizeof buf, "%04d-%02d-%02d %02d:%02d:%02d", tm.tm_year + 1900,
                tm.tm_mon + 1, tm.tm_mday, tm.tm_hour, tm.tm_min, tm.tm_sec);
  std::string out = buf;
  // chrono NaiveTime Display: fraction omitted when zero, else 3, 6 or 9 digits
  const long long frac = static_cast<long long>(ns % 1000000000);
  if (frac % 1000000 == 0 && frac)
    std::snprintf(buf, sizeof buf, ".%03lld", frac / 1000000);
  else if (frac % 1000 == 0 && frac)
    std::snprintf(buf, sizeof buf, ".%06lld", frac / 1000);
  else if (frac)
    std::snprintf(buf, sizeof buf, ".%09lld", frac);
  else
    buf[0] = 0;
  return out + buf + " UTC";
}

}  // namespace bfrs
