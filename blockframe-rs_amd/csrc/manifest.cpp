// manifest.cpp — see manifest.hpp.
#include "manifest.hpp"

#include <cctype>
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

struct Parser {
  const std::string &t;
  size_t p = 0;
  std::string err;
  explicit Parser(const std::string &text) : t(text) {}
  void ws() {
    while (p < t.size() && std::isspace(static_cast<unsigned char>(t[p]))) ++p;
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
    if (p + 4 > t.size()) return fail("short \\u escape");
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
  bool string(std::string *out) {
    if (p >= t.size() || t[p] != '"') return fail("expected string");
    ++p;
    while (p < t.size() && t[p] != '"') {
      char c = t[p++];
      if (c != '\\') {
        out->push_back(c);
        continue;
      }
      if (p >= t.size()) return fail("bad escape");
      c = t[p++];
      switch (c) {
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
          if (cp >= 0xD800 && cp < 0xDC00 && p + 6 <= t.size() && t[p] == '\\' && t[p + 1] == 'u') {
            p += 2;
            uint32_t lo;
            if (!hex4(&lo)) return false;
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
  bool value(Json *v, int depth) {
    if (depth > 64) return fail("nesting too deep");
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
        if (!string(&k)) return false;
        ws();
        if (p >= t.size() || t[p] != ':') return fail("expected ':'");
        ++p;
        if (!value(&v->o[k], depth + 1)) return false;
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
    if (c == '-' || std::isdigit(static_cast<unsigned char>(c))) {
      const size_t s0 = p;
      if (t[p] == '-') ++p;
      while (p < t.size() && std::isdigit(static_cast<unsigned char>(t[p]))) ++p;
      // fractions/exponents are not produced by the manifest writer; accept and truncate
      while (p < t.size() && (t[p] == '.' || t[p] == 'e' || t[p] == 'E' || t[p] == '+' ||
                              t[p] == '-' || std::isdigit(static_cast<unsigned char>(t[p]))))
        ++p;
      v->kind = Json::kInt;
      v->i = std::strtoll(t.substr(s0, p - s0).c_str(), nullptr, 10);
      return true;
    }
    return fail("unexpected character");
  }
};

Json str_array(const std::vector<std::string> &v) {
  Json a = Json::arr();
  for (const auto &s : v) a.a.push_back(Json::str(s));
  return a;
}

bool read_str_array(const Json *j, std::vector<std::string> *out) {
  if (!j || j->kind != Json::kArray) return false;
  for (const auto &e : j->a) {
    if (e.kind != Json::kString) return false;
    out->push_back(e.s);
  }
  return true;
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
// Map keys of leaves/segments/blocks are decimal integers (serde's
// HashMap<i32|usize, _> keys); anything else is a parse error, never an
// exception across the C-ABI.
bool parse_key(const std::string &k, int64_t *out) {
  if (k.empty() || k.size() > 18) return false;
  size_t i = k[0] == '-' ? 1 : 0;
  if (i == k.size()) return false;
  int64_t v = 0;
  for (; i < k.size(); ++i) {
    if (k[i] < '0' || k[i] > '9') return false;
    v = v * 10 + (k[i] - '0');
  }
  *out = k[0] == '-' ? -v : v;
  return true;
}
}  // namespace

bool Manifest::from_json(const std::string &text, Manifest *m, std::string *err) {
  Json j;
  if (!Json::parse(text, &j, err)) return false;
  auto need = [&](const Json *v, Json::Kind k, const char *name) {
    if (!v || v->kind != k) {
      if (err) *err = std::string("manifest: missing or invalid '") + name + "'";
      return false;
    }
    return true;
  };
  if (!need(&j, Json::kObject, "<root>")) return false;
  const Json *v;
  if (!need(v = j.get("original_hash"), Json::kString, "original_hash")) return false;
  m->original_hash = v->s;
  if (!need(v = j.get("name"), Json::kString, "name")) return false;
  m->name = v->s;
  if (!need(v = j.get("size"), Json::kInt, "size")) return false;
  m->size = v->i;
  if ((v = j.get("time_of_creation")) && v->kind == Json::kString) m->time_of_creation = v->s;
  if (!need(v = j.get("tier"), Json::kInt, "tier")) return false;
  m->tier = int(v->i);
  if (!need(v = j.get("segment_size"), Json::kInt, "segment_size")) return false;
  m->segment_size = uint64_t(v->i);
  const Json *ec = j.get("erasure_coding");
  if (!need(ec, Json::kObject, "erasure_coding")) return false;
  if ((v = ec->get("data_shards")) && v->kind == Json::kInt) m->data_shards = int(v->i);
  if ((v = ec->get("parity_shards")) && v->kind == Json::kInt) m->parity_shards = int(v->i);
  if ((v = ec->get("type")) && v->kind == Json::kString) m->ec_type = v->s;
  const Json *mt = j.get("merkle_tree");
  if (!need(mt, Json::kObject, "merkle_tree")) return false;
  if (!need(v = mt->get("root"), Json::kString, "merkle_tree.root")) return false;
  m->root = v->s;
  auto key = [&](const std::string &k, int64_t *out) {
    if (parse_key(k, out)) return true;
    if (err) *err = "manifest: map key '" + k + "' is not an integer";
    return false;
  };
  int64_t id;
  if ((v = mt->get("leaves")) && v->kind == Json::kObject)
    for (const auto &kv : v->o) {
      if (!key(kv.first, &id)) return false;
      if (kv.second.kind == Json::kString) m->leaves[id] = kv.second.s;
    }
  if ((v = mt->get("segments")) && v->kind == Json::kObject)
    for (const auto &kv : v->o) {
      SegmentHashes sh;
      const Json *d = kv.second.get("data");
      if (!d || d->kind != Json::kString || !read_str_array(kv.second.get("parity"), &sh.parity)) {
        if (err) *err = "manifest: bad segments entry";
        return false;
      }
      sh.data = d->s;
      if (!key(kv.first, &id)) return false;
      m->segments[id] = sh;
    }
  if ((v = mt->get("blocks")) && v->kind == Json::kObject)
    for (const auto &kv : v->o) {
      BlockHashes bh;
      if (!read_str_array(kv.second.get("segments"), &bh.segments) ||
          !read_str_array(kv.second.get("parity"), &bh.parity)) {
        if (err) *err = "manifest: bad blocks entry";
        return false;
      }
      if (!key(kv.first, &id)) return false;
      m->blocks[id] = bh;
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
