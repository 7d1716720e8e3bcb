// cjson.hpp — small JSON reader for the host side of libcyclonus_hip.
//
// Inputs crossing the C ABI are the reference's own wire formats: k8s NetworkPolicy JSON
// (cli/utils.go:14-60 reads YAML->JSON), json.Marshal(*matcher.Policy), probe.Resources JSON
// (analyze.go:227-238) and generator.PortProtocol.  Numbers keep their raw text so intstr
// decoding (JSON number => Int, string => String) is exact.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace cyc {
namespace json {

struct Node {
  enum T : uint8_t { Null, Bool, Num, Str, Arr, Obj } t = Null;
  bool b = false;
  std::string s;                                       // Str value / Num raw text
  std::vector<Node> a;                                 // Arr
  std::vector<std::pair<std::string, Node>> o;         // Obj (insertion order)

  bool null() const { return t == Null; }
  bool is_arr() const { return t == Arr; }
  bool is_obj() const { return t == Obj; }
  // encoding/json struct-field lookup: every key equal to the field name exactly or ASCII
  // case-insensitively decodes into that field, in document order, so the LAST such key wins
  // ({"Namespace":"a","namespace":"b"} gives "b", as Go's decoder does).
  const Node* find(std::string_view k) const {
    if (t != Obj) return nullptr;
    const Node* hit = nullptr;
    for (auto& kv : o)
      if (key_eq(kv.first, k)) hit = &kv.second;
    return hit;
  }
  // Pointer, slice, map and interface fields: JSON null sets them to nil, so the last matching
  // key decides and a null there means absent.
  const Node* val(std::string_view k) const {  // non-null member or nullptr
    const Node* n = find(k);
    return (n && n->t != Null) ? n : nullptr;
  }
  // Scalar (string, number, bool) and struct-valued fields: encoding/json leaves them unchanged
  // for a JSON null, so the last NON-null matching key decides ({"Namespace":"a","namespace":null}
  // decodes to "a").
  const Node* sval(std::string_view k) const {
    if (t != Obj) return nullptr;
    const Node* hit = nullptr;
    for (auto& kv : o)
      if (kv.second.t != Null && key_eq(kv.first, k)) hit = &kv.second;
    return hit;
  }
  static bool key_eq(std::string_view a, std::string_view k) {  // exact or ASCII case-insensitive
    if (a.size() != k.size()) return false;
    for (size_t i = 0; i < k.size(); i++) {
      char x = a[i], y = k[i];
      if (x >= 'A' && x <= 'Z') x += 32;
      if (y >= 'A' && y <= 'Z') y += 32;
      if (x != y) return false;
    }
    return true;
  }
  const std::string& str() const {
    if (t != Str) throw std::runtime_error("json: expected a string");
    return s;
  }
  long long i64() const {
    if (t != Num) throw std::runtime_error("json: expected a number");
    char* e = nullptr;
    long long v = std::strtoll(s.c_str(), &e, 10);
    if (!e || *e) throw std::runtime_error("json: expected an integer, got " + s);
    return v;
  }
};

class Reader {
 public:
  Reader(const char* p, size_t n) : p_(p), n_(n) {}
  Node doc() {
    sp();
    Node v = any();
    sp();
    if (i_ != n_) fail("trailing data");
    return v;
  }

 private:
  const char* p_;
  size_t n_, i_ = 0;
  int depth_ = 0;  // nesting of the value being read
  // encoding/json's scanner refuses documents nested deeper than 10000 (Go 1.15+ maxNestingDepth);
  // the same bound keeps this recursive reader's stack use finite on hostile input
  static constexpr int kMaxDepth = 10000;
  [[noreturn]] void fail(const char* m) {
    throw std::runtime_error(std::string("json: ") + m + " at byte " + std::to_string(i_));
  }
  void sp() {
    while (i_ < n_ && (p_[i_] == ' ' || p_[i_] == '\t' || p_[i_] == '\n' || p_[i_] == '\r')) i_++;
  }
  char peek() { return i_ < n_ ? p_[i_] : 0; }
  bool word(std::string_view w) {
    if (n_ - i_ >= w.size() && std::string_view(p_ + i_, w.size()) == w) {
      i_ += w.size();
      return true;
    }
    return false;
  }
  struct Nest {  // depth guard for one nested object / array
    int& d;
    explicit Nest(Reader& r) : d(r.depth_) {
      if (++d > kMaxDepth) r.fail("exceeded max depth");
    }
    ~Nest() { --d; }
  };
  Node any() {
    char c = peek();
    if (c == '{' || c == '[') {
      Nest guard(*this);
      return c == '{' ? object() : array();
    }
    return scalar(c);
  }
  Node object() {
    Node v;
    {
      v.t = Node::Obj;
      i_++;
      sp();
      if (peek() == '}') {
        i_++;
        return v;
      }
      for (;;) {
        sp();
        if (peek() != '"') fail("expected object key");
        std::string k = string();
        sp();
        if (peek() != ':') fail("expected ':'");
        i_++;
        sp();
        v.o.emplace_back(std::move(k), any());
        sp();
        if (peek() == ',') {
          i_++;
          continue;
        }
        if (peek() == '}') {
          i_++;
          return v;
        }
        fail("expected ',' or '}'");
      }
    }
  }
  Node array() {
    Node v;
    {
      v.t = Node::Arr;
      i_++;
      sp();
      if (peek() == ']') {
        i_++;
        return v;
      }
      for (;;) {
        sp();
        v.a.push_back(any());
        sp();
        if (peek() == ',') {
          i_++;
          continue;
        }
        if (peek() == ']') {
          i_++;
          return v;
        }
        fail("expected ',' or ']'");
      }
    }
  }
  Node scalar(char c) {
    Node v;
    if (c == '"') {
      v.t = Node::Str;
      v.s = string();
      return v;
    }
    if (word("true")) {
      v.t = Node::Bool;
      v.b = true;
      return v;
    }
    if (word("false")) {
      v.t = Node::Bool;
      return v;
    }
    if (word("null")) return v;
    if (c == '-' || (c >= '0' && c <= '9')) {
      v.t = Node::Num;
      size_t st = i_++;
      while (i_ < n_) {
        char d = p_[i_];
        if ((d >= '0' && d <= '9') || d == '.' || d == 'e' || d == 'E' || d == '+' || d == '-') i_++;
        else break;
      }
      v.s.assign(p_ + st, i_ - st);
      return v;
    }
    fail("unexpected character");
  }
  unsigned hex4() {
    if (n_ - i_ < 4) fail("short \\u escape");
    unsigned v = 0;
    for (int k = 0; k < 4; k++) {
      char h = p_[i_++];
      v <<= 4;
      if (h >= '0' && h <= '9') v |= unsigned(h - '0');
      else if (h >= 'a' && h <= 'f') v |= unsigned(h - 'a' + 10);
      else if (h >= 'A' && h <= 'F') v |= unsigned(h - 'A' + 10);
      else fail("bad \\u escape");
    }
    return v;
  }
  static void utf8(std::string& o, unsigned cp) {
    if (cp < 0x80) o += char(cp);
    else if (cp < 0x800) {
      o += char(0xC0 | (cp >> 6));
      o += char(0x80 | (cp & 63));
    } else if (cp < 0x10000) {
      o += char(0xE0 | (cp >> 12));
      o += char(0x80 | ((cp >> 6) & 63));
      o += char(0x80 | (cp & 63));
    } else {
      o += char(0xF0 | (cp >> 18));
      o += char(0x80 | ((cp >> 12) & 63));
      o += char(0x80 | ((cp >> 6) & 63));
      o += char(0x80 | (cp & 63));
    }
  }
  std::string string() {
    std::string o;
    i_++;
    for (;;) {
      if (i_ >= n_) fail("unterminated string");
      size_t st = i_;
      while (i_ < n_ && p_[i_] != '"' && p_[i_] != '\\') i_++;
      o.append(p_ + st, i_ - st);
      if (i_ >= n_) fail("unterminated string");
      if (p_[i_] == '"') {
        i_++;
        return o;
      }
      i_++;  // backslash
      if (i_ >= n_) fail("bad escape");
      char e = p_[i_++];
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00) {
            if (n_ - i_ >= 6 && p_[i_] == '\\' && p_[i_ + 1] == 'u') {
              i_ += 2;
              unsigned lo = hex4();
              cp = (lo >= 0xDC00 && lo < 0xE000) ? 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00) : 0xFFFD;
            } else {
              cp = 0xFFFD;
            }
          } else if (cp >= 0xDC00 && cp < 0xE000) {
            cp = 0xFFFD;
          }
          utf8(o, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
  }
};

inline Node parse(const char* p, size_t n) { return Reader(p, n).doc(); }

// Go encoding/json string quoting (json.Marshal escapes <, >, & and U+2028/2029).
inline std::string quote(std::string_view s) {
  static const char* hx = "0123456789abcdef";
  std::string o;
  o.reserve(s.size() + 2);
  o += '"';
  for (size_t i = 0; i < s.size(); i++) {
    unsigned char c = (unsigned char)s[i];
    switch (c) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      default: break;
    }
    if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      o += "\\u00";
      o += hx[c >> 4];
      o += hx[c & 15];
    } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
               ((unsigned char)s[i + 2] & 0xFE) == 0xA8) {
      o += ((unsigned char)s[i + 2] == 0xA8) ? "\\u2028" : "\\u2029";
      i += 2;
    } else {
      o += char(c);
    }
  }
  o += '"';
  return o;
}

}  // namespace json
}  // namespace cyc
