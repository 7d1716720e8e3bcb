// oracle/ojson.hpp — minimal JSON DOM used ONLY by the CPU oracle (test infrastructure).
//
// The oracle decodes the same wire formats the reference's Go code decodes with
// encoding/json (k8s NetworkPolicy objects, probe.Resources, generator.PortProtocol).
// Objects keep insertion order; numbers keep their raw text so that intstr decoding
// (number => Int, string => String; k8s.io/apimachinery intstr.go UnmarshalJSON) can
// be restated exactly.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ojson {

struct Value;
using VP = std::shared_ptr<Value>;

struct Value {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  std::string s;  // string value, or raw number text
  std::vector<VP> arr;
  std::vector<std::pair<std::string, VP>> obj;

  bool is_null() const { return kind == Null; }
  // Go's encoding/json matches object keys case-insensitively (exact match preferred).
  const Value* get(const std::string& k) const {
    if (kind != Object) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return kv.second.get();
    for (auto& kv : obj) {
      if (kv.first.size() != k.size()) continue;
      bool eq = true;
      for (size_t i = 0; i < k.size() && eq; i++) {
        char a = kv.first[i], c = k[i];
        if (a >= 'A' && a <= 'Z') a = char(a - 'A' + 'a');
        if (c >= 'A' && c <= 'Z') c = char(c - 'A' + 'a');
        eq = a == c;
      }
      if (eq) return kv.second.get();
    }
    return nullptr;
  }
  long long as_int() const {
    if (kind != Number) throw std::runtime_error("json: expected number");
    char* end = nullptr;
    long long v = std::strtoll(s.c_str(), &end, 10);
    if (!end || *end != 0) throw std::runtime_error("json: expected integer, got " + s);
    return v;
  }
  const std::string& as_str() const {
    if (kind != String) throw std::runtime_error("json: expected string");
    return s;
  }
};

class Parser {
 public:
  explicit Parser(const std::string& t) : t_(t) {}
  VP parse() {
    ws();
    VP v = value();
    ws();
    if (i_ != t_.size()) err("trailing characters");
    return v;
  }

 private:
  const std::string& t_;
  size_t i_ = 0;
  [[noreturn]] void err(const char* m) {
    throw std::runtime_error(std::string("json parse error: ") + m + " at offset " + std::to_string(i_));
  }
  void ws() {
    while (i_ < t_.size() && (t_[i_] == ' ' || t_[i_] == '\n' || t_[i_] == '\r' || t_[i_] == '\t')) i_++;
  }
  bool lit(const char* w) {
    size_t n = 0;
    while (w[n]) n++;
    if (t_.compare(i_, n, w) == 0) {
      i_ += n;
      return true;
    }
    return false;
  }
  VP value() {
    if (i_ >= t_.size()) err("unexpected end");
    auto v = std::make_shared<Value>();
    char c = t_[i_];
    if (c == '{') {
      v->kind = Value::Object;
      i_++;
      ws();
      if (i_ < t_.size() && t_[i_] == '}') {
        i_++;
        return v;
      }
      for (;;) {
        ws();
        if (i_ >= t_.size() || t_[i_] != '"') err("expected key");
        std::string k = str();
        ws();
        if (i_ >= t_.size() || t_[i_] != ':') err("expected ':'");
        i_++;
        ws();
        v->obj.emplace_back(std::move(k), value());
        ws();
        if (i_ < t_.size() && t_[i_] == ',') {
          i_++;
          continue;
        }
        if (i_ < t_.size() && t_[i_] == '}') {
          i_++;
          break;
        }
        err("expected ',' or '}'");
      }
    } else if (c == '[') {
      v->kind = Value::Array;
      i_++;
      ws();
      if (i_ < t_.size() && t_[i_] == ']') {
        i_++;
        return v;
      }
      for (;;) {
        ws();
        v->arr.push_back(value());
        ws();
        if (i_ < t_.size() && t_[i_] == ',') {
          i_++;
          continue;
        }
        if (i_ < t_.size() && t_[i_] == ']') {
          i_++;
          break;
        }
        err("expected ',' or ']'");
      }
    } else if (c == '"') {
      v->kind = Value::String;
      v->s = str();
    } else if (lit("true")) {
      v->kind = Value::Bool;
      v->b = true;
    } else if (lit("false")) {
      v->kind = Value::Bool;
    } else if (lit("null")) {
      v->kind = Value::Null;
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      v->kind = Value::Number;
      size_t st = i_;
      if (t_[i_] == '-') i_++;
      while (i_ < t_.size() && ((t_[i_] >= '0' && t_[i_] <= '9') || t_[i_] == '.' || t_[i_] == 'e' ||
                                t_[i_] == 'E' || t_[i_] == '+' || t_[i_] == '-'))
        i_++;
      v->s = t_.substr(st, i_ - st);
    } else {
      err("unexpected character");
    }
    return v;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) {
      o += char(cp);
    } else if (cp < 0x800) {
      o += char(0xC0 | (cp >> 6));
      o += char(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      o += char(0xE0 | (cp >> 12));
      o += char(0x80 | ((cp >> 6) & 0x3F));
      o += char(0x80 | (cp & 0x3F));
    } else {
      o += char(0xF0 | (cp >> 18));
      o += char(0x80 | ((cp >> 12) & 0x3F));
      o += char(0x80 | ((cp >> 6) & 0x3F));
      o += char(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i_ + 4 > t_.size()) err("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
      char h = t_[i_++];
      v <<= 4;
      if (h >= '0' && h <= '9') v |= uint32_t(h - '0');
      else if (h >= 'a' && h <= 'f') v |= uint32_t(h - 'a' + 10);
      else if (h >= 'A' && h <= 'F') v |= uint32_t(h - 'A' + 10);
      else err("bad hex digit");
    }
    return v;
  }
  std::string str() {
    std::string o;
    i_++;  // opening quote
    while (i_ < t_.size()) {
      char c = t_[i_++];
      if (c == '"') return o;
      if (c != '\\') {
        o += c;
        continue;
      }
      if (i_ >= t_.size()) break;
      char e = t_[i_++];
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
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= t_.size() && t_[i_] == '\\' && t_[i_ + 1] == 'u') {
            i_ += 2;
            uint32_t lo = hex4();
            if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else cp = 0xFFFD;
          } else if (cp >= 0xD800 && cp < 0xE000) {
            cp = 0xFFFD;
          }
          put_utf8(o, cp);
          break;
        }
        default: err("bad escape");
      }
    }
    err("unterminated string");
  }
};

inline VP parse(const std::string& text) { return Parser(text).parse(); }

// Go encoding/json string encoding (HTML-escaping on, as json.Marshal does).
inline std::string go_quote(const std::string& s) {
  static const char* hx = "0123456789abcdef";
  std::string o = "\"";
  for (size_t i = 0; i < s.size(); i++) {
    unsigned char c = (unsigned char)s[i];
    if (c == '"') o += "\\\"";
    else if (c == '\\') o += "\\\\";
    else if (c == '\n') o += "\\n";
    else if (c == '\r') o += "\\r";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      o += "\\u00";
      o += hx[c >> 4];
      o += hx[c & 15];
    } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
               ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
      o += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
      i += 2;
    } else {
      o += char(c);
    }
  }
  o += "\"";
  return o;
}

}  // namespace ojson
