// Minimal JSON reader/writer for the oracle's fixture I/O (test infrastructure only).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace oj {

struct Value {
  enum Kind { Null, Bool, Int, Dbl, Str, Arr, Obj } kind = Null;
  bool b = false;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::vector<Value> a;
  std::vector<std::pair<std::string, Value>> o;

  bool is_null() const { return kind == Null; }
  const Value* get(const std::string& k) const {
    if (kind != Obj) return nullptr;
    for (auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  bool has(const std::string& k) const {
    const Value* v = get(k);
    return v && !v->is_null();
  }
  int64_t as_int(int64_t dflt = 0) const {
    if (kind == Int) return i;
    if (kind == Dbl) return (int64_t)d;
    if (kind == Bool) return b;
    return dflt;
  }
  double as_dbl() const { return kind == Int ? (double)i : d; }
  bool as_bool(bool dflt = false) const { return kind == Bool ? b : dflt; }
  const std::string& as_str() const {
    static const std::string empty;
    return kind == Str ? s : empty;
  }
  int64_t int_at(const std::string& k, int64_t dflt = 0) const {
    const Value* v = get(k);
    return v ? v->as_int(dflt) : dflt;
  }
  std::string str_at(const std::string& k) const {
    const Value* v = get(k);
    return v ? v->as_str() : std::string();
  }
  bool bool_at(const std::string& k, bool dflt = false) const {
    const Value* v = get(k);
    return v ? v->as_bool(dflt) : dflt;
  }
  const std::vector<Value>& arr_at(const std::string& k) const {
    static const std::vector<Value> empty;
    const Value* v = get(k);
    return (v && v->kind == Arr) ? v->a : empty;
  }
};

class Parser {
 public:
  explicit Parser(const char* p) : p_(p) {}
  Value parse() {
    Value v = value();
    ws();
    if (*p_) throw std::runtime_error("json: trailing data");
    return v;
  }

 private:
  const char* p_;
  void ws() {
    while (*p_ == ' ' || *p_ == '\n' || *p_ == '\t' || *p_ == '\r') ++p_;
  }
  Value value() {
    ws();
    Value v;
    char c = *p_;
    if (c == '{') {
      v.kind = Value::Obj;
      ++p_;
      ws();
      if (*p_ == '}') { ++p_; return v; }
      for (;;) {
        ws();
        std::string k = str();
        ws();
        if (*p_++ != ':') throw std::runtime_error("json: expected ':'");
        v.o.emplace_back(std::move(k), value());
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == '}') { ++p_; break; }
        throw std::runtime_error("json: expected ',' or '}'");
      }
    } else if (c == '[') {
      v.kind = Value::Arr;
      ++p_;
      ws();
      if (*p_ == ']') { ++p_; return v; }
      for (;;) {
        v.a.push_back(value());
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == ']') { ++p_; break; }
        throw std::runtime_error("json: expected ',' or ']'");
      }
    } else if (c == '"') {
      v.kind = Value::Str;
      v.s = str();
    } else if (c == 't' && !strncmp(p_, "true", 4)) {
      v.kind = Value::Bool; v.b = true; p_ += 4;
    } else if (c == 'f' && !strncmp(p_, "false", 5)) {
      v.kind = Value::Bool; v.b = false; p_ += 5;
    } else if (c == 'n' && !strncmp(p_, "null", 4)) {
      p_ += 4;
    } else {
      const char* s = p_;
      bool flt = false;
      if (*p_ == '-' || *p_ == '+') ++p_;
      while ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '-' || *p_ == '+') {
        if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') flt = true;
        ++p_;
      }
      if (p_ == s) throw std::runtime_error("json: bad value");
      std::string num(s, p_ - s);
      if (flt) { v.kind = Value::Dbl; v.d = strtod(num.c_str(), nullptr); }
      else { v.kind = Value::Int; v.i = strtoll(num.c_str(), nullptr, 10); }
    }
    return v;
  }
  static int strncmp(const char* a, const char* b, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      if (a[i] != b[i]) return 1;
      if (!a[i]) return 1;
    }
    return 0;
  }
  std::string str() {
    if (*p_ != '"') throw std::runtime_error("json: expected string");
    ++p_;
    std::string out;
    while (*p_ && *p_ != '"') {
      if (*p_ == '\\') {
        ++p_;
        switch (*p_) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {
            unsigned cp = (unsigned)strtoul(std::string(p_ + 1, 4).c_str(), nullptr, 16);
            p_ += 4;
            if (cp < 0x80) out += (char)cp;
            else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
            else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
            break;
          }
          default: out += *p_;
        }
        ++p_;
      } else {
        out += *p_++;
      }
    }
    if (*p_ != '"') throw std::runtime_error("json: unterminated string");
    ++p_;
    return out;
  }
};

inline Value parse(const std::string& s) { return Parser(s.c_str()).parse(); }

// ---- writer ----
inline void esc(std::string& out, const std::string& s) {
  out += '"';
  for (char c : s) {
    if (c == '"' || c == '\\') { out += '\\'; out += c; }
    else if (c == '\n') out += "\\n";
    else if ((unsigned char)c < 0x20) { char buf[8]; snprintf(buf, 8, "\\u%04x", c); out += buf; }
    else out += c;
  }
  out += '"';
}

}  // namespace oj
