// SPDX-License-Identifier: Apache-2.0
#include "json.h"

#include <cmath>
#include <cstdio>
#include <cerrno>
#include <cstdlib>
#include <cstring>

namespace pdo {
namespace json {

const Value& null_value() {
  static const Value n;
  return n;
}

Value::Value(Array a) : t_(Type::Array), a_(new Array(std::move(a))) {}
Value::Value(Object o) : t_(Type::Object), o_(new Object(std::move(o))) {}
Value::Value(const Value& o) { copy_from(o); }
Value::Value(Value&& o) noexcept
    : t_(o.t_), b_(o.b_), i_(o.i_), d_(o.d_), s_(std::move(o.s_)), a_(std::move(o.a_)), o_(std::move(o.o_)) {
  o.t_ = Type::Null;
}
Value& Value::operator=(const Value& o) {
  if (this != &o) {
    Value tmp(o);
    *this = std::move(tmp);
  }
  return *this;
}
Value& Value::operator=(Value&& o) noexcept {
  if (this != &o) {
    t_ = o.t_;
    b_ = o.b_;
    i_ = o.i_;
    d_ = o.d_;
    s_ = std::move(o.s_);
    a_ = std::move(o.a_);
    o_ = std::move(o.o_);
    o.t_ = Type::Null;
  }
  return *this;
}
Value::~Value() = default;

void Value::copy_from(const Value& o) {
  t_ = o.t_;
  b_ = o.b_;
  i_ = o.i_;
  d_ = o.d_;
  s_ = o.s_;
  if (o.a_) a_.reset(new Array(*o.a_));
  if (o.o_) o_.reset(new Object(*o.o_));
}

int64_t Value::as_int(int64_t def) const {
  if (t_ == Type::Int) return i_;
  if (t_ == Type::Double) return (int64_t)d_;
  return def;
}
double Value::as_double(double def) const {
  if (t_ == Type::Double) return d_;
  if (t_ == Type::Int) return (double)i_;
  return def;
}
const std::string& Value::as_string() const {
  static const std::string empty;
  return t_ == Type::String ? s_ : empty;
}

Array& Value::arr() {
  if (t_ == Type::Null) {
    t_ = Type::Array;
    a_.reset(new Array());
  }
  if (t_ != Type::Array) throw std::runtime_error("json: not an array");
  return *a_;
}
const Array& Value::arr() const {
  static const Array empty;
  return t_ == Type::Array ? *a_ : empty;
}
size_t Value::size() const {
  if (t_ == Type::Array) return a_->size();
  if (t_ == Type::Object) return o_->size();
  return 0;
}
Value& Value::push_back(Value v) {
  arr().push_back(std::move(v));
  return a_->back();
}

Object& Value::obj() {
  if (t_ == Type::Null) {
    t_ = Type::Object;
    o_.reset(new Object());
  }
  if (t_ != Type::Object) throw std::runtime_error("json: not an object");
  return *o_;
}
const Object& Value::obj() const {
  static const Object empty;
  return t_ == Type::Object ? *o_ : empty;
}
const Value* Value::find(const std::string& k) const {
  if (t_ != Type::Object) return nullptr;
  for (auto& m : *o_)
    if (m.first == k) return &m.second;
  return nullptr;
}
Value* Value::find(const std::string& k) {
  if (t_ != Type::Object) return nullptr;
  for (auto& m : *o_)
    if (m.first == k) return &m.second;
  return nullptr;
}
Value& Value::operator[](const std::string& k) {
  Object& o = obj();
  for (auto& m : o)
    if (m.first == k) return m.second;
  o.emplace_back(k, Value());
  return o.back().second;
}
const Value& Value::get(const std::string& k) const {
  const Value* v = find(k);
  return v ? *v : null_value();
}
bool Value::erase(const std::string& k) {
  if (t_ != Type::Object) return false;
  for (auto it = o_->begin(); it != o_->end(); ++it)
    if (it->first == k) {
      o_->erase(it);
      return true;
    }
  return false;
}

const Value& Value::at_path(const std::string& path) const {
  const Value* cur = this;
  size_t start = 0;
  while (start <= path.size()) {
    size_t dot = path.find('.', start);
    std::string key = path.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
    cur = cur->find(key);
    if (!cur) return null_value();
    if (dot == std::string::npos) break;
    start = dot + 1;
  }
  return *cur;
}
Value& Value::ensure_path(const std::string& path) {
  Value* cur = this;
  size_t start = 0;
  while (true) {
    size_t dot = path.find('.', start);
    std::string key = path.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
    cur = &(*cur)[key];
    if (dot == std::string::npos) break;
    start = dot + 1;
  }
  return *cur;
}

bool Value::operator==(const Value& o) const {
  if (is_number() && o.is_number()) {
    if (t_ == Type::Int && o.t_ == Type::Int) return i_ == o.i_;
    return as_double() == o.as_double();
  }
  if (t_ != o.t_) return false;
  switch (t_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::String: return s_ == o.s_;
    case Type::Array: return *a_ == *o.a_;
    case Type::Object: {
      // order-insensitive comparison (semantic equality of objects)
      if (o_->size() != o.o_->size()) return false;
      for (auto& m : *o_) {
        const Value* v = o.find(m.first);
        if (!v || !(*v == m.second)) return false;
      }
      return true;
    }
    default: return false;
  }
}

// ------------------------------------------------------------------ dump
std::string quote(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out.push_back((char)c);
        }
    }
  }
  out.push_back('"');
  return out;
}

static void newline(std::string& out, int indent, int depth) {
  if (indent < 0) return;
  out.push_back('\n');
  out.append((size_t)indent * depth, ' ');
}

void Value::dump_to(std::string& out, int indent, int depth) const {
  switch (t_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: out += std::to_string(i_); break;
    case Type::Double: {
      if (!std::isfinite(d_)) {
        out += "null";
        break;
      }
      char buf[32];
      snprintf(buf, sizeof buf, "%.17g", d_);
      out += buf;
      break;
    }
    case Type::String: out += quote(s_); break;
    case Type::Array: {
      out.push_back('[');
      bool first = true;
      for (auto& v : *a_) {
        if (!first) out.push_back(',');
        first = false;
        newline(out, indent, depth + 1);
        v.dump_to(out, indent, depth + 1);
      }
      if (!a_->empty()) newline(out, indent, depth);
      out.push_back(']');
      break;
    }
    case Type::Object: {
      out.push_back('{');
      bool first = true;
      for (auto& m : *o_) {
        if (!first) out.push_back(',');
        first = false;
        newline(out, indent, depth + 1);
        out += quote(m.first);
        out += indent >= 0 ? ": " : ":";
        m.second.dump_to(out, indent, depth + 1);
      }
      if (!o_->empty()) newline(out, indent, depth);
      out.push_back('}');
      break;
    }
  }
}

std::string Value::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

// ------------------------------------------------------------------ parse
namespace {
struct Parser {
  const char* p;
  const char* end;
  int depth = 0;

  [[noreturn]] void fail(const char* what) {
    throw ParseError(std::string("json parse error: ") + what + " at offset " +
                     std::to_string((long)(p - (end - (end - p)))));
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p;
  }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(end - p) >= n && memcmp(p, s, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  static void utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) {
      out.push_back((char)cp);
    } else if (cp < 0x800) {
      out.push_back((char)(0xC0 | (cp >> 6)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back((char)(0xE0 | (cp >> 12)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      out.push_back((char)(0xF0 | (cp >> 18)));
      out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  unsigned hex4() {
    if (end - p < 4) fail("short \\u escape");
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string str() {
    if (p >= end || *p != '"') fail("expected string");
    ++p;
    std::string out;
    while (true) {
      if (p >= end) fail("unterminated string");
      char c = *p++;
      if (c == '"') break;
      if (c == '\\') {
        if (p >= end) fail("bad escape");
        char e = *p++;
        switch (e) {
          case '"': out.push_back('"'); break;
          case '\\': out.push_back('\\'); break;
          case '/': out.push_back('/'); break;
          case 'b': out.push_back('\b'); break;
          case 'f': out.push_back('\f'); break;
          case 'n': out.push_back('\n'); break;
          case 'r': out.push_back('\r'); break;
          case 't': out.push_back('\t'); break;
          case 'u': {
            unsigned cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              p += 2;
              unsigned lo = hex4();
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            utf8(out, cp);
            break;
          }
          default: fail("unknown escape");
        }
      } else {
        out.push_back(c);
      }
    }
    return out;
  }
  Value num() {
    const char* s = p;
    bool is_float = false;
    if (p < end && (*p == '-' || *p == '+')) ++p;
    while (p < end && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '-' || *p == '+')) {
      if (*p == '.' || *p == 'e' || *p == 'E') is_float = true;
      ++p;
    }
    std::string t(s, p);
    if (t.empty() || t == "-") fail("bad number");
    if (!is_float) {
      errno = 0;
      long long v = strtoll(t.c_str(), nullptr, 10);
      if (errno == 0) return Value((int64_t)v);
    }
    return Value(strtod(t.c_str(), nullptr));
  }
  Value val() {
    if (++depth > 512) fail("nesting too deep");
    ws();
    if (p >= end) fail("unexpected end");
    Value v;
    char c = *p;
    if (c == '{') {
      ++p;
      v = Value::object();
      ws();
      if (p < end && *p == '}') {
        ++p;
      } else {
        while (true) {
          ws();
          std::string k = str();
          ws();
          if (p >= end || *p != ':') fail("expected ':'");
          ++p;
          v.obj().emplace_back(std::move(k), val());
          ws();
          if (p < end && *p == ',') {
            ++p;
            continue;
          }
          if (p < end && *p == '}') {
            ++p;
            break;
          }
          fail("expected ',' or '}'");
        }
      }
    } else if (c == '[') {
      ++p;
      v = Value::array();
      ws();
      if (p < end && *p == ']') {
        ++p;
      } else {
        while (true) {
          v.arr().push_back(val());
          ws();
          if (p < end && *p == ',') {
            ++p;
            continue;
          }
          if (p < end && *p == ']') {
            ++p;
            break;
          }
          fail("expected ',' or ']'");
        }
      }
    } else if (c == '"') {
      v = Value(str());
    } else if (lit("true")) {
      v = Value(true);
    } else if (lit("false")) {
      v = Value(false);
    } else if (lit("null")) {
      v = Value();
    } else {
      v = num();
    }
    --depth;
    return v;
  }
};
}  // namespace

Value Value::parse(const std::string& text) {
  Parser ps{text.data(), text.data() + text.size()};
  Value v = ps.val();
  ps.ws();
  if (ps.p != ps.end) ps.fail("trailing characters");
  return v;
}

}  // namespace json
}  // namespace pdo
