// SPDX-License-Identifier: Apache-2.0
// Minimal, dependency-free JSON DOM for the pdo control plane.
//
// Kubernetes objects travel as JSON; the control plane mutates only a few
// fields of user PodTemplates and must round-trip everything else untouched,
// so objects keep their key order and integers stay integers (no double
// round-trip of resourceVersion / replicas).  Value semantics: copying a
// Value deep-copies it (this replaces the reference's generated DeepCopy,
// api/v1/zz_generated.deepcopy.go).
#pragma once

#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace pdo {
namespace json {

class ParseError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Value;
using Array = std::deque<Value>;  // deque: appends never invalidate references
using Member = std::pair<std::string, Value>;
using Object = std::deque<Member>;

class Value {
 public:
  enum class Type { Null, Bool, Int, Double, String, Array, Object };

  Value() : t_(Type::Null) {}
  Value(std::nullptr_t) : t_(Type::Null) {}
  Value(bool b) : t_(Type::Bool), b_(b) {}
  Value(int i) : t_(Type::Int), i_(i) {}
  Value(int64_t i) : t_(Type::Int), i_(i) {}
  Value(long long i) : t_(Type::Int), i_((int64_t)i) {}
  Value(unsigned i) : t_(Type::Int), i_(i) {}
  Value(double d) : t_(Type::Double), d_(d) {}
  Value(const char* s) : t_(Type::String), s_(s) {}
  Value(std::string s) : t_(Type::String), s_(std::move(s)) {}
  Value(Array a);
  Value(Object o);
  Value(const Value& o);
  Value(Value&& o) noexcept;
  Value& operator=(const Value& o);
  Value& operator=(Value&& o) noexcept;
  ~Value();

  static Value object() { return Value(Object{}); }
  static Value array() { return Value(Array{}); }
  static Value parse(const std::string& text);

  Type type() const { return t_; }
  bool is_null() const { return t_ == Type::Null; }
  bool is_bool() const { return t_ == Type::Bool; }
  bool is_int() const { return t_ == Type::Int; }
  bool is_number() const { return t_ == Type::Int || t_ == Type::Double; }
  bool is_string() const { return t_ == Type::String; }
  bool is_array() const { return t_ == Type::Array; }
  bool is_object() const { return t_ == Type::Object; }

  bool as_bool(bool def = false) const { return t_ == Type::Bool ? b_ : def; }
  int64_t as_int(int64_t def = 0) const;
  double as_double(double def = 0) const;
  const std::string& as_string() const;  // "" when not a string
  std::string str(const std::string& def = "") const { return t_ == Type::String ? s_ : def; }

  // arrays
  Array& arr();
  const Array& arr() const;
  size_t size() const;
  Value& push_back(Value v);
  Value& operator[](size_t i) { return arr()[i]; }
  const Value& operator[](size_t i) const { return arr()[i]; }
  Value& operator[](int i) { return arr()[(size_t)i]; }  // disambiguates literal 0 vs const char*
  const Value& operator[](int i) const { return arr()[(size_t)i]; }

  // objects (insertion-ordered)
  Object& obj();
  const Object& obj() const;
  bool has(const std::string& k) const { return find(k) != nullptr; }
  const Value* find(const std::string& k) const;
  Value* find(const std::string& k);
  Value& operator[](const std::string& k);  // creates (and converts null → object)
  Value& operator[](const char* k) { return (*this)[std::string(k)]; }
  const Value& get(const std::string& k) const;  // Null sentinel when missing
  bool erase(const std::string& k);
  void set(const std::string& k, Value v) { (*this)[k] = std::move(v); }

  // dotted path helpers: "spec.worker.replicas"
  const Value& at_path(const std::string& path) const;
  Value& ensure_path(const std::string& path);

  std::string dump(int indent = -1) const;
  bool operator==(const Value& o) const;
  bool operator!=(const Value& o) const { return !(*this == o); }

 private:
  void dump_to(std::string& out, int indent, int depth) const;
  void destroy();
  void copy_from(const Value& o);

  Type t_;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::string s_;
  std::unique_ptr<Array> a_;
  std::unique_ptr<Object> o_;
};

const Value& null_value();
std::string quote(const std::string& s);

}  // namespace json
}  // namespace pdo
