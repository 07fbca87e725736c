// Minimal JSON value, parser and writer.
//
// The reference depends on nlohmann/json (cpp/utils.hpp:279-294 reads
// models/*.json) and on the external ccutils library for its JSON output
// sections. Neither is available here, so the runtime carries
// this small self-contained implementation (objects keep insertion order so
// reports are stable and diff-able).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace dlnb {

class Json {
 public:
  enum class Type { Null, Bool, Number, String, Array, Object };

  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Number), n_(v), is_int_(true), i_(v) {}
  Json(long v) : type_(Type::Number), n_(static_cast<double>(v)), is_int_(true), i_(v) {}
  Json(long long v) : type_(Type::Number), n_(static_cast<double>(v)), is_int_(true), i_(v) {}
  Json(unsigned v) : Json(static_cast<long long>(v)) {}
  Json(unsigned long v) : Json(static_cast<long long>(v)) {}
  Json(unsigned long long v) : Json(static_cast<long long>(v)) {}
  Json(double v) : type_(Type::Number), n_(v) {}
  Json(float v) : type_(Type::Number), n_(v) {}
  Json(const char* s) : type_(Type::String), s_(s) {}
  Json(const std::string& s) : type_(Type::String), s_(s) {}
  template <typename T>
  Json(const std::vector<T>& v) : type_(Type::Array) {
    for (const auto& x : v) a_.emplace_back(x);
  }

  static Json array() {
    Json j;
    j.type_ = Type::Array;
    return j;
  }
  static Json object() {
    Json j;
    j.type_ = Type::Object;
    return j;
  }
  static Json parse(const std::string& text);  // throws dlnb::Error

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_number() const { return type_ == Type::Number; }
  bool is_string() const { return type_ == Type::String; }
  bool is_object() const { return type_ == Type::Object; }
  bool is_array() const { return type_ == Type::Array; }

  double as_double() const;
  long long as_int() const;
  bool as_bool() const;
  const std::string& as_string() const;

  // Object access (insertion ordered).
  bool contains(const std::string& key) const;
  const Json& at(const std::string& key) const;
  Json& operator[](const std::string& key);  // inserts Null if missing
  const std::vector<std::pair<std::string, Json>>& items() const { return o_; }

  // Array access.
  void push_back(const Json& v);
  size_t size() const;
  const Json& at(size_t i) const;

  std::string dump(int indent = -1) const;

 private:
  void dump_to(std::string& out, int indent, int depth) const;

  Type type_ = Type::Null;
  bool b_ = false;
  double n_ = 0.0;
  bool is_int_ = false;
  long long i_ = 0;
  std::string s_;
  std::vector<Json> a_;
  std::vector<std::pair<std::string, Json>> o_;
};

Json read_json_file(const std::string& path);

}  // namespace dlnb
