#include "dlnb/json.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

#include "dlnb/common.hpp"

namespace dlnb {

namespace {

struct Parser {
  const std::string& t;
  size_t p = 0;

  explicit Parser(const std::string& text) : t(text) {}

  void ws() {
    while (p < t.size() && (t[p] == ' ' || t[p] == '\n' || t[p] == '\r' || t[p] == '\t')) ++p;
  }
  [[noreturn]] void fail(const char* what) { DLNB_THROW("json parse error at offset " << p << ": " << what); }
  char peek() {
    ws();
    if (p >= t.size()) fail("unexpected end");
    return t[p];
  }
  void expect(char c) {
    if (peek() != c) fail("unexpected character");
    ++p;
  }

  Json value() {
    char c = peek();
    if (c == '{') return object();
    if (c == '[') return array();
    if (c == '"') return Json(str());
    if (t.compare(p, 4, "true") == 0) {
      p += 4;
      return Json(true);
    }
    if (t.compare(p, 5, "false") == 0) {
      p += 5;
      return Json(false);
    }
    if (t.compare(p, 4, "null") == 0) {
      p += 4;
      return Json();
    }
    return number();
  }

  Json number() {
    size_t b = p;
    bool is_float = false;
    if (p < t.size() && (t[p] == '-' || t[p] == '+')) ++p;
    while (p < t.size()) {
      char c = t[p];
      if (c >= '0' && c <= '9') {
        ++p;
      } else if (c == '.' || c == 'e' || c == 'E' || c == '-' || c == '+') {
        is_float = true;
        ++p;
      } else {
        break;
      }
    }
    if (b == p) fail("bad value");
    std::string s = t.substr(b, p - b);
    if (!is_float) return Json(std::strtoll(s.c_str(), nullptr, 10));
    return Json(std::strtod(s.c_str(), nullptr));
  }

  std::string str() {
    expect('"');
    std::string out;
    while (p < t.size() && t[p] != '"') {
      char c = t[p++];
      if (c == '\\') {
        if (p >= t.size()) fail("bad escape");
        char e = t[p++];
        switch (e) {
          case 'n': out.push_back('\n'); break;
          case 't': out.push_back('\t'); break;
          case 'r': out.push_back('\r'); break;
          case 'b': out.push_back('\b'); break;
          case 'f': out.push_back('\f'); break;
          case 'u': {
            if (p + 4 > t.size()) fail("bad \\u escape");
            unsigned cp = static_cast<unsigned>(std::strtoul(t.substr(p, 4).c_str(), nullptr, 16));
            p += 4;
            if (cp < 0x80) {
              out.push_back(static_cast<char>(cp));
            } else if (cp < 0x800) {
              out.push_back(static_cast<char>(0xc0 | (cp >> 6)));
              out.push_back(static_cast<char>(0x80 | (cp & 0x3f)));
            } else {
              out.push_back(static_cast<char>(0xe0 | (cp >> 12)));
              out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3f)));
              out.push_back(static_cast<char>(0x80 | (cp & 0x3f)));
            }
            break;
          }
          default: out.push_back(e);
        }
      } else {
        out.push_back(c);
      }
    }
    if (p >= t.size()) fail("unterminated string");
    ++p;
    return out;
  }

  Json array() {
    expect('[');
    Json a = Json::array();
    if (peek() == ']') {
      ++p;
      return a;
    }
    for (;;) {
      a.push_back(value());
      char c = peek();
      ++p;
      if (c == ']') break;
      if (c != ',') fail("expected , or ]");
    }
    return a;
  }

  Json object() {
    expect('{');
    Json o = Json::object();
    if (peek() == '}') {
      ++p;
      return o;
    }
    for (;;) {
      if (peek() != '"') fail("expected key");
      std::string k = str();
      expect(':');
      o[k] = value();
      char c = peek();
      ++p;
      if (c == '}') break;
      if (c != ',') fail("expected , or }");
    }
    return o;
  }
};

void escape_to(std::string& out, const std::string& s) {
  out.push_back('"');
  for (char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\t': out += "\\t"; break;
      case '\r': out += "\\r"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", c);
          out += buf;
        } else {
          out.push_back(c);
        }
    }
  }
  out.push_back('"');
}

}  // namespace

Json Json::parse(const std::string& text) {
  Parser ps(text);
  Json v = ps.value();
  ps.ws();
  if (ps.p != text.size()) ps.fail("trailing characters");
  return v;
}

double Json::as_double() const {
  if (type_ != Type::Number) DLNB_THROW("json value is not a number");
  return n_;
}

long long Json::as_int() const {
  if (type_ != Type::Number) DLNB_THROW("json value is not a number");
  return is_int_ ? i_ : static_cast<long long>(n_);
}

bool Json::as_bool() const {
  if (type_ != Type::Bool) DLNB_THROW("json value is not a bool");
  return b_;
}

const std::string& Json::as_string() const {
  if (type_ != Type::String) DLNB_THROW("json value is not a string");
  return s_;
}

bool Json::contains(const std::string& key) const {
  if (type_ != Type::Object) return false;
  for (const auto& kv : o_)
    if (kv.first == key) return true;
  return false;
}

const Json& Json::at(const std::string& key) const {
  if (type_ != Type::Object) DLNB_THROW("json value is not an object");
  for (const auto& kv : o_)
    if (kv.first == key) return kv.second;
  DLNB_THROW("json key not found: " << key);
}

Json& Json::operator[](const std::string& key) {
  if (type_ == Type::Null) type_ = Type::Object;
  if (type_ != Type::Object) DLNB_THROW("json value is not an object");
  for (auto& kv : o_)
    if (kv.first == key) return kv.second;
  o_.emplace_back(key, Json());
  return o_.back().second;
}

void Json::push_back(const Json& v) {
  if (type_ == Type::Null) type_ = Type::Array;
  if (type_ != Type::Array) DLNB_THROW("json value is not an array");
  a_.push_back(v);
}

size_t Json::size() const {
  if (type_ == Type::Array) return a_.size();
  if (type_ == Type::Object) return o_.size();
  return 0;
}

const Json& Json::at(size_t i) const {
  if (type_ != Type::Array || i >= a_.size()) DLNB_THROW("json array index out of range");
  return a_[i];
}

std::string Json::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  auto nl = [&](int d) {
    if (indent >= 0) {
      out.push_back('\n');
      out.append(static_cast<size_t>(indent * d), ' ');
    }
  };
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Number: {
      if (is_int_) {
        out += std::to_string(i_);
      } else if (!std::isfinite(n_)) {
        out += "null";
      } else {
        char buf[64];
        std::snprintf(buf, sizeof(buf), "%.12g", n_);  // 1e-5 us at a 10-s timeline offset
        out += buf;
      }
      break;
    }
    case Type::String: escape_to(out, s_); break;
    case Type::Array: {
      out.push_back('[');
      for (size_t i = 0; i < a_.size(); ++i) {
        if (i) out.push_back(',');
        if (indent >= 0 && a_[i].type_ >= Type::Array) nl(depth + 1);
        a_[i].dump_to(out, indent, depth + 1);
      }
      out.push_back(']');
      break;
    }
    case Type::Object: {
      out.push_back('{');
      for (size_t i = 0; i < o_.size(); ++i) {
        if (i) out.push_back(',');
        nl(depth + 1);
        escape_to(out, o_[i].first);
        out.push_back(':');
        if (indent >= 0) out.push_back(' ');
        o_[i].second.dump_to(out, indent, depth + 1);
      }
      if (!o_.empty()) nl(depth);
      out.push_back('}');
      break;
    }
  }
}

Json read_json_file(const std::string& path) {
  std::ifstream f(path);
  if (!f) DLNB_THROW("cannot open json file " << path);
  std::stringstream ss;
  ss << f.rdbuf();
  return Json::parse(ss.str());
}

}  // namespace dlnb
