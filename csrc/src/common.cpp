#include "dlnb/common.hpp"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace dlnb {

size_t dtype_size(DType t) {
  switch (t) {
    case DType::BF16: return 2;
    case DType::FP16: return 2;
    case DType::FP32: return 4;
    case DType::FP8_E4M3: return 1;
    case DType::FP8_E5M2: return 1;
  }
  return 0;
}

const char* dtype_name(DType t) {
  switch (t) {
    case DType::BF16: return "bf16";
    case DType::FP16: return "fp16";
    case DType::FP32: return "fp32";
    case DType::FP8_E4M3: return "fp8_e4m3";
    case DType::FP8_E5M2: return "fp8_e5m2";
  }
  return "?";
}

DType parse_dtype(const std::string& s0) {
  std::string s = s0;
  std::transform(s.begin(), s.end(), s.begin(), ::tolower);
  if (s == "bf16" || s == "bfloat16") return DType::BF16;
  if (s == "fp16" || s == "float16" || s == "half") return DType::FP16;
  if (s == "fp32" || s == "float32" || s == "float") return DType::FP32;
  if (s == "fp8" || s == "float8" || s == "fp8_e4m3" || s == "e4m3") return DType::FP8_E4M3;
  if (s == "bf8" || s == "fp8_e5m2" || s == "e5m2") return DType::FP8_E5M2;
  DLNB_THROW("unknown dtype '" << s0 << "'");
}

std::string& last_error_message() {
  thread_local std::string m;
  return m;
}

std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
  return out;
}

bool starts_with(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(0, p.size(), p) == 0;
}

bool ends_with(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0;
}

std::string env_or(const char* name, const std::string& dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::string(v) : dflt;
}

long long env_int(const char* name, long long dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  long long r = std::strtoll(v, &end, 10);
  return (end && *end == '\0') ? r : dflt;
}

float bf16_to_float(uint16_t v) {
  uint32_t u = static_cast<uint32_t>(v) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

uint16_t float_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

float fp16_to_float(uint16_t h) {
  uint32_t sign = (h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1f;
  uint32_t man = h & 0x3ff;
  uint32_t u;
  if (exp == 0) {
    if (man == 0) {
      u = sign;
    } else {  // subnormal
      int e = -1;
      do {
        ++e;
        man <<= 1;
      } while ((man & 0x400) == 0);
      u = sign | ((127 - 15 - e) << 23) | ((man & 0x3ff) << 13);
    }
  } else if (exp == 31) {
    u = sign | 0x7f800000u | (man << 13);
  } else {
    u = sign | ((exp + 127 - 15) << 23) | (man << 13);
  }
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

uint16_t float_to_fp16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  uint32_t sign = (u >> 16) & 0x8000u;
  int32_t exp = static_cast<int32_t>((u >> 23) & 0xff) - 127 + 15;
  uint32_t man = u & 0x7fffffu;
  if (((u >> 23) & 0xff) == 0xff) return static_cast<uint16_t>(sign | 0x7c00u | (man ? 0x200u : 0));
  if (exp >= 31) return static_cast<uint16_t>(sign | 0x7c00u);
  if (exp <= 0) {
    if (exp < -10) return static_cast<uint16_t>(sign);
    man |= 0x800000u;
    uint32_t shift = static_cast<uint32_t>(14 - exp);
    uint32_t half = man >> shift;
    uint32_t rem = man & ((1u << shift) - 1);
    uint32_t mid = 1u << (shift - 1);
    if (rem > mid || (rem == mid && (half & 1))) ++half;
    return static_cast<uint16_t>(sign | half);
  }
  uint32_t half = sign | (static_cast<uint32_t>(exp) << 10) | (man >> 13);
  uint32_t rem = man & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (half & 1))) ++half;
  return static_cast<uint16_t>(half);
}

// OCP FP8 e4m3fn: bias 7, no infinities, 0x7f/0xff are NaN, max 448.
// Decoded through a 256-entry table (the host checks of commtest / the shm
// backend decode millions of elements).
namespace {
float fp8e4m3_decode_slow(uint8_t v) {
  int sign = (v >> 7) & 1;
  int exp = (v >> 3) & 0xf;
  int man = v & 7;
  float r;
  if (exp == 0xf && man == 7) return std::nanf("");
  if (exp == 0)
    r = std::ldexp(static_cast<float>(man) / 8.0f, -6);
  else
    r = std::ldexp(1.0f + static_cast<float>(man) / 8.0f, exp - 7);
  return sign ? -r : r;
}
struct Fp8e4m3Table {
  float v[256];
  Fp8e4m3Table() {
    for (int c = 0; c < 256; ++c) v[c] = fp8e4m3_decode_slow(static_cast<uint8_t>(c));
  }
};
}  // namespace

float fp8e4m3_to_float(uint8_t v) {
  static const Fp8e4m3Table t;
  return t.v[v];
}

// Round to nearest, ties to even, saturating at +-448 (the conversion the
// gfx950 cvt instructions do with saturation on).
uint8_t float_to_fp8e4m3(float f) {
  if (std::isnan(f)) return 0x7f;
  uint8_t sign = std::signbit(f) ? 0x80 : 0;
  float a = std::fabs(f);
  if (a >= 448.0f) return sign | 0x7e;  // saturate to max finite
  if (a < 0.015625f) {
    // subnormal range (below 2^-6): code = round(a / 2^-9); 8 is the
    // smallest normal (exponent 1, mantissa 0), which the same code denotes
    return sign | static_cast<uint8_t>(std::nearbyint(a * 512.0f));
  }
  uint32_t u;
  std::memcpy(&u, &a, 4);
  // keep 3 mantissa bits, round to nearest even (a carry bumps the exponent)
  u += 0x7ffffu + ((u >> 20) & 1u);
  uint32_t code = (u >> 20) - ((127u - 7u) << 3);
  return sign | static_cast<uint8_t>(std::min<uint32_t>(code, 0x7e));
}

// OCP FP8 e5m2: bias 15, IEEE-like with inf/NaN.
float fp8e5m2_to_float(uint8_t v) { return fp16_to_float(static_cast<uint16_t>(v) << 8); }

uint8_t float_to_fp8e5m2(float f) {
  uint16_t h = float_to_fp16(f);
  if ((h & 0x7c00u) == 0x7c00u) return static_cast<uint8_t>(h >> 8) | ((h & 0x3ffu) ? 0x2 : 0);
  uint16_t r = h >> 8;
  uint16_t rem = h & 0xff;
  if (rem > 0x80 || (rem == 0x80 && (r & 1))) ++r;
  return static_cast<uint8_t>(r);
}

}  // namespace dlnb
