// Host SIMD loops of the CPU backend's reductions (comm_shm.cpp), built as
// plain host C++ (no HIP device pass: function multiversioning is host-only)
// for AVX-512, AVX2 and the x86-64 baseline, the widest picked at load time.
// The shared-memory collectives are bound by these conversions + sums, not by
// memory: on the 8-CPU container the 2-rank registered all-reduce went from
// 6.5 to 8.5-9.2 GB/s bus bandwidth and reduce-scatter from 3.5 to 6.6-7.4
// GB/s with 16-wide AVX-512 instead of the 4-wide SSE loops.
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "dlnb/host_simd.hpp"

namespace dlnb {
namespace simd {

namespace {

inline float bf16f(uint16_t v) {
  uint32_t u = static_cast<uint32_t>(v) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// round to nearest even; NaN stays NaN (quiet bit set)
inline uint16_t fbf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint32_t r = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
  const uint32_t n = (u >> 16) | 0x40u;
  return static_cast<uint16_t>((u & 0x7fffffffu) > 0x7f800000u ? n : r);
}

}  // namespace

#define DLNB_SIMD_CLONES __attribute__((target_clones("avx512bw", "avx2", "default")))

DLNB_SIMD_CLONES void acc_bf16(float* __restrict acc, const uint16_t* __restrict src, size_t n) {
  for (size_t i = 0; i < n; ++i) acc[i] += bf16f(src[i]);
}

DLNB_SIMD_CLONES void set_bf16(float* __restrict acc, const uint16_t* __restrict src, size_t n) {
  for (size_t i = 0; i < n; ++i) acc[i] = bf16f(src[i]);
}

DLNB_SIMD_CLONES void acc_f32(float* __restrict acc, const float* __restrict src, size_t n) {
  for (size_t i = 0; i < n; ++i) acc[i] += src[i];
}

DLNB_SIMD_CLONES void store_bf16(uint16_t* __restrict dst, const float* __restrict acc, size_t n) {
  for (size_t i = 0; i < n; ++i) dst[i] = fbf16(acc[i]);
}

}  // namespace simd
}  // namespace dlnb
