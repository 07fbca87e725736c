// Vectorised host loops of the CPU backend's reductions (csrc/host/simd_reduce.cpp,
// multiversioned for AVX-512 / AVX2 / baseline x86-64).
#pragma once

#include <cstddef>
#include <cstdint>

namespace dlnb {
namespace simd {

void acc_bf16(float* acc, const uint16_t* src, size_t n);    // acc[i] += bf16 src[i]
void set_bf16(float* acc, const uint16_t* src, size_t n);    // acc[i]  = bf16 src[i]
void acc_f32(float* acc, const float* src, size_t n);        // acc[i] += src[i]
void store_bf16(uint16_t* dst, const float* acc, size_t n);  // dst[i] = bf16(acc[i]), round to nearest even

}  // namespace simd
}  // namespace dlnb
