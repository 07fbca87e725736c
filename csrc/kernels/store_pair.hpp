// Epilogue store of two adjacent 16 x 16 MFMA output fragments (gfx950).
//
// After a 16x16 MFMA with the operands swapped (B rows as src0, A rows as
// src1: gemm_8phase.hip, gemm_4wave_fp8.hip) lane (r16, h) = lane r16 + 16 h
// holds C[row r16][cols 4h .. 4h+3] of a fragment, so a fragment is one
// 8-byte store per lane: 16 rows x 32 B per store instruction. An epilogue of
// such stores is store-issue bound (cdna_hip_programming.md T21).
//
// Two fragments F0 (cols n .. n+15) and F1 (cols n+16 .. n+31) of the same
// rows become ONE 16-byte store per lane with v_permlane16_swap: it swaps the
// odd 16-lane rows of its first operand with the even rows of its second, so
// swap(F0, F1) per dword leaves lane h = 0 with F0 cols 0..7, h = 1 with F1
// cols 0..7, h = 2 with F0 cols 8..15 and h = 3 with F1 cols 8..15: half the
// store instructions, 16 rows x 64 contiguous bytes each. Needs 16-byte
// aligned rows (ldc % 8 == 0 and a 16-byte aligned C), decided per launch
// (`wide`, wave-uniform); otherwise the two 8-byte stores.
#pragma once

#include <hip/hip_runtime.h>

namespace dlnb {
namespace kernels {
namespace epi {

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;

__device__ __forceinline__ bf16x4_t to_bf16(const f32x4_t& a) {
  bf16x4_t o;
  o[0] = static_cast<__bf16>(a[0]);
  o[1] = static_cast<__bf16>(a[1]);
  o[2] = static_cast<__bf16>(a[2]);
  o[3] = static_cast<__bf16>(a[3]);
  return o;
}

// row: C + (this lane's row) * ldc + (the pair's first column); h = lane / 16.
// NT: non-temporal (streaming) stores - the deadline stand-in's output is
// never read, and lines it leaves dirty in the XCDs' L2s have to be written
// back at the kernel's end-of-kernel release: tens of us that every kernel
// after it on any queue waits for (round 5: one-wave stamp / done kernels
// took ~40 us right after a deadline GEMM ended).
template <bool NT = false>
__device__ __forceinline__ void store_pair(__bf16* row, const f32x4_t& f0, const f32x4_t& f1, int h, bool wide) {
  const bf16x4_t o0 = to_bf16(f0), o1 = to_bf16(f1);
  if (wide) {
    const u32x2_t u0 = __builtin_bit_cast(u32x2_t, o0), u1 = __builtin_bit_cast(u32x2_t, o1);
    const auto s0 = __builtin_amdgcn_permlane16_swap(u0[0], u1[0], false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(u0[1], u1[1], false, false);
    const u32x4_t v = {s0[0], s1[0], s0[1], s1[1]};
    u32x4_t* p = reinterpret_cast<u32x4_t*>(row + (h & 1) * 16 + (h >> 1) * 8);
    if constexpr (NT)
      __builtin_nontemporal_store(v, p);
    else
      *p = v;
  } else {
    bf16x4_t* p0 = reinterpret_cast<bf16x4_t*>(row + 4 * h);
    bf16x4_t* p1 = reinterpret_cast<bf16x4_t*>(row + 16 + 4 * h);
    if constexpr (NT) {
      __builtin_nontemporal_store(o0, p0);
      __builtin_nontemporal_store(o1, p1);
    } else {
      *p0 = o0;
      *p1 = o1;
    }
  }
}

// One fragment alone (an odd fragment count per row): the 8-byte store.
__device__ __forceinline__ void store_one(__bf16* row, const f32x4_t& f, int h) {
  *reinterpret_cast<bf16x4_t*>(row + 4 * h) = to_bf16(f);
}

__device__ __forceinline__ bool wide_ok(const __bf16* C, int ldc) {
  return (ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(C) & 15) == 0;
}

}  // namespace epi
}  // namespace kernels
}  // namespace dlnb
