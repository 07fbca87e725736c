// Host launchers for the hand-written CDNA4 (gfx950) kernels.
//
// The reference has no GPU kernels at all: compute is host usleep()
// (SURVEY.md §2.1 "GPU kernel inventory: none"). These kernels are new
// capability: they put real, stream-ordered work on the MI355X so the
// collectives contend for CUs / HBM / power the way they do in training.
//   * fill_random       - vectorised hash fill (uniform [-1,1)), any dtype
//   * idle_wait         - one wave sleeps on s_memrealtime until a deadline
//                          (the device-side equivalent of the reference's
//                          usleep: the GPU is idle, the stream is busy)
//   * busy_spin         - every CU runs dependent FMAs until a deadline
//   * gemm_tn           - C[M,N] (bf16) = A[M,K] · B[N,K]^T, MFMA 16x16x32
//                          bf16 or OCP-fp8 e4m3 operands, 256x256 tiles,
//                          global_load_lds staging into an XOR-swizzled LDS
//                          image, XCD-aware tile order.
// All launchers take the stream as void* (hipStream_t) so plain C++
// translation units can call them.
#pragma once

#include <cstddef>
#include <cstdint>

#include "dlnb/common.hpp"

namespace dlnb {
namespace kernels {

void fill_random(void* p, size_t count, DType t, uint64_t seed, void* stream);

// Deadline kernels; ticks of the 100 MHz s_memrealtime clock (see
// wallclock_hz()).
void idle_wait(uint64_t ticks, void* stream);
void busy_spin(uint64_t ticks, int blocks, void* stream);
double wallclock_hz(int device);
// One wave stores s_memrealtime into *slot (host-mapped memory) when the
// stream reaches this point.
void stamp(uint64_t* slot, void* stream);
int num_cus(int device);

// GEMM: requires M % 256 == 0, N % 256 == 0, K*elem_size % 128 == 0, leading
// dimensions in elements, 16-byte aligned rows. in_t is BF16 or FP8_E4M3;
// C is always bf16.
bool gemm_shape_ok(int M, int N, int K, DType in_t);
// waves selects the variant: 8 = 8 waves (2 per SIMD, 128x64 per wave)
// double buffered, 2 = the same with software-pipelined fragment reads
// (bf16), 1 = 8 waves with a 3-deep A ring (160 KiB LDS), 4 = 4 waves (1 per
// SIMD, 128x128 per wave), 6 = 8-phase with balanced fragment reads (bf16;
// even K-tile counts, else 3), 7 / 9 = 8-phase balanced / plain with one
// uniform K-tile body, 5 = one wave per SIMD with AGPR accumulators (below);
// 0 = the default: bf16 6, fp8 5 (K % 256 == 0) else 9, where they apply
// (>= 2 K-tiles), else 2 for bf16 / 8 for fp8 (ring if DLNB_GEMM_RING=1, 4
// waves if DLNB_GEMM_WAVES=4).
// 3 = the 8-phase ping-pong schedule (gemm_8phase.hip; needs >= 2 K-tiles).
void gemm_tn(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, DType in_t,
             void* stream, int waves = 0);
bool gemm_8phase_shape_ok(int M, int N, int K, DType in_t);
// 5 = one wave per SIMD, 128 x 128 of C per wave (gemm_4wave.hip; bf16, K % 64 == 0).
bool gemm_4wave_shape_ok(int M, int N, int K, DType in_t);
void gemm_tn_4wave(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                   void* stream);
//   fp8: gemm_4wave_fp8.hip (MX MFMA, K % 256 == 0).
bool gemm_4wave_fp8_shape_ok(int M, int N, int K, DType in_t);
void gemm_tn_4wave_fp8(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                       void* stream);
void gemm_tn_4wave_fp8_deadline(const void* A, const void* B, void* C, int M, int N, int K, uint64_t ticks,
                                uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end,
                                uint64_t* tstart);
void gemm_tn_8phase(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, DType in_t,
                    void* stream, bool balanced = false, bool uniform = false);
void gemm_tn_8phase_deadline(const void* A, const void* B, void* C, int M, int N, int K, DType in_t, uint64_t ticks,
                             uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end,
                             uint64_t* tstart);
// Whether the 8-phase schedule is used where it applies (default on;
// DLNB_GEMM_8PHASE=0 selects the older double-buffered kernel for A/B runs).
bool gemm_8phase_enabled();
int gemm_default_waves();

// Persistent deadline variant (the default stand-in compute): a grid of
// `grid` blocks (<= one per CU: 128 KiB LDS each) walks the M x N tile space
// of C = A.B^T round-robin and stops min(ticks, slice_end) (100 MHz
// s_memrealtime) after t0. t0 is agreed through *slot: the first block of the
// first launch of `epoch` (1..65535, different from the slot's previous task)
// CASes {epoch:16 | t0:48} into it; every other block and every later launch
// with the same epoch reads it. A long task is issued as several launches
// (slices) with increasing slice_end so that collectives on other streams get
// CUs at slice boundaries, as they do between a training step's kernels.
// Leading dimensions are K, K and N.
// tstart (optional, host-mapped): the block that claims the epoch stores the
// task's start (s_memrealtime) there - stall timing without extra kernels.
void gemm_tn_deadline(const void* A, const void* B, void* C, int M, int N, int K, DType in_t, uint64_t ticks,
                      uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end = 0,
                      uint64_t* tstart = nullptr);

// Elementwise "optimizer" stand-in (SGD-momentum on bf16 shards, fp32 math):
// p = p - lr * (m = beta*m + g). Used by the optional --optimizer step.
void sgd_momentum_bf16(void* param, void* mom, const void* grad, size_t n, float lr, float beta, void* stream);

}  // namespace kernels
}  // namespace dlnb
