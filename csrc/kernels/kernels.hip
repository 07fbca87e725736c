// CDNA4 / gfx950 kernels for the dlnb runtime. See dlnb/kernels.hpp for the
// inventory and docs/KERNELS.md for design notes and measured numbers.
#include <hip/hip_runtime.h>

#include <cstdio>
#include "dlnb/common.hpp"
#include <thread>
#include <mutex>
#include <cmath>
#include <vector>
#include <algorithm>
#include <atomic>
#include <chrono>

#include "deadline_sync.hpp"
#include "dlnb/kernels.hpp"

#define DLNB_HIP_CHECK(expr)                                                       \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) DLNB_THROW(#expr << " failed: " << hipGetErrorString(e_)); \
  } while (0)

namespace dlnb {
namespace kernels {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

inline hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

// ------------------------------------------------------------------ fill

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ float u01(uint64_t h, int part) {
  // 21-bit slices of one 64-bit hash -> uniform [-1, 1)
  uint32_t v = static_cast<uint32_t>((h >> (21 * part)) & 0x1fffff);
  return static_cast<float>(v) * (2.0f / 2097152.0f) - 1.0f;
}

__device__ __forceinline__ uint8_t f32_to_e4m3(float f) {
  // Saturating OCP e4m3fn conversion via the hardware packed convert.
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(f, f, 0, false);
  return static_cast<uint8_t>(r & 0xff);
}

__device__ __forceinline__ uint8_t f32_to_e5m2(float f) {
  int r = __builtin_amdgcn_cvt_pk_bf8_f32(f, f, 0, false);
  return static_cast<uint8_t>(r & 0xff);
}

// Each thread produces 8 elements per step (16 B for 2-byte types).
template <typename Tstore, int KIND>
__global__ void fill_kernel(Tstore* __restrict__ p, size_t n8, size_t n, uint64_t seed) {
  size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n8; i += stride) {
    uint64_t h0 = splitmix64(seed ^ (i * 2 + 0));
    uint64_t h1 = splitmix64(seed ^ (i * 2 + 1));
    float f[8];
#pragma unroll
    for (int j = 0; j < 3; ++j) f[j] = u01(h0, j);
#pragma unroll
    for (int j = 0; j < 3; ++j) f[3 + j] = u01(h1, j);
    f[6] = u01(h0 ^ h1, 0);
    f[7] = u01(h0 ^ h1, 1);
    size_t base = i * 8;
    if (KIND == 0) {  // bf16
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = static_cast<__bf16>(f[j]);
      if (base + 8 <= n) {
        *reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(p) + base) = v;
      } else {
        for (int j = 0; j < 8 && base + j < n; ++j) reinterpret_cast<__bf16*>(p)[base + j] = v[j];
      }
    } else if (KIND == 1) {  // fp16
      for (int j = 0; j < 8 && base + j < n; ++j) reinterpret_cast<_Float16*>(p)[base + j] = static_cast<_Float16>(f[j]);
    } else if (KIND == 2) {  // fp32
      for (int j = 0; j < 8 && base + j < n; ++j) reinterpret_cast<float*>(p)[base + j] = f[j];
    } else {  // fp8 (3 = e4m3, 4 = e5m2)
      uint8_t b[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = KIND == 3 ? f32_to_e4m3(f[j]) : f32_to_e5m2(f[j]);
      uint8_t* q = reinterpret_cast<uint8_t*>(p);
      if (base + 8 <= n) {
        uint64_t packed = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) packed |= static_cast<uint64_t>(b[j]) << (8 * j);
        *reinterpret_cast<uint64_t*>(q + base) = packed;
      } else {
        for (int j = 0; j < 8 && base + j < n; ++j) q[base + j] = b[j];
      }
    }
  }
}

// ------------------------------------------------------------- deadlines

__global__ void idle_wait_kernel(uint64_t ticks, uint64_t* start, uint64_t* start2) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (start) __hip_atomic_store(start, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (start2) __hip_atomic_store(start2, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void stamp_kernel(uint64_t* slot) {
  if (threadIdx.x == 0) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_store(slot, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void gate_signal_kernel(uint64_t* gate, const uint64_t* iter, uint32_t tag) {
  if (threadIdx.x == 0) {
    const uint64_t seq = dl::gate_seq(iter, tag);
    __hip_atomic_store(gate + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gate, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void gate_wait_kernel(const uint64_t* gate, const uint64_t* iter, uint32_t tag, uint64_t timeout_ticks,
                                 uint64_t* timeouts, const uint64_t* abort) {
  if (threadIdx.x == 0) {
    const uint64_t it = dl::iter_of(iter);
    const uint64_t want = dl::gate_seq_of(it, tag);
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    // relaxed polls, one acquire at the end: an acquire load invalidates the
    // cache on every poll (buffer_inv), under the compute running beside it.
    // >=: the sequence words only grow (a later replay's raise satisfies it);
    // a poisoned iteration (a replay the abort released) does not wait.
    if (!(iter && it == kPoisonIter)) {
      for (unsigned k = 1; __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want; ++k) {
        __builtin_amdgcn_s_sleep(2);
        if ((k & 63u) == 0 && dl::abort_up(abort)) break;
        if (__builtin_amdgcn_s_memrealtime() - w0 > timeout_ticks) {
          __hip_atomic_fetch_add(timeouts, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

__global__ void set_word_kernel(uint64_t* word, uint64_t value) {
  if (threadIdx.x == 0) __hip_atomic_store(word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// queue probe: a waits for b's store (system scope: the word is host memory)
__global__ void probe_wait_kernel(const uint64_t* word, uint64_t value, uint64_t timeout_ticks, uint64_t* timed_out) {
  if (threadIdx.x == 0) {
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != value) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - w0 > timeout_ticks) {
        __hip_atomic_store(timed_out, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
}

// A lane's last node: the iteration number into the host's done word - a
// relaxed system-scope store (a release would write the L2 back first: ~50 us
// after a collective's copy, measured in round 5) inside the lane's graph.
__global__ void lane_done_kernel(uint64_t* word, const uint64_t* iter) {
  if (threadIdx.x == 0)
    __hip_atomic_store(word, __hip_atomic_load(iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void host_signal_kernel(uint64_t* word, uint64_t value) {
  if (threadIdx.x == 0) __hip_atomic_store(word, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void host_wait_kernel(const uint64_t* word, uint64_t value, uint64_t timeout_ticks, uint64_t* timeouts,
                                 uint64_t* iter_out, uint64_t iter_value, uint64_t tight_ticks, const uint64_t* abort) {
  if (threadIdx.x == 0) {
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    bool aborted = false;
    // relaxed polls (an acquire load would invalidate the L2's system-scope
    // lines on every poll, for the whole iteration an armed replay waits);
    // after tight_ticks (0: never) one poll every ~4 us. The host's abort
    // word ends the wait too: what this held back then runs through on a
    // poisoned iteration word (no compute, no waits: dl::start_task).
    for (unsigned k = 1; __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < value; ++k) {
      const uint64_t el = __builtin_amdgcn_s_memrealtime() - w0;
      if (tight_ticks != 0 && el > tight_ticks)
        __builtin_amdgcn_s_sleep(127);
      else
        __builtin_amdgcn_s_sleep(2);
      if (((k & 63u) == 0 || (tight_ticks != 0 && el > tight_ticks)) && dl::abort_up(abort)) {
        aborted = true;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - w0 > timeout_ticks) {
        __hip_atomic_fetch_add(timeouts, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (iter_out)
      __hip_atomic_store(iter_out, aborted ? kPoisonIter : iter_value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void __launch_bounds__(256) busy_spin_kernel(uint64_t ticks, float* sink, uint64_t* start,
                                                        uint64_t* start2) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (start) __hip_atomic_store(start, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (start2) __hip_atomic_store(start2, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  float x = static_cast<float>(threadIdx.x) * 1e-3f, y = 0.999f;
  for (;;) {
#pragma unroll
    for (int i = 0; i < 64; ++i) x = __builtin_fmaf(x, y, 1e-3f);
    if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
  }
  if (x == -1.0f) sink[threadIdx.x] = x;  // never true; keeps the FMAs live
}

// ------------------------------------------------------------------ GEMM
//
// Tile 256 (M) x 256 (N) x 128 bytes of K per stage (64 bf16 / 128 fp8).
// 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns 128 x 64 of C as
// 8 x 4 MFMA 16x16 accumulators (128 f32 registers).
// LDS = 2 stages x {A, B} x 256 rows x 128 B = 128 KiB, one __shared__ array.
//
// Staging: global_load_lds_dwordx4 writes 1 KiB per wave-instruction
// lane-linearly (LDS = base + 16*lane), so the bank-conflict swizzle is put on
// the per-lane SOURCE address (cdna_hip_programming.md §5.4 rule 21): LDS slot
// q of row r holds 16-byte chunk c = q ^ ((r >> 1) & 7). A fragment read of
// chunk c of row r therefore looks at slot c ^ ((r >> 1) & 7); the 16 lanes of
// each ds_read_b128 lane group then hit 16 distinct 16-B slots of the 256-B
// bank row (conflict-free; checked by hand against the gfx950 lane groups).
//
// Operands are swapped in the MFMA (a <- B rows, b <- A rows) so each lane
// ends up with 4 consecutive N columns of one M row: one 8-byte store per
// accumulator instead of four 2-byte ones.

constexpr int kTile = 256;
constexpr int kRowBytes = 128;
constexpr int kTileBytes = kTile * kRowBytes;  // 32 KiB
constexpr int kStageBytes = 2 * kTileBytes;    // A + B

__device__ __forceinline__ int swz(int row, int chunk) { return row * kRowBytes + ((chunk ^ ((row >> 1) & 7)) << 4); }

// One 256 x 128-byte tile = 2048 16-B slots = 32 wave-instructions of
// global_load_lds_dwordx4, spread over the block's NW waves.
template <int NW>
__device__ __forceinline__ void stage_tile(const char* __restrict__ g, size_t ld_bytes, char* lds_tile, int w,
                                           int lane) {
#pragma unroll
  for (int i = 0; i < 32 / NW; ++i) {
    const int slot = (i * NW + w) * 64 + lane;
    const int r = slot >> 3;
    const int c = (slot & 7) ^ ((r >> 1) & 7);
    const char* src = g + static_cast<size_t>(r) * ld_bytes + (c << 4);
    __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(lds_tile + (i * NW + w) * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ int xcd_remap(int b, int T) {
  // Bijective: blocks that share an XCD (b % 8 equal) get a contiguous range
  // of logical tile ids (cdna_hip_programming.md §5 "XCD swizzle").
  const int q = T / 8, r = T % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// One 128-byte K-tile of MFMA work for a wave owning rows wm*128.. (8
// fragments) and columns wn*WTN.. (FN fragments) of the block tile.
template <bool FP8, bool DEADLINE, int FN, int WTN, bool SWP = false>
__device__ __forceinline__ void ktile_mfma(const char* __restrict__ At, const char* __restrict__ Bt, f32x4 (&acc)[8][FN],
                                           int wm, int wn, int r16, int h) {
  if constexpr (SWP && !FP8 && FN == 4) {
    // Software-pipelined: step 1's 12 fragment reads are interleaved with
    // step 0's 32 MFMAs (2 MFMAs, 1 ds_read, ...), so they are in flight
    // while the matrix cores work instead of after a lgkmcnt(0) drain.
    bf16x8 af[2][8], bfr[2][FN];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      af[0][i] = *reinterpret_cast<const bf16x8*>(At + swz(wm * 128 + i * 16 + r16, h));
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bfr[0][j] = *reinterpret_cast<const bf16x8*>(Bt + swz(wn * WTN + j * 16 + r16, h));
    __builtin_amdgcn_s_setprio(1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      af[1][i] = *reinterpret_cast<const bf16x8*>(At + swz(wm * 128 + i * 16 + r16, 4 + h));
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bfr[1][j] = *reinterpret_cast<const bf16x8*>(Bt + swz(wn * WTN + j * 16 + r16, 4 + h));
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[0][j], af[0][i], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[1][j], af[1][i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  } else if constexpr (!FP8) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[8], bfr[FN];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(At + swz(wm * 128 + i * 16 + r16, ks * 4 + h));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bt + swz(wn * WTN + j * 16 + r16, ks * 4 + h));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  } else if constexpr (DEADLINE) {
    // Deadline (persistent stand-in) variant: the non-scaled 16x16x32 fp8
    // MFMA; the MX path below needs ~48 more VGPRs than the deadline
    // bookkeeping leaves (it would spill), and a deadline kernel's rate
    // does not change how long it runs.
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      long af[8], bfr[FN];
      const int chunk = ks * 2 + (h >> 1), half = (h & 1) * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        af[i] = *reinterpret_cast<const long*>(At + swz(wm * 128 + i * 16 + r16, chunk) + half);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const long*>(Bt + swz(wn * WTN + j * 16 + r16, chunk) + half);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(bfr[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  } else {
    // fp8 e4m3 through the MX-scaled MFMA (16x16x128, unit E8M0 scales =
    // 127): one instruction covers the whole 128-byte K-tile at twice the
    // non-scaled fp8 rate. Lane group h holds K chunks h and h + 4 of its
    // row (not 2h, 2h+1: with the (row >> 1) swizzle those put rows r and
    // r + 4 of one ds_read_b128 lane group on the same banks, 2-way on
    // every read); A and B use the same K order, which is all the product
    // needs (checked exactly by tests/test_gpu_kernels.py).
    i32x8 bfr[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * WTN + j * 16 + r16;
      const int4 lo = *reinterpret_cast<const int4*>(Bt + swz(row, h));
      const int4 hi = *reinterpret_cast<const int4*>(Bt + swz(row, h + 4));
      bfr[j] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wm * 128 + i * 16 + r16;
      const int4 lo = *reinterpret_cast<const int4*>(At + swz(row, h));
      const int4 hi = *reinterpret_cast<const int4*>(At + swz(row, h + 4));
      const i32x8 af = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af, acc[i][j], 0, 0, 0, 127, 0, 127);
      __builtin_amdgcn_s_setprio(0);
    }
  }
}

// Epilogue: lane holds C[m = .. + (lane & 15)][n = .. + 4*(lane >> 4) + 0..3].
template <int FN, int WTN>
__device__ __forceinline__ void store_tile(__bf16* __restrict__ C, int ldc, int tm, int tn, int wm, int wn, int r16,
                                           int h, const f32x4 (&acc)[8][FN]) {
  const int m_base = tm * kTile + wm * 128 + r16;
  const int n_base = tn * kTile + wn * WTN + 4 * h;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bf16x4 o;
      o[0] = static_cast<__bf16>(acc[i][j][0]);
      o[1] = static_cast<__bf16>(acc[i][j][1]);
      o[2] = static_cast<__bf16>(acc[i][j][2]);
      o[3] = static_cast<__bf16>(acc[i][j][3]);
      *reinterpret_cast<bf16x4*>(C + static_cast<size_t>(m_base + i * 16) * ldc + n_base + j * 16) = o;
    }
  }
}

// DEADLINE = false: one launch computes every tile once (grid = tiles).
// DEADLINE = true : persistent stand-in compute. grid <= resident blocks;
//   each block walks the tile space round-robin (wrapping) and the whole
//   grid stops `min(ticks, slice_end)` of the 100 MHz s_memrealtime clock
//   after t0, the time the first block of the first launch of this epoch
//   started (agreed through an epoch-tagged CAS on *slot; later launches of
//   the same epoch reuse t0, so a task cut into slices keeps one absolute
//   deadline however late a slice starts). Thread 0
//   decides once per K-tile and publishes the decision through a
//   double-buffered LDS flag read after the K-tile's barrier, so every wave
//   leaves the K-loop at the same barrier.
// WN = waves along N (WM = 2 along M): WN = 4 -> 8 waves (2 per SIMD) of
// 128 x 64; WN = 2 -> 4 waves (1 per SIMD) of 128 x 128, twice the MFMAs per
// LDS fragment read and the 256 accumulators in AGPRs.
template <bool FP8, bool DEADLINE, int WN, bool SWP = false>
__global__ void __launch_bounds__(128 * WN, WN == 4 ? 2 : 1)
    gemm_tn_256_kernel(const char* __restrict__ A, const char* __restrict__ B, __bf16* __restrict__ C, int M, int N,
                       int K, int lda, int ldb, int ldc, uint64_t* __restrict__ slot, uint32_t epoch,
                       uint64_t ticks, uint64_t slice_end, DlSync sync) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kStageBytes + 16];
  volatile int* stop_flag = reinterpret_cast<volatile int*>(smem + 2 * kStageBytes);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NW = 2 * WN;          // waves per block
  constexpr int FN = kTile / WN / 16;  // 16-wide fragments along N per wave
  constexpr int WTN = kTile / WN;      // wave tile width (N)
  const int wm = w / WN, wn = w % WN;
  const int nt_m = M / kTile, nt_n = N / kTile, T = nt_m * nt_n;
  constexpr uint64_t kMask48 = dl::kMask48;
  uint64_t t0 = 0;
  if constexpr (DEADLINE) {
    if (tid == 0) t0 = dl::agree_t0(slot, epoch, ticks, sync);
  }
  for (int round = 0;; ++round) {
  const int b = xcd_remap(DEADLINE ? (blockIdx.x + round * gridDim.x) % T : blockIdx.x, T);
  // Grouped tile order: GROUP row-tiles share their B panels in L2.
  constexpr int GROUP = 8;
  const int per_group = GROUP * nt_n;
  const int first_m = (b / per_group) * GROUP;
  const int gsz = min(nt_m - first_m, GROUP);
  const int tm = first_m + (b % per_group) % gsz;
  const int tn = (b % per_group) / gsz;

  constexpr int esz = FP8 ? 1 : 2;
  const size_t lda_b = static_cast<size_t>(lda) * esz, ldb_b = static_cast<size_t>(ldb) * esz;
  const char* Ab = A + static_cast<size_t>(tm) * kTile * lda_b;
  const char* Bb = B + static_cast<size_t>(tn) * kTile * ldb_b;
  const int nk = (K * esz) / kRowBytes;

  f32x4 acc[8][FN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage_tile<NW>(Ab, lda_b, smem, w, lane);
  stage_tile<NW>(Bb, ldb_b, smem + kTileBytes, w, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int expired = 0;

  const int r16 = lane & 15, h = lane >> 4;
  for (int kt = 0; kt < nk && !expired; ++kt) {
    const char* cur = smem + (kt & 1) * kStageBytes;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * kStageBytes;
      stage_tile<NW>(Ab + static_cast<size_t>(kt + 1) * kRowBytes, lda_b, nxt, w, lane);
      stage_tile<NW>(Bb + static_cast<size_t>(kt + 1) * kRowBytes, ldb_b, nxt + kTileBytes, w, lane);
    }
    const char* At = cur;
    const char* Bt = cur + kTileBytes;
    ktile_mfma<FP8, DEADLINE, FN, WTN, SWP>(At, Bt, acc, wm, wn, r16, h);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (DEADLINE) {
      // Double-buffered flag: written before barrier kt, read after it; the
      // other slot is rewritten only after every wave passed barrier kt+1.
      if (tid == 0) {
        const uint64_t el = (__builtin_amdgcn_s_memrealtime() - t0) & kMask48;
        stop_flag[kt & 1] = el >= ticks || el >= slice_end;
      }
      __syncthreads();
      expired = __builtin_amdgcn_readfirstlane(stop_flag[kt & 1]);
    } else {
      __syncthreads();
    }
  }
  if (expired) {  // partial tile: the stand-in result is not needed
    if constexpr (DEADLINE) dl::task_done(sync);
    return;
  }

  store_tile<FN, WTN>(C, ldc, tm, tn, wm, wn, r16, h, acc);
  if constexpr (!DEADLINE) return;
  }  // round
}


// ------------------------------------------------------------- optimizer

__global__ void sgd_momentum_kernel(__bf16* __restrict__ p, __bf16* __restrict__ m, const __bf16* __restrict__ g,
                                    size_t n, float lr, float beta, uint64_t* end_stamp, uint32_t* done) {
  size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x * 8;
  for (size_t i = (blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x) * 8; i < n; i += stride) {
    if (i + 8 <= n) {
      bf16x8 pv = *reinterpret_cast<bf16x8*>(p + i);
      bf16x8 mv = *reinterpret_cast<bf16x8*>(m + i);
      bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float mm = beta * static_cast<float>(mv[j]) + static_cast<float>(gv[j]);
        mv[j] = static_cast<__bf16>(mm);
        pv[j] = static_cast<__bf16>(static_cast<float>(pv[j]) - lr * mm);
      }
      *reinterpret_cast<bf16x8*>(p + i) = pv;
      *reinterpret_cast<bf16x8*>(m + i) = mv;
    } else {
      for (size_t k = i; k < n; ++k) {
        float mm = beta * static_cast<float>(m[k]) + static_cast<float>(g[k]);
        m[k] = static_cast<__bf16>(mm);
        p[k] = static_cast<__bf16>(static_cast<float>(p[k]) - lr * mm);
      }
    }
  }
  if (end_stamp) {
    // the kernel's end on the device clock: the last block to finish stores it
    // (and re-arms the counter for the next launch)
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
        __hip_atomic_store(end_stamp, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

int grid_for(size_t work_items, int block) {
  size_t g = (work_items + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

}  // namespace

void fill_random(void* p, size_t count, DType t, uint64_t seed, void* stream) {
  if (count == 0) return;
  size_t n8 = (count + 7) / 8;
  int grid = grid_for(n8, 256);
  seed = seed * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull;
  switch (t) {
    case DType::BF16: hipLaunchKernelGGL((fill_kernel<uint16_t, 0>), grid, 256, 0, S(stream), static_cast<uint16_t*>(p), n8, count, seed); break;
    case DType::FP16: hipLaunchKernelGGL((fill_kernel<uint16_t, 1>), grid, 256, 0, S(stream), static_cast<uint16_t*>(p), n8, count, seed); break;
    case DType::FP32: hipLaunchKernelGGL((fill_kernel<float, 2>), grid, 256, 0, S(stream), static_cast<float*>(p), n8, count, seed); break;
    case DType::FP8_E4M3: hipLaunchKernelGGL((fill_kernel<uint8_t, 3>), grid, 256, 0, S(stream), static_cast<uint8_t*>(p), n8, count, seed); break;
    case DType::FP8_E5M2: hipLaunchKernelGGL((fill_kernel<uint8_t, 4>), grid, 256, 0, S(stream), static_cast<uint8_t*>(p), n8, count, seed); break;
  }
  DLNB_HIP_CHECK(hipGetLastError());
}

void idle_wait(uint64_t ticks, void* stream, uint64_t* start, uint64_t* start2) {
  hipLaunchKernelGGL(idle_wait_kernel, 1, 64, 0, S(stream), ticks, start, start2);
  DLNB_HIP_CHECK(hipGetLastError());
}

namespace {
std::atomic<long> g_gate_signals{0};
std::atomic<long> g_gate_fault{-1};
}  // namespace

void fail_gate_signal(long index) { g_gate_fault.store(index); }

void gate_signal(uint64_t* gate, const uint64_t* iter, uint32_t tag, void* stream) {
  DLNB_REQUIRE(gate != nullptr && tag > 0 && reinterpret_cast<uintptr_t>(gate) % 16 == 0, "gate_signal: bad gate/tag");
  const long k = g_gate_signals.fetch_add(1);
  const long f = g_gate_fault.load();
  if (f >= 0 && k == f) {  // fault injection: this gate is never raised
    std::fprintf(stderr, "[dlnb] fault injection: gate signal %ld of this process is not raised\n", k);
    std::fflush(stderr);
    return;
  }
  hipLaunchKernelGGL(gate_signal_kernel, 1, 64, 0, S(stream), gate, iter, tag);
  DLNB_HIP_CHECK(hipGetLastError());
}

void gate_wait(const uint64_t* gate, const uint64_t* iter, uint32_t tag, uint64_t timeout_ticks, uint64_t* timeouts,
               void* stream, const uint64_t* abort) {
  DLNB_REQUIRE(gate != nullptr && timeouts != nullptr && tag > 0 && reinterpret_cast<uintptr_t>(gate) % 16 == 0,
               "gate_wait: bad gate/tag");
  hipLaunchKernelGGL(gate_wait_kernel, 1, 64, 0, S(stream), gate, iter, tag, timeout_ticks, timeouts, abort);
  DLNB_HIP_CHECK(hipGetLastError());
}

void set_word(uint64_t* word, uint64_t value, void* stream) {
  DLNB_REQUIRE(word != nullptr, "set_word: null word");
  hipLaunchKernelGGL(set_word_kernel, 1, 64, 0, S(stream), word, value);
  DLNB_HIP_CHECK(hipGetLastError());
}

bool queues_independent(void* a, void* b, uint64_t timeout_ticks) {
  void* p = nullptr;
  DLNB_HIP_CHECK(hipHostMalloc(&p, 2 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
  uint64_t* w = static_cast<uint64_t*>(p);
  w[0] = 0;
  w[1] = 0;
  hipLaunchKernelGGL(probe_wait_kernel, 1, 64, 0, S(a), w, 1ull, timeout_ticks, w + 1);
  hipLaunchKernelGGL(host_signal_kernel, 1, 64, 0, S(b), w, 1ull);
  hipError_t e = hipGetLastError();
  const hipError_t ea = hipStreamSynchronize(S(a)), eb = hipStreamSynchronize(S(b));
  const bool ok = __atomic_load_n(w + 1, __ATOMIC_ACQUIRE) == 0;
  (void)hipHostFree(p);
  DLNB_HIP_CHECK(e);
  DLNB_HIP_CHECK(ea);
  DLNB_HIP_CHECK(eb);
  return ok;
}

void lane_done(uint64_t* word, const uint64_t* iter, void* stream) {
  DLNB_REQUIRE(word != nullptr && iter != nullptr, "lane_done: null word");
  hipLaunchKernelGGL(lane_done_kernel, 1, 64, 0, S(stream), word, iter);
  DLNB_HIP_CHECK(hipGetLastError());
}

void host_signal(uint64_t* word, uint64_t value, void* stream) {
  DLNB_REQUIRE(word != nullptr, "host_signal: null word");
  hipLaunchKernelGGL(host_signal_kernel, 1, 64, 0, S(stream), word, value);
  DLNB_HIP_CHECK(hipGetLastError());
}

void host_wait(const uint64_t* word, uint64_t value, uint64_t timeout_ticks, uint64_t* timeouts, void* stream,
               uint64_t* iter_out, uint64_t iter_value, const uint64_t* abort) {
  DLNB_REQUIRE(word != nullptr && timeouts != nullptr, "host_wait: null word");
  // Tight polling for DLNB_HOST_WAIT_TIGHT_US (50), then one poll every ~4 us:
  // an armed replay waits a whole iteration, and its wave's back-to-back
  // host-memory reads slowed the iteration's HBM-bound copies (one-rank
  // hybrid_3d: the 7-ms DP all-reduce copy 7.15-7.30 -> 6.89-6.93 ms, step
  // -0.5 ms; headline 0.05x -0.025 ms; profiles/hostwait_r5.md). 0: tight.
  static const long tight_us = env_int("DLNB_HOST_WAIT_TIGHT_US", 50);
  const uint64_t tight = tight_us > 0 ? static_cast<uint64_t>(tight_us) * 100ull : 0ull;  // 100 MHz ticks
  hipLaunchKernelGGL(host_wait_kernel, 1, 64, 0, S(stream), word, value, timeout_ticks, timeouts, iter_out, iter_value,
                     tight, abort);
  DLNB_HIP_CHECK(hipGetLastError());
}

void stamp(uint64_t* slot, void* stream) {
  hipLaunchKernelGGL(stamp_kernel, 1, 64, 0, S(stream), slot);
  DLNB_HIP_CHECK(hipGetLastError());
}

void busy_spin(uint64_t ticks, int blocks, void* stream, uint64_t* start, uint64_t* start2) {
  hipLaunchKernelGGL(busy_spin_kernel, blocks, 256, 0, S(stream), ticks, static_cast<float*>(nullptr), start, start2);
  DLNB_HIP_CHECK(hipGetLastError());
}

double wallclock_hz_nominal(int device) {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) khz = 100000;
  return static_cast<double>(khz) * 1e3;
}

// One wave answers the host's clock requests (read_clock): for k = 1..n it
// waits for the host's request word (slot[0]) to reach k, reads
// s_memrealtime, and replies with the tick (slot[1]) and then k (slot[2]).
// One request in flight at a time: a wave that streamed its clock into host
// memory as fast as it could (round 5's first version) queued its stores up
// to ~540 us behind (profiles/clock_r5.md). Every wait is bounded (1 s
// without a request ends the kernel), so the grid drains if the host stops.
__global__ void clock_pingpong_kernel(uint64_t* slot, int n, uint64_t idle_ticks) {
  if (threadIdx.x == 0) {
    for (int k = 1; k <= n; ++k) {
      const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
      bool live = true;
      while (__hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < static_cast<uint64_t>(k)) {
        if (__builtin_amdgcn_s_memrealtime() - w0 > idle_ticks) {
          live = false;
          break;
        }
      }
      if (!live) break;
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      __hip_atomic_store(slot + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(slot + 2, static_cast<uint64_t>(k), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

namespace {
// The s_memrealtime clock's rate against the host's steady clock, measured
// once per process and device from two readings >= DLNB_CLOCK_CAL_MS (500)
// apart. A reading (read_clock) is 2048 request / reply round trips with a
// one-wave kernel (clock_pingpong_kernel, ~6 ms): the device's tick lies
// between the host's clock before the request and after the reply, and the
// offset is read at the midpoints of the tightest round trips (what the
// midpoint misses by - unequal request and reply latencies - is the same at
// both readings and drops out of the rate); its uncertainty is the spread of
// those midpoints. (Round 5's first version streamed the clock into host
// memory instead: the stores queued up to ~540 us behind, and the rate's
// uncertainty came out at ~140 ppm - profiles/clock_r5.md.)
// Round 4 paired one stamp with the tightest of 16 launch + synchronize
// brackets (~5.5 us half-width): up to +-20 ppm over 500 ms, the
// size of the headline deltas; this is ~0.1 ppm (wallclock_uncertainty_ppm).
// The MI355X's 100 MHz reference ran 7.6 ppm slow on the box measured
// (profiles/host_boundary_r4.md): a deadline task timed in nominal ticks then
// lasted 21 us longer than the table time per headline iteration; with the
// measured rate the tasks last the table time in host (wall-clock) time.
struct ClockCal {
  std::mutex mu;
  bool begun = false, done = false;
  double hz = 0.0, host_us = 0.0, err_us = 0.0;
  double uncertainty_ppm = -1.0;  // < 0: nominal rate (not measured)
  uint64_t tick = 0;
};
ClockCal& clock_cal(int device) {
  static ClockCal c[64];
  return c[device & 63];
}
double steady_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// Returns false when too few requests were answered (then nothing is read).
bool read_clock(int device, double* host_us, uint64_t* tick, double* err_us) {
  int prev = 0;
  DLNB_HIP_CHECK(hipGetDevice(&prev));
  DLNB_HIP_CHECK(hipSetDevice(device));
  hipStream_t s{};
  DLNB_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void* p = nullptr;
  DLNB_HIP_CHECK(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent));
  uint64_t* slot = static_cast<uint64_t*>(p);
  slot[0] = slot[1] = slot[2] = 0;
  const double nominal = wallclock_hz_nominal(device);
  const int n = 2048;
  hipLaunchKernelGGL(clock_pingpong_kernel, 1, 64, 0, s, slot, n, static_cast<uint64_t>(1.0 * nominal));
  const hipError_t le = hipGetLastError();
  // (h0, h1, tick): the host's clock before its request and after the reply
  struct Rt {
    double h0, h1;
    uint64_t t;
  };
  std::vector<Rt> rs;
  rs.reserve(n);
  const double start = steady_us();
  for (int k = 1; k <= n; ++k) {
    const double h0 = steady_us();
    __atomic_store_n(slot, static_cast<uint64_t>(k), __ATOMIC_RELEASE);
    bool got = true;
    while (__atomic_load_n(slot + 2, __ATOMIC_ACQUIRE) < static_cast<uint64_t>(k)) {
      if (steady_us() - start > 2e6) {
        got = false;
        break;
      }
    }
    if (!got) break;
    const double h1 = steady_us();
    rs.push_back({h0, h1, __atomic_load_n(slot + 1, __ATOMIC_ACQUIRE)});
  }
  __atomic_store_n(slot, static_cast<uint64_t>(n), __ATOMIC_RELEASE);  // ends the kernel's loop either way
  const hipError_t se = hipStreamSynchronize(s);
  (void)hipHostFree(p);
  (void)hipStreamDestroy(s);
  DLNB_HIP_CHECK(hipSetDevice(prev));
  DLNB_HIP_CHECK(le);
  DLNB_HIP_CHECK(se);
  if (rs.size() < 64) return false;
  // The device read its clock between h0 and h1: the pair's midpoint is the
  // host time of tick t to within half its round trip, and the offset
  // (midpoint minus the device time at the nominal rate: 10 ms x 10 ppm is
  // 0.1 us) is read from the tightest round trips (a preempted host only
  // widens one); its uncertainty is the spread of those offsets. What the
  // midpoint misses by (the request's and the reply's unequal latencies) is
  // the same at both readings and drops out of the rate.
  const double b = nominal * 1e-6;  // ticks per us
  const uint64_t tref = rs[rs.size() / 2].t;
  std::vector<size_t> idx(rs.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return rs[x].h1 - rs[x].h0 < rs[y].h1 - rs[y].h0; });
  const size_t m = std::max<size_t>(16, rs.size() / 20);
  std::vector<double> off(m);
  for (size_t j = 0; j < m; ++j) {
    const Rt& r = rs[idx[j]];
    off[j] = 0.5 * (r.h0 + r.h1) - static_cast<double>(static_cast<int64_t>(r.t - tref)) / b;
  }
  std::sort(off.begin(), off.end());
  const double med = off[m / 2];
  // the offsets' spread over the tightest 5 %, as a standard error of their median
  const double iqr = off[3 * m / 4] - off[m / 4];
  *host_us = med;
  *tick = tref;
  *err_us = std::max(iqr / std::sqrt(static_cast<double>(m)), 0.002);
  if (env_int("DLNB_CLOCK_DEBUG", 0) != 0) {
    std::vector<double> rtt(rs.size());
    for (size_t i = 0; i < rs.size(); ++i) rtt[i] = rs[i].h1 - rs[i].h0;
    std::sort(rtt.begin(), rtt.end());
    std::fprintf(stderr,
                 "[dlnb] clock reading: %zu round trips over %.1f us, rtt (us) min %.3f p5 %.3f p50 %.3f max %.3f; "
                 "best %zu offsets (us from median) min %.3f p25 %.3f p75 %.3f max %.3f; err %.4f us\n",
                 rs.size(), rs.back().h1 - rs.front().h0, rtt[0], rtt[rtt.size() / 20], rtt[rtt.size() / 2],
                 rtt.back(), m, off[0] - med, off[m / 4] - med, off[3 * m / 4] - med, off[m - 1] - med, *err_us);
  }
  return true;
}
void clock_cal_begin_locked(int device, ClockCal& c) {
  c.begun = true;
  if (env_int("DLNB_CLOCK_CAL_MS", 500) <= 0 || !read_clock(device, &c.host_us, &c.tick, &c.err_us)) {
    c.hz = wallclock_hz_nominal(device);
    c.done = true;
  }
}
}  // namespace

void clock_cal_begin(int device) {
  ClockCal& c = clock_cal(device);
  std::lock_guard<std::mutex> g(c.mu);
  if (!c.begun) clock_cal_begin_locked(device, c);
}

double wallclock_hz(int device) {
  ClockCal& c = clock_cal(device);
  std::lock_guard<std::mutex> g(c.mu);
  if (c.done) return c.hz;
  if (!c.begun) clock_cal_begin_locked(device, c);
  if (c.done) return c.hz;
  const double window_us = static_cast<double>(env_int("DLNB_CLOCK_CAL_MS", 500)) * 1e3;
  const double waited = steady_us() - c.host_us;
  if (waited < window_us) std::this_thread::sleep_for(std::chrono::duration<double, std::micro>(window_us - waited));
  double h = 0.0, err = 0.0;
  uint64_t t = 0;
  const bool ok = read_clock(device, &h, &t, &err);
  const double nominal = wallclock_hz_nominal(device);
  const double hz = ok ? static_cast<double>(t - c.tick) / ((h - c.host_us) * 1e-6) : 0.0;
  const double unc = ok ? (c.err_us + err) / (h - c.host_us) * 1e6 : 1e9;
  // the rate only with a sane value and an uncertainty well under the ppm
  // the deadline compute cares about (a preempted host, a wrong clock)
  if (ok && t > c.tick && h > c.host_us && std::fabs(hz / nominal - 1.0) < 200e-6 && unc < 2.0) {
    c.hz = hz;
    c.uncertainty_ppm = unc;
  } else {
    std::fprintf(stderr,
                 "[dlnb] warning: device %d clock measured at %.1f Hz (+-%.2f ppm) vs %.0f nominal; using nominal\n",
                 device, hz, unc, nominal);
    c.hz = nominal;
  }
  c.done = true;
  return c.hz;
}

double wallclock_uncertainty_ppm(int device) {
  ClockCal& c = clock_cal(device);
  std::lock_guard<std::mutex> g(c.mu);
  return c.done ? c.uncertainty_ppm : -1.0;
}

int num_cus(int device) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n <= 0) n = 256;
  return n;
}

bool gemm_shape_ok(int M, int N, int K, DType in_t) {
  if (in_t != DType::BF16 && in_t != DType::FP8_E4M3) return false;
  size_t esz = dtype_size(in_t);
  return M > 0 && N > 0 && K > 0 && M % kTile == 0 && N % kTile == 0 && (static_cast<size_t>(K) * esz) % kRowBytes == 0;
}

namespace {

template <bool FP8, bool DEADLINE, int WN, bool SWP = false>
void launch_gemm(int grid, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                 uint64_t* slot, uint32_t epoch, uint64_t ticks, uint64_t slice_end, hipStream_t st,
                 const DlSync& sync = DlSync()) {
  hipLaunchKernelGGL((gemm_tn_256_kernel<FP8, DEADLINE, WN, SWP>), grid, 128 * WN, 0, st, static_cast<const char*>(A),
                     static_cast<const char*>(B), static_cast<__bf16*>(C), M, N, K, lda, ldb, ldc, slot, epoch, ticks,
                     slice_end, sync);
}

// The 8-wave double-buffered kernel (variant 8): bf16 with software-pipelined
// fragment reads, fp8 with the plain MX body. The fallback for shapes the
// 8-phase / 4-wave kernels do not take (a single K-tile).
template <bool DEADLINE>
void dispatch_gemm(DType in_t, int grid, const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                   int ldc, uint64_t* slot, uint32_t epoch, uint64_t ticks, uint64_t slice_end, hipStream_t st,
                   const DlSync& sync = DlSync()) {
  const bool fp8 = in_t == DType::FP8_E4M3;
  if (!DEADLINE && !fp8)
    launch_gemm<false, false, 4, true>(grid, A, B, C, M, N, K, lda, ldb, ldc, slot, epoch, ticks, slice_end, st);
  else if (fp8)
    launch_gemm<true, DEADLINE, 4>(grid, A, B, C, M, N, K, lda, ldb, ldc, slot, epoch, ticks, slice_end, st, sync);
  else
    launch_gemm<false, DEADLINE, 4>(grid, A, B, C, M, N, K, lda, ldb, ldc, slot, epoch, ticks, slice_end, st, sync);
  DLNB_HIP_CHECK(hipGetLastError());
}

}  // namespace

void gemm_tn(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, DType in_t,
             void* stream, int variant) {
  DLNB_REQUIRE(gemm_shape_ok(M, N, K, in_t), "gemm_tn: unsupported shape M=" << M << " N=" << N << " K=" << K << " dtype="
                                                                              << dtype_name(in_t));
  size_t esz = dtype_size(in_t);
  DLNB_REQUIRE(lda >= K && ldb >= K && ldc >= N, "gemm_tn: leading dimensions too small");
  DLNB_REQUIRE((static_cast<size_t>(lda) * esz) % 16 == 0 && (static_cast<size_t>(ldb) * esz) % 16 == 0 && ldc % 4 == 0,
               "gemm_tn: rows must be 16-byte aligned");
  DLNB_REQUIRE(reinterpret_cast<uintptr_t>(A) % 16 == 0 && reinterpret_cast<uintptr_t>(B) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(C) % 8 == 0,
               "gemm_tn: misaligned base pointers");
  DLNB_REQUIRE(variant == 0 || variant == 5 || variant == 6 || variant == 8,
               "gemm_tn: variant must be 0 (default), 5 (4-wave MX, fp8), 6 (8-phase) or 8 (8-wave)");
  const int tiles = (M / kTile) * (N / kTile);
  // 0: fp8 the one-wave-per-SIMD MX kernel where it applies (+5-7 % over the
  // 8-phase one), else the 8-phase kernel where it applies, else 8 waves
  // bf16 where 256 x 32 nf tiles save rounds of tile work (fewer square tiles
  // than CUs, or a partial last round; fp8: inside variant 5)
  if (variant == 0 && in_t == DType::BF16 && gemm_tn_narrow(A, B, C, M, N, K, lda, ldb, ldc, in_t, stream)) return;
  if (variant == 0)
    variant = gemm_4wave_fp8_shape_ok(M, N, K, in_t) ? 5 : gemm_8phase_shape_ok(M, N, K, in_t) ? 6 : 8;
  if (variant == 5 && gemm_4wave_fp8_shape_ok(M, N, K, in_t)) {
    gemm_tn_4wave_fp8(A, B, C, M, N, K, lda, ldb, ldc, stream);
    return;
  }
  if (variant == 5 && in_t == DType::BF16 && gemm_4wave_shape_ok(M, N, K, in_t)) {
    gemm_tn_4wave_bf16(A, B, C, M, N, K, lda, ldb, ldc, stream);
    return;
  }
  if ((variant == 5 || variant == 6) && gemm_8phase_shape_ok(M, N, K, in_t)) {
    gemm_tn_8phase(A, B, C, M, N, K, lda, ldb, ldc, in_t, stream);
    return;
  }
  dispatch_gemm<false>(in_t, tiles, A, B, C, M, N, K, lda, ldb, ldc, nullptr, 0u, 0ull, 0ull, S(stream));
}

void gemm_tn_deadline(const void* A, const void* B, void* C, int M, int N, int K, DType in_t, uint64_t ticks,
                      uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end, const DlSync& sync) {
  if (slice_end == 0) slice_end = ticks;
  DLNB_REQUIRE(gemm_shape_ok(M, N, K, in_t), "gemm_tn_deadline: unsupported shape");
  DLNB_REQUIRE(slot != nullptr && grid > 0 && epoch > 0 && epoch < 65536, "gemm_tn_deadline: bad slot/grid/epoch");
  // fp8: the one-wave-per-SIMD MX kernel where it applies (2665 vs ~2180 TF/s sustained)
  if (gemm_4wave_fp8_shape_ok(M, N, K, in_t)) {
    gemm_tn_4wave_fp8_deadline(A, B, C, M, N, K, ticks, slot, epoch, grid, stream, slice_end, sync);
    return;
  }
  // bf16: DLNB_DEADLINE_BF16=4wave picks the one-wave-per-SIMD kernel (A/B;
  // read at every launch so one process can compare both)
  const bool bf16_4wave = in_t == DType::BF16 && env_or("DLNB_DEADLINE_BF16", "8phase") == "4wave";
  if (in_t == DType::BF16 && bf16_4wave && gemm_4wave_shape_ok(M, N, K, in_t)) {
    gemm_tn_4wave_deadline(A, B, C, M, N, K, in_t, ticks, slot, epoch, grid, stream, slice_end, sync);
    return;
  }
  if (gemm_8phase_shape_ok(M, N, K, in_t)) {
    gemm_tn_8phase_deadline(A, B, C, M, N, K, in_t, ticks, slot, epoch, grid, stream, slice_end, sync);
    return;
  }
  // 8 waves (a single K-tile)
  dispatch_gemm<true>(in_t, grid, A, B, C, M, N, K, K, K, N, slot, epoch, ticks, slice_end, S(stream), sync);
}

// (gemm_8phase.hip, gemm_4wave_fp8.hip)
bool deadline_program_8phase_ok(int M, int N, int K, DType in_t);
void gemm_8phase_deadline_program(const void* A, const void* B, void* C, int M, int N, int K, DType in_t,
                                  const DlTask* tasks, int n, uint64_t* slot, int grid, void* stream, uint32_t epoch);
void gemm_4wave_deadline_program(const void* A, const void* B, void* C, int M, int N, int K, DType in_t,
                                 const DlTask* tasks, int n, uint64_t* slot, int grid, void* stream, uint32_t epoch);

// The same kernel choice as gemm_tn_deadline, for the kernels with a program mode.
namespace {
int program_kernel(int M, int N, int K, DType in_t) {
  if (!gemm_shape_ok(M, N, K, in_t)) return 0;
  if (gemm_4wave_fp8_shape_ok(M, N, K, in_t)) return 4;
  if (in_t == DType::BF16 && env_or("DLNB_DEADLINE_BF16", "8phase") == "4wave" && gemm_4wave_shape_ok(M, N, K, in_t))
    return 4;
  if (gemm_8phase_shape_ok(M, N, K, in_t)) return deadline_program_8phase_ok(M, N, K, in_t) ? 8 : 0;
  return 0;
}
}  // namespace

bool deadline_program_ok(int M, int N, int K, DType in_t) { return program_kernel(M, N, K, in_t) != 0; }

int program_ktiles(int M, int N, int K, DType in_t) {
  if (program_kernel(M, N, K, in_t) == 0) return 0;
  return static_cast<int>(static_cast<size_t>(K) * dtype_size(in_t) / kRowBytes);
}

// The tail tile's K-tile count keeps the kernel's K-tile pairing: the 4-wave
// and the balanced 8-phase bodies run K-tiles in pairs; 2 for all of them.
int program_tail_multiple(int M, int N, int K, DType in_t) { return program_kernel(M, N, K, in_t) != 0 ? 2 : 0; }

void gemm_tn_deadline_program(const void* A, const void* B, void* C, int M, int N, int K, DType in_t,
                              const DlTask* tasks, int n, uint64_t* slot, int grid, void* stream, uint32_t epoch) {
  const int k = program_kernel(M, N, K, in_t);
  DLNB_REQUIRE(k != 0, "gemm_tn_deadline_program: no program-mode kernel for M=" << M << " N=" << N << " K=" << K);
  DLNB_REQUIRE(epoch == 0 || (n == 1 && epoch < 65536), "gemm_tn_deadline_program: a launch epoch needs one task");
  // every block must be resident at once (one 128-KiB-LDS block per CU): a
  // fixed-work task waits for all of them
  int dev = 0;
  DLNB_HIP_CHECK(hipGetDevice(&dev));
  DLNB_REQUIRE(grid > 0 && grid <= num_cus(dev), "gemm_tn_deadline_program: grid " << grid << " exceeds the CUs");
  if (k == 4)
    gemm_4wave_deadline_program(A, B, C, M, N, K, in_t, tasks, n, slot, grid, stream, epoch);
  else
    gemm_8phase_deadline_program(A, B, C, M, N, K, in_t, tasks, n, slot, grid, stream, epoch);
}

void sgd_momentum_bf16(void* param, void* mom, const void* grad, size_t n, float lr, float beta, void* stream,
                       uint64_t* end_stamp, uint32_t* done) {
  if (n == 0) return;
  DLNB_REQUIRE(!end_stamp || done, "sgd_momentum_bf16: an end stamp needs its completion counter");
  int grid = grid_for((n + 7) / 8, 256);
  hipLaunchKernelGGL(sgd_momentum_kernel, grid, 256, 0, S(stream), static_cast<__bf16*>(param),
                     static_cast<__bf16*>(mom), static_cast<const __bf16*>(grad), n, lr, beta, end_stamp, done);
  DLNB_HIP_CHECK(hipGetLastError());
}

}  // namespace kernels
}  // namespace dlnb
