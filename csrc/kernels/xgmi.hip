// Kernels of the "xgmi" backend (see dlnb/xgmi.hpp for the protocol).
//
// Data path: 16-B vector loads/stores, 512 threads per block, every block
// owns one contiguous slice of the per-rank message (the same slice on all
// ranks). Pushes go to the peers' uncached windows over xGMI; peers' targets
// are visited in rank-staggered order so the 7 links of an MI355X carry
// traffic at the same time. Reductions accumulate in fp32 and round once.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dlnb/xgmi.hpp"

#define DLNB_HIP_CHECK(expr)                                                       \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) DLNB_THROW(#expr << " failed: " << hipGetErrorString(e_)); \
  } while (0)

namespace dlnb {
namespace xgmi {

namespace {

constexpr int T = kThreads;

// Every kernel that waits on peers is capped at 64 registers per lane: 8 of
// its waves then fit a SIMD, i.e. kBlocksPerCU blocks of 512 threads per CU,
// which is what the CU budget of a comm lane is computed from
// (comm_xgmi.cpp). Uncapped, the fp8 reductions took 70-72 VGPRs (7 waves /
// SIMD = 3 blocks per CU), so a lane of 4 * max_ctas blocks needed a third
// more CUs than budgeted - blocks of one lane could then queue behind a
// spinning kernel of another (tests/test_tools.py checks the code object).
#define DLNB_XGMI_KERNEL __global__ void __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(8)))

// Flags are raised with a system-scope atomic RMW, not a store: L2 is per
// XCD and not coherent across XCDs, and a plain store made through a peer's
// IPC mapping can sit in the writer's L2 - the waiter, polling its flag
// word, then spins until that line happens to be evicted (seen as
// intermittent multi-second stalls with two ranks on one GPU). Atomics
// execute at the memory side. Epochs only grow, so max == store. The RMW
// itself is relaxed: release_window() orders the data before it.
__device__ __forceinline__ void sys_store(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Polled with an idempotent atomic RMW for the same reason: a plain
// system-scope load can keep hitting a stale line in the poller's own XCD L2.
// (A compare-and-swap that never matches: LLVM folds an idempotent add/or
// into a plain load.) Relaxed: an acquire here would invalidate the whole
// L2 on every poll; acquire_window() runs once after the wait instead.
__device__ __forceinline__ uint32_t sys_load(uint32_t* p) {
  uint32_t v = 0xffffffffu;
  __hip_atomic_compare_exchange_strong(p, &v, 0xffffffffu, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
  return v;
}

// Make this wave's window stores visible to the peers before a flag is
// raised. Uncached windows (the default) never hold data in any cache, so
// completing the stores (vmcnt 0) is all it takes; a system-scope release
// fence would also write back the whole L2 of the XCD (buffer_wbl2) and,
// as __threadfence_system() is acquire-release, invalidate it - once per
// block and piece, costly for every kernel sharing the XCD. This holds for a
// peer on another GPU too: gfx950's system-scope release is exactly that
// L2 write-back followed by vmcnt(0), and the write-back has nothing to do
// for MTYPE-UC lines - a store's vmcnt slot is returned only once the write
// is acknowledged by the memory it targets (local HBM or, through xGMI, the
// peer's). Cached windows (DLNB_XGMI_MEM=fine|coarse) keep the full fence,
// and so does DLNB_XGMI_RELEASE=system on uncached windows: the escape hatch
// if a platform ever acknowledges a remote store earlier (the bench's
// multi-GPU exactness pass runs vmcnt first and system if that fails).
__device__ __forceinline__ void release_window(const Peers& P) {
  if (P.uncached && !P.release_system)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}
// After the peers' flags were seen: drop this CU's L1 lines (the window
// slots were read two pieces ago) - the L2 holds no window data when the
// windows are uncached; cached windows (or the system release mode) take
// the full system-scope acquire.
__device__ __forceinline__ void acquire_window(const Peers& P) {
  if (P.uncached && !P.release_system)
    asm volatile("buffer_inv sc0" ::: "memory");
  else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// Spin until *f >= v (wrap-safe). Every wait has an exit: the host's abort
// word or the timeout (which also raises the error word), so a dead peer
// never leaves a grid that cannot drain. Once any wait of the communicator
// timed out, the later ones give up at their first check instead of each
// waiting out the full timeout (the queued work then drains in moments).
__device__ void wait_geq(uint32_t* f, uint32_t v, const Peers& P) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned k = 1; static_cast<int>(sys_load(f) - v) < 0; ++k) {
    __builtin_amdgcn_s_sleep(1);
    if ((k & 255u) == 0) {
      if (__hip_atomic_load(P.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return;
      if (__hip_atomic_load(P.error_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return;
      if (__builtin_amdgcn_s_memrealtime() - t0 > P.timeout_ticks) {
        __hip_atomic_store(P.error_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
    }
  }
}

__device__ __forceinline__ uint32_t* coll_flag(const Peers& P, int owner, int phase, int src) {
  return P.flags[owner] + kFlagColl + (static_cast<size_t>(phase) * kMaxRanks + src) * kMaxBlocks + blockIdx.x;
}

// Sequence number of this kernel on a counter of the rank's own flag page:
// the value the previous kernel on the communicator published, plus one.
// Every block reads it before any block of the kernel can finish (the last
// block to finish is the one that advances it), so all blocks agree.
__device__ __forceinline__ uint32_t begin_seq(const Peers& P, size_t word) {
  __shared__ uint32_t seq;
  if (threadIdx.x == 0)
    seq = __hip_atomic_load(P.flags[P.rank] + word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  return seq;
}

// Count this block as finished; the last one resets the block counter and
// publishes `seq` for the next kernel (stream order makes it visible there).
// Returns true in thread 0 of the last block.
__device__ __forceinline__ bool end_seq(const Peers& P, size_t word, size_t done, uint32_t seq) {
  __syncthreads();
  if (threadIdx.x != 0) return false;
  uint32_t* f = P.flags[P.rank];
  // relaxed: the counters carry no data; the next kernel on the stream reads
  // them after this kernel's end-of-kernel release
  const uint32_t old = __hip_atomic_fetch_add(f + done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 != gridDim.x) return false;
  __hip_atomic_store(f + done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(f + word, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// This block's window stores are visible system-wide -> raise one flag per
// peer -> wait for every peer's flag of the same block and phase.
__device__ void exchange(const Peers& P, int phase, uint32_t epoch) {
  release_window(P);
  __syncthreads();
  const int t = threadIdx.x;
  if (t < P.nranks && t != P.rank) sys_store(coll_flag(P, t, phase, P.rank), epoch);
  if (t < P.nranks && t != P.rank) wait_geq(coll_flag(P, P.rank, phase, t), epoch, P);
  __syncthreads();
  acquire_window(P);
}

__device__ __forceinline__ void blk_range(size_t n, size_t& lo, size_t& hi) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  lo = min(n, static_cast<size_t>(blockIdx.x) * per);
  hi = min(n, lo + per);
}

__device__ __forceinline__ const uint4* V(const char* p) { return reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ uint4* V(char* p) { return reinterpret_cast<uint4*>(p); }

// dst[i] = src[i] for 16-B vectors i in [lo, hi), 4 loads in flight per thread.
__device__ __forceinline__ void copy_vec(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t lo,
                                         size_t hi) {
  size_t i = lo + threadIdx.x;
  for (; i + 3 * T < hi; i += 4 * T) {
    uint4 a = src[i], b = src[i + T], c = src[i + 2 * T], d = src[i + 3 * T];
    dst[i] = a;
    dst[i + T] = b;
    dst[i + 2 * T] = c;
    dst[i + 3 * T] = d;
  }
  for (; i < hi; i += T) dst[i] = src[i];
}

// Byte tail [from, to) of a message, done by the last block.
__device__ __forceinline__ void copy_tail(char* dst, const char* src, size_t from, size_t to) {
  if (blockIdx.x != gridDim.x - 1) return;
  for (size_t i = from + threadIdx.x; i < to; i += T) dst[i] = src[i];
}

// ---------------------------------------------------------------- dtypes

template <DType D>
struct Elt;
template <>
struct Elt<DType::BF16> {
  static constexpr int N = 8;
  __device__ static float ld(const char* p, size_t i) {
    uint32_t u = static_cast<uint32_t>(reinterpret_cast<const uint16_t*>(p)[i]) << 16;
    return __uint_as_float(u);
  }
  __device__ static void st(char* p, size_t i, float f) {
    __bf16 b = static_cast<__bf16>(f);
    reinterpret_cast<__bf16*>(p)[i] = b;
  }
  __device__ static void unpack(uint4 v, float* f) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = __uint_as_float(w[k] << 16);
      f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  __device__ static uint4 pack(const float* f) {
    typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
    bf16x8 b;
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = static_cast<__bf16>(f[k]);
    return __builtin_bit_cast(uint4, b);
  }
};
template <>
struct Elt<DType::FP16> {
  static constexpr int N = 8;
  __device__ static float ld(const char* p, size_t i) { return static_cast<float>(reinterpret_cast<const _Float16*>(p)[i]); }
  __device__ static void st(char* p, size_t i, float f) { reinterpret_cast<_Float16*>(p)[i] = static_cast<_Float16>(f); }
  __device__ static void unpack(uint4 v, float* f) {
    typedef __attribute__((ext_vector_type(8))) _Float16 h8;
    h8 h = __builtin_bit_cast(h8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = static_cast<float>(h[k]);
  }
  __device__ static uint4 pack(const float* f) {
    typedef __attribute__((ext_vector_type(8))) _Float16 h8;
    h8 h;
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = static_cast<_Float16>(f[k]);
    return __builtin_bit_cast(uint4, h);
  }
};
template <>
struct Elt<DType::FP32> {
  static constexpr int N = 4;
  __device__ static float ld(const char* p, size_t i) { return reinterpret_cast<const float*>(p)[i]; }
  __device__ static void st(char* p, size_t i, float f) { reinterpret_cast<float*>(p)[i] = f; }
  __device__ static void unpack(uint4 v, float* f) {
    f[0] = __uint_as_float(v.x);
    f[1] = __uint_as_float(v.y);
    f[2] = __uint_as_float(v.z);
    f[3] = __uint_as_float(v.w);
  }
  __device__ static uint4 pack(const float* f) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
};
// OCP fp8 (gfx950 converts natively; FP8_E5M2 = "bf8" in the ISA).
template <bool E5M2>
struct Fp8 {
  static constexpr int N = 16;
  __device__ static float cvt(uint32_t w, int sel) {
    if constexpr (E5M2) {
      switch (sel) {
        case 0: return __builtin_amdgcn_cvt_f32_bf8(w, 0);
        case 1: return __builtin_amdgcn_cvt_f32_bf8(w, 1);
        case 2: return __builtin_amdgcn_cvt_f32_bf8(w, 2);
        default: return __builtin_amdgcn_cvt_f32_bf8(w, 3);
      }
    } else {
      switch (sel) {
        case 0: return __builtin_amdgcn_cvt_f32_fp8(w, 0);
        case 1: return __builtin_amdgcn_cvt_f32_fp8(w, 1);
        case 2: return __builtin_amdgcn_cvt_f32_fp8(w, 2);
        default: return __builtin_amdgcn_cvt_f32_fp8(w, 3);
      }
    }
  }
  __device__ static uint32_t pk(float a, float b, float c, float d) {
    int r;
    if constexpr (E5M2) {
      r = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
      r = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, r, true);
    } else {
      r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
      r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
    }
    return static_cast<uint32_t>(r);
  }
  __device__ static float ld(const char* p, size_t i) { return cvt(reinterpret_cast<const uint8_t*>(p)[i], 0); }
  __device__ static void st(char* p, size_t i, float f) {
    reinterpret_cast<uint8_t*>(p)[i] = static_cast<uint8_t>(pk(f, f, f, f) & 0xffu);
  }
  __device__ static void unpack(uint4 v, float* f) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[4 * k + 0] = cvt(w[k], 0);
      f[4 * k + 1] = cvt(w[k], 1);
      f[4 * k + 2] = cvt(w[k], 2);
      f[4 * k + 3] = cvt(w[k], 3);
    }
  }
  __device__ static uint4 pack(const float* f) {
    return make_uint4(pk(f[0], f[1], f[2], f[3]), pk(f[4], f[5], f[6], f[7]), pk(f[8], f[9], f[10], f[11]),
                      pk(f[12], f[13], f[14], f[15]));
  }
};
template <>
struct Elt<DType::FP8_E4M3> : Fp8<false> {};
template <>
struct Elt<DType::FP8_E5M2> : Fp8<true> {};

// Loops over ranks are unrolled to kMaxRanks with a guard, never indexed by
// a run-time count: the per-rank pointer arrays then stay in (scalar)
// registers instead of going to scratch under the 64-register cap.

// Sum of vector i over the first ns sources, unpacked into acc (fp32), in
// source order. The loads of a group of G sources are issued before the first
// is used: on a node 7 of 8 sources are a peer's memory across xGMI (round
// trips of microseconds), and loading one source at a time (what the
// compiler made of a load-add loop: a vmcnt(0) after every load) left each
// thread with a single request in flight. G = 8 (all ranks) where the
// unpacked vector is <= 8 floats, 4 for fp8 (16 floats; 8 loads would not
// fit the 64-register budget beside two 16-float arrays).
template <DType D>
__device__ __forceinline__ void sum_vec(float* acc, const uint4* const* srcs, int ns, size_t i) {
  using E = Elt<D>;
  constexpr int G = E::N <= 8 ? 8 : 4;
  float f[E::N];
#pragma unroll
  for (int g = 0; g < kMaxRanks; g += G) {
    if (g < ns) {
      uint4 v[G];
#pragma unroll
      for (int u = 0; u < G; ++u)
        if (g + u < ns) v[u] = srcs[g + u][i];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        if (g + u < ns) {
          if (g + u == 0) {
            E::unpack(v[u], acc);
          } else {
            E::unpack(v[u], f);
#pragma unroll
            for (int k = 0; k < E::N; ++k) acc[k] += f[k];
          }
        }
      }
    }
  }
}

// out[i] = sum over srcs of vector i, for i in [lo, hi).
template <DType D>
__device__ __forceinline__ void reduce_vec(uint4* out, const uint4* const* srcs, int ns, size_t lo, size_t hi) {
  using E = Elt<D>;
  for (size_t i = lo + threadIdx.x; i < hi; i += T) {
    float acc[E::N];
    sum_vec<D>(acc, srcs, ns, i);
    out[i] = E::pack(acc);
  }
}

// Element tail [e0, e1) (elements), last block only.
template <DType D>
__device__ __forceinline__ void reduce_tail(char* out, const char* const* srcs, int ns, size_t e0, size_t e1) {
  using E = Elt<D>;
  if (blockIdx.x != gridDim.x - 1) return;
  for (size_t i = e0 + threadIdx.x; i < e1; i += T) {
    float a = 0.f;
#pragma unroll
    for (int s = 0; s < kMaxRanks; ++s)
      if (s < ns) a += E::ld(srcs[s], i);
    E::st(out, i, a);
  }
}

// --------------------------------------------------------------- kernels

__device__ __forceinline__ int peer_at(const Peers& P, int j) { return (P.rank + j) % P.nranks; }
// The j-th (0-based) of the n - 1 other ranks this block serves when every
// peer gets its own block of data: blocks start at different peers, so at
// any moment a rank's blocks feed all of its xGMI links instead of every
// block (and so the whole rank) streaming into the same peer.
__device__ __forceinline__ int peer_rot(const Peers& P, int j) {
  return peer_at(P, 1 + (j + static_cast<int>(blockIdx.x)) % (P.nranks - 1));
}

// for (r = 0; r < n; ++r) unrolled to kMaxRanks (see sum_vec)
#define DLNB_FOR_RANKS(r, lo, n) _Pragma("unroll") for (int r = (lo); r < kMaxRanks; ++r) if (r < (n))

// Push vectors [lo, hi) of src to slot `slot_off` of every peer's window
// (and to `own` unless null): 4 loads in flight per thread, each loaded
// vector stored to all peers (rank-staggered) before the next batch.
__device__ __forceinline__ void push_all(const Peers& P, const uint4* __restrict__ src, size_t slot_off,
                                         uint4* __restrict__ own, size_t lo, size_t hi) {
  size_t i = lo + threadIdx.x;
  for (; i + 3 * T < hi; i += 4 * T) {
    uint4 v[4] = {src[i], src[i + T], src[i + 2 * T], src[i + 3 * T]};
    for (int j = 1; j < P.nranks; ++j) {
      uint4* d = V(P.win[peer_at(P, j)] + slot_off);
#pragma unroll
      for (int u = 0; u < 4; ++u) d[i + u * T] = v[u];
    }
    if (own) {
#pragma unroll
      for (int u = 0; u < 4; ++u) own[i + u * T] = v[u];
    }
  }
  for (; i < hi; i += T) {
    const uint4 v = src[i];
    for (int j = 1; j < P.nranks; ++j) V(P.win[peer_at(P, j)] + slot_off)[i] = v;
    if (own) own[i] = v;
  }
}

DLNB_XGMI_KERNEL ag_kernel(Peers P, CollPiece c) {
  const uint32_t ep = begin_seq(P, kCtlCollEpoch);
  const size_t rg = (ep & 1) * c.region;
  const size_t nv = c.bytes / 16;
  size_t lo, hi;
  blk_range(nv, lo, hi);
  char* own = c.recv + static_cast<size_t>(P.rank) * c.recv_stride;
  const bool in_place = own == c.send;
  // push my block into slot[rank] of every peer's window (+ my own recv)
  push_all(P, V(c.send), rg + c.slot * P.rank, in_place ? nullptr : V(own), lo, hi);
  for (int j = 1; j < P.nranks; ++j) copy_tail(P.win[peer_at(P, j)] + rg + c.slot * P.rank, c.send, nv * 16, c.bytes);
  if (!in_place) copy_tail(own, c.send, nv * 16, c.bytes);
  exchange(P, 0, ep);
  for (int j = 1; j < P.nranks; ++j) {
    const int src = peer_at(P, P.nranks - j);
    const char* w = P.win[P.rank] + rg + c.slot * src;
    char* d = c.recv + static_cast<size_t>(src) * c.recv_stride;
    copy_vec(V(d), V(w), lo, hi);
    copy_tail(d, w, nv * 16, c.bytes);
  }
  end_seq(P, kCtlCollEpoch, kCtlCollDone, ep);
}

DLNB_XGMI_KERNEL a2a_kernel(Peers P, CollPiece c) {
  const uint32_t ep = begin_seq(P, kCtlCollEpoch);
  const size_t rg = (ep & 1) * c.region;
  const size_t nv = c.bytes / 16;
  size_t lo, hi;
  blk_range(nv, lo, hi);
  for (int j = 0; j + 1 < P.nranks; ++j) {
    const int p = peer_rot(P, j);
    char* w = P.win[p] + rg + c.slot * P.rank;
    const char* s = c.send + static_cast<size_t>(p) * c.send_stride;
    copy_vec(V(w), V(s), lo, hi);
    copy_tail(w, s, nv * 16, c.bytes);
  }
  {
    char* d = c.recv + static_cast<size_t>(P.rank) * c.recv_stride;
    const char* s = c.send + static_cast<size_t>(P.rank) * c.send_stride;
    copy_vec(V(d), V(s), lo, hi);
    copy_tail(d, s, nv * 16, c.bytes);
  }
  exchange(P, 0, ep);
  for (int j = 1; j < P.nranks; ++j) {
    const int src = peer_at(P, P.nranks - j);
    const char* w = P.win[P.rank] + rg + c.slot * src;
    char* d = c.recv + static_cast<size_t>(src) * c.recv_stride;
    copy_vec(V(d), V(w), lo, hi);
    copy_tail(d, w, nv * 16, c.bytes);
  }
  end_seq(P, kCtlCollEpoch, kCtlCollDone, ep);
}

template <DType D>
DLNB_XGMI_KERNEL rs_kernel(Peers P, CollPiece c) {
  const uint32_t ep = begin_seq(P, kCtlCollEpoch);
  const size_t rg = (ep & 1) * c.region;
  const size_t es = sizeof(uint4) / Elt<D>::N;
  const size_t nv = c.bytes / 16;
  size_t lo, hi;
  blk_range(nv, lo, hi);
  for (int j = 0; j + 1 < P.nranks; ++j) {
    const int p = peer_rot(P, j);
    char* w = P.win[p] + rg + c.slot * P.rank;
    const char* s = c.send + static_cast<size_t>(p) * c.send_stride;
    copy_vec(V(w), V(s), lo, hi);
    copy_tail(w, s, nv * 16, c.bytes);
  }
  exchange(P, 0, ep);
  const uint4* srcs[kMaxRanks];
  const char* srcb[kMaxRanks];
  srcb[0] = c.send + static_cast<size_t>(P.rank) * c.send_stride;
  DLNB_FOR_RANKS(j, 1, P.nranks) srcb[j] = P.win[P.rank] + rg + c.slot * peer_at(P, j);
  DLNB_FOR_RANKS(j, 0, P.nranks) srcs[j] = V(srcb[j]);
  reduce_vec<D>(V(c.recv), srcs, P.nranks, lo, hi);
  reduce_tail<D>(c.recv, srcb, P.nranks, nv * 16 / es, c.bytes / es);
  end_seq(P, kCtlCollEpoch, kCtlCollDone, ep);
}

template <DType D>
DLNB_XGMI_KERNEL ar1_kernel(Peers P, CollPiece c) {
  const uint32_t ep = begin_seq(P, kCtlCollEpoch);
  const size_t rg = (ep & 1) * c.region;
  const size_t es = sizeof(uint4) / Elt<D>::N;
  const size_t nv = c.bytes / 16;
  size_t lo, hi;
  blk_range(nv, lo, hi);
  push_all(P, V(c.send), rg + c.slot * P.rank, nullptr, lo, hi);
  for (int j = 1; j < P.nranks; ++j) copy_tail(P.win[peer_at(P, j)] + rg + c.slot * P.rank, c.send, nv * 16, c.bytes);
  exchange(P, 0, ep);
  // every rank sums in the same (rank) order -> bitwise identical results
  const uint4* srcs[kMaxRanks];
  const char* srcb[kMaxRanks];
  DLNB_FOR_RANKS(r, 0, P.nranks) srcb[r] = r == P.rank ? c.send : P.win[P.rank] + rg + c.slot * r;
  DLNB_FOR_RANKS(r, 0, P.nranks) srcs[r] = V(srcb[r]);
  reduce_vec<D>(V(c.recv), srcs, P.nranks, lo, hi);
  reduce_tail<D>(c.recv, srcb, P.nranks, nv * 16 / es, c.bytes / es);
  end_seq(P, kCtlCollEpoch, kCtlCollDone, ep);
}

// Two-shot (reduce-scatter + all-gather inside one kernel). c.bytes is a
// multiple of 16; chunk p = vectors [p*cv, min((p+1)*cv, nv)).
template <DType D>
DLNB_XGMI_KERNEL ar2_kernel(Peers P, CollPiece c) {
  const uint32_t ep = begin_seq(P, kCtlCollEpoch);
  const size_t rg = (ep & 1) * c.region;
  const size_t nv = c.bytes / 16;
  const size_t cv = (nv + P.nranks - 1) / P.nranks;
  size_t lo, hi;  // this block's slice of a chunk
  blk_range(cv, lo, hi);
  auto chunk_hi = [&](int p, size_t h) { return min(h, nv > p * cv ? nv - p * cv : size_t(0)); };
  // 1. chunk p -> peer p's RS slot[rank]
  for (int j = 0; j + 1 < P.nranks; ++j) {
    const int p = peer_rot(P, j);
    copy_vec(V(P.win[p] + rg + c.slot * P.rank), V(c.send) + p * cv, lo, chunk_hi(p, hi));
  }
  exchange(P, 0, ep);
  // 2. reduce my chunk (rank order), write it to recv and to every peer's AG slot[rank]
  const uint4* srcs[kMaxRanks];
  DLNB_FOR_RANKS(r, 0, P.nranks) srcs[r] = r == P.rank ? V(c.send) + P.rank * cv : V(P.win[P.rank] + rg + c.slot * r);
  uint4* outs[kMaxRanks];
  DLNB_FOR_RANKS(j, 1, P.nranks) outs[j - 1] = V(P.win[peer_at(P, j)] + rg + c.ag_off + c.slot * P.rank);
  // srcs are chunk-relative; recv chunk rank
  {
    using E = Elt<D>;
    const size_t h = chunk_hi(P.rank, hi);
    uint4* out = V(c.recv) + P.rank * cv;
    for (size_t i = lo + threadIdx.x; i < h; i += T) {
      float acc[E::N];
      sum_vec<D>(acc, srcs, P.nranks, i);
      uint4 r = E::pack(acc);
      out[i] = r;
      DLNB_FOR_RANKS(o, 0, P.nranks - 1) outs[o][i] = r;
    }
  }
  exchange(P, 1, ep);
  // 3. copy the peers' reduced chunks out of my AG slots
  for (int j = 1; j < P.nranks; ++j) {
    const int src = peer_at(P, P.nranks - j);
    copy_vec(V(c.recv) + src * cv, V(P.win[P.rank] + rg + c.ag_off + c.slot * src), lo, chunk_hi(src, hi));
  }
  end_seq(P, kCtlCollEpoch, kCtlCollDone, ep);
}

// ------------------------------------------------ zero-copy (registered)

// dst[j][i] = src[i] for every rank j (own first, then rank-staggered), 4
// loads in flight per thread.
__device__ __forceinline__ void push_ptrs(const Peers& P, const uint4* __restrict__ src, char* const* dst, size_t lo,
                                          size_t hi) {
  size_t i = lo + threadIdx.x;
  for (; i + 3 * T < hi; i += 4 * T) {
    uint4 v[4] = {src[i], src[i + T], src[i + 2 * T], src[i + 3 * T]};
    for (int j = 0; j < P.nranks; ++j) {
      uint4* d = V(dst[peer_at(P, j)]);
#pragma unroll
      for (int u = 0; u < 4; ++u) d[i + u * T] = v[u];
    }
  }
  for (; i < hi; i += T) {
    const uint4 v = src[i];
    for (int j = 0; j < P.nranks; ++j) V(dst[peer_at(P, j)])[i] = v;
  }
}

DLNB_XGMI_KERNEL ag_direct_kernel(Peers P, DirectPiece c) {
  const uint32_t ep = begin_seq(P, kCtlCollEpoch);
  exchange(P, 0, ep);  // every rank's receive buffer is free
  const size_t nv = c.bytes / 16;
  size_t lo, hi;
  blk_range(nv, lo, hi);
  push_ptrs(P, V(c.src[P.rank]), c.dst, lo, hi);
  for (int r = 0; r < P.nranks; ++r) copy_tail(c.dst[r], c.src[P.rank], nv * 16, c.bytes);
  exchange(P, 1, ep);  // every rank's block landed in my receive buffer
  end_seq(P, kCtlCollEpoch, kCtlCollDone, ep);
}

DLNB_XGMI_KERNEL a2a_direct_kernel(Peers P, DirectPiece c) {
  const uint32_t ep = begin_seq(P, kCtlCollEpoch);
  exchange(P, 0, ep);  // every rank's receive buffer is free
  const size_t nv = c.bytes / 16;
  size_t lo, hi;
  blk_range(nv, lo, hi);
  // block j of my send -> slot `rank` of rank j's receive buffer; blocks
  // start at different ranks (own block included) so all links carry data
  for (int j = 0; j < P.nranks; ++j) {
    const int r = peer_at(P, (j + static_cast<int>(blockIdx.x)) % P.nranks);
    const char* s = c.src[P.rank] + static_cast<size_t>(r) * c.bytes;
    copy_vec(V(c.dst[r]), V(s), lo, hi);
    copy_tail(c.dst[r], s, nv * 16, c.bytes);
  }
  exchange(P, 1, ep);  // every rank's block for me landed
  end_seq(P, kCtlCollEpoch, kCtlCollDone, ep);
}

template <DType D>
DLNB_XGMI_KERNEL rs_direct_kernel(Peers P, DirectPiece c) {
  const size_t es = sizeof(uint4) / Elt<D>::N;
  const uint32_t ep = begin_seq(P, kCtlCollEpoch);
  exchange(P, 0, ep);  // every rank's send buffer holds its data
  const size_t nv = c.bytes / 16;
  size_t lo, hi;
  blk_range(nv, lo, hi);
  const uint4* srcs[kMaxRanks];
  DLNB_FOR_RANKS(r, 0, P.nranks) srcs[r] = V(c.src[r]);  // rank order: identical sums everywhere
  reduce_vec<D>(V(c.out), srcs, P.nranks, lo, hi);
  reduce_tail<D>(c.out, c.src, P.nranks, nv * 16 / es, c.bytes / es);
  exchange(P, 1, ep);  // every rank is done reading my send buffer
  end_seq(P, kCtlCollEpoch, kCtlCollDone, ep);
}

template <DType D>
DLNB_XGMI_KERNEL ar_direct_kernel(Peers P, DirectPiece c) {
  using E = Elt<D>;
  const uint32_t ep = begin_seq(P, kCtlCollEpoch);
  exchange(P, 0, ep);
  const size_t nv = c.bytes / 16;
  const size_t cv = (nv + P.nranks - 1) / P.nranks;
  const size_t c0 = min(nv, static_cast<size_t>(P.rank) * cv), c1 = min(nv, c0 + cv);
  size_t lo, hi;
  blk_range(c1 - c0, lo, hi);
  const uint4* srcs[kMaxRanks];
  DLNB_FOR_RANKS(r, 0, P.nranks) srcs[r] = V(c.src[r]) + c0;
  // chunk `rank` of every send buffer, summed in rank order, into chunk
  // `rank` of every receive buffer (only this rank reads or writes that
  // chunk anywhere, so send and receive may alias)
  for (size_t i = lo + threadIdx.x; i < hi; i += T) {
    float acc[E::N];
    sum_vec<D>(acc, srcs, P.nranks, i);
    const uint4 v = E::pack(acc);
    for (int j = 0; j < P.nranks; ++j) (V(c.dst[peer_at(P, j)]) + c0)[i] = v;
  }
  exchange(P, 1, ep);
  end_seq(P, kCtlCollEpoch, kCtlCollDone, ep);
}

DLNB_XGMI_KERNEL send_kernel(Peers P, const char* buf, size_t bytes, int dst, size_t off,
                                                 size_t slot) {
  const uint32_t n = begin_seq(P, kCtlSendSeq + dst);
  if (threadIdx.x == 0 && n > 2) wait_geq(P.flags[P.rank] + kFlagP2PConsumed + dst, n - 2, P);
  __syncthreads();
  const size_t nv = bytes / 16;
  size_t lo, hi;
  blk_range(nv, lo, hi);
  char* w = P.win[dst] + off + (n & 1) * slot;
  copy_vec(V(w), V(buf), lo, hi);
  copy_tail(w, buf, nv * 16, bytes);
  release_window(P);
  __syncthreads();
  if (threadIdx.x == 0) sys_store(P.flags[dst] + kFlagP2PSeq + static_cast<size_t>(P.rank) * kMaxBlocks + blockIdx.x, n);
  end_seq(P, kCtlSendSeq + dst, kCtlSendDone + dst, n);
}

DLNB_XGMI_KERNEL recv_kernel(Peers P, char* buf, size_t bytes, int src, size_t off, size_t slot) {
  const uint32_t n = begin_seq(P, kCtlRecvSeq + src);
  if (threadIdx.x == 0) wait_geq(P.flags[P.rank] + kFlagP2PSeq + static_cast<size_t>(src) * kMaxBlocks + blockIdx.x, n, P);
  __syncthreads();
  acquire_window(P);
  const size_t nv = bytes / 16;
  size_t lo, hi;
  blk_range(nv, lo, hi);
  const char* w = P.win[P.rank] + off + (n & 1) * slot;
  copy_vec(V(buf), V(w), lo, hi);
  copy_tail(buf, w, nv * 16, bytes);
  // the last block to finish tells the sender that message n was consumed
  if (end_seq(P, kCtlRecvSeq + src, kCtlRecvDone + src, n)) sys_store(P.flags[src] + kFlagP2PConsumed + P.rank, n);
}

struct LocalArgs {
  const char* src[kMaxLocal];
  char* dst[kMaxLocal];
  int ns, nd;
  size_t count;  // elements
};

// Grid-stride over 16-B vectors (VEC: every pointer 16-B aligned), then the
// element tail; a copy (ns == 1) moves raw vectors, no dtype round trip.
template <DType D, bool VEC>
__global__ void __launch_bounds__(T) local_reduce_kernel(LocalArgs a) {
  using E = Elt<D>;
  const size_t stride = static_cast<size_t>(gridDim.x) * T;
  const size_t tid = static_cast<size_t>(blockIdx.x) * T + threadIdx.x;
  const size_t nv = VEC ? a.count / E::N : 0;
  for (size_t i = tid; i < nv; i += stride) {
    uint4 v = V(a.src[0])[i];
    if (a.ns > 1) {
      float acc[E::N], f[E::N];
      E::unpack(v, acc);
      for (int s = 1; s < a.ns; ++s) {
        E::unpack(V(a.src[s])[i], f);
#pragma unroll
        for (int k = 0; k < E::N; ++k) acc[k] += f[k];
      }
      v = E::pack(acc);
    }
    for (int d = 0; d < a.nd; ++d) V(a.dst[d])[i] = v;
  }
  const size_t es = sizeof(uint4) / E::N;
  for (size_t i = nv * E::N + tid; i < a.count; i += stride) {
    if (a.ns == 1) {
      for (int d = 0; d < a.nd; ++d)
        for (size_t b = 0; b < es; ++b) a.dst[d][i * es + b] = a.src[0][i * es + b];
      continue;
    }
    float x = 0.f;
    for (int s = 0; s < a.ns; ++s) x += E::ld(a.src[s], i);
    for (int d = 0; d < a.nd; ++d) E::st(a.dst[d], i, x);
  }
}

struct CollArgs {
  const char* send[kMaxLocal];
  char* recv[kMaxLocal];
  int W;
  size_t blk;  // elements per rank block
};

// blockIdx.y = the rank block this block works on: the source rank i
// (all-gather, all-to-all) or the destination rank j (reduce-scatter).
template <DType D, LocalColl OP, bool VEC>
__global__ void __launch_bounds__(T) local_coll_kernel(CollArgs a) {
  using E = Elt<D>;
  const int b = blockIdx.y;
  const size_t stride = static_cast<size_t>(gridDim.x) * T;
  const size_t tid = static_cast<size_t>(blockIdx.x) * T + threadIdx.x;
  constexpr size_t es = sizeof(uint4) / E::N;
  const size_t bb = a.blk * es;  // bytes per rank block
  const size_t nv = VEC ? a.blk / E::N : 0;
  for (size_t v = tid; v < nv; v += stride) {
    if constexpr (OP == LocalColl::AllGather) {
      const uint4 x = V(a.send[b])[v];
      for (int j = 0; j < a.W; ++j) V(a.recv[j] + b * bb)[v] = x;
    } else if constexpr (OP == LocalColl::ReduceScatter) {
      float acc[E::N], f[E::N];
      E::unpack(V(a.send[0] + b * bb)[v], acc);
      for (int i = 1; i < a.W; ++i) {
        E::unpack(V(a.send[i] + b * bb)[v], f);
#pragma unroll
        for (int k = 0; k < E::N; ++k) acc[k] += f[k];
      }
      V(a.recv[b])[v] = E::pack(acc);
    } else {
      for (int j = 0; j < a.W; ++j) V(a.recv[j] + b * bb)[v] = V(a.send[b] + j * bb)[v];
    }
  }
  for (size_t e = nv * E::N + tid; e < a.blk; e += stride) {
    if constexpr (OP == LocalColl::ReduceScatter) {
      float x = 0.f;
      for (int i = 0; i < a.W; ++i) x += E::ld(a.send[i] + b * bb, e);
      E::st(a.recv[b], e, x);
    } else {
      for (int j = 0; j < a.W; ++j) {
        const char* src = OP == LocalColl::AllGather ? a.send[b] : a.send[b] + j * bb;
        char* dst = a.recv[j] + b * bb;
        for (size_t k = 0; k < es; ++k) dst[e * es + k] = src[e * es + k];
      }
    }
  }
}

template <DType D, LocalColl OP>
void local_coll_typed(const CollArgs& a, bool vec, dim3 grid, hipStream_t s) {
  if (vec)
    local_coll_kernel<D, OP, true><<<grid, T, 0, s>>>(a);
  else
    local_coll_kernel<D, OP, false><<<grid, T, 0, s>>>(a);
}

template <LocalColl OP>
void local_coll_dtype(const CollArgs& a, DType t, bool vec, dim3 grid, hipStream_t s) {
  switch (t) {
    case DType::BF16: local_coll_typed<DType::BF16, OP>(a, vec, grid, s); break;
    case DType::FP16: local_coll_typed<DType::FP16, OP>(a, vec, grid, s); break;
    case DType::FP32: local_coll_typed<DType::FP32, OP>(a, vec, grid, s); break;
    case DType::FP8_E4M3: local_coll_typed<DType::FP8_E4M3, OP>(a, vec, grid, s); break;
    case DType::FP8_E5M2: local_coll_typed<DType::FP8_E5M2, OP>(a, vec, grid, s); break;
  }
}

template <DType D>
void local_reduce_typed(const LocalArgs& a, bool vec, int blocks, hipStream_t s) {
  if (vec)
    local_reduce_kernel<D, true><<<blocks, T, 0, s>>>(a);
  else
    local_reduce_kernel<D, false><<<blocks, T, 0, s>>>(a);
}

#define DLNB_XGMI_TYPED(KERNEL)                                                                       \
  switch (c.dtype) {                                                                                 \
    case DType::BF16: KERNEL<DType::BF16><<<blocks, T, 0, s>>>(p, c); break;                         \
    case DType::FP16: KERNEL<DType::FP16><<<blocks, T, 0, s>>>(p, c); break;                         \
    case DType::FP32: KERNEL<DType::FP32><<<blocks, T, 0, s>>>(p, c); break;                         \
    case DType::FP8_E4M3: KERNEL<DType::FP8_E4M3><<<blocks, T, 0, s>>>(p, c); break;                 \
    case DType::FP8_E5M2: KERNEL<DType::FP8_E5M2><<<blocks, T, 0, s>>>(p, c); break;                 \
  }

}  // namespace

int blocks_for(size_t bytes, int max_blocks) {
  // ~64 KB per block (512 threads x 16 B x 8) keeps enough stores in flight
  // per CU; small messages use few blocks (fewer flags to exchange).
  size_t b = (bytes + 65535) / 65536;
  if (b < 1) b = 1;
  if (b > static_cast<size_t>(max_blocks)) b = static_cast<size_t>(max_blocks);
  if (b > static_cast<size_t>(kMaxBlocks)) b = kMaxBlocks;
  return static_cast<int>(b);
}

void launch_coll(Op op, const Peers& p, const CollPiece& c, int blocks, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  DLNB_REQUIRE(blocks >= 1 && blocks <= kMaxBlocks, "xgmi: bad block count " << blocks);
  DLNB_REQUIRE(p.nranks >= 1 && p.nranks <= kMaxRanks, "xgmi: bad group size " << p.nranks);
  switch (op) {
    case Op::AllGather: ag_kernel<<<blocks, T, 0, s>>>(p, c); break;
    case Op::AllToAll: a2a_kernel<<<blocks, T, 0, s>>>(p, c); break;
    case Op::ReduceScatter: DLNB_XGMI_TYPED(rs_kernel) break;
    case Op::AllReduceOneShot: DLNB_XGMI_TYPED(ar1_kernel) break;
    case Op::AllReduceTwoShot:
      DLNB_REQUIRE(c.bytes % 16 == 0, "xgmi: two-shot piece must be a multiple of 16 B");
      DLNB_XGMI_TYPED(ar2_kernel) break;
  }
  DLNB_HIP_CHECK(hipGetLastError());
}

void launch_direct(DirectOp op, const Peers& p, const DirectPiece& c, int blocks, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  DLNB_REQUIRE(blocks >= 1 && blocks <= kMaxBlocks, "xgmi: bad block count " << blocks);
  DLNB_REQUIRE(p.nranks >= 1 && p.nranks <= kMaxRanks, "xgmi: bad group size " << p.nranks);
  switch (op) {
    case DirectOp::AllGather: ag_direct_kernel<<<blocks, T, 0, s>>>(p, c); break;
    case DirectOp::AllToAll: a2a_direct_kernel<<<blocks, T, 0, s>>>(p, c); break;
    case DirectOp::ReduceScatter: DLNB_XGMI_TYPED(rs_direct_kernel) break;
    case DirectOp::AllReduce:
      DLNB_REQUIRE(c.bytes % 16 == 0, "xgmi: direct all-reduce needs a multiple of 16 B");
      DLNB_XGMI_TYPED(ar_direct_kernel) break;
  }
  DLNB_HIP_CHECK(hipGetLastError());
}

void launch_local_reduce(char* const* dsts, int nd, const char* const* srcs, int ns, size_t count, DType t,
                         void* stream) {
  DLNB_REQUIRE(ns >= 1 && ns <= kMaxLocal && nd >= 1 && nd <= kMaxLocal,
               "local reduce: " << ns << " sources / " << nd << " destinations (1.." << kMaxLocal << ")");
  if (count == 0) return;
  LocalArgs a{};
  a.ns = ns;
  a.nd = nd;
  a.count = count;
  bool vec = true;
  for (int i = 0; i < ns; ++i) {
    a.src[i] = srcs[i];
    vec = vec && (reinterpret_cast<uintptr_t>(srcs[i]) & 15u) == 0;
  }
  for (int i = 0; i < nd; ++i) {
    a.dst[i] = dsts[i];
    vec = vec && (reinterpret_cast<uintptr_t>(dsts[i]) & 15u) == 0;
  }
  const size_t per_vec = 16 / dtype_size(t);
  const size_t work = vec ? std::max<size_t>(1, count / per_vec) : count;
  const int blocks = static_cast<int>(std::min<size_t>(2048, std::max<size_t>(1, (work + 4 * T - 1) / (4 * T))));
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (t) {
    case DType::BF16: local_reduce_typed<DType::BF16>(a, vec, blocks, s); break;
    case DType::FP16: local_reduce_typed<DType::FP16>(a, vec, blocks, s); break;
    case DType::FP32: local_reduce_typed<DType::FP32>(a, vec, blocks, s); break;
    case DType::FP8_E4M3: local_reduce_typed<DType::FP8_E4M3>(a, vec, blocks, s); break;
    case DType::FP8_E5M2: local_reduce_typed<DType::FP8_E5M2>(a, vec, blocks, s); break;
  }
  DLNB_HIP_CHECK(hipGetLastError());
}

void launch_local_coll(LocalColl op, char* const* recv, const char* const* send, int W, size_t blk, DType t,
                       void* stream) {
  DLNB_REQUIRE(W >= 1 && W <= kMaxLocal, "local collective: " << W << " ranks (1.." << kMaxLocal << ")");
  if (blk == 0) return;
  CollArgs a{};
  a.W = W;
  a.blk = blk;
  const size_t es = dtype_size(t);
  bool vec = (blk * es) % 16 == 0;
  for (int i = 0; i < W; ++i) {
    a.send[i] = send[i];
    a.recv[i] = recv[i];
    vec = vec && (reinterpret_cast<uintptr_t>(send[i]) & 15u) == 0 && (reinterpret_cast<uintptr_t>(recv[i]) & 15u) == 0;
  }
  const size_t work = vec ? std::max<size_t>(1, blk * es / 16) : blk;
  // ~2048 blocks in total across the W rank blocks
  const size_t per = std::max<size_t>(1, std::min<size_t>((work + 4 * T - 1) / (4 * T), 2048 / W));
  const dim3 grid(static_cast<unsigned>(per), static_cast<unsigned>(W));
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (op) {
    case LocalColl::AllGather: local_coll_dtype<LocalColl::AllGather>(a, t, vec, grid, s); break;
    case LocalColl::ReduceScatter: local_coll_dtype<LocalColl::ReduceScatter>(a, t, vec, grid, s); break;
    case LocalColl::AllToAll: local_coll_dtype<LocalColl::AllToAll>(a, t, vec, grid, s); break;
  }
  DLNB_HIP_CHECK(hipGetLastError());
}

namespace {

template <typename K>
void occ(std::vector<KernelOccupancy>& out, const char* name, K kernel) {
  int n = 0;
  DLNB_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, T, 0));
  out.push_back({name, n});
}

#define DLNB_XGMI_OCC_TYPED(KERNEL)                                \
  occ(v, #KERNEL "<bf16>", KERNEL<DType::BF16>);                   \
  occ(v, #KERNEL "<fp16>", KERNEL<DType::FP16>);                   \
  occ(v, #KERNEL "<fp32>", KERNEL<DType::FP32>);                   \
  occ(v, #KERNEL "<fp8_e4m3>", KERNEL<DType::FP8_E4M3>);           \
  occ(v, #KERNEL "<fp8_e5m2>", KERNEL<DType::FP8_E5M2>);

}  // namespace

std::vector<KernelOccupancy> occupancy() {
  std::vector<KernelOccupancy> v;
  occ(v, "ag_kernel", ag_kernel);
  occ(v, "a2a_kernel", a2a_kernel);
  occ(v, "ag_direct_kernel", ag_direct_kernel);
  occ(v, "a2a_direct_kernel", a2a_direct_kernel);
  occ(v, "send_kernel", send_kernel);
  occ(v, "recv_kernel", recv_kernel);
  DLNB_XGMI_OCC_TYPED(rs_kernel)
  DLNB_XGMI_OCC_TYPED(ar1_kernel)
  DLNB_XGMI_OCC_TYPED(ar2_kernel)
  DLNB_XGMI_OCC_TYPED(rs_direct_kernel)
  DLNB_XGMI_OCC_TYPED(ar_direct_kernel)
  return v;
}

int min_blocks_per_cu() {
  static int cached = [] {
    int m = kBlocksPerCU;
    for (const auto& k : occupancy()) m = std::min(m, k.blocks_per_cu);
    return std::max(1, m);
  }();
  return cached;
}

void launch_send(const Peers& p, const char* buf, size_t bytes, int dst, size_t off, size_t slot, int blocks,
                 void* stream) {
  send_kernel<<<blocks, T, 0, static_cast<hipStream_t>(stream)>>>(p, buf, bytes, dst, off, slot);
  DLNB_HIP_CHECK(hipGetLastError());
}

void launch_recv(const Peers& p, char* buf, size_t bytes, int src, size_t off, size_t slot, int blocks,
                 void* stream) {
  recv_kernel<<<blocks, T, 0, static_cast<hipStream_t>(stream)>>>(p, buf, bytes, src, off, slot);
  DLNB_HIP_CHECK(hipGetLastError());
}

}  // namespace xgmi
}  // namespace dlnb
