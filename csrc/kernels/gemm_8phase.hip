// 8-phase ping-pong MFMA GEMM for gfx950: C[M,N] (bf16) = A[M,K] . B[N,K]^T.
//
// Same operand contract as gemm_tn_256_kernel (kernels.hip) - bf16 or OCP
// fp8 e4m3 inputs, 256 x 256 block tile, 128-byte K-tiles, XOR-swizzled
// lane-linear LDS image filled by global_load_lds - but a different schedule
// (cdna_hip_programming.md §5 "The 256² 8-phase template", T3+T4):
//
//   * A K-tile is split into four 128-row half-tiles (A0 A1 | B0 B1, 16 KiB
//     each; two 64 KiB buffers = 128 KiB LDS) and its MFMA work into four
//     phases, one per 128 x 128 quadrant of C, visited (0,0) (0,1) (1,1)
//     (1,0) so every phase after the first reads ONE half-tile's fragments
//     (the B0 fragments of phase 0 stay in registers for phase 3).
//   * Every phase = {ds_read its fragments, issue one half-tile of
//     global_load_lds (2 per thread), counted vmcnt, raw s_barrier, MFMAs
//     under s_setprio(1), raw s_barrier}. The two wave rows run one barrier
//     apart (wave row 1 takes an extra barrier up front), so on every SIMD
//     one wave issues its loads while the other one runs its MFMAs.
//   * Loads stay in flight across barriers: a half-tile is waited for
//     (vmcnt(8) = 4 half-tiles still in flight) four phases after it was
//     issued and read one phase after that wait; a buffer slot is re-staged
//     at least two phases after its last read (the RAW / WAR rules of the
//     staggered schedule; derivation in docs/KERNELS.md).
//
// Variant 3 of dlnb::kernels::gemm_tn (the library's one-shot GEMM).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "deadline_sync.hpp"
#include "dlnb/kernels.hpp"
#include "store_pair.hpp"

namespace dlnb {
namespace kernels {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kT = 256;          // block tile (M and N)
constexpr int kRB = 128;         // bytes of K per K-tile row
constexpr int kHalf = 128 * kRB; // one half-tile: 128 rows x 128 B = 16 KiB
constexpr int kBuf = 4 * kHalf;  // A0 A1 B0 B1
enum : int { kA0 = 0, kA1 = 1, kB0 = 2, kB1 = 3 };

__device__ __forceinline__ int swz(int row, int chunk) { return row * kRB + ((chunk ^ ((row >> 1) & 7)) << 4); }

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at "no wait"), gfx9 encoding.
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// One half-tile: 16 wave-instructions of buffer_load_dwordx4 ... lds, 2 per
// wave (instruction i*8 + w: rows 8 (i*8 + w) .. +7, 128 B each). The swizzle
// is applied to the per-lane source offset (LDS writes are lane-linear): LDS
// slot q of row r holds chunk q ^ ((r >> 1) & 7). The lane offset
// (lane_offset) is loop-invariant; the half-tile's first row is the
// (scalar) resource base and the K-tile the scalar offset, so staging costs
// no per-lane address arithmetic (the per-lane 64-bit global_load_lds
// addresses it replaces cost 10 % in the one-wave-per-SIMD kernel,
// profiles/gemm_bench_r2.md).
__device__ __forceinline__ void stage_half(const char* base, int voff, size_t ld, int soff, char* lds, int w) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, 0x7ffffff0, 0x00020000);
#pragma unroll
  for (int i = 0; i < 2; ++i)  // instruction 1 = instruction 0 + 64 rows (same swizzle phase): a scalar offset
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(lds + (i * 8 + w) * 1024), 16, voff,
                                             soff + i * 64 * static_cast<int>(ld), 0, 0);
}

// The lane's offset within its first staging instruction (w * 64 + lane).
__device__ __forceinline__ int lane_offset(size_t ld, int w, int lane) {
  const int slot = w * 64 + lane;
  const int r = slot >> 3;
  const int q = (slot & 7) ^ ((r >> 1) & 7);
  return static_cast<int>(r * ld) + (q << 4);
}

__device__ __forceinline__ int xcd_remap(int b, int T) {
  const int q = T / 8, r = T % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Fragment registers of one wave. bf16: [k-step][frag] 16-B reads;
// fp8: one 32-B (two-chunk) read pair per fragment covers the whole K-tile.
template <bool FP8>
struct Frags;
template <>
struct Frags<false> {
  bf16x8 a[2][4], bx[2][2], by[2][2];
};
template <>
struct Frags<true> {
  i32x8 a[4], bx[2], by[2];
};

template <bool FP8, int NF>
__device__ __forceinline__ void read_frags(const char* half, int row0, int r16, int h, bf16x8 (&f)[2][NF]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < NF; ++i) f[ks][i] = *reinterpret_cast<const bf16x8*>(half + swz(row0 + i * 16 + r16, ks * 4 + h));
}
template <bool FP8, int NF>
__device__ __forceinline__ void read_frags(const char* half, int row0, int r16, int h, i32x8 (&f)[NF]) {
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int row = row0 + i * 16 + r16;
    // K chunks h and h + 4 (same order for A and B): conflict-free under the
    // swizzle, where chunks 2h, 2h + 1 are 2-way on every ds_read_b128
    const i32x4 lo = *reinterpret_cast<const i32x4*>(half + swz(row, h));
    const i32x4 hi = *reinterpret_cast<const i32x4*>(half + swz(row, h + 4));
    f[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);  // register concat, no element moves
  }
}

// acc[i][j] += A-frags x B-frags for one 64 x 32 sub-tile of a quadrant.
__device__ __forceinline__ void mfma_quadrant(f32x4 (&acc)[4][2], const bf16x8 (&a)[2][4], const bf16x8 (&b)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], a[ks][i], acc[i][j], 0, 0, 0);
}
__device__ __forceinline__ void mfma_quadrant(f32x4 (&acc)[4][2], const i32x8 (&a)[4], const i32x8 (&b)[2]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b[j], a[i], acc[i][j], 0, 0, 0, 127, 0, 127);
}

struct Ctx {
  const char* Ab;  // A rows of this block tile, K-tile 0
  const char* Bb;
  size_t lda, ldb;  // bytes
  char* smem;
  int w, lane, wr, wc, r16, h;
  int last_kt;  // uniform K-loop: staging of K-tiles past the last one re-reads it (never consumed)
  int voffA, voffB;  // staging lane offsets (lane_offset)
};

// Where half-tile `slot` of K-tile t comes from / goes to.
__device__ __forceinline__ void stage(const Ctx& c, int t, int slot) {
  const int tk = min(t, c.last_kt);  // == t except for the uniform loop's two overrun K-tiles
  const bool isA = slot == kA0 || slot == kA1;
  const int hi = slot == kA1 || slot == kB1;
  const char* base = isA ? c.Ab + static_cast<size_t>(hi) * 128 * c.lda : c.Bb + static_cast<size_t>(hi) * 128 * c.ldb;
  stage_half(base, isA ? c.voffA : c.voffB, isA ? c.lda : c.ldb, tk * kRB, c.smem + (t & 1) * kBuf + slot * kHalf, c.w);
}

// Deadline state of the persistent variant: thread 0 (wave row 0) reads the
// clock at the end of phase 2 of every K-tile, writes the stop
// decision in phase 3 into an LDS flag
// (completed before its barrier), and every wave reads it after its own first
// barrier of that phase - the write precedes every read (the rows are one
// barrier apart) and the next write is four phases away.
typedef __attribute__((address_space(3))) volatile int lds_flag_t;
struct Deadline {
  uint64_t t0, ticks, slice_end;
  lds_flag_t* flag;  // 2 ints at the end of the staging array (typed LDS: a
                     // generic pointer becomes a flat store that waits vmcnt(0))
  int tid;
};

// Phase Q of K-tile v. Staging schedule (G = half-tile issued in the phase):
//   Q0: B1(v+1)  Q1: A1(v+1)  Q2: A0(v+2)  Q3: B0(v+2)          (BAL = false)
//   Q0: B1(v+1)  Q1: A1(v+1)  Q2: B0(v+2)  Q3: A0(v+2)          (BAL = true)
// VM = vmcnt after the issue (8 in steady state: retires the half-tile
// issued four phases earlier); STAGE = whether the phase's G exists.
// BAL ("balanced"): fragment reads per phase 8/4/8/4 instead of 12/4/8/0 -
// phase 3 reads the NEXT K-tile's B0 fragments into the register set the
// current tile used for B1, so the two B sets swap roles every K-tile (PAR =
// v & 1; B0(v+1) is staged one phase earlier so it is retired by phase 2).
// Every buffer slot is still restaged >= 2 phases after its last read.
// Returns (DL, phase 3) whether the deadline has passed.
template <bool FP8, bool DL, bool BAL, int Q, int VM, bool STAGE, typename AF, typename BF>
__device__ __forceinline__ bool phase(const Ctx& c, int v, AF& fa, BF& b0r, BF& b1r, f32x4 (&acc)[2][2][4][2],
                                      const Deadline& d, uint64_t& now, bool has_next) {
  // b0r: this K-tile's B0 fragments; b1r: its B1 fragments (BAL: the next
  // K-tile's B0 is read into them in phase 3)
  const char* cur = c.smem + (v & 1) * kBuf;
  if constexpr (Q == 0) {
    if constexpr (!BAL) {
      read_frags<FP8, 2>(cur + kB0 * kHalf, c.wc * 32, c.r16, c.h, b0r);
      __builtin_amdgcn_sched_barrier(0);
    }
    read_frags<FP8, 4>(cur + kA0 * kHalf, c.wr * 64, c.r16, c.h, fa);
  } else if constexpr (Q == 1) {
    read_frags<FP8, 2>(cur + kB1 * kHalf, c.wc * 32, c.r16, c.h, b1r);
  } else if constexpr (Q == 2) {
    read_frags<FP8, 4>(cur + kA1 * kHalf, c.wr * 64, c.r16, c.h, fa);
  } else {
    // The flag write comes first: wave 0 then has no LDS read in flight (phase
    // 2's fragments were consumed by its MFMAs), so the lgkmcnt(0) that
    // completes the write (and the clock read of phase 2) costs the write's
    // own latency only. After the BAL reads below it waited for those 4
    // ds_reads too, once per K-tile in front of the barrier every wave waits
    // at: 27.6 % of wave time waiting vs 20.8 % for the one-shot kernel
    // (profiles/deadline_shapes_r3.md).
    if constexpr (DL) {
      if (d.tid == 0) {
        const uint64_t el = (now - d.t0) & ((1ull << 48) - 1);
        d.flag[v & 1] = el >= d.ticks || el >= d.slice_end;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
    if constexpr (BAL) {
      if (has_next) read_frags<FP8, 2>(c.smem + ((v + 1) & 1) * kBuf + kB0 * kHalf, c.wc * 32, c.r16, c.h, b1r);
    }
  }
  if constexpr (STAGE) {
    if constexpr (Q == 0) stage(c, v + 1, kB1);
    if constexpr (Q == 1) stage(c, v + 1, kA1);
    if constexpr (Q == 2) stage(c, v + 2, BAL ? kB0 : kA0);
    if constexpr (Q == 3) stage(c, v + 2, BAL ? kA0 : kB0);
  }
  wait_vm<VM>();
  raw_barrier();
  // The stop flag is loaded right after the barrier but used only after the
  // MFMA cluster: its LDS latency (and the wait for the prefetch reads issued
  // before the barrier, which the same lgkmcnt covers) hides behind the
  // MFMAs instead of delaying their start once per K-tile.
  int flag = 0;
  if constexpr (DL && Q == 3) flag = d.flag[v & 1];
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_setprio(1);
  if constexpr (Q == 0) mfma_quadrant(acc[0][0], fa, b0r);
  if constexpr (Q == 1) mfma_quadrant(acc[0][1], fa, b1r);
  if constexpr (Q == 2) mfma_quadrant(acc[1][1], fa, b1r);
  if constexpr (Q == 3) mfma_quadrant(acc[1][0], fa, b0r);
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
  // The clock is read at the END of phase 2, once its MFMAs are issued: a
  // scalar-memory read in flight forces every LDS wait behind it to
  // lgkmcnt(0) (they complete out of order), and read at the start of phase 2
  // it made the whole A1 fragment read complete before the phase's first
  // MFMA. Consumed by wave 0 at the start of phase 3 (its latency hides
  // behind the barrier between).
  if constexpr (DL && Q == 2) now = __builtin_amdgcn_s_memrealtime();
  bool stop = false;
  if constexpr (DL && Q == 3) stop = __builtin_amdgcn_readfirstlane(flag) != 0;
  raw_barrier();
  return stop;
}

template <bool FP8, bool DL, bool BAL, int PAR, int V0, int V1, int V2, int V3, bool S01, bool S23>
__device__ __forceinline__ bool ktile(const Ctx& c, int v, Frags<FP8>& f, f32x4 (&acc)[2][2][4][2], const Deadline& d,
                                      bool has_next = true) {
  uint64_t now = 0;
  auto& b0r = (BAL && PAR == 1) ? f.by : f.bx;
  auto& b1r = (BAL && PAR == 1) ? f.bx : f.by;
  phase<FP8, DL, BAL, 0, V0, S01>(c, v, f.a, b0r, b1r, acc, d, now, has_next);
  phase<FP8, DL, BAL, 1, V1, S01>(c, v, f.a, b0r, b1r, acc, d, now, has_next);
  phase<FP8, DL, BAL, 2, V2, S23>(c, v, f.a, b0r, b1r, acc, d, now, has_next);
  return phase<FP8, DL, BAL, 3, V3, S23>(c, v, f.a, b0r, b1r, acc, d, now, has_next);
}

// The last two K-tiles (v = nk-2 stages only tile nk-1, v = nk-1 drains).
template <bool FP8, bool DL, bool BAL, int PAR>
__device__ __forceinline__ bool tail(const Ctx& c, int v, Frags<FP8>& f, f32x4 (&acc)[2][2][4][2], const Deadline& d) {
  if (ktile<FP8, DL, BAL, PAR, 8, 8, 6, 4, true, false>(c, v, f, acc, d)) return true;
  return ktile<FP8, DL, BAL, 1 - PAR, 2, 0, 0, 0, false, false>(c, v + 1, f, acc, d, false);
}

// One 256 x 256 tile of C. Returns false if the deadline stopped it (no
// store; every staged load has been waited for).
template <bool FP8, bool DL, bool BAL, bool UNI = false>
__device__ __forceinline__ bool tile(Ctx& c, const char* __restrict__ A, const char* __restrict__ B,
                                     __bf16* __restrict__ C, int M, int N, int K, int ldc, int b, const Deadline& d,
                                     int GROUP = 8) {
  const int nt_m = M / kT, nt_n = N / kT;
  // GROUP M-tiles share their B panels in L2
  const int per_group = GROUP * nt_n;
  const int first_m = (b / per_group) * GROUP;
  const int gsz = min(nt_m - first_m, GROUP);
  const int tm = first_m + (b % per_group) % gsz;
  const int tn = (b % per_group) / gsz;
  constexpr int esz = FP8 ? 1 : 2;
  c.Ab = A + static_cast<size_t>(tm) * kT * c.lda;
  c.Bb = B + static_cast<size_t>(tn) * kT * c.ldb;
  const int nk = (K * esz) / kRB;  // >= 2 (host checks)
  c.last_kt = UNI ? nk - 1 : 1 << 30;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[qm][qn][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  Frags<FP8> f;

  // Prologue, in the steady-state issue order: A0(0) B0(0) B1(0) A1(0) A0(1) B0(1)
  // (BAL: B0(0) A0(0) B1(0) A1(0) B0(1) A0(1)).
  stage(c, 0, BAL ? kB0 : kA0);
  stage(c, 0, BAL ? kA0 : kB0);
  stage(c, 0, kB1);
  stage(c, 0, kA1);
  stage(c, 1, BAL ? kB0 : kA0);
  stage(c, 1, BAL ? kA0 : kB0);
  wait_vm<8>();  // A0(0), B0(0) landed
  raw_barrier();
  if constexpr (BAL) read_frags<FP8, 2>(c.smem + kB0 * kHalf, c.wc * 32, c.r16, c.h, f.bx);  // B0(0), PAR 0
  if (c.wr == 1) raw_barrier();  // wave row 1 runs one barrier behind

  bool stop = false;
  int v = 0;
  if constexpr (UNI) {
    // One K-tile body for the whole loop (no tail instantiations: less
    // register pressure): the last two K-tiles stage two K-tiles past the
    // end (clamped to the last one: L2 hits, never read), drained below.
    if constexpr (!BAL) {
      for (; v < nk && !stop; ++v) stop = ktile<FP8, DL, false, 0, 8, 8, 8, 8, true, true>(c, v, f, acc, d);
    } else {
      for (; v < nk && !stop; v += 2) {
        stop = ktile<FP8, DL, true, 0, 8, 8, 8, 8, true, true>(c, v, f, acc, d);
        if (!stop) stop = ktile<FP8, DL, true, 1, 8, 8, 8, 8, true, true>(c, v + 1, f, acc, d);
      }
    }
    wait_vm<0>();
  } else if constexpr (!BAL) {
    for (; v < nk - 2 && !stop; ++v) stop = ktile<FP8, DL, false, 0, 8, 8, 8, 8, true, true>(c, v, f, acc, d);
    if (!stop) stop = tail<FP8, DL, false, 0>(c, v, f, acc, d);
  } else {
    // register roles alternate per K-tile: unrolled by two (nk even, host-checked)
    for (; v < nk - 2 && !stop; v += 2) {
      stop = ktile<FP8, DL, true, 0, 8, 8, 8, 8, true, true>(c, v, f, acc, d);
      if (!stop) stop = ktile<FP8, DL, true, 1, 8, 8, 8, 8, true, true>(c, v + 1, f, acc, d);
    }
    if (!stop) stop = tail<FP8, DL, true, 0>(c, v, f, acc, d);
  }
  if (c.wr == 0) raw_barrier();  // re-align the barrier counts of the two rows
  if constexpr (DL) {
    if (stop) {  // partial tile: the stand-in result is not needed
      wait_vm<0>();
      return false;
    }
  }

  // Epilogue: lane holds C[m = .. + r16][n = .. + 4h + 0..3] of each
  // fragment; the j = 0, 1 fragments are adjacent (store_pair.hpp).
  const bool wide = epi::wide_ok(C, ldc);
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = tm * kT + qm * 128 + c.wr * 64 + i * 16 + c.r16;
        const int n = tn * kT + qn * 128 + c.wc * 32;
        epi::store_pair<DL>(C + static_cast<size_t>(m) * ldc + n, acc[qm][qn][i][0], acc[qm][qn][i][1], c.h, wide);
      }
  return true;
}

// DL = false: one launch, grid = tiles. DL = true: persistent stand-in
// compute with the contract of gemm_tn_256_kernel's deadline mode
// (kernels.hip): grid <= resident blocks walks the tiles round-robin and
// stops min(ticks, slice_end) after t0, agreed per epoch through *slot.
template <bool FP8, bool DL, bool BAL = false, bool UNI = false>
__global__ void __launch_bounds__(512, 1)
    gemm_8phase_kernel(const char* __restrict__ A, const char* __restrict__ B, __bf16* __restrict__ C, int M, int N,
                       int K, int lda, int ldb, int ldc, uint64_t* __restrict__ slot, uint32_t epoch, uint64_t ticks,
                       uint64_t slice_end, DlSync sync, int group = 8, const DlTask* __restrict__ prog = nullptr,
                       int ntasks = 0) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf + 16];  // ONE array: staging + deadline flags
  const int tid = threadIdx.x;
  Ctx c;
  c.lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: staging LDS addresses stay scalar
  c.wr = c.w >> 2;  // waves w and w+4 share a SIMD: one per wave row
  c.wc = c.w & 3;
  c.r16 = c.lane & 15;
  c.h = c.lane >> 4;
  c.smem = smem;
  constexpr int esz = FP8 ? 1 : 2;
  c.lda = static_cast<size_t>(lda) * esz;
  c.ldb = static_cast<size_t>(ldb) * esz;
  c.voffA = lane_offset(c.lda, c.w, c.lane);
  c.voffB = lane_offset(c.ldb, c.w, c.lane);
  const int T = (M / kT) * (N / kT);
  Deadline d{0, ticks, slice_end, (lds_flag_t*)(smem + 2 * kBuf), tid};
  if constexpr (!DL) {
    tile<FP8, false, BAL, UNI>(c, A, B, C, M, N, K, ldc, xcd_remap(blockIdx.x, T), d, group);
  } else {
    // one task (prog == nullptr) or the tasks of a program, back to back
    // (epoch: the program's claim protocol, dl::program_seq)
    int round = 0;
    for (int k = 0;; ++k) {
      bool fixed = false;
      if (prog) {
        d.ticks = d.slice_end = prog[k].ticks;  // a uniform (scalar) load: stays in SGPRs
        fixed = d.ticks == 0 && (prog[k].work_rounds | prog[k].tail_kt | prog[k].flags) != 0;
        if (d.ticks == 0 && !fixed) {  // the join task(s), the program's last
          // (two end gates per join task: with more lanes the join is several
          // tasks, the last of which stores the host's done word)
          if (blockIdx.x == 0 && tid == 0)
            for (int j = k; j < ntasks; ++j) dl::join(prog[j].sync);
          return;
        }
      }
      if (tid == 0) {  // only thread 0 reads the clock and decides the stop
        if (prog) {
          const dl::ProgSeq ps = dl::program_seq(prog, k, epoch);
          d.t0 = dl::start_task(slot, ps.seq, ps.ep16, ps.mono, d.ticks, prog[k].sync, ps.it, k > 0).t0;
        } else {
          d.t0 = dl::agree_t0(slot, epoch, ticks, sync);
        }
      }
      if (fixed) {
        // fixed work: work_rounds full tiles, then one tile of tail_kt K-tiles
        // (the deadline never passes: the stop checks compare 48-bit times)
        d.ticks = d.slice_end = 1ull << 48;
        const int rounds = static_cast<int>(prog[k].work_rounds);
        for (int r = 0; r < rounds; ++r, ++round)
          tile<FP8, true, BAL, UNI>(c, A, B, C, M, N, K, ldc, xcd_remap((blockIdx.x + round * gridDim.x) % T, T), d);
        const int tkt = static_cast<int>(prog[k].tail_kt);
        if (tkt > 0) {
          tile<FP8, true, BAL, UNI>(c, A, B, C, M, N, tkt * kRB / esz, ldc,
                                    xcd_remap((blockIdx.x + round * gridDim.x) % T, T), d);
          ++round;
        }
        if (tid == 0) dl::fixed_done(slot, prog[k].sync, prog[k].tend);
        if (k + 1 >= ntasks) return;
        continue;
      }
      if (prog && (prog[k].flags & kTaskGateOnly)) {  // its gates, then its done gate: no tiles
        dl::task_done(prog[k].sync);
        if (k + 1 >= ntasks) return;
        continue;
      }
      while (tile<FP8, true, BAL, UNI>(c, A, B, C, M, N, K, ldc, xcd_remap((blockIdx.x + round * gridDim.x) % T, T),
                                       d))
        ++round;
      ++round;  // the stopped tile's partial work is dropped; the next task starts on the next tile
      if (prog) {
        dl::task_done(prog[k].sync);
        if (k + 1 >= ntasks) return;
      } else {
        dl::task_done(sync);
        return;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Streaming persistent variant (the deadline compute, DL only).
//
// The per-tile kernel above fills the pipeline at the start of every tile
// (six half-tiles staged, the first MFMA waits for two of them) and drains it
// over the last two K-tiles. In the persistent deadline kernel a block runs
// tile after tile, so here the K-tiles of consecutive tiles form ONE stream:
// global K-tile g = r * nk + v of the block's r-th tile, LDS buffer g & 1,
// and the phases of the last two K-tiles of tile r stage K-tiles 0 and 1 of
// tile r + 1 exactly as the steady state would. Right after phase 3 of a
// tile's last K-tile the wave converts and stores its accumulators and zeroes
// them (32 stores per thread), then continues into the next tile's K-tile 0,
// whose half-tiles are already in flight. The 32 stores sit in the in-order
// vmcnt queue between the half-tiles, so that K-tile's four waits count them
// (vmcnt(40) instead of 8; from its successor on the stores are older than
// every half-tile waited for and the count is 8 again). The two counts are a
// uniform branch per phase: a second copy of the K-tile body in the loop
// spills ~160 VGPRs. That branch is why this kernel only pays at short K
// (gemm_tn_8phase_deadline picks it for <= 16 K-tiles).
template <bool FP8>
__device__ __forceinline__ void store_tile(const Ctx& c, __bf16* __restrict__ C, int ldc, int tm, int tn,
                                           f32x4 (&acc)[2][2][4][2]) {
  // This lane's element offset in the tile, made opaque so the compiler
  // cannot hoist the 32 store addresses out of the K-loop (they would stay
  // live across it and spill).
  size_t lane = static_cast<size_t>(c.wr * 64 + c.r16) * ldc + c.wc * 32;
  asm volatile("" : "+v"(lane));
  __bf16* base = C + static_cast<size_t>(tm) * kT * ldc + static_cast<size_t>(tn) * kT + lane;
  const bool wide = epi::wide_ok(C, ldc);
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        epi::store_pair<true>(base + static_cast<size_t>(qm * 128 + i * 16) * ldc + qn * 128, acc[qm][qn][i][0],
                        acc[qm][qn][i][1], c.h, wide);
        acc[qm][qn][i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[qm][qn][i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
}

// Tile coordinates of linear tile index b (GROUP-ed M order, as tile()).
__device__ __forceinline__ void tile_coords(int b, int nt_m, int nt_n, int& tm, int& tn) {
  constexpr int GROUP = 8;
  const int per_group = GROUP * nt_n;
  const int first_m = (b / per_group) * GROUP;
  const int gsz = min(nt_m - first_m, GROUP);
  tm = first_m + (b % per_group) % gsz;
  tn = (b % per_group) / gsz;
}

struct StreamCtx {
  const char* A;
  const char* B;
  int nt_m, nt_n, T, nk;
  // the tile being computed (0) and the next one (1); named, not an array:
  // a runtime-indexed array would live in scratch
  const char *Ab0, *Ab1, *Bb0, *Bb1;
};

// Half-tile `slot` of stream K-tile t (t - base in [0, 2 nk): this tile or the next).
__device__ __forceinline__ void stage_g(const Ctx& c, const StreamCtx& sc, int t, int base, int slot) {
  const int nxt = t - base >= sc.nk;
  const int kt = t - base - nxt * sc.nk;
  const bool isA = slot == kA0 || slot == kA1;
  const int hi = slot == kA1 || slot == kB1;
  const char* ab = nxt ? sc.Ab1 : sc.Ab0;
  const char* bb = nxt ? sc.Bb1 : sc.Bb0;
  const char* src = isA ? ab + static_cast<size_t>(hi) * 128 * c.lda : bb + static_cast<size_t>(hi) * 128 * c.ldb;
  stage_half(src, isA ? c.voffA : c.voffB, isA ? c.lda : c.ldb, kt * kRB, c.smem + (t & 1) * kBuf + slot * kHalf, c.w);
}

// Phase Q of stream K-tile g (g - base = K-tile of the current tile). Same
// body as phase<FP8, true, false, Q, ...> with stream staging.
template <bool FP8, int Q, typename AF, typename BF>
__device__ __forceinline__ bool sphase(const Ctx& c, const StreamCtx& sc, int g, int base, bool after_store, AF& fa,
                                       BF& b0r, BF& b1r, f32x4 (&acc)[2][2][4][2], const Deadline& d, uint64_t& now) {
  const char* cur = c.smem + (g & 1) * kBuf;
  if constexpr (Q == 0) {
    read_frags<FP8, 2>(cur + kB0 * kHalf, c.wc * 32, c.r16, c.h, b0r);
    __builtin_amdgcn_sched_barrier(0);
    read_frags<FP8, 4>(cur + kA0 * kHalf, c.wr * 64, c.r16, c.h, fa);
  } else if constexpr (Q == 1) {
    read_frags<FP8, 2>(cur + kB1 * kHalf, c.wc * 32, c.r16, c.h, b1r);
  } else if constexpr (Q == 2) {
    read_frags<FP8, 4>(cur + kA1 * kHalf, c.wr * 64, c.r16, c.h, fa);
    now = __builtin_amdgcn_s_memrealtime();
  } else {
    if (d.tid == 0) {
      const uint64_t el = (now - d.t0) & ((1ull << 48) - 1);
      d.flag[g & 1] = el >= d.ticks || el >= d.slice_end;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  if constexpr (Q == 0) stage_g(c, sc, g + 1, base, kB1);
  if constexpr (Q == 1) stage_g(c, sc, g + 1, base, kA1);
  if constexpr (Q == 2) stage_g(c, sc, g + 2, base, kA0);
  if constexpr (Q == 3) stage_g(c, sc, g + 2, base, kB0);
  // a uniform branch on the wait count, not a second instance of the whole
  // K-tile body (two bodies in one loop spill ~160 VGPRs)
  if (after_store)
    wait_vm<40>();
  else
    wait_vm<8>();
  raw_barrier();
  bool stop = false;
  if constexpr (Q == 3) stop = __builtin_amdgcn_readfirstlane(d.flag[g & 1]) != 0;
  __builtin_amdgcn_s_setprio(1);
  if constexpr (Q == 0) mfma_quadrant(acc[0][0], fa, b0r);
  if constexpr (Q == 1) mfma_quadrant(acc[0][1], fa, b1r);
  if constexpr (Q == 2) mfma_quadrant(acc[1][1], fa, b1r);
  if constexpr (Q == 3) mfma_quadrant(acc[1][0], fa, b0r);
  __builtin_amdgcn_s_setprio(0);
  raw_barrier();
  return stop;
}

template <bool FP8>
__device__ __forceinline__ bool sktile(const Ctx& c, const StreamCtx& sc, int g, int base, bool after_store,
                                       Frags<FP8>& f, f32x4 (&acc)[2][2][4][2], const Deadline& d) {
  uint64_t now = 0;
  sphase<FP8, 0>(c, sc, g, base, after_store, f.a, f.bx, f.by, acc, d, now);
  sphase<FP8, 1>(c, sc, g, base, after_store, f.a, f.bx, f.by, acc, d, now);
  sphase<FP8, 2>(c, sc, g, base, after_store, f.a, f.bx, f.by, acc, d, now);
  return sphase<FP8, 3>(c, sc, g, base, after_store, f.a, f.bx, f.by, acc, d, now);
}

template <bool FP8>
__global__ void __launch_bounds__(512, 1)
    gemm_8phase_stream_kernel(const char* __restrict__ A, const char* __restrict__ B, __bf16* __restrict__ C, int M,
                              int N, int K, int lda, int ldb, int ldc, uint64_t* __restrict__ slot, uint32_t epoch,
                              uint64_t ticks, uint64_t slice_end, DlSync sync) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf + 16];  // ONE array: staging + deadline flags
  const int tid = threadIdx.x;
  Ctx c;
  c.lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: staging LDS addresses stay scalar
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  c.r16 = c.lane & 15;
  c.h = c.lane >> 4;
  c.smem = smem;
  constexpr int esz = FP8 ? 1 : 2;
  c.lda = static_cast<size_t>(lda) * esz;
  c.ldb = static_cast<size_t>(ldb) * esz;
  c.voffA = lane_offset(c.lda, c.w, c.lane);
  c.voffB = lane_offset(c.ldb, c.w, c.lane);
  Deadline d{0, ticks, slice_end, (lds_flag_t*)(smem + 2 * kBuf), tid};
  if (tid == 0) d.t0 = dl::agree_t0(slot, epoch, ticks, sync);
  StreamCtx sc;
  sc.A = A;
  sc.B = B;
  sc.nt_m = M / kT;
  sc.nt_n = N / kT;
  sc.T = sc.nt_m * sc.nt_n;
  sc.nk = (K * esz) / kRB;  // >= 2 (host checks)
  int tm0, tn0, tm1, tn1;
  int round = 0;
  tile_coords(xcd_remap(blockIdx.x % sc.T, sc.T), sc.nt_m, sc.nt_n, tm0, tn0);
  tile_coords(xcd_remap((blockIdx.x + gridDim.x) % sc.T, sc.T), sc.nt_m, sc.nt_n, tm1, tn1);
  sc.Ab0 = A + static_cast<size_t>(tm0) * kT * c.lda;
  sc.Bb0 = B + static_cast<size_t>(tn0) * kT * c.ldb;
  sc.Ab1 = A + static_cast<size_t>(tm1) * kT * c.lda;
  sc.Bb1 = B + static_cast<size_t>(tn1) * kT * c.ldb;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[qm][qn][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  Frags<FP8> f;

  // Prologue (stream K-tiles 0 and 1), steady-state issue order.
  stage_g(c, sc, 0, 0, kA0);
  stage_g(c, sc, 0, 0, kB0);
  stage_g(c, sc, 0, 0, kB1);
  stage_g(c, sc, 0, 0, kA1);
  stage_g(c, sc, 1, 0, kA0);
  stage_g(c, sc, 1, 0, kB0);
  wait_vm<8>();
  raw_barrier();
  if (c.wr == 1) raw_barrier();  // wave row 1 runs one barrier behind

  int g = 0;     // stream K-tile
  int base = 0;  // stream index of the current tile's K-tile 0
  bool stop = false;
  while (!stop) {
    // K-tile 0 of a tile after the first: the previous tile's 32 stores are in flight
    stop = sktile<FP8>(c, sc, g, base, g == base && base > 0, f, acc, d);
    ++g;
    if (!stop && g == base + sc.nk) {  // tile done: store, advance the tile window
      store_tile<FP8>(c, C, ldc, tm0, tn0, acc);
      base = g;
      ++round;
      tm0 = tm1;
      tn0 = tn1;
      sc.Ab0 = sc.Ab1;
      sc.Bb0 = sc.Bb1;
      tile_coords(xcd_remap((blockIdx.x + (round + 1) * gridDim.x) % sc.T, sc.T), sc.nt_m, sc.nt_n, tm1, tn1);
      sc.Ab1 = A + static_cast<size_t>(tm1) * kT * c.lda;
      sc.Bb1 = B + static_cast<size_t>(tn1) * kT * c.ldb;
    }
  }
  // stopped (partial tile discarded): drain every staged half-tile, re-align the rows
  wait_vm<0>();
  if (c.wr == 0) raw_barrier();
  dl::task_done(sync);
}

}  // namespace

bool gemm_8phase_shape_ok(int M, int N, int K, DType in_t) {
  const size_t esz = dtype_size(in_t);
  return gemm_shape_ok(M, N, K, in_t) && (static_cast<size_t>(K) * esz) / kRB >= 2;
}

void gemm_tn_8phase(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, DType in_t,
                    void* stream) {
  DLNB_REQUIRE(gemm_8phase_shape_ok(M, N, K, in_t), "gemm 8-phase: unsupported shape M=" << M << " N=" << N << " K=" << K);
  const int tiles = (M / kT) * (N / kT);
  const int group = gemm_group();  // M-tiles per L2 group of the tile order (4; DLNB_GEMM_GROUP)
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* a = static_cast<const char*>(A);
  auto* b = static_cast<const char*>(B);
  auto* cc = static_cast<__bf16*>(C);
  const bool even = (static_cast<size_t>(K) * dtype_size(in_t) / kRB) % 2 == 0;
  if (in_t == DType::FP8_E4M3) {
    // fp8: one uniform K-tile body with plain reads (the balanced fp8 build
    // spills under the buffer_load staging, profiles/gemm_bench_r2.md)
    hipLaunchKernelGGL((gemm_8phase_kernel<true, false, false, true>), tiles, 512, 0, st, a, b, cc, M, N, K, lda, ldb,
                       ldc, nullptr, 0u, 0ull, 0ull, DlSync(), group);
  } else if (even) {
    // bf16: balanced fragment reads (unrolled by two K-tiles: even counts)
    hipLaunchKernelGGL((gemm_8phase_kernel<false, false, true>), tiles, 512, 0, st, a, b, cc, M, N, K, lda, ldb, ldc,
                       nullptr, 0u, 0ull, 0ull, DlSync(), group);
  } else {
    hipLaunchKernelGGL((gemm_8phase_kernel<false, false>), tiles, 512, 0, st, a, b, cc, M, N, K, lda, ldb, ldc, nullptr,
                       0u, 0ull, 0ull, DlSync(), group);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) DLNB_THROW("gemm 8-phase launch failed: " << hipGetErrorString(e));
}

// Tile-order group of the per-tile deadline kernels (8; DLNB_DEADLINE_GROUP, A/B knob read per launch).
static int deadline_group() {
  const char* env = std::getenv("DLNB_DEADLINE_GROUP");
  const int g = env ? std::atoi(env) : 0;
  return g > 0 ? g : 8;
}

// The per-tile 8-phase deadline kernel in program mode (bf16, or fp8 K-tiles
// the 4-wave kernel does not take).
bool deadline_program_8phase_ok(int M, int N, int K, DType in_t) {
  // (short-K bf16 too: one launch of its own takes the streaming kernel
  // there, a program the per-tile one - fixed work needs a program for every
  // stand-in shape)
  return gemm_8phase_shape_ok(M, N, K, in_t);
}

void gemm_8phase_deadline_program(const void* A, const void* B, void* C, int M, int N, int K, DType in_t,
                                  const DlTask* tasks, int n, uint64_t* slot, int grid, void* stream, uint32_t epoch) {
  DLNB_REQUIRE(deadline_program_8phase_ok(M, N, K, in_t), "gemm 8-phase deadline program: unsupported shape");
  DLNB_REQUIRE(tasks != nullptr && n > 0 && slot != nullptr && grid > 0, "gemm 8-phase deadline program: bad args");
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* a = static_cast<const char*>(A);
  auto* b = static_cast<const char*>(B);
  auto* cc = static_cast<__bf16*>(C);
  const int nk = static_cast<int>(static_cast<size_t>(K) * dtype_size(in_t) / kRB);
  const DlSync none;
  if (in_t == DType::BF16 && nk % 2 == 0)
    hipLaunchKernelGGL((gemm_8phase_kernel<false, true, true>), grid, 512, 0, st, a, b, cc, M, N, K, K, K, N, slot,
                       epoch, 0ull, 0ull, none, deadline_group(), tasks, n);
  else if (in_t == DType::BF16)
    hipLaunchKernelGGL((gemm_8phase_kernel<false, true>), grid, 512, 0, st, a, b, cc, M, N, K, K, K, N, slot, epoch,
                       0ull, 0ull, none, deadline_group(), tasks, n);
  else
    hipLaunchKernelGGL((gemm_8phase_kernel<true, true, false, true>), grid, 512, 0, st, a, b, cc, M, N, K, K, K, N,
                       slot, epoch, 0ull, 0ull, none, deadline_group(), tasks, n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) DLNB_THROW("gemm 8-phase deadline program launch failed: " << hipGetErrorString(e));
}

void gemm_tn_8phase_deadline(const void* A, const void* B, void* C, int M, int N, int K, DType in_t, uint64_t ticks,
                             uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end,
                             const DlSync& sync) {
  DLNB_REQUIRE(gemm_8phase_shape_ok(M, N, K, in_t), "gemm 8-phase deadline: unsupported shape");
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* a = static_cast<const char*>(A);
  auto* b = static_cast<const char*>(B);
  auto* cc = static_cast<__bf16*>(C);
  // Chosen by shape (profiles/gemm_deadline_stream_r2.md, gemm_bench_r2.md):
  //   bf16, short K (<= 16 K-tiles): the streaming kernel, whose per-tile
  //     pipeline fill / drain savings outweigh its per-phase wait-count
  //     branch only there;
  //   bf16, long K: the per-tile loop, balanced reads when the K-tile count
  //     is even (236 VGPRs, no spills: 1354 vs 1288 TF/s sustained), plain
  //     otherwise;
  //   fp8 (K not a multiple of 256 bytes, else the 4-wave MX kernel runs):
  //     the per-tile loop with one uniform K-tile body (no spills; +7 % at
  //     K = 4096, +24 % at the ViT-H FFN's K = 1280 over the tail
  //     instantiations, +8 % over the streaming kernel).
  const int nk = static_cast<int>(static_cast<size_t>(K) * dtype_size(in_t) / kRB);
  if (in_t == DType::BF16 && nk <= 16) {
    hipLaunchKernelGGL((gemm_8phase_stream_kernel<false>), grid, 512, 0, st, a, b, cc, M, N, K, K, K, N, slot, epoch,
                       ticks, slice_end, sync);
  } else if (in_t == DType::BF16 && nk % 2 == 0) {
    hipLaunchKernelGGL((gemm_8phase_kernel<false, true, true>), grid, 512, 0, st, a, b, cc, M, N, K, K, K, N, slot,
                       epoch, ticks, slice_end, sync, deadline_group());
  } else if (in_t == DType::BF16) {
    hipLaunchKernelGGL((gemm_8phase_kernel<false, true>), grid, 512, 0, st, a, b, cc, M, N, K, K, K, N, slot, epoch,
                       ticks, slice_end, sync, deadline_group());
  } else {
    hipLaunchKernelGGL((gemm_8phase_kernel<true, true, false, true>), grid, 512, 0, st, a, b, cc, M, N, K, K, K, N, slot,
                       epoch, ticks, slice_end, sync, deadline_group());
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) DLNB_THROW("gemm 8-phase deadline launch failed: " << hipGetErrorString(e));
}

}  // namespace kernels
}  // namespace dlnb
