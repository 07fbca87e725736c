// One-wave-per-SIMD MFMA GEMM for gfx950 (bf16): C[M,N] = A[M,K] . B[N,K]^T.
//
// A different point in the design space from the 8-phase ping-pong kernel
// (gemm_8phase.hip, 8 waves = 2 per SIMD, 128 x 64 of C per wave):
//
//   * 4 waves, one per SIMD, each owning a 128 x 128 quadrant of the 256 x 256
//     block tile: 64 accumulator fragments (256 fp32 per lane, all 256 AGPRs),
//     so every A fragment feeds 8 MFMAs and every B fragment 8 (0.25
//     ds_read_b128 per MFMA vs 0.375 for the 128 x 64 wave tile).
//   * The MFMAs are inline asm with the accumulator as a tied "+a" operand:
//     through the builtin, hipcc keeps only part of the accumulators in AGPRs
//     and rotates the rest through VGPRs (~2.5 v_accvgpr moves per MFMA).
//   * The compute unit is a 32-deep K-step (one MFMA K, 64 MFMAs per wave):
//     the wave runs K-step t's MFMAs on fragments read during K-step t-1 and,
//     between them, reads K-step t+1's 16 fragments (pairs 0-15).
//   * Staging is by 64-deep K-tiles of 128-byte rows (one load = 8 full
//     128-B lines) in half-tiles (A0 A1 B0 B1: 128 rows x 128 B = 16 KiB),
//     two K-tiles resident (128 KiB). K-tile T+2 is staged during K-step 2T+1
//     into K-tile T's slots (their last reads were in K-step 2T): 16
//     buffer_load ... lds per wave, one every other MFMA pair. The lane offset
//     of each load is loop-invariant (the K-tile goes in the scalar offset) and
//     the loop runs two K-tiles per iteration, so every LDS address is static:
//     the loop is MFMAs, ds_reads, loads and a few SALU ops. (The first
//     version - global_load_lds with per-lane 64-bit addresses, 64-B rows -
//     spent 30% of the MFMA time on address VALU and issue; probe history in
//     profiles/gemm_bench_r2.md.)
//   * Every K-step ends with the vmcnt wait for what the next one reads,
//     lgkmcnt(0) and ONE barrier.
//   * LDS image per half: row r, 16-B chunk q holds K-chunk q ^ ((r >> 1) & 7)
//     (XOR applied to the per-lane global source offset; LDS-DMA writes
//     lane-linearly), so each 16-lane group of a ds_read_b128 covers all 64
//     banks once (0 bank conflicts measured).
//   * The last K-tiles stage clamped copies of the last K-tile (never read);
//     one vmcnt(0) drains them after the loop.
//
// Variant 5 of dlnb::kernels::gemm_tn (bf16; K a multiple of 64).
#include <hip/hip_runtime.h>

#include "dlnb/kernels.hpp"

namespace dlnb {
namespace kernels {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kT = 256;           // block tile
constexpr int kRB = 128;          // bytes per staged row: 64 bf16 of K
constexpr int kHalf = 128 * kRB;  // one half-tile, 16 KiB

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

__device__ __forceinline__ int xcd_remap(int b, int T) {
  const int q = T / 8, r = T % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * kRB + ((chunk ^ ((row >> 1) & 7)) << 4); }

struct Ctx4 {
  __amdgpu_buffer_rsrc_t ra, rb;  // A / B rows of this block tile as buffer resources
  int voff[2][8];                 // per operand, per staging piece: the lane's byte offset (row * ld + chunk)
  char* smem;
  int w, last_tile;
};

// Half-tile slot h (0 A0, 1 A1, 2 B0, 3 B1) of the K-tile with parity tp.
__device__ __forceinline__ char* slot(const Ctx4& c, int tp, int h) { return c.smem + (tp * 4 + h) * kHalf; }

// Piece p (0..15) of this wave's share of K-tile `tile` (clamped to the last
// one), into the slots of parity tp: half p/4, wave-instruction (p%4)*4 + w
// of its 16 (8 rows x 128 B each). buffer_load ... lds: the lane offset is
// loop-invariant, the K-tile goes in the scalar offset.
__device__ __forceinline__ void stage_piece(const Ctx4& c, int tile, int tp, int p) {
  const int half = p >> 2;
  const int tk = min(tile, c.last_tile);
  const int inst = (p & 3) * 4 + c.w;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(half < 2 ? c.ra : c.rb, (lds_ptr_t)(slot(c, tp, half) + inst * 1024), 16,
                                           c.voff[half >> 1][(half & 1) * 4 + (p & 3)], tk * kRB, 0, 0);
}

// This wave's 16 fragments of one K-step: a[i] = A rows wr*128 + i*16 + r16,
// b[j] = B rows (C columns) wc*128 + j*16 + r16, K chunk 4s + h of the K-tile
// (s = K-step parity). Rows 16 apart share the swizzle phase, so fragment i
// is at the lane's offset plus i * 2 KiB; chunk 4 + h flips offset bit 6.
struct Frag4 {
  bf16x8 a[8], b[8];
};
__device__ __forceinline__ void read_frag(const char* ahalf, const char* bhalf, int off, int g, Frag4& f) {
  if (g < 8)
    f.a[g] = *reinterpret_cast<const bf16x8*>(ahalf + off + g * 2048);
  else
    f.b[g - 8] = *reinterpret_cast<const bf16x8*>(bhalf + off + (g - 8) * 2048);
}

// acc += b . a^T on the matrix core, the accumulator pinned to AGPRs (tied
// "+a" operand). hipcc does not pad hazards inside asm: every reader of an
// accumulator other than the next MFMA of its chain sits behind the pad after
// the loop; the A/B operands come from compiler ds_reads, which hipcc waits
// for.
template <bool ZERO>
__device__ __forceinline__ void mfma(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  if constexpr (ZERO)
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(b), "v"(a));
  else
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// Staging load carried by MFMA pair g (0..31) of an odd K-step: every other
// pair (loads bunched into half of the K-step measured 8-10% slower; spreading
// the fragment reads as well, or dropping the odd K-steps' barrier, changed
// nothing: probe table in profiles/gemm_bench_r2.md).
__device__ constexpr int pair_load(int g) { return (g & 1) ? (g >> 1) : -1; }

// One K-step t, Q = t % 4 (the loop runs four K-steps = two K-tiles per
// iteration, so every LDS address is static): 64 MFMAs on `cur` (i outer, j
// inner) in 32 pairs, pairs 0-15 each carrying one of K-step t+1's fragment
// reads; an odd K-step t = 2T+1 also stages K-tile T+2 (16 loads per wave)
// into the slots of K-tile T, whose last reads were in K-step 2T. The order
// is pinned with sched_barrier. Then the vmcnt wait for what K-step t+1 reads
// (K-tile (t+2)/2, staged two K-steps back: after an odd K-step its own 16
// loads stay in flight, after an even one nothing), lgkmcnt(0) (this wave's
// reads of the slots staged next are done) and the K-step's one barrier.
// FIRST: accumulators start from 0; LAST: no reads, staging or barrier.
template <int Q, bool FIRST, bool LAST>
__device__ __forceinline__ void kstep(const Ctx4& c, int t, int wr, int wc, int off0, int off1, const Frag4& cur,
                                      Frag4& nxt, f32x4 (&acc)[8][8]) {
  constexpr int PAR = Q & 1;
  constexpr int RTP = ((Q + 1) >> 1) & 1;  // parity of K-tile (t+1)/2
  const char* ahalf = slot(c, RTP, wr);
  const char* bhalf = slot(c, RTP, 2 + wc);
  const int roff = PAR ? off0 : off1;  // K-step t+1's parity
#pragma unroll
  for (int g = 0; g < 32; ++g) {
    const int i = g >> 2, j = (g & 3) * 2;
    mfma<FIRST>(acc[i][j], cur.b[j], cur.a[i]);
    mfma<FIRST>(acc[i][j + 1], cur.b[j + 1], cur.a[i]);
    if constexpr (!LAST) {
      if (g < 16) read_frag(ahalf, bhalf, roff, g == 0 ? 0 : g <= 8 ? 7 + g : g - 8, nxt);  // a0, b0..b7, a1..a7
      if constexpr (PAR == 1) {
        const int p = pair_load(g);
        if (p >= 0) stage_piece(c, (t >> 1) + 2, Q >> 1, p);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (!LAST) {
    wait_vm<PAR ? 16 : 0>();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    raw_barrier();
  }
}

__global__ void __launch_bounds__(256, 1)
    gemm_4wave_kernel(const char* __restrict__ A, const char* __restrict__ B, __bf16* __restrict__ C, int M, int N,
                      int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[8 * kHalf];  // 128 KiB, one array
  const int tid = threadIdx.x;
  Ctx4 c;
  const int lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS bases stay scalar
  const int wr = c.w >> 1, wc = c.w & 1;
  const int r16 = lane & 15, h = lane >> 4;
  c.smem = smem;
  const int nt_m = M / kT, nt_n = N / kT, T = nt_m * nt_n;
  const int b = xcd_remap(blockIdx.x, T);
  constexpr int GROUP = 8;
  const int per_group = GROUP * nt_n;
  const int first_m = (b / per_group) * GROUP;
  const int gsz = min(nt_m - first_m, GROUP);
  const int tm = first_m + (b % per_group) % gsz;
  const int tn = (b % per_group) / gsz;
  const int ldab = lda * 2, ldbb = ldb * 2;
  c.ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(A) + static_cast<size_t>(tm) * kT * ldab, 0, 0x7ffffff0,
                                           0x00020000);
  c.rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(B) + static_cast<size_t>(tn) * kT * ldbb, 0, 0x7ffffff0,
                                           0x00020000);
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int li = ((p & 3) * 4 + c.w) * 64 + lane;
    const int r = li >> 3;  // row within the half
    const int q = (li & 7) ^ ((r >> 1) & 7);
    c.voff[0][p] = ((p >> 2) * 128 + r) * ldab + (q << 4);
    c.voff[1][p] = ((p >> 2) * 128 + r) * ldbb + (q << 4);
  }
  const int ns = K / 32;  // K-steps (even: K % 64 == 0, host-checked)
  c.last_tile = ns / 2 - 1;
  const int off0 = swz(r16, h), off1 = off0 ^ 64;

  f32x4 acc[8][8];
  Frag4 f0, f1;

  // K-tiles 0 and 1 (16 loads per wave each); K-tile 0 landed -> read
  // K-step 0; K-tile 1 is waited for at the end of K-step 0.
#pragma unroll
  for (int p = 0; p < 32; ++p) stage_piece(c, p >> 4, p >> 4, p & 15);
  wait_vm<16>();
  raw_barrier();
#pragma unroll
  for (int g = 0; g < 16; ++g) read_frag(slot(c, 0, wr), slot(c, 0, 2 + wc), off0, g, f0);
  kstep<0, true, false>(c, 0, wr, wc, off0, off1, f0, f1, acc);
  int t = 1;
  for (; t <= ns - 5; t += 4) {
    kstep<1, false, false>(c, t, wr, wc, off0, off1, f1, f0, acc);
    kstep<2, false, false>(c, t + 1, wr, wc, off0, off1, f0, f1, acc);
    kstep<3, false, false>(c, t + 2, wr, wc, off0, off1, f1, f0, acc);
    kstep<0, false, false>(c, t + 3, wr, wc, off0, off1, f0, f1, acc);
  }
  if (t < ns - 1) {  // two K-steps left before the last (ns % 4 == 0)
    kstep<1, false, false>(c, t, wr, wc, off0, off1, f1, f0, acc);
    kstep<2, false, false>(c, t + 1, wr, wc, off0, off1, f0, f1, acc);
  }
  kstep<3, false, true>(c, ns - 1, wr, wc, off0, off1, f1, f0, acc);
  wait_vm<0>();  // the clamped staging copies
  // MFMA D -> v_accvgpr_read: the last MFMAs need their wait states before
  // the epilogue reads them (tied, so no reader is hoisted above the pad).
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
               : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]), "+a"(acc[7][4]),
                 "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]));

  // Epilogue: lane holds C[m = .. + r16][n = .. + 4h + 0..3] of each fragment.
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = tm * kT + wr * 128 + i * 16 + r16;
      const int n = tn * kT + wc * 128 + j * 16 + 4 * h;
      const f32x4 a = acc[i][j];
      bf16x4 o;
      o[0] = static_cast<__bf16>(a[0]);
      o[1] = static_cast<__bf16>(a[1]);
      o[2] = static_cast<__bf16>(a[2]);
      o[3] = static_cast<__bf16>(a[3]);
      *reinterpret_cast<bf16x4*>(C + static_cast<size_t>(m) * ldc + n) = o;
    }
}

}  // namespace

bool gemm_4wave_shape_ok(int M, int N, int K, DType in_t) {
  return in_t == DType::BF16 && gemm_shape_ok(M, N, K, in_t) && K % 64 == 0 && K >= 64;
}

void gemm_tn_4wave(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                   void* stream) {
  DLNB_REQUIRE(gemm_4wave_shape_ok(M, N, K, DType::BF16), "gemm 4-wave: unsupported shape M=" << M << " N=" << N
                                                                                           << " K=" << K);
  const int tiles = (M / kT) * (N / kT);
  hipLaunchKernelGGL(gemm_4wave_kernel, tiles, 256, 0, static_cast<hipStream_t>(stream), static_cast<const char*>(A),
                     static_cast<const char*>(B), static_cast<__bf16*>(C), M, N, K, lda, ldb, ldc);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) DLNB_THROW("gemm 4-wave launch failed: " << hipGetErrorString(e));
}

}  // namespace kernels
}  // namespace dlnb
