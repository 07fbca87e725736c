// One-wave-per-SIMD MX-fp8 GEMM for gfx950: C[M,N] (bf16) = A[M,K] . B[N,K]^T,
// A and B OCP fp8 e4m3, unit E8M0 scales (v_mfma_scale_f32_16x16x128_f8f6f4).
//
// Why a 4-wave fp8 kernel: in the 8-phase kernel (gemm_8phase.hip) an fp8
// phase is only 8 MX MFMAs per wave between two barriers, and the waves spend
// 30 % of their time at barriers / waitcnt (PMC at 8192 x 14336 x 4096; the
// MX MFMA runs twice the FLOPs of a bf16 one in the same time, so the
// per-barrier cost doubles relative to compute). Here one K-tile (128 fp8 =
// one MX MFMA K) is 64 MFMAs per wave with two barriers.
//
//   * 4 waves, one per SIMD, 128 x 128 of C per wave: 64 accumulators = all
//     256 AGPRs, MFMAs as inline asm on tied "+a" operands (see
//     gemm_4wave.hip for why).
//   * Fragments: a[i] (A rows wr*128 + 16 i + r16) single-buffered - a[i] of
//     K-tile t+1 is read into a[i]'s registers once row i of K-tile t is done;
//     b[j] double-buffered (two sets alternate per K-tile). 64 + 128 VGPRs.
//     A lane's 32 bytes of K are chunks h and h + 4 of its row (the 8-phase
//     kernel's conflict-free fp8 order).
//   * K-tile t, MFMAs row-major (row i: 8 MFMAs on a[i]):
//       start    vmcnt(8) (B(t+1) landed) + barrier
//       rows 0-3 read B(t+1) into the other B set (16 ds_reads), stage B(t+2)
//                (8 buffer_load ... lds, every other MFMA pair)
//       mid      vmcnt(8) (A(t+1) landed) + lgkmcnt(8) + barrier (every wave's
//                A(t) reads - the last, a[7], in this K-tile's first MFMA pair -
//                are done: A(t+2) may overwrite them)
//       rows 4-7 read A(t+1) (a[0..3] at once, a[4..6] after their rows; a[7]
//                in K-tile t+1's first MFMA pair), stage A(t+2)
//     so every staged operand half has a full K-tile of load latency before
//     its wait, and loads / reads are spread evenly (8 + 16 per half).
//   * LDS: two 64 KiB K-tile buffers of four 128-row half-tiles (A0 A1 B0 B1),
//     the 8-phase kernel's XOR-swizzled image; staging by buffer_load ... lds
//     with loop-invariant lane offsets (K-tile and row block in the scalar
//     offset). Uniform loop: the last K-tiles stage / read clamped copies of
//     the last one (never used) - or, in the streaming kernel, the next
//     tile's first K-tiles.
//   * Kernels: gemm_4wave_fp8_kernel<BF, false> (a block per tile),
//     gemm_4wave_fp8_stream_kernel<BF, false> (persistent, a block's tiles as one
//     K-tile stream; the one-shot default with more tiles than CUs),
//     gemm_4wave_fp8_kernel<BF, true> (the persistent deadline compute stand-in)
//     and gemm_4wave_fp8_stream_kernel<BF, true> (its streaming variant, opt-in);
//     BF = true: bf16 operands in the same byte layout, two 16x16x32 bf16
//     MFMAs per 128-byte K-tile row where fp8 issues one MX MFMA (the same
//     MFMA time per K-tile, the same LDS / staging work: round 4);
//     gemm_4wave_narrow_kernel<NF, BF16> (256 x 32 NF tiles, bf16 or fp8, for
//     outputs whose square tiles would leave CUs idle; see "Narrow-N tiles").
//   * Epilogues store two adjacent fragments per 16-byte store (store_pair.hpp).
//
// Variant 5 of dlnb::kernels::gemm_tn for fp8 (K a multiple of 256 bytes), and
// the narrow-tile path of the default variant for bf16.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "deadline_sync.hpp"
#include "dlnb/kernels.hpp"
#include "store_pair.hpp"

namespace dlnb {
namespace kernels {

namespace {

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kT = 256;           // block tile
constexpr int kRB = 128;          // bytes of K per K-tile row
constexpr int kHalf = 128 * kRB;  // half-tile: 16 KiB
constexpr int kBuf = 4 * kHalf;   // A0 A1 B0 B1

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

struct CtxF {
  __amdgpu_buffer_rsrc_t ra, rb;  // A / B rows of the block tile
  __amdgpu_buffer_rsrc_t ran, rbn;  // the next tile's (streaming kernel; has_next)
  int voffA, voffB;               // lane offset within a staging instruction
  int lda, ldb;                   // bytes
  char* smem;
  int w, last_kt;
  int has_next = 0;  // K-tiles past the last stage the next tile's K-tiles 0, 1 (else clamped copies)
};

// Piece p (0..7) of operand op's (0 A, 1 B) half-tiles of K-tile kt (clamped
// to the last one): half p / 4, this wave's wave-instruction (p % 4) * 4 + w
// (8 rows x 128 B; instruction i covers rows 32 i + 8 w + lane / 8 of the half).
__device__ __forceinline__ void stage_piece(const CtxF& c, int kt, int op, int p) {
  const int half = p >> 2, i = p & 3;
  const bool past = kt > c.last_kt;
  const bool nxt = past && c.has_next;  // the next tile's K-tile kt - nk (same buffer parity: nk even)
  const int tk = nxt ? kt - c.last_kt - 1 : min(kt, c.last_kt);
  const int ld = op ? c.ldb : c.lda;
  char* lds = c.smem + (kt & 1) * kBuf + (op * 2 + half) * kHalf + (i * 4 + c.w) * 1024;
  const __amdgpu_buffer_rsrc_t rs = op ? (nxt ? c.rbn : c.rb) : (nxt ? c.ran : c.ra);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)lds, 16, op ? c.voffB : c.voffA,
                                           tk * kRB + (half * 128 + i * 32) * ld, 0, 0);
}

// The same piece for a K-tile known to be in range (kt <= last_kt, buffer
// parity PAR at compile time): no clamp, no next-tile select, a constant LDS
// buffer - two scalar ops per piece (M0, soffset) instead of a dozen compares
// and selects per K-tile (the main K-loop, ktiles_rest; round 4:
// profiles/gemm_instmix_r4.md measured 38 % more SALU per MFMA than the
// vendor's fp8 kernel, this cut the loop's 67 SALU per K-tile to 32 and gave
// +2-3 % at long K, profiles/gemm_g4_main_r4.md).
template <int PAR>
__device__ __forceinline__ void stage_piece_main(const CtxF& c, int kt, int op, int p) {
  const int half = p >> 2, i = p & 3;
  const int ld = op ? c.ldb : c.lda;
  char* lds = c.smem + PAR * kBuf + (op * 2 + half) * kHalf + (i * 4 + c.w) * 1024;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(op ? c.rb : c.ra, (lds_ptr_t)lds, 16, op ? c.voffB : c.voffA,
                                           kt * kRB + (half * 128 + i * 32) * ld, 0, 0);
}

// One 16-B half of fragment f (rows 16 f + r16 of a half-tile): part 0 = K
// chunk h, part 1 = chunk h + 4 (lane offsets offl / offh).
__device__ __forceinline__ i32x4 read_part(const char* half, int offl, int offh, int f, int part) {
  return *reinterpret_cast<const i32x4*>(half + (part ? offh : offl) + f * 2048);
}

struct FragF {
  i32x4 lo, hi;
  __device__ __forceinline__ i32x8 v() const { return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7); }
};

// acc += b . a^T (MX fp8, unit scales), accumulator pinned to AGPRs. ZERO:
// srcC = 0 (first K-tile).
template <bool ZERO>
__device__ __forceinline__ void mfma(f32x4& acc, const FragF& b, const FragF& a, int scale) {
  const i32x8 bv = b.v(), av = a.v();
  if constexpr (ZERO)
    asm("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0]"
        : "=a"(acc)
        : "v"(bv), "v"(av), "v"(scale));
  else
    asm("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
        : "+a"(acc)
        : "v"(bv), "v"(av), "v"(scale));
}

// bf16 inputs in the same fragment layout (narrow kernel): a lane's K chunks h
// and h + 4 of a 128-byte K-tile row are bf16 K elements 8h..8h+7 and
// 32+8h..32+8h+7, i.e. its operands of the K-tile's two 16x16x32 K-steps.
template <bool ZERO>
__device__ __forceinline__ void mfma_bf16(f32x4& acc, const FragF& b, const FragF& a) {
  if constexpr (ZERO)
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(b.lo), "v"(a.lo));
  else
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b.lo), "v"(a.lo));
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b.hi), "v"(a.hi));
}

// One 32-deep K-step of a bf16 fragment pair (the lo or hi chunks).
template <bool ZERO>
__device__ __forceinline__ void mfma_bf16_step(f32x4& acc, const i32x4& b, const i32x4& a) {
  if constexpr (ZERO)
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(b), "v"(a));
  else
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// Deadline state (DL kernels, the compute stand-in): the clock is read at the
// start of every K-tile and thread 0 writes the stop decision into an LDS flag
// (typed LDS pointer: a generic one becomes a FLAT store that waits vmcnt(0))
// before the K-tile's mid barrier; every wave reads it right after that
// barrier, so all waves leave at the same point. flag[t & 1] is next written
// two K-tiles later, after two more barriers.
typedef __attribute__((address_space(3))) volatile int lds_flag_t;
struct DeadlineF {
  uint64_t t0, ticks, slice_end;
  lds_flag_t* flag;
  int tid;
};

// K-tile t (PAR = t & 1: b[PAR] is this K-tile's B set, b[1 - PAR] receives
// K-tile t+1's). READ7: read this K-tile's a[7] (every K-tile but a tile's
// first, whose fragments the prologue read). Returns (DL) whether the
// deadline has passed; a stopped K-tile has issued every load it would have.
// READ7: read this K-tile's a[7] (false only for a tile whose prologue read
// every fragment). VM < 0 (the streaming kernel's K-tile 0): the two vmcnt
// waits are 63 when after_store (the previous tile's 64 stores are younger
// than the loads waited for and would not fit the counter), else 8 - a
// uniform branch, not a second instantiation of the K-tile body.
// MAIN: t + 2 <= last_kt (stage_piece_main, compile-time buffers).
template <bool BF, int PAR, bool FIRST, bool DL, bool READ7 = !FIRST, int VM = 8, bool MAIN = false>
__device__ __forceinline__ bool ktile(const CtxF& c, int t, int wr, int wc, int offl, int offh, FragF (&a)[8],
                                      FragF (&b)[2][8], f32x4 (&acc)[8][8], int scale, const DeadlineF& d,
                                      bool after_store = false) {
  // PAR == t & 1 (K-tile counts are even); a compile-time buffer when MAIN
  const char* cbuf = c.smem + (MAIN ? PAR : (t & 1)) * kBuf;
  const char* nbuf = c.smem + (MAIN ? 1 - PAR : ((t + 1) & 1)) * kBuf;
  const char* na = nbuf + wr * kHalf;
  const char* nb = nbuf + (2 + wc) * kHalf;
  if (VM >= 0 || !after_store)  // B(t+1) landed (A(t+1) may be in flight)
    wait_vm<(VM >= 0 ? VM : 8)>();
  else
    wait_vm<63>();
  // lgkmcnt(14): this wave's B(t) reads (older than the previous K-tile's 14
  // A parts) are done before any wave restages B(t+2) over them after the
  // barrier; a tile's first K-tile waits for every read before it
  __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | ((FIRST ? 0 : 14) << 8) | (3 << 14));
  raw_barrier();
  bool stop = false;
  uint64_t now = 0;
#pragma unroll
  for (int g = 0; g < 32; ++g) {
    const int i = g >> 2, j = (g & 3) * 2;
    if constexpr (DL) {
      // clock read early (scalar-memory latency hidden behind 8 MFMA pairs);
      // the flag write is followed by exactly 8 LDS reads (pairs 8-15), so the
      // mid wait's lgkmcnt(8) lands it before the barrier
      if (g == 0) now = __builtin_amdgcn_s_memrealtime();
      if (g == 8 && d.tid == 0) {
        const uint64_t el = (now - d.t0) & ((1ull << 48) - 1);
        d.flag[t & 1] = el >= d.ticks || el >= d.slice_end;
      }
    }
    if (g == 16) {
      if (VM >= 0 || !after_store)  // A(t+1) landed (B(t+2) may be in flight)
        wait_vm<(VM >= 0 ? VM : 8)>();
      else
        wait_vm<63>();
      // lgkmcnt(8): this wave's A(t) reads (the last, a[7], in pairs 0-1) are
      // done; the B(t+1) reads of pairs 8-15 may still be in flight (lgkmcnt(0)
      // here stalled on the reads just issued)
      __builtin_amdgcn_s_waitcnt(0xc87f);
      raw_barrier();
      if constexpr (DL) stop = __builtin_amdgcn_readfirstlane(d.flag[t & 1]) != 0;
    }
    if constexpr (BF) {
      // bf16: two 32-deep K-steps per 128-byte K-tile row (lo, hi chunks),
      // together the time of one MX MFMA; the two accumulators alternate so
      // no MFMA waits on the one just issued into the same accumulator (a
      // row's 8 lo K-steps before its 8 hi ones, same-accumulator MFMAs 8
      // apart with no s_nop between them, measured the same, round 4)
      mfma_bf16_step<FIRST>(acc[i][j], b[PAR][j].lo, a[i].lo);
      mfma_bf16_step<FIRST>(acc[i][j + 1], b[PAR][j + 1].lo, a[i].lo);
      mfma_bf16_step<false>(acc[i][j], b[PAR][j].hi, a[i].hi);
      mfma_bf16_step<false>(acc[i][j + 1], b[PAR][j + 1].hi, a[i].hi);
    } else {
      mfma<FIRST>(acc[i][j], b[PAR][j], a[i], scale);
      mfma<FIRST>(acc[i][j + 1], b[PAR][j + 1], a[i], scale);
    }
    // a[7] of THIS K-tile: read here, not right after the MFMA that last read
    // the previous a[7] (its K-tile's A region is restaged only after the mid
    // barrier, which waits for this read)
    if (READ7 && g == 0) a[7].lo = read_part(cbuf + wr * kHalf, offl, offh, 7, 0);
    if (READ7 && g == 1) a[7].hi = read_part(cbuf + wr * kHalf, offl, offh, 7, 1);
    if (g < 16) {
      // B(t+1): fragment g / 2, part g % 2
      if ((g & 1) == 0)
        b[1 - PAR][g >> 1].lo = read_part(nb, offl, offh, g >> 1, 0);
      else
        b[1 - PAR][g >> 1].hi = read_part(nb, offl, offh, g >> 1, 1);
      if (g & 1) {
        if constexpr (MAIN)
          stage_piece_main<PAR>(c, t + 2, 1, g >> 1);
        else
          stage_piece(c, t + 2, 1, g >> 1);
      }
    } else {
      // A(t+1): a[0..1] in pairs 16-19, a[2..3] 20-23, a[4..5] 24-27 (rows 4, 5
      // done), a[6] 28-29 (row 6 done); a[7] in K-tile t+1's first pair
      const int k = g - 16;
      if (k < 14) {
        if ((k & 1) == 0)
          a[k >> 1].lo = read_part(na, offl, offh, k >> 1, 0);
        else
          a[k >> 1].hi = read_part(na, offl, offh, k >> 1, 1);
      }
      if (g & 1) {
        if constexpr (MAIN)
          stage_piece_main<PAR>(c, t + 2, 0, (g - 16) >> 1);
        else
          stage_piece(c, t + 2, 0, (g - 16) >> 1);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return stop;
}

// K-tiles 1 .. nk - 1 of a tile (nk even), after its K-tile 0: the pairs
// whose staging stays inside the tile (t + 3 <= nk - 1) run the clamp-free
// body; the last pair and K-tile keep the general one.
template <bool BF, bool DL>
__device__ __forceinline__ bool ktiles_rest(const CtxF& c, int nk, int wr, int wc, int offl, int offh, FragF (&a)[8],
                                            FragF (&b)[2][8], f32x4 (&acc)[8][8], int scale, const DeadlineF& d,
                                            bool stop) {
  int t = 1;
  for (; t < nk - 3 && !stop; t += 2) {
    stop = ktile<BF, 1, false, DL, true, 8, true>(c, t, wr, wc, offl, offh, a, b, acc, scale, d);
    if (!stop) stop = ktile<BF, 0, false, DL, true, 8, true>(c, t + 1, wr, wc, offl, offh, a, b, acc, scale, d);
  }
  for (; t < nk - 1 && !stop; t += 2) {
    stop = ktile<BF, 1, false, DL>(c, t, wr, wc, offl, offh, a, b, acc, scale, d);
    if (!stop) stop = ktile<BF, 0, false, DL>(c, t + 1, wr, wc, offl, offh, a, b, acc, scale, d);
  }
  if (!stop) stop = ktile<BF, 1, false, DL>(c, nk - 1, wr, wc, offl, offh, a, b, acc, scale, d);
  return stop;
}

// A tile's prologue: stage B(0) A(0) B(1) A(1); once K-tile 0 has landed,
// read all of its fragments (a[], b[0]).
__device__ __forceinline__ void prologue(const CtxF& c, int wr, int wc, int offl, int offh, FragF (&a)[8],
                                         FragF (&b)[2][8]) {
#pragma unroll
  for (int k = 0; k < 32; ++k) stage_piece(c, k >> 4, ((k >> 3) & 1) ^ 1, k & 7);  // kt, op (B first), piece
  wait_vm<16>();
  raw_barrier();
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    a[f].lo = read_part(c.smem + wr * kHalf, offl, offh, f, 0);
    a[f].hi = read_part(c.smem + wr * kHalf, offl, offh, f, 1);
    b[0][f].lo = read_part(c.smem + (2 + wc) * kHalf, offl, offh, f, 0);
    b[0][f].hi = read_part(c.smem + (2 + wc) * kHalf, offl, offh, f, 1);
  }
}

// Convert and store a tile's accumulators: lane holds C[m = .. + r16][n = ..
// + 4h + 0..3] of each fragment. The MFMA D -> v_accvgpr_read wait states
// come first (tied to the last row, so no read is hoisted above them); the
// lane's element offset is made opaque so the 64 store addresses are not
// hoisted out of a tile loop (they would stay live across it and spill).
template <bool NT = false>
__device__ __forceinline__ void store_tile(f32x4 (&acc)[8][8], __bf16* __restrict__ C, int ldc, int tm, int tn, int wr,
                                           int wc, int r16, int h) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
               : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]), "+a"(acc[7][4]),
                 "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]));
  size_t lo = static_cast<size_t>(wr * 128 + r16) * ldc + wc * 128;
  asm volatile("" : "+v"(lo));
  __bf16* base = C + static_cast<size_t>(tm) * kT * ldc + static_cast<size_t>(tn) * kT + lo;
  const bool wide = epi::wide_ok(C, ldc);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; j += 2)
      epi::store_pair<NT>(base + static_cast<size_t>(i * 16) * ldc + j * 16, acc[i][j], acc[i][j + 1], h, wide);
}

// One 256 x 256 tile of C. Returns false if the deadline stopped it (no
// store; every staged load has been waited for).
template <bool BF, bool DL>
__device__ __forceinline__ bool tile4(CtxF& c, const char* __restrict__ A, const char* __restrict__ B,
                                      __bf16* __restrict__ C, int lda, int ldb, int ldc, int K, int tm, int tn,
                                      int lane, const DeadlineF& d) {
  const int wr = c.w >> 1, wc = c.w & 1;
  const int r16 = lane & 15, h = lane >> 4;
  if constexpr (DL) {
    // Tile boundary check: a deadline that passes during the previous tile's
    // epilogue must not cost a whole prologue + first K-tile (measured: 512
    // instead of 500 us per 500-us slice at the ViT-H FFN shape). flag[2] is
    // rewritten only after this tile's last barrier.
    if (d.tid == 0) {
      const uint64_t el = (__builtin_amdgcn_s_memrealtime() - d.t0) & ((1ull << 48) - 1);
      d.flag[2] = el >= d.ticks || el >= d.slice_end;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    raw_barrier();
    if (__builtin_amdgcn_readfirstlane(d.flag[2]) != 0) return false;
  }
  c.ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(A) + static_cast<size_t>(tm) * kT * lda, 0, 0x7ffffff0,
                                           0x00020000);
  c.rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(B) + static_cast<size_t>(tn) * kT * ldb, 0, 0x7ffffff0,
                                           0x00020000);
  const int nk = K / kRB;  // K-tiles (even, >= 2: host-checked)
  c.last_kt = nk - 1;
  const int x = (r16 >> 1) & 7;
  const int offl = r16 * kRB + ((h ^ x) << 4), offh = offl ^ 64;  // chunk h + 4 = offset bit 6 flipped
  int scale = 127;  // E8M0 1.0
  asm volatile("" : "+v"(scale));

  f32x4 acc[8][8];
  FragF a[8], b[2][8];

  prologue(c, wr, wc, offl, offh, a, b);
  bool stop = ktile<BF, 0, true, DL>(c, 0, wr, wc, offl, offh, a, b, acc, scale, d);
  stop = ktiles_rest<BF, DL>(c, nk, wr, wc, offl, offh, a, b, acc, scale, d, stop);
  wait_vm<0>();  // the clamped staging copies (or, stopped, everything in flight)
  // Every wave passes this barrier before the next tile's prologue restages
  // K-tile 1's buffer, whose last reads (the clamped K-tile nk) were this
  // K-tile's; and a stopped block leaves with nothing in flight.
  __builtin_amdgcn_s_waitcnt(0xc07f);
  raw_barrier();
  if constexpr (DL) {
    if (stop) return false;
  }
  store_tile<DL>(acc, C, ldc, tm, tn, wr, wc, r16, h);
  return true;
}

__device__ __forceinline__ void tile_coords(int bid, int nt_m, int nt_n, int group, int& tm, int& tn) {
  const int per_group = group * nt_n;  // group M-tiles share their B panels in L2
  const int first_m = (bid / per_group) * group;
  const int gsz = min(nt_m - first_m, group);
  tm = first_m + (bid % per_group) % gsz;
  tn = (bid % per_group) / gsz;
}

// DL = false: one launch, grid = tiles. DL = true: persistent stand-in
// compute with gemm_tn_deadline's contract (kernels.hip): grid <= resident
// blocks walks the tiles round-robin and stops min(ticks, slice_end) after t0,
// agreed per epoch through *slot.
template <bool BF, bool DL>
__global__ void __launch_bounds__(256, 1)
    gemm_4wave_fp8_kernel(const char* __restrict__ A, const char* __restrict__ B, __bf16* __restrict__ C, int M, int N,
                          int K, int lda, int ldb, int ldc, int group, uint64_t* __restrict__ slot, uint32_t epoch,
                          uint64_t ticks, uint64_t slice_end, DlSync sync, const DlTask* __restrict__ prog = nullptr,
                          int ntasks = 0) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf + 16];  // ONE array: staging + deadline flags
  const int tid = threadIdx.x;
  CtxF c;
  const int lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);
  c.smem = smem;
  c.lda = lda;  // fp8: elements = bytes
  c.ldb = ldb;
  {
    const int r = c.w * 8 + (lane >> 3);  // row within instruction 0 of a half
    const int q = (lane & 7) ^ ((r >> 1) & 7);
    c.voffA = r * lda + (q << 4);
    c.voffB = r * ldb + (q << 4);
  }
  const int nt_m = M / kT, nt_n = N / kT, T = nt_m * nt_n;
  DeadlineF d{0, ticks, slice_end, (lds_flag_t*)(smem + 2 * kBuf), tid};
  int tm, tn;
  if constexpr (!DL) {
    tile_coords(xcd_remap(blockIdx.x, T), nt_m, nt_n, group, tm, tn);
    tile4<BF, false>(c, A, B, C, lda, ldb, ldc, K, tm, tn, lane, d);
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
        // the task's fields are re-read per tile (scalar loads) rather than
        // held across the tile body, which sits at the register limit
        for (int r = 0; r < static_cast<int>(__builtin_nontemporal_load(&prog[k].work_rounds)); ++r, ++round) {
          tile_coords(xcd_remap((blockIdx.x + round * gridDim.x) % T, T), nt_m, nt_n, group, tm, tn);
          tile4<BF, true>(c, A, B, C, lda, ldb, ldc, K, tm, tn, lane, d);
        }
        if (__builtin_nontemporal_load(&prog[k].tail_kt) > 0) {
          tile_coords(xcd_remap((blockIdx.x + round * gridDim.x) % T, T), nt_m, nt_n, group, tm, tn);
          tile4<BF, true>(c, A, B, C, lda, ldb, ldc, static_cast<int>(prog[k].tail_kt) * kRB, tm, tn, lane, d);
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
      for (;; ++round) {
        tile_coords(xcd_remap((blockIdx.x + round * gridDim.x) % T, T), nt_m, nt_n, group, tm, tn);
        if (!tile4<BF, true>(c, A, B, C, lda, ldb, ldc, K, tm, tn, lane, d)) break;
      }
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


// Streaming kernel (persistent: block b computes tiles b, b + grid, ...; DL:
// round-robin over the tile space until the deadline). A block's tiles form
// one K-tile stream: the last two K-tiles of a tile stage the next tile's
// K-tiles 0 and 1 and the last one reads its K-tile-0 fragments, so the next
// tile starts without a prologue (no exposed load latency); the 64
// accumulator stores of a tile sit between its last K-tile and the next
// tile's first, whose waits use vmcnt(63). DL: a stop (decided at a mid
// K-tile barrier, uniform over the block) drains the loads in flight and
// leaves without storing.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const char* base, int tile_row, int ld) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base) + static_cast<size_t>(tile_row) * kT * ld, 0,
                                           0x7ffffff0, 0x00020000);
}

template <bool BF, bool DL>
__global__ void __launch_bounds__(256, 1)
    gemm_4wave_fp8_stream_kernel(const char* __restrict__ A, const char* __restrict__ B, __bf16* __restrict__ C,
                                 int M, int N, int K, int lda, int ldb, int ldc, int group, uint64_t* __restrict__ slot,
                                 uint32_t epoch, uint64_t ticks, uint64_t slice_end, DlSync sync) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf + 16];  // ONE array: staging + deadline flags
  const int tid = threadIdx.x;
  CtxF c;
  const int lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = c.w >> 1, wc = c.w & 1;
  const int r16 = lane & 15, h = lane >> 4;
  c.smem = smem;
  c.lda = lda;
  c.ldb = ldb;
  {
    const int r = c.w * 8 + (lane >> 3);
    const int q = (lane & 7) ^ ((r >> 1) & 7);
    c.voffA = r * lda + (q << 4);
    c.voffB = r * ldb + (q << 4);
  }
  const int nt_m = M / kT, nt_n = N / kT, T = nt_m * nt_n;
  const int G = gridDim.x;
  DeadlineF d{0, ticks, slice_end, (lds_flag_t*)(smem + 2 * kBuf), tid};
  if constexpr (DL) {
    if (tid == 0) d.t0 = dl::agree_t0(slot, epoch, ticks, sync);  // only thread 0 reads the clock
  }
  // one-shot: grid <= T (host), the stream ends after the block's last tile;
  // DL: tile indices wrap, the stream never ends before the deadline
  int cur = DL ? blockIdx.x % T : blockIdx.x;
  auto next_of = [&](int t) { return DL ? (t + G) % T : t + G; };
  int tm, tn, tmn = 0, tnn = 0;
  tile_coords(xcd_remap(cur, T), nt_m, nt_n, group, tm, tn);
  c.ra = rows_rsrc(A, tm, lda);
  c.rb = rows_rsrc(B, tn, ldb);
  c.has_next = DL || next_of(cur) < T;
  if (c.has_next) {
    tile_coords(xcd_remap(next_of(cur), T), nt_m, nt_n, group, tmn, tnn);
    c.ran = rows_rsrc(A, tmn, lda);
    c.rbn = rows_rsrc(B, tnn, ldb);
  }
  const int nk = K / kRB;  // even, >= 2
  c.last_kt = nk - 1;
  const int x = (r16 >> 1) & 7;
  const int offl = r16 * kRB + ((h ^ x) << 4), offh = offl ^ 64;
  int scale = 127;
  asm volatile("" : "+v"(scale));

  f32x4 acc[8][8];
  FragF a[8], b[2][8];

  prologue(c, wr, wc, offl, offh, a, b);
  bool first = true, stop = false;
  for (;;) {
    // (the first tile re-reads the a[7] its prologue read: same data)
    stop = ktile<BF, 0, true, DL, true, -1>(c, 0, wr, wc, offl, offh, a, b, acc, scale, d, !first);
    stop = ktiles_rest<BF, DL>(c, nk, wr, wc, offl, offh, a, b, acc, scale, d, stop);
    if (DL && stop) break;  // partial tile: the stand-in result is not needed
    store_tile<DL>(acc, C, ldc, tm, tn, wr, wc, r16, h);
    if (!c.has_next) break;
    // advance the stream: the next tile's K-tiles 0, 1 are staged, its K-tile-0
    // fragments (but a[7]) read
    cur = next_of(cur);
    tm = tmn;
    tn = tnn;
    c.ra = c.ran;
    c.rb = c.rbn;
    c.has_next = DL || next_of(cur) < T;
    if (c.has_next) {
      tile_coords(xcd_remap(next_of(cur), T), nt_m, nt_n, group, tmn, tnn);
      c.ran = rows_rsrc(A, tmn, lda);
      c.rbn = rows_rsrc(B, tnn, ldb);
    }
    first = false;
  }
  wait_vm<0>();  // the clamped / next-tile staging still in flight
  if constexpr (DL) dl::task_done(sync);
}

// ---------------------------------------------------------------------------
// Narrow-N tiles (one-shot only): 256 x 32·NF of C per block, 128 x 16·NF per
// wave (acc[8][NF] AGPRs), NF in 3..7.
//
// A 256 x 256 tile grid quantises badly on skinny outputs: the ViT-H / GPT-2-L
// FFN down projection (M = 8192 tokens, N = 1280, the C5 stand-in shape) is
// 160 tiles for 256 CUs, so 96 CUs idle for the whole launch. 256 x 160 tiles
// make it exactly 256 (the host picks NF by makespan, gemm_tn_4wave_fp8).
// Same K-tile structure as ktile() above, with the MFMA stream of a K-tile
// (8 rows x NF) and the per-K-tile work laid out by MFMA index m (H = 4 NF
// MFMAs per half):
//   first half   after every odd m: one 16-B part of B(t+1) (2 NF parts); after
//                m = 4p + 3: B(t+2) piece p (NF pieces, 8 rows each: the B tile
//                is 32 NF rows = 4 NF wave-instructions, instruction 4p + w
//                from wave w); after m = 1, 3 (, 5, 7): this K-tile's late
//                row(s) a[7] (NF = 3: a[6], a[7]), read from its own buffer
//   mid          vmcnt(NF) (A(t+1) landed; B(t+2) in flight) + lgkmcnt + barrier
//   second half  A(t+1) parts of the other rows (a[i]'s at least two MFMAs
//                after row i's last, a_part_slot; at NF = 3 row 6 ends too late
//                for that, hence two late rows) and the 8 A(t+2) pieces
// LDS per K-tile buffer: A0 A1 (the 128-row halves, as above) then the B rows
// (32 NF x 128 B); the XOR swizzle phase of a B row is that of its row within
// its 16-row fragment, so the lane offsets offl / offh are the square
// kernel's.
template <int NF>
struct Narrow {
  static constexpr int kB = 2 * kHalf;              // B rows' offset in a buffer
  static constexpr int kBufN = 2 * kHalf + 32 * NF * kRB;  // bytes per K-tile buffer
  static constexpr int kM = 8 * NF;                 // MFMAs per K-tile per wave
  static constexpr int kH = 4 * NF;
  static constexpr int kLate = NF == 3 ? 2 : 1;  // rows read at the start of their own K-tile
  static constexpr int kEarly = 2 * (8 - kLate);  // A parts read in the previous K-tile
  // MFMA index after which part k (0..kEarly-1) of a[k / 2] is read
  static constexpr int a_part_slot(int k) {
    int m = kH - 1;
    for (int q = 0; q <= k; ++q) {
      const int earliest = ((q >> 1) + 1) * NF + 1;  // two MFMAs after row q / 2's last
      m = (m + 1 > earliest) ? m + 1 : earliest;
    }
    return m;
  }
  static_assert(NF >= 3 && NF <= 7, "narrow tile: NF 3..7");
  static_assert(a_part_slot(kEarly - 1) < kM, "A(t+1) reads must fit the K-tile");
};

template <int NF>
__device__ __forceinline__ void stage_piece_n(const CtxF& c, int kt, int op, int p) {
  const int tk = min(kt, c.last_kt);  // past the last K-tile: clamped copies, never read
  char* buf = c.smem + (kt & 1) * Narrow<NF>::kBufN;
  if (op == 0) {  // A: half p / 4, instruction (p % 4) * 4 + w
    const int half = p >> 2, i = p & 3;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(c.ra, (lds_ptr_t)(buf + half * kHalf + (i * 4 + c.w) * 1024), 16,
                                             c.voffA, tk * kRB + (half * 128 + i * 32) * c.lda, 0, 0);
  } else {  // B: instruction 4p + w = rows 32p + 8w .. +7
    __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rb, (lds_ptr_t)(buf + Narrow<NF>::kB + (p * 4 + c.w) * 1024), 16,
                                             c.voffB, tk * kRB + p * 32 * c.ldb, 0, 0);
  }
}

template <int NF, bool BF16, int PAR, bool FIRST, bool READ7 = !FIRST>
__device__ __forceinline__ void ktile_n(const CtxF& c, int t, int wr, int wc, int offl, int offh, FragF (&a)[8],
                                        FragF (&b)[2][NF], f32x4 (&acc)[8][NF], int scale) {
  using NW = Narrow<NF>;
  const char* ca = c.smem + (t & 1) * NW::kBufN + wr * kHalf;
  const char* nbuf = c.smem + ((t + 1) & 1) * NW::kBufN;
  const char* na = nbuf + wr * kHalf;
  const char* nb = nbuf + NW::kB + wc * NF * 2048;
  // B(t+1) landed (A(t+1) may be in flight); lgkmcnt(kEarly): the previous
  // K-tile's B reads (older than its kEarly A parts) are done before any wave
  // restages their region (the first K-tile: every prologue read, whose B(0)
  // reads are its youngest)
  __builtin_amdgcn_s_waitcnt((8 & 15) | (7 << 4) | ((FIRST ? 0 : NW::kEarly) << 8));
  raw_barrier();
#pragma unroll
  for (int m = 0; m < NW::kM; ++m) {
    const int i = m / NF, j = m % NF;
    if (m == NW::kH) {
      wait_vm<NF>();  // A(t+1) landed (B(t+2) in flight)
      // this wave's late-row reads (the K-tile's first LDS reads) are done: at
      // most the 2 NF - 2 kLate + 1 B parts issued after the last are in flight
      constexpr int lg = 2 * NF - 2 * NW::kLate + 1 < 8 ? 2 * NF - 2 * NW::kLate + 1 : 8;
      __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (lg << 8) | (3 << 14));
      raw_barrier();
    }
    if constexpr (BF16)
      mfma_bf16<FIRST>(acc[i][j], b[PAR][j], a[i]);
    else
      mfma<FIRST>(acc[i][j], b[PAR][j], a[i], scale);
    if (m < NW::kH) {
      if (READ7 && (m & 1) && (m >> 1) < 2 * NW::kLate) {  // late row 8 - kLate + r / 2, half r % 2
        const int r = m >> 1, row = 8 - NW::kLate + (r >> 1);
        if (r & 1)
          a[row].hi = read_part(ca, offl, offh, row, 1);
        else
          a[row].lo = read_part(ca, offl, offh, row, 0);
      }
      if (m & 1) {
        const int k = m >> 1;  // B(t+1) part k: fragment k / 2, half k % 2
        if (k & 1)
          b[1 - PAR][k >> 1].hi = read_part(nb, offl, offh, k >> 1, 1);
        else
          b[1 - PAR][k >> 1].lo = read_part(nb, offl, offh, k >> 1, 0);
      }
      if ((m & 3) == 3) stage_piece_n<NF>(c, t + 2, 1, m >> 2);
    } else {
#pragma unroll
      for (int k = 0; k < NW::kEarly; ++k)
        if (NW::a_part_slot(k) == m) {
          if (k & 1)
            a[k >> 1].hi = read_part(na, offl, offh, k >> 1, 1);
          else
            a[k >> 1].lo = read_part(na, offl, offh, k >> 1, 0);
        }
      const int s = m - NW::kH;  // A(t+2) piece p after MFMA kH + floor(p kH / 8)
#pragma unroll
      for (int p = 0; p < 8; ++p)
        if (s == (p * NW::kH) / 8) stage_piece_n<NF>(c, t + 2, 0, p);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int NF, bool BF16>
__global__ void __launch_bounds__(256, 1)
    gemm_4wave_narrow_kernel(const char* __restrict__ A, const char* __restrict__ B, __bf16* __restrict__ C,
                                 int M, int N, int K, int lda, int ldb, int ldc, int group) {
  using NW = Narrow<NF>;
  __shared__ __attribute__((aligned(16))) char smem[2 * NW::kBufN];
  const int tid = threadIdx.x;
  CtxF c;
  const int lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = c.w >> 1, wc = c.w & 1;
  const int r16 = lane & 15, h = lane >> 4;
  c.smem = smem;
  constexpr int esz = BF16 ? 2 : 1;
  lda *= esz;  // bytes from here on
  ldb *= esz;
  c.lda = lda;
  c.ldb = ldb;
  {
    const int r = c.w * 8 + (lane >> 3);
    const int q = (lane & 7) ^ ((r >> 1) & 7);
    c.voffA = r * lda + (q << 4);
    c.voffB = r * ldb + (q << 4);
  }
  constexpr int TN = 32 * NF;
  const int nt_m = M / kT, nt_n = N / TN, T = nt_m * nt_n;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, T), nt_m, nt_n, group, tm, tn);
  c.ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(A) + static_cast<size_t>(tm) * kT * lda, 0, 0x7ffffff0,
                                           0x00020000);
  c.rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(B) + static_cast<size_t>(tn) * TN * ldb, 0, 0x7ffffff0,
                                           0x00020000);
  const int nk = K * esz / kRB;  // even, >= 2 (host-checked)
  c.last_kt = nk - 1;
  const int x = (r16 >> 1) & 7;
  const int offl = r16 * kRB + ((h ^ x) << 4), offh = offl ^ 64;
  int scale = 127;  // E8M0 1.0
  asm volatile("" : "+v"(scale));

  f32x4 acc[8][NF];
  FragF a[8], b[2][NF];

  // Prologue: B(0) A(0) B(1) A(1), then K-tile 0's fragments.
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
    for (int p = 0; p < NF; ++p) stage_piece_n<NF>(c, kt, 1, p);
#pragma unroll
    for (int p = 0; p < 8; ++p) stage_piece_n<NF>(c, kt, 0, p);
  }
  wait_vm<NF + 8>();
  raw_barrier();
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    a[f].lo = read_part(smem + wr * kHalf, offl, offh, f, 0);
    a[f].hi = read_part(smem + wr * kHalf, offl, offh, f, 1);
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    b[0][f].lo = read_part(smem + NW::kB + wc * NF * 2048, offl, offh, f, 0);
    b[0][f].hi = read_part(smem + NW::kB + wc * NF * 2048, offl, offh, f, 1);
  }

  ktile_n<NF, BF16, 0, true>(c, 0, wr, wc, offl, offh, a, b, acc, scale);
  for (int t = 1; t < nk - 1; t += 2) {
    ktile_n<NF, BF16, 1, false>(c, t, wr, wc, offl, offh, a, b, acc, scale);
    ktile_n<NF, BF16, 0, false>(c, t + 1, wr, wc, offl, offh, a, b, acc, scale);
  }
  ktile_n<NF, BF16, 1, false>(c, nk - 1, wr, wc, offl, offh, a, b, acc, scale);
  wait_vm<0>();  // the clamped staging copies

  // MFMA D -> v_accvgpr_read wait states, tied to the last row (no read hoisted above)
#pragma unroll
  for (int j = 0; j < NF; ++j) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(acc[7][j]));
  size_t lo = static_cast<size_t>(wr * 128 + r16) * ldc + wc * 16 * NF;
  asm volatile("" : "+v"(lo));
  __bf16* base = C + static_cast<size_t>(tm) * kT * ldc + static_cast<size_t>(tn) * TN + lo;
  const bool wide = epi::wide_ok(C, ldc);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j + 1 < NF; j += 2)
      epi::store_pair(base + static_cast<size_t>(i * 16) * ldc + j * 16, acc[i][j], acc[i][j + 1], h, wide);
    if constexpr (NF & 1) epi::store_one(base + static_cast<size_t>(i * 16) * ldc + (NF - 1) * 16, acc[i][NF - 1], h);
  }
}

}  // namespace

bool gemm_4wave_fp8_shape_ok(int M, int N, int K, DType in_t) {
  return in_t == DType::FP8_E4M3 && gemm_shape_ok(M, N, K, in_t) && K % 256 == 0 && K >= 256;
}

int gemm_group() {
  const char* env = std::getenv("DLNB_GEMM_GROUP");
  const int g = env ? std::atoi(env) : 0;
  return g > 0 ? g : 4;
}

int gemm_narrow_nf(int M, int N, int cus) {
  // Tile width 32 nf: the fewest rounds of tile work per CU, ceil(tiles / CUs)
  // x nf (a tile's time ~ its width), ties to the wider tile. Fewer square
  // tiles than CUs: any saving (they idle CUs for the whole launch); more: a
  // saving of at least 10 % (a partial last round - 640 square tiles are 2.5
  // rounds, 1024 of 256 x 160 exactly 4 - against the square kernels' higher
  // reuse and, fp8, the streaming kernel). DLNB_GEMM_NARROW_NF=8 pins the
  // square tile (A/B), 3-7 forces a width where it divides N. Read on every
  // call (a getenv per GEMM launch is negligible), so an A/B in one process
  // can change it between launches.
  const char* env = std::getenv("DLNB_GEMM_NARROW_NF");
  const int forced = env ? std::atoi(env) : 0;
  if (forced >= 3 && forced <= 8) return (forced == 8 || N % (32 * forced) == 0) ? forced : 8;
  const long sq = static_cast<long>(M / kT) * (N / kT);
  const long sq_cost = (sq + cus - 1) / cus * 8;
  int best = 8;
  long best_cost = sq_cost;
  for (int nf = 7; nf >= 3; --nf) {
    if (N % (32 * nf) != 0) continue;
    const long t = static_cast<long>(M / kT) * (N / (32 * nf));
    const long cost = (t + cus - 1) / cus * nf;
    if (cost < best_cost) {
      best = nf;
      best_cost = cost;
    }
  }
  if (sq >= cus && best_cost * 10 > sq_cost * 9) return 8;
  return best;
}

bool gemm_tn_narrow(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                    DType in_t, void* stream) {
  static const int cus = [] {
    int dev = 0;
    return hipGetDevice(&dev) == hipSuccess ? num_cus(dev) : 256;
  }();
  const size_t kbytes = static_cast<size_t>(K) * dtype_size(in_t);
  if (!gemm_shape_ok(M, N, K, in_t) || kbytes % 256 != 0) return false;  // an even K-tile count
  const int nf = gemm_narrow_nf(M, N, cus);
  if (nf == 8) return false;
  const int group = gemm_group();
  const int nt = (M / kT) * (N / (32 * nf));
  auto* a = static_cast<const char*>(A);
  auto* b = static_cast<const char*>(B);
  auto* cc = static_cast<__bf16*>(C);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool bf = in_t == DType::BF16;
#define DLNB_NARROW(NF)                                                                                     \
  if (bf)                                                                                                   \
    hipLaunchKernelGGL((gemm_4wave_narrow_kernel<NF, true>), nt, 256, 0, st, a, b, cc, M, N, K, lda, ldb, ldc, \
                       group);                                                                              \
  else                                                                                                      \
    hipLaunchKernelGGL((gemm_4wave_narrow_kernel<NF, false>), nt, 256, 0, st, a, b, cc, M, N, K, lda, ldb, ldc, group)
  switch (nf) {
    case 7: DLNB_NARROW(7); break;
    case 3: DLNB_NARROW(3); break;
    case 4: DLNB_NARROW(4); break;
    case 5: DLNB_NARROW(5); break;
    default: DLNB_NARROW(6); break;
  }
#undef DLNB_NARROW
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) DLNB_THROW("gemm narrow-tile launch failed: " << hipGetErrorString(e));
  return true;
}

namespace {

// The square one-wave-per-SIMD kernels for either dtype: strides and K go in
// as bytes (the staging and K-tile arithmetic work in bytes; bf16 runs two
// 32-deep MFMAs per 128-byte K-tile row where fp8 runs one 128-deep MX MFMA).
template <bool BF>
void launch_4wave(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, void* stream) {
  constexpr int esz = BF ? 2 : 1;
  const int tiles = (M / kT) * (N / kT);
  // M-tiles sharing B panels in L2: 4 (round 4, profiles/gemm_group_r4.md: 3 / 4 / 6 / 8 interleaved - 4 at or
  // above 8 on every fp8 shape, +9 % at short K, where 8 re-read 15-37 % more operand panels from HBM than the
  // vendor). DLNB_GEMM_GROUP overrides (A/B, read per launch).
  const int group = gemm_group();
  // more tiles than CUs: the streaming persistent kernel, one block per CU
  // (+1-5 %, profiles/gemm_bench_r2.md); else a block per tile
  static const int cus = [] {
    int dev = 0;
    return hipGetDevice(&dev) == hipSuccess ? num_cus(dev) : 256;
  }();
  auto* a = static_cast<const char*>(A);
  auto* b = static_cast<const char*>(B);
  auto* c = static_cast<__bf16*>(C);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (tiles > cus)
    hipLaunchKernelGGL((gemm_4wave_fp8_stream_kernel<BF, false>), cus, 256, 0, st, a, b, c, M, N, K * esz,
                       lda * esz, ldb * esz, ldc, group, nullptr, 0u, 0ull, 0ull, DlSync());
  else
    hipLaunchKernelGGL((gemm_4wave_fp8_kernel<BF, false>), tiles, 256, 0, st, a, b, c, M, N, K * esz, lda * esz,
                       ldb * esz, ldc, group, nullptr, 0u, 0ull, 0ull, DlSync());
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) DLNB_THROW("gemm 4-wave launch failed: " << hipGetErrorString(e));
}

}  // namespace

bool gemm_4wave_shape_ok(int M, int N, int K, DType in_t) {
  const size_t kb = static_cast<size_t>(K) * dtype_size(in_t);
  return gemm_shape_ok(M, N, K, in_t) && kb % 256 == 0 && kb >= 256;
}

void gemm_tn_4wave_fp8(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                       void* stream) {
  DLNB_REQUIRE(gemm_4wave_fp8_shape_ok(M, N, K, DType::FP8_E4M3),
               "gemm 4-wave fp8: unsupported shape M=" << M << " N=" << N << " K=" << K);
  // A narrower tile when it saves rounds of tile work: fewer square tiles than
  // CUs (the ViT-H FFN down projection 8192 x 1280: 160 square tiles, 256 of
  // 256 x 160) or a partial last round (gemm_narrow_nf).
  if (gemm_tn_narrow(A, B, C, M, N, K, lda, ldb, ldc, DType::FP8_E4M3, stream)) return;
  launch_4wave<false>(A, B, C, M, N, K, lda, ldb, ldc, stream);
}

void gemm_tn_4wave_bf16(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                        void* stream) {
  DLNB_REQUIRE(gemm_4wave_shape_ok(M, N, K, DType::BF16),
               "gemm 4-wave bf16: unsupported shape M=" << M << " N=" << N << " K=" << K);
  launch_4wave<true>(A, B, C, M, N, K, lda, ldb, ldc, stream);
}

void gemm_tn_4wave_deadline(const void* A, const void* B, void* C, int M, int N, int K, DType in_t, uint64_t ticks,
                            uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end,
                            const DlSync& sync) {
  DLNB_REQUIRE(gemm_4wave_shape_ok(M, N, K, in_t) && in_t != DType::FP16,
               "gemm 4-wave deadline: unsupported shape");
  // The per-tile kernel. (Its streaming twin ran +5 % MFMA per clock at a 5 %
  // lower, power-capped clock on the 224 CUs - the same 2620-2630 TF/s - so
  // it was not kept as a deadline kernel: profiles/gemm_deadline_stream_r2.md.)
  const int esz = static_cast<int>(dtype_size(in_t));
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* a = static_cast<const char*>(A);
  auto* b = static_cast<const char*>(B);
  auto* c = static_cast<__bf16*>(C);
  if (in_t == DType::BF16)
    hipLaunchKernelGGL((gemm_4wave_fp8_kernel<true, true>), grid, 256, 0, st, a, b, c, M, N, K * esz, K * esz,
                       K * esz, N, 8, slot, epoch, ticks, slice_end, sync);
  else
    hipLaunchKernelGGL((gemm_4wave_fp8_kernel<false, true>), grid, 256, 0, st, a, b, c, M, N, K, K, K, N, 8, slot,
                       epoch, ticks, slice_end, sync);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) DLNB_THROW("gemm 4-wave deadline launch failed: " << hipGetErrorString(e));
}

void gemm_4wave_deadline_program(const void* A, const void* B, void* C, int M, int N, int K, DType in_t,
                                 const DlTask* tasks, int n, uint64_t* slot, int grid, void* stream, uint32_t epoch) {
  DLNB_REQUIRE(gemm_4wave_shape_ok(M, N, K, in_t) && in_t != DType::FP16,
               "gemm 4-wave deadline program: unsupported shape");
  DLNB_REQUIRE(tasks != nullptr && n > 0 && slot != nullptr && grid > 0, "gemm 4-wave deadline program: bad args");
  const int esz = static_cast<int>(dtype_size(in_t));
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto* a = static_cast<const char*>(A);
  auto* b = static_cast<const char*>(B);
  auto* c = static_cast<__bf16*>(C);
  const DlSync none;
  if (in_t == DType::BF16)
    hipLaunchKernelGGL((gemm_4wave_fp8_kernel<true, true>), grid, 256, 0, st, a, b, c, M, N, K * esz, K * esz,
                       K * esz, N, 8, slot, epoch, 0ull, 0ull, none, tasks, n);
  else
    hipLaunchKernelGGL((gemm_4wave_fp8_kernel<false, true>), grid, 256, 0, st, a, b, c, M, N, K, K, K, N, 8, slot,
                       epoch, 0ull, 0ull, none, tasks, n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) DLNB_THROW("gemm 4-wave deadline program launch failed: " << hipGetErrorString(e));
}

void gemm_tn_4wave_fp8_deadline(const void* A, const void* B, void* C, int M, int N, int K, uint64_t ticks,
                                uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end,
                                const DlSync& sync) {
  DLNB_REQUIRE(gemm_4wave_fp8_shape_ok(M, N, K, DType::FP8_E4M3), "gemm 4-wave fp8 deadline: unsupported shape");
  gemm_tn_4wave_deadline(A, B, C, M, N, K, DType::FP8_E4M3, ticks, slot, epoch, grid, stream, slice_end, sync);
}

}  // namespace kernels
}  // namespace dlnb
