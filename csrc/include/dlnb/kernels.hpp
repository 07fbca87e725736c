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

// How a deadline task's start is decided (csrc/kernels/deadline_sync.hpp):
// wait for up to two gates (device words a collective's stream raises with
// gate_signal), continue the stream's previous task (chain), and write the
// start to up to two host-mapped stamp slots.
// Counters a deadline task adds to (DlSync::counters, device memory), also
// read by the host (ComputeEngine::chain_counters):
enum DlCounter : int {
  kCappedTasks = 0,    // chained tasks whose first block came later than the absorb cap
  kCappedTicks = 1,    // and the lateness beyond the cap
  kWaitTimeouts = 2,   // gate_wait kernels (a comm lane waiting on a compute gate) that gave up
  kGateTimeouts = 3,   // deadline tasks whose gate wait gave up (agree_t0)
  kAbsorbedTicks = 4,  // lateness chained tasks took out of their own compute (<= the cap each)
  kAbsorbedTasks = 5,  // chained tasks that absorbed any
  kAborted = 6,        // waits (gates, claims, joins, go words) that left because the host raised the abort word
  kLateBlocks = 7,     // program blocks that reached a task after a later task was claimed (skipped it)
  kNumCounters = 8
};
// The iteration word's value after an abort (host_wait stores it instead of
// the iteration when the abort word is up): every deadline task that reads it
// ends at once, every gate wait gives up - a pre-armed replay released by the
// abort runs through without computing or waiting (deadline_sync.hpp).
constexpr uint64_t kPoisonIter = ~0ull;
struct DlSync {
  uint64_t* tstart[2] = {nullptr, nullptr};
  const uint64_t* gate[2] = {nullptr, nullptr};
  uint32_t tag[2] = {0, 0};
  uint32_t chain = 0;  // != 0: continue the stream's previous task, absorbing at most this many ticks of lateness
  uint64_t* counters = nullptr;      // DlCounter words (nullptr: none)
  const uint64_t* iter = nullptr;    // iteration word the gates' sequence numbers carry (nullptr: 0)
  uint64_t gate_timeout = 0;         // ticks a gate wait may last (0: 60 s)
  // A gate the task raises itself when its compute is over (block 0 leaving
  // the kernel, i.e. the deadline passed): the dependent collective's signal
  // without a gate_signal kernel after the task (nullptr: none). Set on the
  // task's last launch only.
  uint64_t* done_gate = nullptr;
  uint32_t done_tag = 0;
  uint32_t pad = 0;
  // Host-mapped abort word (Device::abort_word; nullptr: none): every wait of
  // the task polls it next to what it waits for and gives up once it is
  // non-zero (counted in kAborted); a task whose gate wait saw it ends at once.
  const uint64_t* abort = nullptr;
};
// One task of a compute program (gemm_tn_deadline_program; device memory):
// its start protocol (gates, chain, stamps, done gate) and either
//   * a deadline task: `ticks` of the device clock after its agreed start, or
//   * a fixed-work task (ticks == 0, work_rounds or tail_kt != 0): every block
//     computes work_rounds full 256 x 256 tiles and then one tile of tail_kt
//     K-tiles, however long that takes; it starts once the program's previous
//     task is complete on every block (and its gates are up), the last block
//     to finish stores the end time into *tend and raises the done gate, or
//   * a gate-only task (flags & kTaskGateOnly): the start protocol (its
//     gates), no compute, then its done gate - a wait or an event record of
//     the program's stream between two tasks (ComputeEngine folds them into
//     the program: Device::StreamFold); ticks 1 in a deadline program (the
//     stream's chain continues from when the gates opened), 0 in fixed work;
//   * the join (ticks == 0, no work, no flag): the program's last task (dl::join).
// epoch: the task's index among the stream's program tasks of the iteration.
constexpr uint32_t kTaskGateOnly = 1;
struct DlTask {
  DlSync sync;
  uint64_t ticks = 0;
  uint32_t epoch = 0;
  uint32_t work_rounds = 0;
  uint32_t tail_kt = 0;
  uint32_t flags = 0;
  uint64_t* tend = nullptr;  // fixed-work: end stamp (host-mapped or device memory; nullptr: none)
};
// Device gates: two words {seq, time} in device memory (16-byte aligned).
// seq = iteration << 32 | tag, the iteration read from *iter (the device's
// iteration word, Device::iter_word; nullptr = 0) when the kernel runs: a
// replayed graph repeats its captured tags, and the iteration word (set at
// the head of every replay on every lane) keeps one replay's gates from
// satisfying the next replay's waits, with no reset between them.
// gate_signal: one wave stores the time (s_memrealtime), then seq (release)
// when the stream reaches this point. tag != 0.
void gate_signal(uint64_t* gate, const uint64_t* iter, uint32_t tag, void* stream);
// Fault injection (DLNB_INJECT_FAULT mode=gate): the index-th gate_signal of
// this process (counted from now on, from 0) launches nothing, so whatever
// waits for that gate waits until its timeout - or the host's abort.
void fail_gate_signal(long index);
// One wave waits until the gate carries this iteration's seq for tag (raised
// by gate_signal on another stream), at most timeout ticks; a timeout adds 1
// to *timeouts and lets the stream go on (a wait that can never be satisfied
// - e.g. the raising kernel queued behind this one on the same hardware queue
// - must not hang the GPU).
// The wait gives up as soon as the host-mapped abort word (optional) is up.
// A gate counts as raised once its sequence word is >= the one expected (the
// words only grow within a run: a later replay's raise also satisfies it).
void gate_wait(const uint64_t* gate, const uint64_t* iter, uint32_t tag, uint64_t timeout_ticks, uint64_t* timeouts,
               void* stream, const uint64_t* abort = nullptr);
// One wave stores value into *word (device memory, agent scope): the
// iteration word at the head of a lane.
void set_word(uint64_t* word, uint64_t value, void* stream);
// A probe: does stream a run while a kernel enqueued later on stream b has not?
// (a waits on a word b stores, at most timeout ticks). Returns false when a
// timed out, i.e. both streams feed one hardware queue. Synchronises both.
bool queues_independent(void* a, void* b, uint64_t timeout_ticks);

// Deadline kernels; ticks of the 100 MHz s_memrealtime clock (see
// wallclock_hz()).
// start, start2 (optional, host-mapped): the kernel stores its own start time
// there (s_memrealtime), so stall timers work from the task itself (gap()).
void idle_wait(uint64_t ticks, void* stream, uint64_t* start = nullptr, uint64_t* start2 = nullptr);
void busy_spin(uint64_t ticks, int blocks, void* stream, uint64_t* start = nullptr, uint64_t* start2 = nullptr);
// The deadline clock's rate in Hz: measured against the host's steady clock
// once per process (clock_cal_begin starts the window - the GPU device does
// at creation - and the first wallclock_hz call ends it, sleeping until
// DLNB_CLOCK_CAL_MS (500) have passed; 0 = the attribute's nominal rate).
double wallclock_hz(int device);
double wallclock_hz_nominal(int device);
// The measured rate's uncertainty (ppm: the two readings' standard errors
// over the window); < 0 when the nominal rate is used.
double wallclock_uncertainty_ppm(int device);
void clock_cal_begin(int device);
// One wave stores s_memrealtime into *slot (host-mapped memory) when the
// stream reaches this point.
void stamp(uint64_t* slot, void* stream);
// Host <-> stream handshake words in host-coherent memory (system scope):
// host_signal stores `value`; host_wait holds the stream until *word >= value
// (one wave spinning with s_sleep; after timeout_ticks it gives up and adds
// one to *timeouts, so the stream always drains).
// host_wait also stores iter_value into *iter_out (device memory; optional)
// once released: the pre-armed loop's lane head sets the iteration word.
// With the abort word (optional, host-mapped) up it stops waiting at once,
// stores kPoisonIter into *iter_out and no timeout is counted: what it held
// back runs through without computing or waiting (kernels read the poison).
void host_signal(uint64_t* word, uint64_t value, void* stream);
// *word (host-coherent) = *iter (the device's iteration word) when the stream
// gets here: a lane graph's last node (relaxed: no L2 write-back first).
void lane_done(uint64_t* word, const uint64_t* iter, void* stream);
void host_wait(const uint64_t* word, uint64_t value, uint64_t timeout_ticks, uint64_t* timeouts, void* stream,
               uint64_t* iter_out = nullptr, uint64_t iter_value = 0, const uint64_t* abort = nullptr);
int num_cus(int device);

// GEMM: requires M % 256 == 0, N % 256 == 0, K*elem_size % 128 == 0, leading
// dimensions in elements, 16-byte aligned rows. in_t is BF16 or FP8_E4M3;
// C is always bf16.
bool gemm_shape_ok(int M, int N, int K, DType in_t);
// variant:
//   0 = the default: fp8 5 where it applies (K % 256 == 0), else 6 where it
//       applies (>= 2 K-tiles), else 8; bf16 first the narrow-tile kernel
//       when fewer 256 x 256 tiles than CUs leave some idle (gemm_tn_narrow);
//   5 = one wave per SIMD, 128 x 128 of C per wave, MX MFMA with AGPR
//       accumulators (gemm_4wave_fp8.hip; fp8, K % 256 == 0, or bf16 with two
//       16x16x32 MFMAs per 128-byte K-tile row, K % 128 == 0; the streaming
//       persistent kernel when there are more tiles than CUs, 256 x 32 nf
//       tiles when fewer square tiles than CUs leave some idle);
//   6 = the 8-phase ping-pong schedule, 8 waves (2 per SIMD, 128 x 64 of C
//       each; gemm_8phase.hip; bf16 balanced fragment reads when the K-tile
//       count is even, fp8 one uniform K-tile body; >= 2 K-tiles);
//   8 = 8 waves double-buffered (kernels.hip; bf16 software-pipelined reads):
//       any K, the fallback.
// A variant that does not take a shape falls through to the next that does.
void gemm_tn(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, DType in_t,
             void* stream, int variant = 0);
bool gemm_8phase_shape_ok(int M, int N, int K, DType in_t);
bool gemm_4wave_fp8_shape_ok(int M, int N, int K, DType in_t);
// Tile width 32 nf (nf 3..7, or 8 = the square 256 x 256 tile of the other
// kernels) a one-shot GEMM of an M x N output uses on `cus` CUs: narrower
// tiles when the square ones leave CUs idle - fewer tiles than CUs, or a last
// round at least 10 % short (gemm_4wave_fp8.hip, narrow kernel).
// M-tiles per group of the one-shot GEMMs' tile order (groups walk the N-tiles
// together and share B panels in L2): 4, or DLNB_GEMM_GROUP (read per call).
int gemm_group();
int gemm_narrow_nf(int M, int N, int cus);
// The narrow-tile one-shot GEMM (bf16 or fp8, K * elem_size % 256 == 0); false
// (nothing launched) when gemm_narrow_nf picks the square tile or the shape
// does not fit.
bool gemm_tn_narrow(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                    DType in_t, void* stream);
void gemm_tn_4wave_fp8(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                       void* stream);
// The same one-wave-per-SIMD square kernel for bf16 (K * 2 % 256 == 0).
bool gemm_4wave_shape_ok(int M, int N, int K, DType in_t);
void gemm_tn_4wave_bf16(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                        void* stream);
void gemm_tn_4wave_deadline(const void* A, const void* B, void* C, int M, int N, int K, DType in_t, uint64_t ticks,
                            uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end,
                            const DlSync& sync);
void gemm_tn_4wave_fp8_deadline(const void* A, const void* B, void* C, int M, int N, int K, uint64_t ticks,
                                uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end,
                                const DlSync& sync);
void gemm_tn_8phase(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, DType in_t,
                    void* stream);
void gemm_tn_8phase_deadline(const void* A, const void* B, void* C, int M, int N, int K, DType in_t, uint64_t ticks,
                             uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end,
                             const DlSync& sync);

// Persistent deadline variant (the default stand-in compute): a grid of
// `grid` blocks (<= one per CU: 128 KiB LDS each) walks the M x N tile space
// of C = A.B^T round-robin and stops min(ticks, slice_end) (100 MHz
// s_memrealtime) after t0. t0 is agreed through *slot (a 64-byte line per
// stream): the first block of the first launch of `epoch` (1..65535,
// different from the slot's previous task) claims the task, waits for its
// gates and decides t0 (sync: deadline_sync.hpp); every other block and every
// later launch with the same epoch reads it. A task is one launch by default;
// with DLNB_GEMM_SLICE_US it is issued as several launches (slices) with
// increasing slice_end (compute.cpp; profiles/slice_ab_r3.md).
// Leading dimensions are K, K and N.
// sync.tstart (optional, host-mapped): the claiming block stores the task's
// start (s_memrealtime) there - stall timing without extra kernels.
void gemm_tn_deadline(const void* A, const void* B, void* C, int M, int N, int K, DType in_t, uint64_t ticks,
                      uint64_t* slot, uint32_t epoch, int grid, void* stream, uint64_t slice_end = 0,
                      const DlSync& sync = DlSync());

// A deadline PROGRAM: the tasks of tasks[0..n) (device memory) back to back
// in ONE persistent launch - each task agrees its start exactly like a
// separate gemm_tn_deadline launch (deadline_sync.hpp: gates, chain to the
// previous task's deadline, stamps), runs its tiles until its deadline and
// raises its done gate, then the blocks go on to the next task without
// leaving the kernel. A lane's compute is then one kernel per iteration: no
// kernel boundary (drain, dispatch, fences: 15-30 us per task measured in
// round 5) between two compute tasks, and nothing for a collective's
// one-wave kernels to queue behind at a task boundary. Only where
// deadline_program_ok() (the per-tile 8-phase and one-wave-per-SIMD
// kernels; not the short-K streaming or single-K-tile fallbacks).
// epoch: 0 = the tasks' claim sequence follows the device iteration word
// (programs of a replayed lane graph: sequence = iteration * 4096 + task
// index, monotonic, so a block that reaches a task after a later one was
// claimed skips it - kLateBlocks); otherwise the one-launch epoch protocol of
// gemm_tn_deadline (1..65535, different from the slot's previous task; n must
// be 1): a fixed-work task launched on its own.
bool deadline_program_ok(int M, int N, int K, DType in_t);
void gemm_tn_deadline_program(const void* A, const void* B, void* C, int M, int N, int K, DType in_t,
                              const DlTask* tasks, int n, uint64_t* slot, int grid, void* stream,
                              uint32_t epoch = 0);
// K-tiles (128 bytes of K each) of one 256 x 256 tile of the program kernel
// chosen for this shape, and the granularity of a fixed-work task's tail
// (tail_kt must be a multiple of it, >= 2).
int program_ktiles(int M, int N, int K, DType in_t);
int program_tail_multiple(int M, int N, int K, DType in_t);

// Elementwise "optimizer" stand-in (SGD-momentum on bf16 shards, fp32 math):
// p = p - lr * (m = beta*m + g). Used by the optional --optimizer step.
// end_stamp (optional, host-mapped): the kernel's end time (s_memrealtime),
// stored by its last block; `done` is a zeroed device word it counts blocks
// in (re-armed to 0 by that block).
void sgd_momentum_bf16(void* param, void* mom, const void* grad, size_t n, float lr, float beta, void* stream,
                       uint64_t* end_stamp = nullptr, uint32_t* done = nullptr);

}  // namespace kernels
}  // namespace dlnb
