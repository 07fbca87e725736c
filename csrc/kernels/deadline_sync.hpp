// Start-time agreement of the persistent deadline GEMMs (every deadline
// kernel: kernels.hip, gemm_8phase.hip, gemm_4wave_fp8.hip) and of the
// compute programs' fixed-work tasks.
//
// A deadline task's blocks must all stop `ticks` after ONE start time t0.
// Thread 0 of every block calls start_task(); the slot is one 64-byte line
// per compute stream (ComputeEngine, compute.cpp):
//   word 0: {epoch:16 | t0:48}  the published start of the current task
//   word 1: t0 + ticks (48 bit)  the deadline of the stream's last task
//   word 2: the claim: the sequence of the last task whose start was claimed
//   word 3: fixed-work completions (every block adds 1 per fixed-work task;
//           a task is complete on every block when it is a multiple of the
//           grid - the slot is zeroed with the grid fixed per stream)
// The first block of a task claims word 2 with a CAS and decides t0; every
// other block of the task and every later launch of the same task
// (DLNB_GEMM_SLICE_US slices) waits for word 0 to carry the epoch and reads
// t0 back.
//
// Claim sequences: a launch of its own carries an epoch (1..65535, different
// from the slot's previous task: the kernel boundary orders the tasks). A
// program task of a replayed lane graph carries kProgBit | (iteration * 4096
// + index): monotonic over the run, so a block dispatched late (a collective
// held the CUs) that reaches task k after task k+1 was claimed sees a LARGER
// claim, skips task k (kLateBlocks) and goes on - it never CASes the claim
// back and rewrites the line under task k+1, and a block waiting
// for a publish that was overtaken leaves too.
//
// How the claiming block decides t0 (DlSync, dlnb/kernels.hpp):
//   * gates: two-word device gates {seq, time} that a one-wave kernel on a
//     collective's stream raises when the collective is done
//     (kernels::gate_signal; seq = the device's iteration word << 32 | tag).
//     The block spins until each gate carries at least this iteration's seq
//     (the words only grow) and takes the latest time. With per-lane graphs
//     (the runner's lane mode) the gate is the only ordering between the
//     collective and the task: the task's own kernel holds the stream until
//     the collective is done;
//   * chain (!= 0: the most ticks of lateness to absorb): the task continues
//     the stream's previous task, so it starts at max(previous deadline, the
//     latest gate) - a late launch (queue hop, the previous grid's drain) is
//     absorbed, a late collective is not (the start moves to the time its
//     gate was raised, and that wait is what the strategy's timers report as
//     exposed communication). A first block later than that start by more
//     than `chain` ticks starts the task `chain` ticks before it arrived: a
//     longer delay is not a launch hop (a replayed graph can queue a node
//     behind another stream's collective on one hardware queue) and stays in
//     the iteration time instead of being taken out of the compute. Both the
//     absorbed part and the part beyond the cap are counted (DlCounter);
//   * otherwise t0 = the time the gates opened (now, with no gates).
//   * a fixed-work task (no deadline) starts once the program's previous
//     task is complete on every block (word 3) and its gates are up.
// A gate never raised within gate_timeout (a bug, or a peer that died) ends
// the wait: the task starts then and kGateTimeouts counts it, so the report
// shows it (chain_capped.compute_gate_timeouts) and the CUs are released.
// Every wait also polls the host's abort word (DlSync::abort, every 64 polls)
// and gives up when it is up (kAborted); a deadline task whose wait gave up
// that way - or that reads the poisoned iteration word a released pre-armed
// replay carries (kPoisonIter) - ends at once.
// t0 (as a full 64-bit s_memrealtime value) goes to up to two host-mapped
// stamp slots (the strategy's stall timer, the --timeline span).
// Every access is a relaxed agent-scope atomic (coherent across the XCDs'
// L2s) except the gates' acquire loads: the stand-in GEMM reads its own
// operands, never a collective's output, so the gates order time, not data.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dlnb/kernels.hpp"

namespace dlnb {
namespace kernels {
namespace dl {

constexpr uint64_t kMask48 = (1ull << 48) - 1;
constexpr uint64_t kGateTimeoutTicks = 60ull * 100000000ull;  // 60 s at 100 MHz
constexpr uint64_t kProgBit = 1ull << 63;                      // claim sequences of program tasks

// a at or after b on the 48-bit clock (wraps every 32 days at 100 MHz)
__device__ __forceinline__ bool not_before(uint64_t a, uint64_t b) { return ((a - b) & kMask48) < (1ull << 47); }

__device__ __forceinline__ uint64_t ld(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void count(uint64_t* counters, int i, uint64_t v) {
  if (counters) __hip_atomic_fetch_add(counters + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The host's abort word (host-mapped, system scope; nullptr: none).
__device__ __forceinline__ bool abort_up(const uint64_t* abort) {
  return abort && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

__device__ __forceinline__ uint64_t iter_of(const uint64_t* iter) { return iter ? ld(iter) : 0ull; }

// A gate's expected sequence word for iteration `it` (kernels::gate_signal).
__device__ __forceinline__ uint64_t gate_seq_of(uint64_t it, uint32_t tag) { return (it << 32) | tag; }
__device__ __forceinline__ uint64_t gate_seq(const uint64_t* iter, uint32_t tag) { return gate_seq_of(iter_of(iter), tag); }

// Spin until the gate's sequence word reaches `want`: true with *t = the
// time it was raised; false when the wait gave up - at the timeout
// (kGateTimeouts) or on the host's abort (kAborted, *aborted = true) - with
// *t = now.
__device__ __forceinline__ bool wait_gate(const uint64_t* gate, uint64_t want, uint64_t timeout, const DlSync& s,
                                          uint64_t* t, bool* aborted) {
  const uint64_t w0 = now_ticks();
  for (unsigned k = 1;; ++k) {
    if (ld(gate) >= want) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // once, not per poll
      *t = ld(gate + 1) & kMask48;
      return true;
    }
    __builtin_amdgcn_s_sleep(2);
    if ((k & 63u) == 0 && abort_up(s.abort)) {
      count(s.counters, kAborted, 1ull);
      *aborted = true;
      break;
    }
    if (now_ticks() - w0 > timeout) {
      // never raised: give up rather than hold the CUs forever, and count it
      count(s.counters, kGateTimeouts, 1ull);
      break;
    }
  }
  *t = now_ticks() & kMask48;
  return false;
}

// Claim results of claim()
enum : int { kWon = 0, kFollower = 1, kLate = 2 };

__device__ __forceinline__ int claim(uint64_t* w, uint64_t seq, bool mono) {
  uint64_t c = ld(w);
  for (;;) {
    if (c == seq) return kFollower;
    // a program task claimed after this one: this block is late for it
    if (mono && (c & kProgBit) && c > seq) return kLate;
    if (__hip_atomic_compare_exchange_strong(w, &c, seq, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return kWon;
  }
}

struct Start {
  uint64_t t0;  // the task's start (48 bit); a deadline task that must not run gets now - ticks
  bool skip;    // the block does not run the task (late for it, or the wait gave up on the abort)
};

// The start of one task for thread 0 of a block (see the file comment).
//   seq / ep16: claim sequence and the 16-bit epoch the publish carries;
//   mono: program sequences (a larger claim means this block is late);
//   ticks: the deadline (0: a fixed-work task);
//   it: the iteration word's value (kPoisonIter: aborted);
//   wait_prev: a fixed-work task after another task of the same launch
//     (waits until that one is complete on every block).
__device__ __forceinline__ Start start_task(uint64_t* slot, uint64_t seq, uint32_t ep16, bool mono, uint64_t ticks,
                                            const DlSync& s, uint64_t it, bool wait_prev) {
  const bool fixed = ticks == 0;
  const int r = claim(slot + 2, seq, mono);
  if (r == kLate) {
    count(s.counters, kLateBlocks, 1ull);
    return {(now_ticks() - ticks) & kMask48, true};
  }
  const uint64_t gate_timeout = s.gate_timeout ? s.gate_timeout : kGateTimeoutTicks;
  if (r == kFollower) {
    // Every other block waits for the claimer's t0. Poll fast for a few us
    // (the usual case: the claimer decides at once), then back off: 223
    // blocks polling one line every ~64 cycles while the claimer waits for
    // its gate (a compute program's first task, gated on the iteration's
    // first all-gather) slowed that very all-gather 4x (round 5: 0.76 vs
    // 0.19 ms on the headline). Bounded: the claimer's own waits are (two
    // gates and the previous task), and a task overtaken by a later claim or
    // the host's abort ends the wait too.
    const uint64_t w0 = now_ticks();
    uint64_t cur;
    for (unsigned polls = 1; ((cur = ld(slot)) >> 48) != ep16; ++polls) {
      if (polls < 64)
        __builtin_amdgcn_s_sleep(1);
      else
        __builtin_amdgcn_s_sleep(32);
      if ((polls & 63u) == 0) {
        if (mono) {
          const uint64_t c = ld(slot + 2);
          if ((c & kProgBit) && c > seq) {
            count(s.counters, kLateBlocks, 1ull);
            return {(now_ticks() - ticks) & kMask48, true};
          }
        }
        if (abort_up(s.abort)) {
          count(s.counters, kAborted, 1ull);
          return {(now_ticks() - ticks) & kMask48, true};
        }
        if (now_ticks() - w0 > 4 * gate_timeout) {
          count(s.counters, kGateTimeouts, 1ull);
          return {(now_ticks() - ticks) & kMask48, true};
        }
      }
    }
    return {cur & kMask48, false};
  }
  // the claimer
  bool aborted = s.iter != nullptr && it == kPoisonIter;  // a replay the abort released
  if (aborted) count(s.counters, kAborted, 1ull);
  if (fixed && wait_prev && !aborted) {
    // the previous task is complete when every block has added its completion
    const uint32_t grid = gridDim.x;
    const uint64_t w0 = now_ticks();
    for (unsigned k = 1; ld(slot + 3) % grid != 0; ++k) {
      __builtin_amdgcn_s_sleep(1);
      if ((k & 63u) == 0) {
        if (abort_up(s.abort)) {
          count(s.counters, kAborted, 1ull);
          aborted = true;
          break;
        }
        if (now_ticks() - w0 > gate_timeout) {
          count(s.counters, kGateTimeouts, 1ull);
          break;
        }
      }
    }
  }
  uint64_t gate_t = 0;
  bool gated = false;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (!s.gate[i] || aborted) continue;
    uint64_t t;
    wait_gate(s.gate[i], gate_seq_of(it, s.tag[i]), gate_timeout, s, &t, &aborted);
    gate_t = gated && not_before(gate_t, t) ? gate_t : t;
    gated = true;
  }
  const uint64_t raw = now_ticks();
  const uint64_t now = raw & kMask48;
  uint64_t t0 = now;  // unchained: when the gates opened
  if (aborted) {
    t0 = (now - ticks) & kMask48;  // a deadline task ends at once
  } else if (!fixed) {
    const uint64_t prev = s.chain ? ld(slot + 1) & kMask48 : 0;
    if (prev != 0) {  // 0: nothing to continue (the slot was reset)
      t0 = gated && not_before(gate_t, prev) ? gate_t : prev;
      if (!not_before(now, t0)) {
        t0 = now;  // never in the future
      } else {
        const uint64_t late = (now - t0) & kMask48;
        if (late > s.chain) {
          t0 = (now - s.chain) & kMask48;  // absorb at most `chain` ticks of lateness
          count(s.counters, kCappedTasks, 1ull);  // a wait the chain did not hide
          count(s.counters, kCappedTicks, late - s.chain);
        }
        if (late > 0) {
          count(s.counters, kAbsorbedTasks, 1ull);
          count(s.counters, kAbsorbedTicks, late > s.chain ? s.chain : late);
        }
      }
    }
    __hip_atomic_store(slot + 1, (t0 + ticks) & kMask48, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __hip_atomic_store(slot, (static_cast<uint64_t>(ep16) << 48) | t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t full = raw - ((now - t0) & kMask48);
#pragma unroll
  for (int i = 0; i < 2; ++i)
    if (s.tstart[i]) __hip_atomic_store(s.tstart[i], full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return {t0, aborted && !fixed};
}

// The one-launch protocol (gemm_tn_deadline): epoch 1..65535, the kernel
// boundary orders consecutive tasks.
__device__ __forceinline__ uint64_t agree_t0(uint64_t* slot, uint32_t epoch, uint64_t ticks, const DlSync& s) {
  return start_task(slot, epoch, epoch, false, ticks, s, iter_of(s.iter), false).t0;
}

// The task's own done gate (DlSync::done_gate): raised by thread 0 of block 0
// as the kernel leaves (every block stops at the same deadline, so this is the
// end of the task's compute, not of the last block's drain).
__device__ __forceinline__ void task_done(const DlSync& s) {
  if (!s.done_gate || blockIdx.x != 0 || threadIdx.x != 0) return;
  const uint64_t seq = gate_seq(s.iter, s.done_tag);
  __hip_atomic_store(s.done_gate + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(s.done_gate, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// A fixed-work task's completion (thread 0 of every block, once its tiles are
// done): the block that completes the task on the whole grid stores the end
// time into *tend and raises the task's done gate.
__device__ __forceinline__ void fixed_done(uint64_t* slot, const DlSync& s, uint64_t* tend) {
  // (the time is read before the completion is counted: the next task's
  // claimer, which starts once the count completes, never stamps earlier)
  const uint64_t t = __builtin_amdgcn_s_memrealtime();
  const uint64_t old = __hip_atomic_fetch_add(slot + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((old + 1) % gridDim.x != 0) return;
  if (tend) __hip_atomic_store(tend, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (s.done_gate) {
    __hip_atomic_store(s.done_gate + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(s.done_gate, gate_seq(s.iter, s.done_tag), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// A program's join task (DlTask with ticks == 0 and no work, the last of its
// program): thread 0 of block 0 waits for its gates (the other lanes' end
// gates, as a task's gates: bounded, counted, abort-aware) and then stores
// the iteration number into the host's done word (sync.tstart[0]; relaxed,
// system scope) - the whole iteration done, signalled while the kernel still
// runs - and the time into sync.tstart[1] (optional).
__device__ __forceinline__ void join(const DlSync& s) {
  const uint64_t gate_timeout = s.gate_timeout ? s.gate_timeout : kGateTimeoutTicks;
  const uint64_t it = iter_of(s.iter);
  bool aborted = s.iter != nullptr && it == kPoisonIter;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (!s.gate[i] || aborted) continue;
    uint64_t t;
    wait_gate(s.gate[i], gate_seq_of(it, s.tag[i]), gate_timeout, s, &t, &aborted);
  }
  if (s.tstart[0]) __hip_atomic_store(s.tstart[0], it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (s.tstart[1])
    __hip_atomic_store(s.tstart[1], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A program task's claim sequence and publish epoch: from the iteration word
// and the task's index among the stream's program tasks of the iteration
// (DlTask::epoch, < 4096), so consecutive tasks - the last of one replay and
// the first of the next too - always differ and no slot reset is needed
// between replays; epochs 1..32767 (launches of their own take
// 32768..65534, ComputeEngine). `launch_epoch` != 0: a one-task launch with
// that epoch instead (gemm_tn_deadline_program's epoch argument).
struct ProgSeq {
  uint64_t it, seq;
  uint32_t ep16;
  bool mono;
};
__device__ __forceinline__ ProgSeq program_seq(const DlTask* prog, int k, uint32_t launch_epoch) {
  ProgSeq p;
  p.it = iter_of(prog[0].sync.iter);
  if (launch_epoch != 0) {
    p.seq = launch_epoch;
    p.ep16 = launch_epoch;
    p.mono = false;
    return p;
  }
  const uint64_t q = (p.it * 4096ull + prog[k].epoch) & ~kProgBit;
  p.seq = kProgBit | q;
  p.ep16 = static_cast<uint32_t>(q % 32767ull) + 1u;
  p.mono = true;
  return p;
}

}  // namespace dl
}  // namespace kernels
}  // namespace dlnb
