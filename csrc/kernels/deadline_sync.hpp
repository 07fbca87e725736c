// Start-time agreement of the persistent deadline GEMMs (every deadline
// kernel: kernels.hip, gemm_8phase.hip, gemm_4wave_fp8.hip).
//
// A deadline task's blocks must all stop `ticks` after ONE start time t0.
// Thread 0 of every block calls agree_t0(); the slot is one 64-byte line per
// compute stream (ComputeEngine, compute.cpp):
//   word 0: {epoch:16 | t0:48}  the published start of the current task
//   word 1: t0 + ticks (48 bit)  the deadline of the stream's last task
//   word 2: epoch of the last task whose start was claimed
// The first block of a task (epoch = task number on the stream, never 0)
// claims word 2 with a CAS and decides t0; every other block of the task and
// every later launch of the same task (DLNB_GEMM_SLICE_US slices) waits for
// word 0 to carry the epoch and reads t0 back.
//
// How the claiming block decides t0 (DlSync, dlnb/kernels.hpp):
//   * gates: two-word device gates {seq, time} that a one-wave kernel on a
//     collective's stream raises when the collective is done
//     (kernels::gate_signal; seq = the device's iteration word << 32 | tag).
//     The block spins until each gate carries this iteration's seq and takes
//     the latest time. With per-lane graphs (the runner's lane mode) the gate
//     is the only ordering between the collective and the task: the task's
//     own kernel holds the stream until the collective is done;
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
// A gate never raised within gate_timeout (a bug, or a peer that died) ends
// the wait: the task starts then and kGateTimeouts counts it, so the report
// shows it (chain_capped.compute_gate_timeouts) and the CUs are released.
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

// a at or after b on the 48-bit clock (wraps every 32 days at 100 MHz)
__device__ __forceinline__ bool not_before(uint64_t a, uint64_t b) { return ((a - b) & kMask48) < (1ull << 47); }

__device__ __forceinline__ uint64_t ld(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void count(uint64_t* counters, int i, uint64_t v) {
  if (counters) __hip_atomic_fetch_add(counters + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A gate's expected sequence word this iteration (kernels::gate_signal).
__device__ __forceinline__ uint64_t gate_seq(const uint64_t* iter, uint32_t tag) {
  const uint64_t it = iter ? ld(iter) : 0ull;
  return (it << 32) | tag;
}

__device__ __forceinline__ uint64_t agree_t0(uint64_t* slot, uint32_t epoch, uint64_t ticks, const DlSync& s) {
  uint64_t* claim = slot + 2;
  uint64_t c = ld(claim);
  bool won = false;
  while (c != epoch) {
    if (__hip_atomic_compare_exchange_strong(claim, &c, static_cast<uint64_t>(epoch), __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      won = true;
      break;
    }
  }
  if (!won) {
    // Every other block waits for the claimer's t0. Poll fast for a few us
    // (the usual case: the claimer decides at once), then back off: 223
    // blocks polling one line every ~64 cycles while the claimer waits for
    // its gate (a compute program's first task, gated on the iteration's
    // first all-gather) slowed that very all-gather 4x (round 5: 0.76 vs
    // 0.19 ms on the headline).
    uint64_t cur;
    int polls = 0;
    while (((cur = ld(slot)) >> 48) != epoch) {
      if (++polls < 64)
        __builtin_amdgcn_s_sleep(1);
      else
        __builtin_amdgcn_s_sleep(32);
    }
    return cur & kMask48;
  }
  uint64_t gate_t = 0;
  bool gated = false;
  const uint64_t gate_timeout = s.gate_timeout ? s.gate_timeout : kGateTimeoutTicks;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (!s.gate[i]) continue;
    const uint64_t want = gate_seq(s.iter, s.tag[i]);
    uint64_t t;
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      if (__hip_atomic_load(s.gate[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == want) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // once, not per poll
        t = ld(s.gate[i] + 1) & kMask48;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - w0 > gate_timeout) {
        // never raised: give up rather than hold the CUs forever, and count it
        count(s.counters, kGateTimeouts, 1ull);
        t = __builtin_amdgcn_s_memrealtime() & kMask48;
        break;
      }
    }
    gate_t = gated && not_before(gate_t, t) ? gate_t : t;
    gated = true;
  }
  const uint64_t raw = __builtin_amdgcn_s_memrealtime();
  const uint64_t now = raw & kMask48;
  uint64_t t0 = now;  // unchained: when the gates opened
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
  __hip_atomic_store(slot, (static_cast<uint64_t>(epoch) << 48) | t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t full = raw - ((now - t0) & kMask48);
#pragma unroll
  for (int i = 0; i < 2; ++i)
    if (s.tstart[i]) __hip_atomic_store(s.tstart[i], full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return t0;
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

// A program's join task (DlTask with ticks == 0, the last of its program):
// thread 0 of block 0 waits for its gates (the other lanes' end gates, as a
// task's gates: bounded, counted) and then stores the iteration number into
// the host's done word (sync.tstart[0]; relaxed, system scope) - the whole
// iteration done, signalled while the kernel still runs.
__device__ __forceinline__ void join(const DlSync& s) {
  const uint64_t gate_timeout = s.gate_timeout ? s.gate_timeout : kGateTimeoutTicks;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (!s.gate[i]) continue;
    const uint64_t want = gate_seq(s.iter, s.tag[i]);
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(s.gate[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - w0 > gate_timeout) {
        count(s.counters, kGateTimeouts, 1ull);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  if (s.tstart[0])
    __hip_atomic_store(s.tstart[0], s.iter ? ld(s.iter) : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A program task's epoch: from the iteration word and the task's index among
// the stream's program tasks of the iteration (DlTask::epoch, < 4096), so
// consecutive tasks - the last of one replay and the first of the next too -
// always differ and no slot reset is needed between replays; 1..32767
// (launches of their own take 32768..65534, ComputeEngine).
__device__ __forceinline__ uint32_t program_epoch(const DlTask* prog, int k) {
  const uint64_t it = prog[0].sync.iter ? ld(prog[0].sync.iter) : 0ull;
  return static_cast<uint32_t>((it * 4096ull + prog[k].epoch) % 32767ull) + 1u;
}

}  // namespace dl
}  // namespace kernels
}  // namespace dlnb
