// Synthetic compute that stands in for the model's forward/backward math.
//
// The reference simulates compute with host usleep(µs) read from the stats
// tables (cpp/data_parallel/dp.cpp:93,98; fsdp.cpp:103,120,145;
// hybrid_2d.cpp:111-156), which leaves the GPU idle while collectives run.
// Modes here (all stream ordered):
//   sleep - the stream is busy for exactly the duration, the GPU is idle
//           (one-wave s_memrealtime wait on GPU; nanosleep task on CPU);
//           reference parity.
//   spin  - every CU runs dependent VALU work until the deadline.
//   gemm  - (default on GPU) hand-written MFMA GEMM shaped from the model
//           (M = 8192-token chunk, N = FFN dim, K = hidden dim) run as a
//           persistent kernel on every CU that stops at a device-clock
//           deadline: exactly the table's duration, with the matrix cores
//           and HBM as busy as in training (the reference's usleep leaves
//           the GPU idle, so its collectives never contend with compute).
//   gemm-work - the same GEMM as a fixed amount of work: full-K rounds of
//           256 x 256 tiles over the same persistent grid plus a partial-K
//           tail tile, calibrated at start-up (after a DVFS settle) so the
//           uncontended duration matches the table; contention / clock drops
//           stretch it, like real training compute. A task is a program task
//           of the deadline kernels (one launch, or one task of the lane's
//           compute program): it stamps its own start and end;
//   flops - the same with the table's FLOP count as the work (MI355X-native
//           compute time).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "dlnb/device.hpp"
#include "dlnb/json.hpp"
#include "dlnb/timers.hpp"

namespace dlnb {

enum class ComputeMode { Sleep, Spin, Gemm, GemmWork, Flops };

ComputeMode parse_compute_mode(const std::string& s, DeviceKind dev);
const char* compute_mode_name(ComputeMode m);

struct ComputeShape {
  int hidden = 4096;  // model hidden size (N of the stand-in GEMM: the FFN down projection)
  int ffn = 16384;    // FFN width (K)
  DType dtype = DType::BF16;
  int comm_cus = 32;  // CUs the persistent compute leaves to collectives
  // Ranks sharing the device (loopback rank threads, several processes on one
  // GPU): their deadline tasks are cut into 500-us slices by default so that
  // the ranks' compute interleaves as it would on separate GPUs.
  int ranks_on_device = 1;
};

class ComputeEngine {
 public:
  virtual ~ComputeEngine() = default;
  // Enqueue `us` microseconds of compute; `flops` is the real FLOP count of
  // that piece of work (used by the flops mode).
  virtual void run(Stream& s, double us, double flops) = 0;
  // Same, and the kernel itself writes the task's start time (device clock,
  // Device::stamp_hz) into *start (host-mapped) - only where
  // stamps_task_start() is true. task_ticks(us) = the task's duration in
  // those clock ticks.
  virtual void run_stamped(Stream& s, double us, double flops, uint64_t* start) {
    (void)start;
    run(s, us, flops);
  }
  virtual bool stamps_task_start() const { return false; }
  // A task that continues the previous task on s: the caller guarantees that
  // nothing but event records was enqueued on s in between (no waits, no
  // collectives), so the two are one stretch of compute. The gemm (deadline)
  // mode then ends it at the previous task's deadline + us on the clock the
  // stretch started with, so a kernel-boundary gap between the two is
  // absorbed rather than added (a replayed HIP graph puts consecutive kernels
  // of a stream on different hardware queues: ~10 us per hop, measured in
  // profiles/graph_queues_r2.md). The compute still lasts the table's total.
  // Other modes: run().
  // start (optional): as run_stamped's. done (optional): an event recorded
  // on s once the task is over (Stream::record semantics) - with gate events
  // (lane graphs) a deadline task raises its gate from its own kernel, so no
  // gate_signal kernel sits between two compute tasks.
  virtual void run_chained(Stream& s, double us, double flops, uint64_t* start = nullptr, Event* done = nullptr) {
    run_stamped(s, us, flops, start);
    if (done) s.record(*done);
  }
  virtual uint64_t task_ticks(double us) const { (void)us; return 0; }
  // Fixed-work compute (gemm-work, flops) has no deadline: its tasks stamp
  // their end too, and this is the end slot of the last task enqueued on s
  // (nullptr: the end is start + task_ticks(us)). A stall after a task is
  // timed from there (task_mark()).
  virtual const uint64_t* last_task_end(Stream& s) { (void)s; return nullptr; }
  // Device-side dependency times (gemm mode; csrc/kernels/deadline_sync.hpp).
  // A gate is a device word: signal(s, g) enqueues on s (a collective's
  // stream, after the collective, before the event the compute stream waits
  // on) a one-wave kernel that raises it with a fresh tag and the time.
  // run_gated() enqueues a task whose first block reads its gates (at most
  // 2, signalled before in host order; the caller also waits on their
  // events, so they are already raised) and, with chain = true, starts at
  // max(the stream's previous deadline, the gates' times): the queue hop and
  // launch gap after a stream wait are absorbed, a late collective is not.
  // *start gets the task's effective start (stall timers: the gap to the
  // previous deadline is the exposed wait). gates_task(us): whether a task
  // of us microseconds can use this (else run_stamped).
  virtual bool gates_task(double us) const { (void)us; return false; }
  virtual int make_gate() { DLNB_THROW("this compute mode has no device gates"); }
  virtual void signal(Stream& s, int gate) { (void)s; (void)gate; DLNB_THROW("this compute mode has no device gates"); }
  // The other direction: stream s (a comm lane) waits on the device until the
  // gate carries the tag of its latest signal(), instead of a cross-stream
  // event (no graph edge from the signalling stream; timeout_us bounds it,
  // counted in chain_counters()).
  virtual void wait_gate(Stream& s, int gate, double timeout_us) {
    (void)s; (void)gate; (void)timeout_us;
    DLNB_THROW("this compute mode has no device gates");
  }
  virtual void run_gated(Stream& s, double us, double flops, const std::vector<int>& gates, uint64_t* start,
                         bool chain, Event* done = nullptr) {
    (void)s; (void)us; (void)flops; (void)gates; (void)start; (void)chain; (void)done;
    DLNB_THROW("this compute mode has no device gates");
  }
  // A second host-mapped slot the next deadline task's kernel writes its
  // start into (the --timeline decorator's span start).
  virtual void set_next_start_slot(uint64_t* slot) { (void)slot; }
  // Graph mode: enqueue on s a reset of whatever per-task device state the
  // engine keys by epoch (a replayed graph repeats the captured epochs):
  // reset_clocks every stream's (one graph, at its head), reset_slot only
  // the state of tasks that ran on s (lane graphs: at the tail of s's graph,
  // the lane's own tasks being done by then).
  virtual void reset_clocks(Stream& s) { (void)s; }
  virtual void reset_slot(Stream& s) { (void)s; }
  // Compute programs (lane graphs): the deadline tasks enqueued on s between
  // begin_program(s) and end_program(s) run as ONE persistent kernel
  // (kernels::gemm_tn_deadline_program): each task starts, chains and gates
  // exactly as a launch of its own, with no kernel boundary between two
  // tasks. Nothing but compute tasks may be enqueued on s inside (the caller's
  // compute lane carries only them: gate events folded into the tasks, stall
  // timers from the tasks' own stamps); a task the program cannot take (an
  // idle / spin task) is launched between two programs. begin_program
  // returns false when the engine does not build programs (then tasks launch
  // one by one). after_capture(): upload the task lists of programs built
  // during a graph capture (device memory written outside the capture).
  // end_program(s, join_ok): join_ok = nothing is enqueued on s after the
  // program in this iteration, so a pending lane join (set_lane_join) may
  // end it; otherwise the join is not taken and the lane ends with its own
  // done word (work after the join - the optimizer, a stall stamp -
  // would run outside the iteration the host times).
  virtual bool begin_program(Stream& s) { (void)s; return false; }
  virtual void end_program(Stream& s, bool join_ok) { (void)s; (void)join_ok; }
  virtual void after_capture() {}
  // Programs launched on s so far (a lane of one program per iteration pays
  // no kernel boundaries between its tasks, joined or not).
  virtual long programs_on(Stream& s) { (void)s; return 0; }
  // Whether the last program opened on s was split by a task too short for a
  // program (< 20 us: launched on its own between two launches of the program).
  virtual bool program_split(Stream& s) { (void)s; return false; }
  // Lane join (the runner, lane graphs): the next program ended on s finishes
  // with a join task - thread 0 of block 0 waits for `gates` (the other
  // lanes' end gates, raised with `tag`) and stores the iteration number into
  // *host_done - so the iteration's completion is signalled from inside the
  // still-running compute kernel (a kernel ending around the iteration's
  // last collective costs the one-wave kernels near it ~40 us, round 5).
  // program_joined(s): whether it happened (then the lanes need no done
  // word of their own, nor a slot reset: program epochs follow the
  // iteration word).
  virtual void set_lane_join(Stream& s, const std::vector<uint64_t*>& gates, uint32_t tag, uint64_t* host_done) {
    (void)s; (void)gates; (void)tag; (void)host_done;
  }
  virtual bool program_joined(Stream& s) { (void)s; return false; }
  // Bound (s) of the deadline tasks' gate waits enqueued from here on.
  virtual void set_gate_timeout(double s) { (void)s; }
  // Mean duration (us) of the compute tasks enqueued on s since set_lane_join
  // (a lane capture), each one kernel (deadline / idle / spin / fixed work);
  // < 0 when any task took several launches or none ran. A lane of long
  // single-kernel tasks pays its kernel boundaries on one queue at little
  // cost (the runner keeps such lanes without a compute program).
  virtual double lane_task_us(Stream& s) { (void)s; return -1.0; }
  // Counters of the chained / gated deadline tasks (kernels::DlCounter):
  //   capped: tasks whose first block came later than the absorb cap after
  //     their chained start (a wait, not a launch hop: e.g. a replayed graph
  //     queueing the task behind another stream's collective) and that
  //     lateness beyond the cap, which stays in the iteration time;
  //   absorbed: the lateness (<= the cap per task) chained tasks took out of
  //     their own compute - launch hops and drains the iteration does not see;
  //   timeouts: gate waits that gave up (comm lanes' gate_wait, deadline
  //     tasks' gates; never expected, counted since the engine was made).
  // reset_capped zeroes the capped / absorbed counts (stream-ordered on s);
  // chain_counters reads them (host, after a sync).
  //   aborted: waits that gave up on the host's abort word (Device::abort_word);
  //   late_blocks: program blocks that reached a task after a later one was
  //     claimed (dispatched late) and skipped it.
  struct ChainCounters {
    double capped_tasks = 0, capped_s = 0, absorbed_tasks = 0, absorbed_s = 0;
    double wait_timeouts = 0, gate_timeouts = 0, aborted = 0, late_blocks = 0;
  };
  virtual void reset_capped(Stream& s) { (void)s; }
  virtual bool chain_counters(ChainCounters& c) { (void)c; return false; }
  // Fixed-work modes (gemm-work, flops): time every compute task on the
  // device into t ("compute_task_time", from the task's own start and end
  // stamps) next to its table duration ("compute_task_table"), so the runner
  // can report how much collectives running beside the compute stretch it
  // (compute_stretch). Deadline modes last exactly the table time by
  // construction and record nothing. Every GPU mode also feeds its tasks'
  // start (and end) stamps to t's stall timers.
  virtual void set_task_timers(TimerSet* t) { (void)t; }
  virtual Json describe() const = 0;
  virtual ComputeMode mode() const = 0;
};

std::unique_ptr<ComputeEngine> make_compute_engine(Device& dev, ComputeMode mode, const ComputeShape& shape,
                                                   double time_scale);

// Where a compute task ends on the device clock, for a stall timer after it:
// its end stamp (fixed work) or its start stamp + its deadline ticks.
struct TaskMark {
  const uint64_t* slot = nullptr;
  uint64_t ticks = 0;
};
inline TaskMark task_mark(ComputeEngine& ce, Stream& s, const uint64_t* start, double us) {
  if (const uint64_t* e = ce.last_task_end(s)) return {e, 0};
  return {start, ce.task_ticks(us)};
}

}  // namespace dlnb
