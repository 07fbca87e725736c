// Per-phase timers: device event pairs resolved after each iteration, plus
// host wall-clock values.
//
// Reference: ccutils CCUTILS_MPI_TIMER_DEF/START/STOP host timers whose
// std::vector<float> __timer_vals_<name> are dumped into the JSON sections
// (cpp/data_parallel/dp.cpp:69-70,102-104,260-263; fsdp.cpp:61-66). Here a
// "device" timer is a pair of timestamps taken when a stream reaches two
// points (Device::stamp: a one-wave s_memrealtime kernel on the GPU), so it
// measures the time the stream spent in an operation (a collective's
// duration on its comm stream, or the compute stream's stall waiting for a
// collective = exposed comm). HIP timing events are not used for this: on
// ROCm 7.2 an event recorded right after a cross-stream wait can carry the
// timestamp of the wait's start.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "dlnb/device.hpp"
#include "dlnb/json.hpp"

namespace dlnb {

class TimerSet {
 public:
  explicit TimerSet(Device& dev);
  ~TimerSet();
  TimerSet(const TimerSet&) = delete;
  TimerSet& operator=(const TimerSet&) = delete;
  int begin(Stream& s);
  // The stamp slot of a begin() token (nullptr when disabled), e.g. for pair().
  const uint64_t* at(int token) const { return token < 0 ? nullptr : stamps_ + token; }
  // Returns the end stamp's slot (nullptr when disabled), e.g. for gap().
  const uint64_t* end(int token, Stream& s, const std::string& name);
  // Time the stall of stream s waiting for event e (exposed latency).
  void stall(Stream& s, Event& e, const std::string& name);
  // Stamp-free variant for a wait between two compute tasks on one stream
  // whose kernels stamp their own start (ComputeEngine::run_stamped):
  // slot() hands out a host-mapped stamp slot for the next task's start, and
  // gap() records value = next_start - (prev_start + prev_ticks), i.e. how
  // long the stream sat between the previous task's deadline and the next
  // task's first block (the dependency wait plus the launch).
  uint64_t* slot();
  // clamp: the two ends are not causally ordered (a collective that may
  // finish before the compute it is compared with): a negative value is a
  // real 0, not an error (negatives_json does not count it).
  void gap(const uint64_t* prev_start, uint64_t prev_ticks, const uint64_t* next_start, const std::string& name,
           bool clamp = false);
  // Stall timers from the compute tasks' own start stamps, for any strategy.
  // With set_task_stamps(true) (the engine's kernels stamp their start:
  // deadline / idle / spin compute), the engine takes a slot for every task
  // (task_slot) and reports its start and duration (task_started); a timed
  // operation on the stream (begin / end) moves the stream's reference to its
  // end stamp. stall_before_task(s, e, name) - a wait that the next compute
  // task (or timed operation) on s follows - then records the gap from the
  // previous task's deadline on s to that task's own start: no stamp kernel
  // is queued on s, so no graph executor can place one behind a collective
  // (VERDICT r4 #1). stall_after_task(s, e, name): a wait with untimed work
  // after it (the optimizer), timed from the previous task's deadline to a
  // stamp right after the wait. Either falls back to stall() when no task
  // precedes the wait in the iteration; a stall_before_task that nothing
  // follows is closed by finish_stalls() (the runner, after each
  // enqueue_iteration) with a stamp on s.
  // A task without a deadline (fixed work) reports its own end stamp too
  // (task_started's `end`): the stream's next wait is timed from there.
  // Without a task before it in the iteration, a wait is timed from a stamp
  // right before it (mark: nothing waited for between the two).
  void set_task_stamps(bool on) { task_stamps_ = on; }
  bool task_stamps() const { return task_stamps_ && enabled_; }
  uint64_t* task_slot(Stream& s);
  void task_started(Stream& s, const uint64_t* start, uint64_t ticks, const uint64_t* end = nullptr);
  // A stamp kernel on s now (its slot; nullptr when disabled).
  const uint64_t* mark(Stream& s);
  // value = *b - *a for two stamp slots of this set (a task's own start and
  // end: compute_task_time).
  void pair(const uint64_t* a, const uint64_t* b, const std::string& name);
  void stall_before_task(Stream& s, Event& e, const std::string& name);
  void stall_after_task(Stream& s, Event& e, const std::string& name);
  // The waits pending on s (stall_before_task with no task after them yet)
  // were for an operation on another stream that ended at op_end (its end
  // stamp): they end there (clamped - the operation may have ended before s
  // got to the wait), and s's next wait is timed from the later of its
  // reference and op_end. E.g. the last all-to-all of a backward and the
  // gradient all-reduce queued behind it on the same lane: the compute
  // stream's wait for the all-reduce is not booked on the all-to-all.
  void settle(Stream& s, const uint64_t* op_end);
  // s does not wait for the operation that ends at `end` (another stream's
  // end stamp) - the iteration does (a lane join): `name` is the time from
  // s's reference (its last task's end, or settle's floor) to `end`, clamped.
  // Nothing is enqueued on s. Needs task stamps.
  void stall_until(Stream& s, const uint64_t* end, const std::string& name);
  // A stamp heading the iteration on s (the runner, before the strategy's
  // enqueue; in a single graph the head node every stream's chain follows):
  // s's first wait with no task before it is timed from there, not from a
  // stamp queued right before the wait - in a single graph that one is a
  // sibling of the other streams' first nodes and can run after them (a
  // stage's wait for its first activation read ~0 instead of the forward of
  // the stage before).
  void iteration_start(Stream& s);
  void finish_stalls();
  void add(const std::string& name, double seconds);
  void ensure(const std::string& name);
  // Call after the streams involved have been synchronised. Intervals are
  // causally ordered, so a negative one (mis-ordered stamps) is recorded as
  // 0 and counted per timer (negatives_json: {name: {count, worst_ms}}).
  void resolve();
  void clear();
  Json negatives_json() const;
  bool has_negatives() const { return !negatives_.empty(); }
  // Graph mode: between begin_capture() and end_capture() host values are
  // recorded instead of applied; afterwards the stamp pairs and the recorded
  // host values are re-applied by every resolve() (one per graph replay).
  void begin_capture();
  void end_capture();
  void set_enabled(bool on) { enabled_ = on; }
  bool enabled() const { return enabled_; }
  const std::vector<double>& get(const std::string& name) const;
  double sum(const std::string& name) const;
  Json values_json(const std::string& name) const;

 private:
  Device& dev_;
  uint64_t* stamps_ = nullptr;  // host-readable timestamp slots
  size_t cap_ = 0;
  size_t next_ = 0;
  struct Pending {
    int a, b;
    std::string name;
  };
  std::vector<Pending> pending_;
  struct Gap {
    int prev, next;
    uint64_t prev_ticks;
    std::string name;
    bool clamp;
    int floor;  // >= 0: the interval starts no earlier than this slot
  };
  std::vector<Gap> gaps_;
  bool owns(const uint64_t* p) const { return p >= stamps_ && p < stamps_ + cap_; }
  struct TaskClock {
    const uint64_t* start = nullptr;  // the last task's start slot on the stream
    uint64_t ticks = 0;
    const uint64_t* floor = nullptr;  // settle(): another stream's end stamp the next wait starts after
    std::vector<std::string> pending;  // stall_before_task names since it
  };
  std::map<Stream*, TaskClock> clocks_;
  Stream* origin_ = nullptr;
  const uint64_t* origin_start_ = nullptr;
  void first_reference(Stream& s, TaskClock& c);
  void close_pending(TaskClock& c, const uint64_t* at, bool clamp = false);
  static void restart(TaskClock& c, const uint64_t* start, uint64_t ticks) {
    c.start = start;
    c.ticks = ticks;
    c.floor = nullptr;
  }
  bool task_stamps_ = false;
  std::map<std::string, std::vector<double>> vals_;
  struct Negative {
    long count = 0;
    double worst_s = 0.0;
  };
  std::map<std::string, Negative> negatives_;
  std::vector<std::pair<std::string, double>> captured_adds_;
  bool capturing_ = false, frozen_ = false;
  bool enabled_ = true;
};

}  // namespace dlnb
