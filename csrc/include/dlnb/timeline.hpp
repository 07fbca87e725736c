// Device timeline (--timeline PATH): every collective, point-to-point group
// and compute task of every rank as a span of device time on the stream it
// ran on, written as one Chrome / Perfetto trace (chrome://tracing,
// ui.perfetto.dev) with a process per rank and a track per stream.
//
// The reference has host wall-clock phase timers only (ccutils
// CCUTILS_MPI_TIMER_*, cpp/data_parallel/dp.cpp:69-70,102-104; SURVEY.md §5
// "Tracing / profiling"): vectors of durations, no timeline, nothing on the
// device. Here a span is two Device::stamp()s on the op's own stream (a
// one-wave s_memrealtime kernel on the GPU, captured into the HIP graph with
// the iteration), taken by decorators around the communicators and the
// compute engine, so the strategies need no changes. Every rank calibrates
// its device clock against the host's steady clock once (a stamp bracketed
// by two host reads), so the ranks of one node share one time axis; the
// bracket's half-width is reported per rank as the alignment error.
//
// Cost: two stamp kernels per traced op (a few us each on the op's stream);
// off unless --timeline is given.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "dlnb/comm.hpp"
#include "dlnb/compute.hpp"
#include "dlnb/device.hpp"
#include "dlnb/json.hpp"

namespace dlnb {

class Timeline {
 public:
  // cap = stamp slots per iteration (two per span).
  explicit Timeline(Device& dev, size_t cap = size_t(1) << 16, size_t max_events = size_t(1) << 20);
  ~Timeline();
  Timeline(const Timeline&) = delete;
  Timeline& operator=(const Timeline&) = delete;

  // A span of work on stream s: begin() before the work is enqueued, end()
  // after (same stream). Returns / takes -1 when the slots ran out.
  int begin(Stream& s);
  // The same, but the span's start is written by the work itself (a deadline
  // kernel's start, ComputeEngine::set_next_start_slot) into *slot.
  int begin_external(uint64_t** slot);
  void end(int token, Stream& s, const char* cat, const std::string& name, Json args = Json::object());
  // End a span `dur_ticks` device-clock ticks after its start, without a
  // stamp: a deadline task's span is [start, deadline] (its grid's drain
  // after the deadline belongs to the next chained task, which starts at it).
  void end_after(int token, Stream& s, uint64_t dur_ticks, const char* cat, const std::string& name,
                 Json args = Json::object());
  // End a span at a stamp the work writes itself into *end (host-mapped; a
  // fixed-work task's own end stamp, ComputeEngine::last_task_end), read at
  // collect() like the span's own slots.
  void end_at(int token, Stream& s, const uint64_t* end, const char* cat, const std::string& name,
              Json args = Json::object());
  // Track name of a stream (the first name given wins).
  void label(Stream& s, const std::string& name);
  // Graph mode: the spans enqueued between these are the captured
  // iteration's; every replay rewrites the same slots and collect() re-reads
  // them.
  void begin_capture();
  void end_capture();
  // After the streams were synchronised: record this iteration's spans
  // (iter >= 0) or drop them (warm-up: iter < 0).
  void collect(int iter);
  // Pairs the device clock with the host's steady clock (host-syncs s).
  void calibrate(Stream& s);
  // The host's view of iteration `iter` (now_s() before the enqueue / graph
  // launch and after the streams were synchronised: what the reference times)
  // as a span on a "host" track: host span - device span = the iteration
  // boundary (launch + completion detection).
  void host_iteration(int iter, double t0_s, double t1_s);
  // Graph mode: a stamp on the launch stream right before (which = 0) and
  // right after (1) the graph launch, outside the graph, so host_iteration()
  // can split the boundary into submission, the graph's start, its join back
  // onto the launch stream and the host's completion detection.
  void edge(Stream& s, int which);
  // This rank's events of the last `keep_iters` collected iterations
  // (0 = all): {"rank", "lanes", "events": [[iter, lane, cat, name, ts_us,
  // dur_us, args], ...], "calibration_error_us", "truncated"}; ts_us on the
  // host steady clock.
  Json rank_json(int rank, int keep_iters) const;
  size_t events() const { return events_.size(); }
  bool truncated() const { return truncated_; }

 private:
  int lane_of(Stream& s);
  Device& dev_;
  uint64_t* stamps_ = nullptr;
  size_t cap_ = 0, next_ = 0, max_events_ = 0;
  struct Span {
    int a, b, lane;  // b < 0: the span lasts dur ticks from a (or ends at *end)
    uint64_t dur;
    const uint64_t* end;
    const char* cat;
    std::string name;
    Json args;
  };
  std::vector<Span> spans_;
  struct Event {
    int iter, lane;
    const char* cat;
    std::string name;
    Json args;
    uint64_t t0, t1;
  };
  std::vector<Event> events_;
  std::map<const void*, int> lanes_;
  std::vector<std::string> lane_names_;
  bool frozen_ = false, truncated_ = false, edges_ = false;
  double hz_ = 1e9;
  double host_cal_us_ = 0.0, cal_err_us_ = 0.0;
  uint64_t tick_cal_ = 0;
};

// Decorators that trace every operation into `tl` (which must outlive them).
std::unique_ptr<CommFactory> make_tracing_factory(std::unique_ptr<CommFactory> inner, Timeline* tl);
std::unique_ptr<ComputeEngine> make_tracing_compute(std::unique_ptr<ComputeEngine> inner, Timeline* tl);

// Rank 0: one Chrome trace from every rank's rank_json() (times shifted so
// the earliest event is at 0).
void write_chrome_trace(const std::string& path, const std::vector<Json>& ranks, const Json& meta);

}  // namespace dlnb
