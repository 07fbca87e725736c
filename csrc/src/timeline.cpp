// Device timeline: see dlnb/timeline.hpp.
#include "dlnb/timeline.hpp"

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <limits>

#include "dlnb/common.hpp"

namespace dlnb {

Timeline::Timeline(Device& dev, size_t cap, size_t max_events) : dev_(dev), cap_(cap), max_events_(max_events) {
  stamps_ = dev_.alloc_stamps(cap_);
}

Timeline::~Timeline() {
  if (stamps_) dev_.free_stamps(stamps_, cap_);
}

int Timeline::lane_of(Stream& s) {
  auto it = lanes_.find(&s);
  if (it != lanes_.end()) return it->second;
  const int id = static_cast<int>(lane_names_.size());
  lanes_[&s] = id;
  lane_names_.push_back("stream " + std::to_string(id));
  return id;
}

void Timeline::label(Stream& s, const std::string& name) {
  const bool fresh = lanes_.find(&s) == lanes_.end();
  const int id = lane_of(s);
  if (fresh) lane_names_[static_cast<size_t>(id)] = name;
}

int Timeline::begin(Stream& s) {
  if (frozen_ || next_ + 5 > cap_) {  // 2 for the span; the last 3 slots are calibrate()'s and edge()'s
    if (!frozen_) truncated_ = true;
    return -1;
  }
  const int idx = static_cast<int>(next_++);
  dev_.stamp(s, stamps_ + idx);
  return idx;
}

int Timeline::begin_external(uint64_t** slot) {
  *slot = nullptr;
  if (frozen_ || next_ + 5 > cap_) {
    if (!frozen_) truncated_ = true;
    return -1;
  }
  const int idx = static_cast<int>(next_++);
  *slot = stamps_ + idx;
  return idx;
}

void Timeline::end(int token, Stream& s, const char* cat, const std::string& name, Json args) {
  if (token < 0) return;
  const int idx = static_cast<int>(next_++);  // begin() reserved room for it
  dev_.stamp(s, stamps_ + idx);
  spans_.push_back(Span{token, idx, lane_of(s), 0, nullptr, cat, name, std::move(args)});
}

void Timeline::end_after(int token, Stream& s, uint64_t dur_ticks, const char* cat, const std::string& name,
                         Json args) {
  if (token < 0) return;
  ++next_;  // keep begin()'s accounting (two slots per span)
  spans_.push_back(Span{token, -1, lane_of(s), dur_ticks, nullptr, cat, name, std::move(args)});
}

void Timeline::end_at(int token, Stream& s, const uint64_t* end, const char* cat, const std::string& name,
                      Json args) {
  if (token < 0) return;
  ++next_;  // keep begin()'s accounting (two slots per span)
  spans_.push_back(Span{token, -1, lane_of(s), 0, end, cat, name, std::move(args)});
}

void Timeline::begin_capture() {
  spans_.clear();
  next_ = 0;
  frozen_ = false;
}

void Timeline::end_capture() { frozen_ = true; }

void Timeline::collect(int iter) {
  if (iter >= 0) {
    for (const auto& sp : spans_) {
      if (events_.size() >= max_events_) {
        truncated_ = true;
        break;
      }
      const uint64_t a = __atomic_load_n(stamps_ + sp.a, __ATOMIC_ACQUIRE);
      const uint64_t b = sp.end    ? __atomic_load_n(sp.end, __ATOMIC_ACQUIRE)
                         : sp.b < 0 ? a + sp.dur
                                    : __atomic_load_n(stamps_ + sp.b, __ATOMIC_ACQUIRE);
      events_.push_back(Event{iter, sp.lane, sp.cat, sp.name, sp.args, a, b >= a ? b : a});
    }
  }
  if (frozen_) return;  // a replayed graph rewrites the same slots
  spans_.clear();
  next_ = 0;
}

void Timeline::host_iteration(int iter, double t0_s, double t1_s) {
  if (iter < 0 || events_.size() >= max_events_) return;
  static const int kHostLaneKey = 0;
  auto it = lanes_.find(&kHostLaneKey);
  int lane;
  if (it == lanes_.end()) {
    lane = static_cast<int>(lane_names_.size());
    lanes_[&kHostLaneKey] = lane;
    lane_names_.push_back("host iteration");
  } else {
    lane = it->second;
  }
  auto tick = [&](double t_s) {
    const double d = (t_s * 1e6 - host_cal_us_) * hz_ / 1e6;
    return static_cast<uint64_t>(static_cast<double>(tick_cal_) + d);
  };
  events_.push_back(Event{iter, lane, "host", "iteration (host)", Json::object(), tick(t0_s), tick(t1_s)});
  if (edges_) {
    static const int kEdgeLaneKey = 0;
    auto ie = lanes_.find(&kEdgeLaneKey);
    if (ie == lanes_.end()) {
      lane = static_cast<int>(lane_names_.size());
      lanes_[&kEdgeLaneKey] = lane;
      lane_names_.push_back("graph launch edges");
    } else {
      lane = ie->second;
    }
    const uint64_t e0 = __atomic_load_n(stamps_ + cap_ - 2, __ATOMIC_ACQUIRE);
    const uint64_t e1 = __atomic_load_n(stamps_ + cap_ - 3, __ATOMIC_ACQUIRE);
    events_.push_back(Event{iter, lane, "edge", "before graph launch", Json::object(), e0, e0});
    events_.push_back(Event{iter, lane, "edge", "after graph launch", Json::object(), e1, e1});
  }
}

void Timeline::edge(Stream& s, int which) {
  dev_.stamp(s, stamps_ + cap_ - 2 - (which ? 1 : 0));
  edges_ = true;
}

void Timeline::calibrate(Stream& s) {
  hz_ = dev_.stamp_hz();  // here, not at construction: the rate's measuring window ends at its first use
  // The stamp lands between the two host reads; the best of a few tries
  // (shortest bracket) pairs the clocks.
  double best = std::numeric_limits<double>::max();
  for (int i = 0; i < 5; ++i) {
    uint64_t* slot = stamps_ + cap_ - 1;  // the last slot: begin() never hands it out with a span pending
    s.synchronize();
    const double h0 = now_s() * 1e6;
    dev_.stamp(s, slot);
    s.synchronize();
    const double h1 = now_s() * 1e6;
    const uint64_t t = __atomic_load_n(slot, __ATOMIC_ACQUIRE);
    if (h1 - h0 < best) {
      best = h1 - h0;
      host_cal_us_ = 0.5 * (h0 + h1);
      tick_cal_ = t;
      cal_err_us_ = 0.5 * (h1 - h0);
    }
  }
}

Json Timeline::rank_json(int rank, int keep_iters) const {
  int last = -1;
  for (const auto& e : events_) last = std::max(last, e.iter);
  const int first = keep_iters > 0 ? last - keep_iters + 1 : 0;
  auto host_us = [&](uint64_t t) {
    return host_cal_us_ + (static_cast<double>(t) - static_cast<double>(tick_cal_)) / hz_ * 1e6;
  };
  // Times go out relative to an integer origin (ns on the host clock): the
  // JSON writer keeps 12 significant digits, ~0.1 us of an absolute clock.
  long long origin_ns = 0;
  for (const auto& e : events_)
    if (e.iter >= first) {
      origin_ns = static_cast<long long>(host_us(e.t0) * 1e3);
      break;
    }
  const double origin_us = static_cast<double>(origin_ns) / 1e3;
  Json ev = Json::array();
  for (const auto& e : events_) {
    if (e.iter < first) continue;
    Json row = Json::array();
    row.push_back(e.iter);
    row.push_back(e.lane);
    row.push_back(e.cat);
    row.push_back(e.name);
    row.push_back(host_us(e.t0) - origin_us);
    row.push_back(static_cast<double>(e.t1 - e.t0) / hz_ * 1e6);
    row.push_back(e.args);
    ev.push_back(row);
  }
  Json j = Json::object();
  j["rank"] = rank;
  j["origin_ns"] = origin_ns;
  j["lanes"] = Json(lane_names_);
  j["events"] = ev;
  j["calibration_error_us"] = cal_err_us_;
  j["truncated"] = truncated_;
  return j;
}

void write_chrome_trace(const std::string& path, const std::vector<Json>& ranks, const Json& meta) {
  // every rank's events are relative to its own integer origin_ns
  long long o0 = std::numeric_limits<long long>::max();
  for (const auto& r : ranks)
    if (r.at("events").size()) o0 = std::min(o0, r.at("origin_ns").as_int());
  if (o0 == std::numeric_limits<long long>::max()) o0 = 0;
  auto base_us = [&](const Json& r) { return static_cast<double>(r.at("origin_ns").as_int() - o0) / 1e3; };
  double t0 = std::numeric_limits<double>::max();
  for (const auto& r : ranks) {
    const Json& ev = r.at("events");
    for (size_t i = 0; i < ev.size(); ++i) t0 = std::min(t0, base_us(r) + ev.at(i).at(4).as_double());
  }
  if (t0 == std::numeric_limits<double>::max()) t0 = 0.0;
  Json out = Json::array();
  for (const auto& r : ranks) {
    const int pid = static_cast<int>(r.at("rank").as_int());
    Json pm = Json::object();
    pm["ph"] = "M";
    pm["name"] = "process_name";
    pm["pid"] = pid;
    Json pa = Json::object();
    std::string pname = "rank " + std::to_string(pid);
    if (r.contains("device")) pname += " (" + r.at("device").as_string() + ")";
    pa["name"] = pname;
    pm["args"] = pa;
    out.push_back(pm);
    Json so = Json::object();
    so["ph"] = "M";
    so["name"] = "process_sort_index";
    so["pid"] = pid;
    Json sa = Json::object();
    sa["sort_index"] = pid;
    so["args"] = sa;
    out.push_back(so);
    const Json& lanes = r.at("lanes");
    for (size_t l = 0; l < lanes.size(); ++l) {
      Json tm = Json::object();
      tm["ph"] = "M";
      tm["name"] = "thread_name";
      tm["pid"] = pid;
      tm["tid"] = static_cast<int>(l);
      Json ta = Json::object();
      ta["name"] = lanes.at(l).as_string();
      tm["args"] = ta;
      out.push_back(tm);
    }
    const Json& ev = r.at("events");
    for (size_t i = 0; i < ev.size(); ++i) {
      const Json& e = ev.at(i);
      Json x = Json::object();
      x["ph"] = "X";
      x["pid"] = pid;
      x["tid"] = static_cast<int>(e.at(1).as_int());
      x["cat"] = e.at(2).as_string();
      x["name"] = e.at(3).as_string();
      x["ts"] = base_us(r) + e.at(4).as_double() - t0;
      x["dur"] = e.at(5).as_double();
      Json args = e.at(6);
      args["iter"] = e.at(0).as_int();
      x["args"] = args;
      out.push_back(x);
    }
  }
  Json doc = Json::object();
  doc["traceEvents"] = out;
  doc["displayTimeUnit"] = "ms";
  Json other = meta;
  Json cal = Json::object();
  for (const auto& r : ranks) cal[std::to_string(r.at("rank").as_int())] = r.at("calibration_error_us");
  other["calibration_error_us"] = cal;
  other["time_origin_host_ns"] = o0 + static_cast<long long>(t0 * 1e3);
  doc["otherData"] = other;
  std::ofstream f(path);
  DLNB_REQUIRE(f.good(), "cannot write the timeline to " << path);
  f << doc.dump() << "\n";
}

namespace {

Json op_args(size_t count, DType t, int n) {
  Json a = Json::object();
  a["count"] = static_cast<double>(count);
  a["bytes"] = static_cast<double>(count * dtype_size(t));
  a["dtype"] = dtype_name(t);
  a["ranks"] = n;
  return a;
}

class TracingCommunicator : public Communicator {
 public:
  TracingCommunicator(std::unique_ptr<Communicator> in, Timeline* tl) : in_(std::move(in)), tl_(tl) {
    rank_ = in_->rank();
    size_ = in_->size();
    members_ = in_->members();
    name_ = in_->name();
  }
  std::string backend_name() const override { return in_->backend_name(); }

  void all_reduce(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    traced(s, "all_reduce", count, t, [&] { in_->all_reduce(send, recv, count, t, s); });
  }
  void all_gather(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    traced(s, "all_gather", count * static_cast<size_t>(size_), t, [&] { in_->all_gather(send, recv, count, t, s); });
  }
  void reduce_scatter(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    traced(s, "reduce_scatter", count * static_cast<size_t>(size_), t,
           [&] { in_->reduce_scatter(send, recv, count, t, s); });
  }
  void all_to_all(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    traced(s, "all_to_all", count * static_cast<size_t>(size_), t, [&] { in_->all_to_all(send, recv, count, t, s); });
  }
  void send(const void* buf, size_t count, DType t, int peer, Stream& s) override {
    p2p(s, "send", count, t, peer);
    in_->send(buf, count, t, peer, s);
    if (depth_ == 0) p2p_close();
  }
  void recv(void* buf, size_t count, DType t, int peer, Stream& s) override {
    p2p(s, "recv", count, t, peer);
    in_->recv(buf, count, t, peer, s);
    if (depth_ == 0) p2p_close();
  }
  // A group's operations run as one: one span from the first operation's
  // stream position to the end of the group (the backend launches them at
  // group_end).
  void group_start() override {
    ++depth_;
    in_->group_start();
  }
  void group_end() override {
    in_->group_end();
    if (--depth_ == 0) p2p_close();
  }
  bool wants_peer_buffers() const override { return in_->wants_peer_buffers(); }
  void register_buffer(void* p, size_t bytes) override { in_->register_buffer(p, bytes); }
  std::string async_error() override { return in_->async_error(); }
  void abort() override { in_->abort(); }
  int library_nranks() override { return in_->library_nranks(); }

 private:
  template <class F>
  void traced(Stream& s, const char* op, size_t count, DType t, F&& fn) {
    tl_->label(s, "comm: " + name_);
    const int tok = tl_->begin(s);
    fn();
    tl_->end(tok, s, "comm", std::string(op) + " " + name_, op_args(count, t, size_));
  }
  void p2p(Stream& s, const char* op, size_t count, DType t, int peer) {
    if (!open_) {
      tl_->label(s, "comm: " + name_);
      open_ = true;
      stream_ = &s;
      tok_ = tl_->begin(s);
      ops_.clear();
      bytes_ = 0;
    }
    if (!ops_.empty()) ops_ += ",";
    ops_ += std::string(op) + "(" + std::to_string(peer) + ")";
    bytes_ += static_cast<double>(count * dtype_size(t));
  }
  void p2p_close() {
    if (!open_) return;
    open_ = false;
    Json a = Json::object();
    a["bytes"] = bytes_;
    a["ops"] = ops_;
    tl_->end(tok_, *stream_, "p2p", "p2p " + name_, a);
  }
  std::unique_ptr<Communicator> in_;
  Timeline* tl_;
  int depth_ = 0, tok_ = -1;
  bool open_ = false;
  Stream* stream_ = nullptr;
  std::string ops_;
  double bytes_ = 0;
};

class TracingFactory : public CommFactory {
 public:
  TracingFactory(std::unique_ptr<CommFactory> in, Timeline* tl) : in_(std::move(in)), tl_(tl) {}
  std::string backend_name() const override { return in_->backend_name(); }
  std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members,
                                       size_t capacity_bytes, bool need_p2p, int max_ctas) override {
    return std::make_unique<TracingCommunicator>(in_->create(name, members, capacity_bytes, need_p2p, max_ctas), tl_);
  }

 private:
  std::unique_ptr<CommFactory> in_;
  Timeline* tl_;
};

class TracingCompute : public ComputeEngine {
 public:
  TracingCompute(std::unique_ptr<ComputeEngine> in, Timeline* tl) : in_(std::move(in)), tl_(tl) {}
  void run(Stream& s, double us, double flops) override {
    traced(s, "compute", us, [&] { in_->run(s, us, flops); });
  }
  void run_stamped(Stream& s, double us, double flops, uint64_t* start) override {
    traced(s, "compute", us, [&] { in_->run_stamped(s, us, flops, start); });
  }
  bool stamps_task_start() const override { return in_->stamps_task_start(); }
  void run_chained(Stream& s, double us, double flops, uint64_t* start, Event* done) override {
    traced(s, "compute (chained)", us, [&] { in_->run_chained(s, us, flops, start, done); });
  }
  uint64_t task_ticks(double us) const override { return in_->task_ticks(us); }
  bool gates_task(double us) const override { return in_->gates_task(us); }
  int make_gate() override { return in_->make_gate(); }
  void signal(Stream& s, int gate) override { in_->signal(s, gate); }
  void wait_gate(Stream& s, int gate, double timeout_us) override { in_->wait_gate(s, gate, timeout_us); }
  void run_gated(Stream& s, double us, double flops, const std::vector<int>& gates, uint64_t* start,
                 bool chain, Event* done) override {
    Json a = Json::object();
    a["gates"] = static_cast<int>(gates.size());
    traced(s, chain ? "compute (chained)" : "compute", us,
           [&] { in_->run_gated(s, us, flops, gates, start, chain, done); }, a);
  }
  void set_next_start_slot(uint64_t* slot) override { in_->set_next_start_slot(slot); }
  void reset_clocks(Stream& s) override { in_->reset_clocks(s); }
  void reset_slot(Stream& s) override { in_->reset_slot(s); }
  bool begin_program(Stream& s) override { return in_->begin_program(s); }
  void end_program(Stream& s, bool join_ok) override { in_->end_program(s, join_ok); }
  long programs_on(Stream& s) override { return in_->programs_on(s); }
  bool program_split(Stream& s) override { return in_->program_split(s); }
  const uint64_t* last_task_end(Stream& s) override { return in_->last_task_end(s); }
  void after_capture() override { in_->after_capture(); }
  void set_lane_join(Stream& s, const std::vector<uint64_t*>& gates, uint32_t tag, uint64_t* host_done) override {
    in_->set_lane_join(s, gates, tag, host_done);
  }
  bool program_joined(Stream& s) override { return in_->program_joined(s); }
  void set_gate_timeout(double s) override { in_->set_gate_timeout(s); }
  double lane_task_us(Stream& s) override { return in_->lane_task_us(s); }
  void reset_capped(Stream& s) override { in_->reset_capped(s); }
  bool chain_counters(ChainCounters& c) override { return in_->chain_counters(c); }
  void set_task_timers(TimerSet* t) override { in_->set_task_timers(t); }
  Json describe() const override { return in_->describe(); }
  ComputeMode mode() const override { return in_->mode(); }

 private:
  // A deadline engine's kernels write their task's effective start (after
  // its gates, at the chain's deadline) into the span's first slot, so a
  // wait for a collective shows as exposed communication, not as compute,
  // and an absorbed launch gap not as idle; other engines: a stamp kernel.
  template <class F>
  void traced(Stream& s, const char* name, double us, F&& fn, Json a = Json::object()) {
    tl_->label(s, "compute");
    int tok;
    if (in_->stamps_task_start()) {
      uint64_t* first = nullptr;
      tok = tl_->begin_external(&first);
      in_->set_next_start_slot(first);
    } else {
      tok = tl_->begin(s);
    }
    fn();
    a["table_us"] = us;
    if (!in_->stamps_task_start())
      tl_->end(tok, s, "compute", name, a);
    else if (const uint64_t* e = in_->last_task_end(s))
      tl_->end_at(tok, s, e, "compute", name, a);  // fixed work: the task's own end stamp
    else
      tl_->end_after(tok, s, in_->task_ticks(us), "compute", name, a);
  }
  std::unique_ptr<ComputeEngine> in_;
  Timeline* tl_;
};

}  // namespace

std::unique_ptr<CommFactory> make_tracing_factory(std::unique_ptr<CommFactory> inner, Timeline* tl) {
  return std::make_unique<TracingFactory>(std::move(inner), tl);
}

std::unique_ptr<ComputeEngine> make_tracing_compute(std::unique_ptr<ComputeEngine> inner, Timeline* tl) {
  return std::make_unique<TracingCompute>(std::move(inner), tl);
}

}  // namespace dlnb
