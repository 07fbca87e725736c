#include "dlnb/timers.hpp"

#include <algorithm>
#include "dlnb/common.hpp"

namespace dlnb {

TimerSet::TimerSet(Device& dev) : dev_(dev) {
  cap_ = 1 << 16;
  stamps_ = dev_.alloc_stamps(cap_);
}

TimerSet::~TimerSet() {
  if (stamps_) dev_.free_stamps(stamps_, cap_);
}

int TimerSet::begin(Stream& s) {
  if (!enabled_) return -1;
  DLNB_REQUIRE(next_ < cap_, "too many timer stamps in one iteration");
  int idx = static_cast<int>(next_++);
  dev_.stamp(s, stamps_ + idx);
  if (task_stamps()) {
    auto it = clocks_.find(&s);
    if (it != clocks_.end() && !it->second.pending.empty()) close_pending(it->second, stamps_ + idx);
  }
  return idx;
}

const uint64_t* TimerSet::end(int token, Stream& s, const std::string& name) {
  if (!enabled_ || token < 0) return nullptr;
  DLNB_REQUIRE(next_ < cap_, "too many timer stamps in one iteration");
  int idx = static_cast<int>(next_++);
  dev_.stamp(s, stamps_ + idx);
  pending_.push_back(Pending{token, idx, name});
  if (task_stamps()) {
    auto it = clocks_.find(&s);
    if (it != clocks_.end()) restart(it->second, stamps_ + idx, 0);  // the stream's next wait is timed from here
  }
  return stamps_ + idx;
}

void TimerSet::stall(Stream& s, Event& e, const std::string& name) {
  static const bool timed = env_int("DLNB_STALL_TIMERS", 1) != 0;  // 0: A/B the stamps' own cost
  if (!timed) {
    s.wait(e);
    return;
  }
  // A stamp-wait-stamp pair read short under graph replay (round 4): inside a
  // capture every stall is timed from task stamps (stall_before_task /
  // stall_after_task) or as a gap between stamps nothing waits between.
  DLNB_REQUIRE(!capturing_ || !task_stamps_, "TimerSet::stall(" << name << ") inside a graph capture");
  int t = begin(s);
  s.wait(e);
  end(t, s, name);
}

uint64_t* TimerSet::task_slot(Stream& s) {
  (void)s;
  if (!task_stamps()) return nullptr;
  return slot();
}

void TimerSet::task_started(Stream& s, const uint64_t* start, uint64_t ticks, const uint64_t* end) {
  if (!task_stamps() || !owns(start)) return;
  TaskClock& c = clocks_[&s];
  close_pending(c, start);
  if (end && owns(end))
    restart(c, end, 0);  // fixed work: the task's own end stamp
  else
    restart(c, start, ticks);
}

const uint64_t* TimerSet::mark(Stream& s) {
  if (!enabled_) return nullptr;
  uint64_t* st = slot();
  dev_.stamp(s, st);
  return st;
}

void TimerSet::pair(const uint64_t* a, const uint64_t* b, const std::string& name) {
  if (!enabled_ || !owns(a) || !owns(b)) return;
  pending_.push_back(Pending{static_cast<int>(a - stamps_), static_cast<int>(b - stamps_), name});
}

void TimerSet::stall_before_task(Stream& s, Event& e, const std::string& name) {
  if (!task_stamps()) {
    stall(s, e, name);
    return;
  }
  TaskClock& c = clocks_[&s];
  if (!c.start) {
    // no task before the wait in this iteration: the iteration's head stamp,
    // or a stamp right before the wait (nothing is waited for between the two)
    first_reference(s, c);
  }
  s.wait(e);
  c.pending.push_back(name);
}

void TimerSet::stall_after_task(Stream& s, Event& e, const std::string& name) {
  if (!task_stamps()) {
    stall(s, e, name);
    return;
  }
  TaskClock& c = clocks_[&s];
  if (!c.start) first_reference(s, c);
  s.wait(e);
  DLNB_REQUIRE(next_ < cap_, "too many timer stamps in one iteration");
  uint64_t* st = stamps_ + next_++;
  dev_.stamp(s, st);
  c.pending.push_back(name);  // (after earlier waits with no task between: the first takes the gap)
  close_pending(c, st);
  restart(c, st, 0);
}

void TimerSet::stall_until(Stream& s, const uint64_t* end, const std::string& name) {
  if (!enabled_) return;
  DLNB_REQUIRE(task_stamps() && owns(end), "TimerSet::stall_until(" << name << ") needs task stamps");
  TaskClock& c = clocks_[&s];
  DLNB_REQUIRE(c.start, "TimerSet::stall_until(" << name << "): no task before it on the stream");
  c.pending.push_back(name);
  close_pending(c, end, true);
}

void TimerSet::iteration_start(Stream& s) {
  if (!task_stamps()) return;
  origin_ = &s;
  origin_start_ = mark(s);
}

void TimerSet::first_reference(Stream& s, TaskClock& c) {
  if (&s == origin_ && origin_start_)
    restart(c, origin_start_, 0);
  else
    restart(c, mark(s), 0);
}

void TimerSet::settle(Stream& s, const uint64_t* op_end) {
  if (!task_stamps() || !owns(op_end)) return;
  auto it = clocks_.find(&s);
  if (it == clocks_.end() || !it->second.start || it->second.pending.empty()) return;
  close_pending(it->second, op_end, true);
  it->second.floor = op_end;
}

// A stream's pending stall_before_task waits end where the stream reaches
// `at` (a task's start or a timed operation's begin stamp).
void TimerSet::close_pending(TaskClock& c, const uint64_t* at, bool clamp) {
  for (size_t i = 0; i < c.pending.size(); ++i) {
    if (i == 0) {
      gap(c.start, c.ticks, at, c.pending[i], clamp);
      if (c.floor && enabled_ && c.start && at) gaps_.back().floor = static_cast<int>(c.floor - stamps_);
    } else
      gap(at, 0, at, c.pending[i]);  // one stream cannot tell consecutive waits apart: the first takes the gap
  }
  c.pending.clear();
}

void TimerSet::finish_stalls() {
  for (auto& kv : clocks_) {
    TaskClock& c = kv.second;
    if (c.pending.empty() || !enabled_) continue;
    uint64_t* st = slot();
    dev_.stamp(*kv.first, st);
    close_pending(c, st);
  }
  clocks_.clear();  // the next iteration's first wait has no task before it
  origin_ = nullptr;
  origin_start_ = nullptr;
}

uint64_t* TimerSet::slot() {
  DLNB_REQUIRE(next_ < cap_, "too many timer stamps in one iteration");
  return stamps_ + next_++;
}

void TimerSet::gap(const uint64_t* prev_start, uint64_t prev_ticks, const uint64_t* next_start,
                   const std::string& name, bool clamp) {
  if (!enabled_ || !prev_start || !next_start) return;
  gaps_.push_back(
      Gap{static_cast<int>(prev_start - stamps_), static_cast<int>(next_start - stamps_), prev_ticks, name, clamp, -1});
}

void TimerSet::add(const std::string& name, double seconds) {
  if (capturing_) {
    captured_adds_.emplace_back(name, seconds);
    return;
  }
  if (enabled_) vals_[name].push_back(seconds);
}

void TimerSet::begin_capture() {
  clocks_.clear();
  origin_ = nullptr;
  origin_start_ = nullptr;
  pending_.clear();
  gaps_.clear();
  next_ = 0;
  captured_adds_.clear();
  capturing_ = true;
}

void TimerSet::end_capture() {
  capturing_ = false;
  frozen_ = true;
}

void TimerSet::ensure(const std::string& name) { vals_[name]; }

void TimerSet::resolve() {
  // Called after the streams were synchronised: every stamp has landed.
  const double hz = dev_.stamp_hz();
  if (frozen_ && enabled_)
    for (const auto& a : captured_adds_) vals_[a.first].push_back(a.second);
  // Every interval here is causally ordered (a stall ends after the task or
  // stamp it is timed from; a collective ends after it began): a negative one
  // means mis-ordered stamps. It is recorded as 0 and counted
  // (negatives_json()), never silently clamped.
  auto put = [&](const std::string& name, uint64_t a, uint64_t b, bool clamp = false) {
    if (!enabled_) return;
    if (b >= a || clamp) {  // (clamp: a gap whose ends are not ordered, TimerSet::gap)
      vals_[name].push_back(b >= a ? static_cast<double>(b - a) / hz : 0.0);
      return;
    }
    vals_[name].push_back(0.0);
    Negative& n = negatives_[name];
    ++n.count;
    n.worst_s = std::max(n.worst_s, static_cast<double>(a - b) / hz);
  };
  for (const auto& p : pending_)
    put(p.name, __atomic_load_n(stamps_ + p.a, __ATOMIC_ACQUIRE), __atomic_load_n(stamps_ + p.b, __ATOMIC_ACQUIRE));
  for (const auto& g : gaps_) {
    uint64_t a = __atomic_load_n(stamps_ + g.prev, __ATOMIC_ACQUIRE) + g.prev_ticks;
    if (g.floor >= 0) a = std::max(a, __atomic_load_n(stamps_ + g.floor, __ATOMIC_ACQUIRE));
    put(g.name, a, __atomic_load_n(stamps_ + g.next, __ATOMIC_ACQUIRE), g.clamp);
  }
  if (frozen_) return;  // the same stamps are rewritten by the next replay
  pending_.clear();
  gaps_.clear();
  next_ = 0;
}

void TimerSet::clear() {
  if (!frozen_) {
    pending_.clear();
    gaps_.clear();
    next_ = 0;
  }
  for (auto& kv : vals_) kv.second.clear();
  negatives_.clear();
}

Json TimerSet::negatives_json() const {
  Json j = Json::object();
  for (const auto& kv : negatives_) {
    Json e = Json::object();
    e["count"] = static_cast<double>(kv.second.count);
    e["worst_ms"] = kv.second.worst_s * 1e3;
    j[kv.first] = e;
  }
  return j;
}

const std::vector<double>& TimerSet::get(const std::string& name) const {
  static const std::vector<double> empty;
  auto it = vals_.find(name);
  return it == vals_.end() ? empty : it->second;
}

double TimerSet::sum(const std::string& name) const {
  double s = 0;
  for (double v : get(name)) s += v;
  return s;
}

Json TimerSet::values_json(const std::string& name) const { return Json(get(name)); }

}  // namespace dlnb
