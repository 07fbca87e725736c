#include "dlnb/timers.hpp"

namespace dlnb {

int TimerSet::begin(Stream& s) {
  if (!enabled_) return -1;
  if (next_ == pool_.size()) pool_.push_back(dev_.create_event(true));
  int idx = static_cast<int>(next_++);
  s.record(*pool_[static_cast<size_t>(idx)]);
  return idx;
}

void TimerSet::end(int token, Stream& s, const std::string& name) {
  if (!enabled_ || token < 0) return;
  if (next_ == pool_.size()) pool_.push_back(dev_.create_event(true));
  int idx = static_cast<int>(next_++);
  s.record(*pool_[static_cast<size_t>(idx)]);
  pending_.push_back(Pending{token, idx, name});
}

void TimerSet::stall(Stream& s, Event& e, const std::string& name) {
  int t = begin(s);
  s.wait(e);
  end(t, s, name);
}

void TimerSet::add(const std::string& name, double seconds) {
  if (enabled_) vals_[name].push_back(seconds);
}

void TimerSet::ensure(const std::string& name) { vals_[name]; }

void TimerSet::resolve() {
  for (const auto& p : pending_) {
    double ms = dev_.elapsed_ms(*pool_[static_cast<size_t>(p.a)], *pool_[static_cast<size_t>(p.b)]);
    vals_[p.name].push_back(ms * 1e-3);
  }
  pending_.clear();
  next_ = 0;
}

void TimerSet::clear() {
  pending_.clear();
  next_ = 0;
  for (auto& kv : vals_) kv.second.clear();
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
