// Communication fault injection (tests of the exactness checks): a
// decorator around any backend's communicators that corrupts chosen
// operations in ways a collective implementation can really fail.
//
//   DLNB_COMM_FAULT="mode=swap|skip|delay[,us=X][,op=all_reduce|all_gather|reduce_scatter|all_to_all|recv|send|any]
//                    [,rank=R][,call=K][,every=N][,comm=SUBSTR]" (several specs: separated by ';')
//
//   swap: after the operation, exchange two parts of its output on the
//         operation's stream (device copies, captured into a HIP graph like
//         the operation): the blocks of peers 0 and 1 for all-gather /
//         all-to-all, the two halves of the buffer for the others - a peer
//         or offset misroute;
//   skip: the operation is not issued at all, so its output keeps whatever
//         the buffer held (a stale window, a replay whose kernel did not
//         run). Collectives rendezvous, so a skip applies to every rank
//         (rank is ignored) to keep the job from hanging.
//   delay: the operation runs, then an idle kernel of X us on its stream (a
//         collective that took X longer: the exposed-communication timers
//         downstream of it must grow by exactly X where it is on the critical
//         path - VERDICT r5 #2's value tests); a send: the idle kernel before
//         it (the data leaves X late). A recv inside a group: after the group.
//   rank: world rank that corrupts or delays (swap, delay; default every
//   rank); call: the K-th call (from 0) of that op on each matching
//   communicator (default every call), with every=N: calls K, K+N, K+2N, ...
//   (the K-th op of every iteration that issues N); comm: only communicators
//   whose name contains SUBSTR.
//
// The reference has no fault injection; the exactness pass it backs is
// dlnb commtest --suite (bench.py at N > 1, VERDICT r3 "fp8 gate").
#include <algorithm>
#include <iostream>
#include <map>

#include "dlnb/strategy.hpp"

namespace dlnb {

namespace {

struct FaultSpec {
  std::string mode, op = "any", comm;
  int rank = -1;
  long long call = -1, every = 0;
  double us = 0.0;
};

class FaultyCommunicator : public Communicator {
 public:
  FaultyCommunicator(std::unique_ptr<Communicator> in, Device& dev, const std::vector<FaultSpec>& fs,
                     int world_rank, size_t capacity)
      : in_(std::move(in)), dev_(dev), fs_(fs), world_rank_(world_rank) {
    rank_ = in_->rank();
    size_ = in_->size();
    members_ = in_->members();
    name_ = in_->name();
    // the swap scratch exists before any capture (no allocation inside a graph)
    for (const auto& f : fs_)
      if (f.mode == "swap") tmp_ = dev_.alloc(std::max<size_t>(capacity, 64));
  }
  std::string backend_name() const override { return in_->backend_name(); }

  void all_reduce(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    const FaultSpec* f = hit("all_reduce");
    if (!f) return in_->all_reduce(send, recv, count, t, s);
    if (f->mode == "skip") return;
    in_->all_reduce(send, recv, count, t, s);
    if (f->mode == "delay") return delay(*f, s);
    swap_halves(recv, count, t, s);
  }
  void all_gather(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    const FaultSpec* f = hit("all_gather");
    if (!f) return in_->all_gather(send, recv, count, t, s);
    if (f->mode == "skip") return;
    in_->all_gather(send, recv, count, t, s);
    if (f->mode == "delay") return delay(*f, s);
    swap_blocks(recv, count, t, s);
  }
  void reduce_scatter(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    const FaultSpec* f = hit("reduce_scatter");
    if (!f) return in_->reduce_scatter(send, recv, count, t, s);
    if (f->mode == "skip") return;
    in_->reduce_scatter(send, recv, count, t, s);
    if (f->mode == "delay") return delay(*f, s);
    swap_halves(recv, count, t, s);
  }
  void all_to_all(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    const FaultSpec* f = hit("all_to_all");
    if (!f) return in_->all_to_all(send, recv, count, t, s);
    if (f->mode == "skip") return;
    in_->all_to_all(send, recv, count, t, s);
    if (f->mode == "delay") return delay(*f, s);
    swap_blocks(recv, count, t, s);
  }
  void send(const void* buf, size_t count, DType t, int peer, Stream& s) override {
    // a skipped receive skips the matching send too (every rank skips)
    for (const auto& f : fs_)
      if (f.mode == "skip" && matches(f, "recv") && call_hit(f, sends_)) {
        ++sends_;
        return;
      }
    ++sends_;
    // a delayed send leaves late: the idle kernel goes before it (inside a
    // group: before the group's kernel, which launches at its end)
    const FaultSpec* f = hit("send");
    if (f && f->mode == "delay") dev_.idle(s, f->us);
    in_->send(buf, count, t, peer, s);
  }
  void recv(void* buf, size_t count, DType t, int peer, Stream& s) override {
    const FaultSpec* f = hit("recv");
    if (!f) return in_->recv(buf, count, t, peer, s);
    if (f->mode == "skip") return;
    in_->recv(buf, count, t, peer, s);
    if (f->mode == "delay") return delay(*f, s);
    pending_.push_back({buf, count, t, &s});  // swapped once the group completes
    if (depth_ == 0) flush();
  }
  void group_start() override {
    ++depth_;
    in_->group_start();
  }
  void group_end() override {
    in_->group_end();
    if (--depth_ == 0) flush();
  }
  bool wants_peer_buffers() const override { return in_->wants_peer_buffers(); }
  void register_buffer(void* p, size_t bytes) override { in_->register_buffer(p, bytes); }
  std::string async_error() override { return in_->async_error(); }
  void abort() override { in_->abort(); }
  int library_nranks() override { return in_->library_nranks(); }

 private:
  bool matches(const FaultSpec& f, const char* op) const {
    return (f.op == "any" || f.op == op) && (f.comm.empty() || name_.find(f.comm) != std::string::npos);
  }
  static bool call_hit(const FaultSpec& f, long long k) {
    if (f.call < 0) return true;
    return f.every > 0 ? k % f.every == f.call : k == f.call;
  }
  // The spec (if any) that hits this call of `op` (each op's calls counted once).
  const FaultSpec* hit(const char* op) {
    const long long k = calls_[op]++;
    for (const auto& f : fs_) {
      if (!matches(f, op) || !call_hit(f, k)) continue;
      if (f.mode == "skip" && std::string(op) == "send") continue;  // (skips are keyed on the recv)
      if ((f.mode == "swap" || f.mode == "delay") && f.rank >= 0 && f.rank != world_rank_) continue;
      if (!announced_[&f - fs_.data()]++) {
        std::cerr << "[dlnb] DLNB_COMM_FAULT: " << f.mode << " on " << op << " of " << name_ << " (call " << k
                  << ", rank " << world_rank_ << ")" << std::endl;
      }
      return &f;
    }
    return nullptr;
  }
  // the delay: an idle kernel after the operation (after the group it is in)
  void delay(const FaultSpec& f, Stream& s) {
    if (depth_ > 0) {
      delays_.push_back({f.us, &s});
      return;
    }
    dev_.idle(s, f.us);
  }
  void* scratch(size_t bytes) {
    DLNB_REQUIRE(tmp_.bytes() >= bytes, "DLNB_COMM_FAULT swap: " << bytes << " B exceed the communicator's capacity");
    return tmp_.data();
  }
  void exchange(char* a, char* b, size_t bytes, Stream& s) {
    if (bytes == 0 || a == b) return;
    void* t = scratch(bytes);
    dev_.copy_async(t, a, bytes, s);
    dev_.copy_async(a, b, bytes, s);
    dev_.copy_async(b, t, bytes, s);
  }
  void swap_blocks(void* recv, size_t count, DType t, Stream& s) {
    if (size_ < 2) return swap_halves(recv, count, t, s);
    const size_t b = count * dtype_size(t);
    exchange(static_cast<char*>(recv), static_cast<char*>(recv) + b, b, s);
  }
  void swap_halves(void* buf, size_t count, DType t, Stream& s) {
    const size_t h = count / 2 * dtype_size(t);
    exchange(static_cast<char*>(buf), static_cast<char*>(buf) + h, h, s);
  }
  void flush() {
    for (auto& p : pending_) swap_halves(p.buf, p.count, p.t, *p.s);
    pending_.clear();
    for (auto& d : delays_) dev_.idle(*d.second, d.first);
    delays_.clear();
  }

  struct Pending {
    void* buf;
    size_t count;
    DType t;
    Stream* s;
  };
  std::unique_ptr<Communicator> in_;
  Device& dev_;
  std::vector<FaultSpec> fs_;
  int world_rank_;
  std::map<std::string, long long> calls_;
  long long sends_ = 0;
  int depth_ = 0;
  std::map<long, long> announced_;
  std::vector<Pending> pending_;
  std::vector<std::pair<double, Stream*>> delays_;
  Buffer tmp_;
};

class FaultyFactory : public CommFactory {
 public:
  FaultyFactory(std::unique_ptr<CommFactory> in, Device& dev, std::vector<FaultSpec> f, int world_rank)
      : in_(std::move(in)), dev_(dev), f_(std::move(f)), world_rank_(world_rank) {}
  std::string backend_name() const override { return in_->backend_name(); }
  std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members,
                                       size_t capacity_bytes, bool need_p2p, int max_ctas) override {
    return std::make_unique<FaultyCommunicator>(in_->create(name, members, capacity_bytes, need_p2p, max_ctas), dev_,
                                                f_, world_rank_, capacity_bytes);
  }

 private:
  std::unique_ptr<CommFactory> in_;
  Device& dev_;
  std::vector<FaultSpec> f_;
  int world_rank_;
};

}  // namespace

std::unique_ptr<CommFactory> wrap_comm_faults(std::unique_ptr<CommFactory> inner, Device& dev, int world_rank) {
  const std::string spec = env_or("DLNB_COMM_FAULT", "");
  if (spec.empty()) return inner;
  std::vector<FaultSpec> fs;
  for (auto& one : split(spec, ';')) {
    if (trim(one).empty()) continue;
    FaultSpec f;
    for (auto& kv : split(trim(one), ',')) {
      auto p = split(trim(kv), '=');
      DLNB_REQUIRE(p.size() == 2, "DLNB_COMM_FAULT: expected key=value, got '" << kv << "'");
      if (p[0] == "mode") f.mode = p[1];
      else if (p[0] == "op") f.op = p[1];
      else if (p[0] == "rank") f.rank = std::stoi(p[1]);
      else if (p[0] == "call") f.call = std::stoll(p[1]);
      else if (p[0] == "every") f.every = std::stoll(p[1]);
      else if (p[0] == "comm") f.comm = p[1];
      else if (p[0] == "us") f.us = std::stod(p[1]);
      else DLNB_THROW("DLNB_COMM_FAULT: unknown key '" << p[0] << "'");
    }
    DLNB_REQUIRE(f.mode == "swap" || f.mode == "skip" || f.mode == "delay",
                 "DLNB_COMM_FAULT: mode must be swap, skip or delay");
    DLNB_REQUIRE(f.op == "any" || f.op == "all_reduce" || f.op == "all_gather" || f.op == "reduce_scatter" ||
                     f.op == "all_to_all" || f.op == "recv" || f.op == "send",
                 "DLNB_COMM_FAULT: unknown op '" << f.op << "'");
    DLNB_REQUIRE(f.mode != "delay" || f.us > 0, "DLNB_COMM_FAULT: mode=delay needs us=X > 0");
    DLNB_REQUIRE(f.op != "send" || f.mode == "delay", "DLNB_COMM_FAULT: op=send only for mode=delay");
    fs.push_back(f);
  }
  DLNB_REQUIRE(!fs.empty(), "DLNB_COMM_FAULT: no spec in '" << spec << "'");
  return std::make_unique<FaultyFactory>(std::move(inner), dev, fs, world_rank);
}

}  // namespace dlnb
