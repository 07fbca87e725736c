// "mixed" backend: size-based dispatch between RCCL and our xgmi kernels.
//
// Every group gets an RCCL communicator; groups whose members share one node
// also get an xgmi communicator with windows sized to the dispatch threshold.
// A single-node group whose largest message (the capacity the strategy
// declares) fits under the threshold gets the xgmi communicator only (every
// operation would go there anyway); that is also what lets the dispatcher run
// with several ranks on one GPU, which RCCL refuses.
// Each operation goes to xgmi when its per-rank message is at most
// DLNB_MIXED_XGMI_MAX_KB (default 2048 KiB: the latency-bound range, where a
// one-shot kernel that writes to all 7 peers at once and exchanges one flag
// per block avoids RCCL's per-step protocol), otherwise to RCCL (large,
// bandwidth-bound messages). Point-to-point operations issued between
// group_start() and group_end() are held back and all go to one backend,
// chosen by the largest message of the group, so a group never straddles
// two communicators.
//
// Both communicators of a group issue in the caller's stream order, and the
// choice depends only on message sizes, which every member sees identically,
// so all members route every operation the same way (each backend's
// per-communicator sequence stays consistent across ranks).
//
// Reference equivalent: none (the reference picks one library at compile
// time, Makefile.flags.mk:74-114); the ops replaced are
// cpp/proxy_classes.hpp:149-227.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <sstream>

#include "dlnb/comm.hpp"

namespace dlnb {

namespace {

class MixedComm : public Communicator {
 public:
  MixedComm(std::unique_ptr<Communicator> big, std::unique_ptr<Communicator> small, size_t max_small)
      : big_(std::move(big)), small_(std::move(small)), max_small_(max_small) {
    Communicator& any = big_ ? *big_ : *small_;
    name_ = any.name();
    members_ = any.members();
    rank_ = any.rank();
    size_ = any.size();
  }
  std::string backend_name() const override { return !small_ ? "RCCL" : big_ ? "RCCL+XGMI" : "XGMI"; }

  void all_reduce(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    pick(count * dtype_size(t)).all_reduce(send, recv, count, t, s);
  }
  void all_gather(const void* send, void* recv, size_t send_count, DType t, Stream& s) override {
    pick(send_count * dtype_size(t)).all_gather(send, recv, send_count, t, s);
  }
  void reduce_scatter(const void* send, void* recv, size_t recv_count, DType t, Stream& s) override {
    pick(recv_count * dtype_size(t)).reduce_scatter(send, recv, recv_count, t, s);
  }
  void all_to_all(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    // in place: RCCL when there is one (xgmi stages in-place all-to-alls
    // through its windows, never the zero-copy path)
    Communicator& c = send == recv && big_ ? *big_ : pick(count * dtype_size(t));
    c.all_to_all(send, recv, count, t, s);
  }
  void send(const void* buf, size_t count, DType t, int peer, Stream& s) override {
    p2p(P2P{true, const_cast<void*>(buf), count, t, peer, &s});
  }
  void recv(void* buf, size_t count, DType t, int peer, Stream& s) override { p2p(P2P{false, buf, count, t, peer, &s}); }
  void group_start() override { in_group_ = true; }
  void group_end() override {
    in_group_ = false;
    std::vector<P2P> ops;
    ops.swap(pending_);
    if (ops.empty()) return;
    size_t mx = 0;
    for (const P2P& o : ops) mx = std::max(mx, o.count * dtype_size(o.t));
    Communicator& c = pick(mx);
    c.group_start();
    for (const P2P& o : ops) issue(c, o);
    c.group_end();
  }
  std::string async_error() override {
    std::string e = big_ ? big_->async_error() : "";
    if (e.empty() && small_) e = small_->async_error();
    return e;
  }
  void abort() override {
    if (big_) big_->abort();
    if (small_) small_->abort();
  }
  int library_nranks() override { return big_ ? big_->library_nranks() : -1; }

 private:
  struct P2P {
    bool is_send;
    void* buf;
    size_t count;
    DType t;
    int peer;
    Stream* s;
  };
  // (no RCCL side: the group's messages all fit the threshold; the xgmi
  // communicator still cuts a larger one into window pieces)
  Communicator& pick(size_t bytes) { return small_ && (bytes <= max_small_ || !big_) ? *small_ : *big_; }
  static void issue(Communicator& c, const P2P& o) {
    if (o.is_send)
      c.send(o.buf, o.count, o.t, o.peer, *o.s);
    else
      c.recv(o.buf, o.count, o.t, o.peer, *o.s);
  }
  void p2p(const P2P& o) {
    if (in_group_) {
      pending_.push_back(o);
      return;
    }
    issue(pick(o.count * dtype_size(o.t)), o);
  }

  std::unique_ptr<Communicator> big_, small_;
  size_t max_small_;
  bool in_group_ = false;
  std::vector<P2P> pending_;
};

class MixedFactory : public CommFactory {
 public:
  MixedFactory(HostGroup& world, Device& dev)
      : world_(world), rccl_(make_rccl_factory(world, dev)), xgmi_(make_xgmi_factory(world, dev)) {
    max_small_ = static_cast<size_t>(std::max<long long>(0, env_int("DLNB_MIXED_XGMI_MAX_KB", 2048))) << 10;
  }
  std::string backend_name() const override { return "RCCL+XGMI"; }
  std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members, size_t capacity_bytes,
                                       bool need_p2p, int max_ctas) override {
    std::unique_ptr<Communicator> big, small;
    if (max_small_ > 0 && members.size() > 1 && one_node(name, members))
      small = xgmi_->create("mixed/" + name, members, std::min(capacity_bytes, max_small_), need_p2p, max_ctas);
    if (!small || capacity_bytes > max_small_) big = rccl_->create(name, members, capacity_bytes, need_p2p, max_ctas);
    return std::unique_ptr<Communicator>(new MixedComm(std::move(big), std::move(small), max_small_));
  }

 private:
  // Every member publishes its host name; the group is single-node iff all
  // agree (identical answer on every member).
  bool one_node(const std::string& name, const std::vector<int>& members) {
    std::ostringstream key;
    key << "mixed/" << name << "/";
    for (int m : members) key << m << ",";
    const std::string me = get_hostname();
    world_.store().set(key.str() + "host/" + std::to_string(world_.rank()), me);
    bool same = true;
    for (int m : members) same = same && world_.store().get(key.str() + "host/" + std::to_string(m)) == me;
    return same;
  }

  HostGroup& world_;
  std::unique_ptr<CommFactory> rccl_, xgmi_;
  size_t max_small_ = 0;
};

}  // namespace

std::unique_ptr<CommFactory> make_mixed_factory(HostGroup& world, Device& dev) {
  return std::unique_ptr<CommFactory>(new MixedFactory(world, dev));
}

}  // namespace dlnb
