// Loopback backend: every rank of the job is a thread of one process, all on
// one device (a GPU, or the CPU device for GPU-less tests).
//
// the reference's only way to run N ranks without N
// devices is `mpirun -n N` on the mpi_cpu build (README.md:96); RCCL refuses
// two ranks on one GPU. Here N "ranks" share the process, so the same
// strategy code, timers and report run N-wide on a single MI355X (or on the
// CPU) without IPC, shared memory segments or RCCL.
//
// Ordering. A collective is issued by the LAST member to arrive: its stream
// waits on every other member's "ready" event (recorded when that member
// called in), runs the data movement (one fp32-accumulating multi-source /
// multi-destination kernel on the GPU, host loops on the CPU device) and
// records the group's "done" event; the other members block on the host until
// then and make their streams wait on "done". Point-to-point messages are
// matched FIFO per (src, dst) channel; the member whose post completes the
// match issues the copy on its own stream. Every wait therefore refers to work
// that was enqueued earlier in host time, so there is no cycle even when the
// ranks' streams share the device's (4) hardware queues - the failure mode of
// device-side spin-waits between streams of one process.
//
// Host-level rendezvous is stricter than RCCL's stream-level one: a rank
// blocked in a collective enqueues nothing else. Operations between
// group_start()/group_end() are posted without blocking and completed
// together at group_end(), which is how the strategies issue paired
// send/recv exchanges.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <sstream>

#include "dlnb/comm.hpp"
#include "dlnb/xgmi.hpp"

namespace dlnb {

namespace {

constexpr size_t kRing = 64;  // done events per P2P channel (messages in flight per group)

struct Post {
  const char* send = nullptr;
  char* recv = nullptr;
  size_t bytes = 0;
  Stream* stream = nullptr;
  Event* ready = nullptr;
  uint64_t seq = 0;  // message index on its channel
};

struct Channel {  // src -> dst
  std::deque<Post> sends, recvs;
  uint64_t posted_send = 0, posted_recv = 0, matched = 0;
  std::vector<std::unique_ptr<Event>> done;  // ring of kRing, by message index
};

struct CollArg {
  const char* send;
  char* recv;
  size_t count;
  DType t;
  CollKind kind;
  Stream* stream;
  Event* ready;
};

struct Group {
  int n = 0;
  std::vector<int> members;
  // collectives
  uint64_t issued = 0;
  int arrived = 0;
  std::vector<CollArg> args;
  std::unique_ptr<Event> done;
  // point-to-point
  std::vector<Channel> chans;  // [src * n + dst]
  Channel& chan(int src, int dst) { return chans[static_cast<size_t>(src) * n + dst]; }
};

const char* kind_name(CollKind k) {
  switch (k) {
    case CollKind::AllReduce: return "all_reduce";
    case CollKind::AllGather: return "all_gather";
    case CollKind::ReduceScatter: return "reduce_scatter";
    case CollKind::AllToAll: return "all_to_all";
    default: return "send/recv";
  }
}

}  // namespace

struct LoopbackHub {
  int ranks = 1;
  double timeout_s = 900;
  std::mutex mu;
  std::condition_variable cv;
  bool aborted = false;
  std::string why;
  std::map<std::string, std::weak_ptr<Group>> groups;
  AbortFlag cpu_abort = std::make_shared<std::atomic<bool>>(false);
  int drained = 0;  // rank threads done with the job (loopback_drained)

  // Waits (mu held) until pred() holds; throws on abort or timeout.
  template <typename Pred>
  void wait(std::unique_lock<std::mutex>& g, Pred pred, const std::string& what) {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
    while (!pred()) {
      if (aborted) DLNB_THROW("loopback: " << what << " abandoned: " << why);
      if (cv.wait_until(g, deadline) == std::cv_status::timeout && !pred()) {
        aborted = true;
        why = what + " timed out";
        cv.notify_all();
        DLNB_THROW("loopback: timeout after " << timeout_s << " s in " << what);
      }
    }
  }
};

std::shared_ptr<LoopbackHub> make_loopback_hub(int ranks, double timeout_s) {
  DLNB_REQUIRE(ranks >= 1 && ranks <= xgmi::kMaxLocal, "loopback: 1.." << xgmi::kMaxLocal << " ranks, got " << ranks);
  auto h = std::make_shared<LoopbackHub>();
  h->ranks = ranks;
  h->timeout_s = timeout_s;
  return h;
}

AbortFlag loopback_cpu_abort_flag(LoopbackHub& hub) { return hub.cpu_abort; }

void loopback_drained(LoopbackHub& hub, bool wait, double timeout_s) {
  std::unique_lock<std::mutex> g(hub.mu);
  ++hub.drained;
  hub.cv.notify_all();
  if (wait)
    hub.cv.wait_for(g, std::chrono::duration<double>(timeout_s), [&] { return hub.drained >= hub.ranks; });
}

void loopback_abort(LoopbackHub& hub, const std::string& why) {
  hub.cpu_abort->store(true);  // loopback-cpu: release worker threads blocked on the failed rank's events
  std::lock_guard<std::mutex> g(hub.mu);
  if (!hub.aborted) {
    hub.aborted = true;
    hub.why = why;
  }
  hub.cv.notify_all();
}

namespace {

// dsts[d][i] = sum_s srcs[s][i] on stream s of device dev.
void move(Device& dev, Stream& s, const std::vector<char*>& dsts, const std::vector<const char*>& srcs, size_t count,
          DType t) {
  if (count == 0 || dsts.empty()) return;
  if (dev.kind() == DeviceKind::GPU) {
    if (srcs.size() == 1 && dsts.size() == 1) {
      if (dsts[0] != srcs[0]) dev.copy_async(dsts[0], srcs[0], count * dtype_size(t), s);
      return;
    }
    xgmi::launch_local_reduce(dsts.data(), static_cast<int>(dsts.size()), srcs.data(), static_cast<int>(srcs.size()),
                              count, t, s.native());
    return;
  }
  dev.host_task(s, [dsts, srcs, count, t] {
    const size_t bytes = count * dtype_size(t);
    if (srcs.size() == 1) {
      for (char* d : dsts)
        if (d != srcs[0]) host_copy(d, srcs[0], bytes);
      return;
    }
    host_reduce_sum(t, dsts[0], srcs, count);
    for (size_t i = 1; i < dsts.size(); ++i) host_copy(dsts[i], dsts[0], bytes);
  });
}

class LoopbackComm : public Communicator {
 public:
  LoopbackComm(std::shared_ptr<LoopbackHub> hub, std::shared_ptr<Group> g, Device& dev, const std::string& name,
               const std::vector<int>& members, int world_rank)
      : hub_(std::move(hub)), g_(std::move(g)), dev_(dev) {
    name_ = name;
    members_ = members;
    size_ = static_cast<int>(members.size());
    rank_ = -1;
    for (int i = 0; i < size_; ++i)
      if (members[static_cast<size_t>(i)] == world_rank) rank_ = i;
    DLNB_REQUIRE(rank_ >= 0, "loopback: rank " << world_rank << " is not a member of group " << name);
    coll_ready_ = dev_.create_event(false);
  }
  std::string backend_name() const override { return "LOOPBACK"; }

  void all_reduce(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    collective(CollKind::AllReduce, send, recv, count, t, s);
  }
  void all_gather(const void* send, void* recv, size_t send_count, DType t, Stream& s) override {
    collective(CollKind::AllGather, send, recv, send_count, t, s);
  }
  void reduce_scatter(const void* send, void* recv, size_t recv_count, DType t, Stream& s) override {
    collective(CollKind::ReduceScatter, send, recv, recv_count, t, s);
  }
  void all_to_all(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    DLNB_REQUIRE(send != recv || size_ == 1, "loopback all_to_all is out of place only");
    collective(CollKind::AllToAll, send, recv, count, t, s);
  }
  void send(const void* buf, size_t count, DType t, int peer, Stream& s) override {
    post(true, const_cast<void*>(buf), count * dtype_size(t), peer, s);
  }
  void recv(void* buf, size_t count, DType t, int peer, Stream& s) override {
    post(false, buf, count * dtype_size(t), peer, s);
  }
  void group_start() override { ++in_group_; }
  void group_end() override {
    DLNB_REQUIRE(in_group_ > 0, "loopback: group_end without group_start");
    if (--in_group_ == 0) complete(pending_);
  }
  std::string async_error() override {
    std::lock_guard<std::mutex> g(hub_->mu);
    return hub_->aborted ? hub_->why : "";
  }
  void abort() override { loopback_abort(*hub_, "communicator " + name_ + " aborted by rank " + std::to_string(rank_)); }

 private:
  struct Pending {
    bool is_send;
    int peer;
    uint64_t seq;
    Stream* stream;
  };

  void collective(CollKind kind, const void* send, void* recv, size_t count, DType t, Stream& s) {
    s.record(*coll_ready_);
    std::unique_lock<std::mutex> lk(hub_->mu);
    Group& g = *g_;
    const uint64_t me = g.issued;
    g.args[static_cast<size_t>(rank_)] = {static_cast<const char*>(send), static_cast<char*>(recv), count, t, kind, &s,
                                          coll_ready_.get()};
    if (++g.arrived < g.n) {
      hub_->wait(lk, [&] { return g.issued > me; }, name_ + " " + kind_name(kind));
      lk.unlock();
      s.wait(*g.done);
      return;
    }
    for (int i = 0; i < g.n; ++i) {
      const CollArg& a = g.args[static_cast<size_t>(i)];
      if (a.kind != kind || a.count != count || a.t != t) {
        std::ostringstream os;
        os << "loopback: mismatched collectives on " << name_ << ": rank " << i << " called " << kind_name(a.kind)
           << " x" << a.count << ", rank " << rank_ << " " << kind_name(kind) << " x" << count;
        fail(os.str());
      }
      if (i != rank_) s.wait(*a.ready);
    }
    issue(kind, count, t, s);
    s.record(*g.done);
    g.arrived = 0;
    ++g.issued;
    hub_->cv.notify_all();
  }

  void issue(CollKind kind, size_t count, DType t, Stream& s) {
    Group& g = *g_;
    const size_t n = static_cast<size_t>(g.n), blk = count * dtype_size(t);
    std::vector<const char*> srcs;
    std::vector<char*> dsts;
    if (dev_.kind() == DeviceKind::GPU && kind != CollKind::AllReduce && count > 0) {
      // one launch for the whole collective (instead of n or n^2 pieces)
      for (auto& a : g.args) {
        srcs.push_back(a.send);
        dsts.push_back(a.recv);
      }
      const xgmi::LocalColl op = kind == CollKind::AllGather       ? xgmi::LocalColl::AllGather
                                 : kind == CollKind::ReduceScatter ? xgmi::LocalColl::ReduceScatter
                                                                   : xgmi::LocalColl::AllToAll;
      xgmi::launch_local_coll(op, dsts.data(), srcs.data(), g.n, count, t, s.native());
      return;
    }
    switch (kind) {
      case CollKind::AllReduce:
        for (auto& a : g.args) {
          srcs.push_back(a.send);
          dsts.push_back(a.recv);
        }
        move(dev_, s, dsts, srcs, count, t);
        break;
      case CollKind::ReduceScatter:
        for (size_t j = 0; j < n; ++j) {
          srcs.clear();
          for (auto& a : g.args) srcs.push_back(a.send + j * blk);
          move(dev_, s, {g.args[j].recv}, srcs, count, t);
        }
        break;
      case CollKind::AllGather:
        for (size_t i = 0; i < n; ++i) {
          dsts.clear();
          for (auto& a : g.args) dsts.push_back(a.recv + i * blk);
          move(dev_, s, dsts, {g.args[i].send}, count, t);
        }
        break;
      case CollKind::AllToAll:
        for (size_t i = 0; i < n; ++i)
          for (size_t j = 0; j < n; ++j) move(dev_, s, {g.args[j].recv + i * blk}, {g.args[i].send + j * blk}, count, t);
        break;
      default: break;
    }
  }

  void post(bool is_send, void* buf, size_t bytes, int peer, Stream& s) {
    DLNB_REQUIRE(peer >= 0 && peer < size_ && peer != rank_, "loopback: bad peer " << peer << " in " << name_);
    if (p2p_ready_.empty())
      for (size_t i = 0; i < kRing; ++i) p2p_ready_.push_back(dev_.create_event(false));
    Event* ready = p2p_ready_[ready_next_++ % kRing].get();
    s.record(*ready);
    uint64_t seq;
    {
      std::lock_guard<std::mutex> lk(hub_->mu);
      Channel& c = is_send ? g_->chan(rank_, peer) : g_->chan(peer, rank_);
      if (c.done.empty())  // first message on this channel
        for (size_t i = 0; i < kRing; ++i) c.done.push_back(dev_.create_event(false));
      Post p;
      p.bytes = bytes;
      p.stream = &s;
      p.ready = ready;
      if (is_send) {
        p.send = static_cast<const char*>(buf);
        p.seq = seq = c.posted_send++;
      } else {
        p.recv = static_cast<char*>(buf);
        p.seq = seq = c.posted_recv++;
      }
      (is_send ? c.sends : c.recvs).push_back(p);
      if (!c.sends.empty() && !c.recvs.empty()) {
        // This post completes the oldest pending message of the channel
        // (FIFO: the other side's front matches our new post).
        Post snd = c.sends.front(), rcv = c.recvs.front();
        c.sends.pop_front();
        c.recvs.pop_front();
        if (snd.bytes != rcv.bytes) {
          std::ostringstream os;
          os << "loopback: " << name_ << " message " << snd.seq << " sent " << snd.bytes << " B but received into "
             << rcv.bytes << " B";
          fail(os.str());
        }
        const Post& other = is_send ? rcv : snd;
        s.wait(*other.ready);
        move(dev_, s, {rcv.recv}, {snd.send}, bytes, DType::FP8_E4M3);  // byte copy
        s.record(*c.done[c.matched % kRing]);
        ++c.matched;
        hub_->cv.notify_all();
      }
    }
    pending_.push_back({is_send, peer, seq, &s});
    if (in_group_ == 0) complete(pending_);
  }

  // Blocks until every posted message is matched, then orders each
  // operation's stream after its copy.
  void complete(std::vector<Pending>& ops) {
    std::vector<Event*> waits;
    {
      std::unique_lock<std::mutex> lk(hub_->mu);
      for (const Pending& p : ops) {
        Channel& c = p.is_send ? g_->chan(rank_, p.peer) : g_->chan(p.peer, rank_);
        hub_->wait(lk, [&] { return c.matched > p.seq; },
                   name_ + (p.is_send ? " send to " : " recv from ") + std::to_string(p.peer));
        waits.push_back(c.done[p.seq % kRing].get());
      }
    }
    for (size_t i = 0; i < ops.size(); ++i) ops[i].stream->wait(*waits[i]);
    ops.clear();
  }

  // mu held: wake every waiting rank with the error, then throw it here.
  [[noreturn]] void fail(const std::string& msg) {
    if (!hub_->aborted) {
      hub_->aborted = true;
      hub_->why = msg;
    }
    hub_->cv.notify_all();
    DLNB_THROW(msg);
  }

  std::shared_ptr<LoopbackHub> hub_;
  std::shared_ptr<Group> g_;
  Device& dev_;
  std::unique_ptr<Event> coll_ready_;
  std::vector<std::unique_ptr<Event>> p2p_ready_;
  size_t ready_next_ = 0;
  int in_group_ = 0;
  std::vector<Pending> pending_;
};

class LoopbackFactory : public CommFactory {
 public:
  LoopbackFactory(HostGroup& world, Device& dev, std::shared_ptr<LoopbackHub> hub)
      : world_(world), dev_(dev), hub_(std::move(hub)) {
    DLNB_REQUIRE(hub_ && hub_->ranks == world.size(), "loopback: hub for " << (hub_ ? hub_->ranks : 0)
                                                                          << " ranks, world of " << world.size());
  }
  std::string backend_name() const override { return "LOOPBACK"; }
  std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members, size_t,
                                       bool, int) override {
    DLNB_REQUIRE(!members.empty() && members.size() <= static_cast<size_t>(xgmi::kMaxLocal),
                 "loopback: group " << name << " of " << members.size() << " ranks");
    std::shared_ptr<Group> g;
    {
      std::lock_guard<std::mutex> lk(hub_->mu);
      auto it = hub_->groups.find(name);
      if (it != hub_->groups.end()) g = it->second.lock();
      if (g) {
        DLNB_REQUIRE(g->members == members, "loopback: group " << name << " created with different members");
      } else {
        g = std::make_shared<Group>();
        g->n = static_cast<int>(members.size());
        g->members = members;
        g->args.resize(members.size());
        g->done = dev_.create_event(false);
        g->chans = std::vector<Channel>(members.size() * members.size());
        hub_->groups[name] = g;
      }
    }
    return std::unique_ptr<Communicator>(new LoopbackComm(hub_, g, dev_, name, members, world_.rank()));
  }

 private:
  HostGroup& world_;
  Device& dev_;
  std::shared_ptr<LoopbackHub> hub_;
};

}  // namespace

std::unique_ptr<CommFactory> make_loopback_factory(HostGroup& world, Device& dev, std::shared_ptr<LoopbackHub> hub) {
  return std::unique_ptr<CommFactory>(new LoopbackFactory(world, dev, std::move(hub)));
}

}  // namespace dlnb
