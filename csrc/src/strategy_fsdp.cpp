// Fully sharded data parallelism (FSDP) and hybrid sharding (HSDP).
//
// Reference: cpp/data_parallel/fsdp.cpp. The model is split into U units;
// each unit's parameters are sharded over F ranks (unit group = contiguous
// blocks of F ranks, rank / F; replica group = rank % F, fsdp.cpp:258-265).
// Per iteration (run_fsdp, fsdp.cpp:73-163):
//   forward : all-gather unit 0; for each unit, prefetch-all-gather the next
//             unit while computing this one;
//   backward: prefetch-all-gather unit u-1 while computing unit u, then
//             reduce-scatter unit u's gradient, then (W/F > 1) all-reduce the
//             shard across replicas.
// Shard size = ceil((P/U)/F) per unit (fsdp.cpp:244-255).
//
// MI355X design:
//   * collectives are stream-ordered behind events, never host-blocking, so
//     the reduce-scatter of unit u and the all-gather prefetch of unit u-2
//     run under the backward of unit u-1 (the reference blocks the host on
//     every reduce-scatter). By default (--comm-lanes single) all of a rank's
//     collectives go through ONE high-priority stream and ONE unit
//     communicator in the same program order on every rank: at most one RCCL
//     kernel per rank is in flight, so kernels of different communicators can
//     never hold CUs while waiting on each other across GPUs (the multi-
//     communicator deadlock RCCL/NCCL warn about). At 8 GPUs a 0.5 GB
//     all-gather is ~1.5 ms against ~29 ms of compute per unit, so
//     serialising the lanes costs nothing. --comm-lanes split gives
//     all-gather, reduce-scatter and replica all-reduce their own
//     communicator + stream (concurrent, for experiments);
//   * gathered parameters and full gradients are double-buffered (the
//     reference gathers into a single buffer that the in-flight prefetch and
//     the reduce-scatter share, a race - SURVEY.md §3.2); buffer reuse is
//     ordered by events;
//   * buffers are exactly sized in the wire dtype: llama3_8b at F=8 needs
//     2x shards (2 GB) + 4 unit buffers (2 GB) on a 288 GB MI355X.
#include "dlnb/strategy.hpp"

namespace dlnb {

namespace {

class Fsdp : public Strategy {
 public:
  void setup(Context& ctx) override {
    ctx_ = &ctx;
    const auto& o = ctx.opt;
    const auto& st = ctx.stats;
    U_ = o.num_units;
    F_ = o.sharding_factor;
    const int W = ctx.world();
    DLNB_REQUIRE(W % F_ == 0, "world size " << W << " must be divisible by sharding_factor " << F_);
    R_ = W / F_;
    P_ = st.model_size;
    DLNB_REQUIRE(P_ >= static_cast<uint64_t>(U_), "num_units exceeds the parameter count");
    uint64_t base = P_ / U_, rem = P_ % U_;
    for (int u = 0; u < U_; ++u) {
      uint64_t pu = base + (static_cast<uint64_t>(u) < rem ? 1 : 0);
      shard_.push_back(pu / F_ + (pu % F_ ? 1 : 0));
    }
    max_shard_ = shard_[0];
    fwd_us_ = st.avg_forward_time_us / U_;
    bwd_us_ = st.avg_backward_time_us / U_;
    fwd_flops_ = st.forward_flops / U_;
    bwd_flops_ = st.backward_flops / U_;
    reference_ = o.schedule == "reference";

    Device& dev = *ctx.dev;
    es_ = dtype_size(ctx.wire);
    const int rank = ctx.rank();
    std::vector<int> unit_members, rep_members;
    for (int r = 0; r < W; ++r) {
      if (r / F_ == rank / F_) unit_members.push_back(r);
      if (r % F_ == rank % F_) rep_members.push_back(r);
    }
    const size_t unit_bytes = max_shard_ * F_ * es_;
    const bool split = o.comm_lanes == "split";
    auto own_comm = [&](std::unique_ptr<Communicator> c) {
      comms_.push_back(std::move(c));
      return comms_.back().get();
    };
    auto own_stream = [&](std::unique_ptr<Stream> s) {
      lanes_.push_back(std::move(s));
      return lanes_.back().get();
    };
    ag_comm_ = own_comm(ctx.comms->create("fsdp/unit/" + std::to_string(rank / F_), unit_members, unit_bytes, false, ctx.lane_ctas));
    rs_comm_ = split ? own_comm(ctx.comms->create("fsdp/unit_rs/" + std::to_string(rank / F_), unit_members,
                                                  unit_bytes, false, ctx.lane_ctas))
                     : ag_comm_;
    if (R_ > 1)
      ar_comm_ = own_comm(
          ctx.comms->create("fsdp/replica/" + std::to_string(rank % F_), rep_members, max_shard_ * es_, false, ctx.lane_ctas));

    compute_ = dev.create_stream(false);
    ag_stream_ = own_stream(dev.create_stream(true));
    rs_stream_ = split ? own_stream(dev.create_stream(true)) : ag_stream_;
    if (R_ > 1) ar_stream_ = split ? own_stream(dev.create_stream(true)) : ag_stream_;

    for (int u = 0; u < U_; ++u) {
      params_.push_back(dev.alloc(shard_[u] * es_));
      grads_.push_back(dev.alloc(shard_[u] * es_));
      dev.fill_random(params_.back().data(), shard_[u], ctx.wire, 2000 + u, *compute_);
    }
    // Zero-copy: with a backend that moves data with its own kernels (xgmi),
    // peers write their shards straight into the gather buffers and read
    // their blocks straight out of the full-gradient buffers.
    const bool ag_peer = ag_comm_->wants_peer_buffers(), rs_peer = rs_comm_->wants_peer_buffers();
    for (int b = 0; b < 2; ++b) {
      gathered_[b] = ag_peer ? dev.alloc_peer(unit_bytes) : dev.alloc(unit_bytes);
      full_grad_[b] = rs_peer ? dev.alloc_peer(unit_bytes) : dev.alloc(unit_bytes);
      dev.fill_random(full_grad_[b].data(), max_shard_ * F_, ctx.wire, 3000 + b, *compute_);
      if (ag_peer) ag_comm_->register_buffer(gathered_[b].data(), unit_bytes);
      if (rs_peer) rs_comm_->register_buffer(full_grad_[b].data(), unit_bytes);
    }
    auto mk = [&](std::vector<std::unique_ptr<Event>>& v) {
      for (int u = 0; u < U_; ++u) v.push_back(dev.create_event());
    };
    mk(ag_f_);
    mk(fwd_done_);
    mk(ag_b_);
    mk(bwd_done_);
    mk(rs_done_);
    mk(ar_done_);
    // Device gates (ComputeEngine::run_gated): every compute task continues
    // the previous one's deadline unless a collective it depends on finished
    // later - the gate words the collectives' stream raises carry that time -
    // so the compute stays one unbroken stretch of exactly the table time,
    // with a late collective's wait (and only that) added. Without it each of
    // the 64 tasks of a llama3_8b iteration starts after the cross-queue hop
    // of the replayed graph (~10 us) and overshoots by its launch ramp and
    // drain (~13 us): ~1.2 ms per iteration (profiles/timeline_r3.md). The
    // event waits stay: the gate only dates the dependency, the graph edge
    // still orders it (a kernel spinning on a word raised by a node the graph
    // executor queued behind it on the same hardware queue would never
    // finish). DLNB_DEVICE_GATES=0: plain event waits + run_stamped (A/B).
    ComputeEngine& ce = *ctx.compute;
    gated_ = !reference_ && env_int("DLNB_DEVICE_GATES", 1) != 0 && ce.gates_task(fwd_us_) && ce.gates_task(bwd_us_);
    if (gated_) {
      for (int u = 0; u < U_; ++u) {
        g_ag_f_.push_back(ce.make_gate());
        g_ag_b_.push_back(ce.make_gate());
        g_rs_.push_back(ce.make_gate());
      }
    }
    if (o.optimizer) {
      DLNB_REQUIRE(ctx.wire == DType::BF16, "--optimizer needs --wire-dtype bf16");
      for (int u = 0; u < U_; ++u) mom_.push_back(dev.alloc(shard_[u] * es_));
    }
    compute_->synchronize();
    timers_.reset(new TimerSet(dev));
    for (const char* k : {"allgather", "allgather_wait_fwd", "allgather_wait_bwd", "reduce_scatter", "barrier",
                          "allgather_time", "allreduce_time"})
      timers_->ensure(k);
    stats_.push_back({"allgather", CollKind::AllGather, F_, static_cast<double>(unit_bytes), "allgather_time"});
    stats_.push_back({"reduce_scatter", CollKind::ReduceScatter, F_, static_cast<double>(unit_bytes), "reduce_scatter"});
    if (R_ > 1)
      stats_.push_back({"allreduce", CollKind::AllReduce, R_, static_cast<double>(max_shard_ * es_), "allreduce_time"});
  }

  // One unit's compute on the compute stream after waiting for `dep`. When
  // the engine's kernels stamp their own start, the exposed wait is timed as
  // the gap between the previous task's deadline and this task's start (no
  // stamp kernels: each costs a kernel boundary right after a full-chip
  // GEMM); otherwise with a stamp pair around the wait.
  void compute_after(Event* dep, const char* timer, double us, double flops) {
    ComputeEngine& ce = *ctx_->compute;
    if (ce.stamps_task_start()) {
      if (dep) compute_->wait(*dep);
      uint64_t* st = timers_->slot();
      ce.run_stamped(*compute_, us, flops, st);
      if (timer && prev_.slot) timers_->gap(prev_.slot, prev_.ticks, st, timer);
      prev_ = task_mark(ce, *compute_, st, us);
      return;
    }
    if (dep) {
      if (timer)
        timers_->stall_before_task(*compute_, *dep, timer);
      else
        compute_->wait(*dep);
    }
    ce.run(*compute_, us, flops);
  }
  void compute_after(Event& dep, const char* timer, double us, double flops) { compute_after(&dep, timer, us, flops); }

  // The gated form (after the event waits on the gates' collectives): start
  // at max(previous task's deadline, the gates' times); the first task of
  // the iteration is not chained and has no timer.
  void compute_gated(std::vector<int> gates, const char* timer, double us, double flops, Event* done) {
    ComputeEngine& ce = *ctx_->compute;
    uint64_t* st = timers_->slot();
    ce.run_gated(*compute_, us, flops, gates, st, prev_.slot != nullptr, done);
    if (timer && prev_.slot) timers_->gap(prev_.slot, prev_.ticks, st, timer);
    prev_ = task_mark(ce, *compute_, st, us);
  }

  void enqueue_iteration() override {
    Context& ctx = *ctx_;
    const DType t = ctx.wire;
    prev_ = TaskMark();
    tail_end_ = nullptr;

    ComputeEngine& ce = *ctx.compute;
    // Lane graphs (the runner's gate events): a gated task's own gates are
    // its only ordering after the collectives - the compute stream's event
    // waits (and the records nobody else waits for) would add a gate kernel
    // each, on the compute or the comm lane.
    const bool lane = gated_ && ctx.dev->gate_events();
    // ... and the iteration's 64 compute tasks are one compute program (one
    // persistent kernel: no kernel boundary between two tasks)
    const bool prog = lane && ce.begin_program(*compute_);
    auto gather = [&](int u, Event& done, bool first, int gate) {
      int tk = timers_->begin(*ag_stream_);
      ag_comm_->all_gather(params_[u].data(), gathered_[u & 1].data(), shard_[u], t, *ag_stream_);
      timers_->end(tk, *ag_stream_, first ? "allgather" : "allgather_time");
      if (gated_) ce.signal(*ag_stream_, gate);  // before the record: the event implies the gate
      if (!lane) ag_stream_->record(done);
    };

    // ---- forward
    gather(0, *ag_f_[0], true, gated_ ? g_ag_f_[0] : -1);
    if (reference_) ag_stream_->synchronize();  // blocking Allgather (fsdp.cpp:86-91)
    for (int u = 0; u < U_; ++u) {
      if (u + 1 < U_) {
        // gathered[(u+1)&1] was last read by forward(u-1).
        if (u >= 1) ag_stream_->wait(*fwd_done_[u - 1]);
        gather(u + 1, *ag_f_[u + 1], false, gated_ ? g_ag_f_[u + 1] : -1);
      }
      if (gated_) {
        if (!lane) compute_->wait(*ag_f_[u]);
        // fwd_done_[u] recorded by the task itself (lane graphs: raised from its kernel)
        compute_gated({g_ag_f_[u]}, u == 0 ? nullptr : "allgather_wait_fwd", fwd_us_, fwd_flops_,
                      fwd_done_[u].get());
      } else {
        compute_after(*ag_f_[u], u == 0 ? nullptr : "allgather_wait_fwd", fwd_us_, fwd_flops_);
        compute_->record(*fwd_done_[u]);
      }
    }

    // ---- backward (unit U-1's parameters are still gathered)
    for (int u = U_ - 1; u >= 0; --u) {
      if (u - 1 >= 0) {
        // gathered[(u-1)&1] was last read by backward(u+1), or by forward(U-2).
        ag_stream_->wait(u + 1 <= U_ - 1 ? *bwd_done_[u + 1] : *fwd_done_[u - 1]);
        gather(u - 1, *ag_b_[u - 1], false, gated_ ? g_ag_b_[u - 1] : -1);
      }
      // full_grad[u&1] was last read by the reduce-scatter of unit u+2.
      if (gated_) {
        std::vector<int> gates;
        if (u < U_ - 1) {
          if (!lane) compute_->wait(*ag_b_[u]);
          gates.push_back(g_ag_b_[u]);
        }
        if (u + 2 <= U_ - 1) {
          if (!lane) compute_->wait(*rs_done_[u + 2]);
          gates.push_back(g_rs_[u + 2]);
        }
        compute_gated(gates, u < U_ - 1 ? "allgather_wait_bwd" : nullptr, bwd_us_, bwd_flops_, bwd_done_[u].get());
      } else {
        if (u + 2 <= U_ - 1) compute_->wait(*rs_done_[u + 2]);
        if (u < U_ - 1)
          compute_after(*ag_b_[u], "allgather_wait_bwd", bwd_us_, bwd_flops_);
        else
          compute_after(nullptr, nullptr, bwd_us_, bwd_flops_);
        compute_->record(*bwd_done_[u]);
      }

      rs_stream_->wait(*bwd_done_[u]);
      int tk = timers_->begin(*rs_stream_);
      rs_comm_->reduce_scatter(full_grad_[u & 1].data(), grads_[u].data(), shard_[u], t, *rs_stream_);
      tail_end_ = timers_->end(tk, *rs_stream_, "reduce_scatter");
      if (gated_ && u >= 2) ce.signal(*rs_stream_, g_rs_[u]);  // RS(u) gates bwd(u - 2)
      // (lane graphs: waited for only by the replica all-reduce, the tail's
      // stall and the optimizer)
      if (!lane || R_ > 1 || u == 0) rs_stream_->record(*rs_done_[u]);
      if (reference_) compute_->wait(*rs_done_[u]);  // blocking Reduce_Scatter_block (fsdp.cpp:124)
      if (R_ > 1) {
        ar_stream_->wait(*rs_done_[u]);
        int ta = timers_->begin(*ar_stream_);
        ar_comm_->all_reduce(grads_[u].data(), grads_[u].data(), shard_[u], t, *ar_stream_);
        tail_end_ = timers_->end(ta, *ar_stream_, "allreduce_time");
        ar_stream_->record(*ar_done_[u]);
      }
    }
    // ---- tail: exposed reduce-scatter / replica all-reduce
    const bool tail_gap = gated_ && !ctx.opt.optimizer && tail_end_ && prev_.slot;
    // (the lane join ends the program only when nothing follows it on the
    // compute stream: no stall stamp, no optimizer - ADVICE r5)
    if (prog) ce.end_program(*compute_, tail_gap);
    Event& tail = R_ > 1 ? *ar_done_[0] : *rs_done_[0];
    if (tail_gap) {
      // nothing runs on the compute stream after the last backward: the
      // exposed tail is the last collective's end stamp minus the last
      // deadline, with no wait + stamp pair (a cross-queue hop and two
      // kernels) at the end of the iteration; the iteration still ends when
      // every stream has (graph join / synchronize)
      timers_->gap(prev_.slot, prev_.ticks, tail_end_, "barrier");
    } else {
      timers_->stall_after_task(*compute_, tail, "barrier");
    }
    if (ctx.opt.optimizer) {
      if (R_ > 1)
        for (int u = 1; u < U_; ++u) compute_->wait(*ar_done_[u]);
      for (int u = 0; u < U_; ++u)
        optimizer_step(ctx, *compute_, params_[u].data(), mom_[u].data(), grads_[u].data(), shard_[u]);
    }
  }

  std::vector<Stream*> streams() override {
    std::vector<Stream*> ss = {compute_.get()};
    for (auto& s : lanes_) ss.push_back(s.get());
    return ss;
  }
  bool capturable() const override { return !reference_; }

  void synchronize() override {
    std::vector<Stream*> ss = {compute_.get()};
    std::vector<Communicator*> cs;
    for (auto& s : lanes_) ss.push_back(s.get());
    for (auto& c : comms_) cs.push_back(c.get());
    sync_streams(ss, cs, *ctx_->dev);
    timers_->resolve();
  }

  std::string tail_collective_timer() const override { return R_ > 1 ? "allreduce_time" : "reduce_scatter"; }
  std::string section_id() const override { return "fsdp"; }
  std::string section_title() const override { return "FSDP metrics"; }
  const char* runtime_key() const override { return "runtime"; }

  Json global_json() const override {
    const Context& ctx = *ctx_;
    Json g = Json::object();
    g["model_size_bytes"] = P_ * es_;
    g["model_name"] = ctx.opt.model;
    g["world_size"] = ctx.world();
    g["num_units"] = U_;
    g["sharding_factor"] = F_;
    g["num_replicas"] = R_;
    g["local_batch_size"] = ctx.stats.batch_size;
    g["device"] = ctx.dev->kind() == DeviceKind::CPU ? "CPU" : "GPU";
    g["backend"] = ag_comm_->backend_name();
    g["comm_lanes"] = ctx.opt.comm_lanes;
    g["device_gates"] = gated_;
    g["fwd_time_per_unit_us"] = fwd_us_;
    g["bwd_time_per_unit_us"] = bwd_us_;
    g["allgather_msg_size_bytes"] = max_shard_ * F_ * es_;
    g["reducescatter_msg_size_bytes"] = max_shard_ * es_;
    if (R_ > 1) g["allreduce_msg_size_bytes"] = max_shard_ * es_;
    return g;
  }

  Json rank_json() const override {
    Json r = Json::object();
    for (const char* k : {"runtime", "allgather", "allgather_wait_fwd", "allgather_wait_bwd", "reduce_scatter",
                          "barrier", "allgather_time", "allreduce_time"})
      r[k] = timers_->values_json(k);
    r["rank"] = ctx_->rank();
    return r;
  }

  Json comm_summary() const override { return comm_stats_json(stats_, *timers_); }

 private:
  Context* ctx_ = nullptr;
  int U_ = 1, F_ = 1, R_ = 1;
  uint64_t P_ = 0, max_shard_ = 0;
  size_t es_ = 2;
  bool reference_ = false;
  bool gated_ = false;                         // device gates instead of compute-stream event waits
  std::vector<int> g_ag_f_, g_ag_b_, g_rs_;    // gate per forward / backward all-gather, reduce-scatter
  std::vector<uint64_t> shard_;
  double fwd_us_ = 0, bwd_us_ = 0, fwd_flops_ = 0, bwd_flops_ = 0;
  std::vector<std::unique_ptr<Communicator>> comms_;
  std::vector<std::unique_ptr<Stream>> lanes_;
  Communicator *ag_comm_ = nullptr, *rs_comm_ = nullptr, *ar_comm_ = nullptr;
  std::unique_ptr<Stream> compute_;
  Stream *ag_stream_ = nullptr, *rs_stream_ = nullptr, *ar_stream_ = nullptr;
  std::vector<Buffer> params_, grads_, mom_;
  Buffer gathered_[2], full_grad_[2];
  std::vector<std::unique_ptr<Event>> ag_f_, fwd_done_, ag_b_, bwd_done_, rs_done_, ar_done_;
  std::vector<CommStat> stats_;
  TaskMark prev_;                         // where the previous compute task ended (task_mark)
  const uint64_t* tail_end_ = nullptr;    // end stamp of the iteration's last collective
};

}  // namespace

std::unique_ptr<Strategy> make_fsdp() { return std::unique_ptr<Strategy>(new Fsdp()); }

}  // namespace dlnb
