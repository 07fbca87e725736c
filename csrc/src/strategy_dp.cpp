// Data parallelism with gradient bucketing.
//
// Reference: cpp/data_parallel/dp.cpp. One iteration = forward compute, then
// for each bucket: backward compute of that bucket, then an asynchronous
// all-reduce of the bucket; finally wait for all all-reduces
// (run_data_parallel, dp.cpp:87-106). Bucket sizes: P/nb, the first P%nb
// buckets one larger (dp.cpp:159-164). Timers: runtimes, barrier_time (the
// final wait = exposed communication).
//
// MI355X design: bucket i's backward records an event on the compute stream;
// the all-reduce of bucket i waits on it from a high-priority comm stream.
// One stream per communicator (RCCL serialises a communicator anyway; the
// reference's nb streams on one comm add nothing but ordering hazards).
//
// Extension (absent from the reference): --zero 1|2 shards
// the optimizer state (ZeRO-1) and the gradients (ZeRO-2) over the W ranks.
// Bucket i is padded to W * ceil(size_i / W) elements. ZeRO-1: bucketed
// all-reduce as above, then the optimizer updates this rank's 1/W slice of
// every bucket and the updated parameter slices are all-gathered; ZeRO-2:
// the backward's all-reduces become reduce-scatters into the rank's gradient
// shard (half the bytes per rank). After the gradients (barrier_time = the
// exposed part, as in dp) the optimizer updates the shard bucket by bucket and
// bucket i's parameter all-gather runs under bucket i+1's update; the next
// forward waits for all of them ("param_allgather_exposed").
#include <cmath>

#include "dlnb/strategy.hpp"

namespace dlnb {

// Bucket sizes of a dp run: ratio 1 is the reference's partition (P/nb, the
// first P%nb buckets one larger, dp.cpp:159-164); ratio r < 1 gives bucket i
// (backward order) the share r^i / sum_j r^j, floored, the rounding rest
// going to bucket 0. The weights are built by repeated multiplication and
// summed in order so dlnetbench_amd/parallel/plan.py dp_bucket_sizes()
// reproduces them bit for bit.
std::vector<uint64_t> dp_bucket_sizes(uint64_t P, int nb, double ratio) {
  std::vector<uint64_t> s;
  if (ratio >= 1.0) {
    const uint64_t base = P / nb, rem = P % nb;
    for (int i = 0; i < nb; ++i) s.push_back(base + (static_cast<uint64_t>(i) < rem ? 1 : 0));
    return s;
  }
  std::vector<double> w(static_cast<size_t>(nb));
  double x = 1.0, tot = 0.0;
  for (int i = 0; i < nb; ++i) {
    w[static_cast<size_t>(i)] = x;
    x *= ratio;
  }
  for (double v : w) tot += v;
  uint64_t sum = 0;
  for (double v : w) {
    s.push_back(static_cast<uint64_t>(std::floor(static_cast<double>(P) * v / tot)));
    sum += s.back();
  }
  s[0] += P - sum;
  for (uint64_t v : s) DLNB_REQUIRE(v > 0, "--dp-bucket-ratio " << ratio << " leaves an empty bucket of " << nb);
  return s;
}

namespace {

class DataParallel : public Strategy {
 public:
  void setup(Context& ctx) override {
    ctx_ = &ctx;
    const auto& o = ctx.opt;
    const auto& st = ctx.stats;
    nb_ = o.num_buckets;
    P_ = st.model_size;
    DLNB_REQUIRE(P_ >= static_cast<uint64_t>(nb_), "num_buckets (" << nb_ << ") exceeds the parameter count");
    ratio_ = o.dp_bucket_ratio;
    sizes_ = dp_bucket_sizes(P_, nb_, ratio_);
    fwd_us_ = st.avg_forward_time_us;
    bwd_us_per_bucket_ = st.avg_backward_time_us / nb_;
    // backward compute of bucket i: the reference's bwd/nb, or under a
    // geometric policy the bucket's share of the parameters
    // (time and FLOPs alike: --compute flops sizes a task by its FLOPs)
    for (uint64_t sz : sizes_) {
      const double share = ratio_ >= 1.0 ? 1.0 / nb_ : static_cast<double>(sz) / static_cast<double>(P_);
      bwd_us_.push_back(ratio_ >= 1.0 ? bwd_us_per_bucket_ : st.avg_backward_time_us * share);
      bwd_flops_.push_back(st.backward_flops * share);
    }
    fwd_flops_ = st.forward_flops;
    bwd_flops_per_bucket_ = st.backward_flops / nb_;

    Device& dev = *ctx.dev;
    es_ = dtype_size(ctx.wire);
    zero_ = o.zero;
    W_ = ctx.world();
    for (uint64_t sz : sizes_) shard_.push_back((sz + W_ - 1) / W_);
    std::vector<int> all;
    for (int r = 0; r < ctx.world(); ++r) all.push_back(r);
    // (bucket 0 is the largest under every policy)
    comm_ = ctx.comms->create("dp/world", all, (zero_ ? shard_[0] * W_ : sizes_[0]) * es_, false, ctx.lane_ctas);
    compute_ = dev.create_stream(false);
    comm_stream_ = dev.create_stream(true);
    // Comm gates (GPU deadline compute, plain DP): each backward bucket's
    // compute raises a device gate word on the compute stream and the comm
    // lane waits for it on the device before the bucket's all-reduce, instead
    // of a cross-stream event. The replayed graph then has no edge from the
    // compute chain into the comm chain until the end of the iteration, so the
    // executor keeps each chain on one hardware queue: with event edges it
    // rotated the backward GEMMs over its queues and queued one behind an
    // all-reduce every 4 buckets (profiles/absorb_r4.md: the 5th of 8 waited
    // for the 4th bucket's all-reduce). DLNB_DP_COMM_GATES=1 turns them on
    // (opt-in until measured on hardware; default: event waits).
    ComputeEngine& ce0 = *ctx.compute;
    comm_gates_ = !zero_ && o.schedule != "reference" && env_int("DLNB_DP_COMM_GATES", 0) != 0 &&
                  ce0.gates_task(fwd_us_);
    if (comm_gates_)
      for (int i = 0; i < nb_; ++i) g_ready_.push_back(ce0.make_gate());
    // Out-of-place like the reference unless asked (or forced by memory).
    size_t need = static_cast<size_t>(P_) * es_ * 2;
    in_place_ = o.in_place || (dev.kind() == DeviceKind::GPU && need > dev.free_memory() * 0.85);
    if (zero_ == 2) in_place_ = false;  // the reduce-scatter writes a separate shard
    // Every rank must take the same decision: it sets how many buffers each
    // registers with the communicator (xgmi pairs the k-th registration of
    // every member) and which buffers the collectives read and write. Free
    // memory differs between ranks (several ranks on one GPU, or near the
    // threshold), so agree: in place if any rank needs it.
    in_place_ = ctx.hg().allreduce_max(in_place_ ? 1.0 : 0.0) > 0.5;
    // Zero-copy (xgmi): gradient buckets and all-reduce outputs in peer
    // memory, registered with the communicator, so the collectives read and
    // write peers' buffers directly (see Communicator::register_buffer).
    const bool peer = comm_->wants_peer_buffers();
    auto buf = [&](size_t bytes, bool reg) {
      Buffer b = peer && reg ? dev.alloc_peer(bytes) : dev.alloc(bytes);
      if (peer && reg) comm_->register_buffer(b.data(), bytes);
      return b;
    };
    for (int i = 0; i < nb_; ++i) {
      const uint64_t n = zero_ ? shard_[i] * W_ : sizes_[i];  // padded for ZeRO
      grads_.push_back(buf(n * es_, true));
      if (!in_place_) sums_.push_back(buf((zero_ == 2 ? shard_[i] : n) * es_, zero_ != 2));
      ready_.push_back(dev.create_event());
      dev.fill_random(grads_.back().data(), n, ctx.wire, 1000 + i, *compute_);
      if (zero_) {
        pshard_.push_back(dev.alloc(shard_[i] * es_));
        mshard_.push_back(dev.alloc(shard_[i] * es_));
        pfull_.push_back(buf(shard_[i] * W_ * es_, true));
        dev.fill_random(pshard_.back().data(), shard_[i], ctx.wire, 2000 + i, *compute_);
        opt_done_.push_back(dev.create_event());
      }
    }
    if (zero_) opt_done_word_ = dev.alloc(64);  // the optimizer kernel's block counter (end stamp)
    done_ = dev.create_event();
    ag_done_ = dev.create_event();
    if (o.optimizer && !zero_) {
      DLNB_REQUIRE(ctx.wire == DType::BF16, "--optimizer needs --wire-dtype bf16");
      params_ = dev.alloc(P_ * es_);
      mom_ = dev.alloc(P_ * es_);
    }
    compute_->synchronize();
    timers_.reset(new TimerSet(dev));
    timers_->ensure("barrier_time");
    timers_->ensure("allreduce_time");
    // bytes per op for the bandwidth summary: the first bucket's (the
    // reference's msg size) under the even policy, the mean otherwise
    double op_bytes = 0, shard_bytes = 0;
    for (int i = 0; i < nb_; ++i) {
      op_bytes += static_cast<double>((zero_ ? shard_[i] * W_ : sizes_[i]) * es_) / nb_;
      shard_bytes += static_cast<double>(shard_[i] * W_ * es_) / nb_;
    }
    if (ratio_ >= 1.0) {
      op_bytes = static_cast<double>((zero_ ? shard_[0] * W_ : sizes_[0]) * es_);
      shard_bytes = static_cast<double>(shard_[0] * W_ * es_);
    }
    if (zero_ == 2)
      stats_ = {{"reduce_scatter", CollKind::ReduceScatter, W_, shard_bytes, "reduce_scatter_time"}};
    else
      stats_ = {{"allreduce", CollKind::AllReduce, W_, op_bytes, "allreduce_time"}};
    if (zero_) {
      for (const char* k : {"reduce_scatter_time", "param_allgather_time", "param_allgather_exposed"}) timers_->ensure(k);
      stats_.push_back({"param_allgather", CollKind::AllGather, W_, shard_bytes, "param_allgather_time"});
    }
  }

  // ZeRO-1/2 backward communication, optimizer on the shard, parameter all-gather.
  void enqueue_zero() {
    Context& ctx = *ctx_;
    ComputeEngine& ce = *ctx.compute;
    const int me = comm_->rank();
    // Lane graphs: the forward and backward buckets are one compute program
    // (their ready records folded into the tasks' done gates); it ends before
    // the tail wait and the optimizer steps, which follow it on the compute
    // lane (not joined: the lane ends with its own done word)
    const bool prog = ctx.dev->gate_events() && ce.begin_program(*compute_);
    ce.run(*compute_, fwd_us_, fwd_flops_);
    for (int i = 0; i < nb_; ++i) {
      // only event records on compute_ since the forward: one stretch of compute
      ce.run_chained(*compute_, bwd_us_[i], bwd_flops_[i]);
      compute_->record(*ready_[i]);
      comm_stream_->wait(*ready_[i]);
      const uint64_t n = shard_[i] * W_;
      if (zero_ == 2) {
        int t = timers_->begin(*comm_stream_);
        comm_->reduce_scatter(grads_[i].data(), sums_[i].data(), shard_[i], ctx.wire, *comm_stream_);
        timers_->end(t, *comm_stream_, "reduce_scatter_time");
      } else {
        int t = timers_->begin(*comm_stream_);
        void* out = in_place_ ? grads_[i].data() : sums_[i].data();
        comm_->all_reduce(grads_[i].data(), out, n, ctx.wire, *comm_stream_);
        timers_->end(t, *comm_stream_, "allreduce_time");
      }
    }
    if (prog) ce.end_program(*compute_, false);
    comm_stream_->record(*done_);
    timers_->stall_after_task(*compute_, *done_, "barrier_time");  // exposed gradient communication (as dp)
    // Optimizer step on this rank's slice of each bucket, then that bucket's
    // parameter all-gather, which overlaps the next bucket's update.
    const uint64_t* ag_end = nullptr;
    uint64_t* opt_end = nullptr;
    for (int i = 0; i < nb_; ++i) {
      const void* g = zero_ == 2 ? sums_[i].data()
                                 : (in_place_ ? grads_[i].at(me * shard_[i] * es_) : sums_[i].at(me * shard_[i] * es_));
      // the last step stamps its own end (its kernel's last block): the reference
      // of the exposed parameter all-gather below
      uint64_t* end = i == nb_ - 1 && timers_->enabled() ? timers_->slot() : nullptr;
      if (ctx.wire == DType::BF16) {
        optimizer_step(ctx, *compute_, pshard_[i].data(), mshard_[i].data(), g, shard_[i], end,
                       end ? opt_done_word_.as<uint32_t>() : nullptr);
        opt_end = end;
      }
      compute_->record(*opt_done_[i]);
      comm_stream_->wait(*opt_done_[i]);
      int t = timers_->begin(*comm_stream_);
      comm_->all_gather(pshard_[i].data(), pfull_[i].data(), shard_[i], ctx.wire, *comm_stream_);
      ag_end = timers_->end(t, *comm_stream_, "param_allgather_time");
    }
    // exposed parameter all-gather: from the optimizer's end (its last
    // kernel's own stamp, or a stamp right behind it without the optimizer)
    // to the last all-gather's end stamp - a gap, never a stamp-wait-stamp
    // pair (a stamp kernel queued behind the all-gather read 0 in a single
    // graph); the all-gather may end before the optimizer's last block (it is
    // hidden then: 0)
    const uint64_t* opt_mark = opt_end ? opt_end : timers_->mark(*compute_);
    comm_stream_->record(*ag_done_);
    compute_->wait(*ag_done_);
    if (opt_mark && ag_end) timers_->gap(opt_mark, 0, ag_end, "param_allgather_exposed", true);
  }

  void enqueue_iteration() override {
    if (zero_) {
      enqueue_zero();
      return;
    }
    Context& ctx = *ctx_;
    ComputeEngine& ce = *ctx.compute;
    // Exposed communication (barrier_time, the reference's timer around the
    // final WaitAll, dp.cpp:102-104) from stamps no executor can reorder: the
    // last backward task's own start stamp + its duration (its deadline) to
    // the end stamp of the last all-reduce on the comm stream, when the
    // engine's kernels stamp their start (deadline / sleep / spin compute).
    // A stamp-wait-stamp on the compute stream (stall) otherwise.
    const bool stamped = ce.stamps_task_start();
    TaskMark last;
    const uint64_t* tail_end = nullptr;
    uint64_t* fwd_start = stamped ? timers_->slot() : nullptr;
    // Lane graphs: the forward and the backward buckets are one compute
    // program (one persistent kernel, ComputeEngine::begin_program); each
    // bucket's done event is raised from inside it.
    const bool prog = ctx.dev->gate_events() && !comm_gates_ && ce.begin_program(*compute_);
    ce.run_stamped(*compute_, fwd_us_, fwd_flops_, fwd_start);
    for (int i = 0; i < nb_; ++i) {
      // only event records (or gate signals) on compute_ since the forward: one stretch of compute
      uint64_t* st = stamped && i == nb_ - 1 ? timers_->slot() : nullptr;
      // the bucket's gradients are ready when its backward is: ready_[i] is
      // recorded by the task itself (lane graphs: raised from its own kernel)
      ce.run_chained(*compute_, bwd_us_[i], bwd_flops_[i], st, comm_gates_ ? nullptr : ready_[i].get());
      if (st) last = task_mark(ce, *compute_, st, bwd_us_[i]);
      if (comm_gates_) {
        ce.signal(*compute_, g_ready_[i]);
        // bounded by 4x the compute queued ahead of the signal (the forward and
        // buckets 0..i) + 1 s: never expected to expire
        double ahead = fwd_us_;
        for (int j = 0; j <= i; ++j) ahead += bwd_us_[j];
        ce.wait_gate(*comm_stream_, g_ready_[i], ahead * ctx.opt.time_scale * 4 + 1e6);
      } else {
        comm_stream_->wait(*ready_[i]);
      }
      int t = timers_->begin(*comm_stream_);
      void* out = in_place_ ? grads_[i].data() : sums_[i].data();
      comm_->all_reduce(grads_[i].data(), out, sizes_[i], ctx.wire, *comm_stream_);
      const uint64_t* e = timers_->end(t, *comm_stream_, "allreduce_time");
      if (e) tail_end = e;
    }
    const bool tail_gap = last.slot && tail_end && !ctx.opt.optimizer;
    // (the lane join ends the program only when nothing follows it on the
    // compute stream: no stall stamp, no optimizer - ADVICE r5)
    if (prog) ce.end_program(*compute_, tail_gap);
    if (tail_gap) {
      // nothing follows on the compute stream: the iteration ends when both
      // streams have (graph join, lane done words, synchronize)
      timers_->gap(last.slot, last.ticks, tail_end, "barrier_time");
      // the iteration on the device clock: forward start to the last all-reduce's end
      timers_->gap(fwd_start, 0, tail_end, "device_span_time");
    } else {
      comm_stream_->record(*done_);
      timers_->stall_after_task(*compute_, *done_, "barrier_time");
    }
    if (ctx.opt.optimizer) {
      // Optimizer over the full (replicated) gradient, bucket by bucket.
      size_t off = 0;
      for (int i = 0; i < nb_; ++i) {
        const void* g = in_place_ ? grads_[i].data() : sums_[i].data();
        optimizer_step(ctx, *compute_, params_.at(off * es_), mom_.at(off * es_), g, sizes_[i]);
        off += sizes_[i];
      }
    }
  }

  std::vector<Stream*> streams() override { return {compute_.get(), comm_stream_.get()}; }
  bool capturable() const override { return true; }

  void synchronize() override {
    sync_streams({compute_.get(), comm_stream_.get()}, {comm_.get()}, *ctx_->dev);
    timers_->resolve();
  }

  std::string tail_collective_timer() const override {
    return zero_ ? "param_allgather_time" : "allreduce_time";
  }
  std::string section_id() const override { return "dp"; }
  std::string section_title() const override { return "Data Parallelism"; }

  Json global_json() const override {
    const Context& ctx = *ctx_;
    double avg = 0, sd = 0;
    for (uint64_t s : sizes_) avg += static_cast<double>(s);
    avg /= nb_;
    for (uint64_t s : sizes_) sd += (s - avg) * (s - avg);
    sd = std::sqrt(sd / nb_);
    Json g = Json::object();
    g["comm_gates"] = comm_gates_;
    g["model_name"] = ctx.opt.model;
    g["num_buckets"] = nb_;
    g["local_batch_size"] = ctx.stats.batch_size;
    g["world_size"] = ctx.world();
    g["fwd_rt_whole_model"] = fwd_us_;
    g["bwd_rt_per_bucket"] = bwd_us_per_bucket_;
    g["total_model_size_params"] = P_;
    g["msg_size_avg_bytes"] = avg * es_;
    g["msg_size_std_bytes"] = sd * es_;
    g["device"] = ctx.dev->kind() == DeviceKind::CPU ? "CPU" : "GPU";
    g["backend"] = comm_->backend_name();
    g["in_place"] = in_place_;
    g["bucket_ratio"] = ratio_;
    if (ratio_ < 1.0) {
      g["bucket_policy"] = "geometric";
      g["bucket_sizes"] = Json(sizes_);
      // every bucket's backward compute: time (sleep/spin/gemm modes) and
      // FLOPs (--compute flops) in the same share as its parameters
      g["bwd_us_per_bucket"] = Json(bwd_us_);
      g["bwd_flops_per_bucket"] = Json(bwd_flops_);
    } else {
      g["bucket_policy"] = "even";
    }
    g["zero_stage"] = zero_;
    if (zero_) {
      g["shard_size_params"] = shard_[0];
      g["param_allgather_msg_size_bytes"] = static_cast<double>(shard_[0] * W_ * es_);
    }
    return g;
  }

  Json rank_json() const override {
    Json r = Json::object();
    r["runtimes"] = timers_->values_json("runtimes");
    r["barrier_time"] = timers_->values_json("barrier_time");
    r["allreduce_time"] = timers_->values_json("allreduce_time");
    if (!timers_->get("device_span_time").empty()) r["device_span_time"] = timers_->values_json("device_span_time");
    if (zero_) {
      r["reduce_scatter_time"] = timers_->values_json("reduce_scatter_time");
      r["param_allgather_time"] = timers_->values_json("param_allgather_time");
      r["param_allgather_exposed"] = timers_->values_json("param_allgather_exposed");
    }
    return r;
  }

  Json comm_summary() const override { return comm_stats_json(stats_, *timers_); }

 private:
  Context* ctx_ = nullptr;
  int nb_ = 1;
  uint64_t P_ = 0;
  size_t es_ = 2;
  std::vector<uint64_t> sizes_;
  std::vector<double> bwd_us_;     // backward compute per bucket
  bool comm_gates_ = false;  // backward buckets signal the comm lane through device gates
  std::vector<int> g_ready_;
  std::vector<double> bwd_flops_;  // and its FLOPs
  double ratio_ = 1.0;
  double fwd_us_ = 0, bwd_us_per_bucket_ = 0, fwd_flops_ = 0, bwd_flops_per_bucket_ = 0;
  bool in_place_ = false;
  int zero_ = 0, W_ = 1;
  std::vector<uint64_t> shard_;        // per bucket: ceil(size / W)
  std::vector<Buffer> pshard_, mshard_, pfull_;  // ZeRO: parameter / momentum shards, gathered parameters
  std::vector<std::unique_ptr<Event>> opt_done_;
  Buffer opt_done_word_;
  std::unique_ptr<Event> ag_done_;
  std::unique_ptr<Communicator> comm_;
  std::unique_ptr<Stream> compute_, comm_stream_;
  std::vector<Buffer> grads_, sums_;
  std::vector<std::unique_ptr<Event>> ready_;
  std::unique_ptr<Event> done_;
  Buffer params_, mom_;
  std::vector<CommStat> stats_;
};

}  // namespace

std::unique_ptr<Strategy> make_dp() { return std::unique_ptr<Strategy>(new DataParallel()); }

}  // namespace dlnb
