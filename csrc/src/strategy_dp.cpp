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
#include <cmath>

#include "dlnb/strategy.hpp"

namespace dlnb {

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
    uint64_t base = P_ / nb_, rem = P_ % nb_;
    for (int i = 0; i < nb_; ++i) sizes_.push_back(base + (static_cast<uint64_t>(i) < rem ? 1 : 0));
    fwd_us_ = st.avg_forward_time_us;
    bwd_us_per_bucket_ = st.avg_backward_time_us / nb_;
    fwd_flops_ = st.forward_flops;
    bwd_flops_per_bucket_ = st.backward_flops / nb_;

    Device& dev = *ctx.dev;
    es_ = dtype_size(ctx.wire);
    std::vector<int> all;
    for (int r = 0; r < ctx.world(); ++r) all.push_back(r);
    comm_ = ctx.comms->create("dp/world", all, sizes_[0] * es_, false);
    compute_ = dev.create_stream(false);
    comm_stream_ = dev.create_stream(true);
    // Out-of-place like the reference unless asked (or forced by memory).
    size_t need = static_cast<size_t>(P_) * es_ * 2;
    in_place_ = o.in_place || (dev.kind() == DeviceKind::GPU && need > dev.free_memory() * 0.85);
    for (int i = 0; i < nb_; ++i) {
      grads_.push_back(dev.alloc(sizes_[i] * es_));
      if (!in_place_) sums_.push_back(dev.alloc(sizes_[i] * es_));
      ready_.push_back(dev.create_event());
      dev.fill_random(grads_.back().data(), sizes_[i], ctx.wire, 1000 + i, *compute_);
    }
    done_ = dev.create_event();
    if (o.optimizer) {
      DLNB_REQUIRE(ctx.wire == DType::BF16, "--optimizer needs --wire-dtype bf16");
      params_ = dev.alloc(P_ * es_);
      mom_ = dev.alloc(P_ * es_);
    }
    compute_->synchronize();
    timers_.reset(new TimerSet(dev));
    timers_->ensure("barrier_time");
    timers_->ensure("allreduce_time");
    stats_ = {{"allreduce", CollKind::AllReduce, comm_->size(), static_cast<double>(sizes_[0] * es_), "allreduce_time"}};
  }

  void enqueue_iteration() override {
    Context& ctx = *ctx_;
    ComputeEngine& ce = *ctx.compute;
    ce.run(*compute_, fwd_us_, fwd_flops_);
    for (int i = 0; i < nb_; ++i) {
      ce.run(*compute_, bwd_us_per_bucket_, bwd_flops_per_bucket_);
      compute_->record(*ready_[i]);
      comm_stream_->wait(*ready_[i]);
      int t = timers_->begin(*comm_stream_);
      void* out = in_place_ ? grads_[i].data() : sums_[i].data();
      comm_->all_reduce(grads_[i].data(), out, sizes_[i], ctx.wire, *comm_stream_);
      timers_->end(t, *comm_stream_, "allreduce_time");
    }
    comm_stream_->record(*done_);
    timers_->stall(*compute_, *done_, "barrier_time");
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
    return g;
  }

  Json rank_json() const override {
    Json r = Json::object();
    r["runtimes"] = timers_->values_json("runtimes");
    r["barrier_time"] = timers_->values_json("barrier_time");
    r["allreduce_time"] = timers_->values_json("allreduce_time");
    return r;
  }

  Json comm_summary() const override { return comm_stats_json(stats_, *timers_); }

 private:
  Context* ctx_ = nullptr;
  int nb_ = 1;
  uint64_t P_ = 0;
  size_t es_ = 2;
  std::vector<uint64_t> sizes_;
  double fwd_us_ = 0, bwd_us_per_bucket_ = 0, fwd_flops_ = 0, bwd_flops_per_bucket_ = 0;
  bool in_place_ = false;
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
