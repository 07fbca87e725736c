// DP x CP: context (sequence) parallelism for long-context training.
//
// Extension: the reference has no sequence / context parallelism; long
// sequences only scale its message sizes (SURVEY.md §2.2 "SP / CP /
// ring-attention / Ulysses: absent", §5 "Long-context"). This driver adds the
// two standard schemes on the same comm layer, as the survey's build plan
// suggests (`hybrid_cp`):
//
//   hybrid_cp <model> <num_cp_shards> <base_path> [--cp-algo ring|ulysses]
//
// Layout: CP innermost (cp_id = rank % C, the C ranks of one xGMI-connected
// group share a sequence), data parallel outside (dp_id = rank / C). Every
// rank holds the whole model and 1/C of the sequence of its replica's batch,
// so its compute is fwd/C and bwd/C per layer and the gradient all-reduce runs
// over all W ranks (CP folded into DP, as Megatron does), bucketed by layers
// (--dp-buckets K) and overlapped with the rest of the backward.
//
// Per layer (L = num_layers from models/<model>.json, d = embed dim, d_kv =
// d * num_kv_heads / num_heads, B = batch, s_loc = seq_len / C):
//   ring    forward: C-1 P2P steps around the CP ring, each sending the KV
//           block 2*B*s_loc*d_kv to cp_id+1 and receiving the next one from
//           cp_id-1 (one group call, double-buffered) while the attention of
//           the current block runs; backward: C-1 steps of KV + dKV (twice
//           the bytes) under the blockwise attention backward.
//   ulysses forward: all-to-all of Q,K,V (B*s_loc*(d+2*d_kv) per rank) before
//           the attention and of its output (B*s_loc*d) after, both on the
//           critical path; backward: the mirror (dO, then dQ,dK,dV).
// A layer's compute is split by the roofline model the stats come from
// (python/model_stats.py:128-130): the attention-score part 4*B*N^2*d is the
// share that overlaps the ring (cut into C blocks), the projections and MLP
// (8*B*N*d^2 + 4*B*N*d*H*k) run half before and half after it.
#include <cmath>

#include "dlnb/strategy.hpp"

namespace dlnb {

namespace {

class ContextParallel : public Strategy {
 public:
  void setup(Context& ctx) override {
    ctx_ = &ctx;
    const auto& o = ctx.opt;
    const auto& st = ctx.stats;
    const int W = ctx.world();
    C_ = o.num_cp_shards;
    ring_ = o.cp_algo == "ring";
    reference_ = o.schedule == "reference";
    DLNB_REQUIRE(ctx.have_arch, "hybrid_cp needs models/<model>.json (layer count, heads)");
    L_ = static_cast<int>(ctx.arch.num_layers);
    DLNB_REQUIRE(L_ > 0, "model has no layers: " << ctx.arch.path);
    DLNB_REQUIRE(W % C_ == 0, "world size " << W << " must be divisible by num_cp_shards " << C_);
    DLNB_REQUIRE(st.seq_len % C_ == 0, "seq_len " << st.seq_len << " must be divisible by num_cp_shards " << C_);
    heads_ = ctx.arch.num_heads ? ctx.arch.num_heads : 1;
    kv_heads_ = heads_;
    const Json& raw = ctx.arch.raw;
    if (raw.is_object() && raw.contains("dlnb") && raw.at("dlnb").is_object() && raw.at("dlnb").contains("num_kv_heads")) {
      uint64_t kv = static_cast<uint64_t>(raw.at("dlnb").at("num_kv_heads").as_int());
      if (kv > 0) kv_heads_ = kv;
    }
    if (!ring_)
      DLNB_REQUIRE(heads_ % C_ == 0, "ulysses: num_heads " << heads_ << " must be divisible by num_cp_shards " << C_);
    nbk_ = std::min(o.dp_buckets, L_);
    cp_id_ = ctx.rank() % C_;
    dp_id_ = ctx.rank() / C_;

    const uint64_t B = st.batch_size, d = st.embedded_dim, N = st.seq_len;
    const uint64_t dkv = d * kv_heads_ / heads_;
    s_loc_ = N / C_;
    kv_ = 2 * B * s_loc_ * dkv;
    qkv_ = B * s_loc_ * (d + 2 * dkv);
    out_ = B * s_loc_ * d;
    // Ulysses all-to-all: count per peer (buffers hold C * count).
    qkv_peer_ = (qkv_ + C_ - 1) / C_;
    out_peer_ = (out_ + C_ - 1) / C_;

    const double H = static_cast<double>(st.ffn_dim ? st.ffn_dim : (ctx.arch.ff_dim ? ctx.arch.ff_dim : 4 * d));
    const double k = static_cast<double>(st.top_k ? st.top_k : (ctx.arch.experts_per_tok ? ctx.arch.experts_per_tok : 1));
    const double dn = static_cast<double>(d), Nn = static_cast<double>(N);
    const double score = 4.0 * Nn * Nn * dn, proj = 8.0 * Nn * dn * dn, mlp = 4.0 * Nn * dn * H * k;
    attn_frac_ = score / (score + proj + mlp);
    fwd_layer_us_ = st.avg_forward_time_us / C_ / L_;
    bwd_layer_us_ = st.avg_backward_time_us / C_ / L_;
    fwd_layer_flops_ = st.forward_flops / C_ / L_;
    bwd_layer_flops_ = st.backward_flops / C_ / L_;

    Device& dev = *ctx.dev;
    es_ = dtype_size(ctx.wire);
    std::vector<int> cp_members;
    for (int i = 0; i < C_; ++i) cp_members.push_back(dp_id_ * C_ + i);
    if (C_ > 1) {
      size_t cap = (ring_ ? 2 * kv_ : C_ * std::max(qkv_peer_, out_peer_)) * es_;
      cp_comm_ = ctx.comms->create("cp/" + std::to_string(dp_id_), cp_members, cap, ring_, ctx.lane_ctas);
    }
    // Gradient buckets by layer (backward order); bucket k = layers
    // [k*L/nbk, (k+1)*L/nbk) counted from the last layer.
    const uint64_t P = st.model_size;
    for (int b = 0; b < nbk_; ++b) bucket_.push_back(P / nbk_ + (static_cast<uint64_t>(b) < P % nbk_ ? 1 : 0));
    std::vector<int> all;
    for (int r = 0; r < W; ++r) all.push_back(r);
    dp_comm_ = ctx.comms->create("cpdp/world", all, bucket_[0] * es_, false, ctx.lane_ctas);

    compute_ = dev.create_stream(false);
    cp_stream_ = dev.create_stream(true);
    dp_stream_ = dev.create_stream(true);
    if (C_ > 1) {
      if (ring_) {
        for (int b = 0; b < 2; ++b) {
          kvbuf_[b] = dev.alloc(2 * kv_ * es_);  // backward carries KV + dKV
          dev.fill_random(kvbuf_[b].data(), 2 * kv_, ctx.wire, 5000 + b, *compute_);
        }
      } else {
        a2a_send_ = dev.alloc(C_ * std::max(qkv_peer_, out_peer_) * es_);
        // zero-copy (xgmi): peers write their blocks straight into a2a_recv_
        const bool peer = cp_comm_->wants_peer_buffers();
        const size_t rb = C_ * std::max(qkv_peer_, out_peer_) * es_;
        a2a_recv_ = peer ? dev.alloc_peer(rb) : dev.alloc(rb);
        if (peer) cp_comm_->register_buffer(a2a_recv_.data(), rb);
        dev.fill_random(a2a_send_.data(), C_ * std::max(qkv_peer_, out_peer_), ctx.wire, 5100, *compute_);
      }
    }
    const bool dp_peer = dp_comm_->wants_peer_buffers();  // in-place bucket all-reduces, zero-copy on xgmi
    for (int b = 0; b < nbk_; ++b) {
      grads_.push_back(dp_peer ? dev.alloc_peer(bucket_[b] * es_) : dev.alloc(bucket_[b] * es_));
      if (dp_peer) dp_comm_->register_buffer(grads_.back().data(), bucket_[b] * es_);
      dev.fill_random(grads_.back().data(), bucket_[b], ctx.wire, 5200 + b, *compute_);
      bucket_ready_.push_back(dev.create_event());
    }
    for (int j = 0; j <= C_; ++j) {
      recvd_.push_back(dev.create_event());
      attn_done_.push_back(dev.create_event());
    }
    proj_done_ = dev.create_event();
    a2a_done_ = dev.create_event();
    dp_done_ = dev.create_event();
    if (o.optimizer) {
      DLNB_REQUIRE(ctx.wire == DType::BF16, "--optimizer needs --wire-dtype bf16");
      params_ = dev.alloc(P * es_);
      mom_ = dev.alloc(P * es_);
    }
    compute_->synchronize();
    timers_.reset(new TimerSet(dev));
    for (const char* k : {"cp_fwd_time", "cp_bwd_time", "cp_qkv_time", "cp_out_time", "cp_exposed_time", "dp_comm_time",
                          "dp_exposed_time"})
      timers_->ensure(k);
    if (C_ > 1) {
      if (ring_) {
        stats_.push_back({"cp_ring_sendrecv", CollKind::SendRecv, 2, static_cast<double>(kv_ * es_), "cp_fwd_time"});
        stats_.push_back({"cp_ring_sendrecv_bwd", CollKind::SendRecv, 2, static_cast<double>(2 * kv_ * es_), "cp_bwd_time"});
      } else {
        stats_.push_back({"cp_alltoall_qkv", CollKind::AllToAll, C_, static_cast<double>(C_ * qkv_peer_ * es_), "cp_qkv_time"});
        stats_.push_back({"cp_alltoall_out", CollKind::AllToAll, C_, static_cast<double>(C_ * out_peer_ * es_), "cp_out_time"});
      }
    }
    stats_.push_back({"dp_allreduce", CollKind::AllReduce, W, static_cast<double>(bucket_[0] * es_), "dp_comm_time"});
  }

  // One layer's attention block with the CP communication around it.
  // fwd: forward pass; else backward (messages twice the KV block for ring).
  void attention(bool fwd, double core_us, double core_flops) {
    Context& ctx = *ctx_;
    ComputeEngine& ce = *ctx.compute;
    if (C_ == 1) {
      ce.run(*compute_, core_us, core_flops);
      return;
    }
    if (ring_) {
      const uint64_t n = fwd ? kv_ : 2 * kv_;
      const char* tk = fwd ? "cp_fwd_time" : "cp_bwd_time";
      compute_->record(*proj_done_);
      for (int j = 0; j < C_; ++j) {
        if (j < C_ - 1) {
          // step j ships block j onward and receives block j+1 into the other
          // buffer, which compute read for block j-1
          cp_stream_->wait(j == 0 ? *proj_done_ : *attn_done_[j - 1]);
          int t = timers_->begin(*cp_stream_);
          cp_comm_->group_start();
          cp_comm_->send(kvbuf_[j & 1].data(), n, ctx.wire, (cp_id_ + 1) % C_, *cp_stream_);
          cp_comm_->recv(kvbuf_[(j + 1) & 1].data(), n, ctx.wire, (cp_id_ + C_ - 1) % C_, *cp_stream_);
          cp_comm_->group_end();
          timers_->end(t, *cp_stream_, tk);
          cp_stream_->record(*recvd_[j + 1]);
          if (reference_) timers_->stall_before_task(*compute_, *recvd_[j + 1], "cp_exposed_time");  // no overlap
        }
        if (j > 0 && !reference_) timers_->stall_before_task(*compute_, *recvd_[j], "cp_exposed_time");
        ce.run(*compute_, core_us / C_, core_flops / C_);
        compute_->record(*attn_done_[j]);
      }
    } else {
      // Ulysses: sequence-sharded -> head-sharded before the attention and
      // back after it (forward: Q,K,V then O; backward: dO then dQ,dK,dV).
      ulysses_a2a(fwd ? qkv_peer_ : out_peer_, fwd ? "cp_qkv_time" : "cp_out_time");
      ce.run(*compute_, core_us, core_flops);
      ulysses_a2a(fwd ? out_peer_ : qkv_peer_, fwd ? "cp_out_time" : "cp_qkv_time");
    }
  }

  void ulysses_a2a(uint64_t per_peer, const char* tk) {
    compute_->record(*proj_done_);
    cp_stream_->wait(*proj_done_);
    int t = timers_->begin(*cp_stream_);
    cp_comm_->all_to_all(a2a_send_.data(), a2a_recv_.data(), per_peer, ctx_->wire, *cp_stream_);
    timers_->end(t, *cp_stream_, tk);
    cp_stream_->record(*a2a_done_);
    timers_->stall_before_task(*compute_, *a2a_done_, "cp_exposed_time");
  }

  void enqueue_iteration() override {
    Context& ctx = *ctx_;
    ComputeEngine& ce = *ctx.compute;
    const double a = attn_frac_;
    // Lane graphs: the iteration's compute tasks are one compute program, the
    // CP and DP event waits / records folded into its tasks' gates
    // (Device::StreamFold): the ~200 task boundaries per iteration that made
    // CP's launch-per-task lanes lose to the single graph are gone.
    const bool prog = ctx.dev->gate_events() && !reference_ && ce.begin_program(*compute_);
    const uint64_t* dp_end = nullptr;
    for (int l = 0; l < L_; ++l) {
      ce.run(*compute_, fwd_layer_us_ * (1 - a) / 2, fwd_layer_flops_ * (1 - a) / 2);
      attention(true, fwd_layer_us_ * a, fwd_layer_flops_ * a);
      ce.run(*compute_, fwd_layer_us_ * (1 - a) / 2, fwd_layer_flops_ * (1 - a) / 2);
    }
    int b = 0;
    for (int i = 0; i < L_; ++i) {  // backward, last layer first
      ce.run(*compute_, bwd_layer_us_ * (1 - a) / 2, bwd_layer_flops_ * (1 - a) / 2);
      attention(false, bwd_layer_us_ * a, bwd_layer_flops_ * a);
      ce.run(*compute_, bwd_layer_us_ * (1 - a) / 2, bwd_layer_flops_ * (1 - a) / 2);
      if ((i + 1) * nbk_ / L_ > b) {  // last layer of bucket b done
        compute_->record(*bucket_ready_[b]);
        dp_stream_->wait(*bucket_ready_[b]);
        int t = timers_->begin(*dp_stream_);
        dp_comm_->all_reduce(grads_[b].data(), grads_[b].data(), bucket_[b], ctx.wire, *dp_stream_);
        dp_end = timers_->end(t, *dp_stream_, "dp_comm_time");
        ++b;
      }
    }
    // nothing after the program on the compute stream (no optimizer): it ends
    // in the lane join and the DP tail is a gap (as the pipeline's)
    const bool join = prog && !ctx.opt.optimizer && dp_end && timers_->task_stamps();
    if (prog) ce.end_program(*compute_, join);
    if (join) {
      timers_->stall_until(*compute_, dp_end, "dp_exposed_time");
    } else {
      dp_stream_->record(*dp_done_);
      timers_->stall_after_task(*compute_, *dp_done_, "dp_exposed_time");
    }
    if (ctx.opt.optimizer) {
      size_t off = 0;
      for (int k = 0; k < nbk_; ++k) {
        optimizer_step(ctx, *compute_, params_.at(off * es_), mom_.at(off * es_), grads_[k].data(), bucket_[k]);
        off += bucket_[k];
      }
    }
  }

  std::vector<Stream*> streams() override { return {compute_.get(), cp_stream_.get(), dp_stream_.get()}; }
  bool capturable() const override { return true; }
  // (launch per task: ~200 task boundaries per iteration, slower than the
  // single graph; a compute program - enqueue_iteration - takes lanes)
  bool lanes_without_program() const override { return false; }  // strategy.hpp

  void synchronize() override {
    std::vector<Communicator*> cs = {dp_comm_.get()};
    if (cp_comm_) cs.push_back(cp_comm_.get());
    sync_streams(streams(), cs, *ctx_->dev);
    timers_->resolve();
  }

  std::string tail_collective_timer() const override { return "dp_comm_time"; }
  std::string section_id() const override { return "dp_cp"; }
  std::string section_title() const override { return "Data + Context Parallelism"; }

  Json global_json() const override {
    const Context& ctx = *ctx_;
    Json g = Json::object();
    g["model_name"] = ctx.opt.model;
    g["num_cp_shards"] = C_;
    g["cp_algo"] = ring_ ? "ring" : "ulysses";
    g["local_batch_size"] = ctx.stats.batch_size;
    g["world_size"] = ctx.world();
    g["dp_size"] = ctx.world() / C_;
    g["sequence_length"] = ctx.stats.seq_len;
    g["local_sequence_length"] = s_loc_;
    g["embedded_dim"] = ctx.stats.embedded_dim;
    g["num_heads"] = heads_;
    g["num_kv_heads"] = kv_heads_;
    g["num_layers"] = L_;
    g["attention_fraction"] = attn_frac_;
    g["fwd_rt_per_layer"] = fwd_layer_us_;
    g["bwd_rt_per_layer"] = bwd_layer_us_;
    g["total_model_size_params"] = ctx.stats.model_size;
    if (ring_) {
      g["cp_kv_block_size_bytes"] = static_cast<double>(kv_ * es_);
      g["cp_sendrecv_per_layer"] = C_ - 1;
    } else {
      g["cp_alltoall_qkv_size_bytes"] = static_cast<double>(C_ * qkv_peer_ * es_);
      g["cp_alltoall_out_size_bytes"] = static_cast<double>(C_ * out_peer_ * es_);
    }
    g["num_dp_buckets"] = nbk_;
    g["dp_allreduce_size_bytes"] = static_cast<double>(bucket_[0] * es_);
    g["device"] = ctx.dev->kind() == DeviceKind::CPU ? "CPU" : "GPU";
    g["backend"] = dp_comm_->backend_name();
    return g;
  }

  // Per-iteration sums of timers recorded several times per iteration.
  Json per_iter(const std::string& name, size_t per_iteration) const {
    const auto& v = timers_->get(name);
    Json a = Json::array();
    if (per_iteration == 0) return a;
    for (size_t i = 0; i + per_iteration <= v.size(); i += per_iteration) {
      double s = 0;
      for (size_t k = 0; k < per_iteration; ++k) s += v[i + k];
      a.push_back(s);
    }
    return a;
  }

  Json rank_json() const override {
    Json r = Json::object();
    const size_t comm_per_iter = C_ == 1 ? 0 : ring_ ? 2 * L_ * (C_ - 1) : 4 * L_;
    const size_t stall_per_iter = C_ == 1 ? 0 : ring_ ? 2 * L_ * (C_ - 1) : 4 * L_;
    Json comm = Json::array();
    {
      // cp_comm_time: every CP op of the iteration (fwd + bwd timers merged)
      std::vector<double> all;
      const char* a = ring_ ? "cp_fwd_time" : "cp_qkv_time";
      const char* b = ring_ ? "cp_bwd_time" : "cp_out_time";
      const auto& va = timers_->get(a);
      const auto& vb = timers_->get(b);
      const size_t half = comm_per_iter / 2;
      for (size_t i = 0; half && (i + 1) * half <= va.size() && (i + 1) * half <= vb.size(); ++i) {
        double s = 0;
        for (size_t k = 0; k < half; ++k) s += va[i * half + k] + vb[i * half + k];
        comm.push_back(s);
      }
    }
    r["runtimes"] = timers_->values_json("runtimes");
    r["cp_comm_time"] = comm;
    r["cp_exposed_time"] = per_iter("cp_exposed_time", stall_per_iter);
    r["dp_comm_time"] = per_iter("dp_comm_time", static_cast<size_t>(nbk_));
    r["dp_exposed_time"] = timers_->values_json("dp_exposed_time");
    // the same, one entry per wait / CP operation (in issue order)
    r["cp_exposed_waits"] = timers_->values_json("cp_exposed_time");
    for (const char* k : {"cp_fwd_time", "cp_bwd_time", "cp_qkv_time", "cp_out_time"})
      if (!timers_->get(k).empty()) r[std::string(k) + "_ops"] = timers_->values_json(k);
    r["dp_comm_ops"] = timers_->values_json("dp_comm_time");
    r["cp_id"] = cp_id_;
    r["dp_id"] = dp_id_;
    return r;
  }

  Json comm_summary() const override { return comm_stats_json(stats_, *timers_); }
  double compute_floor_us(const Context& ctx) const override {
    return (ctx.stats.avg_forward_time_us + ctx.stats.avg_backward_time_us) / C_;
  }

 private:
  Context* ctx_ = nullptr;
  int C_ = 1, L_ = 1, nbk_ = 1, cp_id_ = 0, dp_id_ = 0;
  bool ring_ = true, reference_ = false;
  uint64_t heads_ = 1, kv_heads_ = 1, s_loc_ = 0, kv_ = 0, qkv_ = 0, out_ = 0, qkv_peer_ = 0, out_peer_ = 0;
  double attn_frac_ = 0, fwd_layer_us_ = 0, bwd_layer_us_ = 0, fwd_layer_flops_ = 0, bwd_layer_flops_ = 0;
  size_t es_ = 2;
  std::vector<uint64_t> bucket_;
  std::unique_ptr<Communicator> cp_comm_, dp_comm_;
  std::unique_ptr<Stream> compute_, cp_stream_, dp_stream_;
  Buffer kvbuf_[2], a2a_send_, a2a_recv_, params_, mom_;
  std::vector<Buffer> grads_;
  std::vector<std::unique_ptr<Event>> recvd_, attn_done_, bucket_ready_;
  std::unique_ptr<Event> proj_done_, a2a_done_, dp_done_;
  std::vector<CommStat> stats_;
};

}  // namespace

std::unique_ptr<Strategy> make_cp() { return std::unique_ptr<Strategy>(new ContextParallel()); }

}  // namespace dlnb
