// Pipeline-parallel hybrids: DP x PP (hybrid_2d), DP x PP x TP (hybrid_3d),
// DP x PP x EP (hybrid_3d_moe), and the 4-D DP x PP x TP x EP (hybrid_4d,
// an extension: the reference only lists a hybrid_4d binary in .gitignore:6).
//
// Reference: cpp/hybrid_parallel/hybrid_2d.cpp:90-169, hybrid_3d.cpp:94-192,
// hybrid_3d_moe.cpp:104-211. GPipe schedule: every microbatch forward
// (receive activations from stage-1, compute, send to stage+1), then every
// microbatch backward (mirrored), then a data-parallel all-reduce of the
// stage's gradients. hybrid_3d adds 2 tensor-parallel all-reduces after each
// microbatch forward and backward (hybrid_3d.cpp:144-148,179-183);
// hybrid_3d_moe adds 2 x layers_per_stage expert all-to-alls per microbatch
// and direction (hybrid_3d_moe.cpp:161-165,196-200), an all-reduce of the
// non-expert gradients over the EP group and the DP all-reduce of
// non-expert + expert-shard gradients (:202-208).
// Sizes (elements): pipe = s*d*B/mb; TP AR = pipe/T; DP AR = P/S (2d),
// P/(S*T) (3d), NE/S + (P-NE)/S/EP (moe); A2A per peer = (B/mb)*s*2*d/EP
// (top-k = 2); compute per microbatch = fwd/S/mb (/T for 3d).
//
// MI355X design:
//   * each pair of adjacent stages gets its own 2-rank communicator and
//     stream ("link"), so a stage receives microbatch i+1 from its
//     predecessor while it computes microbatch i and while it sends
//     microbatch i-1 to its successor; activation buffers are double
//     buffered and reuse is ordered by events;
//   * TP all-reduces / EP all-to-alls are on the critical path of the layer
//     they belong to, so the compute waits for them - but they run on the
//     inner lane (the DP lane, ordered the same on every member of every
//     group), handed over by an event after the compute task and handed back
//     by one before the next: the compute stream carries only compute, so the
//     lane graphs need no cross-rank collective on the compute lane (VERDICT
//     r5 #5), and the exposed wait (tp_comm_time / ep_comm_time) is timed from
//     the tasks' own stamps like every other stall. The next task is launched
//     behind the wait, so the collective has the whole GPU (a resident
//     compute grid spinning on a gate would leave it the comm CUs only).
//     --schedule reference keeps them on the compute stream (blocking, the
//     reference's order). With --tp-granularity layer (and always for MoE)
//     they are interleaved between the layers' compute slices instead of all
//     issued after the microbatch;
//   * the DP all-reduce can be split into --dp-buckets buckets that overlap
//     the last microbatch's backward;
//   * S = 1 is valid (no P2P), unlike the reference.
#include <cmath>

#include "dlnb/strategy.hpp"

namespace dlnb {

GridCoords grid_coords(int rank, int inner, int stages) {
  return GridCoords{rank % inner, (rank / inner) % stages, rank / (inner * stages)};
}

std::vector<int> inner_group(int rank, int inner, int stages) {
  GridCoords c = grid_coords(rank, inner, stages);
  std::vector<int> v;
  for (int i = 0; i < inner; ++i) v.push_back(c.dp_id * inner * stages + c.stage_id * inner + i);
  return v;
}

std::vector<int> pp_group(int rank, int inner, int stages) {
  GridCoords c = grid_coords(rank, inner, stages);
  std::vector<int> v;
  for (int s = 0; s < stages; ++s) v.push_back(c.dp_id * inner * stages + s * inner + c.inner_id);
  return v;
}

std::vector<int> dp_group(int rank, int inner, int stages, int world) {
  GridCoords c = grid_coords(rank, inner, stages);
  std::vector<int> v;
  for (int d = 0; d < world / (inner * stages); ++d) v.push_back(d * inner * stages + c.stage_id * inner + c.inner_id);
  return v;
}

namespace {

class Pipeline : public Strategy {
 public:
  explicit Pipeline(StrategyKind k) : kind_(k) {}

  void setup(Context& ctx) override {
    ctx_ = &ctx;
    const auto& o = ctx.opt;
    const auto& st = ctx.stats;
    const int W = ctx.world();
    S_ = o.num_stages;
    mb_ = o.num_microbatches;
    has_tp_ = kind_ == StrategyKind::Hybrid3D || kind_ == StrategyKind::Hybrid4D;
    has_ep_ = kind_ == StrategyKind::Hybrid3DMoE || kind_ == StrategyKind::Hybrid4D;
    T_ = has_tp_ ? o.num_tensor_shards : 1;
    E_ = has_ep_ ? o.num_expert_shards : 1;
    inner_ = T_ * E_;  // TP fastest, then EP (hybrid_4d), then stage, then DP replica
    reference_ = o.schedule == "reference";
    // A/B: the round-5 placement of the TP / EP collectives (on the compute
    // stream between the tasks) instead of the inner lane
    inner_on_compute_ = env_int("DLNB_INNER_ON_COMPUTE", 0) != 0;
    one_f_one_b_ = o.pp_schedule == "1f1b";
    interleaved_ = o.pp_schedule == "interleaved";
    dualpipe_ = o.pp_schedule == "dualpipe";
    V_ = interleaved_ ? o.pp_virtual : 1;
    ep_overlap_ = o.ep_overlap && has_ep_ && !reference_;
    skew_ = has_ep_ && E_ > 1 && o.ep_imbalance > 0;
    DLNB_REQUIRE(!(skew_ && ep_overlap_), "--ep-imbalance and --ep-overlap cannot be combined");
    DLNB_REQUIRE(!(ep_overlap_ && has_tp_), "--ep-overlap is not supported with tensor parallelism (hybrid_4d)");
    DLNB_REQUIRE(!((one_f_one_b_ || interleaved_ || dualpipe_) && reference_),
                 "--pp-schedule " << o.pp_schedule << " needs --schedule overlap");
    if (dualpipe_) {
      DLNB_REQUIRE(S_ >= 2 && S_ % 2 == 0, "--pp-schedule dualpipe needs an even number of stages (got " << S_ << ")");
      DLNB_REQUIRE(mb_ % 2 == 0, "--pp-schedule dualpipe needs an even number of microbatches (half enter at each end)");
      DLNB_REQUIRE(o.dp_buckets == 1, "--pp-schedule dualpipe does not split the DP all-reduce (--dp-buckets 1)");
      DLNB_REQUIRE(!ep_overlap_, "--pp-schedule dualpipe cannot be combined with --ep-overlap");
    }
    DLNB_REQUIRE(V_ >= 1, "--pp-virtual must be >= 1");
    DLNB_REQUIRE(ctx.have_arch, "hybrid strategies need models/<model>.json (layer count)");
    L_ = static_cast<int>(ctx.arch.num_layers);
    DLNB_REQUIRE(L_ > 0, "model has no layers: " << ctx.arch.path);
    DLNB_REQUIRE(L_ % S_ == 0, "num_layers " << L_ << " must be divisible by num_stages " << S_);
    DLNB_REQUIRE(st.batch_size % mb_ == 0, "batch size " << st.batch_size << " must be divisible by num_microbatches " << mb_);
    DLNB_REQUIRE(W % (S_ * inner_) == 0, "world size " << W << " must be divisible by stages*"
                                             << (has_tp_ && has_ep_ ? "tensor*expert" : has_ep_ ? "expert" : "tensor")
                                             << " shards = " << S_ * inner_);
    if (has_ep_)
      DLNB_REQUIRE(st.experts % E_ == 0, "experts " << st.experts << " must be divisible by num_expert_shards " << E_);
    dp_size_ = W / (S_ * inner_);
    layers_per_stage_ = L_ / S_;
    if (interleaved_) {
      DLNB_REQUIRE(L_ % (S_ * V_) == 0, "interleaved: num_layers " << L_ << " must be divisible by stages*virtual "
                                                                   << S_ * V_);
      DLNB_REQUIRE(mb_ % S_ == 0, "interleaved: num_microbatches " << mb_ << " must be a multiple of num_stages " << S_);
    }
    layers_per_chunk_ = layers_per_stage_ / V_;

    GridCoords c = grid_coords(ctx.rank(), inner_, S_);
    stage_ = c.stage_id;
    inner_id_ = c.inner_id;
    tp_id_ = inner_id_ % T_;
    ep_id_ = inner_id_ / T_;
    dp_id_ = c.dp_id;

    spmb_ = st.batch_size / mb_;
    pipe_ = st.seq_len * st.embedded_dim * spmb_;
    double tshard = T_;
    fwd_mb_us_ = st.avg_forward_time_us / S_ / (mb_ * tshard);
    bwd_mb_us_ = st.avg_backward_time_us / S_ / (mb_ * tshard);
    fwd_mb_flops_ = st.forward_flops / S_ / (mb_ * tshard);
    bwd_mb_flops_ = st.backward_flops / S_ / (mb_ * tshard);
    const uint64_t P = st.model_size;
    if (kind_ == StrategyKind::Hybrid2D) {
      dp_ar_ = P / S_;
    } else if (kind_ == StrategyKind::Hybrid3D) {
      dp_ar_ = P / (S_ * T_);
      tp_ar_ = pipe_ / T_;
    } else {
      // MoE (hybrid_3d_moe.cpp:340-363); hybrid_4d also shards the
      // non-expert weights and each expert over TP, and the TP ranks of an
      // EP rank dispatch disjoint 1/T of its tokens (sequence-parallel).
      const uint64_t NE = st.non_expert_size;
      ne_ = NE / S_ / T_;
      uint64_t expert = ((P - NE) / S_) / E_ / T_;
      dp_ar_ = ne_ + expert;
      const int top_k = 2;  // hybrid_3d_moe.cpp:357
      a2a_ = (spmb_ * st.seq_len * top_k * st.embedded_dim) / E_ / T_;
      if (has_tp_) tp_ar_ = pipe_ / T_;
      if (has_ep_ && E_ > 1 && o.ep_imbalance > 0) {
        // Expert-load skew: every rank sends the same a2a_*E_ elements per
        // dispatch, split over the EP ranks by Zipf weights 1/(j+1)^A, so EP
        // rank 0 (the hot experts) receives the most; the combine that
        // follows each dispatch sends the tokens back (the transpose).
        std::vector<double> w(static_cast<size_t>(E_));
        double sw = 0;
        for (int j = 0; j < E_; ++j) sw += (w[static_cast<size_t>(j)] = std::pow(1.0 + j, -o.ep_imbalance));
        const uint64_t total = a2a_ * static_cast<uint64_t>(E_);
        uint64_t used = 0;
        skew_counts_.assign(static_cast<size_t>(E_), 0);
        for (int j = 0; j < E_; ++j) used += (skew_counts_[static_cast<size_t>(j)] = static_cast<uint64_t>(total * w[static_cast<size_t>(j)] / sw));
        skew_counts_[0] += total - used;
      }
    }

    if (dualpipe_) {
      // every rank holds two chunks: stage s of the "down" copy and stage
      // S-1-s of the "up" copy, so its gradients (and non-expert part) double
      dp_ar_ *= 2;
      ne_ *= 2;
    }
    sp_ = has_tp_ && o.sequence_parallel;
    tp_shard_ = has_tp_ ? (tp_ar_ + T_ - 1) / T_ : 0;
    Device& dev = *ctx.dev;
    es_ = dtype_size(ctx.wire);
    const int rank = ctx.rank();
    compute_ = dev.create_stream(false);
    std::vector<int> pp = pp_group(rank, inner_, S_);
    // Link communicators between adjacent stages of this pipeline. Created
    // in stage order by every member so creation never deadlocks.
    for (int s = 0; s + 1 < S_; ++s) {
      if (stage_ == s || stage_ == s + 1) {
        std::string nm = "pp/link/" + std::to_string(dp_id_) + "/" + std::to_string(inner_id_) + "/" + std::to_string(s);
        auto comm = ctx.comms->create(nm, {pp[s], pp[s + 1]}, pipe_ * es_, true, ctx.lane_ctas);
        if (stage_ == s) {
          next_ = std::move(comm);
          next_peer_ = 1;
        } else {
          prev_ = std::move(comm);
          prev_peer_ = 0;
        }
      }
    }
    if (interleaved_ && S_ > 1) {
      // The interleaved schedule's ring closes: chunk c of the last stage
      // feeds chunk c+1 of stage 0 over a wrap link.
      if (stage_ == S_ - 1 || stage_ == 0) {
        std::string nm = "pp/wrap/" + std::to_string(dp_id_) + "/" + std::to_string(inner_id_);
        auto comm = ctx.comms->create(nm, {pp[S_ - 1], pp[0]}, pipe_ * es_, true, ctx.lane_ctas);
        if (stage_ == S_ - 1) {
          next_ = std::move(comm);
          next_peer_ = 1;
        } else {
          prev_ = std::move(comm);
          prev_peer_ = 0;
        }
      }
    }
    if (prev_) prev_stream_ = dev.create_stream(true);
    if (next_) next_stream_ = dev.create_stream(true);
    {
      // TP group: same (dp, stage, ep); EP group: same (dp, stage, tp). With
      // one of the two degrees = 1 these are the reference's inner groups
      // (inner_group()); 1-rank groups are kept (the reference issues its
      // TP all-reduces at T = 1 too).
      const int base = dp_id_ * inner_ * S_ + stage_ * inner_;
      const std::string where = std::to_string(dp_id_) + "/" + std::to_string(stage_);
      if (has_tp_) {
        std::vector<int> m;
        for (int t = 0; t < T_; ++t) m.push_back(base + ep_id_ * T_ + t);
        // T > 1: the compute waits for every TP all-reduce, so it gets the
        // backend's own CTA count (no compute program holds the CUs meanwhile:
        // program_ok(); inner_ctas); a 1-rank group (a copy) stays in the lane budget
        tp_comm_ = ctx.comms->create("tp/" + where + "/" + std::to_string(ep_id_), m, tp_shard_ * T_ * es_, false,
                                     T_ > 1 ? inner_ctas(ctx) : ctx.lane_ctas);
      }
      if (has_ep_) {
        std::vector<int> m;
        for (int e = 0; e < E_; ++e) m.push_back(base + e * T_ + tp_id_);
        const uint64_t cap = skew_counts_.empty() ? a2a_ * E_ : std::max<uint64_t>(a2a_ * E_, skew_counts_[0]);
        ep_comm_ = ctx.comms->create("ep/" + where + "/" + std::to_string(tp_id_), m,
                                     std::max<uint64_t>(cap, ne_) * es_, !skew_counts_.empty(),
                                     o.ep_overlap || E_ == 1 ? ctx.lane_ctas : inner_ctas(ctx));
      }
    }
    {
      std::string nm = "dp/" + std::to_string(stage_) + "/" + std::to_string(inner_id_);
      const int nbk = o.dp_buckets;
      dp_comm_ = ctx.comms->create(nm, dp_group(rank, inner_, S_, W), (dp_ar_ / nbk + 1) * es_, false, ctx.lane_ctas);
      dp_stream_ = dev.create_stream(true);
    }
    if (dualpipe_) {
      // Stage s and stage S-1-s hold the same two chunks (one per copy): their
      // gradients are summed over this pair before the DP all-reduce.
      const int lo = std::min(stage_, S_ - 1 - stage_);
      std::vector<int> pair = {pp[lo], pp[S_ - 1 - lo]};
      mirror_comm_ = ctx.comms->create("pp/mirror/" + std::to_string(dp_id_) + "/" + std::to_string(inner_id_) + "/" +
                                           std::to_string(lo),
                                       pair, dp_ar_ * es_, false, ctx.lane_ctas);
      build_dualpipe();
      for (int k = 0; k < 2 * mb_; ++k) dpbuf_.push_back(dev.alloc(pipe_ * es_));
      mirror_ready_ = dev.create_event();
    }

    // Buffers.
    for (int b = 0; b < 2; ++b) {
      if (prev_) {
        act_in_[b] = dev.alloc(pipe_ * es_);
        grad_out_[b] = dev.alloc(pipe_ * es_);
        dev.fill_random(grad_out_[b].data(), pipe_, ctx.wire, 4000 + b, *compute_);
      }
      if (next_) {
        act_out_[b] = dev.alloc(pipe_ * es_);
        grad_in_[b] = dev.alloc(pipe_ * es_);
        dev.fill_random(act_out_[b].data(), pipe_, ctx.wire, 4100 + b, *compute_);
      }
    }
    // Zero-copy (xgmi): the DP gradient (and its all-reduce output) and the
    // expert receive buffer are peer memory registered with their groups.
    const bool dp_peer = dp_comm_->wants_peer_buffers();
    grad_ = dp_peer ? dev.alloc_peer(dp_ar_ * es_) : dev.alloc(dp_ar_ * es_);
    dev.fill_random(grad_.data(), dp_ar_, ctx.wire, 4200, *compute_);
    if (!o.in_place) sum_grad_ = dp_peer ? dev.alloc_peer(dp_ar_ * es_) : dev.alloc(dp_ar_ * es_);
    if (dp_peer) {
      dp_comm_->register_buffer(grad_.data(), grad_.bytes());
      if (!o.in_place) dp_comm_->register_buffer(sum_grad_.data(), sum_grad_.bytes());
    }
    if (has_tp_) {
      tp_buf_ = dev.alloc(tp_shard_ * T_ * es_);
      tp_res_ = dev.alloc(tp_shard_ * T_ * es_);
      dev.fill_random(tp_buf_.data(), tp_shard_ * T_, ctx.wire, 4300, *compute_);
    }
    if (has_ep_) {
      // skew: the hot rank receives E_ * skew_counts_[0] in a dispatch
      const uint64_t n = skew_counts_.empty() ? a2a_ * E_ : std::max<uint64_t>(a2a_ * E_, skew_counts_[0] * E_);
      ep_send_ = dev.alloc(n * es_);
      const bool ep_peer = ep_comm_->wants_peer_buffers();
      ep_recv_ = ep_peer ? dev.alloc_peer(n * es_) : dev.alloc(n * es_);
      if (ep_peer) ep_comm_->register_buffer(ep_recv_.data(), ep_recv_.bytes());
      dev.fill_random(ep_send_.data(), a2a_ * E_, ctx.wire, 4400, *compute_);
      if (ep_overlap_) {
        // The half-microbatch all-to-alls share the DP lane instead of a
        // fifth stream: a middle stage already has compute + dp + prev + next,
        // and with more streams than hardware queues (GPU_MAX_HW_QUEUES = 4)
        // HIP aliases two streams onto one in-order queue, so a collective
        // spinning on its peers can block an unrelated stream's kernel behind
        // it (a cross-rank deadlock). One ordered lane is safe: every member
        // of the EP and DP groups sits at the same stage and enqueues the
        // same sequence.
        ep_stream_ = dp_stream_.get();
        for (int hh = 0; hh < 2; ++hh) {
          chunk_done_[hh] = dev.create_event();
          a2a_done_[hh] = dev.create_event();
        }
      }
    }
    if (o.optimizer) {
      DLNB_REQUIRE(ctx.wire == DType::BF16, "--optimizer needs --wire-dtype bf16");
      params_ = dev.alloc(dp_ar_ * es_);
      mom_ = dev.alloc(dp_ar_ * es_);
    }
    if (has_tp_ || has_ep_) {
      inner_ready_ = dev.create_event();
      inner_done_ = dev.create_event();
    }
    auto mk = [&](std::vector<std::unique_ptr<Event>>& v) {
      for (int i = 0; i < mb_ * V_; ++i) v.push_back(dev.create_event());
    };
    mk(recv_f_);
    mk(fwd_done_);
    mk(send_f_);
    mk(recv_b_);
    mk(bwd_done_);
    mk(send_b_);
    for (int k = 0; k < o.dp_buckets; ++k) {
      bucket_ready_.push_back(dev.create_event());
    }
    dp_done_ = dev.create_event();
    compute_->synchronize();

    timers_.reset(new TimerSet(dev));
    for (const char* k : {"pp_comm_time", "dp_comm_time", "pp_send_time", "pp_recv_time", "dp_exposed_time"})
      timers_->ensure(k);
    if (has_tp_) {
      timers_->ensure("tp_comm_time");
      timers_->ensure("tp_ar_time");
    }
    if (dualpipe_) timers_->ensure("pp_mirror_time");
    if (sp_) {
      timers_->ensure("tp_ag_time");
      timers_->ensure("tp_rs_time");
    }
    if (has_ep_) {
      timers_->ensure("ep_comm_time");
      timers_->ensure("ep_a2a_time");
      timers_->ensure("dp_ep_comm_time");
    }
    if (prev_ || next_) stats_.push_back({"sendrecv", CollKind::SendRecv, 2, static_cast<double>(pipe_ * es_), "pp_send_time"});
    stats_.push_back({"dp_allreduce", CollKind::AllReduce, dp_size_,
                      static_cast<double>(dp_ar_ / (dualpipe_ ? 2 : o.dp_buckets) * es_), "dp_comm_time"});
    if (dualpipe_)
      stats_.push_back({"pp_mirror_allreduce", CollKind::AllReduce, 2, static_cast<double>(dp_ar_ / 2 * es_), "pp_mirror_time"});
    if (has_tp_ && !sp_)
      stats_.push_back({"tp_allreduce", CollKind::AllReduce, T_, static_cast<double>(tp_ar_ * es_), "tp_ar_time"});
    if (has_tp_ && sp_) {
      stats_.push_back({"tp_allgather", CollKind::AllGather, T_, static_cast<double>(tp_shard_ * T_ * es_), "tp_ag_time"});
      stats_.push_back({"tp_reduce_scatter", CollKind::ReduceScatter, T_, static_cast<double>(tp_shard_ * T_ * es_),
                        "tp_rs_time"});
    }
    if (has_ep_)
      stats_.push_back({"ep_alltoall", CollKind::AllToAll, E_,
                        static_cast<double>((ep_overlap_ ? a2a_ / 2 : a2a_) * E_ * es_),
                        ep_overlap_ ? "ep_comm_time" : "ep_a2a_time"});
  }

  // Compute of one microbatch with the inner-group collectives interleaved.
  void micro_compute(double us, double flops) {
    Context& ctx = *ctx_;
    ComputeEngine& ce = *ctx.compute;
    const bool tp_layer = has_tp_ && ctx.opt.tp_granularity == "layer";
    if (has_ep_) {
      const int n = 2 * layers_per_chunk_;
      if (reference_) {
        ce.run(*compute_, us, flops);
        inner_comm(0, n);
        if (has_tp_) inner_comm(tp_layer ? n : 2, 0);
      } else if (ep_overlap_) {
        // Two half-microbatches in flight: the all-to-all of one half runs on
        // the EP lane under the compute of the other (the dual-batch
        // overlap of MoE training); a half's next chunk waits for its own
        // previous all-to-all. One EP lane = one ordered lane per rank.
        for (int i = 0; i < n; ++i) {
          for (int hh = 0; hh < 2; ++hh) {
            if (i > 0) compute_->wait(*a2a_done_[hh]);
            ce.run(*compute_, us / n / 2, flops / n / 2);
            compute_->record(*chunk_done_[hh]);
            ep_stream_->wait(*chunk_done_[hh]);
            ep_alltoall_half(hh);
            ep_stream_->record(*a2a_done_[hh]);
          }
        }
        compute_->wait(*a2a_done_[0]);
        compute_->wait(*a2a_done_[1]);
      } else {
        // hybrid_4d: the TP all-reduce of a slice (attention / expert output)
        // precedes its all-to-all (dispatch / combine).
        for (int i = 0; i < n; ++i) {
          ce.run(*compute_, us / n, flops / n);
          inner_comm(tp_layer ? 1 : 0, 1);
        }
        if (has_tp_ && !tp_layer) inner_comm(2, 0);
      }
    } else if (has_tp_) {
      if (tp_layer) {
        const int slices = 2 * layers_per_chunk_;  // 2 per layer
        for (int i = 0; i < slices; ++i) {
          ce.run(*compute_, us / slices, flops / slices);
          inner_comm(1, 0);
        }
      } else {
        ce.run(*compute_, us, flops);
        inner_comm(2, 0);
      }
    } else {
      ce.run(*compute_, us, flops);
    }
  }

  // One TP all-reduce of the activations, or with --sequence-parallel the
  // Megatron-SP pair that replaces it: all-gather of the sequence shards into
  // the tensor-parallel region, reduce-scatter out of it (same bytes on the
  // wire, activations outside the TP region stay 1/T).
  // tp TP all-reduces, then ep EP all-to-alls, between two compute tasks.
  // Overlap schedules: on the inner lane (dp_stream_), handed the compute
  // stream's work so far by inner_ready_ and handing back inner_done_; the
  // compute stream's next task waits for it, and that wait is the exposed
  // communication (tp_comm_time / ep_comm_time, one entry per collective as
  // the reference's timers: a wait for several is booked on the first). The
  // collectives' own durations on the lane: tp_ar_time / ep_a2a_time (bus
  // bandwidth). --schedule reference: on the compute stream, timed around
  // each one (hybrid_3d.cpp:144-148, hybrid_3d_moe.cpp:161-165).
  void inner_comm(int tp, int ep) {
    if (tp + ep == 0) return;
    if (reference_) {
      for (int i = 0; i < tp; ++i) tp_allreduce(*compute_, "tp_comm_time");
      for (int i = 0; i < ep; ++i) ep_alltoall(*compute_, "ep_comm_time");
      return;
    }
    if (!inner_lane_) {
      // single graph / eager: on the compute stream between the tasks (no
      // cross-stream hop per collective; the compute waits for each anyway)
      for (int i = 0; i < tp; ++i) tp_allreduce(*compute_, "tp_ar_time", "tp_comm_time");
      for (int i = 0; i < ep; ++i) ep_alltoall(*compute_, "ep_a2a_time", "ep_comm_time");
      return;
    }
    compute_->record(*inner_ready_);
    dp_stream_->wait(*inner_ready_);
    for (int i = 0; i < tp; ++i) tp_allreduce(*dp_stream_, "tp_ar_time");
    for (int i = 0; i < ep; ++i) ep_alltoall(*dp_stream_, "ep_a2a_time");
    dp_stream_->record(*inner_done_);
    for (int i = 0; i < tp; ++i) timers_->stall_before_task(*compute_, *inner_done_, "tp_comm_time");
    for (int i = 0; i < ep; ++i) timers_->stall_before_task(*compute_, *inner_done_, "ep_comm_time");
  }

  // timer: the collective's duration; also (optional): the same interval
  // under a second name (on the compute stream it is the exposed wait too)
  void tp_allreduce(Stream& s, const char* timer, const char* also = nullptr) {
    int t = timers_->begin(s);
    if (sp_) {
      int ta = timers_->begin(s);
      tp_comm_->all_gather(tp_buf_.data(), tp_res_.data(), tp_shard_, ctx_->wire, s);
      timers_->end(ta, s, "tp_ag_time");
      int tr = timers_->begin(s);
      tp_comm_->reduce_scatter(tp_res_.data(), tp_buf_.data(), tp_shard_, ctx_->wire, s);
      timers_->end(tr, s, "tp_rs_time");
    } else {
      tp_comm_->all_reduce(tp_buf_.data(), tp_res_.data(), tp_ar_, ctx_->wire, s);
    }
    const uint64_t* e = timers_->end(t, s, timer);
    lane_end(s, e);
    if (also) timers_->pair(timers_->at(t), e, also);
  }

  // The end stamp of the last collective on the inner lane (finish_iteration:
  // TimerSet::settle).
  void lane_end(Stream& s, const uint64_t* end) {
    if (&s == dp_stream_.get()) inner_end_ = end;
  }

  void ep_alltoall(Stream& s, const char* timer, const char* also = nullptr) {
    int t = timers_->begin(s);
    if (skew_)
      ep_alltoallv(s);
    else
      ep_comm_->all_to_all(ep_send_.data(), ep_recv_.data(), a2a_, ctx_->wire, s);
    const uint64_t* e = timers_->end(t, s, timer);
    lane_end(s, e);
    if (also) timers_->pair(timers_->at(t), e, also);
  }

  // --ep-imbalance: all-to-allv as one group of sends / receives. Even calls
  // are dispatches (to EP rank j: skew_counts_[j]), odd calls the matching
  // combines (every peer sends this rank's share back). The block for this
  // rank itself stays local.
  void ep_alltoallv(Stream& s) {
    const bool dispatch = (skew_call_++ & 1) == 0;
    const int me = ep_id_;
    ep_comm_->group_start();
    size_t so = 0, ro = 0;
    for (int j = 0; j < E_; ++j) {
      const uint64_t send_n = dispatch ? skew_counts_[static_cast<size_t>(j)] : skew_counts_[static_cast<size_t>(me)];
      const uint64_t recv_n = dispatch ? skew_counts_[static_cast<size_t>(me)] : skew_counts_[static_cast<size_t>(j)];
      if (j != me) {
        if (send_n) ep_comm_->send(ep_send_.at(so * es_), send_n, ctx_->wire, j, s);
        if (recv_n) ep_comm_->recv(ep_recv_.at(ro * es_), recv_n, ctx_->wire, j, s);
      }
      so += send_n;
      ro += recv_n;
    }
    ep_comm_->group_end();
  }

  // Half-microbatch all-to-all (--ep-overlap): half hh owns its own slice of
  // the send / receive buffers, so the two halves never share memory.
  void ep_alltoall_half(int hh) {
    const uint64_t c0 = a2a_ / 2, c = hh == 0 ? c0 : a2a_ - c0;
    const size_t off = static_cast<size_t>(hh) * c0 * E_ * es_;
    int t = timers_->begin(*ep_stream_);
    ep_comm_->all_to_all(ep_send_.at(off), ep_recv_.at(off), c, ctx_->wire, *ep_stream_);
    timers_->end(t, *ep_stream_, "ep_comm_time");
  }

  void enqueue_gpipe() {
    Context& ctx = *ctx_;
    const DType t = ctx.wire;
    const int nbk = ctx.opt.dp_buckets;

    // ---------------- forward
    for (int i = 0; i < mb_; ++i) {
      const int b = i & 1;
      if (prev_) {
        if (i >= 2) prev_stream_->wait(*fwd_done_[i - 2]);  // act_in[b] consumed
        int tk = timers_->begin(*prev_stream_);
        prev_->recv(act_in_[b].data(), pipe_, t, prev_peer_, *prev_stream_);
        timers_->end(tk, *prev_stream_, "pp_recv_time");
        prev_stream_->record(*recv_f_[i]);
        timers_->stall_before_task(*compute_, *recv_f_[i], "pp_comm_time");
      } else {
        timers_->add("pp_comm_time", 0.0);
      }
      if (next_ && i >= 2) compute_->wait(*send_f_[i - 2]);  // act_out[b] sent
      micro_compute(fwd_mb_us_, fwd_mb_flops_);
      compute_->record(*fwd_done_[i]);
      if (next_) {
        next_stream_->wait(*fwd_done_[i]);
        int tk = timers_->begin(*next_stream_);
        next_->send(act_out_[b].data(), pipe_, t, next_peer_, *next_stream_);
        timers_->end(tk, *next_stream_, "pp_send_time");
        next_stream_->record(*send_f_[i]);
        if (reference_) compute_->wait(*send_f_[i]);  // blocking send
      }
    }
    // ---------------- backward
    for (int i = 0; i < mb_; ++i) {
      const int b = i & 1;
      if (next_) {
        if (i >= 2) next_stream_->wait(*bwd_done_[i - 2]);  // grad_in[b] consumed
        int tk = timers_->begin(*next_stream_);
        next_->recv(grad_in_[b].data(), pipe_, t, next_peer_, *next_stream_);
        timers_->end(tk, *next_stream_, "pp_recv_time");
        next_stream_->record(*recv_b_[i]);
        timers_->stall_before_task(*compute_, *recv_b_[i], "pp_comm_time");
      } else {
        timers_->add("pp_comm_time", 0.0);
      }
      if (prev_ && i >= 2) compute_->wait(*send_b_[i - 2]);
      const bool last = i == mb_ - 1;
      if (last && nbk > 1 && !reference_) {
        // Overlap the DP all-reduce with the last microbatch's backward.
        for (int k = 0; k < nbk; ++k) {
          ctx.compute->run(*compute_, bwd_mb_us_ / nbk, bwd_mb_flops_ / nbk);
          compute_->record(*bucket_ready_[k]);
          dp_stream_->wait(*bucket_ready_[k]);
          dp_allreduce_bucket(k, nbk);
        }
        compute_->record(*bwd_done_[i]);
      } else {
        micro_compute(bwd_mb_us_, bwd_mb_flops_);
        compute_->record(*bwd_done_[i]);
      }
      if (prev_) {
        prev_stream_->wait(*bwd_done_[i]);
        int tk = timers_->begin(*prev_stream_);
        prev_->send(grad_out_[b].data(), pipe_, t, prev_peer_, *prev_stream_);
        timers_->end(tk, *prev_stream_, "pp_send_time");
        prev_stream_->record(*send_b_[i]);
        if (reference_) compute_->wait(*send_b_[i]);
      }
    }
    finish_iteration();
  }

  // DP (and MoE non-expert) gradient synchronisation after the backwards.
  void finish_iteration() {
    Context& ctx = *ctx_;
    const DType t = ctx.wire;
    const int nbk = ctx.opt.dp_buckets;
    // the compute stream's trailing TP / EP waits (after the last backward
    // task) end with the last inner-lane collective; the DP wait below starts
    // there (else the first pending wait took the whole tail)
    if (inner_end_) timers_->settle(*compute_, inner_end_);
    inner_end_ = nullptr;
    if (has_ep_) {
      // Non-expert gradients are replicated across the EP group: all-reduced
      // on the inner lane (the DP all-reduce follows it there; the compute
      // stream waits for both below: dp_exposed_time), or blocking on the
      // compute stream (--schedule reference, hybrid_3d_moe.cpp:202-204).
      Stream& es = reference_ ? *compute_ : *dp_stream_;
      if (!reference_) {
        compute_->record(*inner_ready_);
        dp_stream_->wait(*inner_ready_);
      }
      int tk = timers_->begin(es);
      void* out = ctx.opt.in_place ? grad_.data() : sum_grad_.data();
      ep_comm_->all_reduce(grad_.data(), out, ne_, t, es);
      const uint64_t* e = timers_->end(tk, es, "dp_ep_comm_time");
      if (&es == dp_stream_.get()) dp_end_ = e;
    }
    if (nbk == 1 || reference_) {
      compute_->record(*bucket_ready_[0]);
      dp_stream_->wait(*bucket_ready_[0]);
      if (mirror_comm_ && mirror_early_tick_ < 0) {
        // MoE: the whole pair gradient after the EP all-reduce
        int tm = timers_->begin(*dp_stream_);
        mirror_comm_->all_reduce(grad_.data(), grad_.data(), dp_ar_, t, *dp_stream_);
        dp_end_ = timers_->end(tm, *dp_stream_, "pp_mirror_time");
        dp_allreduce_bucket(0, 1);
      } else if (mirror_comm_) {
        // the half whose chunks finish last (model stage min(s, S-1-s)); the
        // other half was reduced mid-backward (enqueue_dualpipe)
        const size_t half = dp_ar_ / 2;
        void* g = static_cast<char*>(grad_.data()) + half * es_;
        int tm = timers_->begin(*dp_stream_);
        mirror_comm_->all_reduce(g, g, dp_ar_ - half, t, *dp_stream_);
        timers_->end(tm, *dp_stream_, "pp_mirror_time");
        dp_allreduce_bucket(1, 2);
      } else {
        dp_allreduce_bucket(0, 1);
      }
    }
    // With a compute program and nothing after it on the compute stream (no
    // optimizer), the program's join ends the iteration once the other lanes
    // are done, and the DP tail exposed is the DP lane's last end stamp minus
    // the compute's last task (a gap: no wait on the compute stream);
    // otherwise the compute stream waits for the DP lane.
    const bool join = prog_ && !ctx.opt.optimizer && dp_end_ && timers_->task_stamps();
    if (prog_) ctx.compute->end_program(*compute_, join);
    prog_ = false;
    if (join) {
      timers_->stall_until(*compute_, dp_end_, "dp_exposed_time");
    } else {
      dp_stream_->record(*dp_done_);
      timers_->stall_after_task(*compute_, *dp_done_, "dp_exposed_time");
    }
    if (ctx.opt.optimizer) {
      void* g = ctx.opt.in_place ? grad_.data() : sum_grad_.data();
      optimizer_step(ctx, *compute_, params_.data(), mom_.data(), g, dp_ar_);
    }
  }


  // ---------------------------------------------------------------- 1F1B
  // Non-interleaved one-forward-one-backward (PipeDream-flush): stage s runs
  // w = min(S-s-1, mb) warm-up forwards, then alternates F(w+j) / B(j), then
  // drains the remaining backwards. Same bubble as GPipe, at most w+1
  // microbatches in flight. A send and the opposite-direction receive on the
  // same link are posted as ONE group (send_forward_recv_backward /
  // send_backward_recv_forward), so the two sides of a link never block each
  // other; every link op waits only on events already enqueued.
  void prev_link(int send_b, int recv_f) {
    const DType t = ctx_->wire;
    Stream& ls = *prev_stream_;
    if (send_b >= 0) ls.wait(*bwd_done_[send_b]);
    if (recv_f >= 2) ls.wait(*fwd_done_[recv_f - 2]);  // act_in[recv_f & 1] consumed
    int tk = timers_->begin(ls);
    prev_->group_start();
    if (send_b >= 0) prev_->send(grad_out_[send_b & 1].data(), pipe_, t, prev_peer_, ls);
    if (recv_f >= 0) prev_->recv(act_in_[recv_f & 1].data(), pipe_, t, prev_peer_, ls);
    prev_->group_end();
    timers_->end(tk, ls, send_b >= 0 ? "pp_send_time" : "pp_recv_time");
    if (send_b >= 0) ls.record(*send_b_[send_b]);
    if (recv_f >= 0) ls.record(*recv_f_[recv_f]);
  }

  void next_link(int send_f, int recv_b) {
    const DType t = ctx_->wire;
    Stream& ls = *next_stream_;
    if (send_f >= 0) ls.wait(*fwd_done_[send_f]);
    if (recv_b >= 2) ls.wait(*bwd_done_[recv_b - 2]);  // grad_in[recv_b & 1] consumed
    int tk = timers_->begin(ls);
    next_->group_start();
    if (send_f >= 0) next_->send(act_out_[send_f & 1].data(), pipe_, t, next_peer_, ls);
    if (recv_b >= 0) next_->recv(grad_in_[recv_b & 1].data(), pipe_, t, next_peer_, ls);
    next_->group_end();
    timers_->end(tk, ls, send_f >= 0 ? "pp_send_time" : "pp_recv_time");
    if (send_f >= 0) ls.record(*send_f_[send_f]);
    if (recv_b >= 0) ls.record(*recv_b_[recv_b]);
  }

  void fwd_step(int i) {
    if (prev_)
      timers_->stall_before_task(*compute_, *recv_f_[i], "pp_comm_time");
    else
      timers_->add("pp_comm_time", 0.0);
    if (next_ && i >= 2) compute_->wait(*send_f_[i - 2]);  // act_out[i & 1] sent
    micro_compute(fwd_mb_us_, fwd_mb_flops_);
    compute_->record(*fwd_done_[i]);
  }

  void bwd_step(int j) {
    const int nbk = ctx_->opt.dp_buckets;
    if (next_)
      timers_->stall_before_task(*compute_, *recv_b_[j], "pp_comm_time");
    else
      timers_->add("pp_comm_time", 0.0);
    if (prev_ && j >= 2) compute_->wait(*send_b_[j - 2]);  // grad_out[j & 1] sent
    if (j == mb_ - 1 && nbk > 1) {
      for (int k = 0; k < nbk; ++k) {  // DP buckets overlap the last backward
        ctx_->compute->run(*compute_, bwd_mb_us_ / nbk, bwd_mb_flops_ / nbk);
        compute_->record(*bucket_ready_[k]);
        dp_stream_->wait(*bucket_ready_[k]);
        dp_allreduce_bucket(k, nbk);
      }
    } else {
      micro_compute(bwd_mb_us_, bwd_mb_flops_);
    }
    compute_->record(*bwd_done_[j]);
  }

  void enqueue_1f1b() {
    const int w = std::min(S_ - stage_ - 1, mb_);
    const int steady = mb_ - w;
    for (int i = 0; i < w; ++i) {
      if (prev_) prev_link(-1, i);
      fwd_step(i);
      if (next_) next_link(i, -1);
    }
    if (steady > 0 && prev_) prev_link(-1, w);
    for (int j = 0; j < steady; ++j) {
      const int i = w + j;
      fwd_step(i);
      if (next_) next_link(i, j);  // send F(i) + receive B(j)
      bwd_step(j);
      if (prev_) prev_link(j, j + 1 < steady ? i + 1 : -1);  // send B(j) (+ receive F(i+1))
    }
    for (int j = steady; j < mb_; ++j) {
      if (next_) next_link(-1, j);
      bwd_step(j);
      if (prev_) prev_link(j, -1);
    }
    finish_iteration();
  }

  // ------------------------------------------------- interleaved 1F1B
  // Megatron's interleaved (virtual-stage) schedule: each stage holds V
  // model chunks; virtual stage c*S + s is chunk c of stage s, so a
  // microbatch crosses the S-stage ring V times (the last stage's chunk c
  // feeds stage 0's chunk c+1 over the wrap link). Forward k of a stage runs
  // chunk (k/S)%V of microbatch (k/(S*V))*S + k%S; backward k the chunk
  // V-1-(k/S)%V. Warm-up = (S-s-1)*2 + (V-1)*S forwards (all of them when
  // mb == S), then forward/backward pairs, then the remaining backwards; the
  // bubble shrinks from (S-1)(f+b) to (S-1)(f+b)/V. The P2P after each step
  // is Megatron's, split per link: next link {send F, receive B}, previous
  // link {send B, receive F}.
  int chunk_f(int k) const { return (k / S_) % V_; }
  int chunk_b(int k) const { return V_ - 1 - (k / S_) % V_; }
  bool in_f(int k) const { return !(stage_ == 0 && chunk_f(k) == 0); }
  bool out_f(int k) const { return !(stage_ == S_ - 1 && chunk_f(k) == V_ - 1); }
  bool in_b(int k) const { return !(stage_ == S_ - 1 && chunk_b(k) == V_ - 1); }
  bool out_b(int k) const { return !(stage_ == 0 && chunk_b(k) == 0); }

  void fwd_chunk(int k) {
    if (S_ > 1 && in_f(k))
      timers_->stall_before_task(*compute_, *recv_f_[k], "pp_comm_time");
    else
      timers_->add("pp_comm_time", 0.0);
    if (S_ > 1 && k >= 2) compute_->wait(*send_f_[k - 2]);  // act_out[k & 1] sent (no-op if never recorded)
    micro_compute(fwd_mb_us_ / V_, fwd_mb_flops_ / V_);
    compute_->record(*fwd_done_[k]);
  }

  void bwd_chunk(int j) {
    const int nbk = ctx_->opt.dp_buckets;
    const int total = mb_ * V_;
    if (S_ > 1 && in_b(j))
      timers_->stall_before_task(*compute_, *recv_b_[j], "pp_comm_time");
    else
      timers_->add("pp_comm_time", 0.0);
    if (S_ > 1 && j >= 2) compute_->wait(*send_b_[j - 2]);  // grad_out[j & 1] sent
    if (j == total - 1 && nbk > 1) {
      for (int k = 0; k < nbk; ++k) {  // DP buckets overlap the last backward
        ctx_->compute->run(*compute_, bwd_mb_us_ / V_ / nbk, bwd_mb_flops_ / V_ / nbk);
        compute_->record(*bucket_ready_[k]);
        dp_stream_->wait(*bucket_ready_[k]);
        dp_allreduce_bucket(k, nbk);
      }
    } else {
      micro_compute(bwd_mb_us_ / V_, bwd_mb_flops_ / V_);
    }
    compute_->record(*bwd_done_[j]);
  }

  // Link groups of one step (-1 = nothing in that slot).
  void links(int send_f, int recv_b, int send_b, int recv_f) {
    if (S_ == 1) return;
    // With the wrap link the stages form a ring; stage 0 serves its previous
    // link first so a backend whose groups complete on the host (loopback)
    // has no cycle of stages each waiting on its successor. Stream-ordered
    // backends are indifferent to the order (two independent streams).
    const bool prev_first = interleaved_ && stage_ == 0;
    if (prev_first && (send_b >= 0 || recv_f >= 0)) prev_link(send_b, recv_f);
    if (send_f >= 0 || recv_b >= 0) next_link(send_f, recv_b);
    if (!prev_first && (send_b >= 0 || recv_f >= 0)) prev_link(send_b, recv_f);
  }

  void enqueue_interleaved() {
    const int total = mb_ * V_;
    const int w = mb_ == S_ ? total : std::min((S_ - stage_ - 1) * 2 + (V_ - 1) * S_, total);
    const int rem = total - w;
    links(-1, -1, -1, in_f(0) ? 0 : -1);
    for (int k = 0; k < w; ++k) {
      fwd_chunk(k);
      const int rf = k + 1 < total && in_f(k + 1) ? k + 1 : -1;
      const int rb = k == w - 1 && rem > 0 && in_b(0) ? 0 : -1;
      links(out_f(k) ? k : -1, rb, -1, rf);
    }
    for (int j = 0; j < rem; ++j) {
      const int k = w + j;
      fwd_chunk(k);
      bwd_chunk(j);
      const int rf = k + 1 < total && in_f(k + 1) ? k + 1 : -1;
      const int rb = j + 1 < total && in_b(j + 1) ? j + 1 : -1;
      links(out_f(k) ? k : -1, rb, out_b(j) ? j : -1, rf);
    }
    if (rem == 0) links(-1, in_b(0) ? 0 : -1, -1, -1);
    for (int j = rem; j < total; ++j) {
      bwd_chunk(j);
      const int rb = j + 1 < total && in_b(j + 1) ? j + 1 : -1;
      links(-1, rb, out_b(j) ? j : -1, -1);
    }
    finish_iteration();
  }

  // ---------------------------------------------------------- DualPipe
  // Bidirectional pipeline (DeepSeek-V3's DualPipe, without its intra-chunk
  // attention/MLP split): every rank holds stage s of a "down" copy of the
  // model and stage S-1-s of an "up" copy; mb/2 microbatches enter at stage 0
  // and mb/2 at stage S-1, so the pipeline fills from both ends and each
  // link carries activations and gradients both ways at once. The order is a
  // tick schedule every rank computes identically: per tick each rank runs at
  // most one op - a forward within its 1F1B in-flight cap (S - position in
  // that copy: at most S + 1 activations per rank, DualPipe's budget), the
  // copy with fewer forwards issued first, else a backward (oldest first).
  // Forward-first comes within a few (f + b) of mb (f + b) + (S/2 - 1)(f + b)
  // and beats 1F1B's (mb + S - 1)(f + b) (schedule_sim.py); backward-first
  // stalls the steady state. Each op's output is sent at the end of its tick
  // and received by the neighbour at that same tick boundary into a buffer of
  // its own, so every boundary's send/receive groups pair up among themselves
  // (next link, then previous link: a chain, no cycle) - also for backends
  // whose groups complete on the host. Stages s and S-1-s sum their
  // gradients (pair all-reduce) before the DP all-reduce.
  struct DpOp {
    int dir = -1;  // 0 down, 1 up, -1 idle
    int mb = 0;
    bool bwd = false;
  };

  int dp_pos(int s, int dir) const { return dir == 0 ? s : S_ - 1 - s; }

  void build_dualpipe() {
    const int H = mb_ / 2;
    // done tick per (stage, dir, mb) for F and B; -1 = not yet
    std::vector<int> fdone(static_cast<size_t>(S_ * 2 * H), -1), bdone(fdone.size(), -1);
    auto idx = [&](int s, int d, int i) { return static_cast<size_t>((s * 2 + d) * H + i); };
    std::vector<int> nf(static_cast<size_t>(S_ * 2), 0), nb(nf.size(), 0);
    dp_ticks_.clear();
    int remaining = S_ * 2 * H * 2;
    for (int t = 0; remaining > 0; ++t) {
      DLNB_REQUIRE(t < 16 * (mb_ + S_) + 64, "dualpipe schedule did not converge");
      std::vector<DpOp> row(static_cast<size_t>(S_));
      for (int s = 0; s < S_; ++s) {
        DpOp best;
        {
          // forward first: the direction with fewer forwards issued (ties: the copy
          // whose first stage is nearer)
          int order[2] = {0, 1};
          const int f0 = nf[static_cast<size_t>(s * 2)], f1 = nf[static_cast<size_t>(s * 2 + 1)];
          if (f1 < f0 || (f1 == f0 && dp_pos(s, 1) < dp_pos(s, 0))) std::swap(order[0], order[1]);
          for (int d : order) {
            const int i = nf[static_cast<size_t>(s * 2 + d)];
            if (i >= H) continue;
            if (i - nb[static_cast<size_t>(s * 2 + d)] >= S_ - dp_pos(s, d)) continue;  // in-flight cap
            if (dp_pos(s, d) > 0) {
              const int up = d == 0 ? s - 1 : s + 1;
              const int fu = fdone[idx(up, d, i)];
              if (fu < 0 || fu >= t) continue;
            }
            best = DpOp{d, i, false};
            break;
          }
        }
        if (best.dir < 0) {
          // else a backward: the oldest ready microbatch over both directions
          for (int d = 0; d < 2; ++d) {
            const int i = nb[static_cast<size_t>(s * 2 + d)];
            if (i >= nf[static_cast<size_t>(s * 2 + d)]) continue;
            const int fd = fdone[idx(s, d, i)];
            if (fd < 0 || fd >= t) continue;
            if (dp_pos(s, d) < S_ - 1) {
              const int down = d == 0 ? s + 1 : s - 1;  // the next stage of this copy
              const int bd = bdone[idx(down, d, i)];
              if (bd < 0 || bd >= t) continue;
            }
            if (best.dir < 0 || i < best.mb) best = DpOp{d, i, true};
          }
        }
        if (best.dir >= 0) {
          if (best.bwd) {
            bdone[idx(s, best.dir, best.mb)] = t;
            ++nb[static_cast<size_t>(s * 2 + best.dir)];
          } else {
            fdone[idx(s, best.dir, best.mb)] = t;
            ++nf[static_cast<size_t>(s * 2 + best.dir)];
          }
          --remaining;
        }
        row[static_cast<size_t>(s)] = best;
      }
      dp_ticks_.push_back(row);
    }
    // compute-only makespan of this order (the strategy's floor)
    std::vector<double> ffin(fdone.size(), 0), bfin(fdone.size(), 0), free_at(static_cast<size_t>(S_), 0);
    double span = 0;
    for (const auto& row : dp_ticks_)
      for (int s = 0; s < S_; ++s) {
        const DpOp& op = row[static_cast<size_t>(s)];
        if (op.dir < 0) continue;
        double start = free_at[static_cast<size_t>(s)];
        const int d = op.dir, i = op.mb;
        if (!op.bwd) {
          if (dp_pos(s, d) > 0) start = std::max(start, ffin[idx(d == 0 ? s - 1 : s + 1, d, i)]);
          ffin[idx(s, d, i)] = start + fwd_mb_us_;
          free_at[static_cast<size_t>(s)] = ffin[idx(s, d, i)];
        } else {
          start = std::max(start, ffin[idx(s, d, i)]);
          if (dp_pos(s, d) < S_ - 1) start = std::max(start, bfin[idx(d == 0 ? s + 1 : s - 1, d, i)]);
          bfin[idx(s, d, i)] = start + bwd_mb_us_;
          free_at[static_cast<size_t>(s)] = bfin[idx(s, d, i)];
        }
        span = std::max(span, free_at[static_cast<size_t>(s)]);
      }
    dp_floor_us_ = span;
    // The pair's gradient of model stage max(s, S-1-s) is final once the
    // chunks holding it (down copy on the higher rank, up copy on the lower:
    // both at position >= S/2, early in their backward chains) have run their
    // last backward; both ranks reduce it at the end of that same tick, so the
    // all-reduce overlaps the rest of the backward and host-side rendezvous
    // stays tick-ordered.
    const int lo = std::min(stage_, S_ - 1 - stage_), hi = S_ - 1 - lo;
    mirror_early_tick_ = std::max(bdone[idx(lo, 1, H - 1)], bdone[idx(hi, 0, H - 1)]);
    // With EP the non-expert gradients [0, ne_) - which span the early half -
    // are first all-reduced over the EP group on the compute stream at the end
    // of the backward (reference order: EP, then DP); an early pair / DP
    // all-reduce of that range would race it. MoE syncs the whole gradient
    // after the backward instead.
    if (has_ep_) mirror_early_tick_ = -1;
    for (size_t k = 0; k < dp_ticks_.size(); ++k) {
      const DpOp& op = dp_ticks_[k][static_cast<size_t>(stage_)];
      if (op.dir >= 0 && op.bwd) last_bwd_tick_ = static_cast<int>(k);
    }
  }

  // Event / buffer slot of (dir, mb): activations [0, mb), gradients [mb, 2 mb).
  int dp_slot(int dir, int i) const { return dir * (mb_ / 2) + i; }

  // One link's group at a tick boundary: what this rank's op of the tick
  // sends over it, and what the neighbour's op of the tick sends to us.
  void dualpipe_link(bool next, const DpOp& mine, const DpOp& theirs) {
    Communicator* c = next ? next_.get() : prev_.get();
    if (!c) return;
    Stream& ls = next ? *next_stream_ : *prev_stream_;
    const int peer = next ? next_peer_ : prev_peer_;
    // our output travels towards `next` for down-forwards and up-backwards
    const bool send = mine.dir >= 0 && ((mine.dir == 0) != mine.bwd) == next &&
                      (mine.bwd ? dp_pos(stage_, mine.dir) > 0 : dp_pos(stage_, mine.dir) < S_ - 1);
    const int nstage = stage_ + (next ? 1 : -1);
    const bool recv = theirs.dir >= 0 && ((theirs.dir == 0) != theirs.bwd) == !next &&
                      (theirs.bwd ? dp_pos(nstage, theirs.dir) > 0 : dp_pos(nstage, theirs.dir) < S_ - 1);
    if (!send && !recv) return;
    const DType t = ctx_->wire;
    if (send) ls.wait(mine.bwd ? *bwd_done_[dp_slot(mine.dir, mine.mb)] : *fwd_done_[dp_slot(mine.dir, mine.mb)]);
    int tk = timers_->begin(ls);
    c->group_start();
    if (send) c->send(next ? act_out_[0].data() : grad_out_[0].data(), pipe_, t, peer, ls);
    const int slot = recv ? dp_slot(theirs.dir, theirs.mb) : 0;
    if (recv) c->recv(dpbuf_[static_cast<size_t>(theirs.bwd ? mb_ + slot : slot)].data(), pipe_, t, peer, ls);
    c->group_end();
    timers_->end(tk, ls, send ? "pp_send_time" : "pp_recv_time");
    if (recv) ls.record(theirs.bwd ? *recv_b_[slot] : *recv_f_[slot]);
  }

  void enqueue_dualpipe() {
    int tick = 0;
    for (const auto& row : dp_ticks_) {
      const DpOp& op = row[static_cast<size_t>(stage_)];
      if (op.dir >= 0) {
        const int slot = dp_slot(op.dir, op.mb);
        if (!op.bwd) {
          if (dp_pos(stage_, op.dir) > 0)
            timers_->stall_before_task(*compute_, *recv_f_[slot], "pp_comm_time");
          else
            timers_->add("pp_comm_time", 0.0);
          micro_compute(fwd_mb_us_, fwd_mb_flops_);
          compute_->record(*fwd_done_[slot]);
        } else {
          if (dp_pos(stage_, op.dir) < S_ - 1)
            timers_->stall_before_task(*compute_, *recv_b_[slot], "pp_comm_time");
          else
            timers_->add("pp_comm_time", 0.0);
          micro_compute(bwd_mb_us_, bwd_mb_flops_);
          compute_->record(*bwd_done_[slot]);
        }
      }
      if (next_) dualpipe_link(true, op, row[static_cast<size_t>(stage_ + 1)]);
      if (prev_) dualpipe_link(false, op, row[static_cast<size_t>(stage_ - 1)]);
      if (tick == mirror_early_tick_) {
        compute_->record(*mirror_ready_);
        dp_stream_->wait(*mirror_ready_);
        void* g = grad_.data();
        int tm = timers_->begin(*dp_stream_);
        mirror_comm_->all_reduce(g, g, dp_ar_ / 2, ctx_->wire, *dp_stream_);
        timers_->end(tm, *dp_stream_, "pp_mirror_time");
        dp_allreduce_bucket(0, 2);  // and that half's DP all-reduce right behind it
      }
      ++tick;
    }
    finish_iteration();
  }

  void enqueue_iteration() override {
    // Lane graphs: the compute stream's tasks of the iteration are one compute
    // program (one persistent kernel); its event waits and records - the
    // receives', the inner lane's, the sends' and the DP buckets' - fold into
    // the tasks' gates (Device::StreamFold), so no other kernel sits between
    // two tasks on the compute lane
    dp_end_ = nullptr;
    // The TP / EP collectives go on the inner lane under lane graphs (the
    // compute lane must hold only compute and its waits); with the single
    // graph or eager they stay on the compute stream. Ranks sharing a GPU
    // (4 over xgmi, profiles/pipeline_program_r6.md): the inner lane ran C3
    // 795 against 810 ms and C4 2802 against 379 ms on the compute stream.
    inner_lane_ = !inner_on_compute_ && ctx_->dev->gate_events();
    prog_ = ctx_->dev->gate_events() && !reference_ && program_ok() && ctx_->compute->begin_program(*compute_);
    if (dualpipe_)
      enqueue_dualpipe();
    else if (interleaved_)
      enqueue_interleaved();
    else if (one_f_one_b_)
      enqueue_1f1b();
    else
      enqueue_gpipe();
  }

  void dp_allreduce_bucket(int k, int nbk) {
    const uint64_t base = dp_ar_ / nbk, rem = dp_ar_ % nbk;
    const uint64_t off = k * base + std::min<uint64_t>(k, rem);
    const uint64_t n = base + (static_cast<uint64_t>(k) < rem ? 1 : 0);
    void* in = grad_.at(off * es_);
    void* out = ctx_->opt.in_place ? in : sum_grad_.at(off * es_);
    int tk = timers_->begin(*dp_stream_);
    dp_comm_->all_reduce(in, out, n, ctx_->wire, *dp_stream_);
    dp_end_ = timers_->end(tk, *dp_stream_, "dp_comm_time");
  }

  // Whether the compute lane may be one compute program: not with TP or EP
  // groups of > 1 rank. Their collectives sit on the critical path between
  // two compute tasks (the compute waits for each), and a program keeps its
  // grid resident through those waits, leaving the collective only the CUs
  // reserved for communication; with one launch per task the collective gets
  // the CUs the finished task freed. hybrid_3d 1 4 2 on two ranks sharing GPU
  // 0 (profiles/pipeline_program_r6.md): program 82.9 ms, one launch per task
  // 80.6, single graph 80.3 at 32 CTAs per lane.
  // CTAs of TP / EP groups of > 1 rank: the backend's own (0), except with
  // lane graphs on a shared device (DLNB_LANE_SHARED=1): there one rank's
  // spinning collective CTAs can starve another rank's compute task that the
  // collective waits for (a 5-s gate timeout now and then), so the lane budget.
  static int inner_ctas(const Context& ctx) {
    const int forced = env_int("DLNB_INNER_CTAS", -1);
    if (forced >= 0) return forced;
    return ctx.ranks_on_device > 1 && env_int("DLNB_LANE_SHARED", 0) != 0 ? ctx.lane_ctas : 0;
  }
  // DualPipe takes the single graph (below).
  bool program_ok() const {
    const int forced = env_int("DLNB_PIPELINE_PROGRAM", -1);  // A/B: 0 never, 1 always (lane graphs)
    if (forced >= 0) return forced != 0;
    return !(has_tp_ && T_ > 1) && !(has_ep_ && E_ > 1) && !dualpipe_;
  }

  std::vector<Stream*> streams() override {
    std::vector<Stream*> ss = {compute_.get(), dp_stream_.get()};
    if (prev_) ss.push_back(prev_stream_.get());
    if (next_) ss.push_back(next_stream_.get());
    return ss;
  }
  bool capturable() const override { return !reference_; }
  // (TP / EP collectives are on the inner lane: the compute lane carries compute and waits only)
  // DualPipe: its lanes (with or without a program) ran 166-167 ms against
  // 152-162 ms on the single graph, two ranks on one GPU (round 6).
  bool lanes_without_program() const override { return !dualpipe_; }

  void synchronize() override {
    std::vector<Stream*> ss = {compute_.get(), dp_stream_.get()};
    std::vector<Communicator*> cs = {dp_comm_.get()};
    if (prev_) {
      ss.push_back(prev_stream_.get());
      cs.push_back(prev_.get());
    }
    if (next_) {
      ss.push_back(next_stream_.get());
      cs.push_back(next_.get());
    }
    if (tp_comm_) cs.push_back(tp_comm_.get());
    if (ep_comm_) cs.push_back(ep_comm_.get());
    if (mirror_comm_) cs.push_back(mirror_comm_.get());
    sync_streams(ss, cs, *ctx_->dev);
    timers_->resolve();
  }

  double compute_floor_us(const Context&) const override {
    // GPipe / 1F1B: (mb + S - 1)(f + b); interleaved: the bubble / V
    if (dualpipe_) return dp_floor_us_;
    return (mb_ + static_cast<double>(S_ - 1) / V_) * (fwd_mb_us_ + bwd_mb_us_);
  }

  std::string tail_collective_timer() const override { return "dp_comm_time"; }
  std::string section_id() const override {
    return kind_ == StrategyKind::Hybrid2D      ? "dp_pp"
           : kind_ == StrategyKind::Hybrid3D    ? "dp_pp_tp"
           : kind_ == StrategyKind::Hybrid3DMoE ? "dp_pp_ep"
                                                : "dp_pp_tp_ep";
  }
  std::string section_title() const override {
    return kind_ == StrategyKind::Hybrid2D      ? "Data + Pipeline Parallelism"
           : kind_ == StrategyKind::Hybrid3D    ? "Data + Pipeline + Tensor Parallelism"
           : kind_ == StrategyKind::Hybrid3DMoE ? "Data + Pipeline + Expert Parallelism"
                                                : "Data + Pipeline + Tensor + Expert Parallelism";
  }

  Json global_json() const override {
    const Context& ctx = *ctx_;
    Json g = Json::object();
    g["model_name"] = ctx.opt.model;
    g["num_stages"] = S_;
    g["num_microbatches"] = mb_;
    if (has_tp_) g["num_tensor_shards"] = T_;
    if (has_ep_) {
      g["num_expert_shards"] = E_;
      g["num_experts"] = ctx.stats.experts;
      g["sequence_length"] = ctx.stats.seq_len;
      g["embedded_dim"] = ctx.stats.embedded_dim;
    }
    g["samples_per_microbatch"] = spmb_;
    g["local_batch_size"] = ctx.stats.batch_size;
    // hybrid_2d.cpp:453 reports world*B/S; hybrid_3d.cpp:530 dp_size*B.
    g["global_batch_size"] = kind_ == StrategyKind::Hybrid2D
                                 ? static_cast<uint64_t>(ctx.world()) * ctx.stats.batch_size / S_
                                 : static_cast<uint64_t>(dp_size_) * ctx.stats.batch_size;
    g["world_size"] = ctx.world();
    g["dp_size"] = dp_size_;
    g["num_layers"] = L_;
    g["fwd_rt_per_microbatch"] = fwd_mb_us_;
    g["bwd_rt_per_microbatch"] = bwd_mb_us_;
    g["total_model_size_params"] = ctx.stats.model_size;
    g["pipe_msg_size_bytes"] = pipe_ * es_;
    if (has_tp_) g["tp_allreduce_size_bytes"] = tp_ar_ * es_;
    if (has_tp_) g["sequence_parallel"] = sp_;
    if (has_ep_) {
      g["ep_alltoall_size_bytes"] = a2a_ * es_;
      g["ep_allreduce_size_bytes"] = ne_ * es_;
      if (skew_) {
        g["ep_imbalance"] = ctx.opt.ep_imbalance;
        Json c = Json::array();
        for (uint64_t v : skew_counts_) c.push_back(static_cast<double>(v * es_));
        g["ep_dispatch_bytes_per_peer"] = c;  // sent by every rank to EP rank j
      }
    }
    g["dp_allreduce_size_bytes"] = dp_ar_ * es_;
    g["pp_schedule"] = ctx.opt.pp_schedule;
    if (interleaved_) g["pp_virtual_stages"] = V_;
    if (dualpipe_) g["dualpipe_ticks"] = static_cast<uint64_t>(dp_ticks_.size());
    if (has_ep_) g["ep_overlap"] = ep_overlap_;
    if (has_tp_) g["tp_granularity"] = ctx.opt.tp_granularity;
    g["device"] = ctx.dev->kind() == DeviceKind::CPU ? "CPU" : "GPU";
    g["backend"] = dp_comm_->backend_name();
    return g;
  }

  Json rank_json() const override {
    Json r = Json::object();
    r["runtimes"] = timers_->values_json("runtimes");
    r["pp_comm_time"] = timers_->values_json("pp_comm_time");
    r["dp_comm_time"] = timers_->values_json("dp_comm_time");
    if (has_tp_) {
      r["tp_comm_time"] = timers_->values_json("tp_comm_time");  // the compute's waits for TP (exposed)
      r["tp_ar_time"] = timers_->values_json("tp_ar_time");      // each all-reduce on the inner lane
    }
    if (has_ep_) {
      r["ep_comm_time"] = timers_->values_json("ep_comm_time");
      r["ep_a2a_time"] = timers_->values_json("ep_a2a_time");
      r["dp_ep_comm_time"] = timers_->values_json("dp_ep_comm_time");
    }
    r["pp_send_time"] = timers_->values_json("pp_send_time");
    r["pp_recv_time"] = timers_->values_json("pp_recv_time");
    r["dp_exposed_time"] = timers_->values_json("dp_exposed_time");
    if (dualpipe_) {
      r["pp_mirror_time"] = timers_->values_json("pp_mirror_time");
      r["dualpipe_early_sync_tick"] = mirror_early_tick_;  // -1: whole gradient after the backward (MoE)
      r["dualpipe_last_backward_tick"] = last_bwd_tick_;
    }
    r["stage_id"] = stage_;
    if (has_tp_) r["tp_id"] = tp_id_;
    if (has_ep_) r["ep_id"] = ep_id_;
    if (kind_ != StrategyKind::Hybrid2D) r["dp_id"] = dp_id_;
    return r;
  }

  Json comm_summary() const override { return comm_stats_json(stats_, *timers_); }

 private:
  StrategyKind kind_;
  Context* ctx_ = nullptr;
  int S_ = 1, mb_ = 1, inner_ = 1, L_ = 0, layers_per_stage_ = 0, dp_size_ = 1;
  int stage_ = 0, inner_id_ = 0, dp_id_ = 0, tp_id_ = 0, ep_id_ = 0, T_ = 1, E_ = 1;
  bool has_tp_ = false, has_ep_ = false, sp_ = false;
  uint64_t tp_shard_ = 0;  // ceil(tp_ar_ / T): sequence-parallel shard
  bool reference_ = false;
  bool inner_on_compute_ = false;
  bool inner_lane_ = false;  // this enqueue puts the TP / EP collectives on the inner lane
  bool one_f_one_b_ = false, interleaved_ = false, dualpipe_ = false;
  std::vector<std::vector<DpOp>> dp_ticks_;  // [tick][stage]
  double dp_floor_us_ = 0;
  int mirror_early_tick_ = -1;  // tick after which the first half of the mirror all-reduce is issued (-1: none)
  int last_bwd_tick_ = -1;      // this stage's last backward tick (dualpipe)
  std::unique_ptr<Event> mirror_ready_;
  std::vector<Buffer> dpbuf_;  // receive buffers per (dir, microbatch): activations, then gradients
  std::unique_ptr<Communicator> mirror_comm_;
  int V_ = 1, layers_per_chunk_ = 0;
  bool ep_overlap_ = false;
  bool skew_ = false;                   // --ep-imbalance > 0
  std::vector<uint64_t> skew_counts_;   // elements every rank dispatches to EP rank j
  uint64_t skew_call_ = 0;
  Stream* ep_stream_ = nullptr;  // = dp_stream_ (see setup)
  std::unique_ptr<Event> chunk_done_[2], a2a_done_[2];
  std::unique_ptr<Event> inner_ready_, inner_done_;  // compute -> inner lane -> compute (inner_comm)
  uint64_t spmb_ = 0, pipe_ = 0, dp_ar_ = 0, tp_ar_ = 0, ne_ = 0, a2a_ = 0;
  size_t es_ = 2;
  double fwd_mb_us_ = 0, bwd_mb_us_ = 0, fwd_mb_flops_ = 0, bwd_mb_flops_ = 0;
  std::unique_ptr<Communicator> prev_, next_, tp_comm_, ep_comm_, dp_comm_;
  int prev_peer_ = 0, next_peer_ = 1;
  std::unique_ptr<Stream> compute_, prev_stream_, next_stream_, dp_stream_;
  Buffer act_in_[2], act_out_[2], grad_in_[2], grad_out_[2];
  Buffer grad_, sum_grad_, tp_buf_, tp_res_, ep_send_, ep_recv_, params_, mom_;
  std::vector<std::unique_ptr<Event>> recv_f_, fwd_done_, send_f_, recv_b_, bwd_done_, send_b_, bucket_ready_;
  std::unique_ptr<Event> dp_done_;
  const uint64_t* inner_end_ = nullptr;
  const uint64_t* dp_end_ = nullptr;  // the DP lane's last end stamp of the iteration
  bool prog_ = false;                 // the iteration's compute tasks are one compute program
  std::vector<CommStat> stats_;
};

}  // namespace

std::unique_ptr<Strategy> make_pipeline(StrategyKind kind) { return std::unique_ptr<Strategy>(new Pipeline(kind)); }

}  // namespace dlnb
