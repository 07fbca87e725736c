#include "dlnb/compute.hpp"

#include <algorithm>
#include <cmath>
#include <exception>
#include <map>
#include <set>

#include "dlnb/kernels.hpp"
#include "dlnb/timers.hpp"

namespace dlnb {

ComputeMode parse_compute_mode(const std::string& s, DeviceKind dev) {
  if (s == "auto") return dev == DeviceKind::GPU ? ComputeMode::Gemm : ComputeMode::Sleep;
  if (s == "sleep") return ComputeMode::Sleep;
  if (s == "spin") return ComputeMode::Spin;
  if (s == "gemm") return ComputeMode::Gemm;
  if (s == "gemm-work" || s == "gemm_work") return ComputeMode::GemmWork;
  if (s == "flops") return ComputeMode::Flops;
  DLNB_THROW("unknown compute mode '" << s << "' (auto, sleep, spin, gemm, flops)");
}

const char* compute_mode_name(ComputeMode m) {
  switch (m) {
    case ComputeMode::Sleep: return "sleep";
    case ComputeMode::Spin: return "spin";
    case ComputeMode::Gemm: return "gemm";
    case ComputeMode::GemmWork: return "gemm-work";
    case ComputeMode::Flops: return "flops";
  }
  return "?";
}

namespace {

// ------------------------------------------------------------------ CPU

class CpuCompute : public ComputeEngine {
 public:
  CpuCompute(Device& dev, ComputeMode mode, double scale) : dev_(dev), mode_(mode), scale_(scale) {}
  void run(Stream& s, double us, double) override {
    double d = us * scale_;
    if (d <= 0) return;
    if (mode_ == ComputeMode::Spin) {
      dev_.host_task(s, [d] {
        double end = now_s() + d * 1e-6;
        volatile double x = 1.0;
        while (now_s() < end) x = x * 1.0000001 + 1e-9;
      });
    } else {
      // sleep; gemm/flops have no CPU implementation and fall back to sleep.
      dev_.host_task(s, [d] { precise_sleep_us(d); });
    }
  }
  Json describe() const override {
    Json j = Json::object();
    j["mode"] = compute_mode_name(mode_);
    j["effective_mode"] = mode_ == ComputeMode::Spin ? "spin" : "sleep";
    j["time_scale"] = scale_;
    return j;
  }
  ComputeMode mode() const override { return mode_; }

 private:
  Device& dev_;
  ComputeMode mode_;
  double scale_;
};

// ------------------------------------------------------------------ GPU

// Fixed-work calibration of the program kernel: one full-K round (every block
// of the grid one 256 x 256 tile) and one K-tile of the tail tile.
struct FixedCal {
  double round_us = 0.0;
  double ktile_us = 0.0;
};

// The work of one fixed-work task: full-K rounds plus a tail tile of tail_kt
// K-tiles per block, and its uncontended duration.
struct FixedWork {
  uint32_t rounds = 0, tail_kt = 0;
  double us = 0.0;
};

class GpuCompute : public ComputeEngine {
 public:
  GpuCompute(Device& dev, ComputeMode mode, const ComputeShape& shape, double scale)
      : dev_(dev), mode_(mode), scale_(scale) {
    // (the rate itself is taken at the first task, kernels::wallclock_hz; the
    // absorb cap needs no ppm)
    absorb_ticks_ = static_cast<uint32_t>(std::max<double>(
        static_cast<double>(env_int("DLNB_CHAIN_ABSORB_US", 30)) * 1e-6 * kernels::wallclock_hz_nominal(dev.index()), 1.0));
    cus_ = kernels::num_cus(dev.index());
    gate_timeout_ticks_ = static_cast<uint64_t>(static_cast<double>(env_int("DLNB_GATE_TIMEOUT_S", 60)) *
                                                kernels::wallclock_hz_nominal(dev.index()));
    dtype_ = shape.dtype == DType::FP8_E4M3 ? DType::FP8_E4M3 : DType::BF16;
    fixed_ = mode_ == ComputeMode::GemmWork || mode_ == ComputeMode::Flops;
    // The stand-in is the layer's FFN down projection, C[tokens, hidden] =
    // A[tokens, ffn] . W[hidden, ffn]^T: its long K (the FFN width) keeps
    // the per-tile pipeline fill / drain of the persistent kernel small. At
    // the up-projection shape used before (K = hidden) the deadline kernel did
    // 0.725 -> 0.787 less MFMA busy per clock on its CUs (bf16 llama3_8b) and
    // 1810 vs 2672 TF/s (fp8 ViT-H, K = 1280) (profiles/deadline_shapes_r3.md).
    // K: a multiple of 128 (bf16: an even K-tile count, the balanced body) or
    // 256 bytes (fp8: the one-wave-per-SIMD MX kernel).
    const int kmul = dtype_ == DType::FP8_E4M3 ? 256 : 128;
    K_ = std::min(65536, std::max(512, (shape.ffn + kmul - 1) / kmul * kmul));
    N_ = std::min(32768, std::max(1024, (shape.hidden + 255) / 256 * 256));
    // The operands must fit beside the strategy's buffers: at most 1/8 of this
    // rank's share of free memory (ranks sharing the GPU each allocate their
    // own set). Large-FFN models (K = ffn up to 64 Ki) shrink K, keeping its
    // multiple (ffn 53248 x hidden 16384 is ~2.6 GB per rank).
    if (mode_ != ComputeMode::Sleep && mode_ != ComputeMode::Spin) {
      const size_t esz = dtype_size(dtype_);
      const double share = static_cast<double>(dev_.free_memory()) / std::max(1, shape.ranks_on_device) / 8.0;
      auto bytes = [&](int k) {
        return static_cast<double>(kMmax + N_) * k * esz + static_cast<double>(kMmax) * N_ * 2;
      };
      while (K_ > 512 && share > 0 && bytes(K_) > share) K_ = std::max(512, (K_ / 2 + kmul - 1) / kmul * kmul);
    }
    // GEMM operands for every GEMM mode
    if (mode_ != ComputeMode::Sleep && mode_ != ComputeMode::Spin) alloc_operands();
    if (mode_ == ComputeMode::Gemm || fixed_) {
      // one 64-byte line per compute stream; the counters (DlCounter)
      slots_ = dev_.alloc(kSlots * 64);
      counters_ = dev_.alloc(kernels::kNumCounters * sizeof(uint64_t));
      // compute programs' task lists: a device ring (lists captured into a
      // graph, uploaded after the capture) and a host-mapped ring (lists
      // launched at once: written by the host, read by the kernel, no copy)
      prog_dev_ = dev_.alloc(kProgTasks * sizeof(kernels::DlTask));
      prog_host_ = reinterpret_cast<kernels::DlTask*>(dev_.alloc_stamps(kProgTasks * sizeof(kernels::DlTask) / 8));
      auto zs = dev_.create_stream(false);
      dev_.memset_async(slots_.data(), 0, kSlots * 64, *zs);
      dev_.memset_async(counters_.data(), 0, kernels::kNumCounters * sizeof(uint64_t), *zs);
      zs->synchronize();
      // Leave `comm_cus` CUs to collectives: one 128-KiB-LDS block fits per
      // CU, so a grid of CUs - comm_cus blocks never touches those CUs and
      // RCCL / copy kernels on the high-priority comm streams always find
      // room (with the whole chip taken, a comm kernel only starts at a
      // compute boundary, and overlap collapses).
      grid_ = std::max(1, cus_ - std::max(0, shape.comm_cus));
      // Fixed work waits for every block of its grid between two tasks, so
      // ranks sharing the device split the free CUs: all their grids must be
      // resident at once.
      if (fixed_) grid_ = std::max(1, grid_ / std::max(1, shape.ranks_on_device));
    }
    if (mode_ == ComputeMode::Gemm) {
      // One launch per task by default. Cutting a task into relaunched
      // slices (DLNB_GEMM_SLICE_US > 0) was meant to give collectives CUs at
      // slice boundaries, which the comm_cus reservation already does; at
      // 500-us slices every slice also abandons a partial 256 x 256 tile and
      // pays a prologue: 630 vs 679 TF/s per GHz on the headline
      // (profiles/slice_ab_r3.md), and a 4x larger graph.
      // Ranks sharing one GPU (loopback, -d 0,0) keep 500-us slices: with one
      // launch per task a rank's persistent grid holds the CUs for its whole
      // task and the other ranks' compute (and so the collectives that wait
      // for it) serialises behind it - 8 loopback ranks of the llama3_8b FSDP
      // config ran 459 vs 317 ms per iteration (profiles/loopback_w8_r3.md).
      slice_us_ = static_cast<double>(env_int("DLNB_GEMM_SLICE_US", shape.ranks_on_device > 1 ? 500 : 0));
    } else {
      slice_us_ = 0.0;
    }
    if (fixed_) {
      DLNB_REQUIRE(kernels::deadline_program_ok(kMmax, N_, K_, dtype_),
                   "fixed-work compute: no program kernel for the stand-in shape " << kMmax << "x" << N_ << "x" << K_);
      calibrate();
    }
  }
  ~GpuCompute() override {
    // (a task list a kernel may still read is never freed: the process is going away)
    if (prog_host_ && !dev_.abort_raised())
      dev_.free_stamps(reinterpret_cast<uint64_t*>(prog_host_), kProgTasks * sizeof(kernels::DlTask) / 8);
  }

  void reset_clocks(Stream& s) override {
    if (slots_.data()) dev_.memset_async(slots_.data(), 0, kSlots * 64, s);
  }
  void reset_slot(Stream& s) override {
    if (!slots_.data()) return;
    auto it = slot_of_.find(&s);
    if (it != slot_of_.end()) dev_.memset_async(slots_.as<uint64_t>() + it->second * 8, 0, 64, s);
  }
  void reset_capped(Stream& s) override {
    // the capped / absorbed counts (the timeouts stay: counted since start)
    if (!counters_.data()) return;
    uint64_t* c = counters_.as<uint64_t>();
    dev_.memset_async(c + kernels::kCappedTasks, 0, 2 * sizeof(uint64_t), s);
    dev_.memset_async(c + kernels::kAbsorbedTicks, 0, 2 * sizeof(uint64_t), s);
  }
  bool begin_program(Stream& s) override {
    if ((mode_ != ComputeMode::Gemm && !fixed_) || slice_us_ > 0 || env_int("DLNB_COMPUTE_PROGRAMS", 1) == 0 ||
        !kernels::deadline_program_ok(kMmax, N_, K_, dtype_))
      return false;
    Program& p = programs_[&s];
    DLNB_REQUIRE(!p.open, "begin_program: a program is already open on this stream");
    p.open = true;
    p.index = 0;
    p.tasks.clear();
    p.pending.clear();
    p.done_free = false;
    p.split = false;
    if (dev_.gate_events()) {
      // the stream's gate-event waits and records between the tasks become
      // the tasks' gates and done gates (gate-only tasks where none fits):
      // no gate kernel on the stream while its program is being built
      p.fold.e = this;
      p.fold.s = &s;
      dev_.set_stream_fold(s, &p.fold);
    }
    return true;
  }
  void end_program(Stream& s, bool join_ok) override {
    auto it = programs_.find(&s);
    if (it == programs_.end() || !it->second.open) return;
    Program& p = it->second;
    dev_.set_stream_fold(s, nullptr);
    emit_pending(s, p, nullptr, 0);  // waits after the last task: before the join
    auto j = joins_.find(&s);
    if (j != joins_.end() && !p.tasks.empty() && join_ok) {
      // the join task(s): up to two gates each, the last one stores the done word
      const Join& jn = j->second;
      size_t g = 0;
      do {
        kernels::DlTask t;
        t.sync.iter = dev_.iter_word();
        t.sync.counters = counters_.as<uint64_t>();
        t.sync.gate_timeout = gate_timeout_ticks_;
        t.sync.abort = dev_.abort_word();
        for (int i = 0; i < 2 && g < jn.gates.size(); ++i, ++g) {
          t.sync.gate[i] = jn.gates[g];
          t.sync.tag[i] = jn.tag;
        }
        if (g >= jn.gates.size()) t.sync.tstart[0] = jn.host_done;
        t.ticks = 0;
        p.tasks.push_back(t);
      } while (g < jn.gates.size());
      joins_.erase(j);
      joined_.insert(&s);
    }
    flush_program(s);
    p.open = false;
  }
  void set_lane_join(Stream& s, const std::vector<uint64_t*>& gates, uint32_t tag, uint64_t* host_done) override {
    if (mode_ != ComputeMode::Gemm && !fixed_) return;
    joins_[&s] = Join{gates, tag, host_done};
    joined_.erase(&s);
    lane_stats_.clear();
  }
  bool program_joined(Stream& s) override { return joined_.count(&s) != 0; }
  bool program_split(Stream& s) override {
    auto it = programs_.find(&s);
    return it != programs_.end() && it->second.split;
  }
  long programs_on(Stream& s) override {
    auto it = program_count_.find(&s);
    return it == program_count_.end() ? 0 : it->second;
  }
  void set_gate_timeout(double s) override {
    gate_timeout_ticks_ = static_cast<uint64_t>(s * kernels::wallclock_hz_nominal(dev_.index()));
  }
  double lane_task_us(Stream& s) override {
    auto it = lane_stats_.find(&s);
    if (it == lane_stats_.end() || it->second.n == 0 || !it->second.single) return -1.0;
    return it->second.us / static_cast<double>(it->second.n);
  }
  void after_capture() override {
    joins_.clear();  // a join no program took does not carry over
    if (uploads_.empty()) return;
    auto st = dev_.create_stream(false);
    for (const auto& u : uploads_)
      dev_.copy_async(u.dst, u.tasks.data(), u.tasks.size() * sizeof(kernels::DlTask), *st);
    st->synchronize();
    uploads_.clear();
  }

  bool chain_counters(ChainCounters& out) override {
    if (!counters_.data()) return false;
    uint64_t v[kernels::kNumCounters] = {};
    auto st = dev_.create_stream(false);
    dev_.copy_async(v, counters_.data(), sizeof(v), *st);
    st->synchronize();
    out.capped_tasks = static_cast<double>(v[kernels::kCappedTasks]);
    out.capped_s = static_cast<double>(v[kernels::kCappedTicks]) / hz();
    out.absorbed_tasks = static_cast<double>(v[kernels::kAbsorbedTasks]);
    out.absorbed_s = static_cast<double>(v[kernels::kAbsorbedTicks]) / hz();
    out.wait_timeouts = static_cast<double>(v[kernels::kWaitTimeouts]);
    out.gate_timeouts = static_cast<double>(v[kernels::kGateTimeouts]);
    out.aborted = static_cast<double>(v[kernels::kAborted]);
    out.late_blocks = static_cast<double>(v[kernels::kLateBlocks]);
    return true;
  }

  // Every GPU mode's kernels stamp their own start (deadline / idle / spin:
  // the kernel; fixed work: the program task, which also stamps its end).
  bool stamps_task_start() const override { return true; }
  uint64_t task_ticks(double us) const override { return fixed_ ? 0 : ticks(us * scale_); }
  const uint64_t* last_task_end(Stream& s) override {
    auto it = last_end_.find(&s);
    return it == last_end_.end() ? nullptr : it->second;
  }
  void run(Stream& s, double us, double flops) override { run_stamped(s, us, flops, nullptr); }

  void run_chained(Stream& s, double us, double flops, uint64_t* start, Event* done) override {
    if (fixed_) {
      fixed_task(s, us, flops, start, {}, done);
      return;
    }
    if (mode_ == ComputeMode::Gemm && us * scale_ >= 20.0 && chain_live_[slot_for(s)]) {
      note_task(s, us * scale_);
      if (stall_timers_ && !start) start = stall_timers_->task_slot(s);
      StartNote note{stall_timers_, s, start, ticks(us * scale_), nullptr};
      kernels::DlSync sync;
      sync.tstart[0] = start;
      sync.tstart[1] = extra_start_;
      extra_start_ = nullptr;
      deadline_task(s, us * scale_, sync, true, done);
      ++chained_;
      return;
    }
    run_stamped(s, us, flops, start);
    if (done) s.record(*done);
  }

  bool gates_task(double us) const override { return fixed_ || (mode_ == ComputeMode::Gemm && us * scale_ >= 20.0); }

  int make_gate() override {
    DLNB_REQUIRE(mode_ == ComputeMode::Gemm || fixed_, "gates need the gemm (deadline) or fixed-work GPU compute");
    gates_.push_back(dev_.alloc_gate());
    gate_tag_.push_back(0);
    return static_cast<int>(gates_.size()) - 1;
  }

  void signal(Stream& s, int gate) override {
    uint32_t& tag = gate_tag_.at(gate);
    tag = tag == 0xffffffffu ? 1u : tag + 1;
    kernels::gate_signal(gates_.at(gate), dev_.iter_word(), tag, s.native());
  }
  void wait_gate(Stream& s, int gate, double timeout_us) override {
    const uint32_t tag = gate_tag_.at(gate);
    DLNB_REQUIRE(tag != 0, "wait_gate: gate " << gate << " was never signalled");
    kernels::gate_wait(gates_.at(gate), dev_.iter_word(), tag, ticks(timeout_us),
                       counters_.as<uint64_t>() + kernels::kWaitTimeouts, s.native(), dev_.abort_word());
  }

  void run_gated(Stream& s, double us, double flops, const std::vector<int>& gates, uint64_t* start,
                 bool chain, Event* done) override {
    DLNB_REQUIRE(gates_task(us), "run_gated: the task cannot wait on gates (see gates_task)");
    DLNB_REQUIRE(gates.size() <= 2, "run_gated: at most 2 gates per task");
    kernels::DlSync sync;
    for (size_t i = 0; i < gates.size(); ++i) {
      sync.gate[i] = gates_.at(gates[i]);
      sync.tag[i] = gate_tag_.at(gates[i]);
      DLNB_REQUIRE(sync.tag[i] != 0, "run_gated: gate " << gates[i] << " was never signalled");
    }
    if (fixed_) {
      fixed_task(s, us, flops, start, sync, done);
      ++gated_;
      return;
    }
    note_task(s, us * scale_);
    if (stall_timers_ && !start) start = stall_timers_->task_slot(s);
    StartNote note{stall_timers_, s, start, ticks(us * scale_), nullptr};
    sync.tstart[0] = start;
    sync.tstart[1] = extra_start_;
    extra_start_ = nullptr;
    const bool chained = chain && chain_live_[slot_for(s)];
    deadline_task(s, us * scale_, sync, chained, done);
    if (chained) ++chained_;
    ++gated_;
  }

  void set_next_start_slot(uint64_t* slot) override { extra_start_ = slot; }

  // Launch the open program's tasks so far (it stays open for the tasks after).
  void flush_program(Stream& s) {
    auto it = programs_.find(&s);
    if (it == programs_.end()) return;
    // folded waits not taken by a task yet: the launch ends with them (a
    // kernel of its own follows it on the stream)
    if (it->second.open) emit_pending(s, it->second, nullptr, 0);
    if (it->second.tasks.empty()) return;
    it->second.done_free = false;
    std::vector<kernels::DlTask>& ts = it->second.tasks;
    // A program whose first task waits for gates (FSDP: the iteration's first
    // all-gather) is launched only once they are up, behind one-wave gate
    // waits: resident and waiting, its grid would hold the CUs that
    // collective needs (round 5: the headline's first all-gather ran on the 32
    // free CUs, 0.74 instead of 0.19 ms). Its first block then finds them up.
    for (int i = 0; i < 2; ++i)
      if (ts[0].sync.gate[i])
        kernels::gate_wait(ts[0].sync.gate[i], dev_.iter_word(), ts[0].sync.tag[i], gate_timeout_ticks_,
                           counters_.as<uint64_t>() + kernels::kWaitTimeouts, s.native(), dev_.abort_word());
    const kernels::DlTask* dst = place_tasks(s, ts);
    kernels::gemm_tn_deadline_program(A_.data(), B_.data(), C_.data(), kMmax, N_, K_, dtype_, dst,
                                      static_cast<int>(ts.size()), slot_for(s), grid_, s.native(), 0u);
    ++programs_launched_;
    ++program_count_[&s];
    program_tasks_ += static_cast<long>(ts.size());
    ts.clear();
  }

  void run_stamped(Stream& s, double us, double flops, uint64_t* start) override {
    if (fixed_) {
      fixed_task(s, us, flops, start, {}, nullptr);
      return;
    }
    note_task(s, us * scale_);
    if (stall_timers_ && !start) start = stall_timers_->task_slot(s);
    StartNote note{stall_timers_, s, start, ticks(std::max(0.0, us * scale_)), nullptr};
    double d = us * scale_;
    // a task that is not a deadline kernel cannot join the open program
    if (mode_ == ComputeMode::Gemm && d < 20.0) {
      auto pit = programs_.find(&s);
      if (pit != programs_.end() && pit->second.open) pit->second.split = true;
      flush_program(s);
    }
    if (mode_ == ComputeMode::Gemm) chain_live_[slot_for(s)] = false;  // a chain restarts at every unchained task
    if (mode_ == ComputeMode::Sleep || mode_ == ComputeMode::Spin) {
      // the kernel stamps its own start (stall timers: gap() from it)
      uint64_t* extra = extra_start_;
      extra_start_ = nullptr;
      if (d <= 0) {
        if (start) dev_.stamp(s, start);
        if (extra) dev_.stamp(s, extra);
      } else if (mode_ == ComputeMode::Sleep) {
        kernels::idle_wait(ticks(d), s.native(), start, extra);
      } else {
        kernels::busy_spin(ticks(d), cus_, s.native(), start, extra);
      }
      return;
    }
    // Fixed duration, real MFMA work: persistent deadline GEMM (the stand-in
    // keeps the matrix cores and HBM busy for exactly the table's time, so
    // DVFS or contention changes how much work is done, not how long).
    if (d <= 0) {
      if (start) dev_.stamp(s, start);
      if (extra_start_) dev_.stamp(s, extra_start_);
      extra_start_ = nullptr;
      return;
    }
    if (d < 20.0) {
      kernels::busy_spin(ticks(d), cus_, s.native(), start, extra_start_);
      extra_start_ = nullptr;
      return;
    }
    kernels::DlSync sync;
    sync.tstart[0] = start;
    sync.tstart[1] = extra_start_;
    extra_start_ = nullptr;
    deadline_task(s, d, sync, false);
  }

  void set_task_timers(TimerSet* t) override {
    // every task's own start (and, fixed work, end) stamp feeds the stall
    // timers (TimerSet::stall_before_task) and the fixed-work task times
    // (compute_task_time / compute_task_table: compute_stretch)
    task_timers_ = fixed_ ? t : nullptr;
    if (t && env_int("DLNB_TASK_STAMP_TIMERS", 1) != 0) {
      stall_timers_ = t;
      t->set_task_stamps(true);
    } else if (fixed_) {
      stall_timers_ = t;  // fixed work needs its end slots even without the stall timers
    }
  }

  Json describe() const override {
    Json j = Json::object();
    j["mode"] = compute_mode_name(mode_);
    j["time_scale"] = scale_;
    j["wallclock_hz"] = hz();
    j["wallclock_hz_nominal"] = kernels::wallclock_hz_nominal(dev_.index());
    j["wallclock_uncertainty_ppm"] = kernels::wallclock_uncertainty_ppm(dev_.index());
    j["num_cus"] = cus_;
    if (mode_ == ComputeMode::Gemm || fixed_) {
      j["deadline_grid"] = grid_;
      j["comm_reserved_cus"] = cus_ - grid_;
      j["deadline_slice_us"] = slice_us_;
      j["chained_tasks"] = chained_;  // enqueued so far (a captured graph counts its one iteration)
      j["chain_absorb_us"] = absorb_ticks_ / hz() * 1e6;  // most lateness a chained / gated task absorbs
      j["gated_tasks"] = gated_;      // tasks that waited on device gates instead of stream events
      // compute programs enqueued so far (one persistent kernel each) and their tasks
      j["programs"] = programs_launched_;
      j["program_tasks"] = program_tasks_;
    }
    if (A_.data()) {
      j["gemm_dtype"] = dtype_name(dtype_);
      j["gemm_N"] = N_;
      j["gemm_K"] = K_;
    }
    if (fixed_) {
      // the fixed-work unit: one full-K round of 256 x 256 tiles over the grid
      // and one K-tile of a tail tile, measured alone at start-up
      Json f = Json::object();
      f["round_us"] = cal_.round_us;
      f["ktile_us"] = cal_.ktile_us;
      f["grid"] = grid_;
      f["ktiles_per_tile"] = nk_;
      f["tflops"] = round_flops() / (cal_.round_us * 1e-6) / 1e12;
      f["tasks"] = fixed_tasks_;
      f["calibration"] = cal_given_ ? "DLNB_FIXED_WORK_CAL" : "measured";
      j["fixed_work"] = f;
    }
    return j;
  }
  ComputeMode mode() const override { return mode_; }

 private:
  uint64_t ticks(double us) const { return static_cast<uint64_t>(us * 1e-6 * hz() + 0.5); }
  double hz() const {
    if (hz_ <= 0.0) hz_ = kernels::wallclock_hz(dev_.index());
    return hz_;
  }

  // Where a task list goes: captured into a graph, the device ring (written
  // by after_capture, before the first replay); launched at once, the
  // host-mapped ring (the kernel reads it where the host wrote it).
  const kernels::DlTask* place_tasks(Stream& s, const std::vector<kernels::DlTask>& ts) {
    const size_t n = ts.size();
    DLNB_REQUIRE(n <= kProgTasks, "compute program of " << n << " tasks exceeds the ring (" << kProgTasks << ")");
    if (dev_.capturing(s)) {
      if (prog_next_ + n > kProgTasks) prog_next_ = 0;  // (a program runs before the ring comes round again)
      kernels::DlTask* dst = prog_dev_.as<kernels::DlTask>() + prog_next_;
      prog_next_ += n;
      uploads_.push_back(Upload{dst, ts});
      return dst;
    }
    // (16384 entries: an iteration's launches - the host synchronises with
    // every iteration - never come round to a list still being read)
    if (host_next_ + n > kProgTasks) host_next_ = 0;
    kernels::DlTask* dst = prog_host_ + host_next_;
    host_next_ += n;
    std::copy(ts.begin(), ts.end(), dst);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    return dst;
  }

  // One deadline task of d us on s (every slice launch carries the same
  // epoch; the kernels agree its start through the stream's slot line,
  // csrc/kernels/deadline_sync.hpp). chain: start at the stream's previous
  // deadline (or the latest gate) instead of when the first block arrives.
  // done (optional): recorded when the task is over - with gate events its
  // gate is raised by the task's own kernel (DlSync::done_gate, last launch).
  void deadline_task(Stream& s, double d, kernels::DlSync sync, bool chain, Event* done = nullptr) {
    uint64_t* slot = slot_for(s);
    sync.chain = chain ? absorb_ticks_ : 0u;
    sync.counters = counters_.as<uint64_t>();
    sync.iter = dev_.iter_word();
    sync.gate_timeout = gate_timeout_ticks_;
    sync.abort = dev_.abort_word();
    uint64_t* dgate = nullptr;
    uint32_t dtag = 0;
    const bool folded = done && dev_.arm_gate_record(*done, s, &dgate, &dtag);
    const uint64_t total = ticks(d);
    auto pit = programs_.find(&s);
    if (pit != programs_.end() && pit->second.open) {
      // a task of the open program: launched with it (end_program)
      DLNB_REQUIRE(folded || !done, "a program task's done event needs gate events");
      kernels::DlTask t;
      t.sync = sync;
      t.sync.done_gate = dgate;
      t.sync.done_tag = dtag;
      t.ticks = total;
      take_pending(s, pit->second, t.sync);
      DLNB_REQUIRE(pit->second.index < 4096, "more than 4096 program tasks per iteration on one stream");
      t.epoch = pit->second.index++;  // the kernel derives the epoch from it and the iteration word
      pit->second.tasks.push_back(t);
      pit->second.done_free = t.sync.done_gate == nullptr;
      chain_live_[slot] = true;
      return;
    }
    const uint32_t ep = next_epoch(slot);
    const uint64_t slice = slice_us_ > 0 ? std::max<uint64_t>(ticks(slice_us_), 1) : total;
    for (uint64_t end = slice;; end += slice) {
      kernels::DlSync ls = end == slice ? sync : kernels::DlSync();
      ls.abort = sync.abort;
      if (end >= total && folded) {
        ls.done_gate = dgate;
        ls.done_tag = dtag;
        ls.iter = sync.iter;
      }
      kernels::gemm_tn_deadline(A_.data(), B_.data(), C_.data(), kMmax, N_, K_, dtype_, total, slot, ep, grid_,
                                s.native(), std::min(end, total), ls);
      if (end >= total) break;
    }
    if (done && !folded) s.record(*done);
    chain_live_[slot] = true;
  }

  // A launch epoch of its own: 32768..65534 (never 0: a fresh slot reads as
  // epoch 0); program tasks take 1..32767 from the iteration word.
  uint32_t next_epoch(uint64_t* slot) {
    uint32_t& ep0 = epoch_[slot];
    ep0 = ep0 % 32767 + 1;
    return 32767 + ep0;
  }

  // ---- fixed work (gemm-work, flops): program tasks of a given amount of
  // MFMA work that stamp their own start and end (no stamp kernels).
  double round_flops() const { return static_cast<double>(grid_) * 2.0 * kTile * kTile * K_; }
  FixedWork size_work(double us, double flops) const {
    FixedWork w;
    double units;  // in full-K rounds
    if (mode_ == ComputeMode::Flops)
      units = std::max(0.0, flops * scale_) / round_flops();
    else
      units = std::max(0.0, us * scale_) / cal_.round_us;
    w.rounds = static_cast<uint32_t>(std::floor(units));
    // the rest as a tail tile of an even K-tile count (the kernels' pairing)
    const double kt = (units - w.rounds) * nk_;
    uint32_t tail = static_cast<uint32_t>(std::lround(kt / tail_mul_)) * tail_mul_;
    if (tail >= static_cast<uint32_t>(nk_)) {
      ++w.rounds;
      tail = 0;
    }
    w.tail_kt = tail;
    if (w.rounds == 0 && w.tail_kt == 0 && units > 0) w.tail_kt = tail_mul_;
    w.us = w.rounds * cal_.round_us + w.tail_kt * cal_.ktile_us;
    return w;
  }

  void fixed_task(Stream& s, double us, double flops, uint64_t* start, kernels::DlSync sync, Event* done) {
    const FixedWork w = size_work(us, flops);
    note_task(s, w.us);
    if (stall_timers_ && !start) start = stall_timers_->slot();
    uint64_t* end = stall_timers_ ? stall_timers_->slot() : nullptr;
    sync.tstart[0] = start;
    sync.tstart[1] = extra_start_;
    extra_start_ = nullptr;
    sync.counters = counters_.as<uint64_t>();
    sync.iter = dev_.iter_word();
    sync.gate_timeout = gate_timeout_ticks_;
    sync.abort = dev_.abort_word();
    uint64_t* dgate = nullptr;
    uint32_t dtag = 0;
    const bool folded = done && dev_.arm_gate_record(*done, s, &dgate, &dtag);
    sync.done_gate = dgate;
    sync.done_tag = dtag;
    kernels::DlTask t;
    t.sync = sync;
    t.ticks = 0;
    t.work_rounds = w.rounds;
    t.tail_kt = w.tail_kt;
    t.tend = end;
    auto pit = programs_.find(&s);
    if (pit != programs_.end() && pit->second.open) {
      DLNB_REQUIRE(folded || !done, "a program task's done event needs gate events");
      take_pending(s, pit->second, t.sync);
      DLNB_REQUIRE(pit->second.index < 4096, "more than 4096 program tasks per iteration on one stream");
      t.epoch = pit->second.index++;
      pit->second.tasks.push_back(t);
      pit->second.done_free = t.sync.done_gate == nullptr;
    } else {
      // a launch of its own (a one-task program with an epoch of its own):
      // the gates' one-wave waits first, as for a program's first task
      for (int i = 0; i < 2; ++i)
        if (t.sync.gate[i])
          kernels::gate_wait(t.sync.gate[i], dev_.iter_word(), t.sync.tag[i], gate_timeout_ticks_,
                             counters_.as<uint64_t>() + kernels::kWaitTimeouts, s.native(), dev_.abort_word());
      uint64_t* slot = slot_for(s);
      const kernels::DlTask* dst = place_tasks(s, {t});
      kernels::gemm_tn_deadline_program(A_.data(), B_.data(), C_.data(), kMmax, N_, K_, dtype_, dst, 1, slot, grid_,
                                        s.native(), next_epoch(slot));
      if (done && !folded) s.record(*done);
    }
    ++fixed_tasks_;
    if (end) last_end_[&s] = end;
    if (stall_timers_) stall_timers_->task_started(s, start, 0, end);
    if (task_timers_ && start && end) {
      task_timers_->pair(start, end, "compute_task_time");
      task_timers_->add("compute_task_table", (mode_ == ComputeMode::Flops ? w.us : us * scale_) * 1e-6);
    }
  }

  uint64_t* slot_for(Stream& s) {
    auto it = slot_of_.find(&s);
    size_t idx;
    if (it == slot_of_.end()) {
      idx = slot_of_.size();
      DLNB_REQUIRE(idx < kSlots, "too many compute streams");
      slot_of_[&s] = idx;
    } else {
      idx = it->second;
    }
    return slots_.as<uint64_t>() + idx * 8;  // one 64-B line per stream
  }

  void alloc_operands() {
    const int Mmax = kMmax;
    const size_t esz = dtype_size(dtype_);
    A_ = dev_.alloc(static_cast<size_t>(Mmax) * K_ * esz);
    B_ = dev_.alloc(static_cast<size_t>(N_) * K_ * esz);
    C_ = dev_.alloc(static_cast<size_t>(Mmax) * N_ * 2);
    auto s = dev_.create_stream(false);
    dev_.fill_random(A_.data(), static_cast<size_t>(Mmax) * K_, dtype_, 1, *s);
    dev_.fill_random(B_.data(), static_cast<size_t>(N_) * K_, dtype_, 2, *s);
    s->synchronize();
  }

  // Fixed work's unit costs with nothing else running: one-task programs of
  // R full-K rounds (R = 20 and 60: the difference removes the launch and
  // the first tile's ramp) and of a tail of nk / 2 K-tiles after one round.
  void calibrate() {
    nk_ = kernels::program_ktiles(kMmax, N_, K_, dtype_);
    tail_mul_ = static_cast<uint32_t>(std::max(1, kernels::program_tail_multiple(kMmax, N_, K_, dtype_)));
    // DLNB_FIXED_WORK_CAL="round_us:ktile_us" reuses an earlier calibration
    // (the report's compute.fixed_work) instead of measuring: a fixed-work run
    // beside other jobs (tools/interference.py) must do the work it would do
    // alone, not what a contended calibration says fits the table time.
    const std::string given = env_or("DLNB_FIXED_WORK_CAL", "");
    if (!given.empty()) {
      const auto kv = split(trim(given), ':');
      DLNB_REQUIRE(kv.size() == 2, "DLNB_FIXED_WORK_CAL: expected round_us:ktile_us, got '" << given << "'");
      cal_.round_us = std::stod(kv[0]);
      cal_.ktile_us = std::stod(kv[1]);
      DLNB_REQUIRE(cal_.round_us > 0 && cal_.ktile_us > 0, "DLNB_FIXED_WORK_CAL: bad values '" << given << "'");
      cal_given_ = true;
      return;
    }
    auto s = dev_.create_stream(false);
    auto e0 = dev_.create_event(true);
    auto e1 = dev_.create_event(true);
    uint64_t* slot = slot_for(*s);
    auto time_task = [&](uint32_t rounds, uint32_t tail) {
      kernels::DlTask t;
      t.sync.counters = counters_.as<uint64_t>();
      t.sync.abort = dev_.abort_word();
      t.work_rounds = rounds;
      t.tail_kt = tail;
      const kernels::DlTask* dst = place_tasks(*s, {t});
      s->record(*e0);
      kernels::gemm_tn_deadline_program(A_.data(), B_.data(), C_.data(), kMmax, N_, K_, dtype_, dst, 1, slot, grid_,
                                        s->native(), next_epoch(slot));
      s->record(*e1);
      s->synchronize();
      return dev_.elapsed_ms(*e0, *e1) * 1e3;
    };
    // ~0.3 s first so the measurement sees the sustained (DVFS-settled) clock
    // rather than the cold-start boost
    const double probe = std::max(1.0, time_task(8, 0) / 8.0);
    const uint32_t warm = static_cast<uint32_t>(std::min(4000.0, std::max(20.0, 300000.0 / probe)));
    (void)time_task(warm, 0);
    auto best = [&](uint32_t r, uint32_t tail) {
      double b = 1e30;
      for (int i = 0; i < 3; ++i) b = std::min(b, time_task(r, tail));
      return b;
    };
    const uint32_t r1 = 20, r2 = 60;
    const double t1 = best(r1, 0), t2 = best(r2, 0);
    cal_.round_us = std::max(1e-3, (t2 - t1) / (r2 - r1));
    const uint32_t tail = std::max<uint32_t>(tail_mul_, static_cast<uint32_t>(nk_ / 2) / tail_mul_ * tail_mul_);
    const double tt = best(r1, tail);
    cal_.ktile_us = std::max(1e-4, (tt - t1) / tail);
    // the slot's epoch / completion state is this stream's: the line is reset for the strategy's streams
    dev_.memset_async(slot, 0, 64, *s);
    s->synchronize();
    slot_of_.clear();
    epoch_.clear();
  }

  static constexpr int kMmax = 8192;
  static constexpr int kTile = 256;
  static constexpr size_t kSlots = 64;
  Device& dev_;
  ComputeMode mode_;
  double scale_;
  bool fixed_ = false;
  Buffer slots_;
  Buffer counters_;  // kernels::DlCounter words (DlSync::counters)
  // programs: the open task list per stream, the device ring their task lists
  // live in, uploads deferred past a graph capture
  struct Fold : Device::StreamFold {
    GpuCompute* e = nullptr;
    Stream* s = nullptr;
    void fold_wait(const uint64_t* gate, uint32_t tag) override { e->fold_wait(*s, gate, tag); }
    void fold_record(Event& ev) override { e->fold_record(*s, ev); }
  };
  struct Program {
    bool open = false;
    uint32_t index = 0;  // program tasks of the iteration so far (DlTask::epoch)
    std::vector<kernels::DlTask> tasks;
    // folded gate-event waits (gate, tag) the next task takes as its gates
    std::vector<std::pair<const uint64_t*, uint32_t>> pending;
    bool done_free = false;  // tasks.back() has no done gate: a record right after it takes that one
    bool split = false;      // a short task was launched on its own while the program was open
    Fold fold;
  };

  // ---- gate events folded into the open program (Device::StreamFold)
  void fold_wait(Stream& s, const uint64_t* gate, uint32_t tag) {
    Program& p = programs_[&s];
    for (auto& w : p.pending)
      if (w.first == gate) {  // the same gate again: its latest record
        w.second = tag;
        return;
      }
    p.pending.emplace_back(gate, tag);
  }
  void fold_record(Stream& s, Event& ev) {
    Program& p = programs_[&s];
    uint64_t* g = nullptr;
    uint32_t tag = 0;
    DLNB_REQUIRE(dev_.arm_gate_record(ev, s, &g, &tag), "fold_record: not a gate event");
    if (p.pending.empty() && p.done_free && !p.tasks.empty()) {
      // recorded right after a task: that task's done gate
      p.tasks.back().sync.done_gate = g;
      p.tasks.back().sync.done_tag = tag;
      p.done_free = false;
      return;
    }
    emit_pending(s, p, g, tag);
    if (p.tasks.empty() || p.tasks.back().sync.done_gate != g) {
      // nothing pending and no task to carry it: a gate-only task raises it
      kernels::DlTask t = gate_task();
      t.sync.done_gate = g;
      t.sync.done_tag = tag;
      push_task(p, t);
    }
    p.done_free = false;
  }
  kernels::DlTask gate_task() const {
    kernels::DlTask t;
    t.sync.iter = dev_.iter_word();
    t.sync.counters = counters_.as<uint64_t>();
    t.sync.gate_timeout = gate_timeout_ticks_;
    t.sync.abort = dev_.abort_word();
    t.ticks = fixed_ ? 0 : 1;  // (deadline: the stream's chain goes on from when its gates opened)
    t.flags = kernels::kTaskGateOnly;
    return t;
  }
  void push_task(Program& p, const kernels::DlTask& t) {
    DLNB_REQUIRE(p.index < 4096, "more than 4096 program tasks per iteration on one stream");
    kernels::DlTask c = t;
    c.epoch = p.index++;
    p.tasks.push_back(c);
  }
  // The pending waits as gate-only tasks (two gates each); the last one
  // raises done_gate when given.
  void emit_pending(Stream& s, Program& p, uint64_t* done_gate, uint32_t done_tag) {
    (void)s;
    while (!p.pending.empty()) {
      kernels::DlTask t = gate_task();
      for (int i = 0; i < 2 && !p.pending.empty(); ++i) {
        t.sync.gate[i] = p.pending.front().first;
        t.sync.tag[i] = p.pending.front().second;
        p.pending.erase(p.pending.begin());
      }
      if (p.pending.empty() && done_gate) {
        t.sync.done_gate = done_gate;
        t.sync.done_tag = done_tag;
      }
      push_task(p, t);
      p.done_free = false;
    }
  }
  // A task about to join the program takes the pending waits as its gates
  // (those beyond its free gate slots go to gate-only tasks before it).
  void take_pending(Stream& s, Program& p, kernels::DlSync& sync) {
    if (p.pending.empty()) return;
    const size_t free_slots = (sync.gate[0] ? 0u : 1u) + (sync.gate[1] ? 0u : 1u);
    if (p.pending.size() > free_slots) {
      // keep the last free_slots for the task, the rest before it
      std::vector<std::pair<const uint64_t*, uint32_t>> keep(p.pending.end() - static_cast<long>(free_slots),
                                                             p.pending.end());
      p.pending.resize(p.pending.size() - free_slots);
      emit_pending(s, p, nullptr, 0);
      p.pending = keep;
    }
    for (int i = 0; i < 2 && !p.pending.empty(); ++i) {
      if (sync.gate[i]) continue;
      sync.gate[i] = p.pending.front().first;
      sync.tag[i] = p.pending.front().second;
      p.pending.erase(p.pending.begin());
    }
  }
  std::map<Stream*, Program> programs_;
  struct Join {
    std::vector<uint64_t*> gates;
    uint32_t tag;
    uint64_t* host_done;
  };
  std::map<Stream*, Join> joins_;  // set_lane_join, taken by the next end_program
  std::set<Stream*> joined_;
  std::map<Stream*, long> program_count_;  // programs launched per stream (programs_on)
  Buffer prog_dev_;
  size_t prog_next_ = 0;
  kernels::DlTask* prog_host_ = nullptr;  // host-mapped ring (task lists launched at once)
  size_t host_next_ = 0;
  struct Upload {
    kernels::DlTask* dst;
    std::vector<kernels::DlTask> tasks;
  };
  std::vector<Upload> uploads_;
  static constexpr size_t kProgTasks = 16384;
  long programs_launched_ = 0, program_tasks_ = 0, fixed_tasks_ = 0;
  std::vector<uint64_t*> gates_;          // device gates (Device::alloc_gate)
  std::map<Stream*, size_t> slot_of_;
  std::map<uint64_t*, uint32_t> epoch_;
  std::map<uint64_t*, bool> chain_live_;  // the stream's last task was a deadline task a chained one may continue
  std::map<Stream*, const uint64_t*> last_end_;  // fixed work: the end slot of the stream's last task
  std::vector<uint32_t> gate_tag_;        // last tag signalled per gate (never 0 once signalled)
  uint64_t* extra_start_ = nullptr;       // set_next_start_slot
  TimerSet* stall_timers_ = nullptr;      // set_task_timers: task starts for the stall timers
  // lane_task_us: the tasks enqueued per stream since the last set_lane_join
  struct LaneStats {
    long n = 0;
    double us = 0.0;
    bool single = true;  // every task one kernel
  };
  std::map<Stream*, LaneStats> lane_stats_;
  void note_task(Stream& s, double d) {
    LaneStats& st = lane_stats_[&s];
    ++st.n;
    st.us += std::max(0.0, d);
  }
  // Reports a task's start slot and duration to the stall timers once it is enqueued.
  struct StartNote {
    TimerSet* t;
    Stream& s;
    const uint64_t* start;
    uint64_t ticks;
    const uint64_t* end;
    ~StartNote() {
      if (t && std::uncaught_exceptions() == 0) t->task_started(s, start, ticks, end);
    }
  };
  // Lateness a chained task absorbs (deadline_sync.hpp): the replayed graph's
  // queue hop (8-11 us) + the previous grid's drain (~13 us) measured in
  // round 3; anything later is a wait and stays in the iteration time.
  // DLNB_CHAIN_ABSORB_US overrides.
  uint32_t absorb_ticks_ = 1;
  uint64_t gate_timeout_ticks_ = 0;  // a deadline task's gate wait bound (DLNB_GATE_TIMEOUT_S)
  long chained_ = 0;                      // tasks that continued a chain (describe())
  long gated_ = 0;
  int grid_ = 256;
  double slice_us_ = 500;
  mutable double hz_ = 0.0;  // hz()
  int cus_ = 256;
  DType dtype_ = DType::BF16;
  int K_ = 4096, N_ = 16384;
  int nk_ = 0;                 // K-tiles of a full tile (fixed work)
  uint32_t tail_mul_ = 2;      // the tail's K-tile multiple
  FixedCal cal_;
  bool cal_given_ = false;
  Buffer A_, B_, C_;
  TimerSet* task_timers_ = nullptr;
};

}  // namespace

std::unique_ptr<ComputeEngine> make_compute_engine(Device& dev, ComputeMode mode, const ComputeShape& shape,
                                                   double time_scale) {
  if (dev.kind() == DeviceKind::CPU) return std::unique_ptr<ComputeEngine>(new CpuCompute(dev, mode, time_scale));
  return std::unique_ptr<ComputeEngine>(new GpuCompute(dev, mode, shape, time_scale));
}

}  // namespace dlnb
