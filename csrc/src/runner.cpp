// Benchmark runner shared by all strategies: bootstrap, device/backend
// selection, warm-up, run-count estimation, timed runs, loop mode, report.
//
// Reference flow: main() of each driver (e.g. cpp/data_parallel/dp.cpp:127-303):
// parse args -> read stats -> MPI_Init -> topology print -> set device ->
// CCL init -> buffers -> barrier -> warm-up (MPI_Wtime) -> optional
// estimate_runs -> PROXY_LOOP or timed runs -> ccutils JSON section.
// Deviations: estimate_runs averages warm-ups over warm-ups (the reference
// divides a world-sum by the warm-up count, cpp/utils.hpp:127-128) and takes
// the max over ranks; loop mode is a run-time flag (or a *_loop argv[0]).
#include <algorithm>
#include <exception>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <mutex>
#include <sstream>
#include <thread>

#include <sys/prctl.h>

extern char** environ;

#include "dlnb/aux.hpp"
#include "dlnb/kernels.hpp"
#include "dlnb/strategy.hpp"
#include "dlnb/xgmi.hpp"

namespace dlnb {

namespace {
thread_local const uint64_t* t_done_flag = nullptr;
thread_local size_t t_done_n = 0;
thread_local uint64_t t_done_value = 0;

// The run on this thread, for device_failure (set by run_rank).
struct FailGuard {
  Device* dev = nullptr;
  std::vector<Communicator*>* comms = nullptr;
  bool cli_exit = false;  // CLI process owning its ranks: end the process at the first failure
  int rank = 0;
  bool fired = false;
};
thread_local FailGuard* t_fail = nullptr;
std::atomic<bool> g_poisoned{false};
}  // namespace

void device_failure(const std::string& why) {
  FailGuard* f = t_fail;
  if (!f || f->fired) return;
  f->fired = true;
  if (f->dev) f->dev->raise_abort();
  if (f->cli_exit && f->dev) {  // (GPU runs only: a CPU run's failure path is its own, unchanged)
    std::fprintf(stderr,
                 "[dlnb] rank %d error: %s\n[dlnb] rank %d: device waits aborted; exiting without teardown (the "
                 "driver reclaims the GPU queues)\n",
                 f->rank, why.c_str(), f->rank);
    std::fflush(stdout);
    std::fflush(stderr);
    std::_Exit(3);
  }
  if (f->comms)
    for (Communicator* c : *f->comms)
      if (c) c->abort();
}

bool process_poisoned() { return g_poisoned.load(); }

CompletionFlag::CompletionFlag(const uint64_t* flags, size_t n, uint64_t value)
    : prev_(t_done_flag), prev_n_(t_done_n), prev_value_(t_done_value) {
  t_done_flag = flags;
  t_done_n = n;
  t_done_value = value;
}
CompletionFlag::~CompletionFlag() {
  t_done_flag = prev_;
  t_done_n = prev_n_;
  t_done_value = prev_value_;
}

void sync_streams(const std::vector<Stream*>& streams, const std::vector<Communicator*>& comms, Device& dev) {
  (void)dev;
  // Poll period: with the default 50-us timer slack a 20-us sleep woke ~70 us
  // late, and every timed iteration ends inside this loop (the reference times
  // each iteration from the host); slack 1 us + 5-us sleeps bound the wake-up
  // latency to a few us for a fraction of one core.
  thread_local const bool slack_set = [] {  // (timer slack is per thread)
    prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
    return true;
  }();
  (void)slack_set;
  const double timeout = static_cast<double>(env_int("DLNB_TIMEOUT", 900));
  const double t0 = now_s();
  int polls = 0;
  const uint64_t* flag = t_done_flag;
  const size_t nflags = t_done_n;
  const uint64_t want = t_done_value;
  auto done = [&](Stream* s) {
    if (!flag) return s->query();
    for (size_t i = 0; i < nflags; ++i)
      if (__atomic_load_n(flag + i, __ATOMIC_ACQUIRE) < want) return false;
    return true;
  };
  for (Stream* s : streams) {
    while (!done(s)) {
      if (++polls % 64 == 0) {
        for (Communicator* c : comms) {
          if (!c) continue;
          std::string err = c->async_error();
          if (!err.empty()) {
            device_failure("communication failure: " + err);
            for (Communicator* a : comms)
              if (a) a->abort();
            DLNB_THROW("communication failure: " << err);
          }
        }
        if (now_s() - t0 > timeout) {
          std::ostringstream m;
          m << "iteration did not complete within DLNB_TIMEOUT=" << timeout << " s (hung collective or dead peer)";
          if (flag) {
            // lane graphs: which lanes' done words (host-mapped) are behind
            m << "; lane done words (want " << want << "):";
            for (size_t i = 0; i < nflags; ++i) m << " " << __atomic_load_n(flag + i, __ATOMIC_ACQUIRE);
          }
          device_failure(m.str());
          for (Communicator* a : comms)
            if (a) a->abort();
          DLNB_THROW(m.str());
        }
      }
      std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
  }
}

Json comm_stats_json(const std::vector<CommStat>& stats, const TimerSet& t) {
  Json out = Json::object();
  for (const auto& s : stats) {
    const auto& v = t.get(s.timer);
    Json e = Json::object();
    e["kind"] = s.name;
    e["nranks"] = s.nranks;
    e["bytes_per_op"] = s.bytes_per_op;
    e["ops"] = static_cast<long long>(v.size());
    double tot = 0;
    for (double x : v) tot += x;
    e["total_s"] = tot;
    // A 1-rank group moves nothing over a link: its "collective" is a local
    // device copy (or nothing), so it reports busbw 0 and says so.
    e["transport"] = s.nranks > 1 ? "link" : "local-copy";
    if (!v.empty() && tot > 0) {
      double algbw = s.bytes_per_op * v.size() / tot / 1e9;
      e["algbw_GBps"] = algbw;
      e["busbw_GBps"] = algbw * busbw_factor(s.kind, s.nranks);
    }
    out[s.name] = e;
  }
  return out;
}

void optimizer_step(Context& ctx, Stream& s, void* param, void* mom, const void* grad, size_t n, uint64_t* end_stamp,
                    uint32_t* done) {
  if (ctx.dev->kind() == DeviceKind::GPU) {
    kernels::sgd_momentum_bf16(param, mom, grad, n, 1e-4f, 0.9f, s.native(), end_stamp, done);
    return;
  }
  if (end_stamp) {
    // (the CPU device's stamp: when the stream reaches it, i.e. after the task below)
    ctx.dev->host_task(s, [param, mom, grad, n] {
      auto* p = static_cast<uint16_t*>(param);
      auto* m = static_cast<uint16_t*>(mom);
      auto* g = static_cast<const uint16_t*>(grad);
      for (size_t i = 0; i < n; ++i) {
        float mv = 0.9f * bf16_to_float(m[i]) + bf16_to_float(g[i]);
        m[i] = float_to_bf16(mv);
        p[i] = float_to_bf16(bf16_to_float(p[i]) - 1e-4f * mv);
      }
    });
    ctx.dev->stamp(s, end_stamp);
    return;
  }
  ctx.dev->host_task(s, [param, mom, grad, n] {
    auto* p = static_cast<uint16_t*>(param);
    auto* m = static_cast<uint16_t*>(mom);
    auto* g = static_cast<const uint16_t*>(grad);
    for (size_t i = 0; i < n; ++i) {
      float mv = 0.9f * bf16_to_float(m[i]) + bf16_to_float(g[i]);
      m[i] = float_to_bf16(mv);
      p[i] = float_to_bf16(bf16_to_float(p[i]) - 1e-4f * mv);
    }
  });
}

// ------------------------------------------------------------- topology

void print_topology(Context& ctx) {
  // Reference: cpp/netcommunicators.hpp:142-290 builds a switch/node tree
  // from SLURM_TOPOLOGY_ADDR (fake address when SLURM is absent, :154-157).
  // Here each rank also reports its GPU, and rank 0 prints the node's
  // xGMI link matrix.
  std::string addr = env_or("SLURM_TOPOLOGY_ADDR", "");
  if (addr.empty()) addr = "root." + ctx.boot->info.hostname;
  std::ostringstream me;
  me << addr << "|" << ctx.boot->info.hostname << "|" << ctx.dev->name() << "|" << ctx.dev->index();
  auto all = ctx.hg().allgather(me.str());
  if (ctx.rank() != 0) return;
  // path -> ranks
  std::map<std::string, std::vector<int>> leaves;
  std::map<std::string, std::string> dev_of;
  for (size_t r = 0; r < all.size(); ++r) {
    auto f = split(all[r], '|');
    leaves[f[0]].push_back(static_cast<int>(r));
    dev_of[f[0]] = f.size() > 2 ? f[2] : "?";
  }
  std::ostringstream os;
  os << "=== topology: " << all.size() << " ranks on " << leaves.size() << " node(s) ===\n";
  std::vector<std::string> prev;
  for (const auto& kv : leaves) {
    auto parts = split(kv.first, '.');
    size_t common = 0;
    while (common < prev.size() && common < parts.size() - 1 && prev[common] == parts[common]) ++common;
    for (size_t d = common; d < parts.size(); ++d) {
      os << std::string(2 * d, ' ') << (d ? "└─ " : "") << parts[d];
      if (d + 1 == parts.size()) {
        os << "  ranks [";
        for (size_t i = 0; i < kv.second.size(); ++i) os << (i ? "," : "") << kv.second[i];
        os << "]  " << dev_of[kv.first];
      }
      os << "\n";
    }
    prev = parts;
  }
  if (ctx.dev->kind() == DeviceKind::GPU) os << describe_gpu_links();
  std::cout << os.str() << std::flush;
}

namespace {

std::vector<int> parse_device_list(const std::string& s) {
  std::vector<int> v;
  if (s.empty()) return v;
  for (auto& p : split(s, ',')) {
    std::string t = trim(p);
    if (!t.empty()) v.push_back(std::stoi(t));
  }
  return v;
}

double percentile(std::vector<double> v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  double pos = q * (v.size() - 1);
  size_t lo = static_cast<size_t>(std::floor(pos)), hi = static_cast<size_t>(std::ceil(pos));
  return v[lo] + (v[hi] - v[lo]) * (pos - lo);
}

std::unique_ptr<Strategy> make_strategy(StrategyKind k) {
  switch (k) {
    case StrategyKind::DP: return make_dp();
    case StrategyKind::FSDP: return make_fsdp();
    case StrategyKind::HybridCP: return make_cp();
    default: return make_pipeline(k);
  }
}

bool file_exists(const std::string& p) {
  std::ifstream f(p);
  return static_cast<bool>(f);
}

}  // namespace

namespace {

// Wraps the backend's factory and logs every communicator it creates (name,
// members, the library's own rank count) into ctx.comm_log for the report.
class RecordingFactory : public CommFactory {
 public:
  RecordingFactory(std::unique_ptr<CommFactory> inner, std::vector<CommRecord>* log, std::vector<Communicator*>* live)
      : inner_(std::move(inner)), log_(log), live_(live) {}
  std::string backend_name() const override { return inner_->backend_name(); }
  std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members,
                                       size_t capacity_bytes, bool need_p2p, int max_ctas) override {
    auto c = inner_->create(name, members, capacity_bytes, need_p2p, max_ctas);
    log_->push_back({name, c->backend_name(), c->size(), c->library_nranks()});
    return c;
  }
  void add_live(Communicator* c) { live_->push_back(c); }

 private:
  std::unique_ptr<CommFactory> inner_;
  std::vector<CommRecord>* log_;
  std::vector<Communicator*>* live_;
};

// The outermost communicator wrapper (tracing, when --timeline wraps the
// factory afterwards) is what the strategy holds; it reports itself here.
class LiveFactory : public CommFactory {
 public:
  LiveFactory(std::unique_ptr<CommFactory> inner, std::vector<Communicator*>* live)
      : inner_(std::move(inner)), live_(live) {}
  std::string backend_name() const override { return inner_->backend_name(); }
  std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members,
                                       size_t capacity_bytes, bool need_p2p, int max_ctas) override {
    auto c = inner_->create(name, members, capacity_bytes, need_p2p, max_ctas);
    live_->push_back(c.get());
    return c;
  }

 private:
  std::unique_ptr<CommFactory> inner_;
  std::vector<Communicator*>* live_;
};

}  // namespace

Json comm_log_json(const std::vector<CommRecord>& log) {
  Json out = Json::object();
  Json all = Json::array();
  Json rccl = Json::object();
  for (const auto& r : log) {
    Json e = Json::object();
    e["name"] = r.name;
    e["backend"] = r.backend;
    e["nranks"] = r.nranks;
    e["library_nranks"] = r.library_nranks;
    all.push_back(e);
    if (r.library_nranks >= 0) rccl[r.name] = r.library_nranks;
  }
  out["communicators"] = all;
  out["rccl_nranks"] = rccl;
  return out;
}

int collective_lanes(const Options& o, int world) {
  switch (o.strategy) {
    case StrategyKind::DP: return 1;
    case StrategyKind::FSDP: {
      const int F = std::max(1, o.sharding_factor);
      const bool replicas = world / F > 1;
      return o.comm_lanes == "split" ? 2 + (replicas ? 1 : 0) : 1;
    }
    case StrategyKind::HybridCP: return 2;
    default: return o.num_stages > 1 ? 3 : 1;
  }
}

std::string select_backend(Context& ctx, const std::string& requested, const std::string& devices) {
  const RankInfo& ri = ctx.boot->info;
  std::string backend = requested;
  const bool in_process = backend == "loopback" || backend == "loopback-cpu";
  const int ngpu = in_process ? 0 : gpu_device_count();
  if (backend == "auto") backend = ngpu > 0 ? "rccl" : "cpu";
  if (backend == "rccl" || backend == "xgmi" || backend == "mixed") {
    DLNB_REQUIRE(ngpu > 0, "--backend " << backend << " requested but no GPU is visible");
    std::vector<int> list = parse_device_list(devices);
    if (list.empty())
      for (int i = 0; i < ngpu; ++i) list.push_back(i);
    DLNB_REQUIRE(ri.local_rank < static_cast<int>(list.size()),
                 "local rank " << ri.local_rank << " has no device (device list has " << list.size() << ")");
    int dev_index = list[static_cast<size_t>(ri.local_rank)];
    DLNB_REQUIRE(dev_index >= 0 && dev_index < ngpu, "device id " << dev_index << " out of range");
    ctx.ranks_on_device = 0;
    for (int r = 0; r < ri.local_size && r < static_cast<int>(list.size()); ++r)
      ctx.ranks_on_device += list[static_cast<size_t>(r)] == dev_index;
    ctx.dev = make_gpu_device(dev_index);
    ctx.comms = backend == "rccl"    ? make_rccl_factory(ctx.hg(), *ctx.dev)
                : backend == "xgmi" ? make_xgmi_factory(ctx.hg(), *ctx.dev)
                                    : make_mixed_factory(ctx.hg(), *ctx.dev);
  } else if (backend == "cpu") {
    ctx.dev = make_cpu_device();
    ctx.comms = make_shm_factory(ctx.hg(), *ctx.dev);
  } else if (backend == "loopback" || backend == "loopback-cpu") {
    DLNB_REQUIRE(ctx.boot->hub, "--backend " << backend << " runs inside one process (run_benchmark starts the rank threads)");
    if (backend == "loopback-cpu") {
      // CPU device only: no HIP call at all (GPU-less hosts and CPU tests)
      ctx.dev = make_cpu_device(loopback_cpu_abort_flag(*ctx.boot->hub));
      ctx.ranks_on_device = ri.world_size;
    } else {
      // Every rank on the same GPU: the one given by -d (default 0).
      const int ngpu = gpu_device_count();
      DLNB_REQUIRE(ngpu > 0, "--backend loopback needs a GPU (loopback-cpu runs the ranks on the CPU device)");
      std::vector<int> list = parse_device_list(devices);
      const int dev_index = list.empty() ? 0 : list[0];
      for (int d : list)
        DLNB_REQUIRE(d == dev_index, "--backend loopback puts every rank on one device (-d " << devices << ")");
      DLNB_REQUIRE(dev_index >= 0 && dev_index < ngpu, "device id " << dev_index << " out of range");
      ctx.dev = make_gpu_device(dev_index);
      ctx.ranks_on_device = ri.world_size;
    }
    ctx.comms = make_loopback_factory(ctx.hg(), *ctx.dev, ctx.boot->hub);
  } else {
    DLNB_THROW("unknown backend '" << backend << "' (auto, rccl, xgmi, mixed, cpu, loopback, loopback-cpu)");
  }
  ctx.comms = wrap_comm_faults(std::move(ctx.comms), *ctx.dev, ri.rank);
  ctx.comms.reset(new RecordingFactory(std::move(ctx.comms), &ctx.comm_log, &ctx.live_comms));
  return backend;
}

namespace {

Json run_rank(const Options& opt, std::unique_ptr<Bootstrap> boot);

// Set by main_for: this process is a CLI binary, not a library host (Python).
std::atomic<bool> g_cli_process{false};

// State of one loopback job, shared by its rank threads (heap-held so a rank
// thread that outlives run_loopback - detached after a failure - never
// touches a dead stack frame).
struct LoopbackJob {
  Options opt;
  std::shared_ptr<LocalStore> store;
  std::shared_ptr<LoopbackHub> hub;
  std::vector<Json> docs;
  std::mutex mu;
  std::condition_variable done_cv;
  int done = 0;
  std::string first_error;
};

// --backend loopback / loopback-cpu: the job's ranks are threads of this process sharing one
// LocalStore (host barriers / gathers) and one LoopbackHub (collectives). A
// failing rank aborts both (and the job's CPU abort switch), so the others
// leave their waits instead of hanging; the first failure is rethrown.
// Rank threads of loopback jobs still running. A job whose rank threads did
// not drain after a failure detaches them (below); they keep GPU streams and
// buffers until they finally leave their waits, so this process refuses new
// loopback jobs until then (they would share the GPU with the
// next job and may still run at interpreter exit).
std::atomic<int> g_loopback_threads{0};

Json run_loopback(const Options& opt) {
  const int n = opt.ranks;
  DLNB_REQUIRE(n >= 1, "--ranks must be >= 1");
  const int live = g_loopback_threads.load();
  DLNB_REQUIRE(live == 0, "a previous loopback job of this process still has " << live
                              << " rank threads blocked (detached after its failure); run the next job in a new process");
  DLNB_REQUIRE(env_int("WORLD_SIZE", 1) == 1 && env_int("DLNB_WORLD_SIZE", 1) == 1,
               "--backend loopback runs all ranks inside one process: launch it once, not under a multi-rank launcher");
  auto job = std::make_shared<LoopbackJob>();
  job->opt = opt;
  job->store = std::make_shared<LocalStore>();
  job->hub = make_loopback_hub(n, static_cast<double>(env_int("DLNB_STORE_TIMEOUT", 900)));
  job->docs.resize(static_cast<size_t>(n));
  std::vector<std::thread> threads;
  for (int r = 0; r < n; ++r) {
    g_loopback_threads.fetch_add(1);
    threads.emplace_back([job, r, n] {
      try {
        Json d = run_rank(job->opt, bootstrap_loopback(r, n, job->store, job->hub));
        loopback_drained(*job->hub, false, 0);
        std::lock_guard<std::mutex> g(job->mu);
        job->docs[static_cast<size_t>(r)] = std::move(d);
      } catch (const std::exception& e) {
        const std::string msg = "rank " + std::to_string(r) + ": " + e.what();
        {
          std::lock_guard<std::mutex> g(job->mu);
          if (job->first_error.empty()) job->first_error = msg;
        }
        loopback_abort(*job->hub, msg);
        job->store->abort(msg);
      }
      g_loopback_threads.fetch_sub(1);
      std::lock_guard<std::mutex> g(job->mu);
      ++job->done;
      job->done_cv.notify_all();
    });
  }
  // After the first failure the other rank threads get a bounded grace
  // period to leave their waits and tear down. A thread still blocked then
  // must not hold the job forever: the CLI process ends with the rank's
  // error (as a multi-process job would); a library host (Python) gets the
  // error as an exception, with the stuck threads detached (they only hold
  // the job's heap state).
  const double grace_s = static_cast<double>(env_int("DLNB_LOOPBACK_ABORT_GRACE_S", 10));
  std::unique_lock<std::mutex> g(job->mu);
  job->done_cv.wait(g, [&] { return job->done == n || !job->first_error.empty(); });
  if (job->done < n &&
      !job->done_cv.wait_for(g, std::chrono::duration<double>(grace_s), [&] { return job->done == n; })) {
    const int stuck = n - job->done;
    const std::string err = job->first_error;
    g.unlock();
    std::fprintf(stderr, "[dlnb] error: %s\n[dlnb] %d of %d rank threads still blocked %.0f s after the failure\n",
                 err.c_str(), stuck, n, grace_s);
    std::fflush(stderr);
    if (g_cli_process.load()) std::_Exit(2);
    for (auto& t : threads) t.detach();
    throw Error(err + " (" + std::to_string(stuck) +
                " rank threads still blocked were detached; this process runs no further loopback job until they "
                "exit)");
  }
  g.unlock();
  for (auto& t : threads) t.join();
  if (!job->first_error.empty()) throw Error(job->first_error);
  return job->docs[0];
}

}  // namespace

bool cli_process() { return g_cli_process.load(); }

Json run_benchmark(const Options& opt) {
  DLNB_REQUIRE(!process_poisoned(),
               "an earlier run of this process failed and left device work that did not drain: start a new process");
  if (opt.backend == "loopback" || opt.backend == "loopback-cpu") return run_loopback(opt);
  return run_rank(opt, bootstrap_from_env(opt.store_addr));
}

namespace {

Json run_rank_impl(const Options& opt, Context& ctx, std::unique_ptr<Strategy>& strat);

Json run_rank(const Options& opt, std::unique_ptr<Bootstrap> boot) {
  // ctx and the strategy outlive the try block: a failing loopback rank
  // aborts the hub (waking its peers' waits) BEFORE its streams are torn
  // down - their destructors drain queued work that may wait on those peers.
  Context ctx;
  ctx.opt = opt;
  ctx.boot = std::move(boot);
  std::unique_ptr<Strategy> strat;
  FailGuard guard;
  guard.comms = &ctx.live_comms;
  guard.rank = ctx.boot->info.rank;
  guard.cli_exit = g_cli_process.load() && !ctx.boot->hub && env_int("DLNB_FAIL_EXIT", 1) != 0;
  struct GuardScope {
    FailGuard* prev;
    explicit GuardScope(FailGuard* g) : prev(t_fail) { t_fail = g; }
    ~GuardScope() { t_fail = prev; }
  } scope(&guard);
  try {
    Json r = run_rank_impl(opt, ctx, strat);
    t_fail = scope.prev;  // the run is over: strategy teardown is not a failure of it
    return r;
  } catch (const std::exception& e) {
    // The strategy is destroyed before the device (ctx outlives strat): its
    // events, buffers and communicators must not go while a stream task still
    // uses them (a CPU stream waiting on a freed event never returned - seen
    // after a peer died mid-iteration, library host).
    if (ctx.dev && ctx.dev->kind() == DeviceKind::GPU && !ctx.boot->hub) {
      // GPU: abort the device waits (CLI: the process ends here), abort the
      // communicators, then wait - bounded - for the device to drain; work
      // that does not drain keeps everything it may use (nothing is freed) and
      // this process runs nothing more.
      guard.dev = ctx.dev.get();
      device_failure(e.what());
      if (!ctx.dev->abort_and_drain()) {
        g_poisoned.store(true);
        const std::string msg = std::string(e.what()) +
                                " (device work did not drain within DLNB_ABORT_DRAIN_S after the abort: this process "
                                "runs no further benchmark)";
        (void)strat.release();
        (void)ctx.timeline.release();
        (void)ctx.compute.release();
        (void)ctx.comms.release();
        (void)ctx.dev.release();
        throw Error(msg);
      }
    } else if (ctx.dev && !ctx.boot->hub) {
      ctx.dev->abort_and_drain();
    }
    if (ctx.boot->hub) {
      const std::string msg = "rank " + std::to_string(ctx.boot->info.rank) + ": " + e.what();
      loopback_abort(*ctx.boot->hub, msg);
      if (auto* ls = dynamic_cast<LocalStore*>(ctx.boot->store.get())) ls->abort(msg);
      // The other ranks' streams may still hold copies into this rank's
      // buffers or waits on its events: drain this rank's work, then free
      // nothing (ctx / strat destructors) until every rank has drained too.
      try {
        if (ctx.dev) ctx.dev->synchronize();
      } catch (const std::exception&) {
      }
      loopback_drained(*ctx.boot->hub, true, static_cast<double>(env_int("DLNB_LOOPBACK_ABORT_GRACE_S", 10)));
    }
    throw;
  }
}

Json run_rank_impl(const Options& opt, Context& ctx, std::unique_ptr<Strategy>& strat) {
  const RankInfo& ri = ctx.boot->info;

  // ---- backend / device (cpp/utils.hpp:62-117 set_local_device)
  const std::string backend = select_backend(ctx, opt.backend, opt.devices);
  if (t_fail && ctx.dev->kind() == DeviceKind::GPU && !ctx.boot->hub) t_fail->dev = ctx.dev.get();

  // ---- workload
  std::string stats_path = opt.stats_file.empty() ? stats_path_for(opt.base_path, opt.model) : opt.stats_file;
  ctx.stats = parse_model_stats(stats_path);
  if (!opt.base_path.empty()) {
    std::string ap;
    try {
      ap = arch_path_for(opt.base_path, opt.model);
    } catch (const Error&) {
    }
    if (!ap.empty() && file_exists(ap)) {
      ctx.arch = parse_model_arch(ap);
      ctx.have_arch = true;
    }
  }
  ctx.wire = parse_dtype(opt.wire_dtype);
  ComputeShape shape;
  shape.hidden = static_cast<int>(ctx.stats.embedded_dim);
  uint64_t ffn = ctx.stats.ffn_dim ? ctx.stats.ffn_dim : (ctx.have_arch && ctx.arch.ff_dim ? ctx.arch.ff_dim : 4 * ctx.stats.embedded_dim);
  shape.ffn = static_cast<int>(ffn);
  std::string cdt = opt.compute_dtype;
  if (cdt == "auto") cdt = ctx.stats.dtype.find("8") != std::string::npos ? "fp8" : "bf16";
  shape.dtype = parse_dtype(cdt);
  shape.comm_cus = opt.comm_cus;
  shape.ranks_on_device = std::max(1, ctx.ranks_on_device);
  ComputeMode mode = parse_compute_mode(opt.compute, ctx.dev->kind());
  ctx.compute = make_compute_engine(*ctx.dev, mode, shape, opt.time_scale);
  if (!opt.timeline_path.empty()) {
    // every communicator the strategy creates and every compute task it
    // enqueues is traced (dlnb/timeline.hpp)
    ctx.timeline = std::make_unique<Timeline>(*ctx.dev);
    ctx.comms = make_tracing_factory(std::move(ctx.comms), ctx.timeline.get());
    ctx.compute = make_tracing_compute(std::move(ctx.compute), ctx.timeline.get());
  }
  ctx.comms.reset(new LiveFactory(std::move(ctx.comms), &ctx.live_comms));

  if (opt.topology) print_topology(ctx);

  Tracer::get().enable(opt.trace);
  std::unique_ptr<EnergyMeter> meter =
      ctx.dev->kind() == DeviceKind::GPU ? EnergyMeter::open_gpu(ctx.dev->index()) : EnergyMeter::none();
  FaultInjector fault(ri.rank);
  long long iter_no = 0;

  // ---- RCCL CTA budget: every comm lane's collective kernel must find CUs
  // beside the persistent compute (which leaves comm_cus CUs free), so
  // lanes x maxCTAs <= comm_cus; else blocks of one communicator's kernel can
  // sit in the queue while another communicator's kernel holds the free CUs
  // spinning on a peer that waits for them.
  const int lanes = collective_lanes(opt, ri.world_size);
  // xgmi kernels are budgeted too: a lane's kernel gets 4 blocks (512
  // threads, no LDS) per budgeted CU (comm_xgmi.cpp).
  const bool rccl = backend == "rccl" || backend == "mixed" || backend == "xgmi";
  const bool gemm_compute = ctx.compute->mode() == ComputeMode::Gemm;
  if (rccl) {
    if (opt.rccl_max_ctas >= 0)
      ctx.lane_ctas = opt.rccl_max_ctas;
    else
      ctx.lane_ctas = gemm_compute ? std::max(1, opt.comm_cus / lanes) : 0;
    if (ctx.lane_ctas > 0 && gemm_compute && lanes * ctx.lane_ctas > opt.comm_cus && ri.rank == 0)
      std::cerr << "[dlnb] warning: " << lanes << " comm lanes x " << ctx.lane_ctas << " RCCL CTAs > --comm-cus "
                << opt.comm_cus << ": concurrent collectives may not all fit beside the compute" << std::endl;
  }
  strat = make_strategy(opt.strategy);
  {
    TraceRange tr("dlnb:setup");
    strat->setup(ctx);
  }
  DLNB_REQUIRE(strat->streams().size() - 1 <= static_cast<size_t>(lanes),
               strategy_name(opt.strategy) << " uses " << strat->streams().size() - 1
                                           << " comm streams but collective_lanes() budgets " << lanes);
  if (ctx.dev->kind() == DeviceKind::GPU) {
    // More streams than hardware queues makes HIP share an in-order queue
    // between two streams: a collective spinning on its peers can then hold
    // back an unrelated kernel queued behind it on the other stream.
    const char* hwq = std::getenv("GPU_MAX_HW_QUEUES");
    const size_t nq = hwq ? static_cast<size_t>(std::max(1, std::atoi(hwq))) : 4;
    if (strat->streams().size() > nq && ri.rank == 0)
      std::cerr << "[dlnb] warning: " << strat->streams().size() << " streams per rank > GPU_MAX_HW_QUEUES=" << nq
                << "; streams will share hardware queues" << std::endl;
  }
  // DLNB_INJECT_FAULT mode=task: a task that throws on the first stream
  // (CPU devices; library hosts must get the error back, not lose the process)
  auto inject_task = [&] {
    DLNB_REQUIRE(ctx.dev->kind() == DeviceKind::CPU, "DLNB_INJECT_FAULT mode=task needs a CPU device");
    ctx.dev->host_task(*strat->streams()[0], [] { DLNB_THROW("injected fault in a stream task"); });
  };
  // the deadline clock's measured rate (kernels::wallclock_hz): taken here,
  // after setup gave its window time, and never inside a graph capture
  if (ctx.dev->kind() == DeviceKind::GPU) (void)ctx.dev->stamp_hz();
  Timeline* TL = ctx.timeline.get();
  if (TL) TL->calibrate(*strat->streams()[0]);
  TimerSet& T = *strat->timers();
  const char* rkey = strat->runtime_key();
  T.ensure(rkey);
  ctx.compute->set_task_timers(&T);

  // ---- HIP graph: capture one iteration, replay it every iteration.
  // Lane graphs (the default): every stream of the strategy is captured into
  // its own linear graph, launched on that stream, and the streams' ordering
  // is carried by device gates (Device::set_gate_events: an event record
  // raises a gate, a wait spins on it) instead of graph edges. The graph
  // executor then has no fork to spread over its hardware queues: compute
  // stays on the compute stream's queue and every collective on its lane's,
  // so no compute task queues behind a collective (profiles/absorb_r4.md), and
  // every stamp pair on one stream times exactly that stream's work. It needs
  // every stream on a hardware queue of its own (a gate wait would otherwise
  // hold the queue its signal sits behind): probed first, and a single graph
  // with event edges when they share one (lane_graphs.reason says why).
  std::unique_ptr<GraphExec> graph;
  std::vector<std::unique_ptr<GraphExec>> lane_graphs;
  // lane graphs: each lane's last node stores the iteration number here (the
  // host's completion words; Device::lane_done)
  uint64_t* lane_done = nullptr;
  size_t lane_done_n = 0;
  bool joined = false;  // the compute program's join signals the iteration (lane_done[0] alone)
  struct LaneDone {
    Device& d;
    uint64_t*& p;
    size_t& n;
    ~LaneDone() {
      if (p && std::uncaught_exceptions() == 0) d.free_stamps(p, n);
    }
  } lane_done_guard{*ctx.dev, lane_done, lane_done_n};
  Json lane_info = Json::object();
  std::vector<Stream*> lanes_ss;  // streams the replay is launched on (lane graphs: each; else the compute stream)
  std::vector<std::unique_ptr<Stream>> alt_owned;
  std::vector<Stream*> alt_ss;    // lane graphs: the second set, odd replays
  std::vector<Stream*> ss, others;  // --graph: the strategy's streams (compute first)
  // Capture one iteration: lane graphs when `lanes` (the capture may still
  // fall back to the single graph: not linear, no program), else the single
  // graph; `why` is the reason reported when there are no lanes.
  std::function<void(bool, std::string)> build_graph = [&](bool lanes, std::string why) {
    TraceRange tr("dlnb:graph_capture");
    T.begin_capture();
    if (TL) TL->begin_capture();
    if (lanes) {
      ctx.dev->set_gate_events(true);
      // each lane ends by clearing its own deadline slot for the next replay
      lane_done_n = ss.size();
      lane_done = ctx.dev->alloc_stamps(lane_done_n);
      // A compute program on the compute lane ends with a join on the other
      // lanes' end gates and signals the whole iteration from inside the
      // kernel (ComputeEngine::set_lane_join); otherwise every lane ends with
      // its own done word (and clears its deadline slot).
      std::vector<uint64_t*> end_gates;
      for (size_t i = 1; i < ss.size(); ++i) end_gates.push_back(ctx.dev->alloc_gate());
      ctx.compute->set_lane_join(*ss[0], end_gates, 1u, lane_done);
      const long progs0 = ctx.compute->programs_on(*ss[0]);
      lane_graphs = ctx.dev->capture_lanes(
          ss, [&] {
            T.iteration_start(*ss[0]);
            strat->enqueue_iteration();
            T.finish_stalls();
          },
          [&](size_t i) {
            if (ctx.compute->program_joined(*ss[0])) {
              if (i > 0) ctx.dev->signal_gate(*ss[i], end_gates[i - 1], 1u);
            } else {
              ctx.compute->reset_slot(*ss[i]);
              ctx.dev->lane_done(*ss[i], lane_done + i);
            }
            // The graph's last kernel carries its system-scope release (an L2
            // write-back: ~50 us after a collective's copy, round 5 traces):
            // a trailing no-op takes it, after the lane's signal is out.
            if (env_int("DLNB_LANE_TAIL_PAD", 1) != 0) ctx.dev->pad(*ss[i]);
          });
      ctx.compute->after_capture();  // the compute programs' task lists
      joined = ctx.compute->program_joined(*ss[0]);
      // A lane whose graph is not a chain (a library adding its own stream
      // to the capture, e.g. a collective's side work joined back) would be
      // spread over executor streams that may share the compute lane's
      // hardware queue - where a gate wait could hold the node that raises
      // its gate. Then the whole iteration is captured as one graph instead.
      // Lanes pay only when the compute lane is one compute program: a lane
      // of one launch per task puts every kernel boundary (28-60 us: drain,
      // dispatch) on one queue, which the single graph spreads over four
      // (C5 7.40-7.65 ms against 7.27, gemm-work C5 14.5 ms against 7.8:
      // profiles/lanes_r5.md). DLNB_LANE_GRAPHS=2 keeps such lanes anyway.
      bool linear = true;
      for (const auto& g : lane_graphs) linear = linear && g->linear();
      // ... or when its tasks are long single kernels (the pipeline hybrids:
      // one task per micro-batch; their boundaries cost little, while the
      // single graph's executor queues them behind collectives - hybrid_3d
      // S=2 mb=4 on 2 ranks: 100.0 ms with lanes against 104.9-106.7,
      // profiles/lanes_n2_r5.md). DLNB_LANE_MIN_TASK_US (1000).
      const double task_us = ctx.compute->lane_task_us(*ss[0]);
      const bool long_tasks = task_us >= static_cast<double>(env_int("DLNB_LANE_MIN_TASK_US", 1000)) &&
                              strat->lanes_without_program();
      // a compute program per iteration qualifies joined or not (not joined:
      // work follows it on the compute lane, which then ends with its own
      // done word - ADVICE r5)
      // - ONE program launch in the iteration: a task too short for a program
      // (< 20 us) splits it into several launches with kernels between, whose
      // boundaries all land on the compute lane's one queue
      const long progs = ctx.compute->programs_on(*ss[0]) - progs0;
      const bool program_ok = joined || (progs == 1 && !ctx.compute->program_split(*ss[0])) || long_tasks ||
                              env_int("DLNB_LANE_GRAPHS", 1) >= 2;
      lane_info["compute_programs"] = static_cast<double>(progs);
      lane_info["compute_task_us"] = task_us;
      const double verdict = ctx.hg().allreduce_max(!linear ? 2.0 : (!program_ok ? 1.0 : 0.0));
      linear = verdict < 0.5;
      if (linear) {
        lanes_ss = ss;
        // the first replay starts from cleared slots too
        ctx.compute->reset_clocks(*ss[0]);
        ss[0]->synchronize();
        // Every other replay goes to a second set of streams (same
        // priorities: the compute lane normal, the comm lanes high): a
        // launched graph's completion holds its queue for ~70-100 us after
        // its last node (round 5 traces), and the pre-armed next replay would
        // wait behind it. A graph runs on any stream; its nodes do not depend
        // on the one it was captured on.
        // Both sets are streams made here, after setup: replays on the
        // strategy's own streams (made before the communicators) ran their
        // collectives slower - every other iteration 0.13 ms (C5) / 0.3 ms
        // (headline) longer in round 5's A/B - so by default (DLNB_LANE_FRESH)
        // neither set is the capture's.
        // (not with ranks sharing the device, DLNB_LANE_SHARED: two processes'
        // extra stream sets oversubscribe the hardware queues - 2 ranks on one
        // GPU ran 143.4 ms without and 149.5-164.7 with, profiles/lanes_n2_r5.md)
        bool alt = env_int("DLNB_LANE_ALTERNATE", ctx.ranks_on_device > 1 ? 0 : 1) != 0;
        const bool fresh = env_int("DLNB_LANE_FRESH", 1) != 0;
        if (alt) {
          std::vector<Stream*> all = fresh ? std::vector<Stream*>() : ss;
          for (size_t k = 0; k < (fresh ? 2u : 1u); ++k)
            for (size_t i = 0; i < ss.size(); ++i) {
              alt_owned.push_back(ctx.dev->create_stream(i > 0));
              all.push_back(alt_owned.back().get());
            }
          std::string detail;
          alt = ctx.dev->queues_independent(all, 0.05, &detail);
        }
        alt = ctx.hg().allreduce_max(alt ? 0.0 : 1.0) < 0.5;
        if (alt) {
          const size_t n = ss.size();
          if (fresh) {
            lanes_ss.clear();
            for (size_t i = 0; i < n; ++i) lanes_ss.push_back(alt_owned[i].get());
          }
          for (size_t i = 0; i < n; ++i) alt_ss.push_back(alt_owned[(fresh ? n : 0) + i].get());
        } else {
          alt_owned.clear();
        }
      } else {
        // the rejected lanes' shapes (which library added what to a capture)
        Json rej = Json::array();
        for (const auto& g : lane_graphs) {
          Json e = Json::object();
          e["nodes"] = static_cast<double>(g->nodes());
          e["edges"] = static_cast<double>(g->edges());
          e["node_types"] = g->node_types();
          rej.push_back(e);
        }
        lane_info["rejected_lane_graphs"] = rej;
        lane_graphs.clear();
        ctx.dev->free_stamps(lane_done, lane_done_n);  // the single graph signals after its launch
        lane_done = nullptr;
        lane_done_n = 0;
        joined = false;
        ctx.dev->set_gate_events(false);
        lanes = false;
        why = verdict > 1.5 ? "a lane graph is not linear"
                            : "the compute lane is not one compute program (and the strategy's launch-per-task "
                              "lanes do not pay: Strategy::lanes_without_program)";
        T.end_capture();
        if (TL) TL->end_capture();
        T.begin_capture();
        if (TL) TL->begin_capture();
      }
    }
    if (!lanes) {
      // the engine's slot reset heads the graph, before every stream's first node
      graph = ctx.dev->capture(
          *ss[0], others, [&] {
            strat->enqueue_iteration();
            T.finish_stalls();
          }, [&] {
            ctx.compute->reset_clocks(*ss[0]);
            T.iteration_start(*ss[0]);
          });
      ctx.compute->after_capture();  // task lists of the launches captured (fixed-work tasks)
      lanes_ss = {ss[0]};
    }
    T.end_capture();
    if (TL) TL->end_capture();
    lane_info["enabled"] = lanes;
    if (lanes) {
      lane_info["program_join"] = joined;
      lane_info["alternating_streams"] = !alt_ss.empty();
    }
    if (!lanes) lane_info["reason"] = why;
    Json per = Json::array();
    size_t total = 0;
    bool all_linear = true;
    auto describe = [&](const GraphExec& g) {
      Json e = Json::object();
      e["nodes"] = static_cast<double>(g.nodes());
      e["edges"] = static_cast<double>(g.edges());
      e["linear"] = g.linear();
      e["node_types"] = g.node_types();
      total += g.nodes();
      all_linear = all_linear && g.linear();
      per.push_back(e);
    };
    if (lanes)
      for (auto& g : lane_graphs) describe(*g);
    else
      describe(*graph);
    lane_info["graphs"] = per;
    lane_info["linear"] = all_linear;
    if (ri.rank == 0 && !opt.quiet) {
      if (lanes)
        std::cout << "[dlnb] captured one iteration into " << lane_graphs.size() << " lane graphs of " << total
                  << " nodes (" << (all_linear ? "all linear" : "NOT all linear") << ")" << std::endl;
      else
        std::cout << "[dlnb] captured one iteration into a HIP graph of " << total << " nodes"
                  << (why.empty() ? "" : " (no lane graphs: " + why + ")") << std::endl;
    }
    };
  if (opt.graph) {
    DLNB_REQUIRE(ctx.dev->kind() == DeviceKind::GPU, "--graph needs a GPU");
    // xgmi kernels take their epochs from device-side counters, so a replayed
    // graph issues fresh ones; the loopback backends synchronise on the host.
    DLNB_REQUIRE(backend == "rccl" || backend == "xgmi" || backend == "mixed",
                 "--graph needs --backend rccl, xgmi or mixed");
    DLNB_REQUIRE(strat->capturable(), "--graph cannot capture --schedule reference (it blocks the host)");
    ss = strat->streams();
    others.assign(ss.begin() + 1, ss.end());
    std::string why;
    if (env_int("DLNB_LANE_GRAPHS", 1) == 0) {
      why = "DLNB_LANE_GRAPHS=0";
    } else if (ss.size() < 2) {
      why = "one stream";
    } else if (ctx.ranks_on_device > 1 && env_int("DLNB_LANE_SHARED", 0) == 0) {
      // a task spinning on its gate holds its CUs, which another rank's
      // compute on the same device - the one the collective waits for - needs
      // (DLNB_LANE_SHARED=1, with grids that fit side by side - --comm-cus -
      // and no slicing: the multi-rank lane path rehearsed on one GPU)
      why = "ranks share the device";
    } else {
      std::string detail;
      if (!ctx.dev->queues_independent(ss, 0.05, &detail)) why = "streams share a hardware queue (" + detail + ")";
    }
    // every rank takes the same decision, and every rank takes part in it
    bool lanes = ctx.hg().allreduce_max(why.empty() ? 0.0 : 1.0) < 0.5;
    if (!lanes && why.empty()) why = "another rank cannot use lane graphs";
    // Gate waits bounded by 4x the compute floor (at least 15 s) unless
    // DLNB_GATE_TIMEOUT_S is set: a gate that never comes costs the warm-up
    // that much before the safety valve below, not 60 s per wait.
    if (!std::getenv("DLNB_GATE_TIMEOUT_S")) {
      const double t = std::max(15.0, 4.0 * strat->compute_floor_us(ctx) * 1e-6 * opt.time_scale);
      ctx.dev->set_gate_timeout(t);
      ctx.compute->set_gate_timeout(t);
      lane_info["gate_timeout_s"] = t;
    }
    build_graph(lanes, why);
  }
  const bool replay = graph || !lane_graphs.empty();
  Stream* origin = replay ? strat->streams()[0] : nullptr;
  // Device iteration word (gates' sequence numbers): one value per replay,
  // stored at the head of every lane before its graph runs.
  uint64_t dev_iter = 0;
  // the streams replay `it` runs on (lane graphs alternate between two sets)
  auto lanes_for = [&](uint64_t it) -> const std::vector<Stream*>& {
    return !alt_ss.empty() && (it & 1) ? alt_ss : lanes_ss;
  };
  auto launch_graphs = [&](uint64_t it) {
    if (lane_graphs.empty()) {
      graph->launch(*origin);
      return;
    }
    const auto& L = lanes_for(it);
    for (size_t i = 0; i < lane_graphs.size(); ++i) lane_graphs[i]->launch(*L[i]);
  };
  auto enqueue = [&] {
    if (replay) {
      const uint64_t it = ++dev_iter;
      for (Stream* l : lanes_for(it)) ctx.dev->set_iteration(*l, it);
      launch_graphs(it);
    } else {
      T.iteration_start(*strat->streams()[0]);
      strat->enqueue_iteration();
      T.finish_stalls();
    }
  };
  // Host wait for the iteration just enqueued: lane graphs by their done words
  // (the graphs' own completion comes later: each ends with a marker), else
  // the streams.
  auto wait_iteration = [&] {
    if (lane_done) {
      CompletionFlag cf(lane_done, joined ? 1 : lane_done_n, dev_iter);
      strat->synchronize();
    } else {
      strat->synchronize();
    }
  };
  ctx.hg().barrier();

  // ---- warm-up
  std::vector<double> warm;
  for (int i = 0; i < opt.warmup; ++i) {
    fault.at_iteration(iter_no++, inject_task);
    TraceRange tr("dlnb:warmup_iteration");
    double t0 = now_s();
    enqueue();
    wait_iteration();
    warm.push_back(now_s() - t0);
    if (TL) TL->collect(-1);
  }
  // Lane replays that timed out a gate wait, or ran far longer than the
  // compute floor, in the warm-up: re-capture the single graph and warm it
  // once (every rank alike). A safety valve for a first run on hardware the
  // lanes were not measured on (the 8-GPU node); `lane_graphs.fallback`.
  if (!lane_graphs.empty() && !warm.empty()) {
    ComputeEngine::ChainCounters cc;
    double timeouts = static_cast<double>(ctx.dev->gate_event_timeouts());
    if (ctx.compute->chain_counters(cc)) timeouts += cc.wait_timeouts + cc.gate_timeouts;
    const double floor_s = strat->compute_floor_us(ctx) * 1e-6 * opt.time_scale;
    const bool slow = warm.back() > 2.0 * floor_s + static_cast<double>(env_int("DLNB_LANE_WARM_SLACK_S", 5));
    if (ctx.hg().allreduce_max((timeouts > 0 || slow) ? 1.0 : 0.0) > 0.5) {
      const std::string what = timeouts > 0 ? "gate waits timed out in the warm-up"
                                            : "a warm-up replay ran over twice the compute floor";
      if (ri.rank == 0 && !opt.quiet) std::cerr << "[dlnb] lane graphs: " << what << "; the single graph instead\n";
      ctx.dev->synchronize();
      lane_graphs.clear();
      if (lane_done) ctx.dev->free_stamps(lane_done, lane_done_n);
      lane_done = nullptr;
      lane_done_n = 0;
      joined = false;
      alt_ss.clear();
      alt_owned.clear();
      ctx.dev->set_gate_events(false);
      lane_info = Json::object();
      build_graph(false, "lanes fell back after the warm-up");
      lane_info["fallback"] = what;
      fault.at_iteration(iter_no++, inject_task);
      enqueue();
      wait_iteration();
    }
  }
  T.clear();

  int runs = opt.runs;
  if (opt.min_exectime > 0) {
    // Skip the first two warm-ups when there are more (cpp/utils.hpp:121-135).
    double s = 0;
    int n = 0;
    for (size_t i = warm.size() > 2 ? 2 : 0; i < warm.size(); ++i, ++n) s += warm[i];
    double avg = n ? s / n : 1.0;
    avg = ctx.hg().allreduce_max(avg);
    runs = std::max(1, static_cast<int>(std::ceil(opt.min_exectime / std::max(avg, 1e-9))));
    if (ri.rank == 0 && !opt.quiet)
      std::cout << "Estimated runs based on warm-up times to meet minimum execution time: " << runs << std::endl;
  }

  Json doc = Json::object();
  if (opt.loop) {
    // Interference generator (the reference's *_loop builds): no timers,
    // runs forever unless --max-loop-iters bounds it.
    T.set_enabled(false);
    for (long long it = 0; opt.max_loop_iters == 0 || it < opt.max_loop_iters; ++it) {
      fault.at_iteration(iter_no++, inject_task);
      TraceRange tr("dlnb:loop_iteration");
      enqueue();
      wait_iteration();
      if (TL) TL->collect(-1);
    }
    ctx.hg().barrier();
    ctx.hg().store().finish();
    doc["section"] = strat->section_id();
    doc["loop_iterations"] = opt.max_loop_iters;
    return doc;
  }

  // DLNB_TIMELINE_EDGES=1 (with --timeline --graph): a stamp kernel on the
  // launch stream before and after each timed graph launch (Timeline::edge;
  // two more kernels per iteration, so off by default)
  const bool tl_edges = env_int("DLNB_TIMELINE_EDGES", 0) != 0;
  // Graph replays on a GPU (DLNB_PREARM=1, the default): the host runs one
  // launch ahead. Iteration r+1's graph is enqueued while r runs, behind a
  // one-wave kernel that holds the launch stream until the host stores r+2 in
  // a host-coherent "go" word; a kernel after each graph stores r+1 in a
  // "done" word the host polls (CompletionFlag). Each iteration is still
  // timed alone, from the go store to the host seeing its done word, but its
  // start no longer waits for hipGraphLaunch's submission after an idle
  // device (~70 us) and its end not for hipStreamQuery (~20 us)
  // (profiles/host_boundary_r4.md). Iteration 0 is armed before the timed
  // region starts (as the last warm-up iteration would in a longer loop); all
  // of its device work runs inside it, as does the loop's closing device
  // synchronize. DLNB_PREARM=0: launch, then poll the streams (A/B).
  // Lane graphs: every lane has its own go wait and done word; the host
  // waits for all of them (the iteration ends when every stream has).
  const size_t nlanes = lanes_ss.size();
  const size_t nhs = 2 + nlanes;
  uint64_t* hs = nullptr;  // [0] go, [1] go-wait timeouts, [2 + i] lane i done
  if (replay && ctx.dev->kind() == DeviceKind::GPU && env_int("DLNB_PREARM", 1) != 0) hs = ctx.dev->alloc_stamps(nhs);
  struct Handshake {
    Device& d;
    uint64_t*& p;
    size_t n;
    ~Handshake() {
      if (std::uncaught_exceptions() != 0) {
        // The run failed inside the timed loop: abort the device waits before
        // anything is torn down - an armed replay is NOT released (its go
        // wait sees the abort and lets it run through poisoned: no compute,
        // no waits); a CLI process ends here (device_failure). The words are
        // not freed (hipHostFree waits for the device, which may be hung).
        device_failure("exception in the timed loop: " + last_error_message());
        return;
      }
      if (p) d.free_stamps(p, n);
    }
  } handshake{*ctx.dev, hs, nhs};
  // An armed replay waits for its go through the whole iteration before it:
  // its wait's bound (after which it runs anyway, counted in
  // prearm_go_timeouts) is 4x the compute floor + 60 s.
  const double go_timeout_s =
      std::max(60.0, 4.0 * strat->compute_floor_us(ctx) * 1e-6 * opt.time_scale + 60.0);
  std::vector<uint64_t> armed_iter;  // device iteration number of each armed replay
  auto arm = [&](int r) {
    const uint64_t it = ++dev_iter;
    armed_iter.push_back(it);
    const auto& L = lanes_for(it);
    for (size_t i = 0; i < nlanes; ++i) {
      Stream& l = *L[i];
      ctx.dev->host_wait(l, hs, static_cast<uint64_t>(r) + 1, go_timeout_s, hs + 1, it);
      if (TL && tl_edges && i == 0) TL->edge(l, 0);
      if (lane_graphs.empty())
        graph->launch(l);
      else
        lane_graphs[i]->launch(l);
      if (TL && tl_edges && i == 0) TL->edge(l, 1);
      // (lane graphs signal from inside: their last node, lane_done)
      if (!lane_done) ctx.dev->host_signal(l, hs + 2 + i, static_cast<uint64_t>(r) + 1);
    }
  };
  ctx.hg().barrier();
  ctx.compute->reset_capped(*strat->streams()[0]);  // count the timed iterations only
  ctx.dev->synchronize();
  // host time of each arm() (the launches of the next replay): a launch that
  // blocks on the runtime shows up here (profiles/stall_r5.md)
  std::vector<double> arm_s;
  if (hs && runs > 0) arm(0);  // submitted, held until the first go
  // clock / power at each iteration's end (the sampler thread's latest
  // readings, and sclk's range over the iteration: VERDICT r5 #7)
  std::vector<EnergyMeter::Sensors> sensors;
  {
    EnergyMeter::Sensors s0;
    meter->take(s0);  // the first window starts here
  }
  const double T0 = now_s();
  for (int r = 0; r < runs; ++r) {
    fault.at_iteration(iter_no++, inject_task);
    TraceRange tr("dlnb:iteration");
    const double j0 = meter->joules();
    double t0 = now_s();
    if (hs) {
      __atomic_store_n(hs, static_cast<uint64_t>(r) + 1, __ATOMIC_RELEASE);  // go
      if (r + 1 < runs) {
        const double a0 = now_s();
        arm(r + 1);
        arm_s.push_back(now_s() - a0);
      }
      if (lane_done) {
        CompletionFlag cf(lane_done, joined ? 1 : lane_done_n, armed_iter.at(static_cast<size_t>(r)));
        strat->synchronize();
      } else {
        CompletionFlag cf(hs + 2, nlanes, static_cast<uint64_t>(r) + 1);
        strat->synchronize();
      }
    } else {
      if (TL && replay && tl_edges) TL->edge(*origin, 0);
      enqueue();
      if (TL && replay && tl_edges) TL->edge(*origin, 1);
      wait_iteration();
    }
    const double t1 = now_s();
    T.add(rkey, t1 - t0);
    if (TL) {
      TL->collect(r);
      TL->host_iteration(r, t0, t1);
    }
    if (meter->available()) T.add("energy_consumed", meter->joules() - j0);
    EnergyMeter::Sensors sn;
    if (meter->take(sn)) sensors.push_back(sn);
  }
  ctx.dev->synchronize();
  ctx.hg().barrier();
  const double timed_region = ctx.hg().allreduce_max(now_s() - T0);

  // ---- report
  Json rank = strat->rank_json();
  if (hs) {
    rank["prearm_go_timeouts"] = static_cast<double>(__atomic_load_n(hs + 1, __ATOMIC_ACQUIRE));
    Json a = Json::array();
    for (double x : arm_s) a.push_back(x * 1e3);
    rank["prearm_launch_ms"] = a;
  }
  rank["energy_consumed"] = T.values_json("energy_consumed");
  if (!sensors.empty()) {
    Json c = Json::array(), lo = Json::array(), hi = Json::array(), w = Json::array();
    for (const auto& x : sensors) {
      c.push_back(x.sclk_mhz);
      lo.push_back(x.sclk_min_mhz);
      hi.push_back(x.sclk_max_mhz);
      w.push_back(x.power_w);
    }
    rank["iteration_sclk_mhz"] = c;
    rank["iteration_sclk_min_mhz"] = lo;
    rank["iteration_sclk_max_mhz"] = hi;
    rank["iteration_power_w"] = w;
  }
  {
    // the duration of each timed iteration's last collective (ms)
    const std::string tk = strat->tail_collective_timer();
    const auto& v = tk.empty() ? std::vector<double>() : T.get(tk);
    if (runs > 0 && !v.empty() && v.size() % static_cast<size_t>(runs) == 0) {
      const size_t per = v.size() / static_cast<size_t>(runs);
      Json a = Json::array();
      for (int r = 0; r < runs; ++r) a.push_back(v[(static_cast<size_t>(r) + 1) * per - 1] * 1e3);
      rank["iteration_last_collective_ms"] = a;
      rank["iteration_last_collective"] = tk;
    }
  }
  {
    // chained deadline tasks: lateness absorbed (<= the cap each) and beyond
    // the cap (deadline_sync.hpp), gate waits that timed out
    ComputeEngine::ChainCounters cc;
    if (runs > 0 && ctx.compute->chain_counters(cc)) {
      Json c = Json::object();
      c["tasks_per_iter"] = cc.capped_tasks / runs;
      c["ms_per_iter"] = cc.capped_s / runs * 1e3;
      c["absorbed_tasks_per_iter"] = cc.absorbed_tasks / runs;
      c["absorbed_ms_per_iter"] = cc.absorbed_s / runs * 1e3;
      // device gate waits that gave up at their bound (never expected): a comm
      // lane's gate_wait, a deadline task's gate, a gate event's wait
      c["gate_wait_timeouts"] = cc.wait_timeouts + static_cast<double>(ctx.dev->gate_event_timeouts());
      c["compute_gate_timeouts"] = cc.gate_timeouts;
      // waits that left on the host's abort word, program blocks that came late for a task
      c["aborted_waits"] = cc.aborted;
      c["late_blocks"] = cc.late_blocks;
      rank["chain_capped"] = c;
    }
  }
  // intervals whose stamps came out of order (recorded as 0; never expected)
  if (T.has_negatives()) rank["timer_negative_intervals"] = T.negatives_json();
  rank["hostname"] = ri.hostname;
  rank["rank"] = ri.rank;
  rank["local_rank"] = ri.local_rank;
  rank["device_name"] = ctx.dev->name();
  rank["device_index"] = ctx.dev->index();
  rank["comm"] = strat->comm_summary();
  // Fixed-work compute: measured task time / uncontended (table) time over
  // the timed runs. > 1 means the collectives running beside the compute
  // (HBM traffic, CUs, power) slowed it down.
  const double task_s = T.sum("compute_task_time"), table_s = T.sum("compute_task_table");
  if (!T.get("compute_task_time").empty() && table_s > 0) {
    rank["compute_stretch"] = task_s / table_s;
    rank["compute_task_s"] = task_s;
    rank["compute_table_s"] = table_s;
  }
  auto all = ctx.hg().allgather(rank.dump());
  Json timeline_info = nullptr;
  if (TL) {
    Json mine = TL->rank_json(ri.rank, opt.timeline_iters);
    mine["device"] = ctx.dev->name() + " " + std::to_string(ctx.dev->index()) + " @ " + ri.hostname;
    auto parts = ctx.hg().allgather(mine.dump());
    timeline_info = Json::object();
    timeline_info["path"] = opt.timeline_path;
    timeline_info["iterations_kept"] = opt.timeline_iters;
    long long nev = 0;
    bool trunc = false;
    std::vector<Json> docs;
    for (const auto& p : parts) {
      docs.push_back(Json::parse(p));
      nev += static_cast<long long>(docs.back().at("events").size());
      trunc = trunc || docs.back().at("truncated").as_bool();
    }
    timeline_info["events"] = nev;
    timeline_info["truncated"] = trunc;
    if (ri.rank == 0) {
      Json meta = Json::object();
      meta["strategy"] = strategy_name(opt.strategy);
      meta["model"] = opt.model;
      meta["backend"] = backend;
      meta["graph"] = opt.graph;
      meta["world_size"] = ri.world_size;
      write_chrome_trace(opt.timeline_path, docs, meta);
    }
  }

  Json g = strat->global_json();
  Json ext = Json::object();
  ext["strategy"] = strategy_name(opt.strategy);
  ext["schedule"] = opt.schedule;
  {
    size_t nodes = graph ? graph->nodes() : 0;
    for (const auto& g : lane_graphs) nodes += g->nodes();
    ext["graph"] = static_cast<double>(nodes);
  }
  if (opt.graph) ext["lane_graphs"] = lane_info;
  // pre-armed replay loop (each iteration's launch submitted during the one
  // before, released by a host store; DLNB_PREARM=0 launches in the loop)
  ext["prearm"] = hs != nullptr;
  ext["wire_dtype"] = dtype_name(ctx.wire);
  ext["compute"] = ctx.compute->describe();
  ext["stats_file"] = stats_path;
  ext["stats_dtype"] = ctx.stats.dtype;
  ext["stats_device"] = ctx.stats.device;
  ext["warmup"] = opt.warmup;
  ext["runs"] = runs;
  ext["warmup_times"] = Json(warm);
  ext["timed_region_s"] = timed_region;
  ext["energy_source"] = meter->source();
  // ranks of this job on this rank's device (> 1: loopback threads or -d 0,0;
  // the deadline compute then runs in 500-us slices, compute.cpp)
  ext["ranks_on_device"] = ctx.ranks_on_device;
  if (TL) ext["timeline"] = timeline_info;
  {
    Json b = Json::object();
    b["lanes"] = lanes;
    b["comm_cus"] = opt.comm_cus;
    b["max_ctas_per_lane"] = ctx.lane_ctas;  // 0 = RCCL default
    b["applies"] = rccl;
    b["fits"] = !rccl || !gemm_compute || ctx.lane_ctas == 0 ? true : lanes * ctx.lane_ctas <= opt.comm_cus;
    if (backend == "xgmi" || backend == "mixed") {
      // xgmi kernels: blocks per lane = blocks_per_cu x max_ctas, so a lane
      // occupies max_ctas CUs at the measured occupancy
      const int bpc = xgmi::min_blocks_per_cu();
      b["xgmi_blocks_per_cu"] = bpc;
      b["xgmi_blocks_per_lane"] = ctx.lane_ctas > 0 ? bpc * ctx.lane_ctas : 0;
    }
    ext["rccl_cta_budget"] = b;
  }
  {
    Json cl = comm_log_json(ctx.comm_log);
    ext["communicators"] = cl.at("communicators");
    ext["rccl_nranks"] = cl.at("rccl_nranks");
    if (ctx.dev->kind() == DeviceKind::GPU) ext["runtime"] = runtime_info();
  }
  {
    // Collective-library knobs of this run (the reference recorded them as
    // SbatchMan job variables, plots/parser.py:151-154).
    Json env = Json::object();
    for (char** e = environ; e && *e; ++e) {
      std::string kv = *e;
      if (starts_with(kv, "NCCL_") || starts_with(kv, "RCCL_") || starts_with(kv, "HSA_") || starts_with(kv, "DLNB_")) {
        size_t eq = kv.find('=');
        if (eq != std::string::npos) env[kv.substr(0, eq)] = kv.substr(eq + 1);
      }
    }
    ext["env"] = env;
  }
  // Iteration time = max over ranks per run (the slowest rank bounds a step).
  std::vector<Json> ranks;
  for (const auto& s : all) ranks.push_back(Json::parse(s));
  std::vector<double> per_run(static_cast<size_t>(runs), 0.0);
  for (const auto& rj : ranks) {
    const Json& v = rj.at(rkey);
    for (size_t i = 0; i < v.size() && i < per_run.size(); ++i) per_run[i] = std::max(per_run[i], v.at(i).as_double());
  }
  Json it = Json::object();
  it["per_run_max_s"] = Json(per_run);
  it["median_ms"] = percentile(per_run, 0.5) * 1e3;
  double mean = 0;
  for (double x : per_run) mean += x;
  it["mean_ms"] = per_run.empty() ? 0.0 : mean / per_run.size() * 1e3;
  it["p95_ms"] = percentile(per_run, 0.95) * 1e3;
  it["min_ms"] = per_run.empty() ? 0.0 : *std::min_element(per_run.begin(), per_run.end()) * 1e3;
  it["timed_ms_per_iter"] = runs > 0 ? timed_region / runs * 1e3 : 0.0;
  double floor_us = strat->compute_floor_us(ctx);
  it["compute_floor_ms"] = floor_us / 1e3 * opt.time_scale;
  ext["iteration"] = it;
  {
    double worst = 0;
    for (const auto& rj : ranks)
      if (rj.contains("compute_stretch")) worst = std::max(worst, rj.at("compute_stretch").as_double());
    if (worst > 0) ext["compute_stretch"] = worst;  // max over ranks
    // Compute tasks that waited beyond the chain's absorb cap per iteration
    // (the wait stays in the iteration time; max over ranks)
    double ctasks = -1, cms = 0, gto = 0, cgto = 0, ams = 0, atasks = 0;
    for (const auto& rj : ranks)
      if (rj.contains("chain_capped")) {
        const Json& c = rj.at("chain_capped");
        ctasks = std::max(ctasks, c.at("tasks_per_iter").as_double());
        cms = std::max(cms, c.at("ms_per_iter").as_double());
        gto = std::max(gto, c.at("gate_wait_timeouts").as_double());
        cgto = std::max(cgto, c.at("compute_gate_timeouts").as_double());
        ams = std::max(ams, c.at("absorbed_ms_per_iter").as_double());
        atasks = std::max(atasks, c.at("absorbed_tasks_per_iter").as_double());
      }
    if (ctasks >= 0) {
      Json c = Json::object();
      c["tasks_per_iter_max"] = ctasks;
      c["ms_per_iter_max"] = cms;
      c["gate_wait_timeouts_max"] = gto;
      c["compute_gate_timeouts_max"] = cgto;
      // lateness the chained tasks took out of their own compute (launch
      // hops, drains): invisible in the iteration time, shown here
      c["absorbed_ms_per_iter_max"] = ams;
      c["absorbed_tasks_per_iter_max"] = atasks;
      ext["chain_capped"] = c;
    }
  }
  g["dlnb"] = ext;

  doc["section"] = strat->section_id();
  doc["title"] = strat->section_title();
  doc["global"] = g;
  Json rarr = Json::array();
  for (auto& r : ranks) rarr.push_back(r);
  doc["ranks"] = rarr;

  if (ri.rank == 0 && !opt.silent) {
    std::string text = doc.dump();
    std::cout << "<<<DLNB_REPORT_BEGIN " << strat->section_id() << ">>>\n"
              << text << "\n<<<DLNB_REPORT_END " << strat->section_id() << ">>>" << std::endl;
    if (!opt.quiet) {
      std::printf("[dlnb] %s %s W=%d backend=%s compute=%s: iter median %.3f ms (floor %.3f ms), timed %.3f ms/iter\n",
                  strategy_name(opt.strategy), opt.model.c_str(), ri.world_size, backend.c_str(),
                  compute_mode_name(ctx.compute->mode()), it.at("median_ms").as_double(),
                  it.at("compute_floor_ms").as_double(), it.at("timed_ms_per_iter").as_double());
      std::fflush(stdout);
    }
  }
  if (ri.rank == 0 && !opt.json_path.empty()) {
    std::ofstream f(opt.json_path);
    f << doc.dump(1) << "\n";
  }
  ctx.hg().barrier();  // keep the store (rank 0) alive until everyone is done
  ctx.hg().store().finish();
  return doc;
}

}  // namespace

int main_for(StrategyKind kind, int argc, char** argv) {
  Options opt;
  try {
    opt = parse_options(kind, argc, argv);
  } catch (const std::exception& e) {
    std::cerr << e.what() << std::endl;
    return 1;
  }
  std::string prog = argc > 0 ? argv[0] : "";
  if (opt.help) {
    std::cout << usage(kind, prog);
    return 0;
  }
  if (ends_with(prog, "_loop")) opt.loop = true;
  g_cli_process.store(true);
  try {
    run_benchmark(opt);
  } catch (const std::exception& e) {
    std::cerr << "[dlnb] rank " << env_or("RANK", env_or("DLNB_RANK", "0")) << " error: " << e.what() << std::endl;
    return 2;
  }
  return 0;
}

}  // namespace dlnb
