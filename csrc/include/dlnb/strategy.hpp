// Strategy drivers: DP, FSDP/HSDP, DP+PP, DP+PP+TP, DP+PP+EP.
//
// Each driver reproduces the communication of one parallelism strategy with
// the reference's group layout and message-size formulas (SURVEY.md
// §2.2/§2.4) and overlaps it with synthetic compute. Unlike the reference,
// the iteration is enqueued on streams (compute + one stream per
// communicator) and ordered by events, so communication overlaps compute on
// the device without the host thread in the loop; `--schedule reference`
// re-inserts the reference's blocking points for A/B comparisons.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "dlnb/bootstrap.hpp"
#include "dlnb/comm.hpp"
#include "dlnb/compute.hpp"
#include "dlnb/device.hpp"
#include "dlnb/json.hpp"
#include "dlnb/options.hpp"
#include "dlnb/timers.hpp"
#include "dlnb/timeline.hpp"
#include "dlnb/workload.hpp"

namespace dlnb {

// One communicator the run created (recorded by select_backend's factory):
// group name, member count and the library's own rank count.
struct CommRecord {
  std::string name;
  std::string backend;
  int nranks;
  int library_nranks;  // RCCL: ncclCommCount; -1 for backends without one
};

struct Context {
  Options opt;
  std::unique_ptr<Bootstrap> boot;
  std::unique_ptr<Device> dev;
  std::unique_ptr<CommFactory> comms;
  std::vector<CommRecord> comm_log;
  // every communicator the strategy created (outermost wrapper; owned by the
  // strategy): the failure path aborts them all (device_failure)
  std::vector<Communicator*> live_comms;
  std::unique_ptr<ComputeEngine> compute;
  ModelStats stats;
  bool have_arch = false;
  ModelArch arch;
  DType wire = DType::BF16;
  // RCCL CTA cap for communicators whose collectives run on a comm lane
  // (a stream beside the compute); 0 = library default.
  int lane_ctas = 0;
  int ranks_on_device = 1;  // ranks of this job sharing this rank's device (loopback, -d 0,0)
  // --timeline: the spans of this rank (declared last: released before the
  // device whose stamp slots it holds)
  std::unique_ptr<Timeline> timeline;
  int rank() const { return boot->info.rank; }
  int world() const { return boot->info.world_size; }
  HostGroup& hg() { return *boot->world; }
};

// Rank layout shared by the hybrid drivers: inner (TP or EP) fastest, then
// pipeline stage, then data-parallel replica (hybrid_3d.cpp:283-300,
// hybrid_3d_moe.cpp:313-331; hybrid_2d is inner = 1, hybrid_2d.cpp:272-282).
struct GridCoords {
  int inner_id, stage_id, dp_id;
};
GridCoords grid_coords(int rank, int inner, int stages);
std::vector<int> inner_group(int rank, int inner, int stages);  // same (dp, stage)
std::vector<int> pp_group(int rank, int inner, int stages);     // same (dp, inner)
std::vector<int> dp_group(int rank, int inner, int stages, int world);  // same (stage, inner)

class Strategy {
 public:
  virtual ~Strategy() = default;
  virtual void setup(Context& ctx) = 0;
  // Enqueue one iteration (host returns once everything is enqueued; with
  // --schedule reference it may block at the reference's blocking points).
  virtual void enqueue_iteration() = 0;
  // Host-wait for the iteration to finish (with failure detection).
  virtual void synchronize() = 0;
  // Every stream the iteration uses, the compute stream first (graph
  // capture forks the others from it and joins them back).
  virtual std::vector<Stream*> streams() = 0;
  // False when enqueue_iteration() blocks the host (--schedule reference),
  // which a graph capture cannot contain.
  virtual bool capturable() const = 0;
  // Whether lane graphs pay for this strategy when its compute lane is not
  // one compute program (each task a launch of its own, >= 1 ms on average):
  // not when cross-rank collectives sit on the compute stream between the
  // tasks (pipeline TP / EP with more than one shard: hybrid_3d T=2 on 2
  // ranks ran 81.7 ms with lanes against 79.3 on the single graph), nor for
  // CP's ~200 task boundaries per iteration (W=1: 4.16 ms over the floor
  // against 1.3); the pipeline (2 ranks: 100.3 vs 104.8-106.4 ms) and ZeRO DP
  // (21.7 vs 22.7 ms) do (profiles/hostwait_r5.md).
  virtual bool lanes_without_program() const { return true; }
  virtual std::string section_id() const = 0;
  virtual std::string section_title() const = 0;
  // Per-rank key of the host iteration times ("runtimes"; fsdp uses "runtime").
  virtual const char* runtime_key() const { return "runtimes"; }
  virtual Json global_json() const = 0;
  virtual Json rank_json() const = 0;
  // Bus-bandwidth summary per collective kind for this rank (bytes, seconds).
  virtual Json comm_summary() const = 0;
  // Lower bound of an iteration from compute alone (µs): fwd + bwd for
  // dp/fsdp, the pipeline's (mb + S - 1)(f_mb + b_mb), (fwd + bwd) / C for CP.
  virtual double compute_floor_us(const Context& ctx) const {
    return ctx.stats.avg_forward_time_us + ctx.stats.avg_backward_time_us;
  }
  // The timer of the iteration's last collective (the runner reports its
  // last entry per timed iteration: iteration_last_collective_ms).
  virtual std::string tail_collective_timer() const { return ""; }
  TimerSet* timers() { return timers_.get(); }

 protected:
  std::unique_ptr<TimerSet> timers_;
};

std::unique_ptr<Strategy> make_dp();
std::unique_ptr<Strategy> make_fsdp();
std::unique_ptr<Strategy> make_pipeline(StrategyKind kind);  // hybrid_2d / 3d / 3d_moe
std::unique_ptr<Strategy> make_cp();                          // hybrid_cp (extension)

// Upper bound on the comm lanes (streams other than the compute stream that
// carry collectives) a rank of this configuration keeps live at once: dp 1;
// fsdp 1 (--comm-lanes single) or 2 + (replicas > 1) (split); hybrid_cp 2;
// pipelines 3 when S > 1 (prev link, next link, DP lane - which also carries
// the DualPipe mirror and --ep-overlap all-to-alls) else 1. Collectives on
// the compute stream (TP all-reduce, EP all-to-all) never overlap the GEMM
// and are not counted.
int collective_lanes(const Options& o, int world);

// Creates ctx.dev + ctx.comms for a backend (auto | rccl | xgmi | cpu);
// GPU ranks take device list[local_rank] ("-d 0,1,..", default all GPUs).
// Returns the resolved backend name. ctx.boot must be set.
std::string select_backend(Context& ctx, const std::string& requested, const std::string& devices);

// Collective correctness / bandwidth tool: dlnb commtest [options].
int commtest_main(int argc, char** argv);
// dlnb info: one JSON line with the HIP / RCCL runtime this binary bound and
// the xgmi kernels' occupancy (blocks per CU) on the visible GPU.
int info_main(int argc, char** argv);

// Runs a whole benchmark (bootstrap -> setup -> warmup -> timed runs ->
// report). Returns the report document (rank 0 has the gathered ranks).
Json run_benchmark(const Options& opt);

// Entry point shared by the CLI binaries; returns the process exit code.
int main_for(StrategyKind kind, int argc, char** argv);

// Synchronise a set of streams with a deadline; polls communicator async
// errors so a dead peer aborts the job instead of hanging it (the failure
// goes through device_failure before the exception is thrown).
void sync_streams(const std::vector<Stream*>& streams, const std::vector<Communicator*>& comms, Device& dev);

// The failure path of a run on this thread, called where a
// failure is detected (sync_streams' timeout / async error, an exception
// leaving the timed loop, run_rank's catch) BEFORE anything is torn down:
// raises the device's abort word - every device-side wait gives up, a
// pre-armed replay runs through poisoned - and then, in a CLI process that
// owns its ranks (no loopback hub), prints `why` and ends the process at once
// (std::_Exit(3): the kernel driver reclaims the queues; no destructor waits
// on device work that may never finish); otherwise (a library host) aborts
// every communicator of the run. Once per run; a no-op outside one.
void device_failure(const std::string& why);
// Whether a failed run of this process left device work that did not drain
// (Device::abort_and_drain): the process then refuses further runs.
bool process_poisoned();

// While alive on this thread: sync_streams() waits for flags[i] >= value for
// every i < n (host-coherent words a kernel enqueued after each replayed
// graph stores) instead of querying the streams - a single graph joins every
// stream it forked back onto its launch stream before that kernel runs, and
// lane graphs have one word per lane, so the words prove the whole iteration
// complete (runner's pre-armed graph loop).
class CompletionFlag {
 public:
  CompletionFlag(const uint64_t* flags, size_t n, uint64_t value);
  ~CompletionFlag();
  CompletionFlag(const CompletionFlag&) = delete;
  CompletionFlag& operator=(const CompletionFlag&) = delete;

 private:
  const uint64_t* prev_;
  size_t prev_n_;
  uint64_t prev_value_;
};

// Helper shared by the drivers: a stats summary for bus-bandwidth reporting.
struct CommStat {
  std::string name;
  CollKind kind;
  int nranks;
  double bytes_per_op;  // algorithm bytes (nccl-tests convention)
  std::string timer;    // timer key holding the op durations
};
Json comm_stats_json(const std::vector<CommStat>& stats, const TimerSet& t);

void print_topology(Context& ctx);

// HIP runtime / RCCL this process is bound to: versions and the shared
// objects they were loaded from (comm_rccl.cpp).
Json runtime_info();

// The communicator log as report JSON: "communicators" (every group) and
// "rccl_nranks" (group name -> ncclCommCount, RCCL groups only).
Json comm_log_json(const std::vector<CommRecord>& log);

// Elementwise SGD-momentum over a bf16 shard (the optional --optimizer step).
// end_stamp (optional, a TimerSet slot): the step's end on the device clock,
// stored by the kernel itself (GPU: `done` a zeroed device word; CPU: the task).
void optimizer_step(Context& ctx, Stream& s, void* param, void* mom, const void* grad, size_t n,
                    uint64_t* end_stamp = nullptr, uint32_t* done = nullptr);

}  // namespace dlnb
