// Command-line contract.
//
// Positional arguments and the short flags match the reference's easyargs
// definitions (e.g. cpp/data_parallel/dp.cpp:108-122):
//   dp            <model> <num_buckets> <base_path>
//   fsdp          <model> <num_units> <sharding_factor> <base_path>
//   hybrid_2d     <model> <num_stages> <num_microbatches> <base_path>
//   hybrid_3d     <model> <num_stages> <num_microbatches> <num_tensor_shards> <base_path>
//   hybrid_3d_moe <model> <num_stages> <num_microbatches> <num_expert_shards> <base_path>
//   hybrid_cp     <model> <num_cp_shards> <base_path>   (extension: DP x context parallel)
//   hybrid_4d     <model> <num_stages> <num_microbatches> <num_tensor_shards> <num_expert_shards> <base_path>
//                 (extension: DP x PP x TP x EP)
//   flags: -w warmups (3)  -r runs (5; hybrid_3d 3)  -d devices ("")
//          -m min_exectime seconds (0)  -h
// Long options are dlnb extensions (run-time backend, compute model,
// schedule, output file, loop mode instead of separate *_loop builds).
#pragma once

#include <string>
#include <vector>

namespace dlnb {

enum class StrategyKind { DP, FSDP, Hybrid2D, Hybrid3D, Hybrid3DMoE, HybridCP, Hybrid4D };

StrategyKind parse_strategy(const std::string& s);
const char* strategy_name(StrategyKind k);

struct Options {
  StrategyKind strategy = StrategyKind::DP;
  std::string model;
  std::string base_path = ".";
  int num_buckets = 10;
  int num_units = 1;
  int sharding_factor = 1;
  int num_stages = 1;
  int num_microbatches = 1;
  int num_tensor_shards = 1;
  int num_expert_shards = 1;
  int num_cp_shards = 1;
  std::string cp_algo = "ring";  // hybrid_cp: ring (P2P KV blocks) | ulysses (all-to-all)

  int warmup = 3;
  int runs = 5;
  std::string devices;
  double min_exectime = 0;
  bool help = false;

  // dlnb extensions
  std::string backend = "auto";   // auto | rccl | xgmi | cpu | loopback
  int ranks = 2;                  // loopback: in-process ranks (threads) sharing one device
  std::string compute = "auto";   // auto | sleep | spin | gemm | flops
  std::string wire_dtype = "bf16";
  std::string compute_dtype = "auto";  // auto (from stats Dtype) | bf16 | fp8
  std::string schedule = "overlap";    // overlap | reference
  std::string tp_granularity = "microbatch";  // microbatch | layer
  bool sequence_parallel = false;  // TP all-reduce -> all-gather + reduce-scatter (Megatron-SP)
  std::string pp_schedule = "gpipe";          // gpipe (reference) | 1f1b | interleaved
  int pp_virtual = 2;                         // interleaved: model chunks (virtual stages) per stage
  bool ep_overlap = false;  // moe: overlap each half-microbatch's all-to-all with the other half's compute
  double ep_imbalance = 0;  // moe: Zipf exponent of the expert-rank load (0 = uniform all-to-all)
  double dp_bucket_ratio = 1.0;  // dp: geometric bucket sizes (strategy_dp.cpp dp_bucket_sizes)
  int dp_buckets = 1;  // hybrids: DP all-reduce buckets overlapped with the last backward
  bool in_place = false;
  // dp: ZeRO stage. 0 = replicated (reference), 1 = optimizer state sharded
  // (all-reduce grads, step on the 1/W shard, all-gather parameters), 2 =
  // gradients sharded too (bucketed reduce-scatter instead of all-reduce).
  int zero = 0;
  bool optimizer = false;  // add an elementwise optimizer step over the local shard
  bool loop = false;       // the reference's *_loop builds
  long long max_loop_iters = 0;
  double time_scale = 1.0;  // scales every compute duration (tests)
  std::string json_path;
  std::string store_addr;
  std::string stats_file;  // explicit stats path (overrides base_path lookup)
  bool topology = true;
  bool quiet = false;
  bool silent = false;  // print nothing (library use, e.g. bench.py)
  bool trace = false;   // roctx ranges around iterations and phases
  // device timeline (dlnb/timeline.hpp): Chrome trace of every collective,
  // P2P group and compute task of every rank, written by rank 0
  std::string timeline_path;
  int timeline_iters = 2;  // timed iterations kept in it (0 = all)
  int comm_cus = 32;    // CUs left free by the persistent compute for collectives
  // RCCL maxCTAs per communicator on a comm lane: -1 = comm_cus / lanes
  // (runner.cpp, collective_lanes), 0 = RCCL's default, N = N.
  int rccl_max_ctas = -1;
  // fsdp: "single" = every collective of a rank on one in-order comm lane
  // (deadlock-free across communicators), "split" = one lane per collective
  // kind so all-gather / reduce-scatter / replica all-reduce run concurrently.
  std::string comm_lanes = "single";
  bool graph = false;  // capture one iteration into a HIP graph and replay it
};

// Parses argv for the given strategy (argv[0] is the program name). Throws
// dlnb::Error with a usage message on bad input.
Options parse_options(StrategyKind kind, int argc, const char* const* argv);
std::string usage(StrategyKind kind, const std::string& prog);

}  // namespace dlnb
