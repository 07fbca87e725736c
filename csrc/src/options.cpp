#include "dlnb/options.hpp"

#include <cstdlib>
#include <sstream>

#include "dlnb/common.hpp"

namespace dlnb {

StrategyKind parse_strategy(const std::string& s) {
  if (s == "dp") return StrategyKind::DP;
  if (s == "fsdp") return StrategyKind::FSDP;
  if (s == "hybrid_2d" || s == "dp_pp") return StrategyKind::Hybrid2D;
  if (s == "hybrid_3d" || s == "dp_pp_tp") return StrategyKind::Hybrid3D;
  if (s == "hybrid_3d_moe" || s == "dp_pp_ep") return StrategyKind::Hybrid3DMoE;
  if (s == "hybrid_cp" || s == "dp_cp") return StrategyKind::HybridCP;
  if (s == "hybrid_4d" || s == "dp_pp_tp_ep") return StrategyKind::Hybrid4D;
  DLNB_THROW("unknown strategy '" << s << "' (dp, fsdp, hybrid_2d, hybrid_3d, hybrid_3d_moe, hybrid_cp, hybrid_4d)");
}

const char* strategy_name(StrategyKind k) {
  switch (k) {
    case StrategyKind::DP: return "dp";
    case StrategyKind::FSDP: return "fsdp";
    case StrategyKind::Hybrid2D: return "hybrid_2d";
    case StrategyKind::Hybrid3D: return "hybrid_3d";
    case StrategyKind::Hybrid3DMoE: return "hybrid_3d_moe";
    case StrategyKind::HybridCP: return "hybrid_cp";
    case StrategyKind::Hybrid4D: return "hybrid_4d";
  }
  return "?";
}

namespace {

std::vector<std::string> positional_names(StrategyKind k) {
  switch (k) {
    case StrategyKind::DP: return {"model", "num_buckets", "base_path"};
    case StrategyKind::FSDP: return {"model", "num_units", "sharding_factor", "base_path"};
    case StrategyKind::Hybrid2D: return {"model", "num_stages", "num_microbatches", "base_path"};
    case StrategyKind::Hybrid3D: return {"model", "num_stages", "num_microbatches", "num_tensor_shards", "base_path"};
    case StrategyKind::Hybrid3DMoE:
      return {"model", "num_stages", "num_microbatches", "num_expert_shards", "base_path"};
    case StrategyKind::HybridCP: return {"model", "num_cp_shards", "base_path"};
    case StrategyKind::Hybrid4D:
      return {"model", "num_stages", "num_microbatches", "num_tensor_shards", "num_expert_shards", "base_path"};
  }
  return {};
}

int to_int(const std::string& v, const std::string& what) {
  char* end = nullptr;
  long r = std::strtol(v.c_str(), &end, 10);
  if (!end || *end || v.empty()) DLNB_THROW("invalid integer for " << what << ": '" << v << "'");
  return static_cast<int>(r);
}

double to_double(const std::string& v, const std::string& what) {
  char* end = nullptr;
  double r = std::strtod(v.c_str(), &end);
  if (!end || *end || v.empty()) DLNB_THROW("invalid number for " << what << ": '" << v << "'");
  return r;
}

}  // namespace

std::string usage(StrategyKind kind, const std::string& prog) {
  std::ostringstream os;
  os << "Usage: " << prog;
  for (const auto& p : positional_names(kind)) os << " <" << p << ">";
  os << " [options]\n"
     << "  -w, --warmups N        warm-up iterations (default 3)\n"
     << "  -r, --runs N           timed iterations (default " << (kind == StrategyKind::Hybrid3D ? 3 : 5) << ")\n"
     << "  -d, --devices LIST     comma-separated device ids indexed by local rank\n"
     << "  -m, --min_exectime S   run at least S seconds (overrides --runs)\n"
     << "  -h, --help             this help\n"
     << "  --backend B            auto | rccl | xgmi | mixed | cpu | loopback | loopback-cpu\n"
     << "  --ranks N              loopback: ranks run as threads of this process on one GPU\n"
     << "                         (loopback-cpu: on the CPU device), default 2\n"
     << "  --compute C            auto | sleep | spin | gemm | gemm-work | flops\n"
     << "  --wire-dtype T         bf16 | fp16 | fp32 | fp8 (collective element type)\n"
     << "  --compute-dtype T      auto | bf16 | fp8 (GEMM operand type for gemm/flops)\n"
     << "  --schedule S           overlap (stream-ordered) | reference (blocking like DLNetBench)\n"
     << "  --tp-granularity G     microbatch | layer (hybrid_3d, hybrid_4d)\n"
     << "  --sequence-parallel    hybrid_3d/4d: each TP all-reduce becomes all-gather + reduce-scatter (Megatron-SP)\n"
     << "  --pp-schedule gpipe|1f1b|interleaved  hybrids: all forwards then all backwards (reference),\n"
     << "                         one-forward-one-backward, or interleaved 1F1B over --pp-virtual V chunks per stage\n"
     << "  --pp-virtual V         interleaved: model chunks per stage (default 2)\n"
     << "  --ep-overlap           hybrid_3d_moe: two half-microbatches, each one's all-to-all under the other's compute\n"
     << "  --ep-imbalance A       moe: skewed expert load, rank j of an EP group gets a 1/(j+1)^A share of\n"
     << "                         every dispatch (all-to-allv over grouped send/recv); 0 = uniform (reference)\n"
     << "  --dp-buckets K         hybrids: DP all-reduce buckets overlapped with the last backward\n"
     << "                         (hybrid_cp: gradient buckets by layer, overlapped with the backward)\n"
     << "  --dp-bucket-ratio R    dp: bucket i (backward order) holds a share R^i of the parameters, its\n"
     << "                         backward compute the same share (1 = the reference's P/nb; < 1 shrinks\n"
     << "                         the tail so the last, exposed all-reduce is small)\n"
     << "  --cp-algo ring|ulysses hybrid_cp: KV blocks around a P2P ring, or all-to-alls over heads\n"
     << "  --in-place             in-place all-reduce (halves DP buffer memory)\n"
     << "  --zero 0|1|2           dp: ZeRO stage (1: sharded optimizer + parameter all-gather, 2: + gradient\n"
     << "                         reduce-scatter instead of all-reduce)\n"
     << "  --optimizer            add an SGD-momentum step over the local gradient shard\n"
     << "  --loop [--max-loop-iters N]  run iterations forever (interference generator)\n"
     << "  --time-scale F         scale all compute durations by F\n"
     << "  --json PATH            also write the report JSON to PATH\n"
     << "  --stats-file PATH      stats file to use instead of <base>/model_stats/<model>.txt\n"
     << "  --store HOST:PORT      rendezvous store address\n"
     << "  --no-topology          do not print the topology graph\n"
     << "  --quiet                only print the report section\n"
     << "  --silent               print nothing (the report is returned to the caller)\n"
     << "  --trace                emit roctx ranges (rocprofv3 --marker-trace)\n"
     << "  --timeline PATH        device timeline of every rank (Chrome / Perfetto trace JSON, rank 0 writes it)\n"
     << "  --timeline-iters N     timed iterations kept in the timeline (default 2, 0 = all)\n"
     << "  --comm-cus N           CUs the gemm compute leaves free for collectives (default 32)\n"
     << "  --rccl-max-ctas N      RCCL blocks per collective on each comm lane (default: comm-cus / lanes;\n"
     << "                         0 = RCCL's own choice)\n"
     << "  --comm-lanes single|split  fsdp: all collectives on one ordered lane (default) or one per kind\n"
     << "  --graph                capture one iteration into a HIP graph, replay it every iteration (rccl, xgmi, mixed)\n"
     << "env: DLNB_TIMEOUT (s, hang detection), DLNB_INJECT_FAULT=rank=R,iter=I,mode=exit|hang|throw,\n"
     << "     DLNB_STORE_ADDR=host:port, DLNB_NO_ENERGY=1\n";
  return os.str();
}

Options parse_options(StrategyKind kind, int argc, const char* const* argv) {
  Options o;
  o.strategy = kind;
  if (kind == StrategyKind::Hybrid3D) o.runs = 3;  // cpp/hybrid_parallel/hybrid_3d.cpp:62
  std::vector<std::string> pos;
  std::string prog = argc > 0 ? argv[0] : strategy_name(kind);
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* what) -> std::string {
      size_t eq = a.find('=');
      if (starts_with(a, "--") && eq != std::string::npos) return a.substr(eq + 1);
      if (i + 1 >= argc) DLNB_THROW("missing value for " << what << "\n" << usage(kind, prog));
      return argv[++i];
    };
    auto is = [&](const char* s1, const char* s2 = nullptr) {
      std::string head = a.substr(0, a.find('='));
      return head == s1 || (s2 && head == s2);
    };
    if (a == "-h" || a == "--help") {
      o.help = true;
    } else if (is("-w", "--warmups") || is("--warmup")) {
      o.warmup = to_int(val("warmups"), "warmups");
    } else if (is("-r", "--runs")) {
      o.runs = to_int(val("runs"), "runs");
    } else if (is("-d", "--devices")) {
      o.devices = val("devices");
    } else if (is("-m", "--min_exectime") || is("--min-exectime")) {
      o.min_exectime = to_double(val("min_exectime"), "min_exectime");
    } else if (is("--backend")) {
      o.backend = val("backend");
    } else if (is("--ranks")) {
      o.ranks = to_int(val("ranks"), "ranks");
    } else if (is("--compute")) {
      o.compute = val("compute");
    } else if (is("--wire-dtype") || is("--dtype")) {
      o.wire_dtype = val("wire-dtype");
    } else if (is("--compute-dtype")) {
      o.compute_dtype = val("compute-dtype");
    } else if (is("--schedule")) {
      o.schedule = val("schedule");
    } else if (is("--tp-granularity")) {
      o.tp_granularity = val("tp-granularity");
    } else if (a == "--sequence-parallel") {
      o.sequence_parallel = true;
    } else if (a == "--ep-overlap") {
      o.ep_overlap = true;
    } else if (is("--ep-imbalance")) {
      o.ep_imbalance = to_double(val("ep-imbalance"), "ep-imbalance");
      if (o.ep_imbalance < 0) DLNB_THROW("--ep-imbalance must be >= 0");
    } else if (is("--pp-schedule")) {
      o.pp_schedule = val("pp-schedule");
    } else if (is("--pp-virtual")) {
      o.pp_virtual = to_int(val("pp-virtual"), "pp-virtual");
    } else if (is("--cp-algo")) {
      o.cp_algo = val("cp-algo");
    } else if (is("--dp-buckets")) {
      o.dp_buckets = to_int(val("dp-buckets"), "dp-buckets");
    } else if (is("--dp-bucket-ratio")) {
      o.dp_bucket_ratio = to_double(val("dp-bucket-ratio"), "dp-bucket-ratio");
      if (!(o.dp_bucket_ratio > 0 && o.dp_bucket_ratio <= 1)) DLNB_THROW("--dp-bucket-ratio must be in (0, 1]");
    } else if (a == "--in-place") {
      o.in_place = true;
    } else if (is("--zero")) {
      o.zero = to_int(val("zero"), "zero");
    } else if (a == "--optimizer") {
      o.optimizer = true;
    } else if (a == "--loop") {
      o.loop = true;
    } else if (is("--max-loop-iters")) {
      o.max_loop_iters = to_int(val("max-loop-iters"), "max-loop-iters");
    } else if (is("--time-scale")) {
      o.time_scale = to_double(val("time-scale"), "time-scale");
    } else if (is("--json")) {
      o.json_path = val("json");
    } else if (is("--timeline")) {
      o.timeline_path = val("timeline");
    } else if (is("--timeline-iters")) {
      o.timeline_iters = std::stoi(val("timeline-iters"));
      DLNB_REQUIRE(o.timeline_iters >= 0, "--timeline-iters must be >= 0");
    } else if (is("--stats-file")) {
      o.stats_file = val("stats-file");
    } else if (is("--store")) {
      o.store_addr = val("store");
    } else if (a == "--no-topology") {
      o.topology = false;
    } else if (is("--comm-cus")) {
      o.comm_cus = to_int(val("comm-cus"), "comm-cus");
    } else if (is("--rccl-max-ctas")) {
      o.rccl_max_ctas = to_int(val("rccl-max-ctas"), "rccl-max-ctas");
    } else if (a == "--graph") {
      o.graph = true;
    } else if (is("--comm-lanes")) {
      o.comm_lanes = val("comm-lanes");
    } else if (a == "--trace") {
      o.trace = true;
    } else if (a == "--silent") {
      o.silent = o.quiet = true;
      o.topology = false;
    } else if (a == "--quiet") {
      o.quiet = true;
      o.topology = false;
    } else if (a.size() > 1 && a[0] == '-' && !(a[1] >= '0' && a[1] <= '9')) {
      DLNB_THROW("unknown option " << a << "\n" << usage(kind, prog));
    } else {
      pos.push_back(a);
    }
  }
  if (o.help) return o;
  auto names = positional_names(kind);
  if (pos.size() != names.size()) {
    DLNB_THROW("expected " << names.size() << " positional arguments, got " << pos.size() << "\n" << usage(kind, prog));
  }
  o.model = pos[0];
  o.base_path = pos.back();
  switch (kind) {
    case StrategyKind::DP: o.num_buckets = to_int(pos[1], "num_buckets"); break;
    case StrategyKind::FSDP:
      o.num_units = to_int(pos[1], "num_units");
      o.sharding_factor = to_int(pos[2], "sharding_factor");
      break;
    case StrategyKind::Hybrid2D:
      o.num_stages = to_int(pos[1], "num_stages");
      o.num_microbatches = to_int(pos[2], "num_microbatches");
      break;
    case StrategyKind::Hybrid3D:
      o.num_stages = to_int(pos[1], "num_stages");
      o.num_microbatches = to_int(pos[2], "num_microbatches");
      o.num_tensor_shards = to_int(pos[3], "num_tensor_shards");
      break;
    case StrategyKind::Hybrid3DMoE:
      o.num_stages = to_int(pos[1], "num_stages");
      o.num_microbatches = to_int(pos[2], "num_microbatches");
      o.num_expert_shards = to_int(pos[3], "num_expert_shards");
      break;
    case StrategyKind::HybridCP:
      o.num_cp_shards = to_int(pos[1], "num_cp_shards");
      if (o.dp_buckets == 1) o.dp_buckets = 4;  // default: 4 layer buckets
      break;
    case StrategyKind::Hybrid4D:
      o.num_stages = to_int(pos[1], "num_stages");
      o.num_microbatches = to_int(pos[2], "num_microbatches");
      o.num_tensor_shards = to_int(pos[3], "num_tensor_shards");
      o.num_expert_shards = to_int(pos[4], "num_expert_shards");
      break;
  }
  DLNB_REQUIRE(o.warmup >= 0 && o.runs >= 0, "warmups and runs must be >= 0");
  DLNB_REQUIRE(o.num_buckets >= 1 && o.num_units >= 1 && o.sharding_factor >= 1 && o.num_stages >= 1 &&
                   o.num_microbatches >= 1 && o.num_tensor_shards >= 1 && o.num_expert_shards >= 1 &&
                   o.num_cp_shards >= 1,
               "parallelism degrees must be >= 1");
  DLNB_REQUIRE(o.schedule == "overlap" || o.schedule == "reference", "--schedule must be overlap or reference");
  DLNB_REQUIRE(o.pp_schedule == "gpipe" || o.pp_schedule == "1f1b" || o.pp_schedule == "interleaved" ||
                   o.pp_schedule == "dualpipe",
               "--pp-schedule must be gpipe, 1f1b, interleaved or dualpipe");
  DLNB_REQUIRE(o.tp_granularity == "microbatch" || o.tp_granularity == "layer",
               "--tp-granularity must be microbatch or layer");
  DLNB_REQUIRE(o.comm_lanes == "single" || o.comm_lanes == "split", "--comm-lanes must be single or split");
  DLNB_REQUIRE(o.dp_buckets >= 1, "--dp-buckets must be >= 1");
  DLNB_REQUIRE(o.cp_algo == "ring" || o.cp_algo == "ulysses", "--cp-algo must be ring or ulysses");
  DLNB_REQUIRE(o.zero >= 0 && o.zero <= 2, "--zero must be 0, 1 or 2 (ZeRO-3 is the fsdp strategy)");
  DLNB_REQUIRE(o.zero == 0 || kind == StrategyKind::DP, "--zero applies to dp");
  DLNB_REQUIRE(o.time_scale > 0, "--time-scale must be > 0");
  return o;
}

}  // namespace dlnb
