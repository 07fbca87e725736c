#include "dlnb/workload.hpp"

#include <sys/stat.h>
#include <unistd.h>

#include <climits>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>

#include "dlnb/common.hpp"

namespace dlnb {

namespace {

// Canonical key for a stats line: lower-case, everything after the first
// space/paren dropped ("Average_Forward_Time (us)" -> "average_forward_time").
std::string canon_key(const std::string& k) {
  std::string out;
  for (char c : k) {
    if (c == ' ' || c == '(') break;
    out.push_back(static_cast<char>(std::tolower(static_cast<unsigned char>(c))));
  }
  return out;
}

// Order of the first 12 lines in the shipped layout (cpp/utils.hpp:211-253).
const char* kShippedOrder[] = {"forward_flops",          "backward_flops",           "model_size",
                               "non_expert_size",        "average_forward_time",     "average_backward_time",
                               "batch_size",             "ffn_average_forward_time", "ffn_average_backward_time",
                               "experts",                "seq_len",                  "embedded_dim"};

double to_d(const std::string& v, const std::string& key, const std::string& origin) {
  char* end = nullptr;
  double r = std::strtod(v.c_str(), &end);
  if (end == v.c_str()) DLNB_THROW("stats " << origin << ": bad numeric value for " << key << ": '" << v << "'");
  return r;
}

uint64_t to_u(const std::string& v, const std::string& key, const std::string& origin) {
  double d = to_d(v, key, origin);
  if (d < 0) DLNB_THROW("stats " << origin << ": negative value for " << key);
  // Integers in the files can exceed 2^53 only for FLOP counts, which are
  // kept as doubles; parameter counts fit exactly.
  char* end = nullptr;
  unsigned long long u = std::strtoull(v.c_str(), &end, 10);
  if (end != v.c_str() && (*end == '\0' || *end == '.')) return u;
  return static_cast<uint64_t>(d);
}

}  // namespace

ModelStats parse_model_stats_text(const std::string& text, const std::string& origin) {
  std::map<std::string, std::string> kv;
  std::istringstream is(text);
  std::string line;
  int idx = 0;
  while (std::getline(is, line)) {
    line = trim(line);
    if (line.empty() || line[0] == '#') continue;
    size_t colon = line.find(':');
    if (colon == std::string::npos) DLNB_THROW("stats " << origin << ": line without ':' : " << line);
    std::string key = canon_key(trim(line.substr(0, colon)));
    std::string val = trim(line.substr(colon + 1));
    if (key.empty() && idx < 12) key = kShippedOrder[idx];
    kv[key] = val;
    ++idx;
  }
  ModelStats s;
  s.path = origin;
  auto need = [&](const char* k) -> const std::string& {
    auto it = kv.find(k);
    if (it == kv.end()) DLNB_THROW("stats " << origin << ": missing key " << k);
    return it->second;
  };
  auto opt = [&](const char* k) -> const std::string* {
    auto it = kv.find(k);
    return it == kv.end() ? nullptr : &it->second;
  };
  s.forward_flops = to_d(need("forward_flops"), "Forward_Flops", origin);
  s.backward_flops = to_d(need("backward_flops"), "Backward_Flops", origin);
  s.model_size = to_u(need("model_size"), "Model_Size", origin);
  s.avg_forward_time_us = to_d(need("average_forward_time"), "Average_Forward_Time", origin);
  s.avg_backward_time_us = to_d(need("average_backward_time"), "Average_Backward_Time", origin);
  s.batch_size = to_u(need("batch_size"), "Batch_size", origin);
  if (auto v = opt("ffn_average_forward_time")) s.ffn_avg_forward_time_us = to_d(*v, "FFN_fwd", origin);
  if (auto v = opt("ffn_average_backward_time")) s.ffn_avg_backward_time_us = to_d(*v, "FFN_bwd", origin);
  if (auto v = opt("experts")) s.experts = to_u(*v, "Experts", origin);
  s.seq_len = to_u(need("seq_len"), "Seq_len", origin);
  s.embedded_dim = to_u(need("embedded_dim"), "Embedded_dim", origin);
  if (auto v = opt("device")) s.device = *v;
  if (auto v = opt("dtype")) s.dtype = *v;
  if (auto v = opt("bytes_per_element")) s.bytes_per_element = to_d(*v, "Bytes_per_element", origin);
  if (auto v = opt("num_layers")) s.num_layers = to_u(*v, "Num_layers", origin);
  if (auto v = opt("ffn_dim")) s.ffn_dim = to_u(*v, "FFN_dim", origin);
  if (auto v = opt("top_k")) s.top_k = to_u(*v, "Top_k", origin);
  if (auto v = opt("non_expert_size")) {
    s.non_expert_size = to_u(*v, "Non_Expert_size", origin);
    s.format = opt("generator") ? "dlnb" : "shipped";
  } else {
    // python/model_stats.py layout: Model_Size holds the non-expert count.
    s.format = "generator";
    s.non_expert_size = s.experts > 1 ? s.model_size : 0;
  }
  if (s.batch_size == 0) DLNB_THROW("stats " << origin << ": Batch_size must be > 0");
  if (s.experts == 0) s.experts = 1;
  return s;
}

ModelStats parse_model_stats(const std::string& path) {
  std::ifstream f(path);
  if (!f) DLNB_THROW("model stats file does not exist: " << path);
  std::stringstream ss;
  ss << f.rdbuf();
  return parse_model_stats_text(ss.str(), path);
}

Json ModelStats::to_json() const {
  Json j = Json::object();
  j["path"] = path;
  j["format"] = format;
  j["forward_flops"] = forward_flops;
  j["backward_flops"] = backward_flops;
  j["model_size"] = model_size;
  j["non_expert_size"] = non_expert_size;
  j["avg_forward_time_us"] = avg_forward_time_us;
  j["avg_backward_time_us"] = avg_backward_time_us;
  j["batch_size"] = batch_size;
  j["experts"] = experts;
  j["seq_len"] = seq_len;
  j["embedded_dim"] = embedded_dim;
  j["device"] = device;
  j["dtype"] = dtype;
  return j;
}

ModelArch parse_model_arch(const std::string& path) {
  ModelArch a;
  a.path = path;
  a.raw = read_json_file(path);
  auto geti = [&](const char* k, uint64_t d) -> uint64_t {
    return a.raw.contains(k) && a.raw.at(k).is_number() ? static_cast<uint64_t>(a.raw.at(k).as_int()) : d;
  };
  a.num_layers = geti("num_encoder_blocks", 0) + geti("num_decoder_blocks", 0);
  a.embed_dim = geti("embed_dim", 0);
  a.ff_dim = geti("ff_dim", 0);
  a.num_heads = geti("num_heads", 0);
  a.seq_len = geti("seq_len", 0);
  if (a.raw.contains("moe_params") && a.raw.at("moe_params").is_object()) {
    const Json& m = a.raw.at("moe_params");
    if (m.contains("num_experts")) a.num_experts = static_cast<uint64_t>(m.at("num_experts").as_int());
    if (m.contains("num_experts_per_tok")) a.experts_per_tok = static_cast<uint64_t>(m.at("num_experts_per_tok").as_int());
  }
  return a;
}

std::string model_base_name(const std::string& name) {
  size_t last = name.rfind('_');
  if (last == std::string::npos || last == 0) return name;
  size_t second = name.rfind('_', last - 1);
  if (second == std::string::npos) return name;
  return name.substr(0, second);
}

std::string resolve_base_path(const std::string& base) {
  std::string p = base;
  if (p.empty()) p = ".";
  if (p[0] != '/') {
    char buf[PATH_MAX];
    if (!getcwd(buf, sizeof(buf))) DLNB_THROW("getcwd failed");
    p = std::string(buf) + "/" + p;
  }
  struct stat st;
  if (stat(p.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) DLNB_THROW("base path is not a directory: " << p);
  return p;
}

std::string stats_path_for(const std::string& base, const std::string& model) {
  return resolve_base_path(base) + "/model_stats/" + model + ".txt";
}

std::string arch_path_for(const std::string& base, const std::string& model) {
  return resolve_base_path(base) + "/models/" + model_base_name(model) + ".json";
}

}  // namespace dlnb
