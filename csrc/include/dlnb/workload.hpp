// Workload description: model_stats/*.txt tables and models/*.json
// architecture files.
//
// Reference behaviour:
//   * cpp/utils.hpp:200-269 reads the stats file *positionally* (lines 1-12,
//     keys ignored) and truncates the µs times to integers (:228-232).
//   * python/model_stats.py:148-166 writes a *different* layout (no
//     Non_Expert_size line), and the archived A100 set
//     (model_stats/tmp_folder.tar.gz) uses that older order too.
//   * cpp/utils.hpp:279-294 counts layers as num_encoder_blocks +
//     num_decoder_blocks; hybrid drivers find models/<base>.json by stripping
//     the last two '_' fields of the model name (hybrid_2d.cpp:214-216).
// This implementation parses by KEY (falling back to the shipped positional
// order for unknown keys), accepts all three layouts, and keeps the times as
// doubles (deviation #13 in SURVEY.md §7.5).
#pragma once

#include <cstdint>
#include <string>

#include "dlnb/json.hpp"

namespace dlnb {

struct ModelStats {
  std::string path;
  std::string format;  // "shipped" (15 keys incl. Non_Expert_size) | "generator" | "dlnb"
  double forward_flops = 0;
  double backward_flops = 0;
  uint64_t model_size = 0;       // parameters
  uint64_t non_expert_size = 0;  // parameters outside expert MLPs (0 = dense)
  double avg_forward_time_us = 0;
  double avg_backward_time_us = 0;
  uint64_t batch_size = 0;
  double ffn_avg_forward_time_us = 0;
  double ffn_avg_backward_time_us = 0;
  uint64_t experts = 1;
  uint64_t seq_len = 0;
  uint64_t embedded_dim = 0;
  std::string device;
  std::string dtype;  // compute dtype the times were derived for ("bfloat16", "float8", ...)
  double bytes_per_element = 2.0;
  // dlnb extensions (optional trailing keys written by our generator).
  uint64_t num_layers = 0;
  uint64_t ffn_dim = 0;
  uint64_t top_k = 0;

  Json to_json() const;
};

ModelStats parse_model_stats(const std::string& path);
ModelStats parse_model_stats_text(const std::string& text, const std::string& origin = "<text>");

struct ModelArch {
  std::string path;
  uint64_t num_layers = 0;  // num_encoder_blocks + num_decoder_blocks
  uint64_t embed_dim = 0;
  uint64_t ff_dim = 0;
  uint64_t num_heads = 0;
  uint64_t seq_len = 0;
  uint64_t num_experts = 1;
  uint64_t experts_per_tok = 1;
  Json raw;
};

ModelArch parse_model_arch(const std::string& path);

// "llama3_70b_16_bfloat16" -> "llama3_70b" (strip the batch and dtype fields).
std::string model_base_name(const std::string& stats_name);

// Resolve <base>/model_stats/<model>.txt and <base>/models/<model_base>.json.
// `base` is taken relative to the current directory unless absolute
// (cpp/utils.hpp:44-59 get_dnnproxy_base_path); it must be a directory.
std::string resolve_base_path(const std::string& base);
std::string stats_path_for(const std::string& base, const std::string& model);
std::string arch_path_for(const std::string& base, const std::string& model);

}  // namespace dlnb
