// Unified entry point: dlnb <dp|fsdp|hybrid_2d|hybrid_3d|hybrid_3d_moe> <args...>
//                      dlnb commtest [options]   (collective check / bandwidth)
#include <iostream>
#include <string>

#include "dlnb/strategy.hpp"

int main(int argc, char** argv) {
  if (argc < 2 || std::string(argv[1]) == "-h" || std::string(argv[1]) == "--help") {
    std::cout << "Usage: dlnb <dp|fsdp|hybrid_2d|hybrid_3d|hybrid_3d_moe> <args...>  (dlnb <strategy> -h for details)\n"
                 "       dlnb commtest [--backend B] [--bench] ...   (dlnb commtest -h)\n"
                 "       dlnb info    (HIP / RCCL runtime and xgmi kernel occupancy, one JSON line)\n";
    return argc < 2 ? 1 : 0;
  }
  if (std::string(argv[1]) == "info") {
    try {
      return dlnb::info_main(argc - 1, argv + 1);
    } catch (const std::exception& e) {
      std::cerr << "[dlnb] info error: " << e.what() << std::endl;
      return 2;
    }
  }
  if (std::string(argv[1]) == "commtest") {
    try {
      return dlnb::commtest_main(argc - 1, argv + 1);
    } catch (const std::exception& e) {
      std::cerr << "[dlnb] commtest error: " << e.what() << std::endl;
      return 2;
    }
  }
  dlnb::StrategyKind k;
  try {
    k = dlnb::parse_strategy(argv[1]);
  } catch (const std::exception& e) {
    std::cerr << e.what() << std::endl;
    return 1;
  }
  return dlnb::main_for(k, argc - 1, argv + 1);
}
