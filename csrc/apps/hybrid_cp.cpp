// CLI entry point 'hybrid_cp' (DP x context parallel; see dlnb/options.hpp).
#include "dlnb/strategy.hpp"

int main(int argc, char** argv) { return dlnb::main_for(dlnb::StrategyKind::HybridCP, argc, argv); }
