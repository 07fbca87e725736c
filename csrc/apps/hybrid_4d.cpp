// CLI entry point 'hybrid_4d' (DP x PP x TP x EP; see dlnb/options.hpp).
#include "dlnb/strategy.hpp"

int main(int argc, char** argv) { return dlnb::main_for(dlnb::StrategyKind::Hybrid4D, argc, argv); }
