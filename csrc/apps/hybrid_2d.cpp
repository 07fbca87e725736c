// CLI entry point 'hybrid_2d' (reference: see dlnb/options.hpp for the contract).
#include "dlnb/strategy.hpp"

int main(int argc, char** argv) { return dlnb::main_for(dlnb::StrategyKind::Hybrid2D, argc, argv); }
