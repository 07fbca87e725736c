// CLI entry point 'hybrid_3d' (reference: see dlnb/options.hpp for the contract).
#include "dlnb/strategy.hpp"

int main(int argc, char** argv) { return dlnb::main_for(dlnb::StrategyKind::Hybrid3D, argc, argv); }
