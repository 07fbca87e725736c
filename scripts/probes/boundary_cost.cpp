// Probe: what a task boundary on the compute stream costs on MI355X.
// N deadline-GEMM (or idle) tasks of D us back to back on one stream, with
// optional per-task event record, cross-stream event wait (already
// complete) and stamp-kernel pairs. Prints host wall time per task - D.
//   build: make probes   run: build/bin/boundary_cost [gemm|sleep]
#include <chrono>
#include <cstdio>
#include <string>

#include "dlnb/compute.hpp"
#include "dlnb/device.hpp"

using namespace dlnb;

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "gemm";
  auto dev = make_gpu_device(0);
  ComputeShape shape;
  shape.hidden = 4096;
  shape.ffn = 14336;
  auto ce = make_compute_engine(*dev, parse_compute_mode(mode, DeviceKind::GPU), shape, 1.0);
  auto cs = dev->create_stream(false);
  auto other = dev->create_stream(true);
  auto done = dev->create_event();
  auto dep = dev->create_event();
  uint64_t* st = dev->alloc_stamps(4096);
  const int N = 40;
  const double D = 2000.0;
  for (int variant = 0; variant < 5; ++variant) {
    other->record(*dep);
    other->synchronize();
    cs->synchronize();
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; ++i) {
      if (variant == 2 || variant == 4) cs->wait(*dep);
      if (variant == 3 || variant == 4) dev->stamp(*cs, st + 2 * i);
      ce->run(*cs, D, 0.0);
      if (variant == 1 || variant == 4) cs->record(*done);
      if (variant == 3 || variant == 4) dev->stamp(*cs, st + 2 * i + 1);
    }
    cs->synchronize();
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    const char* names[] = {"bare", "record", "wait", "stamps", "record+wait+stamps"};
    std::printf("{\"mode\":\"%s\",\"variant\":\"%s\",\"task_us\":%.0f,\"overhead_us_per_task\":%.2f}\n", mode.c_str(),
                names[variant], D, us / N - D);
  }
  dev->free_stamps(st, 4096);
  return 0;
}
