// Probe: the device's s_memrealtime rate against the host's steady clock.
// Each reading pairs one stamp with the midpoint of the tightest of 20 host
// brackets (launch + hipStreamSynchronize); rate = ticks / host seconds over
// growing intervals, so the bracket error shrinks as 1/interval.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <thread>

__global__ void stamp_kernel(uint64_t* slot) {
  if (threadIdx.x == 0) __hip_atomic_store(slot, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Reading { double host_us, half_us; uint64_t tick; };

static Reading read(uint64_t* slot, hipStream_t s) {
  Reading best{0, 1e30, 0};
  for (int i = 0; i < 20; ++i) {
    (void)hipStreamSynchronize(s);
    const double h0 = now_us();
    hipLaunchKernelGGL(stamp_kernel, 1, 64, 0, s, slot);
    (void)hipStreamSynchronize(s);
    const double h1 = now_us();
    if (0.5 * (h1 - h0) < best.half_us) best = Reading{0.5 * (h0 + h1), 0.5 * (h1 - h0), __atomic_load_n(slot, __ATOMIC_ACQUIRE)};
  }
  return best;
}

int main() {
  int khz = 0;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  uint64_t* slot = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&slot), 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  hipStream_t s;
  (void)hipStreamCreate(&s);
  printf("wallclock attribute: %d kHz\n", khz);
  const Reading a = read(slot, s);
  for (double wait_s : {0.5, 1.0, 2.0, 4.0, 8.0}) {
    std::this_thread::sleep_for(std::chrono::duration<double>(wait_s));
    const Reading b = read(slot, s);
    const double host_s = (b.host_us - a.host_us) * 1e-6;
    const double hz = static_cast<double>(b.tick - a.tick) / host_s;
    const double err_ppm = (a.half_us + b.half_us) / (b.host_us - a.host_us) * 1e6;
    printf("interval %.3f s: %.3f Hz (%+.2f ppm vs %d kHz, bracket +-%.2f ppm; half-widths %.2f / %.2f us)\n", host_s, hz,
           (hz / (khz * 1e3) - 1.0) * 1e6, khz, err_ppm, a.half_us, b.half_us);
    fflush(stdout);
  }
  (void)hipHostFree(slot);
  return 0;
}
