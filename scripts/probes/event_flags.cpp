// Probe: which hipEventCreate* variants succeed on this runtime (GPU box).
#include <hip/hip_runtime.h>
#include <cstdio>
int main() {
  int v = 0; hipRuntimeGetVersion(&v); printf("runtime %d\n", v);
  hipSetDevice(0);
  struct { const char* n; unsigned f; } cases[] = {
    {"Default", hipEventDefault}, {"DisableTiming", hipEventDisableTiming},
    {"DisableSystemFence", hipEventDisableSystemFence},
    {"DisableTiming|DisableSystemFence", hipEventDisableTiming | hipEventDisableSystemFence},
    {"ReleaseToDevice", hipEventReleaseToDevice},
    {"DisableTiming|ReleaseToDevice", hipEventDisableTiming | hipEventReleaseToDevice},
    {"Default again", hipEventDefault}};
  hipEvent_t e;
  printf("hipEventCreate: %s\n", hipGetErrorString(hipEventCreate(&e)));
  for (auto& c : cases) {
    hipError_t r = hipEventCreateWithFlags(&e, c.f);
    printf("%-36s 0x%08x -> %s\n", c.n, c.f, hipGetErrorString(r));
    (void)hipGetLastError();
  }
  return 0;
}
