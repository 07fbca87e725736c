// Round 5 probe: can each stream of an iteration be captured into its own
// linear HIP graph and the lanes be joined by device words instead of graph
// edges?
//   1. queue independence: for every ordered pair (A, B) of the streams a rank
//      uses (compute = normal priority, up to 3 comm lanes = high priority, one
//      more normal stream), a one-wave kernel on A waits for a word that a
//      kernel enqueued AFTER it on B stores. Two streams on one hardware queue
//      time out (bounded 50 ms, counted).
//   2. concurrent capture of two streams into two graphs: node / edge counts
//      (linear: edges == nodes - 1).
//   3. replay of the two lane graphs joined by iteration-tagged gates
//      (compute: 8 x 500 us spin + gate; comm: gate wait + 200 us spin + gate):
//      host time per replay vs the overlapped ideal (4.2 ms) and the serial
//      one (5.8 ms), gate timeouts.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probes/src/lane_probe.hip -o build/bin/lane_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

__global__ void set_word(uint64_t* w, uint64_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(w, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void wait_word(const uint64_t* w, uint64_t v, uint64_t timeout, uint64_t* timeouts) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != v) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        __hip_atomic_fetch_add(timeouts, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
}

// gate = {seq, time}; seq = iter << 32 | tag, iter read from *iter
__global__ void gate_raise(uint64_t* g, const uint64_t* iter, uint32_t tag) {
  if (threadIdx.x == 0) {
    const uint64_t it = __hip_atomic_load(iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(g + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(g, (it << 32) | tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void gate_wait(const uint64_t* g, const uint64_t* iter, uint32_t tag, uint64_t timeout,
                          uint64_t* timeouts) {
  if (threadIdx.x == 0) {
    const uint64_t want = (__hip_atomic_load(iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) << 32) | tag;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(g, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != want) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        __hip_atomic_fetch_add(timeouts, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
}

__global__ void set_iter(uint64_t* iter, uint64_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(iter, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void spin(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static size_t graph_edges(hipGraph_t g) {
  size_t n = 0;
  CK(hipGraphGetEdges(g, nullptr, nullptr, &n));
  return n;
}

int main() {
  CK(hipSetDevice(0));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  const char* hwq = std::getenv("GPU_MAX_HW_QUEUES");
  std::printf("priority range lo=%d hi=%d GPU_MAX_HW_QUEUES=%s\n", lo, hi, hwq ? hwq : "(unset)");
  const int NS = 5;
  hipStream_t s[NS];
  const char* names[NS] = {"compute(n)", "lane1(h)", "lane2(h)", "lane3(h)", "extra(n)"};
  for (int i = 0; i < NS; ++i)
    CK(hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, (i >= 1 && i <= 3) ? hi : lo));
  uint64_t* host = nullptr;
  CK(hipHostMalloc(&host, 64 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
  for (int i = 0; i < 64; ++i) host[i] = 0;
  int clk = 0;
  CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeWallClockRate, 0));
  const double hz = clk * 1e3;
  const uint64_t t50ms = static_cast<uint64_t>(0.05 * hz);

  // ---- 1. pairwise queue independence
  uint64_t* timeouts = host + 0;
  uint64_t seq = 0;
  int shared = 0;
  for (int a = 0; a < NS; ++a)
    for (int b = 0; b < NS; ++b) {
      if (a == b) continue;
      const uint64_t before = *timeouts;
      ++seq;
      hipLaunchKernelGGL(wait_word, 1, 64, 0, s[a], host + 1, seq, t50ms, timeouts);
      hipLaunchKernelGGL(set_word, 1, 64, 0, s[b], host + 1, seq);
      CK(hipStreamSynchronize(s[a]));
      CK(hipStreamSynchronize(s[b]));
      const bool to = *timeouts != before;
      if (to) ++shared;
      std::printf("pair wait-on %-10s signal-from %-10s : %s\n", names[a], names[b], to ? "TIMEOUT (shared queue)" : "ok");
    }
  std::printf("independence: %d of %d ordered pairs timed out\n", shared, NS * (NS - 1));

  // ---- 2. concurrent capture of two lanes
  uint64_t* dev = nullptr;  // [0] iter, [2..] gates (2 words each)
  CK(hipMalloc(&dev, 4096));
  CK(hipMemset(dev, 0, 4096));
  uint64_t* iter = dev;
  auto gate = [&](int i) { return dev + 2 + 2 * i; };
  uint64_t* gto = host + 8;
  const uint64_t t500 = static_cast<uint64_t>(500e-6 * hz), t200 = static_cast<uint64_t>(200e-6 * hz);
  const uint64_t tmo = static_cast<uint64_t>(1.0 * hz);
  hipStream_t C = s[0], M = s[1];
  CK(hipStreamBeginCapture(C, hipStreamCaptureModeThreadLocal));
  CK(hipStreamBeginCapture(M, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < 8; ++i) {
    hipLaunchKernelGGL(spin, 1, 64, 0, C, t500);
    hipLaunchKernelGGL(gate_raise, 1, 64, 0, C, gate(i), iter, 1u + i);
    hipLaunchKernelGGL(gate_wait, 1, 64, 0, M, gate(i), iter, 1u + i, tmo, gto);
    hipLaunchKernelGGL(spin, 1, 64, 0, M, t200);
  }
  hipLaunchKernelGGL(gate_raise, 1, 64, 0, M, gate(8), iter, 9u);
  hipLaunchKernelGGL(gate_wait, 1, 64, 0, C, gate(8), iter, 9u, tmo, gto);
  hipGraph_t gc = nullptr, gm = nullptr;
  CK(hipStreamEndCapture(M, &gm));
  CK(hipStreamEndCapture(C, &gc));
  size_t nc = 0, nm = 0;
  CK(hipGraphGetNodes(gc, nullptr, &nc));
  CK(hipGraphGetNodes(gm, nullptr, &nm));
  std::printf("capture: compute graph %zu nodes %zu edges, comm graph %zu nodes %zu edges\n", nc, graph_edges(gc), nm,
              graph_edges(gm));
  hipGraphExec_t ec = nullptr, em = nullptr;
  CK(hipGraphInstantiate(&ec, gc, nullptr, nullptr, 0));
  CK(hipGraphInstantiate(&em, gm, nullptr, nullptr, 0));

  // ---- 3. replays
  for (int order = 0; order < 2; ++order) {
    std::vector<double> t;
    for (int r = 0; r < 40; ++r) {
      const uint64_t it = 1000 * (order + 1) + r + 1;
      const double t0 = now();
      if (order == 0) {
        hipLaunchKernelGGL(set_iter, 1, 64, 0, C, iter, it);
        CK(hipGraphLaunch(ec, C));
        hipLaunchKernelGGL(set_iter, 1, 64, 0, M, iter, it);
        CK(hipGraphLaunch(em, M));
      } else {  // comm lane first
        hipLaunchKernelGGL(set_iter, 1, 64, 0, M, iter, it);
        CK(hipGraphLaunch(em, M));
        hipLaunchKernelGGL(set_iter, 1, 64, 0, C, iter, it);
        CK(hipGraphLaunch(ec, C));
      }
      CK(hipStreamSynchronize(C));
      CK(hipStreamSynchronize(M));
      t.push_back((now() - t0) * 1e3);
    }
    double mn = 1e9, sum = 0;
    for (size_t i = 5; i < t.size(); ++i) {
      mn = t[i] < mn ? t[i] : mn;
      sum += t[i];
    }
    std::printf("replay (%s first): mean %.3f ms min %.3f ms (overlapped ideal 4.2, serial 5.8); gate timeouts %llu\n",
                order == 0 ? "compute" : "comm", sum / (t.size() - 5), mn, (unsigned long long)*gto);
  }
  // eager (no graph) reference
  {
    std::vector<double> t;
    for (int r = 0; r < 20; ++r) {
      const uint64_t it = 5000 + r;
      const double t0 = now();
      hipLaunchKernelGGL(set_iter, 1, 64, 0, C, iter, it);
      hipLaunchKernelGGL(set_iter, 1, 64, 0, M, iter, it);
      for (int i = 0; i < 8; ++i) {
        hipLaunchKernelGGL(spin, 1, 64, 0, C, t500);
        hipLaunchKernelGGL(gate_raise, 1, 64, 0, C, gate(i), iter, 1u + i);
        hipLaunchKernelGGL(gate_wait, 1, 64, 0, M, gate(i), iter, 1u + i, tmo, gto);
        hipLaunchKernelGGL(spin, 1, 64, 0, M, t200);
      }
      hipLaunchKernelGGL(gate_raise, 1, 64, 0, M, gate(8), iter, 9u);
      hipLaunchKernelGGL(gate_wait, 1, 64, 0, C, gate(8), iter, 9u, tmo, gto);
      CK(hipStreamSynchronize(C));
      CK(hipStreamSynchronize(M));
      t.push_back((now() - t0) * 1e3);
    }
    double sum = 0;
    for (size_t i = 5; i < t.size(); ++i) sum += t[i];
    std::printf("eager: mean %.3f ms; gate timeouts %llu\n", sum / (t.size() - 5), (unsigned long long)*gto);
  }
  std::printf("done\n");
  return 0;
}
