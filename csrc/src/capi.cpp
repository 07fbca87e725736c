// C ABI for the Python package (loaded with ctypes from
// dlnetbench_amd/_lib/libdlnb.so). Every function returns 0 on success and a
// non-zero code on failure; dlnb_last_error() describes the failure.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dlnb/compute.hpp"
#include "dlnb/kernels.hpp"
#include "dlnb/strategy.hpp"
#include "dlnb/workload.hpp"

namespace {
thread_local std::string g_err;

char* dup(const std::string& s) {
  char* p = static_cast<char*>(std::malloc(s.size() + 1));
  std::memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

template <typename F>
int guard(F f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return 1;
  }
}
}  // namespace

extern "C" {

const char* dlnb_version() { return "dlnetbench_amd 0.1.0 (gfx950)"; }

const char* dlnb_last_error() { return g_err.c_str(); }

void dlnb_free(char* p) { std::free(p); }

int dlnb_gpu_count() { return dlnb::gpu_device_count(); }

// Runs a benchmark; *out receives the report JSON (malloc'd, free with
// dlnb_free). argv does not include a program name.
int dlnb_run(const char* strategy, int argc, const char** argv, char** out) {
  return guard([&] {
    dlnb::StrategyKind k = dlnb::parse_strategy(strategy);
    std::vector<const char*> av;
    av.push_back(strategy);
    for (int i = 0; i < argc; ++i) av.push_back(argv[i]);
    dlnb::Options o = dlnb::parse_options(k, static_cast<int>(av.size()), av.data());
    dlnb::Json doc = dlnb::run_benchmark(o);
    if (out) *out = dup(doc.dump());
  });
}

int dlnb_parse_stats(const char* path, char** out) {
  return guard([&] {
    dlnb::ModelStats s = dlnb::parse_model_stats(path);
    if (out) *out = dup(s.to_json().dump());
  });
}

int dlnb_fill_random(void* p, size_t n, int dtype, unsigned long long seed, void* stream) {
  return guard([&] { dlnb::kernels::fill_random(p, n, static_cast<dlnb::DType>(dtype), seed, stream); });
}

int dlnb_gemm_tn(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, int dtype,
                 void* stream) {
  return guard([&] {
    dlnb::kernels::gemm_tn(A, B, C, M, N, K, lda, ldb, ldc, static_cast<dlnb::DType>(dtype), stream);
  });
}

int dlnb_gemm_tn_waves(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, int dtype,
                       int waves, void* stream) {
  return guard([&] {
    dlnb::kernels::gemm_tn(A, B, C, M, N, K, lda, ldb, ldc, static_cast<dlnb::DType>(dtype), stream, waves);
  });
}

int dlnb_gemm_deadline_us(const void* A, const void* B, void* C, int M, int N, int K, int dtype, double us,
                          int device, void* stamp_slot, int grid, void* stream) {
  static uint32_t epoch = 0;
  return guard([&] {
    epoch = epoch % 65535 + 1;
    double hz = dlnb::kernels::wallclock_hz(device);
    if (grid <= 0) grid = dlnb::kernels::num_cus(device);
    dlnb::kernels::gemm_tn_deadline(A, B, C, M, N, K, static_cast<dlnb::DType>(dtype),
                                    static_cast<unsigned long long>(us * 1e-6 * hz), static_cast<uint64_t*>(stamp_slot),
                                    epoch, grid, stream);
  });
}

// The deadline GEMM with the full start protocol (csrc/kernels/deadline_sync.hpp):
// explicit epoch, chain (> 0: continue the slot's previous deadline absorbing at
// most chain_us of lateness), up to two gates (iteration 0) with their tags, a
// start stamp, the DlCounter words (optional, kernels::kNumCounters int64).
int dlnb_gemm_deadline_ex(const void* A, const void* B, void* C, int M, int N, int K, int dtype, double us, int device,
                          void* slot, int grid, void* stream, unsigned epoch, double chain_us, void* gate0, unsigned tag0,
                          void* gate1, unsigned tag1, void* tstart, void* counters) {
  return guard([&] {
    double hz = dlnb::kernels::wallclock_hz(device);
    if (grid <= 0) grid = dlnb::kernels::num_cus(device);
    dlnb::kernels::DlSync sync;
    sync.chain = chain_us > 0 ? static_cast<uint32_t>(std::max(1.0, chain_us * 1e-6 * hz + 0.5)) : 0u;
    sync.gate[0] = static_cast<const uint64_t*>(gate0);
    sync.gate[1] = static_cast<const uint64_t*>(gate1);
    sync.tag[0] = tag0;
    sync.tag[1] = tag1;
    sync.tstart[0] = static_cast<uint64_t*>(tstart);
    sync.counters = static_cast<uint64_t*>(counters);
    dlnb::kernels::gemm_tn_deadline(A, B, C, M, N, K, static_cast<dlnb::DType>(dtype),
                                    static_cast<unsigned long long>(us * 1e-6 * hz), static_cast<uint64_t*>(slot),
                                    epoch, grid, stream, 0, sync);
  });
}

// Raise a two-word gate {seq = tag (iteration 0), time} when the stream gets here.
int dlnb_gate_signal(void* gate, unsigned tag, void* stream) {
  return guard([&] { dlnb::kernels::gate_signal(static_cast<uint64_t*>(gate), nullptr, tag, stream); });
}

// The same with the sequence's iteration read from *iter (device word) when the kernel runs.
int dlnb_gate_signal_iter(void* gate, const void* iter, unsigned tag, void* stream) {
  return guard([&] {
    dlnb::kernels::gate_signal(static_cast<uint64_t*>(gate), static_cast<const uint64_t*>(iter), tag, stream);
  });
}

// One task of a compute program (kernels::DlTask) as the tests describe it:
// ticks > 0 a deadline task; ticks == 0 with work a fixed-work task; neither
// the join.
struct dlnb_task_desc {
  unsigned long long ticks;
  unsigned long long chain_ticks;
  void* gate0;
  void* gate1;
  unsigned tag0, tag1;
  void* tstart0;
  void* tstart1;
  void* done_gate;
  unsigned done_tag;
  unsigned work_rounds;
  unsigned tail_kt;
  unsigned epoch;  // index among the program's tasks
  void* tend;
  unsigned flags;  // kernels::kTaskGateOnly: a gate-only task
};

int dlnb_task_size() { return static_cast<int>(sizeof(dlnb::kernels::DlTask)); }

// A compute program (kernels::gemm_tn_deadline_program) of n described tasks:
// the list is copied into task_buf (device memory, >= n * dlnb_task_size()
// bytes) once the stream is idle, then the program is launched on the stream.
// iter / counters / abort: the device iteration word, the DlCounter words,
// the host-mapped abort word (each optional). epoch: 0 = program claims from
// the iteration word; else a one-task launch epoch.
int dlnb_gemm_program(const void* A, const void* B, void* C, int M, int N, int K, int dtype, const dlnb_task_desc* d,
                      int n, const void* iter, void* counters, const void* abort, double gate_timeout_s, int device,
                      void* slot, void* task_buf, int grid, void* stream, unsigned epoch) {
  return guard([&] {
    DLNB_REQUIRE(n > 0 && d && task_buf && slot, "dlnb_gemm_program: bad arguments");
    if (grid <= 0) grid = dlnb::kernels::num_cus(device);
    const double hz = dlnb::kernels::wallclock_hz_nominal(device);
    std::vector<dlnb::kernels::DlTask> ts(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) {
      dlnb::kernels::DlTask& t = ts[static_cast<size_t>(i)];
      t.ticks = d[i].ticks;
      t.epoch = d[i].epoch;
      t.work_rounds = d[i].work_rounds;
      t.tail_kt = d[i].tail_kt;
      t.flags = d[i].flags;
      t.tend = static_cast<uint64_t*>(d[i].tend);
      t.sync.chain = static_cast<uint32_t>(d[i].chain_ticks);
      t.sync.gate[0] = static_cast<const uint64_t*>(d[i].gate0);
      t.sync.gate[1] = static_cast<const uint64_t*>(d[i].gate1);
      t.sync.tag[0] = d[i].tag0;
      t.sync.tag[1] = d[i].tag1;
      t.sync.tstart[0] = static_cast<uint64_t*>(d[i].tstart0);
      t.sync.tstart[1] = static_cast<uint64_t*>(d[i].tstart1);
      t.sync.done_gate = static_cast<uint64_t*>(d[i].done_gate);
      t.sync.done_tag = d[i].done_tag;
      t.sync.iter = static_cast<const uint64_t*>(iter);
      t.sync.counters = static_cast<uint64_t*>(counters);
      t.sync.abort = static_cast<const uint64_t*>(abort);
      t.sync.gate_timeout = static_cast<uint64_t>(gate_timeout_s * hz);
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (hipStreamSynchronize(st) != hipSuccess) DLNB_THROW("dlnb_gemm_program: stream synchronize failed");
    if (hipMemcpy(task_buf, ts.data(), ts.size() * sizeof(dlnb::kernels::DlTask), hipMemcpyHostToDevice) != hipSuccess)
      DLNB_THROW("dlnb_gemm_program: task list copy failed");
    dlnb::kernels::gemm_tn_deadline_program(A, B, C, M, N, K, static_cast<dlnb::DType>(dtype),
                                            static_cast<const dlnb::kernels::DlTask*>(task_buf), n,
                                            static_cast<uint64_t*>(slot), grid, stream, epoch);
  });
}

int dlnb_program_ktiles(int M, int N, int K, int dtype) {
  return dlnb::kernels::program_ktiles(M, N, K, static_cast<dlnb::DType>(dtype));
}

// Host-mapped, device-visible words (an abort word for the tests): the host
// pointer (the device pointer is returned in *dev).
void* dlnb_host_words(int n, void** dev) {
  void* p = nullptr;
  if (hipHostMalloc(&p, static_cast<size_t>(n) * 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return nullptr;
  std::memset(p, 0, static_cast<size_t>(n) * 8);
  if (dev && hipHostGetDevicePointer(dev, p, 0) != hipSuccess) *dev = p;
  return p;
}
void dlnb_host_words_free(void* p) { (void)hipHostFree(p); }

int dlnb_gemm_narrow_nf(int M, int N, int cus) { return dlnb::kernels::gemm_narrow_nf(M, N, cus); }

int dlnb_gemm_shape_ok(int M, int N, int K, int dtype) {
  return dlnb::kernels::gemm_shape_ok(M, N, K, static_cast<dlnb::DType>(dtype)) ? 1 : 0;
}

int dlnb_idle_wait_us(double us, int device, void* stream) {
  return guard([&] {
    double hz = dlnb::kernels::wallclock_hz(device);
    dlnb::kernels::idle_wait(static_cast<unsigned long long>(us * 1e-6 * hz), stream);
  });
}

int dlnb_busy_spin_us(double us, int device, void* stream) {
  return guard([&] {
    double hz = dlnb::kernels::wallclock_hz(device);
    dlnb::kernels::busy_spin(static_cast<unsigned long long>(us * 1e-6 * hz), dlnb::kernels::num_cus(device), stream);
  });
}

int dlnb_sgd_momentum_bf16(void* p, void* m, const void* g, size_t n, float lr, float beta, void* stream) {
  return guard([&] { dlnb::kernels::sgd_momentum_bf16(p, m, g, n, lr, beta, stream); });
}

double dlnb_wallclock_hz(int device) { return dlnb::kernels::wallclock_hz(device); }

// One wave writes s_memrealtime into *slot when the stream reaches this point.
int dlnb_stamp(void* slot, void* stream) {
  return guard([&] { dlnb::kernels::stamp(static_cast<uint64_t*>(slot), stream); });
}

// Host conversions exposed for tests (OCP fp8 / bf16 rounding parity).
float dlnb_bf16_to_float(unsigned short v) { return dlnb::bf16_to_float(v); }
unsigned short dlnb_float_to_bf16(float f) { return dlnb::float_to_bf16(f); }
float dlnb_fp8e4m3_to_float(unsigned char v) { return dlnb::fp8e4m3_to_float(v); }
unsigned char dlnb_float_to_fp8e4m3(float f) { return dlnb::float_to_fp8e4m3(f); }

}  // extern "C"
