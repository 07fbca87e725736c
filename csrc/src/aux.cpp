#include "dlnb/aux.hpp"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include "dlnb/common.hpp"

namespace dlnb {

// ------------------------------------------------------------ energy meter

namespace {

// Minimal mirror of the amd-smi ABI used here (amd_smi/amdsmi.h).
typedef void* smi_handle;
typedef union {
  struct {
    uint64_t function_number : 3;
    uint64_t device_number : 5;
    uint64_t bus_number : 8;
    uint64_t domain_number : 48;
  } f;
  uint64_t as_uint;
} smi_bdf;
typedef int (*smi_init_t)(uint64_t);
typedef int (*smi_from_bdf_t)(smi_bdf, smi_handle*);
typedef int (*smi_energy_t)(smi_handle, uint64_t*, float*, uint64_t*);
constexpr uint64_t kInitAmdGpus = 1u << 1;

class AmdSmiMeter : public EnergyMeter {
 public:
  bool init(int dev) {
    lib_ = dlopen("libamd_smi.so", RTLD_NOW | RTLD_LOCAL);
    if (!lib_) lib_ = dlopen("/opt/rocm/lib/libamd_smi.so", RTLD_NOW | RTLD_LOCAL);
    if (!lib_) return false;
    auto init = reinterpret_cast<smi_init_t>(dlsym(lib_, "amdsmi_init"));
    auto from_bdf = reinterpret_cast<smi_from_bdf_t>(dlsym(lib_, "amdsmi_get_processor_handle_from_bdf"));
    energy_ = reinterpret_cast<smi_energy_t>(dlsym(lib_, "amdsmi_get_energy_count"));
    if (!init || !from_bdf || !energy_) return false;
    if (init(kInitAmdGpus) != 0) return false;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) return false;
    unsigned dom = 0, b = 0, d = 0, fn = 0;
    if (std::sscanf(bus, "%x:%x:%x.%x", &dom, &b, &d, &fn) != 4) return false;
    smi_bdf bdf;
    bdf.as_uint = 0;
    bdf.f.domain_number = dom;
    bdf.f.bus_number = b;
    bdf.f.device_number = d;
    bdf.f.function_number = fn;
    if (from_bdf(bdf, &h_) != 0) return false;
    uint64_t acc = 0, ts = 0;
    float res = 0;
    if (energy_(h_, &acc, &res, &ts) != 0 || res <= 0) return false;
    bus_ = bus;
    return true;
  }
  bool available() const override { return true; }
  double joules() override {
    uint64_t acc = 0, ts = 0;
    float res = 0;
    if (energy_(h_, &acc, &res, &ts) != 0) return 0.0;
    return static_cast<double>(acc) * res * 1e-6;  // resolution is in µJ
  }
  std::string source() const override { return "amd-smi energy counter (" + bus_ + ")"; }

 private:
  void* lib_ = nullptr;
  smi_handle h_ = nullptr;
  smi_energy_t energy_ = nullptr;
  std::string bus_;
};

}  // namespace

std::unique_ptr<EnergyMeter> EnergyMeter::none() { return std::unique_ptr<EnergyMeter>(new EnergyMeter()); }

std::unique_ptr<EnergyMeter> EnergyMeter::open_gpu(int device_index) {
  if (env_int("DLNB_NO_ENERGY", 0)) return none();
  std::unique_ptr<AmdSmiMeter> m(new AmdSmiMeter());
  if (m->init(device_index)) return std::unique_ptr<EnergyMeter>(m.release());
  return none();
}

// ------------------------------------------------------------------ tracer

Tracer& Tracer::get() {
  static Tracer t;
  return t;
}

void Tracer::enable(bool on) {
  on_ = false;
  if (!on) return;
  if (!lib_) {
    lib_ = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!lib_) lib_ = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!lib_) return;
    push_ = reinterpret_cast<int (*)(const char*)>(dlsym(lib_, "roctxRangePushA"));
    pop_ = reinterpret_cast<int (*)()>(dlsym(lib_, "roctxRangePop"));
    mark_ = reinterpret_cast<void (*)(const char*)>(dlsym(lib_, "roctxMarkA"));
  }
  on_ = push_ && pop_;
}

void Tracer::push(const char* name) {
  if (on_) push_(name);
}
void Tracer::pop() {
  if (on_) pop_();
}
void Tracer::mark(const char* name) {
  if (on_ && mark_) mark_(name);
}

// ---------------------------------------------------------- fault injector

FaultInjector::FaultInjector(int rank) {
  std::string spec = env_or("DLNB_INJECT_FAULT", "");
  if (spec.empty()) return;
  int r = -1;
  long long it = 0;
  std::string mode = "exit";
  for (auto& kv : split(spec, ',')) {
    auto p = split(kv, '=');
    if (p.size() != 2) continue;
    if (p[0] == "rank") r = std::stoi(p[1]);
    if (p[0] == "iter") it = std::stoll(p[1]);
    if (p[0] == "mode") mode = p[1];
  }
  if (r == rank) {
    armed_ = true;
    iter_ = it;
    mode_ = mode;
  }
}

void FaultInjector::at_iteration(long long iter) {
  if (!armed_ || iter != iter_) return;
  std::fprintf(stderr, "[dlnb] DLNB_INJECT_FAULT: injecting '%s' at iteration %lld\n", mode_.c_str(), iter);
  std::fflush(stderr);
  if (mode_ == "exit") std::_Exit(42);
  if (mode_ == "throw") DLNB_THROW("injected fault at iteration " << iter);
  if (mode_ == "hang")
    for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
}

}  // namespace dlnb
