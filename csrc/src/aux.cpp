#include "dlnb/aux.hpp"
#include "dlnb/kernels.hpp"

#include <dirent.h>
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <atomic>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <algorithm>
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
    shut_ = reinterpret_cast<int (*)()>(dlsym(lib_, "amdsmi_shut_down"));
    if (!init || !from_bdf || !energy_) return false;
    if (init(kInitAmdGpus) != 0) return false;
    inited_ = true;
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
  ~AmdSmiMeter() override {
    if (inited_ && shut_) shut_();
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
  int (*shut_)() = nullptr;
  bool inited_ = false;
  std::string bus_;
};

// hwmon sysfs: energy1_input (µJ counter) when the driver exposes it, else
// power1_average / power1_input (µW) integrated by a 5 ms sampling thread
// (the reference's POWER_SAMPLING_RATE_MS, dp.cpp:67). No library is loaded,
// so nothing interferes with the HIP runtime's teardown (amd-smi does: a
// process that initialised it aborts with a heap error at exit on ROCm 7.2).
class HwmonMeter : public EnergyMeter {
 public:
  bool init(int dev) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) return false;
    std::string b = bus;
    for (auto& c : b) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    std::string base = "/sys/bus/pci/devices/" + b + "/hwmon";
    DIR* d = opendir(base.c_str());
    if (!d) return false;
    std::string hw;
    while (dirent* e = readdir(d)) {
      if (std::string(e->d_name).rfind("hwmon", 0) == 0) hw = base + "/" + e->d_name;
    }
    closedir(d);
    if (hw.empty()) return false;
    double v;
    if (read_num(hw + "/energy1_input", v)) {
      energy_path_ = hw + "/energy1_input";
      src_ = "hwmon " + energy_path_;
    }
    for (const char* f : {"power1_average", "power1_input"}) {
      if (read_num(hw + "/" + f, v)) {
        power_path_ = hw + "/" + f;
        if (energy_path_.empty()) src_ = "hwmon " + power_path_ + " sampled every 5 ms";
        break;
      }
    }
    // sclk: hwmon freq1_input (Hz), else the device's pp_dpm_sclk (the level
    // marked '*', MHz)
    if (read_num(hw + "/freq1_input", v))
      sclk_path_ = hw + "/freq1_input";
    else if (read_dpm(std::string("/sys/bus/pci/devices/") + b + "/pp_dpm_sclk", v))
      dpm_path_ = std::string("/sys/bus/pci/devices/") + b + "/pp_dpm_sclk";
    if (energy_path_.empty() && power_path_.empty()) return false;
    stop_ = false;
    th_ = std::thread([this] { sample(); });
    return true;
  }
  bool take(Sensors& out) override {
    std::lock_guard<std::mutex> g(mu_);
    if (!have_) return false;
    out = cur_;
    cur_.sclk_min_mhz = cur_.sclk_max_mhz = cur_.sclk_mhz;  // the next window starts at the latest reading
    return true;
  }
  ~HwmonMeter() override {
    stop_ = true;
    if (th_.joinable()) th_.join();
  }
  bool available() const override { return true; }
  double joules() override {
    if (!energy_path_.empty()) {
      double v = 0;
      return read_num(energy_path_, v) ? v * 1e-6 : 0.0;
    }
    return acc_j_.load();
  }
  std::string source() const override { return src_; }

 private:
  static bool read_num(const std::string& p, double& v) {
    if (p.empty()) return false;
    FILE* f = std::fopen(p.c_str(), "r");
    if (!f) return false;
    bool ok = std::fscanf(f, "%lf", &v) == 1;
    std::fclose(f);
    return ok;
  }
  // "1: 2400Mhz *" -> 2400
  static bool read_dpm(const std::string& p, double& mhz) {
    FILE* f = std::fopen(p.c_str(), "r");
    if (!f) return false;
    char line[128];
    bool ok = false;
    while (std::fgets(line, sizeof(line), f)) {
      if (!std::strchr(line, '*')) continue;
      const char* c = std::strchr(line, ':');
      ok = c && std::sscanf(c + 1, "%lf", &mhz) == 1;
      break;
    }
    std::fclose(f);
    return ok;
  }
  bool read_sclk(double& mhz) const {
    double v;
    if (read_num(sclk_path_, v)) {
      mhz = v * 1e-6;
      return true;
    }
    return !dpm_path_.empty() && read_dpm(dpm_path_, mhz);
  }
  void sample() {
    auto last = std::chrono::steady_clock::now();
    double last_w = 0;
    double v;
    if (read_num(power_path_, v)) last_w = v * 1e-6;
    while (!stop_) {
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
      auto now = std::chrono::steady_clock::now();
      double w = last_w;
      if (read_num(power_path_, v)) w = v * 1e-6;
      double dt = std::chrono::duration<double>(now - last).count();
      if (energy_path_.empty()) acc_j_.store(acc_j_.load() + 0.5 * (w + last_w) * dt);
      last = now;
      last_w = w;
      double mhz = 0;
      const bool clk = read_sclk(mhz);
      std::lock_guard<std::mutex> g(mu_);
      cur_.power_w = w;
      if (clk) {
        if (!have_) cur_.sclk_min_mhz = cur_.sclk_max_mhz = mhz;
        cur_.sclk_mhz = mhz;
        cur_.sclk_min_mhz = std::min(cur_.sclk_min_mhz, mhz);
        cur_.sclk_max_mhz = std::max(cur_.sclk_max_mhz, mhz);
      }
      have_ = true;
    }
  }
  std::string energy_path_, power_path_, sclk_path_, dpm_path_, src_;
  std::mutex mu_;
  Sensors cur_;
  bool have_ = false;
  std::atomic<bool> stop_{true};
  std::atomic<double> acc_j_{0.0};
  std::thread th_;
};

}  // namespace

std::unique_ptr<EnergyMeter> EnergyMeter::none() { return std::unique_ptr<EnergyMeter>(new EnergyMeter()); }

std::unique_ptr<EnergyMeter> EnergyMeter::open_gpu(int device_index) {
  std::string how = env_or("DLNB_ENERGY", "hwmon");  // hwmon | amdsmi | none
  if (env_int("DLNB_NO_ENERGY", 0) || how == "none") return none();
  if (how == "amdsmi") {
    std::unique_ptr<AmdSmiMeter> m(new AmdSmiMeter());
    if (m->init(device_index)) return std::unique_ptr<EnergyMeter>(m.release());
    return none();
  }
  std::unique_ptr<HwmonMeter> h(new HwmonMeter());
  if (h->init(device_index)) return std::unique_ptr<EnergyMeter>(h.release());
  return none();
}

// ------------------------------------------------------------------ tracer

Tracer& Tracer::get() {
  static Tracer t;
  return t;
}

// Process-wide; the rank threads of a loopback job all call enable() with the
// same value, so the flag is set once and never toggled under a live range.
void Tracer::enable(bool on) {
  std::lock_guard<std::mutex> g(mu_);
  if (on && !lib_) {
    lib_ = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!lib_) lib_ = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (lib_) {
      push_ = reinterpret_cast<int (*)(const char*)>(dlsym(lib_, "roctxRangePushA"));
      pop_ = reinterpret_cast<int (*)()>(dlsym(lib_, "roctxRangePop"));
      mark_ = reinterpret_cast<void (*)(const char*)>(dlsym(lib_, "roctxMarkA"));
    }
  }
  const bool want = on && push_ && pop_;
  if (on_.load(std::memory_order_relaxed) != want) on_.store(want, std::memory_order_release);
}

void Tracer::push(const char* name) {
  if (on_.load(std::memory_order_acquire)) push_(name);
}
void Tracer::pop() {
  if (on_.load(std::memory_order_acquire)) pop_();
}
void Tracer::mark(const char* name) {
  if (on_.load(std::memory_order_acquire) && mark_) mark_(name);
}

// ---------------------------------------------------------- fault injector

FaultInjector::FaultInjector(int rank) {
  std::string spec = env_or("DLNB_INJECT_FAULT", "");
  if (spec.empty()) return;
  int r = -1;
  long long it = 0;
  long gate = 0;
  std::string mode = "exit", block;
  for (auto& kv : split(spec, ',')) {
    auto p = split(kv, '=');
    if (p.size() != 2) continue;
    if (p[0] == "rank") r = std::stoi(p[1]);
    if (p[0] == "iter") it = std::stoll(p[1]);
    if (p[0] == "mode") mode = p[1];
    if (p[0] == "block") block = p[1];
    if (p[0] == "gate") gate = std::stol(p[1]);
  }
  // block=TAG: only in the run whose DLNB_BLOCK is TAG (bench.py names each
  // of its child runs, so one phase of the bench can be made to hang)
  if (!block.empty() && env_or("DLNB_BLOCK", "") != block) return;
  if (r == rank) {
    armed_ = true;
    iter_ = it;
    mode_ = mode;
    if (mode_ == "gate") {
      // a device-side hang: the gate-th device gate signal of the run (from
      // the strategy's setup on, so inside the captured graph) is never raised
      std::fprintf(stderr, "[dlnb] DLNB_INJECT_FAULT: gate signal %ld will not be raised\n", gate);
      std::fflush(stderr);
      kernels::fail_gate_signal(gate);
    }
  }
}

void FaultInjector::at_iteration(long long iter, const std::function<void()>& enqueue_failing_task) {
  if (!armed_ || iter != iter_ || mode_ == "gate") return;
  std::fprintf(stderr, "[dlnb] DLNB_INJECT_FAULT: injecting '%s' at iteration %lld\n", mode_.c_str(), iter);
  std::fflush(stderr);
  if (mode_ == "task" && enqueue_failing_task) {
    enqueue_failing_task();
    return;
  }
  if (mode_ == "exit") std::_Exit(42);
  if (mode_ == "throw") DLNB_THROW("injected fault at iteration " << iter);
  if (mode_ == "hang")
    for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
}

}  // namespace dlnb
