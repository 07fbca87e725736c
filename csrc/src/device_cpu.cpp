#include <sys/mman.h>
#include <time.h>
#include <fcntl.h>
#include <sys/syscall.h>
#include <cerrno>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <map>
#include <mutex>
#include <set>
#include <string>

#include "dlnb/device.hpp"

namespace dlnb {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void precise_sleep_us(double us) {
  if (us <= 0) return;
  double t_end = now_s() + us * 1e-6;
  // Sleep for all but the last ~100 µs, then spin: usleep() alone overshoots
  // by 50-100 µs on a loaded host, which the reference silently absorbs
  // into its compute time (cpp/data_parallel/dp.cpp:93,98).
  double coarse = us * 1e-6 - 1e-4;
  if (coarse > 0) {
    timespec ts;
    ts.tv_sec = static_cast<time_t>(coarse);
    ts.tv_nsec = static_cast<long>((coarse - static_cast<double>(ts.tv_sec)) * 1e9);
    while (nanosleep(&ts, &ts) != 0) {
    }
  }
  while (now_s() < t_end) {
  }
}

// ------------------------------------------------------------------ Buffer

Buffer::Buffer(Device* dev, size_t bytes, bool peer) : dev_(dev), bytes_(bytes) {
  ptr_ = bytes ? (peer ? dev->raw_alloc_peer(bytes) : dev->raw_alloc(bytes)) : nullptr;
}

Buffer::~Buffer() {
  if (ptr_ && dev_) dev_->raw_free(ptr_, bytes_);
}

Buffer& Buffer::operator=(Buffer&& o) noexcept {
  if (this != &o) {
    if (ptr_ && dev_) dev_->raw_free(ptr_, bytes_);
    dev_ = o.dev_;
    ptr_ = o.ptr_;
    bytes_ = o.bytes_;
    o.ptr_ = nullptr;
    o.bytes_ = 0;
  }
  return *this;
}

// ---------------------------------------------------------------- CpuEvent

uint64_t CpuEvent::mark_recorded() {
  std::lock_guard<std::mutex> g(mu_);
  return ++recorded_;
}

uint64_t CpuEvent::recorded() {
  std::lock_guard<std::mutex> g(mu_);
  return recorded_;
}

void CpuEvent::complete(uint64_t gen) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (gen > completed_) {
      completed_ = gen;
      t_ = now_s();
    }
  }
  cv_.notify_all();
}

void CpuEvent::wait_for(uint64_t gen) {
  std::unique_lock<std::mutex> g(mu_);
  while (!cv_.wait_for(g, std::chrono::milliseconds(20), [&] { return completed_ >= gen; }))
    if (abort_ && abort_->load()) return;
}

double CpuEvent::time_s() {
  wait_for(recorded());
  std::lock_guard<std::mutex> g(mu_);
  return t_;
}

// --------------------------------------------------------------- CpuStream

struct CpuStreamRegistry {
  std::mutex mu;
  std::set<CpuStream*> live;
};

CpuStream::CpuStream(AbortFlag abort, std::shared_ptr<CpuStreamRegistry> reg)
    : abort_(std::move(abort)), reg_(std::move(reg)), th_([this] { run(); }) {
  if (reg_) {
    std::lock_guard<std::mutex> g(reg_->mu);
    reg_->live.insert(this);
  }
}

CpuStream::~CpuStream() {
  if (reg_) {
    std::lock_guard<std::mutex> g(reg_->mu);
    reg_->live.erase(this);
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  th_.join();
}

void CpuStream::enqueue(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(fn));
    ++inflight_;
  }
  cv_.notify_all();
}

void CpuStream::run() {
  for (;;) {
    std::function<void()> fn;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;
      fn = std::move(q_.front());
      q_.pop_front();
    }
    try {
      if (!abort_ || !abort_->load()) fn();
    } catch (const std::exception& e) {
      // A failed task would leave peers and other streams waiting forever.
      // A CLI rank ends loudly (the launcher tears the job down); in a library
      // host (Python) the device's abort switch drains every stream (later
      // tasks are skipped, event waits return) and synchronize() throws the
      // error to the caller, which can run another job afterwards.
      std::fprintf(stderr, "[dlnb] fatal error on CPU stream: %s\n", e.what());
      std::fflush(stderr);
      if (cli_process()) std::_Exit(17);
      {
        std::lock_guard<std::mutex> g(mu_);
        if (error_.empty()) error_ = e.what();
      }
      if (abort_) abort_->store(true);
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      --inflight_;
    }
    cv_.notify_all();
  }
}

void CpuStream::record(Event& e) {
  auto* ce = dynamic_cast<CpuEvent*>(&e);
  DLNB_REQUIRE(ce, "CPU stream needs a CPU event");
  uint64_t gen = ce->mark_recorded();
  enqueue([ce, gen] { ce->complete(gen); });
}

void CpuStream::wait(Event& e) {
  auto* ce = dynamic_cast<CpuEvent*>(&e);
  DLNB_REQUIRE(ce, "CPU stream needs a CPU event");
  uint64_t gen = ce->recorded();
  if (gen == 0) return;  // never recorded: nothing to wait for (HIP semantics)
  enqueue([ce, gen] { ce->wait_for(gen); });
}

void CpuStream::drain() {
  std::unique_lock<std::mutex> g(mu_);
  cv_.wait(g, [&] { return inflight_ == 0; });
}

bool CpuStream::query() {
  std::lock_guard<std::mutex> g(mu_);
  return inflight_ == 0;
}

void CpuStream::synchronize() {
  std::unique_lock<std::mutex> g(mu_);
  cv_.wait(g, [&] { return inflight_ == 0; });
  if (!error_.empty()) {
    std::string e = error_;
    error_.clear();
    DLNB_THROW("CPU stream task failed: " << e);
  }
}

// --------------------------------------------------------------- CpuDevice

namespace {

std::mutex& peer_mu() {
  static std::mutex m;
  return m;
}
std::map<const void*, int>& peer_fds() {
  static std::map<const void*, int> m;
  return m;
}

class CpuDevice : public Device {
 public:
  explicit CpuDevice(AbortFlag abort) : abort_(std::move(abort)), reg_(std::make_shared<CpuStreamRegistry>()) {}
  DeviceKind kind() const override { return DeviceKind::CPU; }
  std::string name() const override { return "CPU"; }
  int index() const override { return 0; }
  std::unique_ptr<Stream> create_stream(bool) override { return std::unique_ptr<Stream>(new CpuStream(abort_, reg_)); }
  std::unique_ptr<Event> create_event(bool) override { return std::unique_ptr<Event>(new CpuEvent(abort_)); }
  double elapsed_ms(Event& a, Event& b) override {
    auto* ea = dynamic_cast<CpuEvent*>(&a);
    auto* eb = dynamic_cast<CpuEvent*>(&b);
    DLNB_REQUIRE(ea && eb, "CPU events expected");
    return (eb->time_s() - ea->time_s()) * 1e3;
  }
  void* raw_alloc(size_t bytes) override {
    // calloc semantics like the reference's CPU Tensor (proxy_classes.hpp:395-400).
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) DLNB_THROW("host allocation of " << bytes << " bytes failed");
    return p;
  }
  // Peer memory: an anonymous memfd (no name to leak in /dev/shm if the
  // process dies), mapped shared; peers open it through /proc/<pid>/fd.
  void* raw_alloc_peer(size_t bytes) override {
    const int fd = static_cast<int>(syscall(SYS_memfd_create, "dlnb_peer", 0u));
    if (fd < 0) DLNB_THROW("memfd_create failed: " << std::strerror(errno));
    if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
      ::close(fd);
      DLNB_THROW("ftruncate of a " << bytes << "-byte peer buffer failed");
    }
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (p == MAP_FAILED) {
      ::close(fd);
      DLNB_THROW("host peer allocation of " << bytes << " bytes failed");
    }
    std::lock_guard<std::mutex> g(peer_mu());
    peer_fds()[p] = fd;
    return p;
  }
  void raw_free(void* p, size_t bytes) override {
    munmap(p, bytes);
    std::lock_guard<std::mutex> g(peer_mu());
    auto it = peer_fds().find(p);
    if (it != peer_fds().end()) {
      ::close(it->second);
      peer_fds().erase(it);
    }
  }
  void fill_random(void* p, size_t count, DType t, uint64_t seed, Stream& s) override {
    auto* cs = dynamic_cast<CpuStream*>(&s);
    cs->enqueue([p, count, t, seed] {
      uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
      for (size_t i = 0; i < count; ++i) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        float f = static_cast<float>((x >> 40) & 0xffffff) / 8388608.0f - 1.0f;
        switch (t) {
          case DType::BF16: static_cast<uint16_t*>(p)[i] = float_to_bf16(f); break;
          case DType::FP16: static_cast<uint16_t*>(p)[i] = float_to_fp16(f); break;
          case DType::FP32: static_cast<float*>(p)[i] = f; break;
          case DType::FP8_E4M3: static_cast<uint8_t*>(p)[i] = static_cast<uint8_t>(((x >> 20) & 0x77) | ((x >> 8) & 0x80)); break;
          case DType::FP8_E5M2: static_cast<uint8_t*>(p)[i] = float_to_fp8e5m2(f); break;
        }
      }
    });
  }
  void memset_async(void* p, int v, size_t bytes, Stream& s) override {
    dynamic_cast<CpuStream&>(s).enqueue([p, v, bytes] { std::memset(p, v, bytes); });
  }
  void copy_async(void* dst, const void* src, size_t bytes, Stream& s) override {
    dynamic_cast<CpuStream&>(s).enqueue([dst, src, bytes] { std::memcpy(dst, src, bytes); });
  }
  void host_task(Stream& s, std::function<void()> fn) override { dynamic_cast<CpuStream&>(s).enqueue(std::move(fn)); }
  // Like hipDeviceSynchronize: every live stream of this device drained.
  void synchronize() override {
    std::lock_guard<std::mutex> g(reg_->mu);
    for (CpuStream* s : reg_->live) s->synchronize();
  }
  bool abort_and_drain() override {
    abort_->store(true);
    std::lock_guard<std::mutex> g(reg_->mu);
    for (CpuStream* s : reg_->live) s->drain();
    return true;
  }
  bool abort_raised() const override { return abort_->load(); }
  void idle(Stream& s, double us) override {
    dynamic_cast<CpuStream&>(s).enqueue([us] { precise_sleep_us(us); });
  }
  uint64_t* alloc_stamps(size_t n) override { return static_cast<uint64_t*>(std::calloc(n, sizeof(uint64_t))); }
  void free_stamps(uint64_t* p, size_t) override { std::free(p); }
  void stamp(Stream& s, uint64_t* slot) override {
    dynamic_cast<CpuStream&>(s).enqueue([slot] { *slot = static_cast<uint64_t>(now_s() * 1e9); });
  }
  double stamp_hz() const override { return 1e9; }
  size_t total_memory() const override { return static_cast<size_t>(sysconf(_SC_PHYS_PAGES)) * sysconf(_SC_PAGE_SIZE); }
  size_t free_memory() const override { return static_cast<size_t>(sysconf(_SC_AVPHYS_PAGES)) * sysconf(_SC_PAGE_SIZE); }

 private:
  AbortFlag abort_;
  std::shared_ptr<CpuStreamRegistry> reg_;
};

}  // namespace

std::unique_ptr<Device> make_cpu_device(AbortFlag abort) {
  // every CPU device has an abort switch: a failing stream task raises it
  if (!abort) abort = std::make_shared<std::atomic<bool>>(false);
  return std::unique_ptr<Device>(new CpuDevice(std::move(abort)));
}

std::unique_ptr<GraphExec> Device::capture(Stream&, const std::vector<Stream*>&, const std::function<void()>&,
                                           const std::function<void()>&) {
  DLNB_THROW("--graph needs a GPU device (HIP graphs)");
}

std::vector<std::unique_ptr<GraphExec>> Device::capture_lanes(const std::vector<Stream*>&, const std::function<void()>&,
                                                               const std::function<void(size_t)>&) {
  DLNB_THROW("lane graphs need a GPU device (HIP graphs)");
}

void Device::host_signal(Stream&, uint64_t*, uint64_t) { DLNB_THROW("host_signal needs a GPU device"); }
void Device::host_wait(Stream&, const uint64_t*, uint64_t, double, uint64_t*, uint64_t) {
  DLNB_THROW("host_wait needs a GPU device");
}
uint64_t* Device::alloc_gate() { DLNB_THROW("device gates need a GPU device"); }
void Device::set_iteration(Stream&, uint64_t) {}

std::string cpu_peer_source(const void* p) {
  std::lock_guard<std::mutex> g(peer_mu());
  auto it = peer_fds().find(p);
  if (it == peer_fds().end()) return "";
  return "/proc/" + std::to_string(static_cast<long>(getpid())) + "/fd/" + std::to_string(it->second);
}

}  // namespace dlnb
