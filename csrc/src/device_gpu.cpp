// HIP implementation of the device layer (MI355X / gfx950).
#include <hip/hip_runtime.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "dlnb/device.hpp"
#include "dlnb/kernels.hpp"

#define DLNB_HIP_CHECK(expr)                                                       \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) DLNB_THROW(#expr << " failed: " << hipGetErrorString(e_)); \
  } while (0)

namespace dlnb {

namespace {

class GpuDevice;

class GpuEvent : public Event {
 public:
  GpuEvent(bool timing, GpuDevice* dev) : dev(timing ? nullptr : dev) {
    // Dependency-only events: no timestamp and, on HIP >= 7.2, no
    // system-scope fence (an L2 writeback after every GEMM otherwise; the
    // ordering we need is device-local). Timing events keep the defaults.
    unsigned flags = timing ? hipEventDefault : hipEventDisableTiming;
    if (!timing && runtime_version() >= 70200000) flags |= hipEventDisableSystemFence;
    DLNB_HIP_CHECK(hipEventCreateWithFlags(&ev, flags));
  }
  static int runtime_version() {
    static const int v = [] {
      int x = 0;
      if (hipRuntimeGetVersion(&x) != hipSuccess) x = 0;
      return x;
    }();
    return v;
  }
  ~GpuEvent() override { (void)hipEventDestroy(ev); }
  hipEvent_t ev{};
  // gate events (Device::set_gate_events): the device (nullptr for timing
  // events, which never become gates), the gate (allocated at the first gate
  // record) and the tag of the latest record (0: never recorded as a gate)
  GpuDevice* dev = nullptr;
  uint64_t* gate = nullptr;
  uint32_t tag = 0;
  hipStream_t on = nullptr;  // stream of the latest gate record
  uint64_t gen = 0;          // the device's capture generation at that record
};

// The device's live streams (abort_and_drain polls them all).
struct GpuStreamSet {
  std::mutex mu;
  std::set<hipStream_t> live;
};

class GpuStream : public Stream {
 public:
  GpuStream(int device, bool high_priority, std::shared_ptr<GpuStreamSet> set) : set_(std::move(set)) {
    DLNB_HIP_CHECK(hipSetDevice(device));
    int lo = 0, hi = 0;
    DLNB_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // hi is the numerically smallest (= greatest) priority.
    DLNB_HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, high_priority ? hi : lo));
    std::lock_guard<std::mutex> g(set_->mu);
    set_->live.insert(s);
  }
  ~GpuStream() override {
    {
      std::lock_guard<std::mutex> g(set_->mu);
      set_->live.erase(s);
    }
    (void)hipStreamDestroy(s);
  }
  void record(Event& e) override;
  void wait(Event& e) override;
  void synchronize() override { DLNB_HIP_CHECK(hipStreamSynchronize(s)); }
  bool query() override {
    hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return true;
    if (e == hipErrorNotReady) return false;
    DLNB_THROW("hipStreamQuery failed: " << hipGetErrorString(e));
  }
  void* native() override { return s; }
  hipStream_t s{};
  Device::StreamFold* fold = nullptr;  // Device::set_stream_fold

 private:
  std::shared_ptr<GpuStreamSet> set_;
};

class GpuGraphExec : public GraphExec {
 public:
  GpuGraphExec(hipGraphExec_t e, size_t n, size_t edges, std::string types)
      : exec_(e), n_(n), edges_(edges), types_(std::move(types)) {}
  ~GpuGraphExec() override { (void)hipGraphExecDestroy(exec_); }
  void launch(Stream& s) override { DLNB_HIP_CHECK(hipGraphLaunch(exec_, static_cast<hipStream_t>(s.native()))); }
  size_t nodes() const override { return n_; }
  size_t edges() const override { return edges_; }
  std::string node_types() const override { return types_; }

 private:
  hipGraphExec_t exec_;
  size_t n_, edges_;
  std::string types_;
};

std::string graph_node_types(hipGraph_t g, size_t n) {
  std::vector<hipGraphNode_t> nodes(n);
  size_t got = n;
  if (n == 0 || hipGraphGetNodes(g, nodes.data(), &got) != hipSuccess) return "";
  std::map<std::string, int> count;
  for (size_t i = 0; i < got; ++i) {
    hipGraphNodeType t{};
    if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess) continue;
    const char* name = t == hipGraphNodeTypeKernel ? "kernel"
                       : t == hipGraphNodeTypeMemcpy ? "memcpy"
                       : t == hipGraphNodeTypeMemset ? "memset"
                       : t == hipGraphNodeTypeHost ? "host"
                       : t == hipGraphNodeTypeGraph ? "child_graph"
                       : t == hipGraphNodeTypeEmpty ? "empty"
                       : t == hipGraphNodeTypeWaitEvent ? "wait_event"
                       : t == hipGraphNodeTypeEventRecord ? "event_record"
                                                            : "other";
    ++count[name];
  }
  std::string out;
  for (const auto& kv : count) out += (out.empty() ? "" : " ") + kv.first + ":" + std::to_string(kv.second);
  return out;
}

// Instantiate a captured graph (destroying it); node and edge counts kept.
std::unique_ptr<GraphExec> instantiate(hipGraph_t g) {
  size_t n = 0, ne = 0;
  (void)hipGraphGetNodes(g, nullptr, &n);
  (void)hipGraphGetEdges(g, nullptr, nullptr, &ne);
  std::string types = graph_node_types(g, n);
  hipGraphExec_t e = nullptr;
  hipError_t err = hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (err != hipSuccess) DLNB_THROW("hipGraphInstantiate failed: " << hipGetErrorString(err));
  return std::unique_ptr<GraphExec>(new GpuGraphExec(e, n, ne, std::move(types)));
}

void host_trampoline(void* p) {
  auto* fn = static_cast<std::function<void()>*>(p);
  (*fn)();
  delete fn;
}

class GpuDevice : public Device {
 public:
  explicit GpuDevice(int idx) : idx_(idx) {
    DLNB_HIP_CHECK(hipSetDevice(idx_));
    hipDeviceProp_t prop;
    DLNB_HIP_CHECK(hipGetDeviceProperties(&prop, idx_));
    name_ = prop.name;
    arch_ = prop.gcnArchName;
    total_ = prop.totalGlobalMem;
    kernels::clock_cal_begin(idx_);  // the rate is taken at its first use (stamp_hz), after setup
    ensure_pool();                   // gates / iteration word: never allocated while a stream captures
    void* a = nullptr;
    DLNB_HIP_CHECK(hipHostMalloc(&a, 64, hipHostMallocMapped | hipHostMallocCoherent));
    abort_host_ = static_cast<uint64_t*>(a);
    std::memset(abort_host_, 0, 64);
    void* ad = nullptr;
    DLNB_HIP_CHECK(hipHostGetDevicePointer(&ad, a, 0));
    abort_dev_ = static_cast<uint64_t*>(ad);
  }
  ~GpuDevice() override {
    if (pool_) (void)hipFree(pool_);
    // (an abort word a kernel may still poll is never freed: the process is going away)
    if (abort_host_ && !abort_raised()) (void)hipHostFree(abort_host_);
  }
  DeviceKind kind() const override { return DeviceKind::GPU; }
  std::string name() const override { return name_ + " (" + arch_ + ")"; }
  int index() const override { return idx_; }
  std::unique_ptr<Stream> create_stream(bool high_priority) override {
    // DLNB_HIGH_PRIORITY_STREAMS=0: comm lanes on normal-priority queues (A/B)
    static const bool high_ok = env_int("DLNB_HIGH_PRIORITY_STREAMS", 1) != 0;
    return std::unique_ptr<Stream>(new GpuStream(idx_, high_priority && high_ok, streams_));
  }
  std::unique_ptr<Event> create_event(bool timing) override {
    return std::unique_ptr<Event>(new GpuEvent(timing, this));
  }
  double elapsed_ms(Event& a, Event& b) override {
    float ms = 0;
    DLNB_HIP_CHECK(hipEventSynchronize(static_cast<GpuEvent&>(b).ev));
    DLNB_HIP_CHECK(hipEventElapsedTime(&ms, static_cast<GpuEvent&>(a).ev, static_cast<GpuEvent&>(b).ev));
    return ms;
  }
  void* raw_alloc(size_t bytes) override {
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess)
      DLNB_THROW("hipMalloc(" << bytes << " B) failed on device " << idx_ << ": " << hipGetErrorString(e));
    // Zero like the reference's Tensor (proxy_classes.hpp:403-409). The
    // memset runs on the null stream, which our non-blocking streams do not
    // order against: finish it here, or it can land after the first copy or
    // kernel a caller enqueues on its own stream (zeroing fresh data).
    DLNB_HIP_CHECK(hipMemset(p, 0, bytes));
    DLNB_HIP_CHECK(hipStreamSynchronize(nullptr));
    return p;
  }
  void* raw_alloc_peer(size_t bytes) override {
    void* p = nullptr;
    hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
    if (e != hipSuccess)
      DLNB_THROW("hipExtMallocWithFlags(" << bytes << " B, uncached) failed on device " << idx_ << ": "
                                          << hipGetErrorString(e));
    DLNB_HIP_CHECK(hipMemset(p, 0, bytes));
    DLNB_HIP_CHECK(hipStreamSynchronize(nullptr));
    return p;
  }
  void raw_free(void* p, size_t) override { (void)hipFree(p); }
  void fill_random(void* p, size_t count, DType t, uint64_t seed, Stream& s) override {
    kernels::fill_random(p, count, t, seed, s.native());
  }
  void memset_async(void* p, int v, size_t bytes, Stream& s) override {
    DLNB_HIP_CHECK(hipMemsetAsync(p, v, bytes, static_cast<hipStream_t>(s.native())));
  }
  void copy_async(void* dst, const void* src, size_t bytes, Stream& s) override {
    DLNB_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, static_cast<hipStream_t>(s.native())));
  }
  void host_task(Stream& s, std::function<void()> fn) override {
    auto* heap = new std::function<void()>(std::move(fn));
    DLNB_HIP_CHECK(hipLaunchHostFunc(static_cast<hipStream_t>(s.native()), host_trampoline, heap));
  }
  void synchronize() override { DLNB_HIP_CHECK(hipDeviceSynchronize()); }
  const uint64_t* abort_word() override { return abort_dev_; }
  void raise_abort() override { __atomic_store_n(abort_host_, 1ull, __ATOMIC_SEQ_CST); }
  bool abort_raised() const override { return __atomic_load_n(abort_host_, __ATOMIC_ACQUIRE) != 0; }
  bool abort_and_drain() override {
    raise_abort();
    // every device wait gives up on the abort word (and the communicators were
    // aborted by the caller), so the queued work drains; bounded all the same
    const double limit = static_cast<double>(env_int("DLNB_ABORT_DRAIN_S", 20));
    const double t0 = now_s();
    for (;;) {
      bool idle = true;
      {
        std::lock_guard<std::mutex> g(streams_->mu);
        for (hipStream_t s : streams_->live) {
          const hipError_t e = hipStreamQuery(s);
          if (e == hipErrorNotReady) {
            idle = false;
            break;
          }
        }
      }
      if (idle) return true;
      if (now_s() - t0 > limit) return false;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  void idle(Stream& s, double us) override {
    kernels::idle_wait(static_cast<uint64_t>(us * 1e-6 * stamp_hz() + 0.5), s.native());
  }
  uint64_t* alloc_stamps(size_t n) override {
    void* p = nullptr;
    DLNB_HIP_CHECK(hipHostMalloc(&p, n * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(p, 0, n * sizeof(uint64_t));
    return static_cast<uint64_t*>(p);
  }
  void free_stamps(uint64_t* p, size_t) override { (void)hipHostFree(p); }
  void stamp(Stream& s, uint64_t* slot) override { kernels::stamp(slot, s.native()); }
  void host_signal(Stream& s, uint64_t* word, uint64_t value) override { kernels::host_signal(word, value, s.native()); }
  void host_wait(Stream& s, const uint64_t* word, uint64_t value, double timeout_s, uint64_t* timeouts,
                 uint64_t iter_value) override {
    kernels::host_wait(word, value, static_cast<uint64_t>(timeout_s * stamp_hz()), timeouts, s.native(),
                       iter_value ? iter_word() : nullptr, iter_value, abort_dev_);
  }

  // ---- gates: one zeroed device block, carved without HIP calls (gates are
  // taken during graph capture); [0] the iteration word, [1] gate-event wait
  // timeouts, gates from byte 64 on, 16 bytes each.
  uint64_t* alloc_gate() override {
    ensure_pool();
    DLNB_REQUIRE(next_gate_ < kPoolGates, "device gate pool exhausted (" << kPoolGates << " gates)");
    return pool_ + 8 + 2 * next_gate_++;
  }
  uint64_t* iter_word() override {
    ensure_pool();
    return pool_;
  }
  void set_iteration(Stream& s, uint64_t it) override { kernels::set_word(iter_word(), it, s.native()); }
  void lane_done(Stream& s, uint64_t* host_word) override { kernels::lane_done(host_word, iter_word(), s.native()); }
  void pad(Stream& s) override { kernels::set_word(pool_ + 2, 0, s.native()); }  // pool word 2: scratch
  void signal_gate(Stream& s, uint64_t* gate, uint32_t tag) override {
    kernels::gate_signal(gate, iter_word(), tag, s.native());
  }
  void set_gate_events(bool on) override {
    if (on) ensure_pool();
    gate_events_ = on;
  }
  bool gate_events() const override { return gate_events_; }
  bool capturing(Stream& s) override {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    DLNB_HIP_CHECK(hipStreamIsCapturing(static_cast<hipStream_t>(s.native()), &st));
    return st != hipStreamCaptureStatusNone;
  }
  uint64_t gate_event_timeouts() override {
    if (!pool_) return 0;
    uint64_t v = 0;
    DLNB_HIP_CHECK(hipMemcpy(&v, pool_ + 1, sizeof(v), hipMemcpyDeviceToHost));
    return v;
  }
  uint64_t gate_timeout_ticks() {
    static const double s = static_cast<double>(env_int("DLNB_GATE_TIMEOUT_S", 60));
    return static_cast<uint64_t>((gate_timeout_s_ > 0 ? gate_timeout_s_ : s) * stamp_hz());
  }
  void set_gate_timeout(double s) override { gate_timeout_s_ = s; }
  double gate_timeout_s_ = 0.0;
  void gate_mark(GpuEvent& e, hipStream_t s) {
    if (!e.gate) e.gate = alloc_gate();
    e.tag = e.tag == 0xffffffffu ? 1u : e.tag + 1;
    e.on = s;
    e.gen = gen_;
  }
  void gate_record(GpuEvent& e, hipStream_t s) {
    gate_mark(e, s);
    kernels::gate_signal(e.gate, iter_word(), e.tag, s);
  }
  bool arm_gate_record(Event& ev, Stream& s, uint64_t** gate, uint32_t* tag) override {
    auto& e = static_cast<GpuEvent&>(ev);
    if (!gate_events_ || !e.dev) return false;
    gate_mark(e, static_cast<hipStream_t>(s.native()));
    *gate = e.gate;
    *tag = e.tag;
    return true;
  }
  // Whether a wait on s for e's latest gate record must wait at all.
  bool gate_needed(const GpuEvent& e, hipStream_t s) const {
    if (e.tag == 0) return false;  // never recorded: nothing to wait for (as a HIP event)
    if (e.on == s) return false;   // recorded on this stream: already ordered
    // recorded before this capture began (a previous iteration's record): in a
    // replay its gate carries the previous iteration's sequence number and
    // would never match - as a HIP event outside the capture, nothing to wait
    // for inside the graph
    return e.gen == gen_;
  }
  void gate_wait(GpuEvent& e, GpuStream& st) {
    if (!gate_needed(e, st.s)) return;
    if (st.fold) {
      st.fold->fold_wait(e.gate, e.tag);
      return;
    }
    kernels::gate_wait(e.gate, iter_word(), e.tag, gate_timeout_ticks(), pool_ + 1, st.s, abort_dev_);
  }
  void set_stream_fold(Stream& s, StreamFold* f) override { static_cast<GpuStream&>(s).fold = f; }
  bool queues_independent(const std::vector<Stream*>& ss, double timeout_s, std::string* detail) override {
    const uint64_t t = static_cast<uint64_t>(timeout_s * stamp_hz());
    bool ok = true;
    for (size_t a = 0; a < ss.size(); ++a)
      for (size_t b = 0; b < ss.size(); ++b) {
        if (a == b) continue;
        if (!kernels::queues_independent(ss[a]->native(), ss[b]->native(), t)) {
          ok = false;
          if (detail) *detail += (detail->empty() ? "" : ", ") + std::to_string(a) + " waits behind " + std::to_string(b);
        }
      }
    return ok;
  }
  double stamp_hz() const override { return kernels::wallclock_hz(idx_); }
  size_t total_memory() const override { return total_; }
  size_t free_memory() const override {
    size_t f = 0, t = 0;
    if (hipMemGetInfo(&f, &t) != hipSuccess) return 0;
    return f;
  }
  std::unique_ptr<GraphExec> capture(Stream& origin, const std::vector<Stream*>& others,
                                     const std::function<void()>& enqueue,
                                     const std::function<void()>& head) override {
    // Fork/join events exist before the capture starts (no creation inside).
    auto fork = create_event(false);
    std::vector<std::unique_ptr<Event>> joins;
    for (size_t i = 0; i < others.size(); ++i) joins.push_back(create_event(false));
    hipStream_t o = static_cast<hipStream_t>(origin.native());
    DLNB_HIP_CHECK(hipStreamBeginCapture(o, hipStreamCaptureModeThreadLocal));
    try {
      if (head) head();
      origin.record(*fork);
      for (Stream* s : others) s->wait(*fork);
      enqueue();
      for (size_t i = 0; i < others.size(); ++i) {
        others[i]->record(*joins[i]);
        origin.wait(*joins[i]);
      }
    } catch (...) {
      hipGraph_t g = nullptr;
      (void)hipStreamEndCapture(o, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    hipGraph_t g = nullptr;
    DLNB_HIP_CHECK(hipStreamEndCapture(o, &g));
    return instantiate(g);
  }

  std::vector<std::unique_ptr<GraphExec>> capture_lanes(const std::vector<Stream*>& lanes,
                                                        const std::function<void()>& enqueue,
                                                        const std::function<void(size_t)>& tail) override {
    ++gen_;  // gate records from before this capture are not waited for in it
    size_t begun = 0;
    auto end_all = [&] {  // after a failure: end every capture begun, drop the graphs
      for (size_t i = 0; i < begun; ++i) {
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(static_cast<hipStream_t>(lanes[i]->native()), &g);
        if (g) (void)hipGraphDestroy(g);
      }
    };
    try {
      for (; begun < lanes.size(); ++begun)
        DLNB_HIP_CHECK(hipStreamBeginCapture(static_cast<hipStream_t>(lanes[begun]->native()),
                                             hipStreamCaptureModeThreadLocal));
      enqueue();
      if (tail)
        for (size_t i = 0; i < lanes.size(); ++i) tail(i);
    } catch (...) {
      end_all();
      throw;
    }
    std::vector<hipGraph_t> gs(lanes.size(), nullptr);
    hipError_t first = hipSuccess;
    for (size_t i = 0; i < lanes.size(); ++i) {
      hipError_t e = hipStreamEndCapture(static_cast<hipStream_t>(lanes[i]->native()), &gs[i]);
      if (e != hipSuccess && first == hipSuccess) first = e;
    }
    if (first != hipSuccess) {
      for (hipGraph_t g : gs)
        if (g) (void)hipGraphDestroy(g);
      DLNB_THROW("lane capture failed: " << hipGetErrorString(first)
                                         << " (a cross-stream dependency that is not a gate event?)");
    }
    std::vector<std::unique_ptr<GraphExec>> out;
    for (hipGraph_t g : gs) out.push_back(instantiate(g));
    return out;
  }

 private:
  static constexpr size_t kPoolGates = 65536;
  void ensure_pool() {
    if (pool_) return;
    const size_t bytes = 64 + kPoolGates * 16;
    DLNB_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&pool_), bytes));
    DLNB_HIP_CHECK(hipMemset(pool_, 0, bytes));
    DLNB_HIP_CHECK(hipStreamSynchronize(nullptr));
  }
  uint64_t* pool_ = nullptr;
  uint64_t* abort_host_ = nullptr;  // abort word: the host's pointer
  uint64_t* abort_dev_ = nullptr;   // and the kernels'
  std::shared_ptr<GpuStreamSet> streams_ = std::make_shared<GpuStreamSet>();
  size_t next_gate_ = 0;
  uint64_t gen_ = 0;  // capture generation (capture_lanes)
  bool gate_events_ = false;
  int idx_;
  std::string name_, arch_;
  size_t total_ = 0;
};

}  // namespace

void GpuStream::record(Event& e) {
  auto& g = static_cast<GpuEvent&>(e);
  if (g.dev && g.dev->gate_events()) {
    if (fold)
      fold->fold_record(e);
    else
      g.dev->gate_record(g, s);
    return;
  }
  DLNB_HIP_CHECK(hipEventRecord(g.ev, s));
}

void GpuStream::wait(Event& e) {
  auto& g = static_cast<GpuEvent&>(e);
  if (g.dev && g.dev->gate_events()) {
    g.dev->gate_wait(g, *this);
    return;
  }
  DLNB_HIP_CHECK(hipStreamWaitEvent(s, g.ev, 0));
}

std::unique_ptr<Device> make_gpu_device(int local_index) { return std::unique_ptr<Device>(new GpuDevice(local_index)); }

int gpu_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

std::string describe_gpu_links() {
  int n = gpu_device_count();
  if (n <= 0) return "";
  std::string out;
  char buf[256];
  for (int i = 0; i < n; ++i) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), i) != hipSuccess) std::snprintf(bus, sizeof(bus), "?");
    hipDeviceProp_t prop;
    std::string nm = hipGetDeviceProperties(&prop, i) == hipSuccess ? prop.name : "?";
    std::snprintf(buf, sizeof(buf), "  GPU%d  %s  %s  CUs=%d\n", i, bus, nm.c_str(),
                  hipGetDeviceProperties(&prop, i) == hipSuccess ? prop.multiProcessorCount : 0);
    out += buf;
  }
  if (n > 1) {
    out += "  link/hops ";
    for (int j = 0; j < n; ++j) {
      std::snprintf(buf, sizeof(buf), " %8s", ("GPU" + std::to_string(j)).c_str());
      out += buf;
    }
    out += "\n";
    for (int i = 0; i < n; ++i) {
      std::snprintf(buf, sizeof(buf), "  GPU%-6d", i);
      out += buf;
      for (int j = 0; j < n; ++j) {
        if (i == j) {
          std::snprintf(buf, sizeof(buf), " %8s", "-");
        } else {
          uint32_t lt = 0, hops = 0;
          const char* name = "?";
          if (hipExtGetLinkTypeAndHopCount(i, j, &lt, &hops) == hipSuccess) {
            name = lt == HSA_AMD_LINK_INFO_TYPE_XGMI ? "XGMI" : lt == HSA_AMD_LINK_INFO_TYPE_PCIE ? "PCIE" : "OTHER";
          }
          std::snprintf(buf, sizeof(buf), " %5s/%-2u", name, hops);
        }
        out += buf;
      }
      out += "\n";
    }
  }
  return out;
}

}  // namespace dlnb
