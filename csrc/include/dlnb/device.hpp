// Device layer: buffers, streams and events behind one interface for the GPU
// (HIP on MI355X) and the CPU (worker-thread "streams").
//
// Reference: cpp/proxy_classes.hpp:345-444 (Device enum, Tensor<T,Device>
// with calloc / cudaMalloc / hipMalloc / sycl::malloc_device) and the stream
// macros of cpp/data_types.hpp:91-130. The reference drives all ordering from
// the host thread (blocking collectives, usleep compute). Here every strategy
// is *stream ordered*: compute and collectives are enqueued on streams and
// ordered with events, so the host never sits on the critical path. The CPU
// device reproduces the same semantics with one worker thread per stream, so
// the same strategy code runs without a GPU (the reference's mpi_cpu build).
#pragma once

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <functional>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dlnb/common.hpp"

namespace dlnb {

class Event {
 public:
  virtual ~Event() = default;
};

class Stream {
 public:
  virtual ~Stream() = default;
  virtual void record(Event& e) = 0;
  virtual void wait(Event& e) = 0;  // later work on this stream waits for e
  virtual void synchronize() = 0;   // host waits for all enqueued work
  virtual bool query() = 0;         // true when all enqueued work is done
  virtual void* native() = 0;       // hipStream_t on GPU, nullptr on CPU
};

class Device;

// An instantiated HIP graph of one captured iteration (GPU only).
class GraphExec {
 public:
  virtual ~GraphExec() = default;
  virtual void launch(Stream& s) = 0;
  virtual size_t nodes() const = 0;
  virtual size_t edges() const { return 0; }
  // node count per node type ("kernel:12 memcpy:1 ..."), for the report
  virtual std::string node_types() const { return ""; }
  // a chain: every node but the first depends on exactly the one before it,
  // so the executor runs the whole graph on the launch stream's queue
  bool linear() const { return nodes() == 0 || edges() + 1 == nodes(); }
};

// Owning buffer (device memory on GPU, page-aligned host memory on CPU).
class Buffer {
 public:
  Buffer() = default;
  // peer = true: memory peers may read and write directly over xGMI
  // (Device::raw_alloc_peer; see Communicator::register_buffer).
  Buffer(Device* dev, size_t bytes, bool peer = false);
  ~Buffer();
  Buffer(const Buffer&) = delete;
  Buffer& operator=(const Buffer&) = delete;
  Buffer(Buffer&& o) noexcept { *this = std::move(o); }
  Buffer& operator=(Buffer&& o) noexcept;
  void* data() const { return ptr_; }
  size_t bytes() const { return bytes_; }
  template <typename T>
  T* as() const {
    return static_cast<T*>(ptr_);
  }
  char* at(size_t byte_offset) const { return static_cast<char*>(ptr_) + byte_offset; }

 private:
  Device* dev_ = nullptr;
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
};

class Device {
 public:
  virtual ~Device() = default;
  virtual DeviceKind kind() const = 0;
  virtual std::string name() const = 0;
  virtual int index() const = 0;
  virtual std::unique_ptr<Stream> create_stream(bool high_priority) = 0;
  // timing = false: a dependency-only event (no timestamp, device-scope
  // release: no L2 writeback / system fence on AMD, which otherwise costs
  // tens of µs per record after a large GEMM). timing = true: timestamped,
  // still without the system-scope fence.
  virtual std::unique_ptr<Event> create_event(bool timing = false) = 0;
  // Milliseconds from a to b; both must have completed.
  virtual double elapsed_ms(Event& a, Event& b) = 0;
  virtual void* raw_alloc(size_t bytes) = 0;
  // Zeroed memory that other GPUs' kernels access directly through IPC
  // mappings (GPU: uncached, so a peer's stores are never shadowed by a stale
  // line in this device's L2 and this device's stores reach memory when
  // they complete). Freed with raw_free. CPU: a memfd mapping another
  // process of this host maps through /proc (cpu_peer_source).
  virtual void* raw_alloc_peer(size_t bytes) { return raw_alloc(bytes); }
  virtual void raw_free(void* p, size_t bytes) = 0;
  // Fill with deterministic pseudo-random values of type t in [-1, 1)
  // (random data keeps the MFMA units at realistic clocks, unlike zeros).
  virtual void fill_random(void* p, size_t count, DType t, uint64_t seed, Stream& s) = 0;
  virtual void memset_async(void* p, int v, size_t bytes, Stream& s) = 0;
  virtual void copy_async(void* dst, const void* src, size_t bytes, Stream& s) = 0;
  // Enqueue a host callback (CPU: task on the worker; GPU: hipLaunchHostFunc).
  virtual void host_task(Stream& s, std::function<void()> fn) = 0;
  virtual void synchronize() = 0;
  // After a failed iteration, before the strategy (its events, buffers and
  // communicators) is destroyed: stop every stream's queued work and wait for
  // the streams to go idle. CPU devices raise their abort switch (queued
  // tasks are skipped, event waits return) and drain; GPU devices: nothing
  // (the communicators were aborted, the runtime owns the queues).
  // GPU: raise the abort word (below), then wait - at most
  // DLNB_ABORT_DRAIN_S (20) seconds - for every stream of the device to go
  // idle; false when one did not (the caller must not free anything the
  // device may still use: the process is then unusable for another run).
  virtual bool abort_and_drain() { return true; }
  // ---- failure containment: a host-mapped word every device-side wait polls
  // next to what it waits for (the deadline tasks' gates and claims, the
  // programs' joins, gate_wait and the pre-armed replays' go waits). Once
  // raised (raise_abort, a host store: no queue needed) every such wait gives
  // up, a deadline task that waited ends at once, and a pre-armed replay the
  // abort releases runs through on a poisoned iteration word without
  // computing or waiting (kernels::kPoisonIter). abort_word: the device-side
  // pointer the kernels take (nullptr: none).
  virtual const uint64_t* abort_word() { return nullptr; }
  virtual void raise_abort() {}
  virtual bool abort_raised() const { return false; }
  // An idle wait of `us` on s (GPU: a one-wave s_memrealtime wait kernel;
  // CPU: a sleeping task): the comm fault injector's delay.
  virtual void idle(Stream& s, double us) = 0;
  // Timestamps taken when a stream reaches a point (device clock on GPU: a
  // one-wave kernel stores s_memrealtime into host-mapped memory; host clock
  // on CPU). Unlike timing events they are exact across cross-stream waits.
  virtual uint64_t* alloc_stamps(size_t n) = 0;  // zeroed, host-readable
  virtual void free_stamps(uint64_t* p, size_t n) = 0;
  virtual void stamp(Stream& s, uint64_t* slot) = 0;
  // Handshake words (alloc_stamps memory) between the host and a stream:
  // host_signal stores value when the stream reaches it; host_wait holds the
  // stream until the host (or a signal) stored a value >= `value`, at most
  // timeout_s (then it adds 1 to *timeouts and lets the stream go). GPU only.
  // host_wait also stores iter_value into the device's iteration word once
  // released (iter_value 0: leaves it).
  virtual void host_signal(Stream& s, uint64_t* word, uint64_t value);
  virtual void host_wait(Stream& s, const uint64_t* word, uint64_t value, double timeout_s, uint64_t* timeouts,
                         uint64_t iter_value = 0);
  // ---- device gates (GPU): ordering between streams through device words
  // (kernels::gate_signal / gate_wait) instead of graph edges.
  // A gate is two 16-byte-aligned words {seq, time}; seq carries the
  // iteration word (iter_word) so a replayed graph's gates never satisfy the
  // next replay's waits. alloc_gate: a zeroed gate (freed with the device).
  virtual uint64_t* alloc_gate();
  virtual uint64_t* iter_word() { return nullptr; }
  // A no-op kernel on s (GPU): a graph's trailing node.
  virtual void pad(Stream& s) { (void)s; }
  // Raise a gate from alloc_gate with `tag` when s gets here (GPU).
  virtual void signal_gate(Stream& s, uint64_t* gate, uint32_t tag) {
    (void)s; (void)gate; (void)tag;
    DLNB_THROW("device gates need a GPU device");
  }
  // Enqueue on s a store of `it` into the iteration word (a lane's head).
  virtual void set_iteration(Stream& s, uint64_t it);
  // Gate events: while on, recording a dependency-only event (create_event
  // (false)) raises its gate on the recording stream and waiting on it
  // enqueues a one-wave gate_wait on the waiting stream (the mode is read at
  // enqueue time). The runner turns it on for lane graphs: every stream is
  // captured into its own linear graph, with no cross-stream edge for the
  // graph executor to act on (it spreads a forked graph over its hardware
  // queues and can queue a compute node behind a collective,
  // profiles/absorb_r4.md). Waits are bounded (DLNB_GATE_TIMEOUT_S, 60) and
  // counted (gate_event_timeouts).
  virtual void set_gate_events(bool on) { DLNB_REQUIRE(!on, "gate events need a GPU device"); }
  // Bound (s) of the gate-event waits captured from here on (DLNB_GATE_TIMEOUT_S, 60, unless set).
  virtual void set_gate_timeout(double s) { (void)s; }
  // With gate events on: record e on s as a gate a kernel the caller launches
  // on s next raises itself (returns the gate and tag it must store; a
  // deadline task's DlSync::done_gate). False (nothing recorded) otherwise.
  virtual bool arm_gate_record(Event& e, Stream& s, uint64_t** gate, uint32_t* tag) {
    (void)e; (void)s; (void)gate; (void)tag;
    return false;
  }
  virtual bool gate_events() const { return false; }
  // Gate events folded into a consumer instead of gate kernels on s: while a
  // fold is installed on s (a compute program open on it, ComputeEngine),
  // s.wait(e) hands the gate and tag to wait for to fold_wait (nothing when
  // there is nothing to wait for: e never recorded, recorded on s, or before
  // this capture) and s.record(e) hands e to fold_record, which arms it
  // (arm_gate_record) for a kernel it launches on s. nullptr removes it.
  struct StreamFold {
    virtual ~StreamFold() = default;
    virtual void fold_wait(const uint64_t* gate, uint32_t tag) = 0;
    virtual void fold_record(Event& e) = 0;
  };
  virtual void set_stream_fold(Stream& s, StreamFold* f) { (void)s; (void)f; }
  // Enqueue on s a store of the iteration word into *host_word (alloc_stamps
  // memory): the last node of a lane graph, so the host sees the lane done
  // without waiting for the graph's own completion (GPU only).
  virtual void lane_done(Stream& s, uint64_t* host_word) { (void)s; (void)host_word; DLNB_THROW("lane_done needs a GPU"); }
  // Whether s is being captured into a graph (GPU; never on the CPU).
  virtual bool capturing(Stream& s) { (void)s; return false; }
  virtual uint64_t gate_event_timeouts() { return 0; }
  // Whether each stream of `ss` runs while another of them is blocked: every
  // ordered pair is probed (a one-wave wait on one for a store enqueued later
  // on the other, bounded by timeout_s). Two streams on one hardware queue
  // would deadlock gate waits between them. detail: the failing pairs.
  virtual bool queues_independent(const std::vector<Stream*>& ss, double timeout_s, std::string* detail) {
    (void)ss; (void)timeout_s; (void)detail;
    return true;
  }
  virtual double stamp_hz() const = 0;
  virtual size_t total_memory() const = 0;
  virtual size_t free_memory() const = 0;
  // Capture everything `enqueue` puts on `origin` and `others` into one graph:
  // the other streams are forked from origin before and joined back after,
  // so the graph is launched on origin alone. `head` (optional) is enqueued
  // on origin before the fork, so everything of every stream comes after it
  // (the compute engine's slot / gate reset). GPU only.
  virtual std::unique_ptr<GraphExec> capture(Stream& origin, const std::vector<Stream*>& others,
                                             const std::function<void()>& enqueue,
                                             const std::function<void()>& head = {});
  // Lane capture: every stream of `lanes` is captured into its own graph at
  // the same time (no fork / join: the strategy's cross-stream dependencies
  // must be gate events). tail(i) runs after enqueue, still capturing, to add
  // lane i's last nodes. Graph i is launched on lanes[i]. GPU only.
  virtual std::vector<std::unique_ptr<GraphExec>> capture_lanes(const std::vector<Stream*>& lanes,
                                                                const std::function<void()>& enqueue,
                                                                const std::function<void(size_t)>& tail = {});

  Buffer alloc(size_t bytes) { return Buffer(this, bytes); }
  Buffer alloc_peer(size_t bytes) { return Buffer(this, bytes, true); }
};

// ---- CPU implementation (also used by the GPU-less tests) ----

// Abort switch of one job (loopback-cpu: its LoopbackHub owns it): when set,
// CPU-stream event waits give up and queued CPU-stream tasks are dropped, so
// worker threads blocked on a failed rank's events drain and every rank
// thread can unwind. Scoped to the job's device, so another job in the same
// process (or a later --backend cpu run) is never affected.
using AbortFlag = std::shared_ptr<std::atomic<bool>>;

// Generation-counted event with HIP semantics: a wait() captures the most
// recent record() at enqueue time and blocks until that record completes.
class CpuEvent : public Event {
 public:
  explicit CpuEvent(AbortFlag abort = nullptr) : abort_(std::move(abort)) {}
  uint64_t mark_recorded();           // host, at enqueue time
  void complete(uint64_t gen);        // worker, when reached
  uint64_t recorded() ;
  void wait_for(uint64_t gen);        // worker or host
  double time_s();

 private:
  AbortFlag abort_;
  std::mutex mu_;
  std::condition_variable cv_;
  uint64_t recorded_ = 0;
  uint64_t completed_ = 0;
  double t_ = 0;
};

// Live streams of one CPU device (Device::synchronize drains them all).
struct CpuStreamRegistry;

class CpuStream : public Stream {
 public:
  explicit CpuStream(AbortFlag abort = nullptr, std::shared_ptr<CpuStreamRegistry> reg = nullptr);
  ~CpuStream() override;
  void record(Event& e) override;
  void wait(Event& e) override;
  void synchronize() override;
  bool query() override;
  void drain();  // wait until idle; a task's error stays for synchronize()
  void* native() override { return nullptr; }
  void enqueue(std::function<void()> fn);

 private:
  void run();
  AbortFlag abort_;
  std::shared_ptr<CpuStreamRegistry> reg_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  size_t inflight_ = 0;
  bool stop_ = false;
  std::string error_;
  std::thread th_;
};

// CPU device; its streams and events observe `abort` (may be null).
std::unique_ptr<Device> make_cpu_device(AbortFlag abort = nullptr);

// GPU device (HIP). local_index picks the visible device.
std::unique_ptr<Device> make_gpu_device(int local_index);
int gpu_device_count();  // 0 when no GPU / no HIP runtime
// Text matrix of link type (XGMI / PCIE) and hop count between all visible
// GPUs plus each GPU's PCI bus id (empty without GPUs).
std::string describe_gpu_links();

// CPU device peer allocations (Device::alloc_peer on the CPU device): the
// "/proc/<pid>/fd/<fd>" path another process of this host opens to map the
// allocation starting at p, or "" when p is not such an allocation.
std::string cpu_peer_source(const void* p);

// Seconds on a monotonic host clock.
double now_s();
// Precise host sleep (nanosleep + short spin for the tail).
void precise_sleep_us(double us);

}  // namespace dlnb
