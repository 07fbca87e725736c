// Communication layer: one stream-ordered collective/P2P interface with a
// run-time selected backend.
//
// Reference: cpp/proxy_classes.hpp:30-342 defines ProxyCommunicator with
// request/stream "index" slots and three compile-time backends (MPI,
// NCCL/RCCL, oneCCL) chosen by PROXY_ENABLE_* macros. Differences here:
//   * every operation takes the Stream it is ordered on; completion is
//     tracked with Events, so there are no request slots and no Wait(i) /
//     WaitAll(n) (the reference's CCL "Barrier" that was not a barrier,
//     proxy_classes.hpp:189-191, disappears: host barriers live in
//     HostGroup);
//   * the backend is chosen at run time (--backend rccl|xgmi|mixed|cpu);
//   * all-to-all maps to ncclAllToAll instead of a hand-rolled
//     ncclGroupStart + per-peer send/recv loop (proxy_classes.hpp:160-182);
//   * element type is explicit (the MPI backend's hard-coded MPI_FLOAT,
//     proxy_classes.hpp:67,100, is gone).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "dlnb/bootstrap.hpp"
#include "dlnb/common.hpp"
#include "dlnb/device.hpp"

namespace dlnb {

enum class CollKind : int { AllReduce, AllGather, ReduceScatter, AllToAll, SendRecv };

class Communicator {
 public:
  virtual ~Communicator() = default;
  int rank() const { return rank_; }
  int size() const { return size_; }
  const std::vector<int>& members() const { return members_; }  // world ranks
  const std::string& name() const { return name_; }
  virtual std::string backend_name() const = 0;

  // count = elements per rank; send/recv may alias (in place).
  virtual void all_reduce(const void* send, void* recv, size_t count, DType t, Stream& s) = 0;
  // recv holds size()*send_count elements, rank-major.
  virtual void all_gather(const void* send, void* recv, size_t send_count, DType t, Stream& s) = 0;
  // send holds size()*recv_count elements; recv gets this rank's reduced block.
  virtual void reduce_scatter(const void* send, void* recv, size_t recv_count, DType t, Stream& s) = 0;
  // send/recv hold size()*count elements; block j goes to / comes from rank j.
  virtual void all_to_all(const void* send, void* recv, size_t count, DType t, Stream& s) = 0;
  // Point-to-point by group rank. Between group_start()/group_end() the
  // operations progress together (no ordering deadlocks between a send and
  // a recv issued in the same group).
  virtual void send(const void* buf, size_t count, DType t, int peer, Stream& s) = 0;
  virtual void recv(void* buf, size_t count, DType t, int peer, Stream& s) = 0;
  virtual void group_start() {}
  virtual void group_end() {}
  // Zero-copy registration (collective: every member registers its buffer
  // of the same role, in the same order). A backend that moves data with
  // its own kernels can then read a peer's registered send buffer and write
  // a peer's registered receive buffer directly instead of staging through
  // its windows; an operation takes the direct path when its buffers are
  // registered, so registrations and their use must be symmetric across
  // members (the ncclCommRegister rule). wants_peer_buffers(): allocate
  // such buffers with Device::alloc_peer and register them.
  virtual bool wants_peer_buffers() const { return false; }
  virtual void register_buffer(void* p, size_t bytes) { (void)p, (void)bytes; }
  // Returns a non-empty description if the backend detected an
  // asynchronous failure (peer death, network error).
  virtual std::string async_error() { return ""; }
  virtual void abort() {}
  // Ranks the underlying library says the communicator has (RCCL:
  // ncclCommCount), -1 when the backend has no such library object. Reported
  // so a multi-GPU run shows that RCCL really formed an N-rank communicator.
  virtual int library_nranks() { return -1; }

 protected:
  int rank_ = 0;
  int size_ = 1;
  std::vector<int> members_;
  std::string name_;
};

// Creates communicators over subsets of the world.
class CommFactory {
 public:
  virtual ~CommFactory() = default;
  virtual std::string backend_name() const = 0;
  // `members` are world ranks (this rank must be one of them); `name` must
  // be unique per group and identical on all members. capacity_bytes is the
  // largest single message (CPU backend staging size); need_p2p requests
  // point-to-point mailboxes. max_ctas > 0 caps the thread blocks one
  // collective kernel of this communicator may use (RCCL ncclConfig_t
  // maxCTAs; the other backends size their own kernels and ignore it).
  virtual std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members,
                                               size_t capacity_bytes, bool need_p2p, int max_ctas = 0) = 0;
};

std::unique_ptr<CommFactory> make_rccl_factory(HostGroup& world, Device& dev);
std::unique_ptr<CommFactory> make_shm_factory(HostGroup& world, Device& dev);
// Own kernels over IPC-mapped peer windows (one node); see dlnb/xgmi.hpp.
std::unique_ptr<CommFactory> make_xgmi_factory(HostGroup& world, Device& dev);
// Size-based dispatch: xgmi kernels for small messages inside a node, RCCL
// otherwise (comm_mixed.cpp).
std::unique_ptr<CommFactory> make_mixed_factory(HostGroup& world, Device& dev);

// Loopback: N ranks as threads of one process on one device (GPU or CPU),
// sharing one LoopbackHub. Collectives are issued by the last rank to
// arrive, on its own stream, after waiting on every other rank's "ready"
// event; the others wait on its "done" event. Host enqueue order therefore
// orders every dependency, so no stream can wait on work queued behind it
// even when all ranks' streams share the device's few hardware queues.
struct LoopbackHub;
std::shared_ptr<LoopbackHub> make_loopback_hub(int ranks, double timeout_s);
// Wakes every rank blocked in the hub with an error (a rank thread failed).
void loopback_abort(LoopbackHub& hub, const std::string& why);
// The job's CPU abort switch (loopback-cpu devices are created with it;
// loopback_abort sets it).
AbortFlag loopback_cpu_abort_flag(LoopbackHub& hub);
// A rank thread is done with the job: its streams are drained, nothing of it
// is still queued. With `wait`, also blocks (up to timeout_s) until every
// rank of the job is: a failing rank frees its buffers and events only once
// no other rank's queued copy or event wait can still reference them.
void loopback_drained(LoopbackHub& hub, bool wait, double timeout_s);
std::unique_ptr<CommFactory> make_loopback_factory(HostGroup& world, Device& dev, std::shared_ptr<LoopbackHub> hub);

// DLNB_COMM_FAULT set: wraps every communicator of `inner` in a fault
// injector (comm_fault.cpp: swap parts of an op's output, or skip the op);
// otherwise returns inner. Tests of the exactness checks only.
std::unique_ptr<CommFactory> wrap_comm_faults(std::unique_ptr<CommFactory> inner, Device& dev, int world_rank);

// Host-memory helpers of the CPU backends (multi-threaded for large sizes).
// dst[i] = sum over srcs of src[i] (fp32 accumulation); dst may alias a src.
void host_reduce_sum(DType t, void* dst, const std::vector<const char*>& srcs, size_t count);
void host_copy(void* dst, const void* src, size_t bytes);

// Bytes moved per rank for bus-bandwidth accounting (nccl-tests convention):
// busbw = algbw * factor(kind, n).
double busbw_factor(CollKind k, int n);

}  // namespace dlnb
