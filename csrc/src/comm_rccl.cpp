// RCCL backend (collectives over xGMI inside a node, network across nodes).
//
// Reference equivalent: CCLCommunicator, cpp/proxy_classes.hpp:135-253, plus
// the per-driver MPI_Bcast of ncclUniqueId (e.g. cpp/hybrid_parallel/
// hybrid_3d.cpp:330-366). Here unique ids travel through the TCP store and
// every op is enqueued on the caller's stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cstring>
#include <sstream>

#include "dlnb/comm.hpp"
#include "dlnb/json.hpp"

#define DLNB_NCCL_CHECK(expr)                                                            \
  do {                                                                                   \
    ncclResult_t r_ = (expr);                                                            \
    if (r_ != ncclSuccess) DLNB_THROW(#expr << " failed: " << ncclGetErrorString(r_));   \
  } while (0)

namespace dlnb {

namespace {

ncclDataType_t to_nccl(DType t) {
  switch (t) {
    case DType::BF16: return ncclBfloat16;
    case DType::FP16: return ncclFloat16;
    case DType::FP32: return ncclFloat32;
    case DType::FP8_E4M3: return static_cast<ncclDataType_t>(10);  // ncclFloat8e4m3 (RCCL >= 2.24)
    case DType::FP8_E5M2: return static_cast<ncclDataType_t>(11);  // ncclFloat8e5m2
  }
  return ncclBfloat16;
}

hipStream_t hs(Stream& s) { return static_cast<hipStream_t>(s.native()); }

class RcclComm : public Communicator {
 public:
  RcclComm(const std::string& name, const std::vector<int>& members, int my_world_rank, HostGroup& world,
           int max_ctas) {
    name_ = name;
    members_ = members;
    size_ = static_cast<int>(members.size());
    rank_ = -1;
    for (int i = 0; i < size_; ++i)
      if (members[i] == my_world_rank) rank_ = i;
    DLNB_REQUIRE(rank_ >= 0, "rank " << my_world_rank << " is not a member of group " << name);
    std::ostringstream key;
    key << "rccl/" << name << "/";
    for (int m : members) key << m << ",";
    key << "/uid";
    ncclUniqueId id;
    if (rank_ == 0) {
      DLNB_NCCL_CHECK(ncclGetUniqueId(&id));
      world.store().set(key.str(), std::string(reinterpret_cast<const char*>(&id), sizeof(id)));
    } else {
      std::string v = world.store().get(key.str());
      DLNB_REQUIRE(v.size() == sizeof(id), "bad unique id size for " << name);
      std::memcpy(&id, v.data(), sizeof(id));
    }
    // CTA budget (runner.cpp: lanes x max_ctas <= the CUs the persistent
    // compute leaves free), so every block of every concurrently live
    // collective finds a CU and no kernel of one communicator can hold CUs
    // that a peer's kernel of another communicator waits for.
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    if (max_ctas > 0) cfg.maxCTAs = max_ctas;
    cfg.commName = name_.c_str();
    DLNB_NCCL_CHECK(ncclCommInitRankConfig(&comm_, size_, id, rank_, &cfg));
  }
  ~RcclComm() override {
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  std::string backend_name() const override { return "RCCL"; }

  void all_reduce(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    DLNB_NCCL_CHECK(ncclAllReduce(send, recv, count, to_nccl(t), ncclSum, comm_, hs(s)));
  }
  void all_gather(const void* send, void* recv, size_t send_count, DType t, Stream& s) override {
    DLNB_NCCL_CHECK(ncclAllGather(send, recv, send_count, to_nccl(t), comm_, hs(s)));
  }
  void reduce_scatter(const void* send, void* recv, size_t recv_count, DType t, Stream& s) override {
    DLNB_NCCL_CHECK(ncclReduceScatter(send, recv, recv_count, to_nccl(t), ncclSum, comm_, hs(s)));
  }
  void all_to_all(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    DLNB_NCCL_CHECK(ncclAllToAll(send, recv, count, to_nccl(t), comm_, hs(s)));
  }
  void send(const void* buf, size_t count, DType t, int peer, Stream& s) override {
    DLNB_NCCL_CHECK(ncclSend(buf, count, to_nccl(t), peer, comm_, hs(s)));
  }
  void recv(void* buf, size_t count, DType t, int peer, Stream& s) override {
    DLNB_NCCL_CHECK(ncclRecv(buf, count, to_nccl(t), peer, comm_, hs(s)));
  }
  void group_start() override { DLNB_NCCL_CHECK(ncclGroupStart()); }
  void group_end() override { DLNB_NCCL_CHECK(ncclGroupEnd()); }
  std::string async_error() override {
    ncclResult_t r = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
    if (r != ncclSuccess && r != ncclInProgress) return std::string("RCCL async error in ") + name_ + ": " + ncclGetErrorString(r);
    return "";
  }
  void abort() override {
    if (comm_) {
      (void)ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  int library_nranks() override {
    int n = -1;
    if (comm_ && ncclCommCount(comm_, &n) != ncclSuccess) n = -1;
    return n;
  }

 private:
  ncclComm_t comm_ = nullptr;
};

class RcclFactory : public CommFactory {
 public:
  RcclFactory(HostGroup& world, Device& dev) : world_(world), dev_(dev) {
    DLNB_REQUIRE(dev.kind() == DeviceKind::GPU, "the RCCL backend needs a GPU device");
  }
  std::string backend_name() const override { return "RCCL"; }
  std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members, size_t,
                                       bool, int max_ctas) override {
    (void)hipSetDevice(dev_.index());
    return std::unique_ptr<Communicator>(new RcclComm(name, members, world_.rank(), world_, max_ctas));
  }

 private:
  HostGroup& world_;
  Device& dev_;
};

}  // namespace

std::unique_ptr<CommFactory> make_rccl_factory(HostGroup& world, Device& dev) {
  return std::unique_ptr<CommFactory>(new RcclFactory(world, dev));
}

namespace {
std::string lib_of(const void* sym) {
  Dl_info info;
  if (dladdr(sym, &info) && info.dli_fname) return info.dli_fname;
  return "?";
}
}  // namespace

Json runtime_info() {
  // Which HIP runtime and RCCL this process bound (a process that imported
  // torch first binds torch's bundled copies; the CLI binaries and bench.py,
  // which never import torch, bind /opt/rocm's).
  Json j = Json::object();
  int v = 0;
  if (ncclGetVersion(&v) == ncclSuccess) {
    j["rccl_version_code"] = v;
    std::ostringstream s;
    s << v / 10000 << "." << (v / 100) % 100 << "." << v % 100;
    j["rccl_version"] = s.str();
  }
  j["librccl"] = lib_of(reinterpret_cast<const void*>(&ncclGetVersion));
  int hv = 0;
  if (hipRuntimeGetVersion(&hv) == hipSuccess) j["hip_runtime_version"] = hv;
  j["libamdhip64"] = lib_of(reinterpret_cast<const void*>(&hipRuntimeGetVersion));
  return j;
}

double busbw_factor(CollKind k, int n) {
  // nccl-tests convention: a 1-rank collective moves nothing over a link
  // (RCCL runs it as a local device copy), so its bus bandwidth is 0.
  if (n <= 1) return 0.0;
  switch (k) {
    case CollKind::AllReduce: return 2.0 * (n - 1) / n;
    case CollKind::AllGather:
    case CollKind::ReduceScatter:
    case CollKind::AllToAll: return static_cast<double>(n - 1) / n;
    case CollKind::SendRecv: return 1.0;
  }
  return 1.0;
}

}  // namespace dlnb
