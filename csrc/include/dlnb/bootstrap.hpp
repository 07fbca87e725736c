// Process bootstrap without MPI.
//
// The reference bootstraps everything through MPI: MPI_Init, MPI_Comm_split,
// MPI_Bcast of the ncclUniqueId (cpp/data_parallel/dp.cpp:166-188), the
// run-count reduction (cpp/utils.hpp:121-135), local-rank discovery via
// MPI_Comm_split_type(SHARED) (cpp/utils.hpp:74-117) and the topology gather
// (cpp/netcommunicators.hpp:19-47). There is no MPI on the target image, so
// the runtime hosts its own rendezvous: rank 0 runs a small TCP key/value
// store, every rank connects to it, and all host-side coordination (unique-id
// exchange, barriers, gathers of per-rank reports, max-reductions of timers)
// is built on set/get/add. Rank identity comes from the launcher's
// environment (our dlnb launcher, torchrun, Open MPI, Slurm or PMI).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dlnb {

class Store {
 public:
  virtual ~Store() = default;
  virtual void set(const std::string& key, const std::string& value) = 0;
  // Blocks until the key exists (bounded by the store timeout).
  virtual std::string get(const std::string& key) = 0;
  // Atomically adds delta to an integer key (missing = 0); returns the new value.
  virtual long long add(const std::string& key, long long delta) = 0;
  // The job completed cleanly: a server-side store keeps serving until the
  // other ranks disconnect (bounded), so none loses the final barrier reply.
  virtual void finish() {}
};

// In-process store: world_size == 1, or the rank threads of a loopback job.
class LocalStore : public Store {
 public:
  void set(const std::string& key, const std::string& value) override;
  std::string get(const std::string& key) override;
  long long add(const std::string& key, long long delta) override;
  // Every blocked and later get() throws (a rank thread of the job failed).
  void abort(const std::string& why);

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::string> kv_;
  std::string aborted_;
};

// TCP store. The server side (rank 0) runs an accept thread plus one thread
// per client; every rank (including 0) talks to it through a client socket.
class TcpStore : public Store {
 public:
  // is_server: bind host:port (port 0 = ephemeral; read back with port()).
  TcpStore(const std::string& host, int port, bool is_server, double timeout_s);
  ~TcpStore() override;
  void set(const std::string& key, const std::string& value) override;
  std::string get(const std::string& key) override;
  long long add(const std::string& key, long long delta) override;
  void finish() override;
  int port() const { return port_; }

 private:
  struct Server;
  std::string request(uint8_t op, const std::string& key, const std::string& value);
  std::unique_ptr<Server> server_;
  int fd_ = -1;
  int port_ = 0;
  double timeout_s_;
  std::mutex mu_;
};

// Identity of this process within the job.
struct RankInfo {
  int rank = 0;
  int world_size = 1;
  int local_rank = 0;  // index among ranks on the same host
  int local_size = 1;
  std::string hostname;
};

// Host-side process group built on a Store: the MPI_COMM_WORLD replacement.
class HostGroup {
 public:
  HostGroup(std::shared_ptr<Store> store, int rank, int world, std::string ns = "w");
  int rank() const { return rank_; }
  int size() const { return world_; }
  Store& store() { return *store_; }
  std::shared_ptr<Store> store_ptr() { return store_; }

  void barrier();
  std::vector<std::string> allgather(const std::string& value);
  std::string broadcast(const std::string& value, int root);
  double allreduce_max(double v);
  double allreduce_sum(double v);
  // Fresh key prefix, identical on all ranks that call it in the same order.
  std::string next_tag(const char* what);

 private:
  std::shared_ptr<Store> store_;
  int rank_, world_;
  std::string ns_;
  uint64_t seq_ = 0;
};

// Reads rank/world from the environment (DLNB_*, torchrun, OMPI, PMI, Slurm),
// connects to (or hosts) the store and derives local rank from hostnames
// when the launcher did not provide it.
struct LoopbackHub;
struct Bootstrap {
  RankInfo info;
  std::shared_ptr<Store> store;
  std::unique_ptr<HostGroup> world;
  std::shared_ptr<LoopbackHub> hub;  // loopback backend: shared by the job's rank threads
};

// Rank `rank` of an in-process loopback job of `world` threads that share
// `store` and `hub` (--backend loopback --ranks N).
std::unique_ptr<Bootstrap> bootstrap_loopback(int rank, int world, std::shared_ptr<LocalStore> store,
                                              std::shared_ptr<LoopbackHub> hub);

// store_addr: "host:port" (empty = from env DLNB_STORE_ADDR, else
// MASTER_ADDR:(MASTER_PORT+1), else 127.0.0.1:29600).
std::unique_ptr<Bootstrap> bootstrap_from_env(const std::string& store_addr = "");

std::string get_hostname();

}  // namespace dlnb
