#include "dlnb/bootstrap.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cerrno>
#include <cstring>
#include <fstream>
#include <sstream>
#include <thread>

#include "dlnb/common.hpp"

namespace dlnb {

namespace {

enum Op : uint8_t { OP_SET = 1, OP_GET = 2, OP_ADD = 3 };

void write_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      DLNB_THROW("store socket write failed: " << std::strerror(errno));
    }
    p += w;
    n -= static_cast<size_t>(w);
  }
}

bool read_all(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n > 0) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

void write_blob(int fd, const std::string& s) {
  uint32_t n = static_cast<uint32_t>(s.size());
  write_all(fd, &n, 4);
  if (n) write_all(fd, s.data(), n);
}

bool read_blob(int fd, std::string& s) {
  uint32_t n = 0;
  if (!read_all(fd, &n, 4)) return false;
  s.resize(n);
  return n == 0 || read_all(fd, &s[0], n);
}

}  // namespace

// ---------------------------------------------------------------- LocalStore

void LocalStore::set(const std::string& key, const std::string& value) {
  std::lock_guard<std::mutex> g(mu_);
  kv_[key] = value;
  cv_.notify_all();
}

std::string LocalStore::get(const std::string& key) {
  std::unique_lock<std::mutex> g(mu_);
  if (!cv_.wait_for(g, std::chrono::seconds(600), [&] { return kv_.count(key) > 0 || !aborted_.empty(); }))
    DLNB_THROW("local store: timeout waiting for key " << key);
  if (!kv_.count(key)) DLNB_THROW("local store: abandoned waiting for key " << key << ": " << aborted_);
  return kv_[key];
}

void LocalStore::abort(const std::string& why) {
  std::lock_guard<std::mutex> g(mu_);
  if (aborted_.empty()) aborted_ = why.empty() ? "aborted" : why;
  cv_.notify_all();
}

long long LocalStore::add(const std::string& key, long long delta) {
  std::lock_guard<std::mutex> g(mu_);
  long long v = kv_.count(key) ? std::stoll(kv_[key]) : 0;
  v += delta;
  kv_[key] = std::to_string(v);
  cv_.notify_all();
  return v;
}

// ------------------------------------------------------------------ TcpStore

struct TcpStore::Server {
  int listen_fd = -1;
  std::atomic<bool> stop{false};
  std::thread acceptor;
  std::vector<std::thread> workers;
  std::vector<int> client_fds;
  int active = 0;    // connected clients
  int linger_s = 0;  // set by finish()
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::string, std::string> kv;

  void serve(int fd) {
    for (;;) {
      uint8_t op = 0;
      if (!read_all(fd, &op, 1)) break;
      std::string key, val;
      if (!read_blob(fd, key) || !read_blob(fd, val)) break;
      try {
        if (op == OP_SET) {
          {
            std::lock_guard<std::mutex> g(mu);
            kv[key] = val;
          }
          cv.notify_all();
          write_blob(fd, "");
        } else if (op == OP_GET) {
          std::string out;
          {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return stop.load() || kv.count(key) > 0; });
            if (!kv.count(key)) break;  // stopping and the key never came
            out = kv[key];
          }
          write_blob(fd, out);
        } else if (op == OP_ADD) {
          long long v;
          {
            std::lock_guard<std::mutex> g(mu);
            v = kv.count(key) ? std::stoll(kv[key]) : 0;
            v += std::stoll(val);
            kv[key] = std::to_string(v);
          }
          cv.notify_all();
          write_blob(fd, std::to_string(v));
        } else {
          break;
        }
      } catch (...) {
        break;
      }
    }
    ::close(fd);
    {
      std::lock_guard<std::mutex> g(mu);
      --active;
    }
    cv.notify_all();
  }

  void accept_loop() {
    while (!stop.load()) {
      pollfd p{listen_fd, POLLIN, 0};
      int r = ::poll(&p, 1, 200);
      if (r <= 0) continue;
      int fd = ::accept(listen_fd, nullptr, nullptr);
      if (fd < 0) continue;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      std::lock_guard<std::mutex> g(mu);
      client_fds.push_back(fd);
      ++active;
      workers.emplace_back([this, fd] { serve(fd); });
    }
  }

  ~Server() {
    // Graceful first: the other ranks close their connections when they exit;
    // tearing the server down while one of them still waits for the reply of
    // the final barrier would fail that rank. Give them a bounded grace.
    {
      std::unique_lock<std::mutex> g(mu);
      cv.wait_for(g, std::chrono::seconds(linger_s), [&] { return active == 0; });
    }
    stop.store(true);
    cv.notify_all();
    if (acceptor.joinable()) acceptor.join();
    {
      std::lock_guard<std::mutex> g(mu);
      for (int fd : client_fds) ::shutdown(fd, SHUT_RDWR);
    }
    for (auto& t : workers)
      if (t.joinable()) t.join();
    if (listen_fd >= 0) ::close(listen_fd);
  }
};

TcpStore::TcpStore(const std::string& host, int port, bool is_server, double timeout_s)
    : port_(port), timeout_s_(timeout_s) {
  if (is_server) {
    server_.reset(new Server());
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) DLNB_THROW("socket() failed");
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
    addr.sin_port = htons(static_cast<uint16_t>(port));
    if (::bind(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
      ::close(fd);
      DLNB_THROW("store: cannot bind port " << port << ": " << std::strerror(errno));
    }
    if (::listen(fd, 1024) != 0) DLNB_THROW("store: listen failed");
    socklen_t len = sizeof(addr);
    getsockname(fd, reinterpret_cast<sockaddr*>(&addr), &len);
    port_ = ntohs(addr.sin_port);
    server_->listen_fd = fd;
    server_->acceptor = std::thread([this] { server_->accept_loop(); });
  }
  // Connect (retry until the server is up or the timeout expires).
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    std::string h = is_server ? std::string("127.0.0.1") : host;
    if (getaddrinfo(h.c_str(), std::to_string(port_).c_str(), &hints, &res) == 0 && res) {
      int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        // A blocking get() gives up after the store timeout: a rank that died
        // or hangs before a host barrier fails the job instead of hanging it.
        timeval tv;
        tv.tv_sec = static_cast<long>(timeout_s_);
        tv.tv_usec = 0;
        setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        fd_ = fd;
        break;
      }
      if (fd >= 0) ::close(fd);
      freeaddrinfo(res);
    }
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > timeout_s_) DLNB_THROW("store: cannot connect to " << host << ":" << port_ << " within " << timeout_s_ << " s");
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

TcpStore::~TcpStore() {
  if (fd_ >= 0) ::close(fd_);
  server_.reset();
}

std::string TcpStore::request(uint8_t op, const std::string& key, const std::string& value) {
  std::lock_guard<std::mutex> g(mu_);
  write_all(fd_, &op, 1);
  write_blob(fd_, key);
  write_blob(fd_, value);
  std::string out;
  if (!read_blob(fd_, out))
    DLNB_THROW("store: no reply within " << timeout_s_ << " s or connection lost (op " << int(op) << " key " << key
                                         << "): a peer rank died or hangs");
  return out;
}

void TcpStore::finish() {
  if (server_) server_->linger_s = static_cast<int>(env_int("DLNB_STORE_LINGER", 30));
}

void TcpStore::set(const std::string& key, const std::string& value) { request(OP_SET, key, value); }
std::string TcpStore::get(const std::string& key) { return request(OP_GET, key, ""); }
long long TcpStore::add(const std::string& key, long long delta) {
  return std::stoll(request(OP_ADD, key, std::to_string(delta)));
}

// ---------------------------------------------------------------- HostGroup

HostGroup::HostGroup(std::shared_ptr<Store> store, int rank, int world, std::string ns)
    : store_(std::move(store)), rank_(rank), world_(world), ns_(std::move(ns)) {}

std::string HostGroup::next_tag(const char* what) {
  std::ostringstream os;
  os << ns_ << "/" << what << "/" << seq_++;
  return os.str();
}

void HostGroup::barrier() {
  if (world_ == 1) return;
  std::string tag = next_tag("barrier");
  long long n = store_->add(tag + "/cnt", 1);
  if (n == world_) store_->set(tag + "/go", "1");
  store_->get(tag + "/go");
}

std::vector<std::string> HostGroup::allgather(const std::string& value) {
  std::vector<std::string> out(static_cast<size_t>(world_));
  if (world_ == 1) {
    out[0] = value;
    return out;
  }
  std::string tag = next_tag("allgather");
  store_->set(tag + "/" + std::to_string(rank_), value);
  for (int r = 0; r < world_; ++r) out[static_cast<size_t>(r)] = store_->get(tag + "/" + std::to_string(r));
  return out;
}

std::string HostGroup::broadcast(const std::string& value, int root) {
  if (world_ == 1) return value;
  std::string tag = next_tag("bcast");
  if (rank_ == root) {
    store_->set(tag, value);
    return value;
  }
  return store_->get(tag);
}

double HostGroup::allreduce_max(double v) {
  double m = v;
  for (const auto& s : allgather(std::to_string(v))) m = std::max(m, std::stod(s));
  return m;
}

double HostGroup::allreduce_sum(double v) {
  auto all = allgather(std::to_string(v));
  double s = 0;
  for (const auto& x : all) s += std::stod(x);
  return s;
}

// ---------------------------------------------------------------- bootstrap

std::string get_hostname() {
  char buf[256] = {0};
  if (gethostname(buf, sizeof(buf) - 1) != 0) return "unknown";
  return buf;
}

namespace {

int first_env_int(std::initializer_list<const char*> names, int dflt) {
  for (const char* n : names) {
    long long v = env_int(n, -1);
    if (v >= 0) return static_cast<int>(v);
  }
  return dflt;
}

}  // namespace

std::unique_ptr<Bootstrap> bootstrap_loopback(int rank, int world, std::shared_ptr<LocalStore> store,
                                              std::shared_ptr<LoopbackHub> hub) {
  std::unique_ptr<Bootstrap> b(new Bootstrap());
  b->info.rank = rank;
  b->info.world_size = world;
  b->info.local_rank = rank;
  b->info.local_size = world;
  b->info.hostname = get_hostname();
  b->store = store;
  b->world.reset(new HostGroup(store, rank, world));
  b->hub = std::move(hub);
  return b;
}

std::unique_ptr<Bootstrap> bootstrap_from_env(const std::string& store_addr_in) {
  std::unique_ptr<Bootstrap> b(new Bootstrap());
  RankInfo& ri = b->info;
  ri.rank = first_env_int({"DLNB_RANK", "RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID"}, 0);
  ri.world_size =
      first_env_int({"DLNB_WORLD_SIZE", "WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS"}, 1);
  ri.hostname = get_hostname();
  DLNB_REQUIRE(ri.world_size >= 1 && ri.rank >= 0 && ri.rank < ri.world_size,
               "bad rank/world from environment: rank=" << ri.rank << " world=" << ri.world_size);
  double timeout = static_cast<double>(env_int("DLNB_STORE_TIMEOUT", 900));

  if (ri.world_size == 1) {
    b->store = std::make_shared<LocalStore>();
  } else {
    std::string addr = store_addr_in.empty() ? env_or("DLNB_STORE_ADDR", "") : store_addr_in;
    const std::string file = env_or("DLNB_STORE_FILE", "");
    std::string host;
    int port;
    if (addr.empty() && !file.empty()) {
      // File rendezvous: rank 0 serves on an ephemeral port and publishes
      // host:port (write + rename, so readers never see a partial file); no
      // port is chosen ahead of time, so none can be taken in between.
      if (ri.rank == 0) {
        auto st = std::make_shared<TcpStore>("127.0.0.1", 0, true, timeout);
        const std::string tmp = file + ".tmp";
        {
          std::ofstream f(tmp);
          f << env_or("DLNB_STORE_HOST", "127.0.0.1") << ":" << st->port() << "\n";
        }
        DLNB_REQUIRE(std::rename(tmp.c_str(), file.c_str()) == 0, "cannot publish the store address to " << file);
        b->store = st;
      } else {
        auto t0 = std::chrono::steady_clock::now();
        std::string line;
        for (;;) {
          std::ifstream f(file);
          if (f && std::getline(f, line) && !line.empty()) break;
          DLNB_REQUIRE(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < timeout,
                       "rank 0 never published the store address in " << file);
          std::this_thread::sleep_for(std::chrono::milliseconds(20));
        }
        size_t c = line.rfind(':');
        b->store = std::make_shared<TcpStore>(line.substr(0, c), std::stoi(line.substr(c + 1)), false, timeout);
      }
    } else if (!addr.empty()) {
      size_t c = addr.rfind(':');
      DLNB_REQUIRE(c != std::string::npos, "store address must be host:port, got " << addr);
      host = addr.substr(0, c);
      port = std::stoi(addr.substr(c + 1));
    } else {
      host = env_or("MASTER_ADDR", "127.0.0.1");
      port = static_cast<int>(env_int("DLNB_STORE_PORT", env_int("MASTER_PORT", 29599) + 1));
    }
    if (!b->store) b->store = std::make_shared<TcpStore>(host, port, ri.rank == 0, timeout);
  }
  b->world.reset(new HostGroup(b->store, ri.rank, ri.world_size, "world"));

  // Local rank: prefer the launcher's value; otherwise count lower ranks on
  // this host (the MPI_Comm_split_type(SHARED) equivalent).
  auto hosts = b->world->allgather(ri.hostname);
  int lr = 0, ls = 0;
  for (int r = 0; r < ri.world_size; ++r) {
    if (hosts[static_cast<size_t>(r)] == ri.hostname) {
      if (r < ri.rank) ++lr;
      ++ls;
    }
  }
  ri.local_rank = first_env_int({"DLNB_LOCAL_RANK", "LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
                                 "SLURM_LOCALID"},
                                lr);
  ri.local_size = first_env_int({"DLNB_LOCAL_WORLD_SIZE", "LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE"}, ls);
  return b;
}

}  // namespace dlnb
