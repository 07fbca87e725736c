// CPU shared-memory backend: multi-process collectives and point-to-point on
// host buffers, executed on the CPU device's worker-thread streams.
//
// Reference equivalent: the mpi_cpu build (MPICommunicator over calloc'd host
// buffers, cpp/proxy_classes.hpp:53-133, README.md:96), which lets every
// strategy run on a laptop with `mpirun -n N`. MPI is not available on the
// target image, so ranks on one host exchange data through a POSIX shm
// segment per communicator: W staging slots + a result region for
// collectives, and one single-slot mailbox per (src, dst) pair for P2P.
// Synchronisation is a sense-reversing barrier on futexes in the segment.
//
// Zero-copy: buffers allocated with Device::alloc_peer (memfd mappings) and
// registered with the communicator are mapped by every member, so a
// collective on them reads and writes the members' buffers directly: an
// all-reduce moves 2x its bytes per rank (read every member's chunk, write
// the sum into every member's copy) instead of 4.5x through the staging slots.
#include <fcntl.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <atomic>
#include <deque>
#include <cstring>
#include <sstream>
#include <thread>
#include <vector>

#include "dlnb/comm.hpp"
#include "dlnb/host_simd.hpp"

namespace dlnb {

namespace {

constexpr size_t kHeader = 4096;
constexpr size_t kAlign = 4096;

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

struct SegHeader {
  std::atomic<uint32_t> count;
  std::atomic<uint32_t> gen;
  std::atomic<uint32_t> attached;
  uint32_t world;
  uint64_t capacity;
};

struct Mailbox {
  std::atomic<uint32_t> sent;  // futex word
  std::atomic<uint32_t> taken;  // futex word
  uint64_t bytes;
  char pad[48];
};
static_assert(sizeof(Mailbox) == 64, "mailbox header must be one cache line");

long futex(std::atomic<uint32_t>* addr, int op, uint32_t val) {
  timespec ts{0, 2000000};  // 2 ms: re-check deadlines periodically
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, op == FUTEX_WAIT ? &ts : nullptr, nullptr, 0);
}

// Wait until pred() holds; spins briefly, then sleeps on the futex word.
template <typename Pred>
void wait_on(std::atomic<uint32_t>* word, Pred pred, double timeout_s, const char* what) {
  for (int i = 0; i < 2000; ++i) {
    if (pred()) return;
    if (i > 200) sched_yield();
  }
  double t0 = now_s();
  while (!pred()) {
    uint32_t v = word->load(std::memory_order_acquire);
    if (pred()) return;
    futex(word, FUTEX_WAIT, v);
    if (now_s() - t0 > timeout_s) DLNB_THROW("shm backend: timeout in " << what << " after " << timeout_s << " s");
  }
}

void wake(std::atomic<uint32_t>* word) { futex(word, FUTEX_WAKE, INT32_MAX); }

// Sum n elements starting at element off of every source into dst, blockwise
// through an fp32 accumulator (vectorisable inner loops).
void reduce_sum(DType t, void* dst, const std::vector<const char*>& srcs, size_t off, size_t n) {
  const size_t es = dtype_size(t);
  if (srcs.size() == 1) {
    std::memcpy(dst, srcs[0] + off * es, n * es);
    return;
  }
  constexpr size_t BLK = 4096;
  float acc[BLK];
  for (size_t b = 0; b < n; b += BLK) {
    const size_t m = std::min(BLK, n - b);
    const size_t e0 = off + b;
    if (t == DType::BF16)  // the first source initialises the accumulator (one pass fewer)
      simd::set_bf16(acc, reinterpret_cast<const uint16_t*>(srcs[0]) + e0, m);
    else
      for (size_t i = 0; i < m; ++i) acc[i] = 0.f;
    for (size_t si = t == DType::BF16 ? 1 : 0; si < srcs.size(); ++si) {
      const char* s = srcs[si];
      switch (t) {
        case DType::BF16:
          simd::acc_bf16(acc, reinterpret_cast<const uint16_t*>(s) + e0, m);
          break;
        case DType::FP32:
          simd::acc_f32(acc, reinterpret_cast<const float*>(s) + e0, m);
          break;
        case DType::FP16: {
          const uint16_t* p = reinterpret_cast<const uint16_t*>(s) + e0;
          for (size_t i = 0; i < m; ++i) acc[i] += fp16_to_float(p[i]);
          break;
        }
        case DType::FP8_E4M3: {
          const uint8_t* p = reinterpret_cast<const uint8_t*>(s) + e0;
          for (size_t i = 0; i < m; ++i) acc[i] += fp8e4m3_to_float(p[i]);
          break;
        }
        case DType::FP8_E5M2: {
          const uint8_t* p = reinterpret_cast<const uint8_t*>(s) + e0;
          for (size_t i = 0; i < m; ++i) acc[i] += fp8e5m2_to_float(p[i]);
          break;
        }
      }
    }
    char* d = static_cast<char*>(dst) + b * es;
    switch (t) {
      case DType::BF16:
        simd::store_bf16(reinterpret_cast<uint16_t*>(d), acc, m);
        break;
      case DType::FP32: std::memcpy(d, acc, m * 4); break;
      case DType::FP16:
        for (size_t i = 0; i < m; ++i) reinterpret_cast<uint16_t*>(d)[i] = float_to_fp16(acc[i]);
        break;
      case DType::FP8_E4M3:
        for (size_t i = 0; i < m; ++i) reinterpret_cast<uint8_t*>(d)[i] = float_to_fp8e4m3(acc[i]);
        break;
      case DType::FP8_E5M2:
        for (size_t i = 0; i < m; ++i) reinterpret_cast<uint8_t*>(d)[i] = float_to_fp8e5m2(acc[i]);
        break;
    }
  }
}

// Large copies / reductions are split over a few threads: one core cannot
// saturate the socket's memory bandwidth. Threads per rank default to the
// host's cores divided by the ranks on it (DLNB_SHM_THREADS overrides).
int shm_threads() {
  static const int n = [] {
    long long env = env_int("DLNB_SHM_THREADS", 0);
    if (env > 0) return static_cast<int>(env);
    long long local = env_int("DLNB_LOCAL_WORLD_SIZE", env_int("LOCAL_WORLD_SIZE", 1));
    unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    return static_cast<int>(std::max<long long>(1, std::min<long long>(8, hw / std::max<long long>(1, local))));
  }();
  return n;
}

// Runs fn(lo, n) over [0, total) in up to shm_threads() pieces of at least
// min_piece elements; the calling thread takes the first piece.
template <typename F>
void par_range(size_t total, size_t min_piece, F fn) {
  size_t T = std::min<size_t>(static_cast<size_t>(shm_threads()), std::max<size_t>(1, total / min_piece));
  if (T <= 1) {
    fn(size_t(0), total);
    return;
  }
  size_t per = (total + T - 1) / T;
  std::vector<std::thread> th;
  for (size_t i = 1; i < T; ++i) {
    size_t lo = i * per;
    if (lo >= total) break;
    th.emplace_back([=] { fn(lo, std::min(per, total - lo)); });
  }
  fn(size_t(0), std::min(per, total));
  for (auto& t : th) t.join();
}

void par_copy(void* dst, const void* src, size_t bytes) {
  par_range(bytes, size_t(4) << 20, [=](size_t lo, size_t n) {
    std::memcpy(static_cast<char*>(dst) + lo, static_cast<const char*>(src) + lo, n);
  });
}

void par_reduce_sum(DType t, void* dst, const std::vector<const char*>& srcs, size_t off, size_t n) {
  const size_t es = dtype_size(t);
  par_range(n, size_t(1) << 20, [&, dst, off](size_t lo, size_t m) {
    reduce_sum(t, static_cast<char*>(dst) + lo * es, srcs, off + lo, m);
  });
}

class ShmComm : public Communicator {
 public:
  ShmComm(const std::string& name, const std::vector<int>& members, int my_world_rank, HostGroup& world,
          const std::string& job, size_t capacity, bool p2p)
      : world_(&world), job_(job), cap_(round_up(capacity ? capacity : 64, kAlign)), p2p_(p2p) {
    name_ = name;
    members_ = members;
    size_ = static_cast<int>(members.size());
    rank_ = -1;
    for (int i = 0; i < size_; ++i)
      if (members[i] == my_world_rank) rank_ = i;
    DLNB_REQUIRE(rank_ >= 0, "rank " << my_world_rank << " is not a member of group " << name);
    my_world_rank_ = my_world_rank;
    timeout_ = static_cast<double>(env_int("DLNB_TIMEOUT", 900));

    std::ostringstream key;
    key << "shm/" << name << "/";
    for (int m : members) key << m << ",";
    std::string shm_name = "/dlnb_" + job + "_" + std::to_string(std::hash<std::string>()(key.str()) & 0xffffffffffull);
    const size_t W = static_cast<size_t>(size_);
    slots_off_ = kHeader;
    result_off_ = slots_off_ + W * cap_;
    mbox_off_ = result_off_ + cap_;
    size_t mbox_bytes = p2p ? W * W * (64 + cap_) : 0;
    total_ = mbox_off_ + round_up(mbox_bytes, kAlign);

    int fd;
    if (rank_ == 0) {
      shm_unlink(shm_name.c_str());
      fd = shm_open(shm_name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) DLNB_THROW("shm_open(" << shm_name << ") failed: " << std::strerror(errno));
      if (ftruncate(fd, static_cast<off_t>(total_)) != 0) DLNB_THROW("ftruncate shm failed (" << total_ << " B)");
      base_ = static_cast<char*>(mmap(nullptr, total_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
      ::close(fd);
      if (base_ == MAP_FAILED) DLNB_THROW("mmap shm failed");
      hdr()->count.store(0);
      hdr()->gen.store(0);
      hdr()->attached.store(1);
      hdr()->world = static_cast<uint32_t>(W);
      hdr()->capacity = cap_;
      world.store().set(key.str() + "/ready", shm_name);
    } else {
      world.store().get(key.str() + "/ready");
      fd = shm_open(shm_name.c_str(), O_RDWR, 0600);
      if (fd < 0) DLNB_THROW("shm_open(" << shm_name << ") failed: " << std::strerror(errno));
      base_ = static_cast<char*>(mmap(nullptr, total_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
      ::close(fd);
      if (base_ == MAP_FAILED) DLNB_THROW("mmap shm failed");
      hdr()->attached.fetch_add(1);
    }
    barrier();
    if (rank_ == 0) shm_unlink(shm_name.c_str());  // mapping persists; no leak on crash
  }

  ~ShmComm() override {
    for (auto& m : mapped_) munmap(m.first, m.second);
    if (base_ && base_ != MAP_FAILED) munmap(base_, total_);
  }

  std::string backend_name() const override { return "CPU-SHM"; }

  bool wants_peer_buffers() const override { return size_ > 1; }

  // Collective, paired by order across members (the xgmi backend's rule):
  // every member maps every other member's k-th registered buffer.
  // If some member cannot map a peer's buffer (ranks in separate PID
  // namespaces or containers, /proc mounted hidepid), every member keeps the
  // registration slot but marks it unusable, so all of them take the staged
  // path for it (this used to throw on the failing rank only).
  void register_buffer(void* p, size_t bytes) override {
    Reg r;
    r.local = static_cast<char*>(p);
    r.bytes = bytes;
    r.peer.assign(static_cast<size_t>(size_), nullptr);
    r.peer[static_cast<size_t>(rank_)] = r.local;
    if (size_ > 1) {
      const std::string src = cpu_peer_source(p);
      DLNB_REQUIRE(!src.empty(), "shm backend: register_buffer needs a Device::alloc_peer allocation");
      std::ostringstream key;
      key << "shmreg/" << job_ << "/" << name_ << "/";
      for (int m : members_) key << m << ",";
      key << "reg" << regs_.size() << "/";
      world_->store().set(key.str() + std::to_string(rank_), src + " " + std::to_string(bytes));
      std::string why;
      std::vector<std::pair<void*, size_t>> mine;
      for (int q = 0; q < size_; ++q) {
        if (q == rank_) continue;
        std::istringstream in(world_->store().get(key.str() + std::to_string(q)));
        std::string path;
        size_t qb = 0;
        in >> path >> qb;
        DLNB_REQUIRE(qb == bytes, "shm: registration " << regs_.size() << " of " << name_ << ": rank " << q
                                                        << " registered " << qb << " B, this rank " << bytes);
        if (!why.empty()) continue;
        // DLNB_SHM_NO_PEER_MAP=R: rank R behaves as if /proc/<pid>/fd were hidden (tests)
        const int fd = env_int("DLNB_SHM_NO_PEER_MAP", -1) == my_world_rank_ ? -1 : ::open(path.c_str(), O_RDWR);
        if (fd < 0) {
          why = "cannot open peer buffer " + path + ": " + std::strerror(errno);
          continue;
        }
        void* a = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        ::close(fd);
        if (a == MAP_FAILED) {
          why = "cannot map peer buffer " + path;
          continue;
        }
        r.peer[static_cast<size_t>(q)] = static_cast<char*>(a);
        mine.emplace_back(a, bytes);
      }
      // every member's verdict: the registration is usable only if all mapped
      world_->store().set(key.str() + "ok/" + std::to_string(rank_), why.empty() ? "1" : "0");
      bool all_ok = true;
      for (int q = 0; q < size_; ++q) all_ok = all_ok && world_->store().get(key.str() + "ok/" + std::to_string(q)) == "1";
      if (!all_ok) {
        if (!why.empty() && !warned_)
          std::fprintf(stderr, "[dlnb] shm backend: %s; %s uses the staged (copy) path\n", why.c_str(), name_.c_str());
        warned_ = true;
        for (auto& m : mine) munmap(m.first, m.second);
        mine.clear();
        r.usable = false;
      }
      for (auto& m : mine) mapped_.push_back(m);
      // every member mapped every buffer before anyone may free one
      barrier();
    }
    regs_.push_back(std::move(r));
  }

  void all_reduce(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    const size_t bytes = count * dtype_size(t);
    size_t so = 0, ro = 0;
    const Reg* rs = find(send, bytes, so);
    const Reg* rr = find(recv, bytes, ro);
    if (rs && rr) {
      enqueue(s, [=] {
        const size_t es = dtype_size(t);
        barrier();  // every member's send is ready, its previous use of recv done
        size_t lo, n;
        chunk(count, rank_, lo, n);
        std::vector<const char*> srcs;
        for (int q = 0; q < size_; ++q) srcs.push_back(rs->peer[static_cast<size_t>(q)] + so);
        // this rank alone reads and writes chunk `rank_` of every member's buffers
        par_reduce_sum(t, rr->local + ro + lo * es, srcs, lo, n);
        for (int q = 0; q < size_; ++q)
          if (q != rank_) par_copy(rr->peer[static_cast<size_t>(q)] + ro + lo * es, rr->local + ro + lo * es, n * es);
        barrier();  // every chunk written everywhere; nobody reuses send while a peer reads it
      });
      return;
    }
    enqueue(s, [=] {
      const size_t es = dtype_size(t), bytes = count * es;
      check(bytes);
      par_copy(slot(rank_), send, bytes);
      barrier();
      size_t lo, n;
      chunk(count, rank_, lo, n);
      par_reduce_sum(t, base_ + result_off_ + lo * es, all_slots(), lo, n);
      barrier();
      par_copy(recv, base_ + result_off_, bytes);
      barrier();
    });
  }

  void all_gather(const void* send, void* recv, size_t send_count, DType t, Stream& s) override {
    size_t ro = 0;
    if (const Reg* rr = find(recv, send_count * dtype_size(t) * size_, ro)) {
      enqueue(s, [=] {
        const size_t bytes = send_count * dtype_size(t);
        barrier();
        for (int q = 0; q < size_; ++q)
          par_copy(rr->peer[static_cast<size_t>(q)] + ro + static_cast<size_t>(rank_) * bytes, send, bytes);
        barrier();
      });
      return;
    }
    enqueue(s, [=] {
      const size_t bytes = send_count * dtype_size(t);
      check(bytes);
      par_copy(slot(rank_), send, bytes);
      barrier();
      for (int r = 0; r < size_; ++r) par_copy(static_cast<char*>(recv) + r * bytes, slot(r), bytes);
      barrier();
    });
  }

  void reduce_scatter(const void* send, void* recv, size_t recv_count, DType t, Stream& s) override {
    size_t so = 0;
    if (const Reg* rs = find(send, recv_count * dtype_size(t) * size_, so)) {
      enqueue(s, [=] {
        barrier();
        std::vector<const char*> srcs;
        for (int q = 0; q < size_; ++q) srcs.push_back(rs->peer[static_cast<size_t>(q)] + so);
        par_reduce_sum(t, recv, srcs, recv_count * static_cast<size_t>(rank_), recv_count);
        barrier();
      });
      return;
    }
    enqueue(s, [=] {
      const size_t es = dtype_size(t), bytes = recv_count * es * size_;
      check(bytes);
      par_copy(slot(rank_), send, bytes);
      barrier();
      par_reduce_sum(t, recv, all_slots(), recv_count * rank_, recv_count);
      barrier();
    });
  }

  void all_to_all(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    size_t so = 0;
    const Reg* rs = send != recv ? find(send, count * dtype_size(t) * size_, so) : nullptr;
    if (rs) {
      enqueue(s, [=] {
        const size_t blk = count * dtype_size(t);
        barrier();
        for (int q = 0; q < size_; ++q)
          par_copy(static_cast<char*>(recv) + static_cast<size_t>(q) * blk,
                   rs->peer[static_cast<size_t>(q)] + so + static_cast<size_t>(rank_) * blk, blk);
        barrier();
      });
      return;
    }
    enqueue(s, [=] {
      const size_t blk = count * dtype_size(t);
      check(blk * size_);
      par_copy(slot(rank_), send, blk * size_);
      barrier();
      for (int r = 0; r < size_; ++r) par_copy(static_cast<char*>(recv) + r * blk, slot(r) + rank_ * blk, blk);
      barrier();
    });
  }

  void send(const void* buf, size_t count, DType t, int peer, Stream& s) override {
    const size_t bytes = count * dtype_size(t);
    auto op = [=] { do_send(buf, bytes, peer); };
    if (in_group_) {
      group_sends_.push_back(op);
      group_stream_ = &s;
    } else {
      enqueue(s, op);
    }
  }

  void recv(void* buf, size_t count, DType t, int peer, Stream& s) override {
    const size_t bytes = count * dtype_size(t);
    auto op = [=] { do_recv(buf, bytes, peer); };
    if (in_group_) {
      group_recvs_.push_back(op);
      group_stream_ = &s;
    } else {
      enqueue(s, op);
    }
  }

  // Group: all sends (buffered into mailboxes) go first, then the receives,
  // so a group never deadlocks on its own send/recv pairs.
  void group_start() override { in_group_ = true; }
  void group_end() override {
    in_group_ = false;
    if (!group_stream_) return;
    auto sends = std::move(group_sends_);
    auto recvs = std::move(group_recvs_);
    group_sends_.clear();
    group_recvs_.clear();
    Stream* s = group_stream_;
    group_stream_ = nullptr;
    enqueue(*s, [sends, recvs] {
      for (auto& f : sends) f();
      for (auto& f : recvs) f();
    });
  }

 private:
  SegHeader* hdr() { return reinterpret_cast<SegHeader*>(base_); }
  char* slot(int r) { return base_ + slots_off_ + static_cast<size_t>(r) * cap_; }
  Mailbox* mbox(int src, int dst) {
    return reinterpret_cast<Mailbox*>(base_ + mbox_off_ + (static_cast<size_t>(src) * size_ + dst) * (64 + cap_));
  }
  std::vector<const char*> all_slots() {
    std::vector<const char*> v;
    for (int r = 0; r < size_; ++r) v.push_back(slot(r));
    return v;
  }
  void check(size_t bytes) {
    if (bytes > cap_) DLNB_THROW("shm backend: message of " << bytes << " B exceeds group capacity " << cap_ << " B (" << name_ << ")");
  }
  void chunk(size_t count, int r, size_t& lo, size_t& n) {
    size_t base = count / size_, rem = count % size_;
    lo = r * base + std::min<size_t>(r, rem);
    n = base + (static_cast<size_t>(r) < rem ? 1 : 0);
  }
  void enqueue(Stream& s, std::function<void()> fn) {
    auto* cs = dynamic_cast<CpuStream*>(&s);
    DLNB_REQUIRE(cs, "the CPU shm backend needs CPU streams (use --backend rccl on a GPU)");
    cs->enqueue(std::move(fn));
  }

  void barrier() {
    SegHeader* h = hdr();
    uint32_t g = h->gen.load(std::memory_order_acquire);
    if (h->count.fetch_add(1, std::memory_order_acq_rel) + 1 == static_cast<uint32_t>(size_)) {
      h->count.store(0, std::memory_order_relaxed);
      h->gen.fetch_add(1, std::memory_order_acq_rel);
      wake(&h->gen);
    } else {
      wait_on(&h->gen, [&] { return h->gen.load(std::memory_order_acquire) != g; }, timeout_, "barrier");
    }
  }

  void do_send(const void* buf, size_t bytes, int peer) {
    DLNB_REQUIRE(p2p_, "group " << name_ << " was created without point-to-point support");
    check(bytes);
    Mailbox* m = mbox(rank_, peer);
    // Wait until the previous message was taken.
    wait_on(&m->taken, [&] { return m->taken.load(std::memory_order_acquire) == m->sent.load(std::memory_order_acquire); },
            timeout_, "send");
    std::memcpy(reinterpret_cast<char*>(m) + 64, buf, bytes);
    m->bytes = bytes;
    m->sent.fetch_add(1, std::memory_order_release);
    wake(&m->sent);
  }

  void do_recv(void* buf, size_t bytes, int peer) {
    DLNB_REQUIRE(p2p_, "group " << name_ << " was created without point-to-point support");
    Mailbox* m = mbox(peer, rank_);
    wait_on(&m->sent, [&] { return m->sent.load(std::memory_order_acquire) != m->taken.load(std::memory_order_acquire); },
            timeout_, "recv");
    DLNB_REQUIRE(m->bytes == bytes, "shm recv size mismatch: expected " << bytes << " got " << m->bytes);
    std::memcpy(buf, reinterpret_cast<char*>(m) + 64, bytes);
    m->taken.fetch_add(1, std::memory_order_release);
    wake(&m->taken);
  }

  struct Reg {
    char* local = nullptr;
    size_t bytes = 0;
    std::vector<char*> peer;  // by group rank (own entry = local)
    bool usable = true;       // every member mapped every peer's buffer
  };
  bool warned_ = false;
  int my_world_rank_ = 0;
  // The registration holding [p, p + bytes) on this rank, with p's offset.
  const Reg* find(const void* p, size_t bytes, size_t& off) const {
    const char* c = static_cast<const char*>(p);
    for (const auto& r : regs_)
      if (r.usable && c >= r.local && c + bytes <= r.local + r.bytes) {
        off = static_cast<size_t>(c - r.local);
        return &r;
      }
    return nullptr;
  }

  HostGroup* world_ = nullptr;
  std::string job_;
  std::deque<Reg> regs_;  // stable addresses: queued tasks hold Reg pointers
  std::vector<std::pair<void*, size_t>> mapped_;
  size_t cap_;
  bool p2p_;
  char* base_ = nullptr;
  size_t total_ = 0, slots_off_ = 0, result_off_ = 0, mbox_off_ = 0;
  double timeout_ = 900;
  bool in_group_ = false;
  std::vector<std::function<void()>> group_sends_, group_recvs_;
  Stream* group_stream_ = nullptr;
};

class ShmFactory : public CommFactory {
 public:
  ShmFactory(HostGroup& world, Device& dev) : world_(world) {
    DLNB_REQUIRE(dev.kind() == DeviceKind::CPU, "the cpu backend needs the CPU device (buffers in host memory)");
    // Job id shared by all ranks so segment names never collide across jobs.
    char buf[32];
    std::snprintf(buf, sizeof(buf), "%d_%lx", static_cast<int>(getpid()), static_cast<unsigned long>(now_s() * 1e6));
    job_ = world.broadcast(buf, 0);
  }
  std::string backend_name() const override { return "CPU-SHM"; }
  std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members, size_t cap,
                                       bool p2p, int) override {
    return std::unique_ptr<Communicator>(new ShmComm(name, members, world_.rank(), world_, job_, cap, p2p));
  }

 private:
  HostGroup& world_;
  std::string job_;
};

}  // namespace

std::unique_ptr<CommFactory> make_shm_factory(HostGroup& world, Device& dev) {
  return std::unique_ptr<CommFactory>(new ShmFactory(world, dev));
}

void host_reduce_sum(DType t, void* dst, const std::vector<const char*>& srcs, size_t count) {
  par_reduce_sum(t, dst, srcs, 0, count);
}

void host_copy(void* dst, const void* src, size_t bytes) { par_copy(dst, src, bytes); }

}  // namespace dlnb
