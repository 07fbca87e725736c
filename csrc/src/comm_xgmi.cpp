// "xgmi" backend: our own collective / P2P kernels over IPC-mapped peer
// windows (protocol and kernels: dlnb/xgmi.hpp, csrc/kernels/xgmi.hip).
//
// Setup per communicator: each member allocates its window + flag array in
// uncached device memory, publishes hipIpcMemHandles through the job's TCP
// store and opens every peer's handles; the members must share one node
// (xGMI). Each operation is cut into pieces that fit one parity region of
// the windows and each piece is one kernel on the caller's stream. The
// kernel takes its epoch from a per-communicator counter in device memory
// (identical on all members because every member issues the same sequence
// of operations on a communicator - the same rule RCCL has), so the ops
// capture into HIP graphs and replay with fresh epochs. Ops on one
// communicator must be stream-ordered.
//
// Selection: --backend xgmi (GPU only). Several ranks may share one GPU
// (-d 0,0): IPC works within a device, which is how the kernels are tested
// on a 1-GPU machine; RCCL refuses that configuration.
//
// Tunables (env): DLNB_XGMI_REGION_MB (per-parity collective region, default
// 256), DLNB_XGMI_P2P_MB (per-source, per-parity P2P slot, default 128),
// DLNB_XGMI_BLOCKS (max blocks per kernel, default 256),
// DLNB_XGMI_ONESHOT_KB (all-reduce one-shot threshold, default 256),
// DLNB_XGMI_TIMEOUT_S (device-side wait timeout, default 600).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <sstream>

#include "dlnb/comm.hpp"
#include "dlnb/xgmi.hpp"

#define DLNB_HIP_CHECK(expr)                                                       \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) DLNB_THROW(#expr << " failed: " << hipGetErrorString(e_)); \
  } while (0)

namespace dlnb {

namespace {

using xgmi::CollPiece;
using xgmi::Op;

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

std::string hex(const void* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) {
    s += d[b[i] >> 4];
    s += d[b[i] & 15];
  }
  return s;
}

void unhex(const std::string& s, void* p, size_t n) {
  DLNB_REQUIRE(s.size() == 2 * n, "xgmi: bad handle encoding");
  auto v = [](char c) { return c <= '9' ? c - '0' : c - 'a' + 10; };
  unsigned char* b = static_cast<unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) b[i] = static_cast<unsigned char>(v(s[2 * i]) << 4 | v(s[2 * i + 1]));
}

hipStream_t hs(Stream& s) { return static_cast<hipStream_t>(s.native()); }

// PCI bus id of a device ("0000:a4:00.0"): how a peer names its GPU in the
// store record, independent of each process's device ordinals.
std::string pci_id(int dev) {
  char buf[64] = {0};
  if (hipDeviceGetPCIBusId(buf, sizeof(buf), dev) != hipSuccess) return "?";
  return buf;
}

class XgmiComm : public Communicator {
 public:
  XgmiComm(const std::string& name, const std::vector<int>& members, int my_world_rank, HostGroup& world,
           size_t capacity, bool p2p, int max_ctas) {
    name_ = name;
    members_ = members;
    world_ = &world;
    size_ = static_cast<int>(members.size());
    rank_ = -1;
    for (int i = 0; i < size_; ++i)
      if (members[i] == my_world_rank) rank_ = i;
    DLNB_REQUIRE(rank_ >= 0, "rank " << my_world_rank << " is not a member of group " << name);
    DLNB_REQUIRE(size_ <= xgmi::kMaxRanks, "xgmi backend: group " << name << " has " << size_ << " ranks (max "
                                                                 << xgmi::kMaxRanks << ", one node)");
    max_blocks_ = static_cast<int>(std::max<long long>(1, std::min<long long>(xgmi::kMaxBlocks, env_int("DLNB_XGMI_BLOCKS", 256))));
    // CU budget of this comm lane (runner.cpp): blocks_per_cu of these
    // blocks fit a CU beside nothing else (the measured occupancy of the
    // least-occupant kernel; every kernel is register-capped for 4), so the
    // lane's kernels never need more CUs than the budget even when several
    // lanes' kernels are live at once.
    if (max_ctas > 0) max_blocks_ = std::min(max_blocks_, xgmi::min_blocks_per_cu() * max_ctas);
    oneshot_ = static_cast<size_t>(env_int("DLNB_XGMI_ONESHOT_KB", 256)) << 10;
    const size_t cap = std::max<size_t>(capacity, 4096);
    // Collective region per parity: AG/RS/A2A need W slots of a piece, the
    // two-shot all-reduce 2W slots of a chunk (~2 x piece).
    region_ = p2p ? (size_t(1) << 20)
                  : std::min(round_up(2 * cap + 2 * size_ * 256, 1 << 20),
                             static_cast<size_t>(env_int("DLNB_XGMI_REGION_MB", 256)) << 20);
    p2p_slot_ = p2p ? std::min(round_up(cap, 256), static_cast<size_t>(env_int("DLNB_XGMI_P2P_MB", 128)) << 20) : 0;
    p2p_off_ = 2 * region_;
    win_bytes_ = p2p_off_ + static_cast<size_t>(size_) * 2 * p2p_slot_;

    DLNB_HIP_CHECK(hipGetDevice(&dev_));
    // Uncached by default (peers' xGMI stores are never shadowed by a stale
    // L2 line); DLNB_XGMI_MEM=fine|coarse for experiments.
    const std::string mem = env_or("DLNB_XGMI_MEM", "uncached");
    const unsigned flags = mem == "coarse" ? hipDeviceMallocDefault
                           : mem == "fine" ? hipDeviceMallocFinegrained
                                           : hipDeviceMallocUncached;
    DLNB_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&win_), win_bytes_, flags));
    DLNB_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), xgmi::kFlagBytes, flags));
    DLNB_HIP_CHECK(hipMemset(flags_, 0, xgmi::kFlagBytes));
    DLNB_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_words_), 64, hipHostMallocMapped));
    std::memset(host_words_, 0, 64);
    uint32_t* dev_words = nullptr;
    DLNB_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_words), host_words_, 0));
    DLNB_HIP_CHECK(hipDeviceSynchronize());

    // Exchange IPC handles (and host names: the group must share a node).
    hipIpcMemHandle_t hw, hf;
    DLNB_HIP_CHECK(hipIpcGetMemHandle(&hw, win_));
    DLNB_HIP_CHECK(hipIpcGetMemHandle(&hf, flags_));
    std::ostringstream key;
    key << "xgmi/" << name << "/";
    for (int m : members) key << m << ",";
    const std::string me = get_hostname() + " " + hex(&hw, sizeof(hw)) + " " + hex(&hf, sizeof(hf)) + " " + pci_id(dev_);
    world.store().set(key.str() + std::to_string(rank_), me);
    std::memset(&peers_, 0, sizeof(peers_));
    for (int r = 0; r < size_; ++r) {
      if (r == rank_) {
        peers_.win[r] = win_;
        peers_.flags[r] = flags_;
        continue;
      }
      std::istringstream in(world.store().get(key.str() + std::to_string(r)));
      std::string host, sw, sf, pci;
      in >> host >> sw >> sf >> pci;
      DLNB_REQUIRE(host == get_hostname(), "xgmi backend: group " << name << " spans hosts (" << host << " and "
                                                                  << get_hostname() << "); use --backend rccl");
      require_peer_access(name, r, pci);
      hipIpcMemHandle_t pw, pf;
      unhex(sw, &pw, sizeof(pw));
      unhex(sf, &pf, sizeof(pf));
      void* a = nullptr;
      void* b = nullptr;
      DLNB_HIP_CHECK(hipIpcOpenMemHandle(&a, pw, hipIpcMemLazyEnablePeerAccess));
      DLNB_HIP_CHECK(hipIpcOpenMemHandle(&b, pf, hipIpcMemLazyEnablePeerAccess));
      peers_.win[r] = static_cast<char*>(a);
      peers_.flags[r] = static_cast<uint32_t*>(b);
      opened_.push_back(a);
      opened_.push_back(b);
    }
    peers_.abort_word = dev_words;
    peers_.error_word = dev_words + 16;
    peers_.timeout_ticks = static_cast<uint64_t>(env_int("DLNB_XGMI_TIMEOUT_S", 600)) * 100000000ull;
    peers_.rank = rank_;
    peers_.nranks = size_;
    peers_.uncached = mem != "coarse" && mem != "fine";
    const std::string rel = env_or("DLNB_XGMI_RELEASE", "vmcnt");
    DLNB_REQUIRE(rel == "vmcnt" || rel == "system", "DLNB_XGMI_RELEASE must be vmcnt or system (got " << rel << ")");
    peers_.release_system = rel == "system";
    // Nobody may free its window before every member has mapped it.
    const std::string done = key.str() + "opened";
    if (world.store().add(done, 1) == size_) world.store().set(done + "/go", "1");
    world.store().get(done + "/go");
  }

  ~XgmiComm() override {
    (void)hipDeviceSynchronize();
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    if (win_) (void)hipFree(win_);
    if (flags_) (void)hipFree(flags_);
    if (host_words_) (void)hipHostFree(host_words_);
  }

  std::string backend_name() const override { return "XGMI"; }

  bool wants_peer_buffers() const override { return size_ > 1; }

  // Collective: every member maps every other member's buffer of this
  // registration (the k-th registration of each member pairs with the k-th of
  // the others). The buffer must be an allocation of its own (Device::alloc_peer).
  void register_buffer(void* p, size_t bytes) override {
    Reg r;
    std::memset(&r, 0, sizeof(r));
    r.local = static_cast<char*>(p);
    r.bytes = bytes;
    r.peer[rank_] = r.local;
    if (size_ > 1) {
      hipIpcMemHandle_t h;
      DLNB_HIP_CHECK(hipIpcGetMemHandle(&h, p));
      std::ostringstream key;
      key << "xgmi/" << name_ << "/";
      for (int m : members_) key << m << ",";
      key << "reg" << regs_.size() << "/";
      world_->store().set(key.str() + std::to_string(rank_), hex(&h, sizeof(h)) + " " + std::to_string(bytes));
      for (int q = 0; q < size_; ++q) {
        if (q == rank_) continue;
        std::istringstream in(world_->store().get(key.str() + std::to_string(q)));
        std::string sh;
        size_t qb = 0;
        in >> sh >> qb;
        DLNB_REQUIRE(qb == bytes, "xgmi: registration " << regs_.size() << " of " << name_ << ": rank " << q
                                                         << " registered " << qb << " B, this rank " << bytes);
        hipIpcMemHandle_t ph;
        unhex(sh, &ph, sizeof(ph));
        void* a = nullptr;
        DLNB_HIP_CHECK(hipIpcOpenMemHandle(&a, ph, hipIpcMemLazyEnablePeerAccess));
        r.peer[q] = static_cast<char*>(a);
        opened_.push_back(a);
      }
      // nobody may free the buffer before every member mapped it (freeing is
      // stream-ordered after the last use anyway; this orders the setup)
      const std::string done = key.str() + "opened";
      if (world_->store().add(done, 1) == size_) world_->store().set(done + "/go", "1");
      world_->store().get(done + "/go");
    }
    regs_.push_back(r);
  }

  void all_gather(const void* send, void* recv, size_t send_count, DType t, Stream& s) override {
    const size_t es = dtype_size(t), bytes = send_count * es;
    size_t off = 0;
    if (const Reg* r = size_ > 1 && bytes > 0 ? find(recv, bytes * size_, off) : nullptr) {
      xgmi::DirectPiece c = direct(t, bytes);
      c.src[rank_] = static_cast<const char*>(send);
      for (int q = 0; q < size_; ++q) c.dst[q] = r->peer[q] + off + static_cast<size_t>(rank_) * bytes;
      launch_direct(xgmi::DirectOp::AllGather, c, bytes, s);
      return;
    }
    const size_t piece = piece_bytes(region_ / size_, es);
    for (size_t off = 0; off < bytes; off += piece) {
      CollPiece c = base(t);
      c.bytes = std::min(piece, bytes - off);
      c.send = static_cast<const char*>(send) + off;
      c.recv = static_cast<char*>(recv) + off;
      c.recv_stride = bytes;
      c.slot = round_up(c.bytes, 256);
      launch(Op::AllGather, c, s);
    }
  }

  void reduce_scatter(const void* send, void* recv, size_t recv_count, DType t, Stream& s) override {
    const size_t es = dtype_size(t), bytes = recv_count * es;
    size_t off = 0;
    if (const Reg* r = size_ > 1 && bytes > 0 ? find(send, bytes * size_, off) : nullptr) {
      xgmi::DirectPiece c = direct(t, bytes);
      for (int q = 0; q < size_; ++q) c.src[q] = r->peer[q] + off + static_cast<size_t>(rank_) * bytes;
      c.out = static_cast<char*>(recv);
      launch_direct(xgmi::DirectOp::ReduceScatter, c, bytes, s);
      return;
    }
    const size_t piece = piece_bytes(region_ / size_, es);
    for (size_t off = 0; off < bytes; off += piece) {
      CollPiece c = base(t);
      c.bytes = std::min(piece, bytes - off);
      c.send = static_cast<const char*>(send) + off;
      c.recv = static_cast<char*>(recv) + off;
      c.send_stride = bytes;
      c.slot = round_up(c.bytes, 256);
      launch(Op::ReduceScatter, c, s);
    }
  }

  void all_to_all(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    const size_t es = dtype_size(t), bytes = count * es;
    size_t off = 0;
    // In place goes through the windows: each block reads its slice of every
    // send block before the exchange and writes the same slice of the receive
    // blocks after it, while the zero-copy path writes peers' receive buffers
    // that may still be their unread send buffers.
    if (const Reg* r = size_ > 1 && bytes > 0 && send != recv ? find(recv, bytes * size_, off) : nullptr) {
      xgmi::DirectPiece c = direct(t, bytes);
      c.src[rank_] = static_cast<const char*>(send);
      for (int q = 0; q < size_; ++q) c.dst[q] = r->peer[q] + off + static_cast<size_t>(rank_) * bytes;
      launch_direct(xgmi::DirectOp::AllToAll, c, bytes, s);
      return;
    }
    const size_t piece = piece_bytes(region_ / size_, es);
    for (size_t off = 0; off < bytes; off += piece) {
      CollPiece c = base(t);
      c.bytes = std::min(piece, bytes - off);
      c.send = static_cast<const char*>(send) + off;
      c.recv = static_cast<char*>(recv) + off;
      c.send_stride = c.recv_stride = bytes;
      c.slot = round_up(c.bytes, 256);
      launch(Op::AllToAll, c, s);
    }
  }

  void all_reduce(const void* send, void* recv, size_t count, DType t, Stream& s) override {
    const size_t es = dtype_size(t), bytes = count * es;
    const char* sp = static_cast<const char*>(send);
    char* rp = static_cast<char*>(recv);
    if (size_ == 1) {
      if (send != recv) DLNB_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, hs(s)));
      return;
    }
    // One-shot for latency-bound sizes: every rank pushes the whole buffer.
    const size_t one_max = std::min(oneshot_, piece_bytes(region_ / size_, es));
    // Registered send and receive buffers, above the one-shot range: rank r
    // sums chunk r straight out of every peer's send buffer and writes it
    // into every peer's receive buffer (no window staging).
    size_t offs = 0, offr = 0;
    const Reg* rs = bytes > one_max && bytes % 16 == 0 ? find(send, bytes, offs) : nullptr;
    const Reg* rr = rs ? find(recv, bytes, offr) : nullptr;
    if (rs && rr) {
      xgmi::DirectPiece c = direct(t, bytes);
      for (int q = 0; q < size_; ++q) {
        c.src[q] = rs->peer[q] + offs;
        c.dst[q] = rr->peer[q] + offr;
      }
      launch_direct(xgmi::DirectOp::AllReduce, c, bytes / size_, s);
      return;
    }
    if (bytes <= one_max) {
      CollPiece c = base(t);
      c.bytes = bytes;
      c.send = sp;
      c.recv = rp;
      c.slot = round_up(bytes, 256);
      launch(Op::AllReduceOneShot, c, s);
      return;
    }
    // Two-shot on 16-B multiples; a ragged tail (< 16 B) goes one-shot.
    const size_t body = bytes / 16 * 16;
    // chunk = ceil(piece / W) rounded to 256 B per slot: 2 W slots < region
    const size_t piece = std::max<size_t>(16 * size_, (region_ / 2 - size_ * 512) / 16 * 16);
    for (size_t off = 0; off < body; off += piece) {
      CollPiece c = base(t);
      c.bytes = std::min(piece, body - off);
      c.send = sp + off;
      c.recv = rp + off;
      const size_t chunk = (c.bytes / 16 + size_ - 1) / size_ * 16;
      c.slot = round_up(chunk, 256);
      c.ag_off = c.slot * size_;
      launch(Op::AllReduceTwoShot, c, s);
    }
    if (body < bytes) {
      CollPiece c = base(t);
      c.bytes = bytes - body;
      c.send = sp + body;
      c.recv = rp + body;
      c.slot = 256;
      launch(Op::AllReduceOneShot, c, s);
    }
  }

  // Messages larger than a P2P slot travel as several chunks. Inside a group
  // the chunks of all operations are issued round-robin (send chunk r, recv
  // chunk r, ...): a send's chunk r waits for the peer to drain chunk r-2,
  // so two ranks exchanging large messages must interleave their receives
  // with their sends or both would stall behind their own sends.
  void send(const void* buf, size_t count, DType t, int peer, Stream& s) override {
    p2p_op(true, const_cast<void*>(buf), count * dtype_size(t), peer, s);
  }
  void recv(void* buf, size_t count, DType t, int peer, Stream& s) override {
    p2p_op(false, buf, count * dtype_size(t), peer, s);
  }
  void group_start() override { in_group_ = true; }
  void group_end() override {
    in_group_ = false;
    std::vector<P2POp> ops;
    ops.swap(pending_);
    size_t rounds = 0;
    for (auto& o : ops) rounds = std::max(rounds, chunks(o.bytes));
    for (size_t r = 0; r < rounds; ++r)
      for (auto& o : ops)
        if (r < chunks(o.bytes)) p2p_chunk(o, r);
  }

  std::string async_error() override {
    if (__atomic_load_n(host_words_ + 16, __ATOMIC_ACQUIRE))
      return "xgmi: a device-side wait timed out in " + name_ + " (a peer died or hangs)";
    return "";
  }
  void abort() override { __atomic_store_n(host_words_, 1u, __ATOMIC_RELEASE); }

 private:
  // Before any kernel touches a peer window: a member on another GPU must be
  // reachable by peer access (xGMI), or the first load from its window faults
  // the device instead of failing this setup. Ranks sharing one GPU (the
  // 1-GPU test setup) need nothing; a peer GPU outside this process's visible
  // set cannot be checked here and is left to the IPC mapping.
  void require_peer_access(const std::string& name, int r, const std::string& pci) {
    int peer_dev = -1;
    if (pci == "?" || hipDeviceGetByPCIBusId(&peer_dev, pci.c_str()) != hipSuccess || peer_dev == dev_) {
      (void)hipGetLastError();
      return;
    }
    int ok = 0;
    DLNB_HIP_CHECK(hipDeviceCanAccessPeer(&ok, dev_, peer_dev));
    DLNB_REQUIRE(ok, "xgmi backend: group " << name << ": GPU " << dev_ << " cannot access the GPU of member " << r
                                            << " (" << pci << ", device " << peer_dev
                                            << ") by peer access; use --backend rccl");
    hipError_t e = hipDeviceEnablePeerAccess(peer_dev, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
      DLNB_THROW("xgmi backend: hipDeviceEnablePeerAccess(" << peer_dev << ") failed: " << hipGetErrorString(e));
    (void)hipGetLastError();
  }

  struct P2POp {
    bool is_send;
    char* buf;
    size_t bytes;
    int peer;
    Stream* s;
  };
  size_t chunks(size_t bytes) const { return bytes == 0 ? 1 : (bytes + p2p_slot_ - 1) / p2p_slot_; }
  void p2p_op(bool is_send, void* buf, size_t bytes, int peer, Stream& s) {
    DLNB_REQUIRE(p2p_slot_ > 0, "xgmi: communicator " << name_ << " was created without point-to-point support");
    DLNB_REQUIRE(peer >= 0 && peer < size_ && peer != rank_, "xgmi: bad peer " << peer);
    P2POp o{is_send, static_cast<char*>(buf), bytes, peer, &s};
    if (in_group_) {
      pending_.push_back(o);
      return;
    }
    for (size_t r = 0; r < chunks(bytes); ++r) p2p_chunk(o, r);
  }
  void p2p_chunk(const P2POp& o, size_t r) {
    const size_t off = r * p2p_slot_;
    const size_t n = o.bytes == 0 ? 0 : std::min(p2p_slot_, o.bytes - off);
    const size_t p = static_cast<size_t>(o.peer);
    const int nb = xgmi::blocks_for(n, max_blocks_);
    // source s's two slots (message parity) in the receiver's window
    if (o.is_send) {
      const size_t woff = p2p_off_ + static_cast<size_t>(rank_) * 2 * p2p_slot_;
      xgmi::launch_send(peers_, o.buf + off, n, o.peer, woff, p2p_slot_, nb, hs(*o.s));
      debug("send", n, *o.s);
    } else {
      const size_t woff = p2p_off_ + p * 2 * p2p_slot_;
      xgmi::launch_recv(peers_, o.buf + off, n, o.peer, woff, p2p_slot_, nb, hs(*o.s));
      debug("recv", n, *o.s);
    }
  }

  struct Reg {
    char* local;
    size_t bytes;
    char* peer[xgmi::kMaxRanks];  // each member's buffer of this registration, mapped here
  };
  // The registration holding [p, p + n) on this rank (offset returned).
  const Reg* find(const void* p, size_t n, size_t& off) const {
    const char* c = static_cast<const char*>(p);
    for (const Reg& r : regs_)
      if (c >= r.local && c + n <= r.local + r.bytes) {
        off = static_cast<size_t>(c - r.local);
        return &r;
      }
    return nullptr;
  }
  xgmi::DirectPiece direct(DType t, size_t bytes) const {
    xgmi::DirectPiece c;
    std::memset(&c, 0, sizeof(c));
    c.dtype = t;
    c.bytes = bytes;
    return c;
  }
  // `work` = bytes each rank moves per block slice group (blocks_for's unit)
  void launch_direct(xgmi::DirectOp op, const xgmi::DirectPiece& c, size_t work, Stream& s) {
    xgmi::launch_direct(op, peers_, c, xgmi::blocks_for(work, max_blocks_), hs(s));
    ++direct_ops_;
    debug("direct", c.bytes, s);
  }

  // Largest piece (bytes per rank block) fitting `slot_cap`, element aligned.
  static size_t piece_bytes(size_t slot_cap, size_t es) {
    size_t p = (slot_cap / 256) * 256;
    p = p / es * es;
    return std::max(p, es);
  }
  CollPiece base(DType t) {
    CollPiece c;
    std::memset(&c, 0, sizeof(c));
    c.dtype = t;
    c.region = region_;
    return c;
  }
  void launch(Op op, const CollPiece& c, Stream& s) {
    xgmi::launch_coll(op, peers_, c, xgmi::blocks_for(c.bytes, max_blocks_), hs(s));
    debug("coll", c.bytes, s);
  }
  // DLNB_XGMI_DEBUG=1: synchronise after every kernel and dump the flags.
  void debug(const char* what, size_t bytes, Stream& s) {
    static const bool on = env_int("DLNB_XGMI_DEBUG", 0) != 0;
    if (!on) return;
    DLNB_HIP_CHECK(hipStreamSynchronize(hs(s)));
    std::vector<uint32_t> f(xgmi::kFlagWords);
    DLNB_HIP_CHECK(hipMemcpy(f.data(), flags_, f.size() * 4, hipMemcpyDeviceToHost));
    std::fprintf(stderr, "[xgmi-debug] %s r%d %s epoch=%u bytes=%zu err=%u coll0=[", name_.c_str(), rank_, what,
                 f[xgmi::kCtlCollEpoch], bytes, host_words_[16]);
    for (int r = 0; r < size_; ++r) std::fprintf(stderr, "%u ", f[xgmi::kFlagColl + r * xgmi::kMaxBlocks]);
    std::fprintf(stderr, "] seq0=[");
    for (int r = 0; r < size_; ++r) std::fprintf(stderr, "%u ", f[xgmi::kFlagP2PSeq + r * xgmi::kMaxBlocks]);
    std::fprintf(stderr, "] consumed=[");
    for (int r = 0; r < size_; ++r) std::fprintf(stderr, "%u ", f[xgmi::kFlagP2PConsumed + r]);
    std::fprintf(stderr, "] sent=[");
    for (int r = 0; r < size_; ++r) std::fprintf(stderr, "%u ", f[xgmi::kCtlSendSeq + r]);
    std::fprintf(stderr, "] received=[");
    for (int r = 0; r < size_; ++r) std::fprintf(stderr, "%u ", f[xgmi::kCtlRecvSeq + r]);
    std::fprintf(stderr, "]\n");
  }

  int dev_ = 0;
  int max_blocks_ = 64;
  size_t oneshot_ = 0, region_ = 0, p2p_slot_ = 0, p2p_off_ = 0, win_bytes_ = 0;
  char* win_ = nullptr;
  uint32_t* flags_ = nullptr;
  uint32_t* host_words_ = nullptr;  // [0] abort, [16] error
  std::vector<void*> opened_;
  xgmi::Peers peers_;
  HostGroup* world_ = nullptr;
  std::vector<Reg> regs_;
  size_t direct_ops_ = 0;
  bool in_group_ = false;
  std::vector<P2POp> pending_;
};

class XgmiFactory : public CommFactory {
 public:
  XgmiFactory(HostGroup& world, Device& dev) : world_(world) {
    DLNB_REQUIRE(dev.kind() == DeviceKind::GPU, "the xgmi backend needs a GPU device");
  }
  std::string backend_name() const override { return "XGMI"; }
  std::unique_ptr<Communicator> create(const std::string& name, const std::vector<int>& members,
                                       size_t capacity_bytes, bool need_p2p, int max_ctas) override {
    return std::unique_ptr<Communicator>(
        new XgmiComm(name, members, world_.rank(), world_, capacity_bytes, need_p2p, max_ctas));
  }

 private:
  HostGroup& world_;
};

}  // namespace

std::unique_ptr<CommFactory> make_xgmi_factory(HostGroup& world, Device& dev) {
  return std::unique_ptr<CommFactory>(new XgmiFactory(world, dev));
}

}  // namespace dlnb
