// Device side of the "xgmi" backend: collectives and point-to-point copies
// done by our own kernels through IPC-mapped peer windows (SURVEY.md §7.2
// step 7). Every rank owns one window (uncached device memory, so stores
// that peers make over xGMI are never shadowed by a stale L2 line) plus a
// small flag array; each rank maps all peers' windows with
// hipIpcOpenMemHandle. A collective is one kernel per piece: every block
// owns the same slice of the message on every rank, pushes its slice to all
// peers with 16-B stores (the 7 xGMI links run concurrently, staggered by
// rank so no link is hot-spotted), fences at system scope, raises one flag
// per peer and waits for the peers' flags for the same block, then finishes
// locally (copy-out or fp32-accumulated reduction). No grid-wide barrier,
// no host involvement; windows alternate between two parity regions, so a
// piece never waits for a peer to finish reading the previous one (stream
// order on the peer guarantees piece k-2 is fully consumed when any of its
// blocks reached piece k-1's flags).
//
// Sequence numbers live on the device: a collective's epoch (and with it the
// parity region) and a point-to-point message's number are read from
// per-communicator counters in the rank's own flag page when the kernel
// starts, and the last block of the kernel to finish advances them. Kernel
// arguments therefore carry no sequence state, so a captured HIP graph that
// is replayed issues fresh epochs on every replay exactly like eager launches
// (every member still issues the same sequence of kernels per communicator).
//
// Reference equivalent: none (the reference only calls NCCL/RCCL/MPI,
// cpp/proxy_classes.hpp:135-253); this is new MI355X-native capability.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "dlnb/common.hpp"

namespace dlnb {
namespace xgmi {

constexpr int kMaxRanks = 8;     // one node: 8 MI355X, fully connected by xGMI
constexpr int kMaxBlocks = 1024;  // per-block flags
constexpr int kThreads = 512;

// Flag words (uint32) in each rank's flag array.
constexpr size_t kFlagColl = 0;                                    // [phase 2][src 8][block]
constexpr size_t kFlagP2PSeq = 2 * kMaxRanks * kMaxBlocks;         // [src 8][block]
constexpr size_t kFlagP2PConsumed = kFlagP2PSeq + kMaxRanks * kMaxBlocks;  // [dst 8]
// Local-only control words (never touched by peers):
constexpr size_t kCtl = kFlagP2PConsumed + 64;
constexpr size_t kCtlCollEpoch = kCtl;           // last finished collective epoch
constexpr size_t kCtlCollDone = kCtl + 1;        // blocks of the running collective that finished
constexpr size_t kCtlSendSeq = kCtl + 16;        // [dst 8] last message number sent to dst
constexpr size_t kCtlSendDone = kCtl + 32;       // [dst 8] finished blocks of the running send
constexpr size_t kCtlRecvSeq = kCtl + 48;        // [src 8] last message number received from src
constexpr size_t kCtlRecvDone = kCtl + 64;       // [src 8] finished blocks of the running receive
constexpr size_t kFlagWords = kCtl + 80;
constexpr size_t kFlagBytes = 128 * 1024;
static_assert(kFlagWords * 4 <= kFlagBytes, "flag page too small");

struct Peers {
  char* win[kMaxRanks];        // each rank's window, mapped in this process
  uint32_t* flags[kMaxRanks];  // each rank's flag array, mapped in this process
  uint32_t* abort_word;        // host-mapped: non-zero = give up waiting
  uint32_t* error_word;        // host-mapped: set by a kernel that timed out
  uint64_t timeout_ticks;      // s_memrealtime ticks (100 MHz) before a wait gives up
  int rank;
  int nranks;
  int uncached;                // windows + flags in uncached memory (the default; see release_window)
  int release_system;          // DLNB_XGMI_RELEASE=system: system-scope release/acquire even when uncached
};

// Blocks of a peer-waiting kernel that fit one CU (every such kernel is
// register-capped for this; see DLNB_XGMI_KERNEL in xgmi.hip).
constexpr int kBlocksPerCU = 4;

// Occupancy (blocks per CU, hipOccupancyMaxActiveBlocksPerMultiprocessor)
// of every peer-waiting kernel and dtype on the current device, as
// {"rs_kernel<fp8_e4m3>", n} pairs; min_blocks_per_cu() is the smallest.
struct KernelOccupancy {
  const char* name;
  int blocks_per_cu;
};
std::vector<KernelOccupancy> occupancy();
int min_blocks_per_cu();

enum class Op : int { AllGather, ReduceScatter, AllReduceOneShot, AllReduceTwoShot, AllToAll };

struct CollPiece {
  const char* send;
  char* recv;
  size_t bytes;        // bytes per rank block of this piece
  size_t send_stride;  // bytes between rank blocks in send (RS, A2A)
  size_t recv_stride;  // bytes between rank blocks in recv (AG, A2A)
  size_t region;       // bytes per parity region (epoch e uses region (e & 1))
  size_t slot;         // bytes between source slots inside the region
  size_t ag_off;       // two-shot: offset of the all-gather slots inside the region
  DType dtype;
};

// Zero-copy collectives on registered buffers (Communicator::register_buffer):
// one kernel per operation, no window staging. Every block owns the same
// slice on all ranks; its phase-0 flags say "ready" (this rank's kernel has
// started, so everything its stream did to its buffers before is complete)
// and its phase-1 flags "done with your buffers" (the kernel - and with it
// the next use of the buffers on that rank - cannot finish before every peer
// is done reading / writing them).
//   AllGather:     dst[r] = rank r's receive buffer at this rank's block; src[me] = send
//   ReduceScatter: src[r] = rank r's send buffer at this rank's block; out = receive buffer
//   AllReduce:     src[r] = rank r's send buffer, dst[r] = rank r's receive buffer (may alias);
//                  rank me sums chunk me of every src and writes it into every dst
//   AllToAll:      src[me] = send (W blocks); dst[r] = rank r's receive buffer at this rank's block
enum class DirectOp : int { AllGather, ReduceScatter, AllReduce, AllToAll };
struct DirectPiece {
  const char* src[kMaxRanks];
  char* dst[kMaxRanks];
  char* out;
  size_t bytes;  // AG / RS: bytes per rank block; AR: the whole message (multiple of 16)
  DType dtype;
};
void launch_direct(DirectOp op, const Peers& p, const DirectPiece& c, int blocks, void* stream);

// Number of blocks a piece of `bytes` per rank uses (identical on all ranks).
int blocks_for(size_t bytes, int max_blocks);

void launch_coll(Op op, const Peers& p, const CollPiece& c, int blocks, void* stream);

// Point-to-point: message n (1-based, counted on the device) of the
// (me -> dst) channel goes to dst's window at `off + (n & 1) * slot`; the
// sender waits until dst consumed message n-2. The receiver's last block to
// finish signals "consumed n" back to the sender.
void launch_send(const Peers& p, const char* buf, size_t bytes, int dst, size_t off, size_t slot, int blocks,
                 void* stream);
void launch_recv(const Peers& p, char* buf, size_t bytes, int src, size_t off, size_t slot, int blocks,
                 void* stream);

// Loopback backend (all ranks in one process on one device): for i < count,
// dsts[d][i] = sum over s of srcs[s][i] (fp32 accumulation, one rounding;
// ns == 1 is a bit-exact copy to nd destinations). In place safe: every
// element is read from all sources before any destination is written.
constexpr int kMaxLocal = 16;
void launch_local_reduce(char* const* dsts, int nd, const char* const* srcs, int ns, size_t count, DType t,
                         void* stream);

// One launch for a whole loopback collective of W ranks (send[r] / recv[r]
// per rank, blk elements per rank block):
//   AllGather:     recv[j][i*blk + e] = send[i][e]
//   ReduceScatter: recv[j][e]         = sum_i send[i][j*blk + e]  (fp32 accumulation)
//   AllToAll:      recv[j][i*blk + e] = send[i][j*blk + e]        (out of place)
enum class LocalColl : int { AllGather, ReduceScatter, AllToAll };
void launch_local_coll(LocalColl op, char* const* recv, const char* const* send, int W, size_t blk, DType t,
                       void* stream);

}  // namespace xgmi
}  // namespace dlnb
