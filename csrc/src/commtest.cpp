// dlnb commtest: correctness and bandwidth of every collective of a backend.
//
//   dlnb commtest [--backend auto|rccl|xgmi|cpu] [-d 0,1,..] [--dtype bf16]
//                 [--sizes 1,7,4096,...] [--bench] [--iters N] [--warmup N] [--graph]
//
// Check mode (default): every rank fills its buffers with exact small
// integers v(rank, i), runs all-reduce (out-of-place and in-place),
// all-gather, reduce-scatter, all-to-all and a ring send/recv for each size,
// copies the results back and compares with the closed-form expectation
// (exact in every wire dtype at <= 8 ranks). Bench mode prints algbw/busbw
// per collective and size (nccl-tests conventions, SURVEY.md §5 "Metrics"),
// so RCCL and the xgmi kernels can be compared on one node.
//
// --registered: the buffers are peer memory (Device::alloc_peer) registered
// with the communicator, so backends with zero-copy paths (xgmi) read and
// write peers' buffers directly instead of staging through their windows.
//
// --graph (GPU): check mode captures every collective of a size plus the ring
// send/recv into one HIP graph and replays it three times with new inputs
// uploaded between replays (each replay must see fresh sequence numbers);
// bench mode captures the timed loop of one op and replays it.
//
// Reference equivalent: none (DLNetBench relies on nccl-tests externally).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <algorithm>
#include <thread>
#include <sstream>

#include "dlnb/strategy.hpp"
#include "dlnb/xgmi.hpp"

namespace dlnb {

namespace {

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Check patterns (the fp8 pass used 1.0 everywhere, so a block
// from the wrong peer, offset or replay passed). Every value is exact in every
// wire dtype, both fp8 formats included, and is a hash of its coordinates:
//   data(r, i)  (all-gather, all-to-all, send/recv): one of 48 values
//               k * 2^(e-2), k = 4..7, e = -3..8 (0.125 .. 448: exact with e5m2's
//               2 mantissa bits, so in e4m3, fp16, bf16, fp32), hashed from
//               (r, i): a block from another peer, another offset (any
//               distance, the 8 / 16-element vector widths included) or the
//               previous replay (its offset moves with the replay) differs in
//               ~47 of 48 elements;
//   red(r, i)   (all-reduce, reduce-scatter) fp8: one-hot - only rank
//               owner(i) = hash(i) % W contributes, a table value, the others
//               0: the sum is exact, and a dropped, doubled, misrouted or stale
//               contribution changes it; other dtypes: 1..8 hashed from (r, i)
//               on every rank (sums <= 64: exact integers).
// Outputs are poisoned (all bits set: NaN in every float format) before every
// operation and every graph replay, so an operation that writes nothing fails.
uint64_t mix(uint64_t a, uint64_t b) {
  uint64_t x = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull);
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

float table_val(uint64_t h) {
  const int k = 4 + static_cast<int>(h % 4);
  const int e = -3 + static_cast<int>((h >> 2) % 12);
  return std::ldexp(static_cast<float>(k), e - 2);
}

bool is_fp8(DType t) { return t == DType::FP8_E4M3 || t == DType::FP8_E5M2; }

// DLNB_COMMTEST_LEGACY_PATTERN=1: the round-3 patterns ((rank % 8 + 1) * (i % 4 + 1),
// fp8: 1.0 everywhere), kept so a test can show which faults they missed.
bool legacy_pattern() {
  static const bool on = env_int("DLNB_COMMTEST_LEGACY_PATTERN", 0) != 0;
  return on;
}
float legacy_val(int rank, size_t i, DType t) {
  if (is_fp8(t)) return 1.0f;
  return static_cast<float>((rank % 8 + 1) * static_cast<int>(i % 4 + 1));
}

float data_val(int rank, size_t i, DType t) {
  if (legacy_pattern()) return legacy_val(rank, i, t);
  return table_val(mix(static_cast<uint64_t>(rank) + 1, i));
}

float red_val(int rank, size_t i, DType t, int W) {
  if (legacy_pattern()) return legacy_val(rank, i, t);
  if (is_fp8(t)) {
    const int owner = static_cast<int>(mix(0x5EEDull, i) % static_cast<uint64_t>(W));
    return rank == owner ? table_val(mix(0xABCull, i)) : 0.0f;
  }
  return static_cast<float>(1 + mix(static_cast<uint64_t>(rank) + 101, i) % 8);
}

void encode(DType t, float f, void* p, size_t i) {
  switch (t) {
    case DType::BF16: static_cast<uint16_t*>(p)[i] = float_to_bf16(f); break;
    case DType::FP16: static_cast<uint16_t*>(p)[i] = float_to_fp16(f); break;
    case DType::FP32: static_cast<float*>(p)[i] = f; break;
    case DType::FP8_E4M3: static_cast<uint8_t*>(p)[i] = float_to_fp8e4m3(f); break;
    case DType::FP8_E5M2: static_cast<uint8_t*>(p)[i] = float_to_fp8e5m2(f); break;
  }
}

float decode(DType t, const void* p, size_t i) {
  switch (t) {
    case DType::BF16: return bf16_to_float(static_cast<const uint16_t*>(p)[i]);
    case DType::FP16: return fp16_to_float(static_cast<const uint16_t*>(p)[i]);
    case DType::FP32: return static_cast<const float*>(p)[i];
    case DType::FP8_E4M3: return fp8e4m3_to_float(static_cast<const uint8_t*>(p)[i]);
    case DType::FP8_E5M2: return fp8e5m2_to_float(static_cast<const uint8_t*>(p)[i]);
  }
  return 0.f;
}

struct Tester {
  Context& ctx;
  Communicator& comm;
  Stream& s;
  DType t;
  size_t es;
  int W, me;
  long long failures = 0;
  // --registered: buffers of the maximum size, registered once (a
  // registration pairs buffers by order across ranks, so they are not
  // re-created per size); get(.., i) hands out buffer i of the pool.
  std::vector<Buffer>* pool = nullptr;
  // also check an in-place all-to-all (backends that support it: xgmi)
  bool inplace_a2a = false;
  // Buffer i of at least `bytes`: a fresh allocation kept in `keep`, or the
  // registered pool's buffer i.
  void* get(std::vector<Buffer>& keep, size_t bytes, size_t i) {
    if (!pool || pool->empty()) {
      keep.push_back(ctx.dev->alloc(std::max<size_t>(1, bytes)));
      return keep.back().data();
    }
    DLNB_REQUIRE(i < pool->size() && bytes <= (*pool)[i].bytes(), "commtest: registered pool too small");
    return (*pool)[i].data();
  }

  void upload(void* b, const std::vector<char>& h) {
    ctx.dev->copy_async(b, h.data(), h.size(), s);
    s.synchronize();
  }
  std::vector<char> download(const void* b, size_t bytes) {
    std::vector<char> h(bytes);
    ctx.dev->copy_async(h.data(), b, bytes, s);
    s.synchronize();
    return h;
  }
  // host vector of n elements: element i = data(rank, off + i) or red(rank, off + i)
  std::vector<char> pattern(int rank, size_t off, size_t n) {
    std::vector<char> h(n * es);
    for (size_t i = 0; i < n; ++i) encode(t, data_val(rank, off + i, t), h.data(), i);
    return h;
  }
  std::vector<char> red_pattern(int rank, size_t off, size_t n) {
    std::vector<char> h(n * es);
    for (size_t i = 0; i < n; ++i) encode(t, red_val(rank, off + i, t, W), h.data(), i);
    return h;
  }
  float val(int rank, size_t i) const { return data_val(rank, i, t); }
  // all bits set: NaN in bf16, fp16, fp32 and both fp8 formats
  void poison(void* b, size_t bytes) { upload(b, std::vector<char>(bytes, static_cast<char>(0xFF))); }
  void expect(const char* what, size_t n, const std::vector<char>& got, size_t i, float want) {
    float g = decode(t, got.data(), i);
    if (g != want) {
      if (failures < 10)
        std::fprintf(stderr, "[commtest] rank %d %s n=%zu: element %zu = %g, expected %g\n", me, what, n, i, g, want);
      ++failures;
    }
  }
  float sum_over_ranks(size_t i) {
    float a = 0.f;
    for (int r = 0; r < W; ++r) a += red_val(r, i, t, W);
    return a;
  }

  void check(size_t n) {
    const long long before = failures;
    std::vector<Buffer> keep;
    void* a = get(keep, n * W * es, 0);
    void* b = get(keep, n * W * es, 1);
    // all-reduce out of place
    upload(a, red_pattern(me, 0, n));
    poison(b, n * es);
    comm.all_reduce(a, b, n, t, s);
    auto got = download(b, n * es);
    for (size_t i = 0; i < n; ++i) expect("all_reduce", n, got, i, sum_over_ranks(i));
    // all-reduce in place (fresh input: an out-of-place op must not have touched it, but check that apart)
    upload(a, red_pattern(me, 0, n));
    comm.all_reduce(a, a, n, t, s);
    got = download(a, n * es);
    for (size_t i = 0; i < n; ++i) expect("all_reduce(in-place)", n, got, i, sum_over_ranks(i));
    // all-gather
    upload(a, pattern(me, 0, n));
    poison(b, n * W * es);
    comm.all_gather(a, b, n, t, s);
    got = download(b, n * W * es);
    for (int r = 0; r < W; ++r)
      for (size_t i = 0; i < n; ++i) expect("all_gather", n, got, r * n + i, val(r, i));
    // reduce-scatter: send has W blocks of n, element j = red(me, j)
    upload(a, red_pattern(me, 0, n * W));
    poison(b, n * es);
    comm.reduce_scatter(a, b, n, t, s);
    got = download(b, n * es);
    for (size_t i = 0; i < n; ++i) expect("reduce_scatter", n, got, i, sum_over_ranks(me * n + i));
    // all-to-all: block p of rank r's send = data(r, p*n + i) -> recv block p on me = data(p, me*n + i)
    upload(a, pattern(me, 0, n * W));
    poison(b, n * W * es);
    comm.all_to_all(a, b, n, t, s);
    got = download(b, n * W * es);
    for (int p = 0; p < W; ++p)
      for (size_t i = 0; i < n; ++i) expect("all_to_all", n, got, p * n + i, val(p, me * n + i));
    if (inplace_a2a) {
      upload(a, pattern(me, 0, n * W));
      comm.all_to_all(a, a, n, t, s);
      got = download(a, n * W * es);
      for (int p = 0; p < W; ++p)
        for (size_t i = 0; i < n; ++i) expect("all_to_all(in-place)", n, got, p * n + i, val(p, me * n + i));
    }
    s.synchronize();
    if (failures != before) std::fprintf(stderr, "[commtest] rank %d: n=%zu FAILED\n", me, n);
  }

  // One graph holding all collectives of size n and a ring send/recv,
  // replayed `reps` times; inputs change between replays, outputs are
  // compared after each.
  void check_graph(Communicator& link, size_t n, int reps) {
    const long long before = failures;
    const size_t nb = n * W * es;
    std::vector<Buffer> keep;
    void *ar_in = get(keep, nb, 0), *ar_out = get(keep, nb, 1), *ar_ip = get(keep, nb, 2);
    void *ag_out = get(keep, nb, 3), *blk_in = get(keep, nb, 4), *rs_out = get(keep, nb, 5);
    void *a2a_out = get(keep, nb, 6), *p_in = get(keep, nb, 7), *p_out = get(keep, nb, 8);
    void *a2a_in = get(keep, nb, 9), *ag_in = get(keep, nb, 10);
    const int next = (me + 1) % W, prev = (me + W - 1) % W;
    auto g = ctx.dev->capture(s, {}, [&] {
      comm.all_reduce(ar_in, ar_out, n, t, s);
      comm.all_reduce(ar_ip, ar_ip, n, t, s);
      comm.all_gather(ag_in, ag_out, n, t, s);
      comm.reduce_scatter(blk_in, rs_out, n, t, s);
      comm.all_to_all(a2a_in, a2a_out, n, t, s);
      if (W > 1) {
        link.group_start();
        link.send(p_in, n, t, next, s);
        link.recv(p_out, n, t, prev, s);
        link.group_end();
      }
    });
    for (int rep = 0; rep < reps; ++rep) {
      // rank r's inputs at replay rep: data / red(r, 7 * rep + i); every output poisoned
      const size_t o = static_cast<size_t>(rep) * 7;
      upload(ar_in, red_pattern(me, o, n));
      upload(ar_ip, red_pattern(me, o, n));
      upload(blk_in, red_pattern(me, o, n * W));
      upload(a2a_in, pattern(me, o, n * W));
      upload(p_in, pattern(me, o, n));
      upload(ag_in, pattern(me, o, n));
      for (void* out : {ar_out, ag_out, rs_out, a2a_out, p_out}) poison(out, nb);
      g->launch(s);
      auto got = download(ar_out, n * es);
      for (size_t i = 0; i < n; ++i) expect("graph all_reduce", n, got, i, sum_over_ranks(o + i));
      got = download(ar_ip, n * es);
      for (size_t i = 0; i < n; ++i) expect("graph all_reduce(in-place)", n, got, i, sum_over_ranks(o + i));
      got = download(ag_out, n * W * es);
      for (int r = 0; r < W; ++r)
        for (size_t i = 0; i < n; ++i) expect("graph all_gather", n, got, r * n + i, val(r, o + i));
      got = download(rs_out, n * es);
      for (size_t i = 0; i < n; ++i) expect("graph reduce_scatter", n, got, i, sum_over_ranks(o + me * n + i));
      got = download(a2a_out, n * W * es);
      for (int p = 0; p < W; ++p)
        for (size_t i = 0; i < n; ++i) expect("graph all_to_all", n, got, p * n + i, val(p, o + me * n + i));
      if (W > 1) {
        got = download(p_out, n * es);
        for (size_t i = 0; i < n; ++i) expect("graph send/recv", n, got, i, val(prev, o + i));
      }
    }
    s.synchronize();
    if (failures != before) std::fprintf(stderr, "[commtest] rank %d: graph n=%zu FAILED\n", me, n);
  }

  void check_p2p(Communicator& link, size_t n) {
    if (W < 2) return;
    std::vector<Buffer> keep;
    void* a = get(keep, n * es, 0);
    void* b = get(keep, n * es, 1);
    const int next = (me + 1) % W, prev = (me + W - 1) % W;
    for (int rep = 0; rep < 3; ++rep) {  // several messages: exercises the double-buffered slots
      upload(a, pattern(me, static_cast<size_t>(rep) * 7, n));
      poison(b, n * es);
      link.group_start();
      link.send(a, n, t, next, s);
      link.recv(b, n, t, prev, s);
      link.group_end();
      auto got = download(b, n * es);
      for (size_t i = 0; i < n; ++i) expect("send/recv", n, got, i, val(prev, static_cast<size_t>(rep) * 7 + i));
    }
  }
};

std::unique_ptr<CommFactory> factory_for(Context& ctx, const std::string& b) {
  std::unique_ptr<CommFactory> f;
  if (b == "rccl") f = make_rccl_factory(ctx.hg(), *ctx.dev);
  else if (b == "xgmi") f = make_xgmi_factory(ctx.hg(), *ctx.dev);
  else if (b == "mixed") f = make_mixed_factory(ctx.hg(), *ctx.dev);
  else if (b == "cpu") f = make_shm_factory(ctx.hg(), *ctx.dev);
  else DLNB_THROW("commtest --suite: unknown backend " << b << " (rccl, xgmi, mixed, cpu)");
  return wrap_comm_faults(std::move(f), *ctx.dev, ctx.rank());
}

// Modes a backend is checked in: eager enqueue and HIP-graph replay; xgmi
// also with registered (zero-copy) buffers, eager and replayed.
std::vector<std::string> suite_modes(const std::string& b) {
  if (b == "xgmi") return {"staged", "registered", "graph", "registered_graph"};
  if (b == "cpu") return {"eager"};
  return {"eager", "graph"};
}

// --suite: the exactness pass of a multi-GPU job (bench.py runs it as a
// child of every rank before any timed phase). For each backend, mode and
// wire dtype it checks every collective plus a ring send/recv at every size
// exactly, and reports one JSON line (rank 0): per-combination results,
// "exact": {backend: ok, backend_mode: ok}, the xgmi release mode that
// passed and the RCCL communicator's own rank count (ncclCommCount).
// xgmi runs with DLNB_XGMI_RELEASE as set (default vmcnt); with
// --release-fallback a failing xgmi backend is re-checked with the
// system-scope release/acquire.
int run_suite(Context& ctx, const std::vector<std::string>& backends, const std::vector<std::string>& dtypes,
              std::vector<size_t> sizes, bool fallback, const std::string& json_path) {
  const int W = ctx.world(), me = ctx.rank();
  if (sizes.empty()) sizes = {4097, 300000, (size_t(1) << 21) + 5};
  size_t maxn = 1, maxes = 1;
  for (size_t n : sizes) maxn = std::max(maxn, n);
  std::vector<DType> types;
  for (const auto& d : dtypes) {
    types.push_back(parse_dtype(d));
    maxes = std::max(maxes, dtype_size(types.back()));
  }
  std::vector<int> all;
  for (int r = 0; r < W; ++r) all.push_back(r);
  const double t_start = now();
  Json results = Json::array();
  Json exact = Json::object();
  Json release_used = nullptr;
  int rccl_nranks = -1;
  auto stream = ctx.dev->create_stream(true);
  int uid = 0;
  for (const std::string& b : backends) {
    std::vector<std::string> releases = {""};
    if (b == "xgmi" || b == "mixed") {
      releases = {env_or("DLNB_XGMI_RELEASE", "vmcnt")};
      if (fallback && releases[0] != "system") releases.push_back("system");
    }
    const std::string saved_release = env_or("DLNB_XGMI_RELEASE", "");
    bool backend_ok = false;
    Json per_mode = Json::object();
    for (const std::string& rel : releases) {
      if (!rel.empty()) setenv("DLNB_XGMI_RELEASE", rel.c_str(), 1);
      auto fac = factory_for(ctx, b);
      backend_ok = true;
      per_mode = Json::object();
      // registered and unregistered modes use separate communicators (a
      // registration is permanent); graph and eager share one.
      for (bool want_reg : {false, true}) {
        std::vector<std::string> modes;
        for (const auto& m : suite_modes(b))
          if ((m.find("registered") != std::string::npos) == want_reg) modes.push_back(m);
        if (modes.empty()) continue;
        const std::string tag = "suite/" + std::to_string(uid++) + "/" + b;
        auto comm = fac->create(tag + "/world", all, maxn * W * maxes, false);
        auto link = fac->create(tag + "/link", all, maxn * maxes, true);
        if (b == "rccl" && comm->library_nranks() >= 0) rccl_nranks = comm->library_nranks();
        std::vector<Buffer> pool;
        if (want_reg && comm->wants_peer_buffers()) {
          for (int i = 0; i < 11; ++i) {
            pool.push_back(ctx.dev->alloc_peer(std::max<size_t>(16, maxn * W * maxes)));
            comm->register_buffer(pool.back().data(), pool.back().bytes());
          }
        }
        for (const std::string& mode : modes) {
          const bool graph = mode.find("graph") != std::string::npos;
          bool mode_ok = true;
          for (DType t : types) {
            const double t0 = now();
            Tester T{ctx, *comm, *stream, t, dtype_size(t), W, me};
            T.pool = pool.empty() ? nullptr : &pool;
            T.inplace_a2a = comm->backend_name() == "XGMI";
            std::string error;
            try {
              for (size_t n : sizes) {
                if (graph) {
                  T.check_graph(*link, n, 3);
                } else {
                  T.check(n);
                  T.check_p2p(*link, n);
                }
              }
              stream->synchronize();
            } catch (const std::exception& e) {
              error = e.what();
              ++T.failures;
            }
            for (Communicator* c : {comm.get(), link.get()}) {
              std::string err = c->async_error();
              if (!err.empty()) {
                if (error.empty()) error = err;
                ++T.failures;
              }
            }
            const long long fails = static_cast<long long>(ctx.hg().allreduce_sum(static_cast<double>(T.failures)));
            const bool ok = fails == 0;
            mode_ok = mode_ok && ok;
            if (!ok) std::fprintf(stderr, "[commtest] suite %s/%s/%s%s%s: %lld failures %s\n", b.c_str(), mode.c_str(),
                                  dtype_name(t), rel.empty() ? "" : " release=", rel.c_str(), fails, error.c_str());
            Json r = Json::object();
            r["backend"] = b;
            r["mode"] = mode;
            r["dtype"] = dtype_name(t);
            if (!rel.empty()) r["release"] = rel;
            r["ok"] = ok;
            r["failures"] = fails;
            r["seconds"] = now() - t0;
            if (!error.empty()) r["error"] = error.substr(0, 200);
            results.push_back(r);
          }
          per_mode[b + "_" + mode] = mode_ok;
          backend_ok = backend_ok && mode_ok;
        }
        stream->synchronize();
        ctx.hg().barrier();  // nobody frees a registered buffer a peer still maps
      }
      if (backend_ok) {
        if (!rel.empty()) release_used = rel;
        break;
      }
    }
    if (!saved_release.empty())
      setenv("DLNB_XGMI_RELEASE", saved_release.c_str(), 1);
    else
      unsetenv("DLNB_XGMI_RELEASE");
    exact[b] = backend_ok;
    for (const auto& kv : per_mode.items()) exact[kv.first] = kv.second;
  }
  bool all_ok = true;
  for (const auto& kv : exact.items()) all_ok = all_ok && kv.second.as_bool();
  // The verdicts are all-reduced, so every rank holds the same report; each
  // writes --json (so every rank of a job can act on it), rank 0 prints it.
  Json j = Json::object();
  j["commtest"] = "suite";
  j["world_size"] = W;
  j["rank"] = me;
  Json sz = Json::array();
  for (size_t n : sizes) sz.push_back(static_cast<double>(n));
  j["sizes"] = sz;
  j["exact"] = exact;
  j["ok"] = all_ok;
  j["xgmi_release"] = release_used;
  j["rccl_nranks"] = rccl_nranks;
  j["results"] = results;
  j["seconds"] = now() - t_start;
  if (ctx.dev->kind() == DeviceKind::GPU) j["runtime"] = runtime_info();
  if (me == 0) std::cout << j.dump() << std::endl;
  if (!json_path.empty()) {
    std::ofstream f(json_path);
    f << j.dump(1) << "\n";
  }
  return all_ok ? 0 : 3;
}

}  // namespace

int info_main(int argc, char** argv) {
  (void)argc, (void)argv;
  Json j = Json::object();
  j["version"] = "dlnetbench_amd 0.1.0 (gfx950)";
  const int ngpu = gpu_device_count();
  j["gpus"] = ngpu;
  if (ngpu > 0) {
    j["runtime"] = runtime_info();
    Json occ = Json::object();
    for (const auto& k : xgmi::occupancy()) occ[k.name] = k.blocks_per_cu;
    j["xgmi_occupancy_blocks_per_cu"] = occ;
    j["xgmi_min_blocks_per_cu"] = xgmi::min_blocks_per_cu();
    j["xgmi_threads_per_block"] = xgmi::kThreads;
  }
  std::cout << j.dump() << std::endl;
  return 0;
}

int commtest_main(int argc, char** argv) {
  std::string backend = "auto", devices, dtype = "bf16", sizes_s, json_path, backends_s = "rccl,xgmi",
              dtypes_s = "bf16,fp8_e4m3";
  bool bench = false, graph = false, registered = false, suite = false, fallback = false;
  int iters = 20, warmup = 5, ranks = 2;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* what) -> std::string {
      if (i + 1 >= argc) DLNB_THROW("missing value for " << what);
      return argv[++i];
    };
    if (a == "--backend") backend = val("--backend");
    else if (a == "-d" || a == "--devices") devices = val("-d");
    else if (a == "--dtype") dtype = val("--dtype");
    else if (a == "--sizes") sizes_s = val("--sizes");
    else if (a == "--bench") bench = true;
    else if (a == "--graph") graph = true;
    else if (a == "--registered") registered = true;
    else if (a == "--suite") suite = true;
    else if (a == "--backends") backends_s = val("--backends");
    else if (a == "--dtypes") dtypes_s = val("--dtypes");
    else if (a == "--release-fallback") fallback = true;
    else if (a == "--iters") iters = std::stoi(val("--iters"));
    else if (a == "--warmup") warmup = std::stoi(val("--warmup"));
    else if (a == "--ranks") ranks = std::stoi(val("--ranks"));
    else if (a == "--json") json_path = val("--json");
    else if (a == "-h" || a == "--help") {
      std::cout << "Usage: dlnb commtest [--backend auto|rccl|xgmi|mixed|cpu|loopback|loopback-cpu] [--ranks N] [-d 0,1,..]\n"
                   "                     [--dtype bf16|fp16|fp32|fp8_e4m3|fp8_e5m2]\n"
                   "                     [--sizes n1,n2,..] [--bench] [--iters N] [--warmup N] [--graph]\n"
                   "  sizes are elements per rank; check mode verifies every collective exactly\n"
                   "  --graph: capture the operations into a HIP graph and replay it (rccl, xgmi)\n"
                   "  --registered: peer-memory buffers registered with the communicator (zero-copy paths)\n"
                   "       dlnb commtest --suite [--backends rccl,xgmi] [--dtypes bf16,fp8_e4m3] [--sizes ..]\n"
                   "                     [--release-fallback] [--json PATH]\n"
                   "  exactness pass over every backend x mode (eager/graph, xgmi staged/registered) x dtype;\n"
                   "  one JSON line with \"exact\": {backend: ok, ...}, the xgmi release mode and ncclCommCount\n";
      return 0;
    } else DLNB_THROW("unknown option " << a);
  }
  auto body = [&](std::unique_ptr<Bootstrap> boot) -> int {
  Context ctx;
  ctx.boot = std::move(boot);
  if (suite) {
    std::vector<std::string> bs, ds;
    for (auto& x : split(backends_s, ',')) bs.push_back(trim(x));
    for (auto& x : split(dtypes_s, ',')) ds.push_back(trim(x));
    DLNB_REQUIRE(!bs.empty(), "commtest --suite: no backends");
    std::vector<size_t> sz;
    if (!sizes_s.empty())
      for (auto& x : split(sizes_s, ',')) sz.push_back(static_cast<size_t>(std::stoull(x)));
    select_backend(ctx, bs[0], devices);
    const int rc = run_suite(ctx, bs, ds, sz, fallback, json_path);
    ctx.hg().barrier();
    ctx.hg().store().finish();
    return rc;
  }
  const std::string be = select_backend(ctx, backend, devices);
  DLNB_REQUIRE(!graph || be == "rccl" || be == "xgmi" || be == "mixed", "commtest --graph needs a GPU backend");
  const DType t = parse_dtype(dtype);
  const int W = ctx.world(), me = ctx.rank();
  std::vector<size_t> sizes;
  if (sizes_s.empty()) {
    if (bench)
      for (size_t n = 1024; n <= (size_t(256) << 20); n *= 4) sizes.push_back(n);
    else
      sizes = {1, 7, 8, 100, 4097, 65536, 300007, (size_t(1) << 21) + 5};
  } else {
    for (auto& x : split(sizes_s, ',')) sizes.push_back(static_cast<size_t>(std::stoull(x)));
  }
  size_t maxn = 1;
  for (size_t n : sizes) maxn = std::max(maxn, n);
  std::vector<int> all;
  for (int r = 0; r < W; ++r) all.push_back(r);
  const size_t es = dtype_size(t);
  auto comm = ctx.comms->create("commtest/world", all, maxn * W * es, false);
  auto link = ctx.comms->create("commtest/link", all, maxn * es, true);
  auto stream = ctx.dev->create_stream(true);
  Tester T{ctx, *comm, *stream, t, es, W, me};
  T.inplace_a2a = comm->backend_name() == "XGMI";
  const bool reg = registered && comm->wants_peer_buffers();
  std::vector<Buffer> pool;
  if (reg && !bench) {
    for (int i = 0; i < 11; ++i) {
      pool.push_back(ctx.dev->alloc_peer(std::max<size_t>(16, maxn * W * es)));
      comm->register_buffer(pool.back().data(), pool.back().bytes());
    }
    T.pool = &pool;
  }
  long long total_fail = 0;
  if (!bench) {
    const bool verbose = env_int("DLNB_COMMTEST_VERBOSE", 0) != 0;
    for (size_t n : sizes) {
      const double t0 = now();
      if (verbose) std::fprintf(stderr, "[commtest] rank %d: collectives n=%zu\n", me, n);
      if (graph) {
        T.check_graph(*link, n, 3);
        continue;
      }
      T.check(n);
      const double t1 = now();
      if (verbose) std::fprintf(stderr, "[commtest] rank %d: send/recv n=%zu (collectives took %.3f s)\n", me, n, t1 - t0);
      T.check_p2p(*link, n);
      if (verbose) std::fprintf(stderr, "[commtest] rank %d: n=%zu send/recv took %.3f s\n", me, n, now() - t1);
    }
    // a device-side wait that timed out is a failure even if the data came
    for (Communicator* c : {comm.get(), link.get()}) {
      std::string err = c->async_error();
      if (!err.empty()) {
        std::fprintf(stderr, "[commtest] rank %d: %s\n", me, err.c_str());
        ++T.failures;
      }
    }
    total_fail = static_cast<long long>(ctx.hg().allreduce_sum(static_cast<double>(T.failures)));
    if (me == 0) {
      Json j = Json::object();
      j["commtest"] = "check";
      j["backend"] = comm->backend_name();
      j["graph"] = graph;
      j["registered"] = reg;
      j["world_size"] = W;
      j["dtype"] = dtype_name(t);
      Json sz = Json::array();
      for (size_t n : sizes) sz.push_back(static_cast<double>(n));
      j["sizes"] = sz;
      j["failures"] = static_cast<double>(total_fail);
      j["ok"] = total_fail == 0;
      std::cout << j.dump() << std::endl;
    }
  } else {
    Buffer a = reg ? ctx.dev->alloc_peer(maxn * W * es) : ctx.dev->alloc(maxn * W * es);
    Buffer b = reg ? ctx.dev->alloc_peer(maxn * W * es) : ctx.dev->alloc(maxn * W * es);
    if (reg) {
      comm->register_buffer(a.data(), a.bytes());
      comm->register_buffer(b.data(), b.bytes());
    }
    ctx.dev->fill_random(a.data(), maxn * W, t, 7 + me, *stream);
    stream->synchronize();
    struct K {
      const char* name;
      CollKind kind;  // bus-bandwidth accounting
      bool copy;      // the local D2D copy roofline, not a collective
    };
    // "copy": one device-to-device copy of the rank's n elements (the local
    // HBM roofline the collectives' kernels are compared against);
    // "sendrecv": a ring exchange on the point-to-point communicator (send n
    // to the next rank, receive n from the previous one: nccl-tests sendrecv).
    std::vector<K> kinds = {{"all_reduce", CollKind::AllReduce, false},
                            {"all_gather", CollKind::AllGather, false},
                            {"reduce_scatter", CollKind::ReduceScatter, false},
                            {"all_to_all", CollKind::AllToAll, false},
                            {"copy", CollKind::SendRecv, true}};
    if (W > 1) kinds.push_back({"sendrecv", CollKind::SendRecv, false});
    const int next = (me + 1) % W, prev = (me + W - 1) % W;
    for (size_t n : sizes) {
      for (const K& k : kinds) {
        auto op = [&] {
          if (k.copy) {
            ctx.dev->copy_async(b.data(), a.data(), n * es, *stream);
            return;
          }
          switch (k.kind) {
            case CollKind::SendRecv:
              link->group_start();
              link->send(a.data(), n, t, next, *stream);
              link->recv(b.data(), n, t, prev, *stream);
              link->group_end();
              break;
            case CollKind::AllReduce: comm->all_reduce(a.data(), b.data(), n, t, *stream); break;
            case CollKind::AllGather: comm->all_gather(a.data(), b.data(), n, t, *stream); break;
            case CollKind::ReduceScatter: comm->reduce_scatter(a.data(), b.data(), n, t, *stream); break;
            default: comm->all_to_all(a.data(), b.data(), n, t, *stream); break;
          }
        };
        std::unique_ptr<GraphExec> g;
        if (graph)
          g = ctx.dev->capture(*stream, {}, [&] {
            for (int it = 0; it < iters; ++it) op();
          });
        for (int w = 0; w < warmup; ++w) op();
        stream->synchronize();
        ctx.hg().barrier();
        const double t0 = now();
        if (g)
          g->launch(*stream);
        else
          for (int it = 0; it < iters; ++it) op();
        stream->synchronize();
        const double dt = ctx.hg().allreduce_max(now() - t0) / iters;
        // algorithm bytes per rank (nccl-tests): AR/RS/A2A n*W... AG output
        double bytes = static_cast<double>(n) * es;
        if (k.kind != CollKind::AllReduce && k.kind != CollKind::SendRecv) bytes *= W;
        if (me == 0) {
          Json j = Json::object();
          j["commtest"] = "bench";
          j["backend"] = comm->backend_name();
          j["graph"] = graph;
          j["registered"] = reg;
          j["op"] = k.name;
          j["world_size"] = W;
          j["dtype"] = dtype_name(t);
          j["count"] = static_cast<double>(n);
          j["bytes"] = bytes;
          j["time_us"] = dt * 1e6;
          j["algbw_GBps"] = bytes / dt / 1e9;
          j["busbw_GBps"] = k.copy ? 0.0 : bytes / dt / 1e9 * busbw_factor(k.kind, W);
          std::cout << j.dump() << std::endl;
        }
      }
    }
  }
  stream->synchronize();
  ctx.hg().barrier();
  ctx.hg().store().finish();
  return total_fail == 0 ? 0 : 3;
  };
  if (backend != "loopback" && backend != "loopback-cpu") return body(bootstrap_from_env(""));
  // loopback: the ranks are threads of this process (see comm_loopback.cpp)
  auto store = std::make_shared<LocalStore>();
  auto hub = make_loopback_hub(ranks, static_cast<double>(env_int("DLNB_STORE_TIMEOUT", 900)));
  std::vector<int> rc(static_cast<size_t>(ranks), 0);
  std::vector<std::thread> threads;
  for (int r = 0; r < ranks; ++r)
    threads.emplace_back([&, r] {
      try {
        rc[static_cast<size_t>(r)] = body(bootstrap_loopback(r, ranks, store, hub));
      } catch (const std::exception& e) {
        std::fprintf(stderr, "[commtest] rank %d: %s\n", r, e.what());
        rc[static_cast<size_t>(r)] = 2;
        loopback_abort(*hub, e.what());
        store->abort(e.what());
      }
    });
  for (auto& t : threads) t.join();
  return *std::max_element(rc.begin(), rc.end());
}

}  // namespace dlnb
