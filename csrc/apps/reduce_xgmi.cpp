// reduce_xgmi — cross-GPU reduction benchmark: one process per MI355X, RCCL over xGMI.
//
// Two semantics:
//   --mode=vector  reduce.c on GPUs: each rank holds N/P elements, element-wise ncclReduce to
//                  root 0 (or ncclAllReduce), {MAX,MIN,SUM} x {INT,DOUBLE} x RETRY_COUNT, output
//                  byte-compatible with mpi/reduce.c:67-69,80-82,94-96 (GB = 2^30 B of total data).
//   --mode=scalar  the north star: every rank reduces its contiguous shard of a global array with
//                  the single-pass HIP kernel, then a 1-element ncclAllReduce — the hybrid
//                  local-reduce + scalar MPI_Reduce of the vendored simpleMPI
//                  (cuda/C/src/simpleMPI/simpleMPI.cpp:92-98) on RCCL.
// Launch: torchrun / mpirun / srun (see comm.hpp); rank r uses GPU LOCAL_RANK % device_count.
// Timing: host barrier, then `--iters` back-to-back iterations on one stream (optionally replayed
// from a hipGraph, --graph), stream drained with an RCCL async-error watchdog; the MAX over
// ranks of the per-iteration time is reported (fixes reduce.c's root-only, barrier-less rdtsc,
// bug B8). Verification: vector mode checks sampled indices against the host-combined inputs of
// all ranks; scalar mode checks the all-reduced value against the host fold of every rank's
// local result and each local result against the ladder's kernel 6 (an independent kernel).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "mireduce/version.hpp"
#include "mireduce/check.hpp"
#include "mireduce/cli.hpp"
#include "mireduce/comm.hpp"
#include "mireduce/cpu_reference.hpp"
#include "mireduce/device.hpp"
#include "mireduce/direct.hpp"
#include "mireduce/peer_access.hpp"
#include "mireduce/fault.hpp"
#include "mireduce/ladder.hpp"
#include "mireduce/mt19937.hpp"
#include "mireduce/reduce.hpp"
#include "mireduce/report.hpp"
#include "mireduce/timer.hpp"
#include "mireduce/trace.hpp"
#include "mireduce/xrank.hpp"

using namespace mireduce;

namespace {

constexpr uint64_t kNumInts = 512ull * 1024 * 1024;     // mpi/constants.h:1
constexpr uint64_t kNumDoubles = 256ull * 1024 * 1024;  // mpi/constants.h:2

const std::set<std::string> kKnown = {"mode", "collective", "dtypes", "ops", "ints", "doubles", "longs", "floats",
                                      "n", "retries", "warmup", "iters", "root", "json", "graph", "mt19937",
                                      "noverify", "seed", "help", "version", "unroll", "block", "wg-per-cu", "policy",
                                      "units", "timeout", "trace", "single-process", "inject-fault",
                                      "direct-grid"};

struct Ctx {
  LaunchEnv env;
  int device = 0;
  std::unique_ptr<TcpBootstrap> boot;
  std::unique_ptr<RcclComm> comm;      // RCCL collectives
  std::unique_ptr<DirectAllreduce> direct;  // --collective=direct|direct-reduce (peer reads over xGMI)
  int direct_grid = 0;                       // workgroups per direct collective (0: one per CU)
  hipStream_t stream = nullptr;
  int retries = 5, warmup = 1, iters = 10, root = 0;
  std::string mode = "vector", collective, json;
  bool graph = false, verify = true, mt = false;
  uint64_t seed = 0x5EED;
  double timeout_s = 300;
  double direct_timeout_s = 10;  // device-side wait bound of the direct kernels (--timeout sets both)
  bool units_gb = false;  // gnuplot column in 2^30 (reduce.c) unless --units=gb
  ReduceConfig kcfg;
  FaultInjector fault;  // --inject-fault / MIREDUCE_INJECT_FAULT (failure-detection tests)
  long fault_step = 0;  // counts timed collectives / steps on this rank
};

// Fault injection "corrupt": make this rank's contribution at element `i` wrong for one timed
// batch (SUM: +1, MIN: lowest, MAX: highest); returns the original bytes for restore.
template <class T>
T corrupt_element(void* d, uint64_t i, Op o) {
  T v;
  HIP_CHECK(hipMemcpy(&v, static_cast<T*>(d) + i, sizeof(T), hipMemcpyDeviceToHost));
  const T bad = o == Op::Sum ? wrap_add(v, T(1))
                             : (o == Op::Min ? std::numeric_limits<T>::lowest() : std::numeric_limits<T>::max());
  HIP_CHECK(hipMemcpy(static_cast<T*>(d) + i, &bad, sizeof(T), hipMemcpyHostToDevice));
  return v;
}

struct SavedElement {
  void* ptr = nullptr;
  unsigned char bytes[8] = {0};
  size_t size = 0;
};

SavedElement corrupt_any(void* d, uint64_t i, DType t, Op o) {
  SavedElement s;
  s.size = dtype_size(t);
  s.ptr = static_cast<unsigned char*>(d) + i * s.size;
  switch (t) {
    case DType::Int32: { const int32_t v = corrupt_element<int32_t>(d, i, o); std::memcpy(s.bytes, &v, 4); break; }
    case DType::Int64: { const int64_t v = corrupt_element<int64_t>(d, i, o); std::memcpy(s.bytes, &v, 8); break; }
    case DType::Float32: { const float v = corrupt_element<float>(d, i, o); std::memcpy(s.bytes, &v, 4); break; }
    case DType::Float64: { const double v = corrupt_element<double>(d, i, o); std::memcpy(s.bytes, &v, 8); break; }
    default: break;
  }
  return s;
}

void restore_element(const SavedElement& s) {
  if (s.ptr) HIP_CHECK(hipMemcpy(s.ptr, s.bytes, s.size, hipMemcpyHostToDevice));
}

uint64_t global_count(DType t, uint64_t ints, uint64_t longs, uint64_t floats, uint64_t doubles) {
  switch (t) {
    case DType::Int32: return ints;
    case DType::Int64: return longs;
    case DType::Float32: return floats;
    case DType::Float64: return doubles;
    default: break;
  }
  return 0;
}

void sync_stream(Ctx& c) {
  if (c.comm) c.comm->synchronize(c.stream, c.timeout_s);
  else HIP_CHECK(hipStreamSynchronize(c.stream));
  // The direct kernels never hang on a lost peer: their bounded waits set a sticky error word.
  if (c.direct && c.direct->error())
    throw Error("direct: a peer's barrier flag never arrived (device-side wait timed out after --timeout)");
}

bool is_direct(const Ctx& c) { return c.collective == "direct" || c.collective == "direct-reduce"; }
// Collectives that need no RCCL communicator (and so may share one GPU between ranks in tests).
bool needs_no_rccl(const Ctx& c) { return is_direct(c) || c.collective == "fused"; }

// Time `iters` repetitions of `body` on the stream (optionally as one hipGraph replay).
template <class F>
double time_iters(Ctx& c, F&& body) {
  hipGraphExec_t exec = nullptr;
  hipGraph_t graph = nullptr;
  if (c.graph) {
    HIP_CHECK(hipStreamBeginCapture(c.stream, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < c.iters; ++i) body();
    HIP_CHECK(hipStreamEndCapture(c.stream, &graph));
    HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphLaunch(exec, c.stream));  // upload / first replay outside the clock
    sync_stream(c);
  }
  c.boot->barrier();
  const double t0 = StopWatch::now_s();
  if (c.graph) HIP_CHECK(hipGraphLaunch(exec, c.stream));
  else
    for (int i = 0; i < c.iters; ++i) body();
  sync_stream(c);
  const double dt = (StopWatch::now_s() - t0) / c.iters;
  if (exec) HIP_CHECK(hipGraphExecDestroy(exec));
  if (graph) HIP_CHECK(hipGraphDestroy(graph));
  return c.boot->max_double(dt);
}

// The RCCL tuning knobs this process ran with (tools/sweep.py --rccl-knobs sets them per point):
// "NCCL_ALGO=Ring NCCL_PROTO=Simple ..." for every NCCL_* / RCCL_* variable set, "" for none.
std::string rccl_env() {
  std::string out;
  for (const char* k : {"NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_BUFFSIZE",
                        "NCCL_NTHREADS", "RCCL_MSCCL_ENABLE", "RCCL_MSCCLPP_ENABLE"}) {
    if (const char* v = std::getenv(k)) {
      if (!out.empty()) out += ' ';
      out += std::string(k) + '=' + v;
    }
  }
  return out;
}

void emit(Ctx& c, DType t, Op o, double bytes_total, double dt, Json extra) {
  const double gib = bytes_total / dt / kGiB;
  const double gb = bytes_total / dt / kGB;
  if (c.env.rank == c.root) {
    std::printf("%s\n", gnuplot_line(dtype_gnuplot_name(t), op_name(o), c.env.world, c.units_gb ? gb : gib).c_str());
    std::fflush(stdout);
    if (!c.json.empty()) {
      extra.set("app", "reduce_xgmi").set("mode", c.mode).set("collective", c.collective)
          .set("dtype", dtype_gnuplot_name(t)).set("op", op_name(o)).set("ranks", c.env.world)
          .set("bytes_total", bytes_total).set("seconds", dt).set("gib_per_s", gib).set("gb_per_s", gb)
          .set("iters", c.iters).set("graph", c.graph).set("rccl_version", RcclComm::version())
          .set("launcher", c.env.launcher).set("rccl_env", rccl_env());
      extra.write_file(c.json);
    }
  }
}

// ------------------------------------------------------------------------------ vector mode
template <class T>
bool check_samples(Ctx& c, Op o, const void* d_send, const void* d_recv, uint64_t count) {
  const int kS = 16;
  std::vector<uint64_t> idx(kS);
  for (int s = 0; s < kS; ++s) idx[s] = (static_cast<uint64_t>(s) * 2654435761ull + 7) % count;
  std::vector<T> mine(kS), got(kS), all(static_cast<size_t>(kS) * c.env.world);
  for (int s = 0; s < kS; ++s) {
    HIP_CHECK(hipMemcpy(&mine[s], static_cast<const T*>(d_send) + idx[s], sizeof(T), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(&got[s], static_cast<const T*>(d_recv) + idx[s], sizeof(T), hipMemcpyDeviceToHost));
  }
  c.boot->allgather(mine.data(), all.data(), kS * sizeof(T));
  const bool holder = c.collective == "allreduce" || c.collective == "direct" || c.env.rank == c.root;
  int ok = 1;
  if (holder) {
    for (int s = 0; s < kS; ++s) {
      T e = all[s];
      for (int r = 1; r < c.env.world; ++r) {
        const T v = all[static_cast<size_t>(r) * kS + s];
        if (o == Op::Sum) e = wrap_add(e, v);
        else if (o == Op::Min) e = MinOp::apply(e, v);
        else e = MaxOp::apply(e, v);
      }
      if constexpr (std::is_floating_point_v<T>) {
        const double tol = o == Op::Sum ? 1e-12 * c.env.world * (std::fabs(static_cast<double>(e)) + 1.0) : 0.0;
        if (std::fabs(static_cast<double>(e) - static_cast<double>(got[s])) > tol) ok = 0;
      } else if (e != got[s]) {
        ok = 0;
      }
    }
  }
  std::vector<int> oks(c.env.world);
  c.boot->allgather(&ok, oks.data(), sizeof ok);
  return std::all_of(oks.begin(), oks.end(), [](int v) { return v != 0; });
}

bool run_vector(Ctx& c, const std::vector<DType>& dtypes, const std::vector<Op>& ops,
                const std::vector<uint64_t>& counts) {
  struct B {
    DType t;
    uint64_t count;
    DeviceBuffer send, recv;
  };
  std::vector<B> bufs;
  for (size_t k = 0; k < dtypes.size(); ++k) {
    const DType t = dtypes[k];
    B b{t, std::max<uint64_t>(1, counts[k] / c.env.world), {}, {}};
    b.send.allocate(b.count * dtype_size(t));
    b.recv.allocate(b.count * dtype_size(t));
    if (c.mt) {  // reduce.c's exact data: MT19937 seeded {rank,0x123,...}, host-generated, H2D
      Mt19937 g;
      const uint64_t seeds[6] = {static_cast<uint64_t>(c.env.rank), 0x123, 0x234, 0x345, 0x456, 0x789};
      g.init_by_array(seeds, 6);
      std::vector<unsigned char> h(b.count * dtype_size(t));
      for (uint64_t i = 0; i < b.count; ++i) {
        if (t == DType::Int32) reinterpret_cast<int32_t*>(h.data())[i] = static_cast<int32_t>(g.genrand_int32());
        else if (t == DType::Float64) reinterpret_cast<double*>(h.data())[i] = g.genrand_res53();
        else if (t == DType::Float32) reinterpret_cast<float*>(h.data())[i] = static_cast<float>(g.genrand_res53());
        else reinterpret_cast<int64_t*>(h.data())[i] = (static_cast<int64_t>(g.genrand_int32()) << 32) | g.genrand_int32();
      }
      HIP_CHECK(hipMemcpy(b.send.get(), h.data(), h.size(), hipMemcpyHostToDevice));
    } else {
      FillSpec fs;
      fs.pattern = dtype_is_float(t) ? Pattern::Uniform : Pattern::FullRange;
      fs.seed = c.seed + static_cast<uint64_t>(c.env.rank);  // rank-seeded like reduce.c:38-41
      fill_device(b.send.get(), b.count, t, fs, c.stream);
    }
    bufs.push_back(std::move(b));
  }
  HIP_CHECK(hipStreamSynchronize(c.stream));
  if (is_direct(c)) {  // registered (IPC-shared) buffers sized for the largest dtype
    size_t mx = 0;
    for (auto& b : bufs) mx = std::max(mx, b.count * dtype_size(b.t));
    c.direct = std::make_unique<DirectAllreduce>(c.device, mx, c.direct_grid, c.direct_timeout_s);
    const std::vector<char> mine = c.direct->handles();
    std::vector<char> all(mine.size() * c.env.world);
    c.boot->allgather(mine.data(), all.data(), mine.size());
    std::vector<std::vector<char>> hs(c.env.world);
    for (int r = 0; r < c.env.world; ++r)
      hs[r].assign(all.begin() + static_cast<long>(r * mine.size()), all.begin() + static_cast<long>((r + 1) * mine.size()));
    c.direct->connect(c.env.rank, c.env.world, hs);
    c.boot->barrier();  // every rank mapped every peer before the first collective
  }
  auto body_for = [&](B& b, Op o) {
    return [&c, &b, o] {
      TraceRange tr("reduce_xgmi.vector_collective");
      if (c.collective == "reduce") c.comm->reduce(b.send.get(), b.recv.get(), b.count, b.t, o, c.root, c.stream);
      else if (c.collective == "allreduce") c.comm->allreduce(b.send.get(), b.recv.get(), b.count, b.t, o, c.stream);
      else if (c.collective == "direct") c.direct->allreduce(b.count, b.t, o, c.stream);
      else c.direct->reduce(b.count, b.t, o, c.root, c.stream);
    };
  };
  auto stage = [&](B& b) {  // direct mode: this dtype's data into the registered input buffer
    if (c.direct) {
      HIP_CHECK(hipMemcpyAsync(c.direct->in(), b.send.get(), b.count * dtype_size(b.t), hipMemcpyDeviceToDevice, c.stream));
      HIP_CHECK(hipStreamSynchronize(c.stream));  // (the kernel's entry barrier orders it for the peers)
    }
  };
  const void* (*in_ptr)(Ctx&, B&) = [](Ctx& cc, B& bb) -> const void* { return cc.direct ? cc.direct->in() : bb.send.get(); };
  const void* (*out_ptr)(Ctx&, B&) = [](Ctx& cc, B& bb) -> const void* { return cc.direct ? cc.direct->out() : bb.recv.get(); };
  const int saved_iters = c.iters;
  c.iters = 1;
  const bool saved_graph = c.graph;
  c.graph = false;
  for (int w = 0; w < c.warmup; ++w)
    for (auto& b : bufs) {
      stage(b);
      time_iters(c, body_for(b, Op::Sum));  // reduce.c:61-64
    }
  c.iters = saved_iters;
  c.graph = saved_graph;
  if (c.env.rank == c.root) std::printf("%s\n", gnuplot_header().c_str());
  bool ok = true;
  for (int x = 0; x < c.retries; ++x) {
    for (auto& b : bufs) {
      stage(b);
      for (Op o : ops) {
        HIP_CHECK(hipMemsetAsync(const_cast<void*>(out_ptr(c, b)), 0, b.count * dtype_size(b.t), c.stream));  // bzero (reduce.c:74)
        SavedElement saved;
        if (c.fault.at(c.env.rank, c.fault_step++, "vector collective") && b.count)
          saved = corrupt_any(const_cast<void*>(in_ptr(c, b)), 7 % b.count, b.t, o);  // a sampled index
        const double dt = time_iters(c, body_for(b, o));
        restore_element(saved);  // the check compares against the clean inputs
        const double bytes = static_cast<double>(b.count) * c.env.world * dtype_size(b.t);
        const double algbw = static_cast<double>(b.count) * dtype_size(b.t) / dt / kGB;
        const bool all = c.collective == "allreduce" || c.collective == "direct";
        const double busbw = all ? algbw * 2.0 * (c.env.world - 1) / c.env.world : algbw;
        bool vok = true;
        if (c.verify && x == 0) {
          switch (b.t) {
            case DType::Int32: vok = check_samples<int32_t>(c, o, in_ptr(c, b), out_ptr(c, b), b.count); break;
            case DType::Int64: vok = check_samples<int64_t>(c, o, in_ptr(c, b), out_ptr(c, b), b.count); break;
            case DType::Float32: vok = check_samples<float>(c, o, in_ptr(c, b), out_ptr(c, b), b.count); break;
            case DType::Float64: vok = check_samples<double>(c, o, in_ptr(c, b), out_ptr(c, b), b.count); break;
            default: break;
          }
          ok = ok && vok;
        }
        Json j;
        j.set("count_per_rank", b.count).set("algbw_gb_per_s", algbw).set("busbw_gb_per_s", busbw).set("retry", x);
        if (c.verify && x == 0) j.set("verified", vok);
        emit(c, b.t, o, bytes, dt, j);
      }
    }
  }
  return ok;
}

// ------------------------------------------------------------------------------ scalar mode
bool run_scalar(Ctx& c, const std::vector<DType>& dtypes, const std::vector<Op>& ops,
                const std::vector<uint64_t>& counts) {
  Workspace ws(c.device);
  DeviceBuffer out(8), loc(8), oracle(8);
  // --collective=fused: the kernel's finisher folds every rank's partial through IPC mailboxes
  // (xrank.hpp) — one kernel per global reduction, no RCCL.
  std::unique_ptr<XrankChannel> channel;
  ReduceConfig step_cfg = c.kcfg;
  if (c.collective == "fused") {
    channel = std::make_unique<XrankChannel>(c.device, c.direct_timeout_s);
    const IpcHandleBytes mine = channel->handle();
    std::vector<IpcHandleBytes> all(c.env.world);
    c.boot->allgather(mine.data(), all.data(), mine.size());
    channel->connect(c.env.rank, c.env.world, all);
    c.boot->barrier();  // every rank mapped every mailbox before the first launch
    step_cfg.xrank = channel->device_desc();
  }
  if (c.env.rank == c.root) std::printf("%s\n", gnuplot_header().c_str());
  bool ok = true;
  for (size_t k = 0; k < dtypes.size(); ++k) {
    const DType t = dtypes[k];
    const uint64_t n = counts[k];
    const uint64_t base = n / c.env.world, rem = n % c.env.world;
    const uint64_t count = base + (static_cast<uint64_t>(c.env.rank) < rem ? 1 : 0);
    const uint64_t offset = c.env.rank * base + std::min<uint64_t>(c.env.rank, rem);
    DeviceBuffer x(std::max<uint64_t>(count, 1) * dtype_size(t));
    FillSpec fs;
    fs.pattern = dtype_is_float(t) ? Pattern::Uniform : Pattern::FullRange;
    fs.seed = c.seed;
    fs.offset = offset;  // one logical global array, independent of the rank count
    fill_device(x.get(), count, t, fs, c.stream);
    HIP_CHECK(hipStreamSynchronize(c.stream));
    for (Op o : ops) {
      const DType acc = default_acc(t, o);
      auto body = [&] {
        TraceRange tr("reduce_xgmi.scalar_step");
        reduce(x.get(), count, t, o, acc, out.get(), ws, c.stream, step_cfg);
        if (!channel) c.comm->allreduce(out.get(), out.get(), 1, acc, o, c.stream);
      };
      for (int w = 0; w < c.warmup; ++w) {
        body();
        sync_stream(c);
      }
      for (int x_ = 0; x_ < c.retries; ++x_) {
        SavedElement saved;
        if (c.fault.at(c.env.rank, c.fault_step++, "scalar step") && count) saved = corrupt_any(x.get(), 0, t, o);
        const double dt = time_iters(c, body);
        restore_element(saved);
        if (channel && channel->error())
          throw Error("fused: a peer's partial never arrived (device-side wait timed out after --timeout)");
        if (ws.error())  // polled fan-in reached its wait bound: the results are poisoned
          throw Error("polled fan-in: a launch reached its wait bound (device-side error word set)");
        Json j;
        j.set("n_total", n).set("count_per_rank", count).set("retry", x_);
        bool vok = true;
        if (c.verify && x_ == 0) {
          unsigned char g[8] = {0}, l[8] = {0}, orc[8] = {0};
          HIP_CHECK(hipMemcpy(g, out.get(), 8, hipMemcpyDeviceToHost));
          reduce(x.get(), count, t, o, acc, loc.get(), ws, c.stream, c.kcfg);
          // Independent oracle for the local result: the ladder's kernel 6 (a different kernel,
          // grid and fold order), not the streaming kernel's other mode.
          DeviceBuffer lscratch(ladder_scratch_bytes(6, count, 256, 1024));
          ladder_reduce(6, x.get(), count, t, o, acc, oracle.get(), lscratch.get(), 256, 1024, c.stream);
          HIP_CHECK(hipStreamSynchronize(c.stream));
          HIP_CHECK(hipMemcpy(l, loc.get(), 8, hipMemcpyDeviceToHost));
          HIP_CHECK(hipMemcpy(orc, oracle.get(), 8, hipMemcpyDeviceToHost));
          std::vector<unsigned char> all(8 * static_cast<size_t>(c.env.world));
          c.boot->allgather(l, all.data(), 8);
          std::vector<unsigned char> packed(dtype_size(acc) * c.env.world);
          for (int r = 0; r < c.env.world; ++r) std::memcpy(&packed[r * dtype_size(acc)], &all[r * 8], dtype_size(acc));
          unsigned char host_fold[8] = {0};
          cpu_fold(packed.data(), c.env.world, acc, o, host_fold);
          if (dtype_is_float(acc) && o == Op::Sum) {
            const double gv = acc_as_double(g, acc), hv = acc_as_double(host_fold, acc);
            const double lv = acc_as_double(l, acc), ov = acc_as_double(orc, acc);
            vok = std::fabs(gv - hv) <= 1e-12 * (std::fabs(hv) + 1.0) && std::fabs(lv - ov) <= 1e-9 * (std::fabs(ov) + 1.0);
          } else {
            vok = std::memcmp(g, host_fold, dtype_size(acc)) == 0 && std::memcmp(l, orc, dtype_size(acc)) == 0;
          }
          std::vector<int> oks(c.env.world);
          int mine = vok ? 1 : 0;
          c.boot->allgather(&mine, oks.data(), sizeof mine);
          vok = std::all_of(oks.begin(), oks.end(), [](int v) { return v != 0; });
          ok = ok && vok;
          j.set("verified", vok).set("result", acc_as_double(g, acc));
        }
        emit(c, t, o, static_cast<double>(n) * dtype_size(t), dt, j);
      }
    }
  }
  return ok;
}

// ------------------------------------------------------------------------------ single process
// One process drives every visible GPU (simpleMultiGPU.cpp:185-310): per-GPU local
// reduce on its own stream, then either one grouped ncclAllReduce over an ncclCommInitAll set
// (--collective=allreduce) or a host fold of the per-GPU scalars (--collective=host, the
// simpleMultiGPU way). Scalar mode only.
bool run_single_process(Ctx& c, const std::vector<DType>& dtypes, const std::vector<Op>& ops,
                        const std::vector<uint64_t>& counts, int ndev_req) {
  const int avail = device_count();
  const int ndev = ndev_req > 0 ? std::min(ndev_req, avail) : avail;
  std::vector<int> devs(ndev);
  for (int i = 0; i < ndev; ++i) devs[i] = i;
  const bool host_fold = c.collective == "host";
  c.env.world = ndev;  // the NODES column / JSON "ranks" count GPUs in this mode
  std::unique_ptr<RcclGroup> group;
  if (!host_fold) group = std::make_unique<RcclGroup>(devs);
  struct Dev {
    hipStream_t s = nullptr;
    std::unique_ptr<Workspace> ws;
    DeviceBuffer x, out, oracle;
    uint64_t count = 0, offset = 0;
  };
  std::vector<Dev> d(ndev);
  for (int i = 0; i < ndev; ++i) {
    HIP_CHECK(hipSetDevice(devs[i]));
    HIP_CHECK(hipStreamCreateWithFlags(&d[i].s, hipStreamNonBlocking));
    d[i].ws = std::make_unique<Workspace>(devs[i]);
    d[i].out.allocate(8);
    d[i].oracle.allocate(8);
  }
  std::vector<hipStream_t> streams;
  for (auto& x : d) streams.push_back(x.s);
  auto sync_all = [&] {
    for (int i = 0; i < ndev; ++i) {
      HIP_CHECK(hipSetDevice(devs[i]));
      HIP_CHECK(hipStreamSynchronize(d[i].s));
    }
  };
  std::printf("%s\n", gnuplot_header().c_str());
  bool ok = true;
  for (size_t k = 0; k < dtypes.size(); ++k) {
    const DType t = dtypes[k];
    const uint64_t n = counts[k];
    for (int i = 0; i < ndev; ++i) {
      const uint64_t base = n / ndev, rem = n % ndev;
      d[i].count = base + (static_cast<uint64_t>(i) < rem ? 1 : 0);
      d[i].offset = i * base + std::min<uint64_t>(i, rem);
      HIP_CHECK(hipSetDevice(devs[i]));
      d[i].x.allocate(std::max<uint64_t>(d[i].count, 1) * dtype_size(t));
      FillSpec fs;
      fs.pattern = dtype_is_float(t) ? Pattern::Uniform : Pattern::FullRange;
      fs.seed = c.seed;
      fs.offset = d[i].offset;
      fill_device(d[i].x.get(), d[i].count, t, fs, d[i].s);
    }
    sync_all();
    for (Op o : ops) {
      const DType acc = default_acc(t, o);
      const size_t as = dtype_size(acc);
      unsigned char folded[8] = {0};
      auto step = [&] {
        for (int i = 0; i < ndev; ++i) {
          HIP_CHECK(hipSetDevice(devs[i]));
          reduce(d[i].x.get(), d[i].count, t, o, acc, d[i].out.get(), *d[i].ws, d[i].s, c.kcfg);
        }
        if (group) {
          std::vector<const void*> snd;
          std::vector<void*> rcv;
          for (auto& x : d) {
            snd.push_back(x.out.get());
            rcv.push_back(x.out.get());
          }
          group->allreduce(snd, rcv, 1, acc, o, streams);
        }
      };
      auto finish = [&] {  // host fold of the per-GPU scalars (simpleMultiGPU.cpp:263-275)
        sync_all();
        if (!host_fold) return;
        std::vector<unsigned char> parts(as * ndev);
        for (int i = 0; i < ndev; ++i) {
          HIP_CHECK(hipSetDevice(devs[i]));
          HIP_CHECK(hipMemcpy(&parts[i * as], d[i].out.get(), as, hipMemcpyDeviceToHost));
        }
        cpu_fold(parts.data(), ndev, acc, o, folded);
      };
      for (int w = 0; w < c.warmup; ++w) {
        step();
        finish();
      }
      for (int x_ = 0; x_ < c.retries; ++x_) {
        const double t0 = StopWatch::now_s();
        for (int it = 0; it < c.iters; ++it) {
          step();
          if (host_fold) finish();
        }
        finish();
        const double dt = (StopWatch::now_s() - t0) / c.iters;
        const double bytes = static_cast<double>(n) * dtype_size(t);
        Json j;
        j.set("single_process", true).set("devices", ndev).set("n_total", n).set("retry", x_);
        if (c.verify && x_ == 0) {
          // oracle: the two-launch path per GPU, folded on the host
          std::vector<unsigned char> parts(as * ndev);
          ReduceConfig two = c.kcfg;
          two.single_pass = false;
          for (int i = 0; i < ndev; ++i) {
            HIP_CHECK(hipSetDevice(devs[i]));
            reduce(d[i].x.get(), d[i].count, t, o, acc, d[i].oracle.get(), *d[i].ws, d[i].s, two);
            HIP_CHECK(hipStreamSynchronize(d[i].s));
            HIP_CHECK(hipMemcpy(&parts[i * as], d[i].oracle.get(), as, hipMemcpyDeviceToHost));
          }
          unsigned char expect[8] = {0}, got[8] = {0};
          cpu_fold(parts.data(), ndev, acc, o, expect);
          if (host_fold) {
            std::memcpy(got, folded, as);
          } else {
            HIP_CHECK(hipSetDevice(devs[0]));
            HIP_CHECK(hipMemcpy(got, d[0].out.get(), as, hipMemcpyDeviceToHost));
          }
          bool vok;
          if (dtype_is_float(acc) && o == Op::Sum) {
            const double gv = acc_as_double(got, acc), ev = acc_as_double(expect, acc);
            vok = std::fabs(gv - ev) <= 1e-9 * (std::fabs(ev) + 1.0);
          } else {
            vok = std::memcmp(got, expect, as) == 0;
          }
          for (int i = 0; i < ndev; ++i) vok = vok && d[i].ws->error() == 0;  // fan-in error words
          ok = ok && vok;
          j.set("verified", vok);
        }
        emit(c, t, o, bytes, dt, j);
      }
    }
  }
  for (int i = 0; i < ndev; ++i) {
    HIP_CHECK(hipSetDevice(devs[i]));
    HIP_CHECK(hipStreamDestroy(d[i].s));
  }
  return ok;
}

void usage() {
  std::printf(
      "reduce_xgmi — RCCL-over-xGMI reduction benchmark (one process per GPU)\n"
      "  --mode=vector|scalar        reduce.c element-wise reduce | global array -> one value\n"
      "  --collective=reduce|allreduce|direct|direct-reduce|fused (vector default: reduce, like MPI_Reduce;\n"
      "               scalar: allreduce; direct*: one-kernel peer reads over xGMI via IPC, no RCCL;\n"
      "               fused (scalar): the reduction kernel folds every rank's partial, no RCCL)\n"
      "  --dtypes=INT,DOUBLE  --ops=MAX,MIN,SUM  --retries=5  --warmup=1  --iters=10  --root=0\n"
      "  --ints=N --doubles=N --longs=N --floats=N   global element counts (reduce.c defaults)\n"
      "  --n=N                        global count for every dtype (scalar mode north star: 1e9)\n"
      "  --graph                      replay the timed iterations from a captured hipGraph (any collective)\n"
      "  --direct-grid=N              workgroups per direct collective (default: one per CU; same on all ranks)\n"
      "  --single-process[=N]         one process drives N (all) GPUs, scalar mode: grouped RCCL over\n"
      "                               ncclCommInitAll (--collective=allreduce) or host fold (--collective=host)\n"
      "  --mt19937                    vector mode: reduce.c's exact per-rank MT19937 data (host-generated)\n"
      "  --units=gib|gb               GNUPlot column unit (default gib = reduce.c's 2^30)\n"
      "  --json=PATH  --noverify  --seed=N  --block= --unroll= --wg-per-cu= --policy=auto|nt|default\n"
      "  --timeout=S                  RCCL wait deadline / direct kernels' device-side wait bound (s);\n"
      "                               bootstrap: MIREDUCE_BOOTSTRAP_TIMEOUT\n"
      "  --inject-fault=KIND[@RANK][:STEP]  exit|hang|corrupt|delay=<ms> at a timed collective (tests);\n"
      "                               nopeer: RANK's peer-access preflight says no (fused/direct decline)\n"
      "launch: torchrun --nproc-per-node=8 --master-addr 127.0.0.1 ... | mpirun -np 8 ...\n");
}

}  // namespace

int main(int argc, char** argv) {
  CmdArgs args;
  try {
    args = CmdArgs(argc, argv);
  } catch (const CliError& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return EXIT_FAILURE;
  }
  if (args.has("version")) {  // build provenance (version.hpp)
    std::printf("reduce_xgmi (mireduce) native source %s\n", mireduce::source_hash());
    return 0;
  }
  if (args.has("help")) {
    usage();
    return EXIT_SUCCESS;
  }
  Ctx c;
  c.env = launch_env_from_environment();
  std::vector<DType> dtypes = {DType::Int32, DType::Float64};
  std::vector<Op> ops = {Op::Max, Op::Min, Op::Sum};
  uint64_t ints = kNumInts, doubles = kNumDoubles, longs = 0, floats = 0, n_all = 0;
  try {
    for (const auto& u : args.unknown(kKnown))
      if (c.env.rank == 0) std::fprintf(stderr, "warning: unknown flag --%s ignored\n", u.c_str());
    c.mode = args.str_or("mode", "vector");
    if (c.mode != "vector" && c.mode != "scalar") throw CliError("--mode must be vector|scalar");
    c.collective = args.str_or("collective", c.mode == "vector" ? "reduce" : "allreduce");
    if (args.has("single-process")) {
      if (c.mode != "scalar") throw CliError("--single-process is scalar-mode only");
      if (c.collective != "allreduce" && c.collective != "host")
        throw CliError("--single-process takes --collective=allreduce|host");
      if (c.env.world != 1) throw CliError("--single-process runs without a multi-process launcher");
    } else if (c.collective != "reduce" && c.collective != "allreduce" && c.collective != "direct" &&
               c.collective != "direct-reduce" && c.collective != "fused") {
      throw CliError("--collective must be reduce|allreduce|direct|direct-reduce|fused");
    }
    if (c.mode == "scalar" && (c.collective == "direct" || c.collective == "direct-reduce"))
      throw CliError("direct collectives are vector-mode only");
    if (c.mode == "scalar" && c.collective != "allreduce" && c.collective != "fused" &&
        !(args.has("single-process") && c.collective == "host"))
      throw CliError("scalar mode uses --collective=allreduce|fused (or host with --single-process)");
    if (c.mode == "vector" && c.collective == "fused") throw CliError("--collective=fused is scalar-mode only");
    std::vector<std::string> list;
    if (args.get_list("dtypes", &list)) {
      dtypes.clear();
      for (auto& s : list) {
        DType t;
        if (!parse_dtype(s, &t)) throw CliError("unknown dtype " + s);
        if (dtype_is_half(t)) throw CliError("--dtypes=" + s + ": bf16/half are reduced by the single-GPU reduction app and the Python API; the cross-rank apps keep the reduce.c types (INT, LONG, FLOAT, DOUBLE)");
        dtypes.push_back(t);
      }
    }
    if (args.get_list("ops", &list)) {
      ops.clear();
      for (auto& s : list) {
        Op o;
        if (!parse_op(s, &o)) throw CliError("unknown op " + s);
        if (op_is_fused(o)) throw CliError("--ops=" + s + ": the element-wise cross-rank benchmark keeps reduce.c's MAX/MIN/SUM");
        ops.push_back(o);
      }
    }
    args.get_uint("ints", &ints);
    args.get_uint("doubles", &doubles);
    longs = ints;
    floats = doubles;
    args.get_uint("longs", &longs);
    args.get_uint("floats", &floats);
    if (args.get_uint("n", &n_all)) ints = doubles = longs = floats = n_all;
    c.retries = args.int_or<int>("retries", c.retries);
    c.warmup = args.int_or<int>("warmup", c.warmup);
    c.iters = std::max(1, args.int_or<int>("iters", c.iters));
    c.root = args.int_or<int>("root", c.root);
    c.json = args.str_or("json", "");
    c.graph = args.has("graph");
    c.direct_grid = args.int_or<int>("direct-grid", 0);
    if (c.direct_grid < 0 || c.direct_grid > kMaxDirectBlocks) throw CliError("--direct-grid must be 0..1024");
    set_tracing(args.has("trace"));
    c.mt = args.has("mt19937");
    c.verify = !args.has("noverify");
    c.seed = args.int_or<uint64_t>("seed", c.seed);
    c.units_gb = args.str_or("units", "gib") == "gb";
    double to = 0;
    if (args.get_double("timeout", &to)) c.timeout_s = c.direct_timeout_s = to;
    try {
      c.fault = FaultInjector::from_flag_or_env(args.str_or("inject-fault", ""));
    } catch (const std::invalid_argument& e) {
      throw CliError(e.what());
    }
    c.kcfg.block = args.int_or<int>("block", 0);
    c.kcfg.unroll = args.int_or<int>("unroll", 0);
    c.kcfg.wg_per_cu = args.int_or<int>("wg-per-cu", 0);
    {
      const std::string pol = args.str_or("policy", "auto");
      c.kcfg.policy = pol == "nt" ? 1 : (pol == "default" ? 0 : -1);
    }
    if (c.root < 0 || c.root >= c.env.world) throw CliError("--root out of range");
  } catch (const CliError& e) {
    if (c.env.rank == 0) std::fprintf(stderr, "error: %s\n", e.what());
    return EXIT_FAILURE;
  }

  const int ndev = device_count();
  if (ndev == 0) {
    std::fprintf(stderr, "[rank %d] no HIP device\n", c.env.rank);
    return EXIT_FAILURE;
  }
  if (args.has("single-process")) {
    bool sp_ok = false;
    try {
      c.boot = std::make_unique<TcpBootstrap>(c.env);  // world 1: no sockets
      std::vector<uint64_t> counts;
      for (DType t : dtypes) counts.push_back(global_count(t, ints, longs, floats, doubles));
      sp_ok = run_single_process(c, dtypes, ops, counts, args.int_or<int>("single-process", 0));
      if (c.verify) std::fprintf(stderr, "[reduce_xgmi] verification %s\n", sp_ok ? "PASSED" : "FAILED");
    } catch (const Error& e) {
      std::fprintf(stderr, "error: %s\n", e.what());
    }
    return sp_ok ? EXIT_SUCCESS : EXIT_FAILURE;
  }
  c.device = c.env.local_rank % ndev;
  HIP_CHECK(hipSetDevice(c.device));
  HIP_CHECK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
  bool ok = false;
  try {
    c.boot = std::make_unique<TcpBootstrap>(c.env);
    if (!needs_no_rccl(c)) {  // direct / fused need no RCCL (and may share one GPU between ranks)
      c.comm = std::make_unique<RcclComm>(*c.boot, c.device);
      install_comm_abort_hook(c.comm.get());
    } else {
      // The IPC-mapped paths store to / load from peers' memory from inside kernels: agree that
      // every pair of GPUs can map each other BEFORE any handle is opened, and decline on every
      // rank together otherwise (simpleP2P.cu:250-275 checks the same before enabling anything).
      const std::string why = peer_preflight(*c.boot, c.device, &c.fault);
      if (!why.empty())
        throw Error("--collective=" + c.collective + " needs peer access between every pair of GPUs: " + why);
    }
    if (c.env.rank == 0) {
      DeviceInfo di = device_info(c.device);
      std::fprintf(stderr, "[reduce_xgmi] %d ranks (%s), %s %s, RCCL %d, mode=%s collective=%s\n", c.env.world,
                   c.env.launcher.c_str(), di.name.c_str(), di.arch.c_str(), RcclComm::version(), c.mode.c_str(),
                   c.collective.c_str());
    }
    std::vector<uint64_t> counts;
    for (DType t : dtypes) counts.push_back(global_count(t, ints, longs, floats, doubles));
    ok = c.mode == "vector" ? run_vector(c, dtypes, ops, counts) : run_scalar(c, dtypes, ops, counts);
    if (c.verify && c.env.rank == 0) std::fprintf(stderr, "[reduce_xgmi] verification %s\n", ok ? "PASSED" : "FAILED");
    c.boot->barrier();
  } catch (const Error& e) {
    std::fprintf(stderr, "[rank %d] error: %s\n", c.env.rank, e.what());
    if (c.comm) c.comm->abort();
    ok = false;
  }
  install_comm_abort_hook(nullptr);
  c.direct.reset();
  c.comm.reset();
  c.boot.reset();
  HIP_CHECK(hipStreamDestroy(c.stream));
  return ok ? EXIT_SUCCESS : EXIT_FAILURE;
}
