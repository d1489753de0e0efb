// reduction — single-GPU SUM/MIN/MAX benchmark, CLI-compatible with the CUDA SDK sample the
// reference modified (cuda/C/src/reduction/reduction.cpp).
//
// Parity map:
//   main (reduction.cpp:84-204)        -> main: QA banner, log file, --method (required,
//                                         case-sensitive), --type (case-insensitive, default int),
//                                         --device, dispatch over (dtype x op), QA exit status
//   runTest{Sum,Min,Max} (:661-1034)   -> run_test: defaults n=2^24, threads=256, data generation,
//                                         planning, warm-up, 100 timed iterations, throughput line,
//                                         CPU verification
//   benchmarkReduce* (:297-568)        -> time_iterations: first-level kernel + device or host
//                                         (--cpufinal / --cputhresh) finalisation, per-iteration
//                                         hipEvent timing
//   getNumBlocksAndThreads (:272-291)  -> plan_reduce (persistent grid for 256 CUs)
//   shmoo (:576-657, disabled: B6)     -> run_shmoo (implemented)
//   sum/min/maxreduceCPU (:214-249)    -> cpu_reduce (compensated / exact)
// Kernels: --kernel=7 (default) mireduce single-pass streaming kernel; 8 = the same first level +
// a separate finalize launch (the reference's two-launch structure); 0..6 = the Harris
// whitepaper ladder re-expressed for wave64 (csrc/kernels/ladder.hip), 6 being the reference's
// "kernel 6" algorithm (multiple elements per thread, LDS tree, unrolled last wave).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "mireduce/version.hpp"
#include "mireduce/arg_reduce.hpp"
#include "mireduce/check.hpp"
#include "mireduce/cli.hpp"
#include "mireduce/cpu_reference.hpp"
#include "mireduce/device.hpp"
#include "mireduce/ladder.hpp"
#include "mireduce/log.hpp"
#include "mireduce/qa.hpp"
#include "mireduce/reduce.hpp"
#include "mireduce/report.hpp"
#include "mireduce/timer.hpp"
#include "mireduce/trace.hpp"

using namespace mireduce;

namespace {

struct Options {
  DType dtype = DType::Int32;
  std::string type_name = "int";
  Op op = Op::Sum;
  DType acc = DType::Int32;
  bool acc_given = false;
  uint64_t n = 1ull << 24;  // reduction.cpp:665
  int threads = 0;          // 0 = tuned plan (kernels 7/8) / 256 (ladder); reference 256 (reduction.cpp:666)
  int kernel = 7;
  int max_blocks = 0;       // 0 = persistent grid (reference default 64, reduction.cpp:668)
  bool cpufinal = false;
  int cputhresh = 1;        // reduction.cpp:670
  int iterations = 100;     // reduction.cpp:731
  bool batch_timing = false;  // one event pair around all iterations (throughput) vs per iteration
  bool cold = false;          // flush L2 + Infinity Cache before every timed iteration
  int unroll = 0;
  int window = -1;  // streaming body's load window: -1 tuned, 0 hipcc's schedule, 2 | 4
  int64_t segment_bytes = 0;  // segmented launches: 0 auto (8 GiB above 16 GiB), < 0 one launch, > 0 size
  int wg_per_cu = 0;
  int policy = -1;
  Pattern pattern = Pattern::SmallInt;  // rand() & 0xFF (reduction.cpp:698-705)
  uint64_t seed = 1;
  bool device_fill = false;
  bool verify = true;
  std::string json;
  int device = 0;
  bool arg = false;  // --arg: the position of the MIN/MAX too (arg_reduce.hpp)
};

const std::set<std::string> kKnown = {
    "method", "type", "n", "threads", "kernel", "maxblocks", "cpufinal", "cputhresh", "shmoo",
    "device", "qatest", "noprompt", "prompt", "help", "version", "quiet", "iterations", "acc", "unroll", "window",
    "segment-bytes",
    "wg-per-cu", "policy", "pattern", "seed", "fill", "noverify", "json", "log", "master-log",
    "countdown", "shmoo-max", "trace", "timing", "cold", "arg"};

void usage() {
  std::printf(
      "reduction --method=SUM|MIN|MAX [options]\n"
      "  --type=int|int64|float|double  element type (case-insensitive, default int)\n"
      "  --n=N            elements (default 16777216; k/M/G suffixes and 1e9 accepted)\n"
      "  --threads=N             workgroup size, a power of two (default: tuned plan; 256 = reference);\n"
      "                          kernels 0..6 take 1..1024, kernels 7/8 256|512|1024 (smaller: 256)\n"
      "  --kernel=0..8    7 = single-pass (default), 8 = two-launch, 0..6 = Harris ladder\n"
      "  --maxblocks=N    cap the grid (default: persistent grid, 8 WG/CU)\n"
      "  --cpufinal       fold the per-workgroup partials on the host\n"
      "  --cputhresh=N    fold on the host when <= N partials remain\n"
      "  --shmoo          sweep n = 1..32M (powers of two, --shmoo-max=N) over kernels, print CSV\n"
      "  --timing=per-iter|batch  event pair per iteration (reference, default) or around all (shmoo default)\n"
      "  --cold           overwrite a 1 GiB scratch buffer before every timed iteration (evicts the\n"
      "                   256 MB Infinity Cache and the L2s): HBM numbers for small arrays; per-iter timing\n"
      "  --iterations=100 --acc=TYPE --unroll=2|4|8 --wg-per-cu=N --policy=auto|nt|default\n"
      "  --window=0|2|4   streaming body: hipcc's load schedule (0) or an explicit window (default: tuned)\n"
      "  --segment-bytes=N  arrays above 16 GiB run as 8 GiB launches (0, default); -1 one launch; N bytes\n"
      "  --pattern=smallint|uniform|fullrange|iotamod --seed=N --fill=host|device --noverify\n"
      "  --device=N --json=PATH --log=FILE|none --master-log=FILE|none (default SdkMasterLog.csv) --qatest\n"
      "  --prompt --countdown\n"
      "  --trace          roctx ranges per iteration (rocprofv3 --marker-trace)\n"
      "  --arg            with MIN/MAX: also the first index of the extreme (arg-reduction kernel)\n");
}

size_t pick_threads_for_fill() {
  unsigned hc = std::thread::hardware_concurrency();
  return hc ? std::min<unsigned>(hc, 16) : 1;
}

// Host fill in parallel (identical values to the serial / device fill: element i = f(seed, i)).
void parallel_fill_host(void* p, uint64_t n, DType t, const FillSpec& s) {
  const size_t th = n > (1u << 22) ? pick_threads_for_fill() : 1;
  const uint64_t chunk = (n + th - 1) / th;
  std::vector<std::thread> pool;
  for (size_t k = 0; k < th; ++k) {
    const uint64_t b = std::min<uint64_t>(n, k * chunk), e = std::min<uint64_t>(n, b + chunk);
    if (b >= e) continue;
    FillSpec sk = s;
    sk.offset = s.offset + b;
    void* pk = static_cast<char*>(p) + b * dtype_size(t);
    pool.emplace_back([=] { fill_host(pk, e - b, t, sk); });
  }
  for (auto& x : pool) x.join();
}

constexpr size_t kFlushBytes = size_t(1) << 30;  // > 256 MB MALL + 8 x 4 MB L2, written untimed

struct Buffers {
  DeviceBuffer in, out, partials, ladder;  // ladder: ping-pong scratch of kernels 0..6
  DeviceBuffer flush;                      // --cold: cache-eviction scratch
  std::vector<unsigned char> host;  // input copy (for CPU verification)
  void* pinned = nullptr;           // --cpufinal partials landing zone
  size_t pinned_bytes = 0;
  ~Buffers() {
    if (pinned) (void)hipHostFree(pinned);
  }
  // Grow the landing zone to hold `bytes` (stream-synchronised by the caller first). The ladder's
  // first pass leaves as many partials as it launches blocks, and kernels 0..5 have no --maxblocks
  // cap: e.g. --kernel=0 --threads=64 --cpufinal leaves n/64 partials.
  void ensure_pinned(size_t bytes) {
    if (bytes <= pinned_bytes) return;
    if (pinned) HIP_CHECK(hipHostFree(pinned));
    pinned = nullptr;
    HIP_CHECK(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
    pinned_bytes = bytes;
  }
};

// One full reduction of d_in (timed region body). Returns nothing; result lands in out
// (device) or in *host_result (host finalisation).
struct Runner {
  const Options& o;
  Workspace& ws;
  Buffers& b;
  hipStream_t s;
  LaunchPlan plan{};
  bool host_fold = false;

  ReduceConfig cfg() const {
    ReduceConfig c;
    c.block = o.threads;
    c.unroll = o.unroll;
    c.window = o.window;
    c.segment_bytes = o.segment_bytes;
    c.wg_per_cu = o.wg_per_cu;
    c.max_blocks = o.max_blocks;
    c.policy = o.policy;
    c.single_pass = (o.kernel == 7);
    return c;
  }

  int passes = 0;             // kernel launches of the last run_once
  uint64_t host_folded = 0;   // partials folded on the host by the last run_once (0: none)
  const void* result_dev = nullptr;  // where the device result of the last run_once is

  // The reference's host fold of what the relaunch loop left (reduction.cpp:332,362-370).
  bool host_fold_partials(const void* partials, uint64_t left, unsigned char* host_out) {
    const size_t bytes = left * dtype_size(o.acc);
    if (bytes > b.pinned_bytes) {  // (only the warm-up call can grow it: same n, same plan after)
      HIP_CHECK(hipStreamSynchronize(s));
      b.ensure_pinned(bytes);
    }
    HIP_CHECK(hipMemcpyAsync(b.pinned, partials, bytes, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    cpu_fold(b.pinned, left, o.acc, o.op, host_out);
    host_folded = left;
    return true;
  }

  // One timed reduction, as benchmarkReduce* (reduction.cpp:319-374): first pass, then relaunches
  // on the partials while more than --cputhresh remain (none with --cpufinal), then a host fold of
  // what is left. Returns true if the result was produced on the host into host_out.
  bool run_once(uint64_t n, unsigned char* host_out) {
    TraceRange tr("reduction.iteration");
    const void* in = b.in.get();
    host_folded = 0;
    result_dev = b.out.get();
    if (o.kernel <= 6) {
      const int mb = o.max_blocks > 0 ? o.max_blocks : 64;  // reference default (reduction.cpp:668)
      const int th = o.threads ? o.threads : 256;            // reference default (reduction.cpp:666)
      const size_t need = ladder_scratch_bytes(o.kernel, n, th, mb);
      if (b.ladder.bytes() < need) {  // grows during the warm-up call only
        HIP_CHECK(hipStreamSynchronize(s));
        b.ladder.allocate(need);
      }
      const LadderPasses lp = ladder_reduce_passes(o.kernel, in, n, o.dtype, o.op, o.acc, b.out.get(), b.ladder.get(),
                                                   th, mb, o.cputhresh, o.cpufinal, s);
      plan.block = th;
      plan.grid = lp.first_grid;
      passes = lp.passes;
      return lp.left > 1 ? host_fold_partials(lp.partials, lp.left, host_out) : false;
    }
    const bool want_host = o.cpufinal || o.cputhresh > 1;
    if (!want_host) {
      plan = reduce(in, n, o.dtype, o.op, o.acc, b.out.get(), ws, s, cfg());
      passes = plan.single_pass ? 1 : 2;
      return false;
    }
    const ReducePasses rp = reduce_passes(in, n, o.dtype, o.op, o.acc, b.partials.get(), ws.max_grid(), ws.num_cus(),
                                          o.cputhresh, o.cpufinal, s, cfg());
    plan = rp.plan;
    passes = rp.passes;
    if (rp.left > 1 || o.cpufinal) return host_fold_partials(rp.partials, rp.left, host_out);
    result_dev = rp.partials;  // one partial left: the result, in place like d_odata[0]
    return false;
  }
};

struct Timing {
  std::vector<double> ms;  // per iteration, hipEvent (or host clock for host-folded runs)
  double avg_ms = 0;
  bool host_result = false;
  unsigned char result[8] = {0};
};

Timing time_iterations(Runner& r, uint64_t n, int iters) {
  Timing t;
  EventTimer ev;
  HIP_CHECK(hipDeviceSynchronize());
  const bool host_path = r.o.cpufinal || r.o.cputhresh > 1;
  if (r.o.cold && r.b.flush.bytes() < kFlushBytes) r.b.flush.allocate(kFlushBytes);
  if (r.o.batch_timing && !host_path && !r.o.cold) {  // back-to-back launches, one event pair: throughput
    ev.start(r.s);
    for (int i = 0; i < iters; ++i) r.run_once(n, t.result);
    ev.stop(r.s);
    const double ms = ev.elapsed_ms();
    t.ms.assign(iters, ms / iters);
    t.avg_ms = ms / iters;
    HIP_CHECK(hipMemcpy(t.result, r.result_dev, dtype_size(r.o.acc), hipMemcpyDeviceToHost));
    return t;
  }
  for (int i = 0; i < iters; ++i) {
    if (r.o.cold) {  // evict the array from L2 / MALL outside the event pair
      HIP_CHECK(hipMemsetAsync(r.b.flush.get(), i & 0xFF, kFlushBytes, r.s));
      HIP_CHECK(hipStreamSynchronize(r.s));
    }
    const double h0 = StopWatch::now_s();
    ev.start(r.s);
    const bool host = r.run_once(n, t.result);
    ev.stop(r.s);
    if (host) {
      t.ms.push_back((StopWatch::now_s() - h0) * 1e3);
      t.host_result = true;
    } else {
      t.ms.push_back(ev.elapsed_ms());
    }
  }
  double sum = 0;
  for (double m : t.ms) sum += m;
  t.avg_ms = iters ? sum / iters : 0;
  if (!t.host_result) HIP_CHECK(hipMemcpy(t.result, r.result_dev, dtype_size(r.o.acc), hipMemcpyDeviceToHost));
  return t;
}

std::string fmt_result(const unsigned char* p, DType acc) {
  char buf[64];
  if (dtype_is_float(acc)) std::snprintf(buf, sizeof buf, "%f", acc_as_double(p, acc));
  else std::snprintf(buf, sizeof buf, "%" PRId64, acc_as_int64(p, acc));
  return buf;
}

// --arg: first index of the minimum / maximum and its value (csrc/kernels/arg_reduce.hip),
// verified against the host reference cpu_arg_reduce_rows (same first-occurrence rule).
bool run_arg_test(const Options& o, Workspace& ws, hipStream_t s) {
  Logger& L = Logger::instance();
  L.log(kLogBoth, "METHOD: ARG%s\n", op_name(o.op));
  L.log(kLogBoth, "%" PRIu64 " elements\n", o.n);
  const size_t es = dtype_size(o.dtype);
  DeviceBuffer in(std::max<uint64_t>(o.n, 1) * es), val(8), idx(8);
  const size_t need = arg_reduce_scratch_bytes(1, o.n, o.dtype, ws.num_cus());
  DeviceBuffer scratch(std::max<size_t>(need, 256));
  HIP_CHECK(hipMemsetAsync(scratch.get(), 0, scratch.bytes(), s));
  FillSpec fs;
  fs.pattern = o.pattern;
  fs.seed = o.seed;
  std::vector<unsigned char> host;
  const bool host_copy = !o.device_fill || (o.verify && o.n <= (1ull << 30));
  if (host_copy) {
    host.resize(o.n * es);
    parallel_fill_host(host.data(), o.n, o.dtype, fs);
  }
  if (o.device_fill) fill_device(in.get(), o.n, o.dtype, fs, s);
  else HIP_CHECK(hipMemcpy(in.get(), host.data(), o.n * es, hipMemcpyHostToDevice));
  HIP_CHECK(hipDeviceSynchronize());
  ArgTune tune;
  tune.wg_per_cu = o.wg_per_cu;
  tune.unroll = o.unroll;
  auto once = [&] {
    return arg_reduce_rows(in.get(), 1, o.n, o.dtype, o.op, val.get(), idx.as<int64_t>(), scratch.get(), ws.num_cus(),
                           s, tune);
  };
  const ArgPlan plan = once();  // warm-up
  HIP_CHECK(hipStreamSynchronize(s));
  L.log(kLogBoth, "%d blocks\n\n", plan.grid);
  EventTimer ev;
  std::vector<double> ms;
  if (o.batch_timing) {
    ev.start(s);
    for (int i = 0; i < o.iterations; ++i) once();
    ev.stop(s);
    ms.assign(o.iterations, ev.elapsed_ms() / o.iterations);
  } else {
    for (int i = 0; i < o.iterations; ++i) {
      ev.start(s);
      once();
      ev.stop(s);
      ms.push_back(ev.elapsed_ms());
    }
  }
  double sum = 0;
  for (double m : ms) sum += m;
  const double secs = sum / ms.size() * 1e-3, bytes = static_cast<double>(o.n) * es;
  L.log(kLogBoth | kLogMaster, "%s\n", throughput_line(secs > 0 ? 1.0e-9 * bytes / secs : 0.0, secs, o.n, 1,
                                                       static_cast<unsigned>(plan.block)).c_str());
  int64_t gi = 0;
  unsigned char gv[8] = {0};
  HIP_CHECK(hipMemcpy(&gi, idx.get(), 8, hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(gv, val.get(), es, hipMemcpyDeviceToHost));
  L.log(kLogBoth, "\nGPU result = index %" PRId64 "\n", gi);
  bool ok = true;
  if (o.verify && host_copy) {
    int64_t ci = 0;
    unsigned char cv[8] = {0};
    cpu_arg_reduce_rows(host.data(), 1, o.n, o.dtype, o.op, cv, &ci);
    L.log(kLogBoth, "CPU result = index %" PRId64 "\n\n", ci);
    ok = gi == ci && std::memcmp(gv, cv, es) == 0;
  }
  if (!o.json.empty()) {
    Stats st = compute_stats(ms);
    DeviceInfo di = device_info(o.device);
    Json j;
    j.set("app", "reduction").set("method", std::string("ARG") + op_name(o.op)).set("type", dtype_cli_name(o.dtype))
        .set("n", o.n).set("bytes", static_cast<uint64_t>(bytes)).set("grid", plan.grid).set("splits", plan.splits)
        .set("unroll", plan.unroll).set("wg_per_cu", plan.wg_per_cu).set("iterations", o.iterations)
        .set("avg_ms", secs * 1e3).set("median_ms", st.median).set("min_ms", st.min).set("max_ms", st.max)
        .set("std_ms", st.stddev).set("gb_per_s", secs > 0 ? bytes / secs / kGB : 0.0)
        .set("gib_per_s", secs > 0 ? bytes / secs / kGiB : 0.0).set("bytes_per_GB", kGB).set("index", gi)
        .set("verified", o.verify && host_copy).set("passed", ok).set("device", di.name).set("arch", di.arch)
        .set("cus", di.cus).set("iteration_ms", ms);
    j.write_file(o.json);
  }
  return ok;
}

bool run_test(Options& o, Workspace& ws, hipStream_t s) {
  Logger& L = Logger::instance();
  L.log(kLogBoth, "METHOD: %s\n", op_name(o.op));
  L.log(kLogBoth, "%" PRIu64 " elements\n", o.n);
  if (o.threads) L.log(kLogBoth, "%d threads (max)\n", o.threads);
  else L.log(kLogBoth, "tuned threads (max)\n");

  Buffers b;
  const size_t es = dtype_size(o.dtype);
  b.in.allocate(std::max<uint64_t>(o.n, 1) * es);
  b.out.allocate(8);
  b.partials.allocate(2 * static_cast<size_t>(std::max(ws.max_grid(), 1 << 16)) * 8);  // ping-pong passes
  b.ensure_pinned(static_cast<size_t>(std::max(ws.max_grid(), 1 << 16)) * 8);

  FillSpec fs;
  fs.pattern = o.pattern;
  fs.seed = o.seed;
  const bool host_copy = !o.device_fill || (o.verify && o.n <= (1ull << 30));
  if (host_copy) {
    b.host.resize(o.n * es);
    parallel_fill_host(b.host.data(), o.n, o.dtype, fs);
  }
  if (o.device_fill) fill_device(b.in.get(), o.n, o.dtype, fs, s);
  else if (o.n) HIP_CHECK(hipMemcpy(b.in.get(), b.host.data(), o.n * es, hipMemcpyHostToDevice));
  HIP_CHECK(hipDeviceSynchronize());

  Runner r{o, ws, b, s};
  unsigned char scratch[8];
  r.run_once(o.n, scratch);  // warm-up (reduction.cpp:729)
  HIP_CHECK(hipDeviceSynchronize());
  L.log(kLogBoth, "%d blocks\n\n", r.plan.grid);

  Timing t = time_iterations(r, o.n, o.iterations);
  // device-side error word of the polled fan-in (a finisher reached its wait bound: results poisoned)
  const unsigned fan_err = ws.error();
  if (fan_err) {
    L.log(kLogBoth, "FAN-IN ERROR: a launch reached the polled fan-in's wait bound (result poisoned)\n");
    ws.reset(s);
    HIP_CHECK(hipStreamSynchronize(s));
  }
  const double secs = t.avg_ms * 1e-3;
  const double bytes = static_cast<double>(o.n) * es;
  L.log(kLogBoth | kLogMaster, "%s\n", throughput_line(secs > 0 ? 1.0e-9 * bytes / secs : 0.0, secs, o.n, 1,
                                                       static_cast<unsigned>(r.plan.block)).c_str());

  bool ok = fan_err == 0;
  unsigned char cpu[8] = {0};
  double tol = 0;
  bool checked = false;
  std::string oracle = "host reference (Kahan / exact)";
  if (o.verify && host_copy) {
    cpu_reduce(b.host.data(), o.n, o.dtype, o.op, o.acc, cpu);
    checked = true;
    if (dtype_is_float(o.acc)) {
      const double g = acc_as_double(t.result, o.acc), c = acc_as_double(cpu, o.acc);
      // SUMSQ is a sum too; its terms are non-negative, so its Σ|.| is the result itself
      const bool summed = o.op == Op::Sum || o.op == Op::SumSq;
      const double abs_sum = o.op == Op::SumSq ? std::fabs(c) : (summed ? cpu_abs_sum(b.host.data(), o.n, o.dtype) : 0.0);
      tol = summed ? sum_tolerance(o.dtype, o.acc, o.n, abs_sum) : 0.0;
      ok = ok && (summed ? std::fabs(g - c) <= tol : g == c);
    } else {
      ok = ok && acc_as_int64(t.result, o.acc) == acc_as_int64(cpu, o.acc);
    }
  } else if (o.verify) {
    // Huge device-filled arrays (no host copy), independent oracles:
    //  * --pattern=iotamod: the closed-form result (no device code involved);
    //  * reference element types: the ladder's kernel 6 (a different kernel, grid and fold);
    //  * bf16/fp16 or fused ops: the other streaming path (two-launch vs single-pass).
    checked = true;
    const bool summed_f = dtype_is_float(o.acc) && (o.op == Op::Sum || o.op == Op::SumSq);
    if (o.pattern == Pattern::IotaMod && analytic_iotamod(o.n, 0, o.dtype, o.op, o.acc, cpu)) {
      oracle = "closed-form iotamod";
      if (summed_f && o.acc == DType::Float32) {
        const double g = acc_as_double(t.result, o.acc), c = acc_as_double(cpu, o.acc);
        tol = sum_tolerance(o.dtype, o.acc, o.n, std::fabs(c));
        ok = ok && std::fabs(g - c) <= tol;
      } else {
        ok = ok && std::memcmp(t.result, cpu, dtype_size(o.acc)) == 0;  // exact: integer-valued terms
      }
    } else {
      Options o2 = o;
      const bool ladder_ok = !dtype_is_half(o.dtype) && !op_is_fused(o.op);
      o2.kernel = ladder_ok ? 6 : (o.kernel == 8 ? 7 : 8);
      o2.threads = ladder_ok ? 256 : o.threads;
      o2.max_blocks = ladder_ok ? 1024 : o.max_blocks;
      o2.cpufinal = false;
      o2.cputhresh = 1;
      oracle = ladder_ok ? "ladder kernel 6" : (o2.kernel == 7 ? "single-pass kernel 7" : "two-launch kernel 8");
      Runner r2{o2, ws, b, s};
      r2.run_once(o.n, scratch);
      HIP_CHECK(hipStreamSynchronize(s));
      HIP_CHECK(hipMemcpy(cpu, r2.result_dev, dtype_size(o.acc), hipMemcpyDeviceToHost));
      if (summed_f) {
        const double g = acc_as_double(t.result, o.acc), c = acc_as_double(cpu, o.acc);
        tol = 1e-9 * std::fabs(c) + 1e-12;
        ok = ok && std::fabs(g - c) <= tol;
      } else {
        ok = ok && std::memcmp(t.result, cpu, dtype_size(o.acc)) == 0;
      }
    }
  }
  L.log(kLogBoth, "\nGPU result = %s\n", fmt_result(t.result, o.acc).c_str());
  if (checked) L.log(kLogBoth, "CPU result = %s\n\n", fmt_result(cpu, o.acc).c_str());
  if (r.passes > 1 || r.host_folded)
    L.log(kLogBoth, "%d kernel pass(es), %" PRIu64 " partial(s) folded on the host\n", r.passes, r.host_folded);

  if (!o.json.empty()) {
    Stats st = compute_stats(t.ms);
    DeviceInfo di = device_info(o.device);
    Json j;
    j.set("app", "reduction").set("method", op_name(o.op)).set("type", dtype_cli_name(o.dtype))
        .set("acc", dtype_cli_name(o.acc)).set("n", o.n).set("bytes", static_cast<uint64_t>(bytes))
        .set("kernel", o.kernel).set("block", r.plan.block).set("grid", r.plan.grid).set("unroll", r.plan.unroll).set("window", r.plan.window).set("segments", static_cast<int64_t>(r.plan.segments))
        .set("nontemporal", r.plan.nontemporal).set("cpufinal", o.cpufinal)
        .set("iterations", o.iterations).set("cold", o.cold).set("timing", o.batch_timing && !o.cold ? "batch" : "per-iter").set("avg_ms", t.avg_ms).set("median_ms", st.median).set("min_ms", st.min)
        .set("max_ms", st.max).set("std_ms", st.stddev).set("gb_per_s", secs > 0 ? bytes / secs / kGB : 0.0)
        .set("gib_per_s", secs > 0 ? bytes / secs / kGiB : 0.0).set("bytes_per_GB", kGB)
        .set("gpu_result", acc_as_double(t.result, o.acc)).set("verified", checked ? ok : fan_err == 0)
        .set("tolerance", tol).set("device", di.name).set("arch", di.arch).set("cus", di.cus)
        .set("passes", r.passes).set("host_folded", r.host_folded).set("cputhresh", o.cputhresh)
        .set("oracle", checked ? oracle : std::string("none")).set("fanin_error", static_cast<int64_t>(fan_err))
        .set("iteration_ms", t.ms);
    j.write_file(o.json);
  }
  return ok;
}

void run_shmoo(Options o, Workspace& ws, hipStream_t s, uint64_t max_n) {
  // Reference: shmoo<T>(1, 33554432, ...) over kernels 0..6 (reduction.cpp:576-657, disabled);
  // the OpenCL twin prints a kernel x size table (oclReduction.cpp:392-455).
  std::printf("n,bytes,kernel,avg_ms,GB/s\n");
  const size_t es = dtype_size(o.dtype);
  Buffers b;
  b.in.allocate(max_n * es);
  b.out.allocate(8);
  b.partials.allocate(static_cast<size_t>(1 << 16) * 8);
  FillSpec fs;
  fs.pattern = o.pattern;
  fs.seed = o.seed;
  fill_device(b.in.get(), max_n, o.dtype, fs, s);
  HIP_CHECK(hipDeviceSynchronize());
  const int kernels[] = {0, 1, 2, 3, 4, 5, 6, 8, 7};
  for (uint64_t n = 1; n <= max_n; n *= 2) {
    for (int k : kernels) {
      if (k <= 6 && (dtype_is_half(o.dtype) || op_is_fused(o.op))) continue;  // ladder: reference types/ops only
      o.kernel = k;
      o.cpufinal = false;
      o.cputhresh = 1;
      Runner r{o, ws, b, s};
      unsigned char scratch[8];
      r.run_once(n, scratch);
      Timing t = time_iterations(r, n, o.iterations);
      const double bytes = static_cast<double>(n) * es;
      std::printf("%" PRIu64 ",%.0f,%d,%.6f,%.4f\n", n, bytes, k, t.avg_ms,
                  t.avg_ms > 0 ? 1e-9 * bytes / (t.avg_ms * 1e-3) : 0.0);
      std::fflush(stdout);
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  const char* const* cargv = argv;
  qa_start(argc, cargv);
  CmdArgs args;
  try {
    args = CmdArgs(argc, cargv);
  } catch (const CliError& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return EXIT_FAILURE;
  }
  if (args.has("version")) {  // build provenance (version.hpp)
    std::printf("reduction (mireduce) native source %s\n", mireduce::source_hash());
    return 0;
  }
  if (args.has("help")) {
    usage();
    qa_finish_exit(argc, cargv, QaStatus::Passed);
  }
  Logger& L = Logger::instance();
  const std::string log = args.str_or("log", "reduction.txt");
  if (log != "none") L.set_log_file(log);  // shrSetLogFileName("reduction.txt") (reduction.cpp:88)
  // shrLogEx(LOGBOTH | MASTER) appends to SdkMasterLog.csv by default (shrUtils.h:86)
  const std::string master = args.str_or("master-log", "SdkMasterLog.csv");
  if (master != "none") L.set_master_file(master);
  L.set_quiet(args.has("quiet"));
  set_tracing(args.has("trace"));
  for (const auto& u : args.unknown(kKnown)) std::fprintf(stderr, "warning: unknown flag --%s ignored\n", u.c_str());

  Options o;
  std::string method;
  if (!args.has("method")) {  // reduction.cpp:124-128
    std::fprintf(stderr, "MISSING --method FLAG.\nYou must provide --method={ SUM | MIN | MAX }.\n");
    std::exit(1);
  }
  args.get_str("method", &method);
  if (!parse_op_strict(method, &o.op)) {  // case-sensitive strcmp (reduction.cpp:165-199)
    std::fprintf(stderr, "No --method specified!\n");
    std::exit(1);
  }
  try {
    std::string ty;
    if (args.get_str("type", &ty)) {
      if (!parse_dtype(ty, &o.dtype)) {
        std::fprintf(stderr, "warning: unknown --type=%s, using int (reduction.cpp:106-108)\n", ty.c_str());
        o.dtype = DType::Int32;
      }
      o.type_name = ty;
    }
    o.acc = default_acc(o.dtype, o.op);
    // Parity mode: the reference accumulates int SUM in int (reduction_kernel.cu). Default here
    // widens (B7); --acc=int restores the 32-bit wrap.
    std::string acc;
    if (args.get_str("acc", &acc)) {
      if (!parse_dtype(acc, &o.acc) || !acc_supported(o.dtype, o.op, o.acc)) throw CliError("unsupported --acc=" + acc);
      o.acc_given = true;
    }
    args.get_uint("n", &o.n);
    o.threads = args.int_or<int>("threads", o.threads);
    o.kernel = args.int_or<int>("kernel", o.kernel);
    o.max_blocks = args.int_or<int>("maxblocks", o.max_blocks);
    o.cpufinal = args.has("cpufinal");
    o.cputhresh = args.int_or<int>("cputhresh", o.cputhresh);
    o.iterations = args.int_or<int>("iterations", o.iterations);
    o.unroll = args.int_or<int>("unroll", o.unroll);
    o.window = args.int_or<int>("window", o.window);
    o.segment_bytes = args.int_or<int64_t>("segment-bytes", o.segment_bytes);
    o.wg_per_cu = args.int_or<int>("wg-per-cu", o.wg_per_cu);
    {
      const std::string pol = args.str_or("policy", "auto");
      o.policy = pol == "nt" ? 1 : (pol == "default" ? 0 : -1);
    }
    std::string pat = args.str_or("pattern", "smallint");
    if (pat == "smallint") o.pattern = Pattern::SmallInt;
    else if (pat == "uniform") o.pattern = Pattern::Uniform;
    else if (pat == "fullrange") o.pattern = Pattern::FullRange;
    else if (pat == "iotamod") o.pattern = Pattern::IotaMod;
    else throw CliError("unknown --pattern=" + pat);
    o.seed = args.int_or<uint64_t>("seed", o.seed);
    o.device_fill = args.str_or("fill", "host") == "device";
    o.verify = !args.has("noverify");
    o.json = args.str_or("json", "");
    o.device = args.int_or<int>("device", 0);
    {
      const std::string tm = args.str_or("timing", args.has("shmoo") ? "batch" : "per-iter");
      if (tm != "batch" && tm != "per-iter") throw CliError("--timing must be per-iter|batch");
      o.batch_timing = tm == "batch";
      o.cold = args.has("cold");
    }
    if (o.kernel < 0 || o.kernel > 8) throw CliError("--kernel must be 0..8");
    if (op_is_fused(o.op) && !dtype_is_float(o.dtype))
      throw CliError(std::string("--method=") + op_name(o.op) + " needs --type=float|double|bf16|half");
    if (o.kernel <= 6 && op_is_fused(o.op))
      throw CliError("--kernel 0..6 (the reference's ladder) implement SUM/MIN/MAX; SUMSQ/AMAX use kernels 7/8");
    if (o.kernel <= 6 && dtype_is_half(o.dtype))
      throw CliError("--kernel 0..6 (the reference's ladder) covers int/int64/float/double; bf16/half use kernels 7/8");
    // The reference accepts any power of two up to 512 (reduction.cpp:272-291, instantiations
    // reduction_kernel.cu:292-343). The ladder (0..6) runs every one of them (and 1024); the
    // streaming kernels (7/8) use whole-CU workgroups of 256/512/1024 — a smaller request is
    // rounded up to 256 with a note, so parity runs of the reference's flag values still run.
    if (o.threads != 0 && (o.threads < 1 || o.threads > 1024 || (o.threads & (o.threads - 1))))
      throw CliError("--threads must be a power of two in [1, 1024]");
    if (o.kernel >= 7 && o.threads != 0 && o.threads < 256) {
      std::fprintf(stderr, "note: --threads=%d: kernels 7/8 use 256/512/1024-thread workgroups; using 256\n",
                   o.threads);
      o.threads = 256;
    }
    if (o.kernel <= 6 && o.threads == 0) o.threads = 256;
    if (o.iterations < 1) throw CliError("--iterations must be >= 1");
    o.arg = args.has("arg");
    if (o.arg && o.op != Op::Min && o.op != Op::Max) throw CliError("--arg needs --method=MIN or MAX");
    if (o.arg && (o.kernel != 7 || o.cpufinal || o.cputhresh > 1 || args.has("shmoo")))
      throw CliError("--arg runs the arg-reduction kernel only (no --kernel/--cpufinal/--cputhresh/--shmoo)");
  } catch (const CliError& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return EXIT_FAILURE;
  }

  const int ndev = device_count();
  if (ndev == 0 || o.device >= ndev) {
    L.log(kLogBoth, "Error: no usable HIP device (found %d).\n\n", ndev);
    qa_finish_exit(argc, cargv, QaStatus::Waived);
  }
  DeviceInfo di = device_info(o.device);
  if (di.arch.rfind("gfx950", 0) != 0) {  // kernels are built for gfx950 only (cf. reduction.cpp:148-155)
    L.log(kLogBoth, "Error: device %d (%s, %s) is not gfx950 (MI355X).\n\n", o.device, di.name.c_str(), di.arch.c_str());
    qa_finish_exit(argc, cargv, QaStatus::Waived);
  }
  HIP_CHECK(hipSetDevice(o.device));
  L.log(kLogBoth, "Using Device %d: %s\n\n", o.device, di.name.c_str());
  L.log(kLogBoth, "Reducing array of type %s\n\n", dtype_cli_name(o.dtype));

  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  bool ok = true;
  try {
    Workspace ws(o.device);
    if (args.has("shmoo")) {
      run_shmoo(o, ws, s, args.int_or<uint64_t>("shmoo-max", 33554432ull));
    } else if (o.arg) {
      ok = run_arg_test(o, ws, s);
    } else {
      ok = run_test(o, ws, s);
    }
  } catch (const Error& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    ok = false;
  }
  HIP_CHECK(hipStreamDestroy(s));
  L.close();
  qa_finish_exit(argc, cargv, ok ? QaStatus::Passed : QaStatus::Failed);
}
