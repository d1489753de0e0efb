// pybind11 binding: cuda_mpi_reductions_amd._C
//
// Exposes the native HIP kernels, the host reference reducers and MT19937 to Python. Tensors
// cross the boundary as raw device pointers + HIP stream handles (taken from torch on the Python
// side), so this module has no libtorch dependency and builds in seconds.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstring>
#include <memory>

#include "mireduce/arg_reduce.hpp"
#include "mireduce/check.hpp"
#include "mireduce/cpu_reference.hpp"
#include "mireduce/direct.hpp"
#include "mireduce/final_line.hpp"
#include "mireduce/ladder.hpp"
#include "mireduce/moments.hpp"
#include "mireduce/mt19937.hpp"
#include "mireduce/reduce.hpp"
#include "mireduce/reduce_dim.hpp"
#include "mireduce/reduce_many.hpp"
#include "mireduce/trace.hpp"
#include "mireduce/types.hpp"
#include "mireduce/version.hpp"
#include "mireduce/xrank.hpp"

namespace py = pybind11;
using namespace mireduce;

namespace {

template <class T>
T* as_ptr(uintptr_t p) { return reinterpret_cast<T*>(p); }

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

py::dict plan_dict(const LaunchPlan& p) {
  py::dict d;
  d["block"] = p.block;
  d["unroll"] = p.unroll;
  d["grid"] = p.grid;
  d["nontemporal"] = p.nontemporal;
  d["window"] = p.window;
  d["single_pass"] = p.single_pass;
  d["xskew"] = p.xskew;
  d["head"] = p.head;
  d["nvec"] = p.nvec;
  d["tail"] = p.tail;
  d["segments"] = p.segments;
  d["segment_elems"] = p.segment_elems;
  return d;
}

constexpr int kSkewAuto = -2147483647 - 1;  // ReduceConfig::xcd_skew's "tuned default"

ReduceConfig make_cfg(int block, int unroll, int wg_per_cu, int max_blocks, int policy, bool single_pass,
                      int window = -1, int xcd_skew = kSkewAuto, int64_t segment_bytes = 0) {
  ReduceConfig c;
  c.segment_bytes = segment_bytes;
  c.window = window;
  c.xcd_skew = xcd_skew;
  c.block = block;
  c.unroll = unroll;
  c.wg_per_cu = wg_per_cu;
  c.max_blocks = max_blocks;
  c.policy = policy;
  c.single_pass = single_pass;
  return c;
}

py::object acc_to_py(const void* p, DType acc) {
  if (dtype_is_float(acc)) return py::float_(acc_as_double(p, acc));
  return py::int_(acc_as_int64(p, acc));
}

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "mireduce native core: gfx950 HIP reduction kernels, host references, MT19937";

  py::register_exception<Error>(m, "NativeError");

  m.attr("DTYPE_INT32") = static_cast<int>(DType::Int32);
  m.attr("DTYPE_INT64") = static_cast<int>(DType::Int64);
  m.attr("DTYPE_FLOAT32") = static_cast<int>(DType::Float32);
  m.attr("DTYPE_FLOAT64") = static_cast<int>(DType::Float64);
  m.attr("DTYPE_BFLOAT16") = static_cast<int>(DType::BFloat16);
  m.attr("DTYPE_FLOAT16") = static_cast<int>(DType::Float16);
  m.attr("OP_SUM") = static_cast<int>(Op::Sum);
  m.attr("OP_MIN") = static_cast<int>(Op::Min);
  m.attr("OP_MAX") = static_cast<int>(Op::Max);
  m.attr("OP_SUMSQ") = static_cast<int>(Op::SumSq);
  m.attr("OP_AMAX") = static_cast<int>(Op::AbsMax);
  // Build provenance: hash of the csrc tree this module was built from (tools/source_hash.py).
  m.def("source_hash", [] { return std::string(source_hash()); });

  // Read and clear the calling thread's sticky HIP error (e.g. left behind by an aborted
  // stream capture, which would otherwise fail the next unrelated kernel-launch check).
  m.def("hip_get_last_error", [] {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? std::string() : std::string(hipGetErrorName(e)) + ": " + hipGetErrorString(e);
  });

  // Capture state of a stream (0 none, 1 active, 2 invalidated) and a forced end of capture:
  // recovery after a capture aborted by an exception (bench falls back to eager issue).
  m.def("stream_capture_status", [](uintptr_t stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    const hipError_t e = hipStreamIsCapturing(as_stream(stream), &st);
    if (e != hipSuccess) (void)hipGetLastError();
    return static_cast<int>(st);
  });
  m.def("end_capture", [](uintptr_t stream) {
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(as_stream(stream), &g);
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    return e == hipSuccess ? std::string() : std::string(hipGetErrorName(e));
  });

  m.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });

  m.def("device_info", [](int dev) {
    hipDeviceProp_t p;
    check_hip(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
    py::dict d;
    d["name"] = std::string(p.name);
    d["arch"] = std::string(p.gcnArchName);
    d["cus"] = p.multiProcessorCount;
    d["total_mem"] = static_cast<uint64_t>(p.totalGlobalMem);
    d["clock_khz"] = p.clockRate;
    d["mem_clock_khz"] = p.memoryClockRate;
    d["mem_bus_width"] = p.memoryBusWidth;
    d["l2_bytes"] = p.l2CacheSize;
    d["pci_bus_id"] = p.pciBusID;
    int rt = 0;
    (void)hipRuntimeGetVersion(&rt);
    d["hip_runtime"] = rt;
    return d;
  });

  m.def("mem_info", [](int dev) {
    int prev = 0;
    check_hip(hipGetDevice(&prev), "hipGetDevice");
    check_hip(hipSetDevice(dev), "hipSetDevice");
    size_t free_b = 0, total_b = 0;
    check_hip(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    check_hip(hipSetDevice(prev), "hipSetDevice");
    return py::make_tuple(free_b, total_b);
  });

  py::class_<Workspace, std::shared_ptr<Workspace>>(m, "Workspace")
      .def(py::init<int, int>(), py::arg("device") = -1, py::arg("max_grid") = 16384)
      .def_property_readonly("device", &Workspace::device)
      .def_property_readonly("num_cus", &Workspace::num_cus)
      .def_property_readonly("max_grid", &Workspace::max_grid)
      .def_property_readonly("partials_ptr", [](const Workspace& w) { return reinterpret_cast<uintptr_t>(w.partials()); })
      .def("reset", [](Workspace& w, uintptr_t stream) { w.reset(as_stream(stream)); }, py::arg("stream") = 0)
      .def("error", &Workspace::error)
      .def_property_readonly("fan_ptr", [](const Workspace& w) { return reinterpret_cast<uintptr_t>(w.fan()); });

  // Prepared launch for per-step loops: launch(stream) is one positional-argument call.
  py::class_<BoundReduce>(m, "BoundReduce")
      .def(py::init([](Workspace& ws, uintptr_t in, uint64_t n, int dtype, int op, int acc, uintptr_t out,
                       int block, int unroll, int wg_per_cu, int max_blocks, int policy,
                       bool single_pass, uintptr_t xrank, int window, int xcd_skew,
                       int64_t segment_bytes) {
             ReduceConfig cfg = make_cfg(block, unroll, wg_per_cu, max_blocks, policy, single_pass,
                                         window, xcd_skew, segment_bytes);
             cfg.xrank = as_ptr<const void>(xrank);
             return new BoundReduce(as_ptr<const void>(in), n, static_cast<DType>(dtype), static_cast<Op>(op),
                                    static_cast<DType>(acc), as_ptr<void>(out), ws, cfg);
           }),
           py::arg("ws"), py::arg("in_ptr"), py::arg("n"), py::arg("dtype"), py::arg("op"), py::arg("acc"),
           py::arg("out_ptr"), py::arg("block") = 0, py::arg("unroll") = 0, py::arg("wg_per_cu") = 0,
           py::arg("max_blocks") = 0, py::arg("policy") = -1,
           py::arg("single_pass") = true, py::arg("xrank") = 0, py::arg("window") = -1,
           py::arg("xcd_skew") = kSkewAuto, py::arg("segment_bytes") = 0,
           py::keep_alive<1, 2>())
      .def("launch", [](const BoundReduce& b, uintptr_t stream, uintptr_t out) { b.launch(as_stream(stream), as_ptr<void>(out)); },
           py::arg("stream"), py::arg("out_ptr") = 0)
      .def_property_readonly("plan", [](const BoundReduce& b) { return plan_dict(b.plan()); })
      .def("error", &BoundReduce::error);

  // Fused cross-rank finish (xrank.hpp): exchange handle() bytes with every rank, connect(), then
  // pass desc_ptr as BoundReduce(..., xrank=desc_ptr).
  py::class_<XrankChannel, std::shared_ptr<XrankChannel>>(m, "XrankChannel")
      .def(py::init<int, double>(), py::arg("device") = -1, py::arg("timeout_s") = 2.0)
      .def("handle", [](const XrankChannel& c) {
        const IpcHandleBytes h = c.handle();
        return py::bytes(h.data(), h.size());
      })
      .def("connect", [](XrankChannel& c, int rank, int world, const std::vector<py::bytes>& handles) {
        std::vector<IpcHandleBytes> hs(handles.size());
        for (size_t i = 0; i < handles.size(); ++i) {
          const std::string s = handles[i];
          if (s.size() != sizeof(IpcHandleBytes)) throw Error("XrankChannel.connect: bad handle size");
          std::memcpy(hs[i].data(), s.data(), s.size());
        }
        c.connect(rank, world, hs);
      }, py::arg("rank"), py::arg("world"), py::arg("handles"))
      .def_property_readonly("connected", &XrankChannel::connected)
      .def_property_readonly("desc_ptr", [](const XrankChannel& c) { return reinterpret_cast<uintptr_t>(c.device_desc()); })
      .def_property_readonly("rank", &XrankChannel::rank)
      .def_property_readonly("world", &XrankChannel::world)
      .def("error", &XrankChannel::error)
      .def("epoch", &XrankChannel::epoch)
      .def("clear_error", &XrankChannel::clear_error)
      .def("set_stamps", [](XrankChannel& c, uintptr_t p, unsigned cap) { c.set_stamps(as_ptr<uint64_t>(p), cap); },
           py::arg("stamps_ptr"), py::arg("cap"))
      .def_property_readonly("ticks_per_us", &XrankChannel::ticks_per_us);
  m.attr("XRANK_MAX_RANKS") = kMaxXrankRanks;

  // bench.py's one result line, printed exactly once even if the process is killed (final_line.hpp).
  m.def("arm_final_line", [](const std::string& line) { arm_final_line(line); }, py::arg("line"));
  m.def("disarm_final_line", &disarm_final_line);
  m.def("emit_final_line", [](const std::string& line) {
    py::gil_scoped_release nogil;
    return emit_final_line(line);
  }, py::arg("line"));
  m.def("final_line_emitted", &final_line_emitted);

  // Stream-ordered device copy between raw pointers (registered IPC buffers <-> torch tensors).
  m.def("memcpy_d2d", [](uintptr_t dst, uintptr_t src, uint64_t bytes, uintptr_t stream) {
    check_hip(hipMemcpyAsync(as_ptr<void>(dst), as_ptr<const void>(src), bytes, hipMemcpyDeviceToDevice,
                             as_stream(stream)), "hipMemcpyAsync");
  }, py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("stream") = 0);

  // One-kernel direct all-reduce / reduce over IPC-mapped peer buffers (direct.hpp): exchange
  // handles() with every rank, connect(), copy data into in_ptr, then allreduce()/reduce().
  py::class_<DirectAllreduce, std::shared_ptr<DirectAllreduce>>(m, "DirectAllreduce")
      .def(py::init<int, size_t, int, double>(), py::arg("device") = -1, py::arg("bytes") = 16,
           py::arg("grid") = 0, py::arg("timeout_s") = 10.0)
      .def("handles", [](const DirectAllreduce& d) {
        const std::vector<char> h = d.handles();
        return py::bytes(h.data(), h.size());
      })
      .def("connect", [](DirectAllreduce& d, int rank, int world, const std::vector<py::bytes>& all) {
        std::vector<std::vector<char>> hs;
        for (const auto& b : all) {
          const std::string s = b;
          hs.emplace_back(s.begin(), s.end());
        }
        d.connect(rank, world, hs);
      }, py::arg("rank"), py::arg("world"), py::arg("handles"))
      .def_property_readonly("in_ptr", [](const DirectAllreduce& d) { return reinterpret_cast<uintptr_t>(d.in()); })
      .def_property_readonly("out_ptr", [](const DirectAllreduce& d) { return reinterpret_cast<uintptr_t>(d.out()); })
      .def_property_readonly("bytes", &DirectAllreduce::bytes)
      .def_property_readonly("grid", &DirectAllreduce::grid)
      .def_property_readonly("connected", &DirectAllreduce::connected)
      .def("allreduce", [](DirectAllreduce& d, uint64_t count, int dtype, int op, uintptr_t stream) {
        d.allreduce(count, static_cast<DType>(dtype), static_cast<Op>(op), as_stream(stream));
      }, py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("stream") = 0)
      .def("reduce", [](DirectAllreduce& d, uint64_t count, int dtype, int op, int root, uintptr_t stream) {
        d.reduce(count, static_cast<DType>(dtype), static_cast<Op>(op), root, as_stream(stream));
      }, py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("root") = 0, py::arg("stream") = 0)
      .def("read_peers", [](DirectAllreduce& d, uint64_t bytes_each, uintptr_t stream) {
        d.read_peers(bytes_each, as_stream(stream));
      })
      .def("error", &DirectAllreduce::error)
      .def("epoch", &DirectAllreduce::epoch);

  m.def(
      "reduce",
      [](Workspace& ws, uintptr_t in, uint64_t n, int dtype, int op, int acc, uintptr_t out,
         uintptr_t stream, int block, int unroll, int wg_per_cu, int max_blocks,
         int policy, bool single_pass, uint64_t fanin_bound_ticks, int debug_delay_wg,
         uint64_t debug_delay_ticks, int window, uintptr_t xrank, uintptr_t wg_stamps, int xcd_skew,
         uint64_t debug_delay_anchor_ticks, int64_t segment_bytes) {
        ReduceConfig cfg = make_cfg(block, unroll, wg_per_cu, max_blocks, policy, single_pass, window,
                                    xcd_skew, segment_bytes);
        cfg.xrank = as_ptr<const void>(xrank);
        cfg.debug_wg_stamps = as_ptr<uint64_t>(wg_stamps);
        cfg.fanin_bound_ticks = fanin_bound_ticks;
        cfg.debug_delay_wg = debug_delay_wg;
        cfg.debug_delay_ticks = debug_delay_ticks;
        cfg.debug_delay_anchor_ticks = debug_delay_anchor_ticks;
        const LaunchPlan p = reduce(as_ptr<const void>(in), n, static_cast<DType>(dtype),
                                    static_cast<Op>(op), static_cast<DType>(acc),
                                    as_ptr<void>(out), ws, as_stream(stream), cfg);
        return plan_dict(p);
      },
      py::arg("ws"), py::arg("in_ptr"), py::arg("n"), py::arg("dtype"), py::arg("op"),
      py::arg("acc"), py::arg("out_ptr"), py::arg("stream") = 0, py::arg("block") = 0,
      py::arg("unroll") = 0, py::arg("wg_per_cu") = 0, py::arg("max_blocks") = 0,
      py::arg("policy") = -1, py::arg("single_pass") = true,
      py::arg("fanin_bound_ticks") = 0, py::arg("debug_delay_wg") = -1,
      py::arg("debug_delay_ticks") = 0, py::arg("window") = -1, py::arg("xrank") = 0, py::arg("wg_stamps") = 0,
      py::arg("xcd_skew") = kSkewAuto, py::arg("debug_delay_anchor_ticks") = 0, py::arg("segment_bytes") = 0);

  m.def(
      "plan",
      [](uintptr_t in, uint64_t n, int dtype, int num_cus, int max_grid, int block, int unroll,
         int wg_per_cu, int max_blocks, int policy, bool single_pass, int window,
         int op, int xcd_skew, int64_t segment_bytes) {
        MIREDUCE_REQUIRE(op >= 0 && op < kNumOps, "op out of range");
        const ReduceConfig cfg = make_cfg(block, unroll, wg_per_cu, max_blocks, policy, single_pass,
                                          window, xcd_skew, segment_bytes);
        LaunchPlan p = plan_reduce(as_ptr<const void>(in), n, static_cast<DType>(dtype), cfg, num_cus, max_grid,
                                   static_cast<Op>(op));
        plan_segmentation(n, static_cast<DType>(dtype), cfg, p, std::min(256, max_grid));
        return plan_dict(p);
      },
      py::arg("in_ptr"), py::arg("n"), py::arg("dtype"), py::arg("num_cus") = 256,
      py::arg("max_grid") = 16384, py::arg("block") = 0, py::arg("unroll") = 0,
      py::arg("wg_per_cu") = 0, py::arg("max_blocks") = 0,
      py::arg("policy") = -1, py::arg("single_pass") = true, py::arg("window") = -1,
      py::arg("op") = 0, py::arg("xcd_skew") = kSkewAuto, py::arg("segment_bytes") = 0);

  m.def(
      "reduce_partials",
      [](uintptr_t in, uint64_t n, int dtype, int op, int acc, uintptr_t partials, int max_grid,
         int num_cus, uintptr_t stream, int block, int unroll, int wg_per_cu, int max_blocks, int policy) {
        ReduceConfig c = make_cfg(block, unroll, wg_per_cu, max_blocks, policy, false);
        return plan_dict(reduce_partials(as_ptr<const void>(in), n, static_cast<DType>(dtype),
                                         static_cast<Op>(op), static_cast<DType>(acc),
                                         as_ptr<void>(partials), max_grid, num_cus,
                                         as_stream(stream), c));
      },
      py::arg("in_ptr"), py::arg("n"), py::arg("dtype"), py::arg("op"), py::arg("acc"),
      py::arg("partials_ptr"), py::arg("max_grid"), py::arg("num_cus"), py::arg("stream") = 0,
      py::arg("block") = 0, py::arg("unroll") = 0, py::arg("wg_per_cu") = 0,
      py::arg("max_blocks") = 0, py::arg("policy") = -1);

  m.def(
      "reduce_finalize",
      [](uintptr_t partials, uint64_t count, int acc, int op, uintptr_t out, uintptr_t stream) {
        reduce_finalize(as_ptr<const void>(partials), count, static_cast<DType>(acc),
                        static_cast<Op>(op), as_ptr<void>(out), as_stream(stream));
      },
      py::arg("partials_ptr"), py::arg("count"), py::arg("acc"), py::arg("op"), py::arg("out_ptr"),
      py::arg("stream") = 0);

  m.def(
      "combine_elementwise",
      [](uintptr_t inout, uintptr_t other, uint64_t n, int dtype, int op, uintptr_t stream) {
        combine_elementwise(as_ptr<void>(inout), as_ptr<const void>(other), n,
                            static_cast<DType>(dtype), static_cast<Op>(op), as_stream(stream));
      },
      py::arg("inout_ptr"), py::arg("other_ptr"), py::arg("n"), py::arg("dtype"), py::arg("op"),
      py::arg("stream") = 0);

  m.def(
      "fill_device",
      [](uintptr_t ptr, uint64_t n, int dtype, int pattern, uint64_t seed, uint64_t offset,
         double value, uintptr_t stream) {
        FillSpec s;
        s.pattern = static_cast<Pattern>(pattern);
        s.seed = seed;
        s.offset = offset;
        s.value = value;
        fill_device(as_ptr<void>(ptr), n, static_cast<DType>(dtype), s, as_stream(stream));
      },
      py::arg("ptr"), py::arg("n"), py::arg("dtype"), py::arg("pattern") = 0,
      py::arg("seed") = 0x5EED, py::arg("offset") = 0, py::arg("value") = 0.0,
      py::arg("stream") = 0);

  m.def(
      "fill_host",
      [](uintptr_t ptr, uint64_t n, int dtype, int pattern, uint64_t seed, uint64_t offset,
         double value) {
        FillSpec s;
        s.pattern = static_cast<Pattern>(pattern);
        s.seed = seed;
        s.offset = offset;
        s.value = value;
        py::gil_scoped_release nogil;
        fill_host(as_ptr<void>(ptr), n, static_cast<DType>(dtype), s);
      },
      py::arg("ptr"), py::arg("n"), py::arg("dtype"), py::arg("pattern") = 0,
      py::arg("seed") = 0x5EED, py::arg("offset") = 0, py::arg("value") = 0.0);

  m.def(
      "cpu_reduce",
      [](uintptr_t ptr, uint64_t n, int dtype, int op, int acc, int threads) {
        alignas(8) unsigned char out[8] = {0};
        {
          py::gil_scoped_release nogil;
          cpu_reduce(as_ptr<const void>(ptr), n, static_cast<DType>(dtype), static_cast<Op>(op),
                     static_cast<DType>(acc), out, threads);
        }
        return acc_to_py(out, static_cast<DType>(acc));
      },
      py::arg("ptr"), py::arg("n"), py::arg("dtype"), py::arg("op"), py::arg("acc"),
      py::arg("threads") = 0);

  m.def(
      "cpu_abs_sum",
      [](uintptr_t ptr, uint64_t n, int dtype, int threads) {
        py::gil_scoped_release nogil;
        return cpu_abs_sum(as_ptr<const void>(ptr), n, static_cast<DType>(dtype), threads);
      },
      py::arg("ptr"), py::arg("n"), py::arg("dtype"), py::arg("threads") = 0);

  m.def("sum_tolerance", [](int dtype, int acc, uint64_t n, double abs_sum) {
    return sum_tolerance(static_cast<DType>(dtype), static_cast<DType>(acc), n, abs_sum);
  });

  m.def("default_acc", [](int dtype, int op) {
    return static_cast<int>(default_acc(static_cast<DType>(dtype), static_cast<Op>(op)));
  });

  m.def("acc_supported", [](int dtype, int op, int acc) {
    return acc_supported(static_cast<DType>(dtype), static_cast<Op>(op), static_cast<DType>(acc));
  });

  m.def(
      "ladder_reduce",
      [](int kernel, uintptr_t in, uint64_t n, int dtype, int op, int acc, uintptr_t out, uintptr_t scratch,
         int threads, int max_blocks, uintptr_t stream) {
        return ladder_reduce(kernel, as_ptr<const void>(in), n, static_cast<DType>(dtype), static_cast<Op>(op),
                             static_cast<DType>(acc), as_ptr<void>(out), as_ptr<void>(scratch), threads, max_blocks,
                             as_stream(stream));
      },
      py::arg("kernel"), py::arg("in_ptr"), py::arg("n"), py::arg("dtype"), py::arg("op"), py::arg("acc"),
      py::arg("out_ptr"), py::arg("scratch_ptr"), py::arg("threads") = 256, py::arg("max_blocks") = 64,
      py::arg("stream") = 0);

  m.def("ladder_scratch_bytes", &ladder_scratch_bytes, py::arg("kernel"), py::arg("n"), py::arg("threads") = 256,
        py::arg("max_blocks") = 64);

  m.def("ladder_geometry", [](int kernel, uint64_t n, int threads, int max_blocks) {
    int b = 0, t = 0;
    ladder_geometry(kernel, n, threads, max_blocks, &b, &t);
    return py::make_tuple(b, t);
  });

  m.def("compiled_variants", &compiled_variants);

  // One launch over a list of same-typed tensors (csrc/kernels/reduce_many.hip).
  py::class_<BoundReduceMany>(m, "BoundReduceMany")
      .def(py::init([](const std::vector<uintptr_t>& ptrs, const std::vector<uint64_t>& counts, int dtype, int op,
                       int acc, uintptr_t out, int device, int num_cus, uintptr_t stream) {
             std::vector<const void*> p;
             p.reserve(ptrs.size());
             for (uintptr_t v : ptrs) p.push_back(as_ptr<const void>(v));
             return new BoundReduceMany(p, counts, static_cast<DType>(dtype), static_cast<Op>(op),
                                        static_cast<DType>(acc), as_ptr<void>(out), device, num_cus, as_stream(stream));
           }),
           py::arg("ptrs"), py::arg("counts"), py::arg("dtype"), py::arg("op"), py::arg("acc"), py::arg("out_ptr"),
           py::arg("device"), py::arg("num_cus"), py::arg("stream") = 0)
      .def("launch", [](const BoundReduceMany& b, uintptr_t stream, uintptr_t out) { b.launch(as_stream(stream), as_ptr<void>(out)); },
           py::arg("stream"), py::arg("out_ptr") = 0)
      .def_property_readonly("tensors", &BoundReduceMany::tensors)
      .def_property_readonly("segments", &BoundReduceMany::segments)
      .def_property_readonly("grid", &BoundReduceMany::grid);

  // Reductions along one axis of a row-major [rows, cols] matrix (csrc/kernels/reduce_dim.hip).
  auto dim_dict = [](const DimPlan& p) {
    py::dict d;
    d["grid"] = p.grid;
    d["block"] = p.block;
    d["lanes_per_row"] = p.lanes_per_row;
    d["splits"] = p.splits;
    return d;
  };
  m.def(
      "reduce_rows",
      [dim_dict](uintptr_t in, uint64_t rows, uint64_t cols, int dtype, int op, int acc, uintptr_t out,
                 uintptr_t scratch, int num_cus, uintptr_t stream) {
        return dim_dict(reduce_rows(as_ptr<const void>(in), rows, cols, static_cast<DType>(dtype), static_cast<Op>(op),
                                    static_cast<DType>(acc), as_ptr<void>(out), as_ptr<void>(scratch), num_cus,
                                    as_stream(stream)));
      },
      py::arg("in_ptr"), py::arg("rows"), py::arg("cols"), py::arg("dtype"), py::arg("op"), py::arg("acc"),
      py::arg("out_ptr"), py::arg("scratch_ptr"), py::arg("num_cus"), py::arg("stream") = 0);
  m.def(
      "reduce_cols",
      [dim_dict](uintptr_t in, uint64_t outer, uint64_t rows, uint64_t cols, int dtype, int op, int acc, uintptr_t out,
                 uintptr_t scratch, int num_cus, uintptr_t stream) {
        return dim_dict(reduce_cols(as_ptr<const void>(in), outer, rows, cols, static_cast<DType>(dtype), static_cast<Op>(op),
                                    static_cast<DType>(acc), as_ptr<void>(out), as_ptr<void>(scratch), num_cus,
                                    as_stream(stream)));
      },
      py::arg("in_ptr"), py::arg("outer"), py::arg("rows"), py::arg("cols"), py::arg("dtype"), py::arg("op"),
      py::arg("acc"), py::arg("out_ptr"), py::arg("scratch_ptr"), py::arg("num_cus"), py::arg("stream") = 0);
  m.def("reduce_rows_scratch_bytes", [](uint64_t rows, uint64_t cols, int dtype, int num_cus) {
    return reduce_rows_scratch_bytes(rows, cols, static_cast<DType>(dtype), num_cus);
  });
  m.def("reduce_cols_scratch_bytes", [](uint64_t outer, uint64_t rows, uint64_t cols, int dtype, int acc, int num_cus) {
    return reduce_cols_scratch_bytes(outer, rows, cols, static_cast<DType>(dtype), static_cast<DType>(acc), num_cus);
  });

  m.def(
      "arg_reduce_rows",
      [](uintptr_t in, uint64_t rows, uint64_t cols, int dtype, int op, uintptr_t out_value, uintptr_t out_index,
         uintptr_t scratch, int num_cus, uintptr_t stream, int unroll, int wg_per_cu) {
        ArgTune tune;
        tune.unroll = unroll;
        tune.wg_per_cu = wg_per_cu;
        const ArgPlan p = arg_reduce_rows(as_ptr<const void>(in), rows, cols, static_cast<DType>(dtype),
                                          static_cast<Op>(op), as_ptr<void>(out_value), as_ptr<int64_t>(out_index),
                                          as_ptr<void>(scratch), num_cus, as_stream(stream), tune);
        py::dict d;
        d["grid"] = p.grid;
        d["block"] = p.block;
        d["lanes_per_row"] = p.lanes_per_row;
        d["splits"] = p.splits;
        d["unroll"] = p.unroll;
        d["wg_per_cu"] = p.wg_per_cu;
        return d;
      },
      py::arg("in_ptr"), py::arg("rows"), py::arg("cols"), py::arg("dtype"), py::arg("op"), py::arg("out_value_ptr"),
      py::arg("out_index_ptr"), py::arg("scratch_ptr"), py::arg("num_cus"), py::arg("stream") = 0,
      py::arg("unroll") = 0, py::arg("wg_per_cu") = 0);
  m.def(
      "loc_pack",
      [](uintptr_t value, uintptr_t index, int64_t offset, int dtype, uintptr_t pair, uintptr_t stream) {
        loc_pack(as_ptr<const void>(value), as_ptr<const int64_t>(index), offset, static_cast<DType>(dtype),
                 as_ptr<uint64_t>(pair), as_stream(stream));
      },
      py::arg("value_ptr"), py::arg("index_ptr"), py::arg("offset"), py::arg("dtype"), py::arg("pair_ptr"),
      py::arg("stream") = 0);
  m.def(
      "loc_pick",
      [](uintptr_t pairs, int world, int dtype, int op, uintptr_t out_index, uintptr_t out_value, uintptr_t stream) {
        loc_pick(as_ptr<const uint64_t>(pairs), world, static_cast<DType>(dtype), static_cast<Op>(op),
                 as_ptr<int64_t>(out_index), as_ptr<void>(out_value), as_stream(stream));
      },
      py::arg("pairs_ptr"), py::arg("world"), py::arg("dtype"), py::arg("op"), py::arg("out_index_ptr"),
      py::arg("out_value_ptr") = 0, py::arg("stream") = 0);
  m.def("arg_reduce_scratch_bytes", [](uint64_t rows, uint64_t cols, int dtype, int num_cus) {
    return arg_reduce_scratch_bytes(rows, cols, static_cast<DType>(dtype), num_cus);
  });
  m.def(
      "cpu_arg_reduce_rows",
      [](uintptr_t in, uint64_t rows, uint64_t cols, int dtype, int op, uintptr_t out_value, uintptr_t out_index) {
        py::gil_scoped_release nogil;
        cpu_arg_reduce_rows(as_ptr<const void>(in), rows, cols, static_cast<DType>(dtype), static_cast<Op>(op),
                            as_ptr<void>(out_value), as_ptr<int64_t>(out_index));
      },
      py::arg("in_ptr"), py::arg("rows"), py::arg("cols"), py::arg("dtype"), py::arg("op"), py::arg("out_value_ptr"),
      py::arg("out_index_ptr"));

  m.def(
      "moments",
      [](uintptr_t in, uint64_t n, int dtype, uintptr_t out5, uintptr_t partials, int max_grid, int num_cus,
         uintptr_t stream) {
        moments_device(as_ptr<const void>(in), n, static_cast<DType>(dtype), as_ptr<double>(out5),
                       as_ptr<void>(partials), max_grid, num_cus, as_stream(stream));
      },
      py::arg("in_ptr"), py::arg("n"), py::arg("dtype"), py::arg("out_ptr"), py::arg("partials_ptr"),
      py::arg("max_grid"), py::arg("num_cus"), py::arg("stream") = 0);
  m.def("moments_partials_bytes", &moments_partials_bytes);

  m.def("set_tracing", &set_tracing, "enable roctx ranges (rocprofv3 --marker-trace)");
  m.def("tracing", &tracing);
  m.def("trace_push", [](const std::string& name) { if (tracing()) trace_push(name.c_str()); });
  m.def("trace_pop", [] { if (tracing()) trace_pop(); });

  m.def("synchronize", [](int dev) {
    if (dev >= 0) check_hip(hipSetDevice(dev), "hipSetDevice");
    py::gil_scoped_release nogil;
    check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
  }, py::arg("device") = -1);

  py::class_<Mt19937>(m, "Mt19937")
      .def(py::init<uint32_t>(), py::arg("seed") = 5489u)
      .def("init_genrand", &Mt19937::init_genrand)
      .def("init_by_array",
           [](Mt19937& g, const std::vector<uint64_t>& key) { g.init_by_array(key.data(), key.size()); })
      .def("genrand_int32", &Mt19937::genrand_int32)
      .def("genrand_int31", &Mt19937::genrand_int31)
      .def("genrand_real1", &Mt19937::genrand_real1)
      .def("genrand_real2", &Mt19937::genrand_real2)
      .def("genrand_real3", &Mt19937::genrand_real3)
      .def("genrand_res53", &Mt19937::genrand_res53)
      .def("fill_int32",
           [](Mt19937& g, uintptr_t ptr, uint64_t n) {
             int32_t* p = as_ptr<int32_t>(ptr);
             py::gil_scoped_release nogil;
             for (uint64_t i = 0; i < n; ++i) p[i] = static_cast<int32_t>(g.genrand_int32());
           })
      .def("fill_res53", [](Mt19937& g, uintptr_t ptr, uint64_t n) {
        double* p = as_ptr<double>(ptr);
        py::gil_scoped_release nogil;
        for (uint64_t i = 0; i < n; ++i) p[i] = g.genrand_res53();
      });
}
