// bandwidth_test — measured HBM3E roofline for the reduction kernels.
//
// Reference: the vendored bandwidthTest (cuda/C/src/bandwidthTest/bandwidthTest.cu:867,903-925):
// device-to-device copy bandwidth counted as 2 x bytes (read + write) / time, plus H2D / D2H.
// Added: a read-only stream (the reduction kernel itself, bytes / time) and a write-only stream
// (hipMemsetAsync), so every reduction number can be read against what this GPU's HBM delivers
// for the same direction of traffic.
#include <hip/hip_runtime_api.h>

#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

#include "mireduce/check.hpp"
#include "mireduce/cli.hpp"
#include "mireduce/device.hpp"
#include "mireduce/reduce.hpp"
#include "mireduce/report.hpp"

using namespace mireduce;

int main(int argc, char** argv) {
  CmdArgs args;
  try {
    args = CmdArgs(argc, argv);
  } catch (const CliError& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return EXIT_FAILURE;
  }
  if (args.has("help")) {
    std::printf("bandwidth_test [--size=BYTES (default 2G)] [--iters=20] [--device=0] [--host] [--json=PATH]\n");
    return EXIT_SUCCESS;
  }
  uint64_t size = 2ull << 30;
  args.get_uint("size", &size);
  const int iters = args.int_or<int>("iters", 20);
  const int dev = args.int_or<int>("device", 0);
  const std::string json = args.str_or("json", "");
  if (device_count() <= dev) {
    std::fprintf(stderr, "no HIP device %d\n", dev);
    return EXIT_FAILURE;
  }
  HIP_CHECK(hipSetDevice(dev));
  DeviceInfo di = device_info(dev);
  std::printf("Device %d: %s (%s, %d CUs)\n", dev, di.name.c_str(), di.arch.c_str(), di.cus);
  size -= size % 64;
  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  DeviceBuffer a(size), b(size), out(8);
  FillSpec fs;
  fill_device(a.get(), size / 8, DType::Float64, fs, s);
  HIP_CHECK(hipMemsetAsync(b.get(), 0, size, s));
  HIP_CHECK(hipStreamSynchronize(s));
  Workspace ws(dev);
  EventTimer ev;
  Json j;
  j.set("device", di.name).set("arch", di.arch).set("bytes", size).set("iters", iters);

  auto measure = [&](const char* name, double bytes_per_iter, auto&& body) {
    body();
    HIP_CHECK(hipStreamSynchronize(s));
    ev.start(s);
    for (int i = 0; i < iters; ++i) body();
    ev.stop(s);
    const double ms = ev.elapsed_ms() / iters;
    const double gbps = bytes_per_iter / (ms * 1e-3) / kGB;
    std::printf("%-34s %12.1f GB/s   (%.4f ms per pass, %" PRIu64 " bytes)\n", name, gbps, ms, size);
    j.set(std::string(name), gbps);
  };

  measure("Device to Device copy (2x bytes)", 2.0 * size, [&] {
    HIP_CHECK(hipMemcpyAsync(b.get(), a.get(), size, hipMemcpyDeviceToDevice, s));
  });
  measure("Read stream (mireduce f64 sum)", static_cast<double>(size), [&] {
    reduce(a.get(), size / 8, DType::Float64, Op::Sum, DType::Float64, out.get(), ws, s);
  });
  measure("Read stream (f32 sum, f64 acc)", static_cast<double>(size), [&] {
    reduce(a.get(), size / 4, DType::Float32, Op::Sum, DType::Float64, out.get(), ws, s);
  });
  measure("Write stream (hipMemsetAsync)", static_cast<double>(size), [&] {
    HIP_CHECK(hipMemsetAsync(b.get(), 0, size, s));
  });
  if (args.has("host")) {
    const size_t hb = std::min<uint64_t>(size, 1ull << 30);
    void* h = nullptr;
    HIP_CHECK(hipHostMalloc(&h, hb, hipHostMallocDefault));
    measure("Host to Device (pinned)", static_cast<double>(hb), [&] {
      HIP_CHECK(hipMemcpyAsync(a.get(), h, hb, hipMemcpyHostToDevice, s));
    });
    measure("Device to Host (pinned)", static_cast<double>(hb), [&] {
      HIP_CHECK(hipMemcpyAsync(h, a.get(), hb, hipMemcpyDeviceToHost, s));
    });
    HIP_CHECK(hipHostFree(h));
  }
  if (!json.empty()) j.write_file(json);
  HIP_CHECK(hipStreamDestroy(s));
  return EXIT_SUCCESS;
}
