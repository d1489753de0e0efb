// bandwidth_test — measured HBM3E roofline for the reduction kernels.
//
// Reference: the vendored bandwidthTest (cuda/C/src/bandwidthTest/bandwidthTest.cu:867,903-925):
// device-to-device copy bandwidth counted as 2 x bytes (read + write) / time, plus H2D / D2H.
// Added: a read-only stream (the reduction kernel itself, bytes / time) and a write-only stream
// (hipMemsetAsync), so every reduction number can be read against what this GPU's HBM delivers
// for the same direction of traffic.
//
// --peer: the xGMI roofline (the vendored simpleP2P, cuda/C/src/simpleP2P/simpleP2P.cu:250-275
// peer enable, :314-329 100 timed peer copies reported in GiB/s) for EVERY ordered device pair:
// hipMemcpyPeerAsync copy GiB/s, a peer-read kernel's per-link GB/s, and all links at once (every
// device reads all its peers concurrently: per-device ingress and node aggregate). Fewer than two
// visible devices: WAIVED (QA protocol), exit 0.
#include <hip/hip_runtime_api.h>

#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

#include "mireduce/version.hpp"
#include "mireduce/check.hpp"
#include "mireduce/cli.hpp"
#include "mireduce/device.hpp"
#include "mireduce/peer.hpp"
#include "mireduce/qa.hpp"
#include "mireduce/reduce.hpp"
#include "mireduce/report.hpp"

using namespace mireduce;

namespace {

int run_peer(int argc, char** argv, const CmdArgs& args) {
  qa_start(argc, argv);
  const int ndev = device_count();
  if (ndev < 2) {
    std::printf("Peer-to-peer (xGMI) bandwidth: %d visible device(s), needs >= 2 -> WAIVED\n", ndev);
    qa_finish_exit(argc, argv, QaStatus::Waived);
  }
  uint64_t size = 64ull << 20;  // simpleP2P: 16M floats (simpleP2P.cu:293)
  args.get_uint("size", &size);
  size -= size % 64;
  const int iters = args.int_or<int>("iters", 100);  // simpleP2P.cu:314
  const std::string json = args.str_or("json", "");
  std::vector<void*> buf(ndev, nullptr);
  std::vector<uint32_t*> sink(ndev, nullptr);
  std::vector<hipStream_t> st(ndev);
  std::vector<hipEvent_t> e0(ndev), e1(ndev);  // per device: an event must belong to its stream's device
  std::vector<int> access(static_cast<size_t>(ndev) * ndev, 0);
  for (int d = 0; d < ndev; ++d) {
    HIP_CHECK(hipSetDevice(d));
    HIP_CHECK(hipMalloc(&buf[d], size));
    HIP_CHECK(hipMemset(buf[d], d + 1, size));
    HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&sink[d]), 4096 * sizeof(uint32_t)));
    HIP_CHECK(hipStreamCreateWithFlags(&st[d], hipStreamNonBlocking));
    HIP_CHECK(hipEventCreate(&e0[d]));
    HIP_CHECK(hipEventCreate(&e1[d]));
  }
  auto elapsed_ms = [&](int d) {
    HIP_CHECK(hipEventSynchronize(e1[d]));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0[d], e1[d]));
    return static_cast<double>(ms);
  };
  for (auto [s, d] : peer_pairs(ndev)) {  // simpleP2P.cu:250-275: check, then enable both ways
    int can = 0;
    HIP_CHECK(hipDeviceCanAccessPeer(&can, d, s));  // can d map s's memory?
    access[static_cast<size_t>(s) * ndev + d] = can;
    if (can) {
      HIP_CHECK(hipSetDevice(d));
      const hipError_t e = hipDeviceEnablePeerAccess(s, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(e);
      (void)hipGetLastError();
    }
  }
  std::printf("Peer-to-peer (xGMI) bandwidth: %d devices, %" PRIu64 " bytes per transfer, %d iterations\n", ndev,
              size, iters);
  Json j;
  j.set("mode", "peer").set("devices", ndev).set("bytes", size).set("iters", iters);
  std::vector<double> copy(static_cast<size_t>(ndev) * ndev, 0.0), read(copy.size(), 0.0);
  bool ok = true;
  for (auto [s, d] : peer_pairs(ndev)) {
    const size_t k = static_cast<size_t>(s) * ndev + d;
    if (!access[k]) {
      ok = false;
      continue;
    }
    // copy s -> d issued on the destination's stream (warm-up, then `iters` timed)
    HIP_CHECK(hipSetDevice(d));
    HIP_CHECK(hipMemcpyPeerAsync(buf[d], d, buf[s], s, size, st[d]));
    HIP_CHECK(hipStreamSynchronize(st[d]));
    HIP_CHECK(hipEventRecord(e0[d], st[d]));
    for (int i = 0; i < iters; ++i) HIP_CHECK(hipMemcpyPeerAsync(buf[d], d, buf[s], s, size, st[d]));
    HIP_CHECK(hipEventRecord(e1[d], st[d]));
    copy[k] = static_cast<double>(size) * iters / (elapsed_ms(d) * 1e-3) / kGiB;  // simpleP2P.cu:328-329
    // d's kernel reads s's buffer over the link
    PeerSources one{};
    one.p[0] = buf[s];
    peer_read(one, 1, size, sink[d], 0, st[d]);
    HIP_CHECK(hipStreamSynchronize(st[d]));
    HIP_CHECK(hipEventRecord(e0[d], st[d]));
    for (int i = 0; i < iters; ++i) peer_read(one, 1, size, sink[d], 0, st[d]);
    HIP_CHECK(hipEventRecord(e1[d], st[d]));
    read[k] = static_cast<double>(size) * iters / (elapsed_ms(d) * 1e-3) / kGB;
  }
  std::printf("hipMemcpyPeerAsync copy, src -> dst\n%s", peer_matrix(ndev, copy, "GiB/s").c_str());
  std::printf("peer-read kernel, dst reads src\n%s", peer_matrix(ndev, read, "GB/s").c_str());
  // All links at once: every device reads every peer concurrently (one kernel per device).
  std::vector<double> ingress(ndev, 0.0);
  {
    auto all_srcs = [&](int d, int* n) {
      PeerSources ps{};
      *n = 0;
      for (int s = 0; s < ndev && *n < kMaxPeerSources; ++s)
        if (s != d && access[static_cast<size_t>(s) * ndev + d]) ps.p[(*n)++] = buf[s];
      return ps;
    };
    for (int rep = 0; rep < 2; ++rep) {  // rep 0: warm-up
      for (int d = 0; d < ndev; ++d) {
        HIP_CHECK(hipSetDevice(d));
        int n = 0;
        const PeerSources ps = all_srcs(d, &n);
        if (!n) continue;
        HIP_CHECK(hipEventRecord(e0[d], st[d]));
        for (int i = 0; i < (rep ? iters : 1); ++i) peer_read(ps, n, size, sink[d], 256 * n, st[d]);
        HIP_CHECK(hipEventRecord(e1[d], st[d]));
      }
      for (int d = 0; d < ndev; ++d) {
        HIP_CHECK(hipSetDevice(d));
        HIP_CHECK(hipStreamSynchronize(st[d]));
        int n = 0;
        all_srcs(d, &n);
        if (rep && n) ingress[d] = static_cast<double>(size) * n * iters / (elapsed_ms(d) * 1e-3) / kGB;
      }
    }
  }
  double node = 0;
  std::printf("all peers at once (each device reads its %d peers concurrently)\n", ndev - 1);
  for (int d = 0; d < ndev; ++d) {
    std::printf("  device %d ingress %10.1f GB/s  (%.1f GB/s per link)\n", d, ingress[d], ingress[d] / (ndev - 1));
    node += ingress[d];
  }
  std::printf("  node aggregate %10.1f GB/s\n", node);
  std::vector<std::string> keys;
  for (auto [s, d] : peer_pairs(ndev)) {
    const size_t k = static_cast<size_t>(s) * ndev + d;
    j.set("copy_gibps_" + std::to_string(s) + "_" + std::to_string(d), copy[k]);
    j.set("read_gbps_" + std::to_string(s) + "_" + std::to_string(d), read[k]);
  }
  for (int d = 0; d < ndev; ++d) j.set("ingress_gbps_" + std::to_string(d), ingress[d]);
  j.set("node_ingress_gbps", node).set("all_pairs_peer_access", ok);
  if (!json.empty()) j.write_file(json);
  for (int d = 0; d < ndev; ++d) {
    HIP_CHECK(hipSetDevice(d));
    HIP_CHECK(hipStreamDestroy(st[d]));
    HIP_CHECK(hipEventDestroy(e0[d]));
    HIP_CHECK(hipEventDestroy(e1[d]));
    HIP_CHECK(hipFree(sink[d]));
    HIP_CHECK(hipFree(buf[d]));
  }
  qa_finish_exit(argc, argv, ok ? QaStatus::Passed : QaStatus::Failed);
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
    std::printf("bandwidth_test (mireduce) native source %s\n", mireduce::source_hash());
    return 0;
  }
  if (args.has("help")) {
    std::printf("bandwidth_test [--size=BYTES (default 2G)] [--iters=20] [--device=0] [--host] [--json=PATH]\n"
                "bandwidth_test --peer [--size=BYTES (default 64M)] [--iters=100] [--json=PATH] [--qatest]\n");
    return EXIT_SUCCESS;
  }
  if (args.has("peer")) return run_peer(argc, argv, args);
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
  {
    DeviceBuffer sk(4096 * sizeof(uint32_t));
    PeerSources self{};
    self.p[0] = a.get();
    measure("Read stream (peer_read kernel, local)", static_cast<double>(size), [&] {
      peer_read(self, 1, size, sk.as<uint32_t>(), 0, s);
    });
  }
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
