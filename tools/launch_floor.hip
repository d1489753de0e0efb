// Where does the per-launch fixed cost of the streaming reduction go? Every
// variant is replayed from a captured hipGraph of back-to-back launches on one stream (the bench's
// headline protocol: each launch completes before the next starts), hipEvents around the replay,
// rounds interleaved; printed: microseconds per launch (median over rounds) for
//   empty1 / empty768      an empty kernel, 1 / 768 workgroups of 256 threads: the launch floor;
//   args1                  one workgroup that reads the production kernel's Args (by value, ~200 B
//                          of kernarg) and stores one word: + the kernarg fetch;
//   poll768                768 workgroups that each publish a tagged slot and a finisher that polls
//                          them (the production fan-in alone, no data); _coarse: the words in
//                          ordinary device memory instead of uncached;
//   reduce_<n>             the production kern::reduce_stream (tuned plan, polled fan-in) over n
//                          doubles, its result checked against a host sum (_coarse: on a Workspace
//                          made with SlotMemory::Coarse).
//   build: make launch_floor     run: build/bin/launch_floor [--rounds=7] [--launches=200]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../csrc/kernels/reduce_kernels.hpp"

using namespace mireduce;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      std::exit(2);                                                                            \
    }                                                                                          \
  } while (0)

__global__ __launch_bounds__(256) void empty_kernel(int) {}

__global__ __launch_bounds__(256) void args_kernel(kern::Args a) {
  if (blockIdx.x == 0 && threadIdx.x == 0)
    *static_cast<uint64_t*>(a.out) = a.nvec + a.head + a.tail + static_cast<uint64_t>(a.two_pass) + a.fan_bound;
}

// The polled fan-in without data: every workgroup publishes (epoch << 32 | 1) to its slot, the last
// one polls all slots (bounded) and advances the epoch; the same uncached Workspace words.
__global__ __launch_bounds__(256) void poll_kernel(uint64_t* slots, unsigned* fan, uint64_t* out) {
  const unsigned e = __builtin_amdgcn_readfirstlane(__hip_atomic_load(fan, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  const uint64_t tag = static_cast<uint64_t>(e) << 32;
  if (threadIdx.x == 0) __hip_atomic_store(slots + blockIdx.x, tag | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x != gridDim.x - 1) return;
  uint64_t sum = 0;
  for (unsigned i = threadIdx.x; i < gridDim.x; i += 256) {
    uint64_t w;
    const uint64_t t0 = wall_clock64();
    do {
      w = __hip_atomic_load(slots + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } while ((w >> 32) != e && wall_clock64() - t0 < 100000000ull);
    sum += w & 0xffffffffull;
  }
  __shared__ uint64_t red[4];
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    *out = red[0] + red[1] + red[2] + red[3];
    __hip_atomic_store(fan, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <class F>
double replay_us(F&& enqueue, int launches, hipStream_t s) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < launches; ++i) enqueue(s);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));  // upload + warm
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return ms * 1e3 / launches;
}

int main(int argc, char** argv) {
  int rounds = 7, launches = 200;
  for (int i = 1; i < argc; ++i) {
    if (!std::strncmp(argv[i], "--rounds=", 9)) rounds = std::atoi(argv[i] + 9);
    if (!std::strncmp(argv[i], "--launches=", 11)) launches = std::atoi(argv[i] + 11);
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Workspace ws(0, 16384);
  Workspace ws_coarse(0, 16384, SlotMemory::Coarse);  // the A/B workspace: fan-in words in ordinary memory
  const std::vector<uint64_t> sizes = {1024, 1ull << 24, 125000000};
  const uint64_t nmax = sizes.back();
  double* x = nullptr;
  CK(hipMalloc(&x, nmax * 8));
  std::vector<double> h(nmax);
  for (uint64_t i = 0; i < nmax; ++i) h[i] = static_cast<double>((i * 2654435761ull) % 1000) * 0.001;
  CK(hipMemcpy(x, h.data(), nmax * 8, hipMemcpyHostToDevice));
  double* out = nullptr;
  uint64_t* scratch = nullptr;
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&scratch, 16384 * 8));
  CK(hipMemset(scratch, 0, 16384 * 8));
  unsigned* pfan = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&pfan), 64, hipDeviceMallocUncached));
  CK(hipMemset(pfan, 0, 64));
  uint64_t* pslots = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&pslots), 16384 * 8, hipDeviceMallocUncached));
  CK(hipMemset(pslots, 0, 16384 * 8));
  unsigned* cfan = nullptr;
  uint64_t* cslots = nullptr;
  CK(hipMalloc(&cfan, 64));
  CK(hipMemset(cfan, 0, 64));
  CK(hipMalloc(&cslots, 16384 * 8));
  CK(hipMemset(cslots, 0, 16384 * 8));
  kern::Args dummy{};
  dummy.out = scratch;

  struct V {
    std::string name;
    std::function<void(hipStream_t)> enqueue;
    uint64_t n;  // > 0: a reduction to check
  };
  std::vector<V> vars;
  vars.push_back({"empty1", [](hipStream_t st) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(256), 0, st, 0); }, 0});
  vars.push_back({"empty768", [](hipStream_t st) { hipLaunchKernelGGL(empty_kernel, dim3(768), dim3(256), 0, st, 0); }, 0});
  vars.push_back({"args1", [&](hipStream_t st) { hipLaunchKernelGGL(args_kernel, dim3(1), dim3(256), 0, st, dummy); }, 0});
  vars.push_back({"poll768", [&](hipStream_t st) {
                    hipLaunchKernelGGL(poll_kernel, dim3(768), dim3(256), 0, st, pslots, pfan, scratch);
                  }, 0});
  vars.push_back({"poll768_coarse", [&](hipStream_t st) {
                    hipLaunchKernelGGL(poll_kernel, dim3(768), dim3(256), 0, st, cslots, cfan, scratch);
                  }, 0});
  const size_t fixed = vars.size();
  std::vector<std::unique_ptr<BoundReduce>> bound;
  for (uint64_t n : sizes) {
    for (int coarse = 0; coarse < 2; ++coarse) {
      bound.emplace_back(new BoundReduce(x, n, DType::Float64, Op::Sum, DType::Float64, out, coarse ? ws_coarse : ws));
      BoundReduce* b = bound.back().get();
      vars.push_back({"reduce_" + std::to_string(n) + (coarse ? "_coarse" : ""), [b](hipStream_t st) { b->launch(st); }, n});
    }
  }
  std::vector<std::vector<double>> us(vars.size());
  std::vector<size_t> order(vars.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::mt19937 rng(7);
  bool ok = true;
  for (int r = 0; r < rounds; ++r) {
    std::shuffle(order.begin(), order.end(), rng);
    for (size_t k : order) {
      us[k].push_back(replay_us(vars[k].enqueue, launches, s));
      if (vars[k].n) {
        double got = 0, want = 0;
        CK(hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < vars[k].n; ++i) want += h[i];
        if (!(std::fabs(got - want) <= 1e-9 * std::fabs(want) + 1e-9)) {
          std::fprintf(stderr, "%s: got %.17g want %.17g\n", vars[k].name.c_str(), got, want);
          ok = false;
        }
      }
    }
  }
  std::printf("variant        us/launch (median of %d rounds x %d graph-replayed launches)  min     plan\n", rounds,
              launches);
  for (size_t k = 0; k < vars.size(); ++k) {
    std::vector<double> v = us[k];
    std::sort(v.begin(), v.end());
    std::string plan;
    if (vars[k].n) {
      const LaunchPlan& p = bound[k - fixed]->plan();
      plan = std::to_string(p.block) + "x" + std::to_string(p.unroll) + " grid " + std::to_string(p.grid) +
             " window " + std::to_string(p.window) + " xskew " + std::to_string(p.xskew);
    }
    std::printf("%-14s %10.3f %10.3f  %s\n", vars[k].name.c_str(), v[v.size() / 2], v.front(), plan.c_str());
  }
  unsigned err = ws.error() | ws_coarse.error();
  std::printf("fan-in error word %u, results %s\n", err, ok ? "verified" : "WRONG");
  return ok && err == 0 ? 0 : 1;
}
