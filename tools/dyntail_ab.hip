// Experiment (round 4, not the production path): does a workgroup-level DYNAMIC tail beat the
// static XCD-weighted split? After the XCD skew, workgroup end times still spread 17-30 us over an
// 8 GB kernel, run-to-run noise no static weighting can remove (docs/TUNING.md, "What is left of the
// tail"). Here every workgroup streams `static_rounds` interleaved rounds (b, b + grid, ...), then
// claims the remaining tiles one at a time from a counter in uncached memory: the claim for the tile
// after next is issued at the start of a step and broadcast through LDS at its end, so its latency
// hides under the current tile's consume. Compared, same box, interleaved rounds, hipEvent per
// launch, every result checked:
//   prod s0 / prod s20   the production kern::reduce_stream (256 x 8, window 4, polled fan-in):
//                        equal rounds / the anchored XCD-weighted split (19 extra rounds at 1e9)
//   dyn K                this kernel, the last K rounds of tiles dynamic (s20+dyn K: after the
//                        weighted split's static rounds; partials folded on the
//                        host after timing: no fan-in in the timed launch, which favours it by the
//                        production fan-in's ~1 us)
//   build: make dyntail_ab      run: build/bin/dyntail_ab [--n=1e9] [--rounds=5] [--iters=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

constexpr unsigned kDone = 0xffffffffu;

// ctr[0]: claims of this launch, ctr[1]: workgroups done (the last one zeroes both for the next
// launch; kernel boundaries order that against the next launch's claims). A claim is one returning
// global atomic from lane 0, written as inline asm: hipcc's own atomicAdd here either went through
// the atomic optimizer's lane loop or waited for the return at once (vmcnt(0): the window drained
// every step). The asm's result is read only after the next tile's loads (>= 5 issued after it), so
// a vmcnt(4) wait — which the step's own waits have already satisfied — covers it.
__device__ __forceinline__ unsigned claim_issue(unsigned* ctr) {
  unsigned c = 0;
  if (threadIdx.x == 0)
    asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(c) : "v"(ctr), "v"(1u) : "memory");
  return c;
}
__device__ __forceinline__ unsigned claim_read(unsigned c) {
  // >= 5 loads were issued after the atomic, so vmcnt(4) covers it (the step's own waits already did)
  asm volatile("s_waitcnt vmcnt(4)" : "+v"(c) : : "memory");
  return __builtin_amdgcn_readfirstlane(c);
}
template <int BLOCK, int UNROLL, int WIN>
__global__ __launch_bounds__(BLOCK) void dyn_tail(const double* __restrict__ x, uint64_t nvec, uint32_t static_rounds,
                                                  uint32_t extra, unsigned* ctr, double* partials) {
  using V = kern::Vec16<double>::type;
  __shared__ double lds[BLOCK / 64];
  __shared__ unsigned claim[2];
  double acc[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) acc[u] = 0.0;
  const V* vin = reinterpret_cast<const V*>(x);
  constexpr uint64_t kTile = static_cast<uint64_t>(BLOCK) * UNROLL;
  constexpr uint32_t kStride = BLOCK * 16;
  const uint32_t voff = threadIdx.x * 16;
  const uint32_t ntiles = static_cast<uint32_t>(nvec / kTile), grid = gridDim.x;
  const uint32_t sr0 = static_rounds * grid <= ntiles ? static_rounds : ntiles / grid;
  const uint32_t sr = sr0 > 0 ? sr0 : 1;  // >= 1 static tile per workgroup (the grid <= ntiles here)
  const uint32_t half = grid / 2, ex = sr * grid + extra * half <= ntiles ? extra : 0u;
  const uint32_t p0 = sr * grid + ex * half;  // first dynamic tile
  const bool wave0 = threadIdx.x < 64;
  auto claim_tile = [&](unsigned c) { return p0 + c < ntiles ? p0 + c : kDone; };
  // the first claim: made now, used when the static tiles run out (its wait is long over by then)
  const unsigned c0 = claim_issue(ctr);
  uint32_t t = blockIdx.x;
  __amdgpu_buffer_rsrc_t rp = kern::tile_rsrc(vin + static_cast<uint64_t>(t) * kTile);
  V buf[WIN];
#pragma unroll
  for (int j = 0; j < WIN; ++j) buf[j] = kern::ld_buf_nt<V>(rp, voff, j * kStride);
  auto step = [&](uint32_t t_next) {  // consume the current tile, load t_next's first WIN vectors
    const __amdgpu_buffer_rsrc_t rq = kern::tile_rsrc(vin + static_cast<uint64_t>(t_next) * kTile);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      acc[u] += buf[u % WIN][0] + buf[u % WIN][1];
      const int j = u + WIN;
      buf[u % WIN] = j < UNROLL ? kern::ld_buf_nt<V>(rp, voff, j * kStride)
                                : kern::ld_buf_nt<V>(rq, voff, (j - UNROLL) * kStride);
      __builtin_amdgcn_sched_barrier(0);
    }
    rp = rq;
  };
  // static phase: tiles b, b + grid, ... (sr of them), then `ex` more rounds for the odd
  // workgroups interleaved among themselves (the XCD-weighted split, by blockIdx parity: this
  // tool launches on the null stream, where workgroup b runs on XCC b % 8)
#pragma nounroll
  for (uint32_t k = 1; k < sr; ++k) {
    t += grid;
    step(t);
  }
  if ((blockIdx.x & 1u) && ex > 0) {
    t = sr * grid + (blockIdx.x >> 1);
    step(t);
#pragma nounroll
    for (uint32_t k = 1; k < ex; ++k) {
      t += half;
      step(t);
    }
  }
  // the first dynamic tile (broadcast), then one claim ahead per step
  if (wave0) claim[0] = claim_tile(claim_read(c0));
  __syncthreads();
  uint32_t t_nxt = __builtin_amdgcn_readfirstlane(claim[0]);
  int slot = 1;
#pragma nounroll
  while (t_nxt != kDone) {
    const unsigned c = claim_issue(ctr);  // the tile after next
    step(t_nxt);
    if (wave0) claim[slot] = claim_tile(claim_read(c));
    __syncthreads();
    t_nxt = __builtin_amdgcn_readfirstlane(claim[slot]);  // uniform: no waterfall around the loads
    slot ^= 1;
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {  // the last tile
    acc[u] += buf[u % WIN][0] + buf[u % WIN][1];
    const int j = u + WIN;
    if (j < UNROLL) buf[u % WIN] = kern::ld_buf_nt<V>(rp, voff, j * kStride);
  }
  for (uint64_t i = static_cast<uint64_t>(ntiles) * kTile + blockIdx.x * BLOCK + threadIdx.x; i < nvec;
       i += static_cast<uint64_t>(grid) * BLOCK)
    acc[0] += vin[i][0] + vin[i][1];
#pragma unroll
  for (int u = 1; u < UNROLL; ++u) acc[0] += acc[u];
  const double v = kern::block_reduce<SumOp, double, BLOCK>(acc[0], lds);
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = v;
    if (atomicAdd(ctr + 1, 1u) == grid - 1) {  // the last workgroup: every claim of this launch is made
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void fill(double* x, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    x[i] = static_cast<double>(i & 1023);  // exact sums
}

int main(int argc, char** argv) {
  uint64_t n = 1000000000ull;
  int rounds = 5, iters = 20;
  for (int i = 1; i < argc; ++i) {
    if (!std::strncmp(argv[i], "--n=", 4)) n = static_cast<uint64_t>(std::atof(argv[i] + 4));
    else if (!std::strncmp(argv[i], "--rounds=", 9)) rounds = std::atoi(argv[i] + 9);
    else if (!std::strncmp(argv[i], "--iters=", 8)) iters = std::atoi(argv[i] + 8);
  }
  constexpr int B = 256, U = 8, W = 4;
  double* x;
  double* out;
  unsigned* ctr;
  CK(hipMalloc(&x, n * 8));
  CK(hipMalloc(&out, 8));
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&ctr), 256, hipDeviceMallocUncached));
  CK(hipMemset(ctr, 0, 256));
  fill<<<4096, 256>>>(x, n);
  CK(hipDeviceSynchronize());
  const uint64_t full = n / 1024, rem = n % 1024;
  const double expect = static_cast<double>(full) * (1023.0 * 1024.0 / 2.0) + static_cast<double>(rem) * (rem - 1) / 2.0;
  Workspace ws(0);
  const uint64_t nvec = n / 2;  // hipMalloc: 256-byte aligned, no head; n even
  if (n % 2) {
    std::fprintf(stderr, "--n must be even\n");
    return 2;
  }
  const uint64_t ntiles = nvec / (B * U);
  const int grid = ws.num_cus();
  const uint32_t rounds_all = static_cast<uint32_t>(ntiles / grid);

  struct Var {
    std::string name;
    int skew;   // production: extra rounds for the favoured XCC parity (-1: dyn, -2: skewed dyn)
    int dynk;   // dyn: rounds left dynamic
  };
  std::vector<Var> vars = {{"prod s0", 0, 0}, {"prod s20", 19, 0}};
  for (int kk : {2, 4, 8}) vars.push_back({"dyn K=" + std::to_string(kk), -1, kk});
  for (int kk : {1, 2, 4, 8}) vars.push_back({"s20+dyn K=" + std::to_string(kk), -2, kk});

  auto prod_args = [&](int skew) {
    kern::Args a{};
    a.head_ptr = x;
    a.body = x;
    a.nvec = nvec;
    a.partials = ws.partials();
    a.out = out;
    a.slots = ws.slots();
    a.fan = ws.fan();
    a.fan_slots = static_cast<unsigned>(ws.max_grid());
    a.fan_bound = kern::kFanBoundTicks;
    a.delay_wg = -1;
    a.xskew = skew;
    const uint64_t half = grid / 2;
    a.x_ra = skew ? (ntiles - static_cast<uint64_t>(skew) * half) / grid : ntiles / grid;
    a.x_dd = static_cast<uint64_t>(skew);
    return a;
  };
  double* dpart;
  CK(hipMalloc(&dpart, grid * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> ms(vars.size());
  for (int r = 0; r < rounds; ++r) {
    std::vector<size_t> order(vars.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::srand(r + 5);
    for (size_t i = order.size(); i > 1; --i) std::swap(order[i - 1], order[std::rand() % i]);
    for (size_t i : order) {
      const Var& v = vars[i];
      auto launch = [&]() {
        if (v.skew >= 0) {
          detail::launch_stream<SumOp, double, double, B, U, true, W>(prod_args(v.skew), grid, 0);
        } else {
          // -1: equal static rounds; -2: the weighted split's common rounds (19 extra for the odd
          // workgroups, as production at 1e9) minus the K dynamic ones
          const uint32_t d = v.skew == -2 ? 19u : 0u;
          const uint32_t ra = static_cast<uint32_t>((ntiles - static_cast<uint64_t>(d) * (grid / 2)) / grid);
          hipLaunchKernelGGL((dyn_tail<B, U, W>), dim3(grid), dim3(B), 0, 0, x, nvec,
                             ra > static_cast<uint32_t>(v.dynk) ? ra - v.dynk : 0u, d, ctr, dpart);
        }
      };
      launch();  // warm-up
      for (int it = 0; it < iters; ++it) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms[i].push_back(t);
      }
      double got = 0;
      if (v.skew >= 0) {
        CK(hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost));
      } else {
        std::vector<double> h(grid);
        CK(hipMemcpy(h.data(), dpart, grid * 8, hipMemcpyDeviceToHost));
        for (double p : h) got += p;
      }
      if (got != expect || ws.error()) {
        std::fprintf(stderr, "WRONG RESULT %s: %.17g vs %.17g (fan-in error %u)\n", v.name.c_str(), got, expect,
                     ws.error());
        return 3;
      }
    }
  }
  std::printf("n=%llu doubles (%.3f GB), grid %d, %u rounds, %d rounds x %d launches, hipEvent per launch\n",
              static_cast<unsigned long long>(n), n * 8e-9, grid, rounds_all, rounds, iters);
  std::printf("%-12s %10s %10s %10s %8s\n", "variant", "med us", "p10 us", "min us", "TB/s");
  for (size_t i = 0; i < vars.size(); ++i) {
    std::vector<double> v = ms[i];
    std::sort(v.begin(), v.end());
    const double med = v[v.size() / 2] * 1e3, p10 = v[v.size() / 10] * 1e3, mn = v[0] * 1e3;
    std::printf("%-12s %10.1f %10.1f %10.1f %8.3f\n", vars[i].name.c_str(), med, p10, mn, n * 8.0 / (med * 1e-6) / 1e12);
  }
  return 0;
}
