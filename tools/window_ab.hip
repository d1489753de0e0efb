// Production-kernel A/B of the streaming body's load schedule (profiles/r3_window/): hipcc's own
// schedule (WIN 0) against an explicit in-flight window of WIN loads per thread
// (reduce_kernels.hpp stream_window_seq), for the plans that matter at the headline sizes. The real
// kern::reduce_stream with the polled fan-in and a Workspace, hipEvent per launch, rounds
// interleaved in a shuffled order, median per variant; every launch's result is checked.
//   build: make window_ab        run: build/bin/window_ab [--n=1e9] [--rounds=7] [--iters=20] [--type=float]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
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

struct Var {
  const char* name;
  int block, unroll, wpc;
  void (*fn)(const kern::Args&, int, hipStream_t);
};

template <int B, int U, int W, class T = double>
Var mk(const char* name, int wpc) {
  return {name, B, U, wpc, detail::launch_stream<SumOp, T, double, B, U, true, W>};
}

// Control: the first window implementation (plain-pointer nontemporal loads, no sched_barrier
// between consume and load), a reduced copy of the kernel body without the fan-in epilogue: the
// partials go to a.partials and the result is folded by a second launch.
template <int BLOCK, int UNROLL, int WIN>
__global__ __launch_bounds__(BLOCK) void global_window(kern::Args a) {
  using V = kern::Vec16<double>::type;
  __shared__ double lds[BLOCK / 64];
  double acc[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) acc[u] = 0.0;
  const V* base = static_cast<const V*>(a.body) + threadIdx.x;
  constexpr uint64_t kTile = static_cast<uint64_t>(BLOCK) * UNROLL;
  const uint64_t ntiles = a.nvec / kTile, g = gridDim.x;
  uint64_t t = blockIdx.x;
  if (t < ntiles) {
    V buf[WIN];
#pragma unroll
    for (int j = 0; j < WIN; ++j) buf[j] = __builtin_nontemporal_load(base + t * kTile + j * BLOCK);
    for (; t + g < ntiles; t += g) {
      const V* p = base + t * kTile;
      const V* q = base + (t + g) * kTile;
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        acc[u] += buf[u % WIN][0] + buf[u % WIN][1];
        const int j = u + WIN;
        buf[u % WIN] = __builtin_nontemporal_load(j < UNROLL ? p + j * BLOCK : q + (j - UNROLL) * BLOCK);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const V* p = base + t * kTile;
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      acc[u] += buf[u % WIN][0] + buf[u % WIN][1];
      const int j = u + WIN;
      if (j < UNROLL) buf[u % WIN] = __builtin_nontemporal_load(p + j * BLOCK);
    }
  }
  const V* vin = static_cast<const V*>(a.body);
  for (uint64_t i = ntiles * kTile + blockIdx.x * BLOCK + threadIdx.x; i < a.nvec; i += g * BLOCK)
    acc[0] += vin[i][0] + vin[i][1];
#pragma unroll
  for (int u = 1; u < UNROLL; ++u) acc[0] += acc[u];
  const double v = kern::block_reduce<SumOp, double, BLOCK>(acc[0], lds);
  if (threadIdx.x == 0) static_cast<double*>(a.partials)[blockIdx.x] = v;
}

template <int B, int U, int W>
void launch_global_window(const kern::Args& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((global_window<B, U, W>), dim3(grid), dim3(B), 0, s, a);
  hipLaunchKernelGGL((kern::finalize<SumOp, double>), dim3(1), dim3(256), 0, s,
                     static_cast<const double*>(a.partials), static_cast<uint64_t>(grid), static_cast<double*>(a.out),
                     nullptr, nullptr, 0u);
}

template <int B, int U, int W>
Var mkg(const char* name, int wpc) {
  return {name, B, U, wpc, launch_global_window<B, U, W>};
}

// Control: the STRICT window (consume first, then issue the next load: at most WIN in flight) with
// the production buffer loads — the form the production body had as its WIN < 0 instantiation until
// round 6 (1-70 % slower than the loose window, profiles/r3_window/), kept here only. Interleaved
// tiles, partials + finalize like global_window.
template <int BLOCK, int UNROLL, int WIN>
__global__ __launch_bounds__(BLOCK) void strict_window(kern::Args a) {
  using V = kern::Vec16<double>::type;
  __shared__ double lds[BLOCK / 64];
  double acc[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) acc[u] = 0.0;
  const V* vin = static_cast<const V*>(a.body);
  constexpr uint64_t kTile = static_cast<uint64_t>(BLOCK) * UNROLL;
  constexpr uint32_t kStride = BLOCK * 16;
  const uint64_t ntiles = a.nvec / kTile, g = gridDim.x;
  const uint32_t voff = threadIdx.x * 16;
  uint64_t t = blockIdx.x;
  if (t < ntiles) {
    __amdgpu_buffer_rsrc_t rp = kern::tile_rsrc(vin + t * kTile);
    V buf[WIN];
#pragma unroll
    for (int j = 0; j < WIN; ++j) buf[j] = kern::ld_buf_nt<V>(rp, voff, j * kStride);
    for (; t + g < ntiles; t += g) {
      const __amdgpu_buffer_rsrc_t rq = kern::tile_rsrc(vin + (t + g) * kTile);
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        acc[u] += buf[u % WIN][0] + buf[u % WIN][1];
        __builtin_amdgcn_sched_barrier(0);  // strict: the consume completes before the next load issues
        const int j = u + WIN;
        buf[u % WIN] = j < UNROLL ? kern::ld_buf_nt<V>(rp, voff, j * kStride)
                                  : kern::ld_buf_nt<V>(rq, voff, (j - UNROLL) * kStride);
        __builtin_amdgcn_sched_barrier(0);
      }
      rp = rq;
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      acc[u] += buf[u % WIN][0] + buf[u % WIN][1];
      const int j = u + WIN;
      if (j < UNROLL) buf[u % WIN] = kern::ld_buf_nt<V>(rp, voff, j * kStride);
    }
  }
  for (uint64_t i = ntiles * kTile + blockIdx.x * BLOCK + threadIdx.x; i < a.nvec; i += g * BLOCK)
    acc[0] += vin[i][0] + vin[i][1];
#pragma unroll
  for (int u = 1; u < UNROLL; ++u) acc[0] += acc[u];
  const double v = kern::block_reduce<SumOp, double, BLOCK>(acc[0], lds);
  if (threadIdx.x == 0) static_cast<double*>(a.partials)[blockIdx.x] = v;
}

template <int B, int U, int W>
void launch_strict_window(const kern::Args& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((strict_window<B, U, W>), dim3(grid), dim3(B), 0, s, a);
  hipLaunchKernelGGL((kern::finalize<SumOp, double>), dim3(1), dim3(256), 0, s,
                     static_cast<const double*>(a.partials), static_cast<uint64_t>(grid), static_cast<double*>(a.out),
                     nullptr, nullptr, 0u);
}

template <int B, int U, int W>
Var mks(const char* name, int wpc) {
  return {name, B, U, wpc, launch_strict_window<B, U, W>};
}

template <class T>
__global__ void fill(T* x, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    x[i] = static_cast<T>(i & 1023);  // exact sums (fp64 accumulation)
}

int main(int argc, char** argv) {
  uint64_t n = 1000000000ull;
  int rounds = 7, iters = 20;
  bool f32 = false;
  for (int i = 1; i < argc; ++i) {
    if (!std::strncmp(argv[i], "--n=", 4)) n = static_cast<uint64_t>(std::atof(argv[i] + 4));
    else if (!std::strncmp(argv[i], "--rounds=", 9)) rounds = std::atoi(argv[i] + 9);
    else if (!std::strncmp(argv[i], "--iters=", 8)) iters = std::atoi(argv[i] + 8);
    else if (!std::strcmp(argv[i], "--type=float")) f32 = true;
  }
  const size_t es = f32 ? 4 : 8;
  // l<D>: buffer loads, D registers, the next load issued before the consume (D + 1 in flight at
  // issue; the production window, template WIN = D); w<D>: strict, consume first (strict_window);
  // g<D>: the first (plain-pointer) window, control.
  std::vector<Var> vars64 = {
      mk<256, 8, 0>("256x8x1 hipcc", 1),  mk<256, 2, 0>("256x2x3 hipcc", 3),  mk<512, 16, 0>("512x16x1 hipcc", 1),
      mk<256, 8, 4>("256x8x1 l4", 1),     mk<256, 8, 8>("256x8x1 l8", 1),     mk<256, 8, 2>("256x8x1 l2", 1),
      mk<256, 4, 2>("256x4x2 l2", 2),     mk<256, 4, 4>("256x4x2 l4", 2),     mk<256, 4, 2>("256x4x3 l2", 3),
      mk<512, 8, 2>("512x8x1 l2", 1),     mk<512, 8, 4>("512x8x1 l4", 1),     mk<512, 4, 2>("512x4x1 l2", 1),
      mk<256, 8, 2>("256x8x2 l2", 2),     mk<256, 8, 4>("256x8x2 l4", 2),     mkg<256, 4, 2>("256x4x2 g2", 2),
      mks<256, 8, 4>("256x8x1 w4", 1),    mks<256, 8, 8>("256x8x1 w8", 1),
  };  std::vector<Var> vars32 = {
      mk<512, 4, 0, float>("f32 512x4x1 hipcc", 1), mk<256, 2, 0, float>("f32 256x2x3 hipcc", 3),
      mk<256, 8, 0, float>("f32 256x8x1 hipcc", 1),
      mk<512, 4, 2, float>("f32 512x4x1 l2", 1),   mk<512, 4, 4, float>("f32 512x4x1 l4", 1),
      mk<256, 8, 4, float>("f32 256x8x1 l4", 1),   mk<256, 4, 2, float>("f32 256x4x2 l2", 2),
      mk<512, 8, 4, float>("f32 512x8x1 l4", 1),   mk<256, 8, 2, float>("f32 256x8x2 l2", 2),
  };
  std::vector<Var>& vars = f32 ? vars32 : vars64;


  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  void* x;
  double* out;
  CK(hipMalloc(&x, n * es));
  CK(hipMalloc(&out, 8));
  if (f32) fill<float><<<4096, 256>>>(static_cast<float*>(x), n);
  else fill<double><<<4096, 256>>>(static_cast<double*>(x), n);
  CK(hipDeviceSynchronize());
  // closed form of sum(i & 1023)
  const uint64_t full = n / 1024, rem = n % 1024;
  const double expect = static_cast<double>(full) * (1023.0 * 1024.0 / 2.0) + static_cast<double>(rem) * (rem - 1) / 2.0;
  Workspace ws(0);
  auto args_for = [&](const Var& v, int& grid) {
    ReduceConfig c;
    c.block = v.block;
    c.unroll = v.unroll;
    c.wg_per_cu = v.wpc;
    LaunchPlan p = plan_reduce(x, n, f32 ? DType::Float32 : DType::Float64, c, ws.num_cus(), ws.max_grid());
    kern::Args a{};
    a.head_ptr = x;
    a.body = x;
    a.head = p.head;
    a.nvec = p.nvec;
    a.tail = p.tail;
    a.partials = ws.partials();
    a.out = out;
    a.slots = ws.slots();
    a.fan = ws.fan();
    a.fan_bound = kern::kFanBoundTicks;
    a.delay_wg = -1;
    grid = p.grid;
    return a;
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> ms(vars.size());
  for (int r = 0; r < rounds; ++r) {
    std::vector<size_t> order(vars.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::srand(r + 11);
    for (size_t i = order.size(); i > 1; --i) std::swap(order[i - 1], order[std::rand() % i]);
    for (size_t i : order) {
      int grid = 0;
      const kern::Args a = args_for(vars[i], grid);
      vars[i].fn(a, grid, 0);  // warm-up
      for (int it = 0; it < iters; ++it) {
        CK(hipEventRecord(e0));
        vars[i].fn(a, grid, 0);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms[i].push_back(t);
      }
      double got = 0;
      CK(hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost));
      if (got != expect || ws.error()) {
        std::fprintf(stderr, "WRONG RESULT %s: %.17g vs %.17g (fan-in error %u)\n", vars[i].name, got, expect, ws.error());
        return 3;
      }
    }
  }
  std::printf("n=%llu %s (%.3f GB), %d CUs, %d rounds x %d launches, hipEvent per launch\n",
              static_cast<unsigned long long>(n), f32 ? "floats" : "doubles", n * es * 1e-9, cus, rounds, iters);
  std::printf("%-18s %10s %10s %10s %8s\n", "variant", "med us", "p10 us", "min us", "TB/s");
  for (size_t i = 0; i < vars.size(); ++i) {
    std::vector<double> v = ms[i];
    std::sort(v.begin(), v.end());
    const double med = v[v.size() / 2] * 1e3, p10 = v[v.size() / 10] * 1e3, mn = v[0] * 1e3;
    std::printf("%-18s %10.1f %10.1f %10.1f %8.3f\n", vars[i].name, med, p10, mn, n * double(es) / (med * 1e-6) / 1e12);
  }
  return 0;
}
