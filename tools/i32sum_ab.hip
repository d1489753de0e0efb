// Experiment (round 4, not the production path): int32 SUM into int64 with less VALU work.
// The production body sign-extends every element and adds it in 64 bits (v_ashrrev + v_mov +
// v_lshl_add_u64: 3 ops per element); with the window-4 plan at one workgroup per CU that VALU
// work starves the stream, so int32 SUM runs the window-2 plan at two workgroups per CU, ~1.3 %
// behind the other types (docs/TUNING.md, "Open leads"). Here each element x = hi * 2^16 + lo is
// split by two dot2 instructions into 32-bit sums of its unsigned low halves (v_dot2_u32_u16
// against (1, 0)) and signed high halves (v_dot2_i32_i16 against (0, 1)): 2 ops per element, no
// carries, exact while a thread's halves sum below 2^31 (16384 tiles of 8 vectors per slot; the
// host checks), folded into int64 once at the end. Same box, interleaved rounds, hipEvent per
// launch, every result exact:
//   prod w2x2   the production plan (256 x 8, window 2, 2 workgroups per CU, polled fan-in)
//   prod w4x1   the production body with the window-4 plan at 1 workgroup per CU
//   dot2 w4x1   this kernel, 256 x 8, window 4, 1 workgroup per CU (partials folded on the host)
//   build: make i32sum_ab      run: build/bin/i32sum_ab [--n=2e9] [--rounds=5] [--iters=20]
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

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void add_halves(uint32_t& lo, int32_t& hi, int32_t x) {
  const u16x2 xu = __builtin_bit_cast(u16x2, x);
  const i16x2 xs = __builtin_bit_cast(i16x2, x);
  lo = __builtin_amdgcn_udot2(xu, u16x2{1, 0}, lo, false);
  hi = __builtin_amdgcn_sdot2(xs, i16x2{0, 1}, hi, false);
}

// Tiles of workgroup b: the weighted split by blockIdx parity (this tool launches on the null
// stream, where XCC = b % 8): `ra` common rounds, `dd` more for the odd workgroups, then the
// leftover (< grid tiles) one each, odd workgroups first. dd = 0: plain interleaved rounds.
template <int BLOCK, int UNROLL, int WIN>
__global__ __launch_bounds__(BLOCK) void i32sum_dot2(const int32_t* __restrict__ x, uint64_t nvec, uint32_t ra,
                                                     uint32_t dd, int64_t* partials) {
  using V = kern::Vec16<int32_t>::type;  // 4 x int32
  __shared__ int64_t lds[BLOCK / 64];
  uint32_t lo[UNROLL];
  int32_t hi[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) lo[u] = 0, hi[u] = 0;
  const V* vin = reinterpret_cast<const V*>(x);
  constexpr uint64_t kTile = static_cast<uint64_t>(BLOCK) * UNROLL;
  constexpr uint32_t kStride = BLOCK * 16;
  const uint32_t voff = threadIdx.x * 16;
  const uint32_t ntiles = static_cast<uint32_t>(nvec / kTile), grid = gridDim.x, half = grid / 2, b = blockIdx.x;
  const bool fav = (b & 1u) != 0 && dd > 0;
  const uint32_t base2 = ra * grid + dd * half, rank2 = dd == 0 ? b : (fav ? (b >> 1) : half + (b >> 1));
  const uint32_t n_tiles = ra + (fav ? dd : 0u) + (base2 + rank2 < ntiles ? 1u : 0u);
  auto tile_of = [&](uint32_t i) -> uint32_t {  // i-th tile of this workgroup (scalar arithmetic)
    if (i < ra) return b + i * grid;
    if (fav && i < ra + dd) return ra * grid + (b >> 1) + (i - ra) * half;
    return base2 + rank2;
  };
  uint32_t t = tile_of(0);
  if (n_tiles > 0) {
    __amdgpu_buffer_rsrc_t rp = kern::tile_rsrc(vin + static_cast<uint64_t>(t) * kTile);
    V buf[WIN];
#pragma unroll
    for (int j = 0; j < WIN; ++j) buf[j] = kern::ld_buf_nt<V>(rp, voff, j * kStride);
#pragma nounroll
    for (uint32_t i = 1; i < n_tiles; ++i) {
      t = __builtin_amdgcn_readfirstlane(tile_of(i));
      const __amdgpu_buffer_rsrc_t rq = kern::tile_rsrc(vin + static_cast<uint64_t>(t) * kTile);
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
        for (int k = 0; k < 4; ++k) add_halves(lo[u], hi[u], buf[u % WIN][k]);
        const int j = u + WIN;
        buf[u % WIN] = j < UNROLL ? kern::ld_buf_nt<V>(rp, voff, j * kStride)
                                  : kern::ld_buf_nt<V>(rq, voff, (j - UNROLL) * kStride);
        __builtin_amdgcn_sched_barrier(0);
      }
      rp = rq;
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
      for (int k = 0; k < 4; ++k) add_halves(lo[u], hi[u], buf[u % WIN][k]);
      const int j = u + WIN;
      if (j < UNROLL) buf[u % WIN] = kern::ld_buf_nt<V>(rp, voff, j * kStride);
    }
  }
  int64_t acc = 0;
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) acc += static_cast<int64_t>(hi[u]) * 65536 + static_cast<int64_t>(lo[u]);
  for (uint64_t i = static_cast<uint64_t>(ntiles) * kTile + blockIdx.x * BLOCK + threadIdx.x; i < nvec;
       i += static_cast<uint64_t>(grid) * BLOCK)
    for (int k = 0; k < 4; ++k) acc += vin[i][k];
  const int64_t v = kern::block_reduce<SumOp, int64_t, BLOCK>(acc, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = v;
}

__global__ void fill(int32_t* x, uint64_t n) {  // full-range values: both halves vary, signs mixed
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z ^= z >> 29;
    x[i] = static_cast<int32_t>(static_cast<uint32_t>(z * 0xBF58476D1CE4E5B9ull >> 32));
  }
}

int main(int argc, char** argv) {
  uint64_t n = 2000000000ull;
  int rounds = 5, iters = 20;
  for (int i = 1; i < argc; ++i) {
    if (!std::strncmp(argv[i], "--n=", 4)) n = static_cast<uint64_t>(std::atof(argv[i] + 4));
    else if (!std::strncmp(argv[i], "--rounds=", 9)) rounds = std::atoi(argv[i] + 9);
    else if (!std::strncmp(argv[i], "--iters=", 8)) iters = std::atoi(argv[i] + 8);
  }
  if (n % 4) {
    std::fprintf(stderr, "--n must be a multiple of 4\n");
    return 2;
  }
  constexpr int B = 256, U = 8;
  int32_t* x;
  int64_t* out;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&out, 8));
  fill<<<4096, 256>>>(x, n);
  CK(hipDeviceSynchronize());
  std::vector<int32_t> h(n);
  CK(hipMemcpy(h.data(), x, n * 4, hipMemcpyDeviceToHost));
  int64_t expect = 0;
  for (int32_t v : h) expect += v;
  std::vector<int32_t>().swap(h);
  Workspace ws(0);
  const uint64_t nvec = n / 4, ntiles = nvec / (B * U);
  const int cus = ws.num_cus();
  if (ntiles / cus >= 16384) {
    std::fprintf(stderr, "array too large for the unflushed 32-bit halves (%llu tiles per workgroup)\n",
                 static_cast<unsigned long long>(ntiles / cus));
    return 2;
  }
  struct Var {
    std::string name;
    int kind;  // 0: prod window 2 x 2 WG/CU, 1: prod window 4 x 1, 2: dot2 window 4 x 1; 3/4: 1/2 + skew 20
  };
  std::vector<Var> vars = {{"prod w2x2", 0}, {"prod w4x1", 1}, {"dot2 w4x1", 2}, {"prod w4x1 s20", 3},
                           {"dot2 w4x1 s20", 4}};
  const uint32_t kSkew = static_cast<uint32_t>((ntiles / cus * 20 + 500) / 1000);  // 20 permille of the rounds
  auto prod_args = [&](int grid, uint32_t skew = 0) {
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
    a.x_ra = ntiles / grid;  // equal rounds (the production default for int32 SUM)
    if (skew) {              // the anchored weighted split (polled: the fan-in epoch tags the anchor)
      a.xskew = static_cast<int>(skew);
      a.x_ra = (ntiles - static_cast<uint64_t>(skew) * (grid / 2)) / grid;
      a.x_dd = skew;
    }
    return a;
  };
  int64_t* dpart;
  CK(hipMalloc(&dpart, cus * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> ms(vars.size());
  for (int r = 0; r < rounds; ++r) {
    std::vector<size_t> order(vars.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::srand(r + 3);
    for (size_t i = order.size(); i > 1; --i) std::swap(order[i - 1], order[std::rand() % i]);
    for (size_t i : order) {
      const Var& v = vars[i];
      auto launch = [&]() {
        if (v.kind == 0)
          detail::launch_stream<SumOp, int32_t, int64_t, B, U, true, 2>(prod_args(2 * cus), 2 * cus, 0);
        else if (v.kind == 1)
          detail::launch_stream<SumOp, int32_t, int64_t, B, U, true, 4>(prod_args(cus), cus, 0);
        else if (v.kind == 3)
          detail::launch_stream<SumOp, int32_t, int64_t, B, U, true, 4>(prod_args(cus, kSkew), cus, 0);
        else {
          const uint32_t dd = v.kind == 4 ? kSkew : 0u;
          const uint32_t ra = static_cast<uint32_t>((ntiles - static_cast<uint64_t>(dd) * (cus / 2)) / cus);
          hipLaunchKernelGGL((i32sum_dot2<B, U, 4>), dim3(cus), dim3(B), 0, 0, x, nvec, ra, dd, dpart);
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
      int64_t got = 0;
      if (v.kind != 2 && v.kind != 4) {
        CK(hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost));
      } else {
        std::vector<int64_t> p(cus);
        CK(hipMemcpy(p.data(), dpart, cus * 8, hipMemcpyDeviceToHost));
        for (int64_t q : p) got += q;
      }
      if (got != expect || ws.error()) {
        std::fprintf(stderr, "WRONG RESULT %s: %lld vs %lld (fan-in error %u)\n", v.name.c_str(),
                     static_cast<long long>(got), static_cast<long long>(expect), ws.error());
        return 3;
      }
    }
  }
  std::printf("n=%llu int32 (%.3f GB), %d CUs, %d rounds x %d launches, hipEvent per launch\n",
              static_cast<unsigned long long>(n), n * 4e-9, cus, rounds, iters);
  std::printf("%-12s %10s %10s %10s %8s\n", "variant", "med us", "p10 us", "min us", "TB/s");
  for (size_t i = 0; i < vars.size(); ++i) {
    std::vector<double> v = ms[i];
    std::sort(v.begin(), v.end());
    const double med = v[v.size() / 2] * 1e3, p10 = v[v.size() / 10] * 1e3, mn = v[0] * 1e3;
    std::printf("%-12s %10.1f %10.1f %10.1f %8.3f\n", vars[i].name.c_str(), med, p10, mn, n * 4.0 / (med * 1e-6) / 1e12);
  }
  return 0;
}
