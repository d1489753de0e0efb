// Fused multi-statistic reduction: one streaming pass computes Σ(x-K), Σ(x-K)², min and max
// (K = x[0], the shifted-data algorithm, so the variance does not cancel catastrophically when
// |mean| >> std). Pattern reference: the fused Σx / Σx² tree of the vendored MonteCarlo sample
// (cuda/C/src/MonteCarlo/MonteCarlo_reduction.cuh:20-38,47-63), SURVEY.md §2.4.
//
// Same streaming structure as reduce_stream (16-byte nt loads, UNROLL loads in flight, wave64
// butterflies); four accumulators per lane. Two launches: per-workgroup partials (4 doubles),
// then one workgroup folds them — the partial block is only 32 B x grid.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "mireduce/check.hpp"
#include "mireduce/half.hpp"
#include "mireduce/moments.hpp"
#include "mireduce/ops.hpp"
#include "mireduce/vec16.hpp"

namespace mireduce {
namespace kern {

struct Mom {
  double s, q, mn, mx;
};

__device__ __forceinline__ Mom mom_combine(Mom a, Mom b) {
  return {a.s + b.s, a.q + b.q, MinOp::apply(a.mn, b.mn), MaxOp::apply(a.mx, b.mx)};
}

__device__ __forceinline__ Mom mom_shfl(Mom v, int off) {
  return {__shfl_xor(v.s, off, 64), __shfl_xor(v.q, off, 64), __shfl_xor(v.mn, off, 64), __shfl_xor(v.mx, off, 64)};
}

template <int BLOCK>
__device__ __forceinline__ Mom block_mom(Mom v, Mom* lds) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = mom_combine(v, mom_shfl(v, off));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  if (wave == 0) {
    const Mom id{0.0, 0.0, MinOp::identity<double>(), MaxOp::identity<double>()};
    v = lane < BLOCK / 64 ? lds[lane] : id;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = mom_combine(v, mom_shfl(v, off));
  }
  return v;
}

template <class T>
__device__ __forceinline__ double first_value(const void* p) {
  return static_cast<double>(*static_cast<const T*>(p));
}

// One element: shifted Σ and Σ² in fp64; MIN/MAX in the narrowest exact type E (fp32 for fp32 /
// bf16 / f16 storage, which halves the fp64 VALU work per element: 6.4-6.7 TB/s -> see
// profiles/r1_session3/moments_bw.jsonl), widened to fp64 only when the partials are combined.
template <class E>
__device__ __forceinline__ void mom_step(E x, double K, double& s, double& q, E& mn, E& mx) {
  const double d = static_cast<double>(x) - K;
  s += d;
  q = __builtin_fma(d, d, q);
  mn = MinOp::apply(mn, x);
  mx = MaxOp::apply(mx, x);
}

template <class T, int BLOCK, int UNROLL>
__global__ __launch_bounds__(BLOCK) void moments_stream(const T* __restrict__ in, uint64_t n, Mom* __restrict__ partials) {
  using V = typename Vec16<T>::type;
  using E = std::conditional_t<std::is_same_v<T, double>, double, float>;
  constexpr int N = Vec16<T>::N;
  __shared__ Mom lds[BLOCK / 64];
  const double K = n ? static_cast<double>(in[0]) : 0.0;
  double s[UNROLL], q[UNROLL];
  E mn[UNROLL], mx[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    s[u] = 0.0;
    q[u] = 0.0;
    mn[u] = MinOp::identity<E>();
    mx[u] = MaxOp::identity<E>();
  }
  const uint64_t nvec = n / N;
  const V* vin = reinterpret_cast<const V*>(in);
  constexpr uint64_t kTile = static_cast<uint64_t>(BLOCK) * UNROLL;
  const uint64_t ntiles = nvec / kTile;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const V* p = vin + t * kTile + threadIdx.x;
    V v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(p + u * BLOCK);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
      for (int k = 0; k < N; ++k) mom_step<E>(elem<T, E>(v[u], k), K, s[u], q[u], mn[u], mx[u]);
    }
  }
  // remaining vectors, then the < N scalar tail (input is 16-byte aligned: checked on the host)
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * BLOCK;
  for (uint64_t i = ntiles * kTile + static_cast<uint64_t>(blockIdx.x) * BLOCK + threadIdx.x; i < nvec; i += stride) {
    const V v = vin[i];
#pragma unroll
    for (int k = 0; k < N; ++k) mom_step<E>(elem<T, E>(v, k), K, s[0], q[0], mn[0], mx[0]);
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x < n - nvec * N)
    mom_step<E>(static_cast<E>(in[nvec * N + threadIdx.x]), K, s[0], q[0], mn[0], mx[0]);
  Mom m{s[0], q[0], static_cast<double>(mn[0]), static_cast<double>(mx[0])};
#pragma unroll
  for (int u = 1; u < UNROLL; ++u)
    m = mom_combine(m, Mom{s[u], q[u], static_cast<double>(mn[u]), static_cast<double>(mx[u])});
  m = block_mom<BLOCK>(m, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = m;
}

template <class T>
__global__ __launch_bounds__(256) void moments_finalize(const Mom* __restrict__ partials, int count,
                                                        const void* __restrict__ first, uint64_t n,
                                                        double* __restrict__ out) {
  __shared__ Mom lds[4];
  Mom m{0.0, 0.0, MinOp::identity<double>(), MaxOp::identity<double>()};
  for (int i = threadIdx.x; i < count; i += 256) m = mom_combine(m, partials[i]);
  m = block_mom<256>(m, lds);
  if (threadIdx.x == 0) {
    double K = 0.0;
    if (n) K = first_value<T>(first);
    out[0] = K;
    out[1] = m.s;
    out[2] = m.q;
    out[3] = m.mn;
    out[4] = m.mx;
  }
}

}  // namespace kern

namespace {
template <class T>
void launch_moments(const void* in, size_t n, double* out5, kern::Mom* p, int max_grid, int num_cus, hipStream_t stream) {
  constexpr int kBlock = 256, kUnroll = 4;
  constexpr size_t vec = kern::Vec16<T>::N;
  const uint64_t tiles = (n / vec + kBlock * kUnroll - 1) / (kBlock * kUnroll);
  int grid = static_cast<int>(std::min<uint64_t>(std::max<uint64_t>(tiles, 1), static_cast<uint64_t>(num_cus) * 3));
  grid = std::min(grid, max_grid);
  hipLaunchKernelGGL((kern::moments_stream<T, kBlock, kUnroll>), dim3(grid), dim3(kBlock), 0, stream,
                     static_cast<const T*>(in), static_cast<uint64_t>(n), p);
  MIREDUCE_HIP_THROW(hipGetLastError());
  hipLaunchKernelGGL(kern::moments_finalize<T>, dim3(1), dim3(256), 0, stream, p, grid, in, static_cast<uint64_t>(n), out5);
  MIREDUCE_HIP_THROW(hipGetLastError());
}
}  // namespace

void moments_device(const void* in, size_t n, DType t, double* out5, void* partials, int max_grid, int num_cus,
                    hipStream_t stream) {
  MIREDUCE_REQUIRE(dtype_is_float(t), "moments: float32, float64, bfloat16 or float16 input");
  MIREDUCE_REQUIRE(reinterpret_cast<uintptr_t>(in) % 16 == 0, "moments: input must be 16-byte aligned");
  auto* p = static_cast<kern::Mom*>(partials);
  switch (t) {
    case DType::Float64: launch_moments<double>(in, n, out5, p, max_grid, num_cus, stream); break;
    case DType::Float32: launch_moments<float>(in, n, out5, p, max_grid, num_cus, stream); break;
    case DType::BFloat16: launch_moments<bf16_t>(in, n, out5, p, max_grid, num_cus, stream); break;
    case DType::Float16: launch_moments<f16_t>(in, n, out5, p, max_grid, num_cus, stream); break;
    default: break;
  }
}

size_t moments_partials_bytes(int max_grid) { return static_cast<size_t>(max_grid) * sizeof(kern::Mom); }

}  // namespace mireduce
