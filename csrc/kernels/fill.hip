// On-device synthetic data generation (SURVEY.md §2.2 C14 → kernels/fill.hip).
//
// The reference fills host memory with rand()&0xFF (reduction.cpp:698-705) or MT19937
// (reduce.c:51-57) and copies it to the device. At 288 GB per GPU that is hours of host time,
// so here every element is generated in place from (seed, global index) — see rng.hpp — with
// 16-byte stores; fill_host produces the identical values for verification.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mireduce/check.hpp"
#include "mireduce/reduce.hpp"
#include "mireduce/rng.hpp"

namespace mireduce {
namespace kern {

template <class T>
__global__ __launch_bounds__(256) void fill_kernel(T* __restrict__ out, uint64_t n, FillSpec s) {
  constexpr int N = 16 / sizeof(T);
  using V = T __attribute__((ext_vector_type(N)));
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  const uint64_t nvec = n / N;
  V* vout = reinterpret_cast<V*>(out);
  for (uint64_t i = tid; i < nvec; i += stride) {
    V v;
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = pattern_value<T>(s.pattern, s.seed, s.offset + i * N + k, s.value);
    __builtin_nontemporal_store(v, vout + i);
  }
  for (uint64_t i = nvec * N + tid; i < n; i += stride)
    out[i] = pattern_value<T>(s.pattern, s.seed, s.offset + i, s.value);
}

template <class T>
__global__ __launch_bounds__(256) void fill_kernel_scalar(T* __restrict__ out, uint64_t n, FillSpec s) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride)
    out[i] = pattern_value<T>(s.pattern, s.seed, s.offset + i, s.value);
}

// 16-bit floats: eight 2-byte patterns per 16-byte store.
template <class H>
__global__ __launch_bounds__(256) void fill_kernel_half(uint16_t* __restrict__ out, uint64_t n, FillSpec s) {
  using V = uint16_t __attribute__((ext_vector_type(8)));
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  const uint64_t nvec = reinterpret_cast<uintptr_t>(out) % 16 == 0 ? n / 8 : 0;
  V* vout = reinterpret_cast<V*>(out);
  for (uint64_t i = tid; i < nvec; i += stride) {
    V v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = pattern_half_bits<H>(s.pattern, s.seed, s.offset + i * 8 + k, s.value);
    __builtin_nontemporal_store(v, vout + i);
  }
  for (uint64_t i = nvec * 8 + tid; i < n; i += stride) out[i] = pattern_half_bits<H>(s.pattern, s.seed, s.offset + i, s.value);
}

}  // namespace kern

namespace {
template <class T>
void launch_fill(void* ptr, size_t n, const FillSpec& s, hipStream_t st) {
  if (n == 0) return;
  uint64_t blocks = (n / (16 / sizeof(T)) + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 8192) blocks = 8192;
  if (reinterpret_cast<uintptr_t>(ptr) % 16 == 0)
    hipLaunchKernelGGL(kern::fill_kernel<T>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st,
                       static_cast<T*>(ptr), static_cast<uint64_t>(n), s);
  else
    hipLaunchKernelGGL(kern::fill_kernel_scalar<T>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       st, static_cast<T*>(ptr), static_cast<uint64_t>(n), s);
}

template <class H>
void launch_fill_half(void* ptr, size_t n, const FillSpec& s, hipStream_t st) {
  if (n == 0) return;
  uint64_t blocks = (n / 8 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(kern::fill_kernel_half<H>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st,
                     static_cast<uint16_t*>(ptr), static_cast<uint64_t>(n), s);
}

template <class H>
void host_fill_half(void* ptr, size_t n, const FillSpec& s) {
  uint16_t* p = static_cast<uint16_t*>(ptr);
  for (size_t i = 0; i < n; ++i) p[i] = pattern_half_bits<H>(s.pattern, s.seed, s.offset + i, s.value);
}

template <class T>
void host_fill(void* ptr, size_t n, const FillSpec& s) {
  T* p = static_cast<T*>(ptr);
  for (size_t i = 0; i < n; ++i) p[i] = pattern_value<T>(s.pattern, s.seed, s.offset + i, s.value);
}
}  // namespace

void fill_device(void* ptr, size_t n, DType t, const FillSpec& spec, hipStream_t stream) {
  switch (t) {
    case DType::Int32: launch_fill<int32_t>(ptr, n, spec, stream); break;
    case DType::Int64: launch_fill<int64_t>(ptr, n, spec, stream); break;
    case DType::Float32: launch_fill<float>(ptr, n, spec, stream); break;
    case DType::Float64: launch_fill<double>(ptr, n, spec, stream); break;
    case DType::BFloat16: launch_fill_half<bf16_t>(ptr, n, spec, stream); break;
    case DType::Float16: launch_fill_half<f16_t>(ptr, n, spec, stream); break;
  }
  MIREDUCE_HIP_THROW(hipGetLastError());
}

void fill_host(void* ptr, size_t n, DType t, const FillSpec& spec) {
  switch (t) {
    case DType::Int32: host_fill<int32_t>(ptr, n, spec); break;
    case DType::Int64: host_fill<int64_t>(ptr, n, spec); break;
    case DType::Float32: host_fill<float>(ptr, n, spec); break;
    case DType::Float64: host_fill<double>(ptr, n, spec); break;
    case DType::BFloat16: host_fill_half<bf16_t>(ptr, n, spec); break;
    case DType::Float16: host_fill_half<f16_t>(ptr, n, spec); break;
  }
}

}  // namespace mireduce
