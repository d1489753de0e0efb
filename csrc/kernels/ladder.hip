// Harris-whitepaper reduction ladder (kernels 0..6) for gfx950 wave64; see ladder.hpp.
//
// Mapping to the reference / whitepaper (cuda/C/src/reduction/doc/reduction.pdf):
//   k0  p.7-10  interleaved addressing, divergent `tid % (2s)` branch
//   k1  p.11-13 interleaved addressing, strided index (LDS bank conflicts)
//   k2  p.14-16 sequential addressing
//   k3  p.17-19 first add during global load (half the blocks)
//   k4  p.20-23 unroll the last wave — here a 64-lane __shfl_xor butterfly, not the 32-lane
//               volatile-LDS lockstep of reduction_kernel.cu:110-122 (wrong on CDNA)
//   k5  p.24-28 completely unrolled tree (template BLOCK)
//   k6  p.29-34 multiple elements per thread, grid-stride, fixed grid — the reference's kernel 6
//               (sumreduce6/minreduce6/maxreduce6, reduction_kernel.cu:74-253) with the correct
//               pair guard `i + BLOCK < n` (bug B1) and identity init (bug B2)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mireduce/check.hpp"
#include "mireduce/ladder.hpp"
#include "mireduce/ops.hpp"

namespace mireduce {
namespace ladder {

// Butterfly over the first `width` lanes (a power of two <= 64): lane l only ever reads lane
// l ^ off < width, so a block of fewer than 64 threads (the reference accepts --threads down to 1,
// reduction.cpp:272-291) never reads an inactive lane.
template <class OpT, class AccT>
__device__ __forceinline__ AccT wave_tail(AccT v, unsigned width = 64) {
#pragma unroll
  for (unsigned off = 32; off > 0; off >>= 1)
    if (off < width) v = OpT::apply(v, __shfl_xor(v, off, 64));
  return v;
}

template <class AccT>
__device__ __forceinline__ AccT* lds_array() {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  return reinterpret_cast<AccT*>(smem_raw);
}

// k0..k2: one element per thread, LDS tree over the whole block.
template <int K, class OpT, class Tin, class AccT>
__global__ void k012(const Tin* __restrict__ in, uint64_t n, AccT* __restrict__ out) {
  AccT* sdata = lds_array<AccT>();
  const unsigned tid = threadIdx.x;
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + tid;
  sdata[tid] = i < n ? static_cast<AccT>(in[i]) : OpT::template identity<AccT>();
  __syncthreads();
  if constexpr (K == 0) {
    for (unsigned s = 1; s < blockDim.x; s *= 2) {
      if (tid % (2 * s) == 0) sdata[tid] = OpT::apply(sdata[tid], sdata[tid + s]);
      __syncthreads();
    }
  } else if constexpr (K == 1) {
    for (unsigned s = 1; s < blockDim.x; s *= 2) {
      const unsigned index = 2 * s * tid;
      if (index < blockDim.x) sdata[index] = OpT::apply(sdata[index], sdata[index + s]);
      __syncthreads();
    }
  } else {
    for (unsigned s = blockDim.x / 2; s > 0; s >>= 1) {
      if (tid < s) sdata[tid] = OpT::apply(sdata[tid], sdata[tid + s]);
      __syncthreads();
    }
  }
  if (tid == 0) out[blockIdx.x] = sdata[0];
}

// k3/k4: two elements per thread at load; k4 finishes the last 64 values with shuffles.
template <int K, class OpT, class Tin, class AccT>
__global__ void k34(const Tin* __restrict__ in, uint64_t n, AccT* __restrict__ out) {
  AccT* sdata = lds_array<AccT>();
  const unsigned tid = threadIdx.x;
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * (blockDim.x * 2) + tid;
  AccT v = i < n ? static_cast<AccT>(in[i]) : OpT::template identity<AccT>();
  if (i + blockDim.x < n) v = OpT::apply(v, static_cast<AccT>(in[i + blockDim.x]));
  sdata[tid] = v;
  __syncthreads();
  if constexpr (K == 3) {
    for (unsigned s = blockDim.x / 2; s > 0; s >>= 1) {
      if (tid < s) sdata[tid] = OpT::apply(sdata[tid], sdata[tid + s]);
      __syncthreads();
    }
    if (tid == 0) out[blockIdx.x] = sdata[0];
  } else {
    for (unsigned s = blockDim.x / 2; s > 64; s >>= 1) {
      if (tid < s) sdata[tid] = OpT::apply(sdata[tid], sdata[tid + s]);
      __syncthreads();
    }
    if (tid < 64) {
      v = sdata[tid];
      if (blockDim.x >= 128) v = OpT::apply(v, sdata[tid + 64]);
      v = wave_tail<OpT>(v, blockDim.x < 64 ? blockDim.x : 64);
      if (tid == 0) out[blockIdx.x] = v;
    }
  }
}

// Unrolled block tree from BLOCK values in LDS to one value, last wave by shuffles.
template <int BLOCK, class OpT, class AccT>
__device__ __forceinline__ void unrolled_tail(AccT* sdata, AccT v, AccT* out) {
  const unsigned tid = threadIdx.x;
  if constexpr (BLOCK >= 1024) { if (tid < 512) sdata[tid] = v = OpT::apply(v, sdata[tid + 512]); __syncthreads(); }
  if constexpr (BLOCK >= 512) { if (tid < 256) sdata[tid] = v = OpT::apply(v, sdata[tid + 256]); __syncthreads(); }
  if constexpr (BLOCK >= 256) { if (tid < 128) sdata[tid] = v = OpT::apply(v, sdata[tid + 128]); __syncthreads(); }
  if (tid < 64) {
    if constexpr (BLOCK >= 128) v = OpT::apply(v, sdata[tid + 64]);
    v = wave_tail<OpT>(v, BLOCK < 64 ? BLOCK : 64);
    if (tid == 0) out[blockIdx.x] = v;
  }
}

template <int BLOCK, class OpT, class Tin, class AccT>
__global__ __launch_bounds__(BLOCK) void k5(const Tin* __restrict__ in, uint64_t n, AccT* __restrict__ out) {
  AccT* sdata = lds_array<AccT>();
  const unsigned tid = threadIdx.x;
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * (BLOCK * 2) + tid;
  AccT v = i < n ? static_cast<AccT>(in[i]) : OpT::template identity<AccT>();
  if (i + BLOCK < n) v = OpT::apply(v, static_cast<AccT>(in[i + BLOCK]));
  sdata[tid] = v;
  __syncthreads();
  unrolled_tail<BLOCK, OpT>(sdata, v, out);
}

template <int BLOCK, class OpT, class Tin, class AccT>
__global__ __launch_bounds__(BLOCK) void k6(const Tin* __restrict__ in, uint64_t n, AccT* __restrict__ out) {
  AccT* sdata = lds_array<AccT>();
  const unsigned tid = threadIdx.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * (BLOCK * 2) + tid;
  const uint64_t grid_size = static_cast<uint64_t>(BLOCK) * 2 * gridDim.x;
  AccT v = OpT::template identity<AccT>();
  while (i < n) {
    v = OpT::apply(v, static_cast<AccT>(in[i]));
    if (i + BLOCK < n) v = OpT::apply(v, static_cast<AccT>(in[i + BLOCK]));
    i += grid_size;
  }
  sdata[tid] = v;
  __syncthreads();
  unrolled_tail<BLOCK, OpT>(sdata, v, out);
}

uint64_t next_pow2(uint64_t x) {
  if (x <= 1) return 1;
  --x;
  for (int s = 1; s < 64; s <<= 1) x |= x >> s;
  return x + 1;
}

template <int BLOCK, class OpT, class Tin, class AccT>
void launch_block(int kernel, const Tin* in, uint64_t n, AccT* dst, int blocks, hipStream_t s) {
  const size_t smem = static_cast<size_t>(BLOCK) * sizeof(AccT);
  if (kernel == 5) hipLaunchKernelGGL((k5<BLOCK, OpT, Tin, AccT>), dim3(blocks), dim3(BLOCK), smem, s, in, n, dst);
  else hipLaunchKernelGGL((k6<BLOCK, OpT, Tin, AccT>), dim3(blocks), dim3(BLOCK), smem, s, in, n, dst);
}

template <class OpT, class Tin, class AccT>
void launch(int kernel, const void* vin, uint64_t n, AccT* dst, int blocks, int threads, hipStream_t s) {
  const Tin* in = static_cast<const Tin*>(vin);
  const size_t smem = static_cast<size_t>(threads) * sizeof(AccT);
  switch (kernel) {
    case 0: hipLaunchKernelGGL((k012<0, OpT, Tin, AccT>), dim3(blocks), dim3(threads), smem, s, in, n, dst); break;
    case 1: hipLaunchKernelGGL((k012<1, OpT, Tin, AccT>), dim3(blocks), dim3(threads), smem, s, in, n, dst); break;
    case 2: hipLaunchKernelGGL((k012<2, OpT, Tin, AccT>), dim3(blocks), dim3(threads), smem, s, in, n, dst); break;
    case 3: hipLaunchKernelGGL((k34<3, OpT, Tin, AccT>), dim3(blocks), dim3(threads), smem, s, in, n, dst); break;
    case 4: hipLaunchKernelGGL((k34<4, OpT, Tin, AccT>), dim3(blocks), dim3(threads), smem, s, in, n, dst); break;
    default:
      switch (threads) {
        case 1: launch_block<1, OpT>(kernel, in, n, dst, blocks, s); break;
        case 2: launch_block<2, OpT>(kernel, in, n, dst, blocks, s); break;
        case 4: launch_block<4, OpT>(kernel, in, n, dst, blocks, s); break;
        case 8: launch_block<8, OpT>(kernel, in, n, dst, blocks, s); break;
        case 16: launch_block<16, OpT>(kernel, in, n, dst, blocks, s); break;
        case 32: launch_block<32, OpT>(kernel, in, n, dst, blocks, s); break;
        case 64: launch_block<64, OpT>(kernel, in, n, dst, blocks, s); break;
        case 128: launch_block<128, OpT>(kernel, in, n, dst, blocks, s); break;
        case 256: launch_block<256, OpT>(kernel, in, n, dst, blocks, s); break;
        case 512: launch_block<512, OpT>(kernel, in, n, dst, blocks, s); break;
        case 1024: launch_block<1024, OpT>(kernel, in, n, dst, blocks, s); break;
        default: throw Error("ladder: threads must be a power of two in [1, 1024]");
      }
  }
  MIREDUCE_HIP_THROW(hipGetLastError());
}

template <class OpT, class T, class AccT>
LadderPasses run(int kernel, const void* in, uint64_t n, void* out, void* scratch, int max_threads, int max_blocks,
                 uint64_t cpu_thresh, bool cpu_final, hipStream_t s) {
  int blocks = 0, threads = 0;
  ladder_geometry(kernel, n, max_threads, max_blocks, &blocks, &threads);
  AccT* a = static_cast<AccT*>(scratch);
  AccT* b = a + std::max(blocks, 1);
  AccT* dst = blocks == 1 ? static_cast<AccT*>(out) : a;
  launch<OpT, T, AccT>(kernel, in, n, dst, blocks, threads, s);
  LadderPasses r;
  r.first_grid = blocks;
  r.passes = 1;
  uint64_t left = static_cast<uint64_t>(blocks);
  AccT* cur = a;
  AccT* other = b;
  // The reference's relaunch loop (reduction.cpp:344-357): the same kernel on the partials while
  // more than cputhresh remain (ping-pong buffers instead of in place); --cpufinal stops after the
  // first pass (reduction.cpp:328-340). What is left (> 1) is folded on the host by the caller.
  while (!cpu_final && left > std::max<uint64_t>(cpu_thresh, 1)) {
    int b2 = 0, t2 = 0;
    ladder_geometry(kernel, left, max_threads, max_blocks, &b2, &t2);
    AccT* d2 = b2 == 1 ? static_cast<AccT*>(out) : other;
    launch<OpT, AccT, AccT>(kernel, cur, left, d2, b2, t2, s);
    left = static_cast<uint64_t>(b2);
    ++r.passes;
    std::swap(cur, other);
  }
  r.left = left;
  r.partials = left > 1 ? static_cast<const void*>(cur) : out;
  return r;
}

}  // namespace ladder

void ladder_geometry(int kernel, uint64_t n, int max_threads, int max_blocks, int* blocks, int* threads) {
  uint64_t t, b;
  if (kernel < 3) {
    t = n < static_cast<uint64_t>(max_threads) ? ladder::next_pow2(n) : max_threads;
    b = (n + t - 1) / t;
  } else {
    t = n < 2ull * max_threads ? ladder::next_pow2((n + 1) / 2) : max_threads;
    b = (n + t * 2 - 1) / (t * 2);
  }
  if (t < 1) t = 1;  // (any power of two: sub-wave blocks reduce over their active lanes only)
  if (kernel == 6 && b > static_cast<uint64_t>(max_blocks)) b = max_blocks;
  if (b < 1) b = 1;
  MIREDUCE_REQUIRE(b <= 0x7FFFFFFFull, "ladder: grid too large; use kernel 6 or 7 for this size");
  *blocks = static_cast<int>(b);
  *threads = static_cast<int>(t);
}

size_t ladder_scratch_bytes(int kernel, uint64_t n, int max_threads, int max_blocks) {
  int b = 0, t = 0;
  ladder_geometry(kernel, n, max_threads, max_blocks, &b, &t);
  return 2 * (static_cast<size_t>(b) + 1) * 8;
}

int ladder_reduce(int kernel, const void* in, uint64_t n, DType t, Op op, DType acc, void* out, void* scratch,
                  int max_threads, int max_blocks, hipStream_t s) {
  return ladder_reduce_passes(kernel, in, n, t, op, acc, out, scratch, max_threads, max_blocks, 1, false, s).first_grid;
}

LadderPasses ladder_reduce_passes(int kernel, const void* in, uint64_t n, DType t, Op op, DType acc, void* out,
                                  void* scratch, int max_threads, int max_blocks, uint64_t cpu_thresh, bool cpu_final,
                                  hipStream_t s) {
  MIREDUCE_REQUIRE(kernel >= 0 && kernel <= 6, "ladder kernel must be 0..6");
  MIREDUCE_REQUIRE(acc_supported(t, op, acc), "unsupported (dtype, op, accumulator) combination");
  MIREDUCE_REQUIRE(!op_is_fused(op), "ladder kernels 0..6 implement the reference's SUM/MIN/MAX");
  MIREDUCE_REQUIRE(!dtype_is_half(t), "ladder kernels 0..6 cover the reference's element types (int, float, double, "
                                      "int64); bf16/half use the streaming kernel (7/8)");
  using namespace ladder;
#define MIREDUCE_LADDER_CASE(OPT, T, A) \
  return run<OPT, T, A>(kernel, in, n, out, scratch, max_threads, max_blocks, cpu_thresh, cpu_final, s)
  switch (op) {
    case Op::Sum:
      switch (t) {
        case DType::Int32: if (acc == DType::Int64) MIREDUCE_LADDER_CASE(SumOp, int32_t, int64_t); MIREDUCE_LADDER_CASE(SumOp, int32_t, int32_t);
        case DType::Int64: MIREDUCE_LADDER_CASE(SumOp, int64_t, int64_t);
        case DType::Float32: if (acc == DType::Float64) MIREDUCE_LADDER_CASE(SumOp, float, double); MIREDUCE_LADDER_CASE(SumOp, float, float);
        case DType::Float64: MIREDUCE_LADDER_CASE(SumOp, double, double);
        default: break;
      }
      break;
    case Op::Min:
      switch (t) {
        case DType::Int32: MIREDUCE_LADDER_CASE(MinOp, int32_t, int32_t);
        case DType::Int64: MIREDUCE_LADDER_CASE(MinOp, int64_t, int64_t);
        case DType::Float32: MIREDUCE_LADDER_CASE(MinOp, float, float);
        case DType::Float64: MIREDUCE_LADDER_CASE(MinOp, double, double);
        default: break;
      }
      break;
    default:
      break;
    case Op::Max:
      switch (t) {
        case DType::Int32: MIREDUCE_LADDER_CASE(MaxOp, int32_t, int32_t);
        case DType::Int64: MIREDUCE_LADDER_CASE(MaxOp, int64_t, int64_t);
        case DType::Float32: MIREDUCE_LADDER_CASE(MaxOp, float, float);
        case DType::Float64: MIREDUCE_LADDER_CASE(MaxOp, double, double);
        default: break;
      }
      break;
  }
#undef MIREDUCE_LADDER_CASE
  throw Error("ladder: unsupported combination");
}

}  // namespace mireduce
