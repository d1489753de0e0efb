// Kernels of the direct (peer-read) all-reduce; see direct.hpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mireduce/check.hpp"
#include "mireduce/direct.hpp"
#include "mireduce/ops.hpp"

namespace mireduce {
namespace kern {

struct PeerPtrs {
  const void* p[kMaxDirectPeers];
};

// One lane per workgroup: system-scope acquire (invalidate non-coherent cached lines of
// peer-written memory), its wait, then the workgroup barrier (CDNA guide §6 G16 consumer order).
__device__ __forceinline__ void acquire_system() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// Every wave drains its stores, workgroup barrier, one lane releases at system scope (writes
// back dirty L2 lines) and waits for it (guide §6 G16 producer order, Pitfall 12).
__device__ __forceinline__ void release_system() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// out[begin, end) = op over p of in_p[begin, end)  (16-byte vectors + scalar tail)
template <class OpT, class T>
__global__ __launch_bounds__(256) void direct_reduce_scatter(PeerPtrs ins, int world, T* __restrict__ out,
                                                             uint64_t begin, uint64_t end) {
  acquire_system();
  constexpr int N = 16 / sizeof(T);
  using V = T __attribute__((ext_vector_type(N)));
  const uint64_t vb = begin / N, ve = end / N;  // begin is vector-aligned (direct_chunk)
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t i = vb + static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < ve; i += stride) {
    V acc = __builtin_nontemporal_load(static_cast<const V*>(ins.p[0]) + i);
    for (int p = 1; p < world; ++p) {
      const V v = __builtin_nontemporal_load(static_cast<const V*>(ins.p[p]) + i);
#pragma unroll
      for (int k = 0; k < N; ++k) acc[k] = OpT::apply(acc[k], v[k]);
    }
    reinterpret_cast<V*>(out)[i] = acc;
  }
  if (blockIdx.x == 0) {
    for (uint64_t i = ve * N + threadIdx.x; i < end; i += 256) {
      T acc = static_cast<const T*>(ins.p[0])[i];
      for (int p = 1; p < world; ++p) acc = OpT::apply(acc, static_cast<const T*>(ins.p[p])[i]);
      out[i] = acc;
    }
  }
  release_system();
}

// dst[b_p, e_p) = src_p[b_p, e_p) for every peer p != self (the all-gather / gather phase).
__global__ __launch_bounds__(256) void direct_gather(PeerPtrs outs, int world, int self, char* __restrict__ dst,
                                                     uint64_t count, uint64_t elem, uint64_t chunk_elems) {
  acquire_system();
  using V = uint32_t __attribute__((ext_vector_type(4)));
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (int p = 0; p < world; ++p) {
    if (p == self) continue;
    const uint64_t b = std::min<uint64_t>(count, p * chunk_elems) * elem;
    const uint64_t e = std::min<uint64_t>(count, (p + 1) * chunk_elems) * elem;
    const uint64_t vb = b / 16, ve = e / 16;  // b is 16-byte aligned
    const char* src = static_cast<const char*>(outs.p[p]);
    for (uint64_t i = vb + static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < ve; i += stride)
      reinterpret_cast<V*>(dst)[i] = __builtin_nontemporal_load(reinterpret_cast<const V*>(src) + i);
    if (blockIdx.x == 0)
      for (uint64_t i = ve * 16 + threadIdx.x; i < e; i += 256) dst[i] = src[i];
  }
  release_system();
}

}  // namespace kern

void direct_chunk(size_t count, size_t elem_size, int world, int r, size_t* begin, size_t* end) {
  const size_t vec = 16 / elem_size;
  size_t per = (count + world - 1) / world;
  per = (per + vec - 1) / vec * vec;
  *begin = std::min(count, static_cast<size_t>(r) * per);
  *end = std::min(count, static_cast<size_t>(r + 1) * per);
}

namespace {
int grid_for(size_t bytes) {
  const size_t vecs = (bytes + 15) / 16;
  return static_cast<int>(std::max<size_t>(1, std::min<size_t>(2048, (vecs + 255) / 256)));
}

template <class OpT, class T>
void launch_rs(const kern::PeerPtrs& ins, int world, void* out, uint64_t b, uint64_t e, hipStream_t s) {
  hipLaunchKernelGGL((kern::direct_reduce_scatter<OpT, T>), dim3(grid_for((e - b) * sizeof(T))), dim3(256), 0, s, ins,
                     world, static_cast<T*>(out), b, e);
}

template <class OpT>
void rs_by_type(DType t, const kern::PeerPtrs& ins, int world, void* out, uint64_t b, uint64_t e, hipStream_t s) {
  switch (t) {
    case DType::Int32: launch_rs<OpT, int32_t>(ins, world, out, b, e, s); break;
    case DType::Int64: launch_rs<OpT, int64_t>(ins, world, out, b, e, s); break;
    case DType::Float32: launch_rs<OpT, float>(ins, world, out, b, e, s); break;
    case DType::Float64: launch_rs<OpT, double>(ins, world, out, b, e, s); break;
    default: MIREDUCE_REQUIRE(false, "direct: int32, int64, float32 or float64 only");
  }
}
}  // namespace

DirectPeers::DirectPeers(TcpBootstrap& boot, int device, size_t bytes, bool finegrained)
    : boot_(boot), rank_(boot.rank()), world_(boot.world()), device_(device), bytes_(bytes), finegrained_(finegrained) {
  MIREDUCE_REQUIRE(world_ <= kMaxDirectPeers, "direct: too many ranks");
  bytes_ = (std::max<size_t>(bytes, 16) + 255) / 256 * 256;
  if (finegrained_) {
    MIREDUCE_HIP_THROW(hipExtMallocWithFlags(&in_, bytes_, hipDeviceMallocFinegrained));
    MIREDUCE_HIP_THROW(hipExtMallocWithFlags(&out_, bytes_, hipDeviceMallocFinegrained));
  } else {
    MIREDUCE_HIP_THROW(hipMalloc(&in_, bytes_));
    MIREDUCE_HIP_THROW(hipMalloc(&out_, bytes_));
  }
  hipIpcMemHandle_t mine[2];
  MIREDUCE_HIP_THROW(hipIpcGetMemHandle(&mine[0], in_));
  MIREDUCE_HIP_THROW(hipIpcGetMemHandle(&mine[1], out_));
  std::vector<hipIpcMemHandle_t> all(2 * static_cast<size_t>(world_));
  boot_.allgather(mine, all.data(), sizeof mine);
  peer_in_.assign(world_, nullptr);
  peer_out_.assign(world_, nullptr);
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) {
      peer_in_[r] = in_;
      peer_out_[r] = out_;
      continue;
    }
    MIREDUCE_HIP_THROW(hipIpcOpenMemHandle(&peer_in_[r], all[2 * r], hipIpcMemLazyEnablePeerAccess));
    MIREDUCE_HIP_THROW(hipIpcOpenMemHandle(&peer_out_[r], all[2 * r + 1], hipIpcMemLazyEnablePeerAccess));
  }
  boot_.barrier();
}

DirectPeers::~DirectPeers() {
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) continue;
    if (peer_in_.size() > static_cast<size_t>(r) && peer_in_[r]) (void)hipIpcCloseMemHandle(peer_in_[r]);
    if (peer_out_.size() > static_cast<size_t>(r) && peer_out_[r]) (void)hipIpcCloseMemHandle(peer_out_[r]);
  }
  (void)hipFree(in_);
  (void)hipFree(out_);
}

void DirectPeers::reduce_scatter(size_t count, DType t, Op op, hipStream_t s) {
  MIREDUCE_REQUIRE(count * dtype_size(t) <= bytes_, "direct: count exceeds the registered buffers");
  kern::PeerPtrs ins{};
  for (int r = 0; r < world_; ++r) ins.p[r] = peer_in_[r];
  size_t b = 0, e = 0;
  direct_chunk(count, dtype_size(t), world_, rank_, &b, &e);
  if (e > b) {
    switch (op) {
      case Op::Sum: rs_by_type<SumOp>(t, ins, world_, out_, b, e, s); break;
      case Op::Min: rs_by_type<MinOp>(t, ins, world_, out_, b, e, s); break;
      case Op::Max: rs_by_type<MaxOp>(t, ins, world_, out_, b, e, s); break;
      default: MIREDUCE_REQUIRE(false, "direct: SUM, MIN or MAX");
    }
    MIREDUCE_HIP_THROW(hipGetLastError());
  }
  MIREDUCE_HIP_THROW(hipStreamSynchronize(s));
  boot_.barrier();  // every chunk reduced and released before anyone gathers
}

void DirectPeers::gather_chunks(size_t count, DType t, hipStream_t s) {
  kern::PeerPtrs outs{};
  for (int r = 0; r < world_; ++r) outs.p[r] = peer_out_[r];
  size_t b = 0, e = 0;
  direct_chunk(count, dtype_size(t), world_, 0, &b, &e);
  const uint64_t chunk = e - b;
  hipLaunchKernelGGL(kern::direct_gather, dim3(grid_for(count * dtype_size(t))), dim3(256), 0, s, outs, world_, rank_,
                     static_cast<char*>(out_), static_cast<uint64_t>(count), static_cast<uint64_t>(dtype_size(t)),
                     chunk);
  MIREDUCE_HIP_THROW(hipGetLastError());
}

void DirectPeers::allreduce(size_t count, DType t, Op op, hipStream_t s) {
  reduce_scatter(count, t, op, s);
  gather_chunks(count, t, s);
  MIREDUCE_HIP_THROW(hipStreamSynchronize(s));
  boot_.barrier();  // nobody rewrites its chunk while a peer may still read it
}

void DirectPeers::reduce(size_t count, DType t, Op op, int root, hipStream_t s) {
  reduce_scatter(count, t, op, s);
  if (rank_ == root) gather_chunks(count, t, s);
  MIREDUCE_HIP_THROW(hipStreamSynchronize(s));
  boot_.barrier();
}

}  // namespace mireduce
