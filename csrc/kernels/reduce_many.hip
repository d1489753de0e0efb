// One launch, many tensors; see reduce_many.hpp.
//
// The bound list is a table of segments {pointer, [begin, end), tensor}: short tensors are one
// segment, long ones are cut into ~equal segments so the workgroups share the bytes evenly. A
// workgroup takes segments grid-stride (its descriptor comes in through scalar loads), streams the
// range with the 16-byte nt loads of the full reduction (scalar head/tail for any alignment), and
// reduces across its 256 lanes (wave butterflies + one LDS slot per wave). A tensor with one
// segment is written directly; otherwise each segment publishes its partial write-through (sc1)
// and takes the tensor's ticket, and the last one folds the tensor's partials in segment order and
// resets the ticket (the single-pass scheme of reduce.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "mireduce/check.hpp"
#include "mireduce/half.hpp"
#include "mireduce/ops.hpp"
#include "mireduce/reduce_many.hpp"
#include "mireduce/vec16.hpp"

namespace mireduce {
namespace kern {

constexpr int kManyBlock = 256;
constexpr int kManyUnroll = 8;

struct Seg {
  const void* ptr;
  uint64_t begin, end;  // element range of the tensor
  uint32_t tensor;
  uint32_t pad;
};

struct TensorInfo {
  uint32_t first_seg, nseg;
};

struct ManyArgs {
  const Seg* segs;
  const TensorInfo* info;
  uint32_t nseg;
  void* out;
  void* partials;
  unsigned* tickets;
};

template <class OpT, class T, class AccT>
__global__ __launch_bounds__(kManyBlock) void many_kernel(ManyArgs a) {
  using V = typename Vec16<T>::type;
  constexpr int N = Vec16<T>::N;
  constexpr int U = kManyUnroll;
  constexpr int kWaves = kManyBlock / 64;
  __shared__ AccT lds[kWaves];
  __shared__ int last;
  const int tid = threadIdx.x;
  // A workgroup streams one segment at a time (its 256 lanes read 4 KB contiguous per load
  // round): fewer, wider concurrent streams than a wave per segment (13 GB bf16 parameter list:
  // 5.4 -> 6.3 TB/s, profiles/r1_session3/reduce_many/).
  for (uint32_t s = blockIdx.x; s < a.nseg; s += gridDim.x) {  // workgroup-uniform
    const Seg g = a.segs[s];
    const T* p = static_cast<const T*>(g.ptr);
    AccT acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = OpT::template identity<AccT>();
    const uintptr_t addr = reinterpret_cast<uintptr_t>(p + g.begin);
    uint64_t head = addr % 16 ? (16 - addr % 16) / sizeof(T) : 0;
    if (head > g.end - g.begin) head = g.end - g.begin;
    if (static_cast<uint64_t>(tid) < head) acc[0] = OpT::apply(acc[0], OpT::pre(static_cast<AccT>(p[g.begin + tid])));
    const uint64_t vb = g.begin + head;
    const uint64_t nvec = (g.end - vb) / N;
    const V* vp = reinterpret_cast<const V*>(p + vb);
    uint64_t i = tid;
    for (; i + (U - 1) * kManyBlock < nvec; i += U * kManyBlock) {
      V v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(vp + i + u * kManyBlock);
      __builtin_amdgcn_sched_barrier(0);  // all loads out before the first use
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < N; ++k) acc[u] = OpT::apply(acc[u], OpT::pre(elem<T, AccT>(v[u], k)));
      }
    }
    for (; i < nvec; i += kManyBlock) {
      const V v = __builtin_nontemporal_load(vp + i);
#pragma unroll
      for (int k = 0; k < N; ++k) acc[0] = OpT::apply(acc[0], OpT::pre(elem<T, AccT>(v, k)));
    }
    const uint64_t tb = vb + nvec * N;
    if (static_cast<uint64_t>(tid) < g.end - tb) acc[1] = OpT::apply(acc[1], OpT::pre(static_cast<AccT>(p[tb + tid])));
#pragma unroll
    for (int u = 1; u < U; ++u) acc[0] = OpT::apply(acc[0], acc[u]);
    AccT v = acc[0];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = OpT::apply(v, __shfl_xor(v, off, 64));
    if ((tid & 63) == 0) lds[tid >> 6] = v;
    __syncthreads();
    const TensorInfo ti = a.info[g.tensor];
    if (tid == 0) {
#pragma unroll
      for (int w = 1; w < kWaves; ++w) v = OpT::apply(v, lds[w]);
      AccT* out = static_cast<AccT*>(a.out);
      if (ti.nseg == 1) {
        out[g.tensor] = v;
        last = 0;
      } else {
        AccT* part = static_cast<AccT*>(a.partials);
        store_sc1(&part[s], v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(&a.tickets[g.tensor], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == ti.nseg - 1;
        if (last) __hip_atomic_store(&a.tickets[g.tensor], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
    if (last) {  // last segment of this tensor: every lane folds a strided share of its partials
      // (a fixed order — lane j takes j, j + 256, ... — then the fixed butterfly: deterministic)
      const AccT* part = static_cast<const AccT*>(a.partials) + ti.first_seg;
      AccT t = OpT::template identity<AccT>();
      for (uint32_t j = tid; j < ti.nseg; j += kManyBlock) t = OpT::apply(t, load_sc1(&part[j]));
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) t = OpT::apply(t, __shfl_xor(t, off, 64));
      if ((tid & 63) == 0) lds[tid >> 6] = t;
      __syncthreads();
      if (tid == 0) {
#pragma unroll
        for (int w = 1; w < kWaves; ++w) t = OpT::apply(t, lds[w]);
        static_cast<AccT*>(a.out)[g.tensor] = t;
      }
    }
    __syncthreads();  // lds is rewritten by the next segment
  }
}

}  // namespace kern

namespace {

using ManyFn = void (*)(const kern::ManyArgs&, int, hipStream_t);
using ManyOccFn = int (*)();

template <class OpT, class T, class AccT>
void launch_many(const kern::ManyArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((kern::many_kernel<OpT, T, AccT>), dim3(grid), dim3(kern::kManyBlock), 0, s, a);
}

template <class OpT, class T, class AccT>
int many_resident() {
  static const int n = [] {
    int r = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&r, kern::many_kernel<OpT, T, AccT>, kern::kManyBlock, 0) !=
            hipSuccess || r < 1)
      r = 1;
    return std::min(r, 8);
  }();
  return n;
}

struct ManyEntry {
  ManyFn fn;
  ManyOccFn occ;
};

template <class OpT, class T, class AccT>
constexpr ManyEntry many_entry() {
  return {launch_many<OpT, T, AccT>, many_resident<OpT, T, AccT>};
}

ManyEntry many_lookup(Op op, DType t, DType acc) {
  MIREDUCE_REQUIRE(acc_supported(t, op, acc), "unsupported (dtype, op, accumulator) combination");
#define MIREDUCE_MANY(OPV, OPT)                                                                          \
  if (op == OPV) {                                                                                       \
    switch (t) {                                                                                         \
      case DType::Int32: return acc == DType::Int64 ? many_entry<OPT, int32_t, int64_t>() : many_entry<OPT, int32_t, int32_t>(); \
      case DType::Int64: return many_entry<OPT, int64_t, int64_t>();                                     \
      case DType::Float32: return acc == DType::Float64 ? many_entry<OPT, float, double>() : many_entry<OPT, float, float>(); \
      case DType::Float64: return many_entry<OPT, double, double>();                                     \
      case DType::BFloat16: return many_entry<OPT, bf16_t, float>();                                     \
      case DType::Float16: return many_entry<OPT, f16_t, float>();                                       \
    }                                                                                                    \
  }
  MIREDUCE_MANY(Op::Sum, SumOp)
  MIREDUCE_MANY(Op::Min, MinOp)
  MIREDUCE_MANY(Op::Max, MaxOp)
#undef MIREDUCE_MANY
  if (op == Op::SumSq) {
    switch (t) {
      case DType::Float32: return acc == DType::Float64 ? many_entry<SumSqOp, float, double>() : many_entry<SumSqOp, float, float>();
      case DType::Float64: return many_entry<SumSqOp, double, double>();
      case DType::BFloat16: return many_entry<SumSqOp, bf16_t, float>();
      case DType::Float16: return many_entry<SumSqOp, f16_t, float>();
      default: break;
    }
  }
  if (op == Op::AbsMax) {
    switch (t) {
      case DType::Float32: return many_entry<AbsMaxOp, float, float>();
      case DType::Float64: return many_entry<AbsMaxOp, double, double>();
      case DType::BFloat16: return many_entry<AbsMaxOp, bf16_t, float>();
      case DType::Float16: return many_entry<AbsMaxOp, f16_t, float>();
      default: break;
    }
  }
  throw Error("reduce_many: unsupported combination");
}

}  // namespace

BoundReduceMany::BoundReduceMany(const std::vector<const void*>& ptrs, const std::vector<uint64_t>& counts, DType t,
                                 Op op, DType acc, void* out, int device, int num_cus, hipStream_t stream)
    : tensors_(ptrs.size()), t_(t), acc_(acc), op_(op), out_(out) {
  MIREDUCE_REQUIRE(ptrs.size() == counts.size(), "reduce_many: pointer and count lists differ in length");
  MIREDUCE_REQUIRE(!ptrs.empty(), "reduce_many: empty tensor list");
  MIREDUCE_REQUIRE(out != nullptr, "reduce_many: output pointer is null");
  (void)many_lookup(op, t, acc);  // validates the combination
  const size_t es = dtype_size(t);
  const uint64_t N = 16 / es;
  uint64_t total = 0;
  for (size_t i = 0; i < ptrs.size(); ++i) {
    MIREDUCE_REQUIRE(reinterpret_cast<uintptr_t>(ptrs[i]) % es == 0, "reduce_many: misaligned tensor");
    total += counts[i];
  }
  // Segment length: about four segments per resident workgroup over the whole list, at least one
  // full unrolled round of the workgroup (32 KB), at most 4 MB; a multiple of the vector width.
  const uint64_t wgs = static_cast<uint64_t>(num_cus) * 4;
  uint64_t seg = total / std::max<uint64_t>(1, wgs * 4);
  seg = std::max<uint64_t>(seg, static_cast<uint64_t>(kern::kManyBlock) * kern::kManyUnroll * N);
  seg = std::min<uint64_t>(seg, (4ull << 20) / es);
  if (const char* e = std::getenv("MIREDUCE_MANY_SEG_KB"); e && std::atoi(e) > 0)  // A/B runs
    seg = std::max<uint64_t>(N, static_cast<uint64_t>(std::atoi(e)) * 1024 / es);
  seg = (seg + N - 1) / N * N;
  std::vector<kern::Seg> segs;
  std::vector<kern::TensorInfo> info(ptrs.size());
  for (size_t i = 0; i < ptrs.size(); ++i) {
    const uint64_t n = counts[i];
    const uint64_t ns = std::max<uint64_t>(1, (n + seg - 1) / seg);
    info[i].first_seg = static_cast<uint32_t>(segs.size());
    info[i].nseg = static_cast<uint32_t>(ns);
    for (uint64_t j = 0; j < ns; ++j) {
      kern::Seg g{};
      g.ptr = ptrs[i];
      g.begin = std::min<uint64_t>(n, j * seg);
      g.end = std::min<uint64_t>(n, (j + 1) * seg);
      g.tensor = static_cast<uint32_t>(i);
      segs.push_back(g);
    }
  }
  MIREDUCE_REQUIRE(segs.size() < (1ull << 31), "reduce_many: too many segments");
  segments_ = segs.size();
  int prev = 0;
  MIREDUCE_HIP_THROW(hipGetDevice(&prev));
  if (device >= 0) MIREDUCE_HIP_THROW(hipSetDevice(device));
  const size_t seg_bytes = segs.size() * sizeof(kern::Seg);
  const size_t info_off = (seg_bytes + 255) / 256 * 256;
  const size_t table_bytes = info_off + info.size() * sizeof(kern::TensorInfo);
  MIREDUCE_HIP_THROW(hipMalloc(&table_, table_bytes));
  MIREDUCE_HIP_THROW(hipMalloc(&partials_, std::max<size_t>(segs.size(), 1) * 8));
  MIREDUCE_HIP_THROW(hipMalloc(reinterpret_cast<void**>(&tickets_), ptrs.size() * sizeof(unsigned)));
  MIREDUCE_HIP_THROW(hipMemsetAsync(tickets_, 0, ptrs.size() * sizeof(unsigned), stream));
  MIREDUCE_HIP_THROW(hipMemcpyAsync(table_, segs.data(), seg_bytes, hipMemcpyHostToDevice, stream));
  MIREDUCE_HIP_THROW(hipMemcpyAsync(static_cast<char*>(table_) + info_off, info.data(),
                                    info.size() * sizeof(kern::TensorInfo), hipMemcpyHostToDevice, stream));
  MIREDUCE_HIP_THROW(hipStreamSynchronize(stream));  // the host vectors die with this constructor
  int resident = many_lookup(op, t, acc).occ();
  if (const char* e = std::getenv("MIREDUCE_MANY_WG_PER_CU"); e && std::atoi(e) > 0)  // A/B runs
    resident = std::min(resident, std::atoi(e));
  const uint64_t blocks = segs.size();
  grid_ = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(blocks, static_cast<uint64_t>(num_cus) * resident)));
  MIREDUCE_HIP_THROW(hipSetDevice(prev));
}

BoundReduceMany::~BoundReduceMany() {
  (void)hipFree(table_);
  (void)hipFree(partials_);
  (void)hipFree(tickets_);
}

void BoundReduceMany::launch(hipStream_t stream, void* out) const {
  const size_t seg_bytes = segments_ * sizeof(kern::Seg);
  kern::ManyArgs a{};
  a.segs = static_cast<const kern::Seg*>(table_);
  a.info = reinterpret_cast<const kern::TensorInfo*>(static_cast<const char*>(table_) + (seg_bytes + 255) / 256 * 256);
  a.nseg = static_cast<uint32_t>(segments_);
  a.out = out ? out : out_;
  a.partials = partials_;
  a.tickets = tickets_;
  many_lookup(op_, t_, acc_).fn(a, grid_, stream);
  MIREDUCE_HIP_THROW(hipGetLastError());
}

}  // namespace mireduce
