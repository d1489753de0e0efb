// One-kernel direct all-reduce / reduce over xGMI peer mappings; see direct.hpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "mireduce/check.hpp"
#include "mireduce/direct.hpp"
#include "mireduce/peer.hpp"
#include "mireduce/ops.hpp"

namespace mireduce {
namespace kern {

// Per-workgroup cross-rank barrier `phase` of launch `e`: workgroup b of this rank meets
// workgroup b of every other rank. Lane p of wave 0 raises this rank's flag in rank p's array
// and then waits for rank p's flag in its own (the world raises leave in one store round).
// release: make this workgroup's earlier stores visible at system scope first (every wave drains
// its stores, then one system-scope release fence writes back the L2).
__device__ __forceinline__ void peer_barrier(const DirectDesc* d, int phase, unsigned e, unsigned err,
                                             bool release) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    const int world = d->world;
    const uint64_t slot = (static_cast<uint64_t>(phase) * kMaxDirectBlocks + blockIdx.x) * kMaxDirectRanks;
    if (lane < world) {
      __hip_atomic_store(d->sig[lane] + slot + d->rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned* mine = d->sig[d->rank] + slot + lane;
      const uint64_t limit = err ? 0 : d->timeout_ticks;
      const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
      while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != e) {
        if (static_cast<uint64_t>(wall_clock64()) - t0 > limit) {
          __hip_atomic_fetch_or(d->ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // peers' data, not stale cached lines
  }
  __syncthreads();
}

// Vectors [v0, v1) of chunk `c` handled by this workgroup (the same split on every rank).
__device__ __forceinline__ void block_range(uint64_t nvec, uint64_t* v0, uint64_t* v1) {
  const uint64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  *v0 = std::min<uint64_t>(nvec, blockIdx.x * per);
  *v1 = std::min<uint64_t>(nvec, *v0 + per);
}

// Elements per (full) chunk: ceil(count / world) rounded up to whole 16-byte vectors; chunk r is
// [r * per, (r + 1) * per) clipped to count (direct_chunk on the host).
template <class T>
__device__ __forceinline__ uint64_t chunk_elems(uint64_t count, int world) {
  constexpr uint64_t N = 16 / sizeof(T);
  const uint64_t per = (count + world - 1) / world;
  return (per + N - 1) / N * N;
}

// Vectors per thread per loop trip in the W-rank kernel: small worlds have few peer loads per
// vector, so each thread takes U vectors and issues all U * W loads before combining (at least
// 4 loads in flight per lane; a 1- or 2-rank pass with one or two was latency-bound).
template <int W>
constexpr int direct_unroll() {
  return W >= 4 ? 1 : (W >= 2 ? 2 : 4);
}

// W > 0: exactly W ranks, every peer's load of U vectors issued before any is combined.
// W == 0: any world (runtime loop).
template <class OpT, class T, int W>
__global__ __launch_bounds__(kDirectBlock) void direct_kernel(const DirectDesc* __restrict__ d, uint64_t count,
                                                               int gather_rank) {
  constexpr int N = 16 / sizeof(T);
  constexpr int U = W > 0 ? direct_unroll<W>() : 1;
  using V = T __attribute__((ext_vector_type(N)));
  __shared__ unsigned s_epoch, s_err;
  if (threadIdx.x == 0) {
    s_epoch = __hip_atomic_load(d->ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_err = __hip_atomic_load(d->ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const unsigned e = s_epoch;
  const int world = W > 0 ? W : d->world;
  const int rank = d->rank;

  // ---- barrier 0: every rank's input is complete (earlier kernels / copies on its stream)
  peer_barrier(d, 0, e, s_err, true);

  // ---- reduce-scatter: this rank's chunk, every rank's input read over xGMI
  // Workgroup b owns the same vector sub-range [v0, v1) of EVERY chunk, in both phases (a full
  // chunk's split, clipped to a short last chunk), so per-workgroup barriers order all accesses.
  const uint64_t per = chunk_elems<T>(count, world);
  const uint64_t perv = per / N;
  uint64_t v0, v1;
  block_range(perv, &v0, &v1);
  {
    const uint64_t cb = std::min<uint64_t>(count, rank * per);
    const uint64_t ce = std::min<uint64_t>(count, cb + per);
    const uint64_t nvec = (ce - cb) / N;
    const uint64_t r1 = std::min(v1, nvec);
    T* out = reinterpret_cast<T*>(d->out[rank]);
    if constexpr (W > 0) {
      for (uint64_t i0 = v0 + threadIdx.x; i0 < r1; i0 += U * kDirectBlock) {
        V v[U][W];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint64_t i = i0 + static_cast<uint64_t>(u) * kDirectBlock;
          if (i < r1)
#pragma unroll
            for (int p = 0; p < W; ++p)
              v[u][p] = __builtin_nontemporal_load(reinterpret_cast<const V*>(d->in[p]) + cb / N + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint64_t i = i0 + static_cast<uint64_t>(u) * kDirectBlock;
          if (i >= r1) continue;
          V acc = v[u][0];
#pragma unroll
          for (int p = 1; p < W; ++p)
#pragma unroll
            for (int k = 0; k < N; ++k) acc[k] = OpT::apply(acc[k], v[u][p][k]);
          reinterpret_cast<V*>(out)[cb / N + i] = acc;
        }
      }
    } else {
      for (uint64_t i = v0 + threadIdx.x; i < r1; i += kDirectBlock) {
        const uint64_t off = cb / N + i;
        V acc = __builtin_nontemporal_load(reinterpret_cast<const V*>(d->in[0]) + off);
        for (int p = 1; p < world; ++p) {
          const V v = __builtin_nontemporal_load(reinterpret_cast<const V*>(d->in[p]) + off);
#pragma unroll
          for (int k = 0; k < N; ++k) acc[k] = OpT::apply(acc[k], v[k]);
        }
        reinterpret_cast<V*>(out)[off] = acc;
      }
    }
    if (blockIdx.x == gridDim.x - 1) {  // sub-vector tail (last chunk only)
      for (uint64_t i = cb + nvec * N + threadIdx.x; i < ce; i += kDirectBlock) {
        T acc = reinterpret_cast<const T*>(d->in[0])[i];
        for (int p = 1; p < world; ++p) acc = OpT::apply(acc, reinterpret_cast<const T*>(d->in[p])[i]);
        out[i] = acc;
      }
    }
  }

  // ---- barrier 1: every chunk reduced and visible
  peer_barrier(d, 1, e, s_err, true);

  // ---- all-gather (every rank, or only the reduce's root): this workgroup's sub-range of every
  //      other rank's chunk, all owners read in the same pass
  if (gather_rank < 0 || gather_rank == rank) {
    T* mine = reinterpret_cast<T*>(d->out[rank]);
    if constexpr (W > 0) {
      uint64_t nv[W];  // whole vectors in chunk p (only the last non-empty chunk can be short)
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const uint64_t b = std::min<uint64_t>(count, p * per);
        nv[p] = p == rank ? 0 : (std::min<uint64_t>(count, b + per) - b) / N;
      }
      for (uint64_t i0 = v0 + threadIdx.x; i0 < v1; i0 += U * kDirectBlock) {
        V v[U][W];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint64_t i = i0 + static_cast<uint64_t>(u) * kDirectBlock;
#pragma unroll
          for (int p = 0; p < W; ++p)
            if (i < v1 && i < nv[p])
              v[u][p] = __builtin_nontemporal_load(reinterpret_cast<const V*>(d->out[p]) + p * perv + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint64_t i = i0 + static_cast<uint64_t>(u) * kDirectBlock;
#pragma unroll
          for (int p = 0; p < W; ++p)
            if (i < v1 && i < nv[p]) reinterpret_cast<V*>(mine)[p * perv + i] = v[u][p];
        }
      }
    } else {
      for (int p = 0; p < world; ++p) {
        if (p == rank) continue;
        const uint64_t b = std::min<uint64_t>(count, p * per);
        const uint64_t n = (std::min<uint64_t>(count, b + per) - b) / N;
        const uint64_t e1 = std::min(v1, n);
        for (uint64_t i = v0 + threadIdx.x; i < e1; i += kDirectBlock)
          reinterpret_cast<V*>(mine)[p * perv + i] = __builtin_nontemporal_load(reinterpret_cast<const V*>(d->out[p]) + p * perv + i);
      }
    }
    if (blockIdx.x == gridDim.x - 1) {  // sub-vector tails (the last non-empty chunk only)
      for (int p = 0; p < world; ++p) {
        if (p == rank) continue;
        const uint64_t b = std::min<uint64_t>(count, p * per);
        const uint64_t e1 = std::min<uint64_t>(count, b + per);
        for (uint64_t i = b + (e1 - b) / N * N + threadIdx.x; i < e1; i += kDirectBlock)
          mine[i] = reinterpret_cast<const T*>(d->out[p])[i];
      }
    }
  }

  // ---- barrier 2: no peer still reads this rank's input / output (the next collective may
  //      overwrite them); then the last workgroup publishes the epoch for the next launch.
  peer_barrier(d, 2, e, s_err, false);
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(d->ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(d->ctl + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(d->ctl, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
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

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int dev) {
    MIREDUCE_HIP_THROW(hipGetDevice(&prev));
    MIREDUCE_HIP_THROW(hipSetDevice(dev));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

constexpr size_t kSigBytes = static_cast<size_t>(kDirectPhases) * kMaxDirectBlocks * kMaxDirectRanks * sizeof(unsigned);

using DirectFn = void (*)(const DirectDesc*, uint64_t, int, int, hipStream_t);

template <class OpT, class T, int W>
void launch_w(const DirectDesc* d, uint64_t count, int gather, int grid, hipStream_t s) {
  hipLaunchKernelGGL((kern::direct_kernel<OpT, T, W>), dim3(grid), dim3(kDirectBlock), 0, s, d, count, gather);
}

template <class OpT, class T>
DirectFn pick_world(int world) {
  switch (world) {
    case 1: return launch_w<OpT, T, 1>;
    case 2: return launch_w<OpT, T, 2>;
    case 3: return launch_w<OpT, T, 3>;
    case 4: return launch_w<OpT, T, 4>;
    case 5: return launch_w<OpT, T, 5>;
    case 6: return launch_w<OpT, T, 6>;
    case 7: return launch_w<OpT, T, 7>;
    case 8: return launch_w<OpT, T, 8>;
    default: return launch_w<OpT, T, 0>;
  }
}

template <class OpT>
DirectFn pick_type(DType t, int world) {
  switch (t) {
    case DType::Int32: return pick_world<OpT, int32_t>(world);
    case DType::Int64: return pick_world<OpT, int64_t>(world);
    case DType::Float32: return pick_world<OpT, float>(world);
    case DType::Float64: return pick_world<OpT, double>(world);
    default: MIREDUCE_REQUIRE(false, "direct: int32, int64, float32 or float64 only");
  }
  return nullptr;
}

}  // namespace

DirectAllreduce::DirectAllreduce(int device, size_t bytes, int grid, double timeout_s) : timeout_s_(timeout_s) {
  MIREDUCE_REQUIRE(timeout_s > 0, "direct: timeout must be positive");
  if (device < 0) MIREDUCE_HIP_THROW(hipGetDevice(&device));
  device_ = device;
  DeviceGuard g(device_);
  int cus = 0;
  MIREDUCE_HIP_THROW(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_));
  grid_ = grid > 0 ? grid : std::max(1, cus);
  MIREDUCE_REQUIRE(grid_ <= kMaxDirectBlocks, "direct: grid exceeds kMaxDirectBlocks");
  bytes_ = (std::max<size_t>(bytes, 16) + 255) / 256 * 256;
  // Fine-grained data buffers (peers read them over xGMI); uncached flags (polled while peers write).
  MIREDUCE_HIP_THROW(hipExtMallocWithFlags(&in_, bytes_, hipDeviceMallocFinegrained));
  MIREDUCE_HIP_THROW(hipExtMallocWithFlags(&out_, bytes_, hipDeviceMallocFinegrained));
  MIREDUCE_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), kSigBytes, hipDeviceMallocUncached));
  MIREDUCE_HIP_THROW(hipMemset(sig_, 0, kSigBytes));
  MIREDUCE_HIP_THROW(hipMalloc(reinterpret_cast<void**>(&ctl_), 256));
  MIREDUCE_HIP_THROW(hipMemset(ctl_, 0, 256));
  MIREDUCE_HIP_THROW(hipMalloc(reinterpret_cast<void**>(&desc_), sizeof(DirectDesc)));
  MIREDUCE_HIP_THROW(hipDeviceSynchronize());
}

DirectAllreduce::~DirectAllreduce() {
  DeviceGuard g(device_);
  for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
  (void)hipFree(sink_);
  (void)hipFree(desc_);
  (void)hipFree(ctl_);
  (void)hipFree(sig_);
  (void)hipFree(out_);
  (void)hipFree(in_);
  // An ignored failure above (e.g. closing a mapping of a peer that already exited) must not stay
  // behind as the thread's last error: the next launch's hipGetLastError() check would report it.
  (void)hipGetLastError();
}

std::vector<char> DirectAllreduce::handles() const {
  std::vector<char> h(kHandleBytes);
  void* bufs[3] = {in_, out_, sig_};
  for (int k = 0; k < 3; ++k) {
    hipIpcMemHandle_t m;
    MIREDUCE_HIP_THROW(hipIpcGetMemHandle(&m, bufs[k]));
    std::memcpy(h.data() + k * sizeof(IpcHandleBytes), &m, sizeof m);
  }
  const int32_t gr = grid_;
  std::memcpy(h.data() + 3 * sizeof(IpcHandleBytes), &gr, sizeof gr);
  return h;
}

void DirectAllreduce::connect(int rank, int world, const std::vector<std::vector<char>>& all) {
  MIREDUCE_REQUIRE(!connected_, "direct: already connected");
  MIREDUCE_REQUIRE(world >= 1 && world <= kMaxDirectRanks, "direct: world must be 1..16");
  MIREDUCE_REQUIRE(rank >= 0 && rank < world, "direct: rank out of range");
  MIREDUCE_REQUIRE(all.size() == static_cast<size_t>(world), "direct: one handle set per rank");
  DeviceGuard g(device_);
  DirectDesc d{};
  for (int r = 0; r < world; ++r) {
    MIREDUCE_REQUIRE(all[r].size() == kHandleBytes, "direct: bad handle size");
    int32_t gr = 0;
    std::memcpy(&gr, all[r].data() + 3 * sizeof(IpcHandleBytes), sizeof gr);
    MIREDUCE_REQUIRE(gr == grid_, "direct: every rank must use the same grid");
    if (r == rank) {
      d.in[r] = static_cast<const char*>(in_);
      d.out[r] = static_cast<char*>(out_);
      d.sig[r] = sig_;
      continue;
    }
    void* p[3] = {nullptr, nullptr, nullptr};
    for (int k = 0; k < 3; ++k) {
      hipIpcMemHandle_t m;
      std::memcpy(&m, all[r].data() + k * sizeof(IpcHandleBytes), sizeof m);
      MIREDUCE_HIP_THROW(hipIpcOpenMemHandle(&p[k], m, hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(p[k]);
    }
    d.in[r] = static_cast<const char*>(p[0]);
    peer_in_.push_back(p[0]);
    d.out[r] = static_cast<char*>(p[1]);
    d.sig[r] = static_cast<unsigned*>(p[2]);
  }
  d.ctl = ctl_;
  d.rank = rank;
  d.world = world;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_) != hipSuccess || khz <= 0) khz = 100000;
  d.timeout_ticks = static_cast<uint64_t>(timeout_s_ * 1e3 * khz);
  MIREDUCE_HIP_THROW(hipMemcpy(desc_, &d, sizeof d, hipMemcpyHostToDevice));
  MIREDUCE_HIP_THROW(hipDeviceSynchronize());
  rank_ = rank;
  world_ = world;
  connected_ = true;
}

void DirectAllreduce::launch(size_t count, DType t, Op op, int gather_rank, hipStream_t s) {
  MIREDUCE_REQUIRE(connected_, "direct: connect() first");
  MIREDUCE_REQUIRE(count * dtype_size(t) <= bytes_, "direct: count exceeds the registered buffers");
  DirectFn fn = nullptr;
  switch (op) {
    case Op::Sum: fn = pick_type<SumOp>(t, world_); break;
    case Op::Min: fn = pick_type<MinOp>(t, world_); break;
    case Op::Max: fn = pick_type<MaxOp>(t, world_); break;
    default: MIREDUCE_REQUIRE(false, "direct: SUM, MIN or MAX");
  }
  (void)hipGetLastError();  // report this launch's error only
  fn(desc_, count, gather_rank, grid_, s);
  MIREDUCE_HIP_THROW(hipGetLastError());
}

void DirectAllreduce::allreduce(size_t count, DType t, Op op, hipStream_t s) { launch(count, t, op, -1, s); }

void DirectAllreduce::reduce(size_t count, DType t, Op op, int root, hipStream_t s) {
  MIREDUCE_REQUIRE(root >= 0 && root < world_, "direct: root out of range");
  launch(count, t, op, root, s);
}

void DirectAllreduce::read_peers(size_t bytes_each, hipStream_t s) {
  MIREDUCE_REQUIRE(connected_, "direct: connect() first");
  MIREDUCE_REQUIRE(bytes_each <= bytes_, "direct: read_peers beyond the registered buffers");
  DeviceGuard g(device_);
  PeerSources src{};
  int n = 0;
  if (peer_in_.empty()) src.p[n++] = in_;
  for (const void* p : peer_in_) src.p[n++] = p;
  const int grid = 128 * n;  // peer_read's default: 128 workgroups per source
  if (!sink_) MIREDUCE_HIP_THROW(hipMalloc(reinterpret_cast<void**>(&sink_), 128 * kMaxPeerSources * sizeof(uint32_t)));
  peer_read(src, n, bytes_each, sink_, grid, s);
}

unsigned DirectAllreduce::error() const {
  unsigned v = 0;
  DeviceGuard g(device_);
  MIREDUCE_HIP_THROW(hipMemcpy(&v, ctl_ + 1, sizeof v, hipMemcpyDeviceToHost));
  return v;
}

unsigned DirectAllreduce::epoch() const {
  unsigned v = 0;
  DeviceGuard g(device_);
  MIREDUCE_HIP_THROW(hipMemcpy(&v, ctl_, sizeof v, hipMemcpyDeviceToHost));
  return v;
}

}  // namespace mireduce
