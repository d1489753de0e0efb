// Reductions along one axis of a row-major [rows, cols] matrix; see reduce_dim.hpp.
//
// Rows (reduce the contiguous axis). Short rows (<= 32 vectors) are handled by groups of `lpr`
// lanes of one wave, 64/lpr rows per wave; long rows by one workgroup per row *segment*, cut into
// `splits` segments so that even a handful of rows keeps every CU streaming. Loads are
// the full reduction's 16-byte nt vectors (vec16.hpp) with per-segment scalar head/tail, so any
// row length and base alignment works. When a row
// is split, each segment publishes its partial write-through (sc1) and takes a per-row ticket;
// the last arriver folds the row's partials in segment order (deterministic) and resets the
// ticket — the single-pass scheme of reduce.hip (threadFenceReduction_kernel.cu:116-171 idea).
//
// Columns (reduce the strided axis). Each thread owns 16 bytes of adjacent columns (or one
// column when rows are not 16-byte aligned) and walks down its rows with four rows in flight; a
// wave's loads of one row are contiguous. Few columns and many rows: the rows are split into
// ranges whose partial columns a second launch folds in range order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "mireduce/check.hpp"
#include "mireduce/half.hpp"
#include "mireduce/ops.hpp"
#include "mireduce/reduce_dim.hpp"
#include "mireduce/vec16.hpp"

namespace mireduce {
namespace kern {

constexpr int kDimBlock = 256;
constexpr int kRowUnroll = 8;  // vectors in flight per lane (8 KB per wave)
constexpr int kColUnroll = 8;  // rows in flight per thread

// 16 readable bytes: the load target of lanes that have nothing to load (branch-free issue).
template <class V>
__device__ V g_dummy_vec;

struct RowArgs {
  const void* in;
  uint64_t rows, cols;
  uint64_t splits;   // segments per row
  uint64_t seg_len;  // elements per segment (multiple of the vector width)
  int lpr;           // lanes per segment (power of two, 1..64)
  int aligned;       // short rows: base and row length multiples of 16 bytes
  int nt_out;        // short rows, pipelined loop: non-temporal result stores (MIREDUCE_DIM_NT_OUT)
  void* out;
  void* partials;    // [rows * splits] AccT (splits > 1)
  unsigned* tickets; // [rows] (splits > 1)
};

// Long rows: a workgroup streams one row segment at a time (256 lanes, 4 KB contiguous per load
// round) — fewer, wider concurrent streams than a wave per segment, as in reduce_many.hip.
template <class OpT, class T, class AccT>
__global__ __launch_bounds__(kDimBlock) void rows_kernel(RowArgs a) {
  using V = typename Vec16<T>::type;
  constexpr int N = Vec16<T>::N;
  constexpr int U = kRowUnroll;
  constexpr int kWaves = kDimBlock / 64;
  __shared__ AccT lds[kWaves];
  const int tid = threadIdx.x;
  const uint64_t nseg = a.rows * a.splits;
  const T* base = static_cast<const T*>(a.in);
  for (uint64_t seg = blockIdx.x; seg < nseg; seg += gridDim.x) {  // workgroup-uniform
    AccT acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = OpT::template identity<AccT>();
    const uint64_t r = seg / a.splits;
    const uint64_t b = (seg % a.splits) * a.seg_len;
    const uint64_t e = std::min<uint64_t>(a.cols, b + a.seg_len);
    const T* p = base + r * a.cols;
    if (b < e) {
      const uintptr_t addr = reinterpret_cast<uintptr_t>(p + b);
      uint64_t head = addr % 16 ? (16 - addr % 16) / sizeof(T) : 0;
      if (head > e - b) head = e - b;
      if (static_cast<uint64_t>(tid) < head) acc[0] = OpT::apply(acc[0], OpT::pre(static_cast<AccT>(p[b + tid])));
      const uint64_t vb = b + head;
      const uint64_t nvec = (e - vb) / N;
      const V* vp = reinterpret_cast<const V*>(p + vb);
      uint64_t i = tid;
      for (; i + static_cast<uint64_t>(U - 1) * kDimBlock < nvec; i += static_cast<uint64_t>(U) * kDimBlock) {
        V v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(vp + i + static_cast<uint64_t>(u) * kDimBlock);
        // all loads out before the first use: MIN/MAX's inline v_min/v_max otherwise made hipcc
        // wait for each load in turn (one 16-byte load in flight per lane)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int k = 0; k < N; ++k) acc[u] = OpT::apply(acc[u], OpT::pre(elem<T, AccT>(v[u], k)));
        }
      }
      for (; i < nvec; i += kDimBlock) {
        const V v = __builtin_nontemporal_load(vp + i);
#pragma unroll
        for (int k = 0; k < N; ++k) acc[0] = OpT::apply(acc[0], OpT::pre(elem<T, AccT>(v, k)));
      }
      const uint64_t tb = vb + nvec * N;
      if (static_cast<uint64_t>(tid) < e - tb) acc[1] = OpT::apply(acc[1], OpT::pre(static_cast<AccT>(p[tb + tid])));
    }
#pragma unroll
    for (int u = 1; u < U; ++u) acc[0] = OpT::apply(acc[0], acc[u]);
    AccT v = acc[0];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = OpT::apply(v, __shfl_xor(v, off, 64));
    if ((tid & 63) == 0) lds[tid >> 6] = v;
    __syncthreads();
    if (tid == 0) {
#pragma unroll
      for (int w = 1; w < kWaves; ++w) v = OpT::apply(v, lds[w]);
      AccT* out = static_cast<AccT*>(a.out);
      if (a.splits == 1) {
        out[r] = v;
      } else {
        AccT* part = static_cast<AccT*>(a.partials);
        store_sc1(&part[seg], v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(&a.tickets[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == a.splits - 1) {  // last segment of row r: fold in segment order
          __hip_atomic_store(&a.tickets[r], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          AccT t = OpT::template identity<AccT>();
          for (uint64_t j = 0; j < a.splits; ++j) t = OpT::apply(t, load_sc1(&part[r * a.splits + j]));
          out[r] = t;
        }
      }
    }
    __syncthreads();  // lds is rewritten by the next segment
  }
}

// Short rows (every row fits in one vector per lane of its lpr-lane group, lpr < 64): a wave takes
// kRowUnroll batches of 64/lpr consecutive rows per iteration so each lane has kRowUnroll 16-byte
// loads in flight, instead of one load per loop trip.
// ALIGNED (base and row length multiples of 16 bytes): rows are whole vectors — no per-row
// alignment arithmetic or head/tail loops (8 / 64-column bf16 rows: VALU-bound without it).
// PIPE (aligned rows only): two register batches, the next batch's loads issued before the current
// one is folded, so a wave keeps 2 x kRowUnroll vectors in flight across loop trips instead of
// draining to zero at every trip's fold (the single-batch loop waits one full memory latency per
// trip: 2.7 TB/s at one workgroup per CU for 8-column bf16 rows).
template <class OpT, class T, class AccT, bool ALIGNED, bool PIPE = false>
__global__ __launch_bounds__(kDimBlock) void short_rows_kernel(RowArgs a) {
  using V = typename Vec16<T>::type;
  constexpr int N = Vec16<T>::N;
  constexpr int U = kRowUnroll;
  const int lane = threadIdx.x & 63;
  const int lpr = a.lpr;
  const int per_wave = 64 / lpr;
  const int sub = lane / lpr, sl = lane % lpr;
  const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * (kDimBlock / 64) + (threadIdx.x >> 6);
  const uint64_t batch = static_cast<uint64_t>(per_wave) * U;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * (kDimBlock / 64) * batch;
  const T* base = static_cast<const T*>(a.in);
  AccT* out = static_cast<AccT*>(a.out);
  if constexpr (ALIGNED && PIPE) {
    const uint64_t vecs = a.cols / N;
    const V* vbase = reinterpret_cast<const V*>(base);
    auto load = [&](uint64_t row0, V* v) {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const uint64_t r = row0 + static_cast<uint64_t>(j) * per_wave + sub;
        const bool ok = r < a.rows && static_cast<uint64_t>(sl) < vecs;
        v[j] = __builtin_nontemporal_load(ok ? vbase + r * vecs + sl : &g_dummy_vec<V>);
      }
    };
    auto fold = [&](uint64_t row0, const V* v) {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const uint64_t r = row0 + static_cast<uint64_t>(j) * per_wave + sub;
        AccT acc = OpT::template identity<AccT>();
        if (r < a.rows && static_cast<uint64_t>(sl) < vecs) {
#pragma unroll
          for (int k = 0; k < N; ++k) acc = OpT::apply(acc, OpT::pre(elem<T, AccT>(v[j], k)));
        }
        for (int off = lpr >> 1; off > 0; off >>= 1) acc = OpT::apply(acc, __shfl_xor(acc, off, 64));
        if (sl == 0 && r < a.rows) {
          if (a.nt_out) __builtin_nontemporal_store(acc, out + r);  // streaming output, no L2 reuse
          else out[r] = acc;
        }
      }
    };
    uint64_t row0 = wave * batch;
    if (row0 >= a.rows) return;  // wave-uniform; the kernel has no workgroup barrier
    V va[U], vb[U];
    load(row0, va);
    for (;;) {  // wave-uniform trips, unrolled by two so the batches stay in fixed registers
      const uint64_t r1 = row0 + stride;
      if (r1 < a.rows) load(r1, vb);
      __builtin_amdgcn_sched_barrier(0);
      fold(row0, va);
      if (r1 >= a.rows) break;
      const uint64_t r2 = r1 + stride;
      if (r2 < a.rows) load(r2, va);
      __builtin_amdgcn_sched_barrier(0);
      fold(r1, vb);
      if (r2 >= a.rows) break;
      row0 = r2;
    }
    return;
  }
  for (uint64_t row0 = wave * batch; row0 < a.rows; row0 += stride) {  // wave-uniform loop
    // Issue all U loads first, without branches: a lane with no vector in its row (or past the
    // last row) loads the dummy vector instead (a branch per load made hipcc wait for every load
    // before issuing the next).
    V v[U];
    bool has[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t r = row0 + static_cast<uint64_t>(j) * per_wave + sub;
      if constexpr (ALIGNED) {
        const uint64_t vecs = a.cols / N;
        has[j] = r < a.rows && static_cast<uint64_t>(sl) < vecs;
        const V* src = has[j] ? reinterpret_cast<const V*>(base) + r * vecs + sl : &g_dummy_vec<V>;
        v[j] = __builtin_nontemporal_load(src);
      } else {
        const T* p = base + r * a.cols;
        const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
        uint64_t h = addr % 16 ? (16 - addr % 16) / sizeof(T) : 0;
        if (h > a.cols) h = a.cols;
        has[j] = r < a.rows && static_cast<uint64_t>(sl) < (a.cols - h) / N;
        const V* src = has[j] ? reinterpret_cast<const V*>(p + h) + sl : &g_dummy_vec<V>;
        v[j] = __builtin_nontemporal_load(src);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t r = row0 + static_cast<uint64_t>(j) * per_wave + sub;
      AccT acc = OpT::template identity<AccT>();
      if (has[j]) {
#pragma unroll
        for (int k = 0; k < N; ++k) acc = OpT::apply(acc, OpT::pre(elem<T, AccT>(v[j], k)));
      }
      if (!ALIGNED && r < a.rows) {  // scalar head / tail (rows not 16-byte aligned, or lengths not a multiple of N)
        const T* p = base + r * a.cols;
        const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
        uint64_t h = addr % 16 ? (16 - addr % 16) / sizeof(T) : 0;
        if (h > a.cols) h = a.cols;
        for (uint64_t i = sl; i < h; i += lpr) acc = OpT::apply(acc, OpT::pre(static_cast<AccT>(p[i])));
        const uint64_t tb = h + (a.cols - h) / N * N;
        for (uint64_t i = tb + sl; i < a.cols; i += lpr) acc = OpT::apply(acc, OpT::pre(static_cast<AccT>(p[i])));
      }
      for (int off = lpr >> 1; off > 0; off >>= 1) acc = OpT::apply(acc, __shfl_xor(acc, off, 64));
      if (sl == 0 && r < a.rows) out[r] = acc;
    }
  }
}

struct ColArgs {
  const void* in;
  uint64_t rows, cols;      // one [rows, cols] slab
  uint64_t outer;           // slabs (blockIdx.z + z0 indexes them)
  uint64_t z0;
  uint64_t rows_per_split;
  int tpc;    // column threads per workgroup (power of two); kDimBlock / tpc row groups
  void* out;  // splits == 1: the result [outer][cols]; else partials [splits][outer][cols]
};

// VEC: each thread owns N adjacent columns (rows and base 16-byte aligned); else one column.
// A workgroup is G row groups x T column threads (T = a.tpc, a power of two <= 256): narrow slabs
// (few columns) put the spare lanes on interleaved rows instead of idling, and the G partial
// columns are folded through LDS by a fixed pairwise tree (deterministic).
template <class OpT, class T, class AccT, bool VEC>
__global__ __launch_bounds__(kDimBlock) void cols_kernel(ColArgs a) {
  using V = typename Vec16<T>::type;
  constexpr int N = VEC ? Vec16<T>::N : 1;
  __shared__ AccT lds[kDimBlock * N];
  const int tpc = a.tpc;
  const int G = kDimBlock / tpc;
  const int g = threadIdx.x / tpc, tc = threadIdx.x % tpc;
  const uint64_t c0 = (static_cast<uint64_t>(blockIdx.x) * tpc + tc) * N;
  const bool live = c0 < a.cols;
  const uint64_t o = a.z0 + blockIdx.z;
  const uint64_t r0 = static_cast<uint64_t>(blockIdx.y) * a.rows_per_split;
  const uint64_t r1 = std::min<uint64_t>(a.rows, r0 + a.rows_per_split);
  const T* base = static_cast<const T*>(a.in) + o * a.rows * a.cols;
  AccT acc[N];
#pragma unroll
  for (int k = 0; k < N; ++k) acc[k] = OpT::template identity<AccT>();
  if (live) {
    const uint64_t step = static_cast<uint64_t>(G);
    uint64_t r = r0 + g;
    if constexpr (VEC) {
      for (; r + (kColUnroll - 1) * step < r1; r += kColUnroll * step) {
        V v[kColUnroll];
#pragma unroll
        for (int u = 0; u < kColUnroll; ++u)
          v[u] = __builtin_nontemporal_load(reinterpret_cast<const V*>(base + (r + u * step) * a.cols + c0));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < kColUnroll; ++u) {
#pragma unroll
          for (int k = 0; k < N; ++k) acc[k] = OpT::apply(acc[k], OpT::pre(elem<T, AccT>(v[u], k)));
        }
      }
      for (; r < r1; r += step) {
        const V v = __builtin_nontemporal_load(reinterpret_cast<const V*>(base + r * a.cols + c0));
#pragma unroll
        for (int k = 0; k < N; ++k) acc[k] = OpT::apply(acc[k], OpT::pre(elem<T, AccT>(v, k)));
      }
    } else {
      for (; r + (kColUnroll - 1) * step < r1; r += kColUnroll * step) {
        T v[kColUnroll];
#pragma unroll
        for (int u = 0; u < kColUnroll; ++u) v[u] = base[(r + u * step) * a.cols + c0];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < kColUnroll; ++u) acc[0] = OpT::apply(acc[0], OpT::pre(static_cast<AccT>(v[u])));
      }
      for (; r < r1; r += step) acc[0] = OpT::apply(acc[0], OpT::pre(static_cast<AccT>(base[r * a.cols + c0])));
    }
  }
  if (G > 1) {  // fold the G row groups of each column: a fixed pairwise tree through LDS
#pragma unroll
    for (int k = 0; k < N; ++k) lds[threadIdx.x * N + k] = acc[k];
    __syncthreads();
    for (int half = G >> 1; half > 0; half >>= 1) {
      if (g < half) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
          acc[k] = OpT::apply(acc[k], lds[((g + half) * tpc + tc) * N + k]);
          lds[threadIdx.x * N + k] = acc[k];
        }
      }
      __syncthreads();
    }
    if (g != 0) return;
  }
  if (!live) return;
  AccT* out = static_cast<AccT*>(a.out) + (static_cast<uint64_t>(blockIdx.y) * a.outer + o) * a.cols;
#pragma unroll
  for (int k = 0; k < N; ++k) out[c0 + k] = acc[k];
}

// out[c] = op over s of partials[s * cols + c]. A workgroup is SG split groups x CT columns
// (CT = ct, a power of two <= 256): with few columns the splits are spread over the spare lanes
// (split group g takes s = g, g + SG, ...) and folded by a fixed pairwise tree in LDS, so a
// 2048-way split of 8 columns is not one thread walking 2048 dependent loads.
template <class OpT, class AccT>
__global__ __launch_bounds__(kDimBlock) void cols_fold(const AccT* __restrict__ partials, uint64_t splits,
                                                       uint64_t cols, int ct, AccT* __restrict__ out) {
  __shared__ AccT lds[kDimBlock];
  const int SG = kDimBlock / ct;
  const int g = threadIdx.x / ct, tc = threadIdx.x % ct;
  const uint64_t c = static_cast<uint64_t>(blockIdx.x) * ct + tc;
  AccT t = OpT::template identity<AccT>();
  if (c < cols)
    for (uint64_t s = g; s < splits; s += SG) t = OpT::apply(t, partials[s * cols + c]);
  if (SG > 1) {
    lds[threadIdx.x] = t;
    __syncthreads();
    for (int half = SG >> 1; half > 0; half >>= 1) {
      if (g < half) {
        t = OpT::apply(t, lds[(g + half) * ct + tc]);
        lds[threadIdx.x] = t;
      }
      __syncthreads();
    }
  }
  if (g == 0 && c < cols) out[c] = t;
}

}  // namespace kern

// ----------------------------------------------------------------------------------------------
namespace {

constexpr uint64_t kMaxRowSplits = 1024;

uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

struct RowLayout {
  int lpr;
  uint64_t splits, seg_len, waves;
  int grid;
};

constexpr int kMaxResident = 8;  // workgroups per CU assumed by the scratch-size bounds

// Persistent grids are sized to what can be resident at once (a partial second round of
// workgroups would leave most CUs idle at the end: 2048 column-kernel workgroups at 7 resident
// per CU ran 15 % slower than a grid that fits).
template <class K>
int resident_per_cu(K kernel) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, kern::kDimBlock, 0) != hipSuccess || n < 1) n = 1;
  return std::min(n, kMaxResident);
}

RowLayout row_layout(size_t rows, size_t cols, DType t, int num_cus, int resident = kMaxResident) {
  RowLayout L{};
  const uint64_t N = 16 / dtype_size(t);
  const uint64_t vecs = (cols + N - 1) / N;
  const uint64_t target_waves = static_cast<uint64_t>(num_cus) * 16;
  if (vecs <= 32) {  // short rows: a group of lpr lanes per row, 64/lpr rows per wave
    L.lpr = static_cast<int>(next_pow2(std::max<uint64_t>(vecs, 1)));
    L.splits = 1;
  } else {
    L.lpr = 64;  // long rows: a workgroup per segment (rows_kernel)
    const uint64_t min_seg_vecs = static_cast<uint64_t>(kern::kDimBlock) * kern::kRowUnroll;  // one full round
    const uint64_t by_len = std::max<uint64_t>(1, vecs / min_seg_vecs);
    const uint64_t want = rows ? (target_waves + rows - 1) / rows : 1;
    L.splits = std::max<uint64_t>(1, std::min({want, by_len, kMaxRowSplits}));
  }
  L.seg_len = ((cols + L.splits - 1) / L.splits + N - 1) / N * N;
  uint64_t blocks;
  if (L.lpr < 64) {  // short rows: rows per wave trip = (64 / lpr) x kRowUnroll, 4 waves per workgroup
    const uint64_t per_wave = (64 / L.lpr) * kern::kRowUnroll;
    L.waves = (rows + per_wave - 1) / per_wave;
    blocks = (L.waves + 3) / 4;
  } else {  // long rows: one workgroup per segment
    L.waves = rows * L.splits * 4;
    blocks = rows * L.splits;
  }
  L.grid = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(blocks, static_cast<uint64_t>(num_cus) * resident)));
  return L;
}

struct ColLayout {
  bool vec;
  uint64_t threads, splits, rows_per_split;
  int blocks, tpc;
};

ColLayout col_layout(const void* in, size_t outer, size_t rows, size_t cols, DType t, int num_cus,
                     int resident = kMaxResident) {
  ColLayout L{};
  const size_t es = dtype_size(t);
  const uint64_t N = 16 / es;
  L.vec = reinterpret_cast<uintptr_t>(in) % 16 == 0 && (cols * es) % 16 == 0;
  L.threads = L.vec ? cols / N : cols;
  L.tpc = static_cast<int>(std::min<uint64_t>(kern::kDimBlock, next_pow2(std::max<uint64_t>(L.threads, 1))));
  L.blocks = static_cast<int>((L.threads + L.tpc - 1) / L.tpc);
  const uint64_t G = kern::kDimBlock / L.tpc;  // row groups share a workgroup's columns
  const uint64_t target = static_cast<uint64_t>(num_cus) * resident;  // resident workgroups
  const uint64_t all = static_cast<uint64_t>(L.blocks) * outer;
  uint64_t splits = all ? target / all : 1;
  splits = std::max<uint64_t>(1, std::min<uint64_t>({splits, (rows + 16 * G - 1) / (16 * G), 65535}));
  L.rows_per_split = rows ? (rows + splits - 1) / splits : 1;
  L.splits = rows ? (rows + L.rows_per_split - 1) / L.rows_per_split : 1;
  return L;
}

// Resident workgroups per CU the persistent grids are sized for. Measured (tools/dim_wg_sweep.sh,
// profiles/r1_session3/reduce_dim/wg_sweep_bf16.txt, 4 GB bf16): column reductions stream best
// with ONE workgroup per CU (488281 x 4096: 4.6 -> 6.8 TB/s; fewer concurrent DRAM streams, as in
// the full reduction), long rows of >= 64 KB with two (30517 x 65536: 6.9 -> 7.2), shorter rows
// need the occupancy limit (a workgroup per 8 KB row has little in flight).
// MIREDUCE_DIM_WG_PER_CU=k overrides every choice (A/B runs).
int wg_cap(int occ, int preferred) {
  static const int env = [] {
    const char* e = std::getenv("MIREDUCE_DIM_WG_PER_CU");
    return e ? std::atoi(e) : 0;
  }();
  const int cap = env > 0 ? env : preferred;
  return cap > 0 ? std::min(occ, cap) : occ;
}

// Aligned short rows: the two-batch pipelined loop (short_rows_kernel PIPE). MIREDUCE_DIM_SHORT_PIPE=0
// selects the single-batch loop (A/B runs).
bool short_pipe() {
  static const bool on = [] {
    const char* e = std::getenv("MIREDUCE_DIM_SHORT_PIPE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Pipelined short rows: MIREDUCE_DIM_NT_OUT=1 writes the results with non-temporal stores (one
// AccT per row is up to a quarter of the traffic at 8 columns); plain stores by default until an
// A/B on the GPU says otherwise (tools/gpu/r3zb.sh).
bool short_nt_out() {
  static const bool on = [] {
    const char* e = std::getenv("MIREDUCE_DIM_NT_OUT");
    return e && e[0] == '1';
  }();
  return on;
}

using RowFn = void (*)(const kern::RowArgs&, int, hipStream_t);
using OccFn = int (*)(bool);  // resident workgroups per CU of the (short-row | vector) variant
using ColFn = void (*)(const kern::ColArgs&, dim3, bool, hipStream_t);
using FoldFn = void (*)(const void*, uint64_t, uint64_t, void*, hipStream_t);

template <class OpT, class T, class AccT>
void launch_rows(const kern::RowArgs& a, int grid, hipStream_t s) {
  if (a.lpr < 64 && a.aligned && short_pipe())
    hipLaunchKernelGGL((kern::short_rows_kernel<OpT, T, AccT, true, true>), dim3(grid), dim3(kern::kDimBlock), 0, s, a);
  else if (a.lpr < 64 && a.aligned)
    hipLaunchKernelGGL((kern::short_rows_kernel<OpT, T, AccT, true>), dim3(grid), dim3(kern::kDimBlock), 0, s, a);
  else if (a.lpr < 64)
    hipLaunchKernelGGL((kern::short_rows_kernel<OpT, T, AccT, false>), dim3(grid), dim3(kern::kDimBlock), 0, s, a);
  else
    hipLaunchKernelGGL((kern::rows_kernel<OpT, T, AccT>), dim3(grid), dim3(kern::kDimBlock), 0, s, a);
}

template <class OpT, class T, class AccT>
void launch_cols(const kern::ColArgs& a, dim3 grid, bool vec, hipStream_t s) {
  if (vec)
    hipLaunchKernelGGL((kern::cols_kernel<OpT, T, AccT, true>), grid, dim3(kern::kDimBlock), 0, s, a);
  else
    hipLaunchKernelGGL((kern::cols_kernel<OpT, T, AccT, false>), grid, dim3(kern::kDimBlock), 0, s, a);
}

template <class OpT, class AccT>
void launch_fold(const void* partials, uint64_t splits, uint64_t cols, void* out, hipStream_t s) {
  const int ct = static_cast<int>(std::min<uint64_t>(kern::kDimBlock, next_pow2(std::max<uint64_t>(cols, 1))));
  const unsigned blocks = static_cast<unsigned>((cols + ct - 1) / ct);
  hipLaunchKernelGGL((kern::cols_fold<OpT, AccT>), dim3(blocks), dim3(kern::kDimBlock), 0, s,
                     static_cast<const AccT*>(partials), splits, cols, ct, static_cast<AccT*>(out));
}

template <class OpT, class T, class AccT>
int rows_resident(bool short_rows) {
  static const int s = std::min(resident_per_cu(kern::short_rows_kernel<OpT, T, AccT, false>),
                                resident_per_cu(kern::short_rows_kernel<OpT, T, AccT, true, true>));
  static const int l = resident_per_cu(kern::rows_kernel<OpT, T, AccT>);
  return short_rows ? s : l;
}

template <class OpT, class T, class AccT>
int cols_resident(bool vec) {
  static const int v = resident_per_cu(kern::cols_kernel<OpT, T, AccT, true>);
  static const int sc = resident_per_cu(kern::cols_kernel<OpT, T, AccT, false>);
  return vec ? v : sc;
}

struct DimEntry {
  RowFn rows;
  ColFn cols;
  FoldFn fold;
  OccFn rows_occ;
  OccFn cols_occ;
};

template <class OpT, class T, class AccT>
constexpr DimEntry entry() {
  return {launch_rows<OpT, T, AccT>, launch_cols<OpT, T, AccT>, launch_fold<OpT, AccT>,
          rows_resident<OpT, T, AccT>, cols_resident<OpT, T, AccT>};
}

// (op, dtype, acc) -> kernels; the same 20 combinations as the full reduction.
DimEntry lookup(Op op, DType t, DType acc) {
  MIREDUCE_REQUIRE(acc_supported(t, op, acc), "unsupported (dtype, op, accumulator) combination");
#define MIREDUCE_DIM(OPV, OPT)                                                                        \
  if (op == OPV) {                                                                                    \
    switch (t) {                                                                                      \
      case DType::Int32: return acc == DType::Int64 ? entry<OPT, int32_t, int64_t>() : entry<OPT, int32_t, int32_t>(); \
      case DType::Int64: return entry<OPT, int64_t, int64_t>();                                       \
      case DType::Float32: return acc == DType::Float64 ? entry<OPT, float, double>() : entry<OPT, float, float>(); \
      case DType::Float64: return entry<OPT, double, double>();                                       \
      case DType::BFloat16: return entry<OPT, bf16_t, float>();                                       \
      case DType::Float16: return entry<OPT, f16_t, float>();                                         \
    }                                                                                                 \
  }
  MIREDUCE_DIM(Op::Sum, SumOp)
  MIREDUCE_DIM(Op::Min, MinOp)
  MIREDUCE_DIM(Op::Max, MaxOp)
#undef MIREDUCE_DIM
  // fused ops: floating types only (acc_supported)
  if (op == Op::SumSq) {
    switch (t) {
      case DType::Float32: return acc == DType::Float64 ? entry<SumSqOp, float, double>() : entry<SumSqOp, float, float>();
      case DType::Float64: return entry<SumSqOp, double, double>();
      case DType::BFloat16: return entry<SumSqOp, bf16_t, float>();
      case DType::Float16: return entry<SumSqOp, f16_t, float>();
      default: break;
    }
  }
  if (op == Op::AbsMax) {
    switch (t) {
      case DType::Float32: return entry<AbsMaxOp, float, float>();
      case DType::Float64: return entry<AbsMaxOp, double, double>();
      case DType::BFloat16: return entry<AbsMaxOp, bf16_t, float>();
      case DType::Float16: return entry<AbsMaxOp, f16_t, float>();
      default: break;
    }
  }
  throw Error("reduce_dim: unsupported combination");
}

}  // namespace

// Rows split only when rows < num_cus x 16 (row_layout's target_waves), so every split launch's
// per-row tickets fit one fixed region at the start of the scratch; the partials always start
// after it (a row-count-dependent boundary let a later, taller launch read an earlier launch's
// partial bits as tickets — the kernels leave only the ticket words zero).
size_t row_ticket_region_bytes(int num_cus) {
  return (static_cast<size_t>(num_cus) * 16 * sizeof(unsigned) + 255) / 256 * 256;
}

size_t reduce_rows_scratch_bytes(size_t rows, size_t cols, DType t, int num_cus) {
  const RowLayout L = row_layout(rows, cols, t, num_cus);
  if (L.splits <= 1) return 0;
  return row_ticket_region_bytes(num_cus) + rows * L.splits * 8;
}

size_t reduce_cols_scratch_bytes(size_t outer, size_t rows, size_t cols, DType t, DType acc, int num_cus) {
  // An aligned base (vector layout: fewer threads, so the most row splits) bounds every base.
  const ColLayout L = col_layout(nullptr, outer, rows, cols, t, num_cus);
  return L.splits > 1 ? L.splits * outer * cols * dtype_size(acc) : 0;
}

DimPlan reduce_rows(const void* in, size_t rows, size_t cols, DType t, Op op, DType acc, void* out,
                    void* scratch, int num_cus, hipStream_t stream) {
  const DimEntry e = lookup(op, t, acc);
  MIREDUCE_REQUIRE(out != nullptr, "reduce_rows: output pointer is null");
  MIREDUCE_REQUIRE(reinterpret_cast<uintptr_t>(in) % dtype_size(t) == 0, "reduce_rows: misaligned input");
  DimPlan plan;
  if (rows == 0) return plan;
  const bool short_rows = row_layout(rows, cols, t, num_cus).lpr < 64;
  const bool long_rows = !short_rows && cols * dtype_size(t) >= 65536;
  const RowLayout L = row_layout(rows, cols, t, num_cus, wg_cap(e.rows_occ(short_rows), long_rows ? 2 : 0));
  kern::RowArgs a{};
  a.in = in;
  a.rows = rows;
  a.cols = cols;
  a.splits = L.splits;
  a.seg_len = L.seg_len;
  a.lpr = L.lpr;
  a.aligned = reinterpret_cast<uintptr_t>(in) % 16 == 0 && (cols * dtype_size(t)) % 16 == 0;
  a.out = out;
  a.nt_out = short_nt_out() ? 1 : 0;
  if (L.splits > 1) {
    MIREDUCE_REQUIRE(scratch != nullptr, "reduce_rows: this shape needs scratch (reduce_rows_scratch_bytes)");
    MIREDUCE_REQUIRE(rows < static_cast<size_t>(num_cus) * 16, "reduce_rows: split rows exceed the ticket region");
    a.tickets = static_cast<unsigned*>(scratch);
    a.partials = static_cast<char*>(scratch) + row_ticket_region_bytes(num_cus);
  }
  e.rows(a, L.grid, stream);
  MIREDUCE_HIP_THROW(hipGetLastError());
  plan.grid = L.grid;
  plan.lanes_per_row = L.lpr;
  plan.splits = L.splits;
  return plan;
}

DimPlan reduce_cols(const void* in, size_t outer, size_t rows, size_t cols, DType t, Op op, DType acc, void* out,
                    void* scratch, int num_cus, hipStream_t stream) {
  const DimEntry e = lookup(op, t, acc);
  MIREDUCE_REQUIRE(out != nullptr, "reduce_cols: output pointer is null");
  MIREDUCE_REQUIRE(reinterpret_cast<uintptr_t>(in) % dtype_size(t) == 0, "reduce_cols: misaligned input");
  DimPlan plan;
  if (cols == 0 || outer == 0) return plan;
  MIREDUCE_REQUIRE(rows > 0, "reduce_cols: empty reduction axis");
  const bool vec = col_layout(in, outer, rows, cols, t, num_cus).vec;
  const ColLayout L = col_layout(in, outer, rows, cols, t, num_cus, wg_cap(e.cols_occ(vec), 1));
  kern::ColArgs a{};
  a.in = in;
  a.rows = rows;
  a.cols = cols;
  a.outer = outer;
  a.rows_per_split = L.rows_per_split;
  a.tpc = L.tpc;
  if (L.splits > 1) {
    MIREDUCE_REQUIRE(scratch != nullptr, "reduce_cols: this shape needs scratch (reduce_cols_scratch_bytes)");
    a.out = scratch;
  } else {
    a.out = out;
  }
  constexpr uint64_t kMaxZ = 65535;
  for (uint64_t z0 = 0; z0 < outer; z0 += kMaxZ) {  // grid.z indexes slabs
    a.z0 = z0;
    const unsigned nz = static_cast<unsigned>(std::min<uint64_t>(kMaxZ, outer - z0));
    e.cols(a, dim3(static_cast<unsigned>(std::max(L.blocks, 1)), static_cast<unsigned>(L.splits), nz), L.vec, stream);
    MIREDUCE_HIP_THROW(hipGetLastError());
  }
  if (L.splits > 1) {
    e.fold(scratch, L.splits, outer * cols, out, stream);
    MIREDUCE_HIP_THROW(hipGetLastError());
  }
  plan.grid = static_cast<int>(std::min<uint64_t>(INT32_MAX, static_cast<uint64_t>(std::max(L.blocks, 1)) * L.splits * outer));
  plan.splits = L.splits;
  plan.lanes_per_row = L.vec ? static_cast<int>(16 / dtype_size(t)) : 1;
  return plan;
}

}  // namespace mireduce
