// Arg-reductions (first index of the max / min, and its value); see arg_reduce.hpp.
//
// Long rows (and whole arrays: rows = 1) use the streaming shape of reduce_dim.hip's rows_kernel:
// one workgroup per row *segment*, 16-byte nt loads, kArgUnroll vectors in flight per lane, per-row
// tickets when a row is split. What an index adds is kept out of the hot loop: a lane keeps P*N
// running bests (one per vector slot k, P slot groups) together with the 32-bit *trip number* at
// which each improved — within one slot the trips visit strictly increasing indices, so a strict
// comparison keeps the first occurrence and costs one compare + two selects per element. Slot
// bests become (value, index) pairs only once per segment; pairs fold with
// "better value, or same value and smaller index" (NaN the extreme, first NaN wins), which is a
// total order, so the cross-lane butterflies, the workgroup fold and the fold of a split row's
// segment partials (by all 256 lanes of the last-arriving workgroup) give the same answer in any
// order.
//
// Short rows (<= 256 columns, e.g. router logits over experts) use lane groups: lpr lanes per row,
// each lane reading M scalar elements per row, kArgUnroll batches of rows per wave trip, all
// loads issued branch-free (lanes past the end read a dummy) before the first compare.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <limits>
#include <type_traits>

#include "mireduce/arg_reduce.hpp"
#include "mireduce/check.hpp"
#include "mireduce/half.hpp"
#include "mireduce/vec16.hpp"

namespace mireduce {
namespace kern {

constexpr int kArgBlock = 256;
constexpr int kArgUnroll = 8;      // short rows: row batches per wave trip
constexpr int kArgLongUnroll = 4;  // long rows: default vectors in flight per lane (tile = U x 256)
constexpr int64_t kNoIndex = std::numeric_limits<int64_t>::max();
constexpr uint32_t kNoTrip = 0xffffffffu;
constexpr uint32_t kNoIndex32 = 0xffffffffu;  // short rows index within the row in 32 bits

// Comparison domain: 16-bit floats compare as fp32, everything else as itself.
template <class T> struct ArgKey { using type = T; };
template <> struct ArgKey<bf16_t> { using type = float; };
template <> struct ArgKey<f16_t> { using type = float; };

template <bool MAX, class K>
struct ArgCmp {
  static constexpr bool kFloat = std::is_floating_point_v<K>;
  __device__ static K identity() {
    if constexpr (kFloat) return MAX ? -static_cast<K>(__builtin_huge_val()) : static_cast<K>(__builtin_huge_val());
    else return MAX ? std::numeric_limits<K>::lowest() : std::numeric_limits<K>::max();
  }
  // x strictly beats the running best b: NaN beats every number, nothing beats a NaN best.
  __device__ static bool beats(K x, K b) {
    if constexpr (kFloat) return (MAX ? !(x <= b) : !(x >= b)) && b == b;
    else return MAX ? x > b : x < b;
  }
  __device__ static bool same(K a, K b) {
    if constexpr (kFloat) return a == b || (a != a && b != b);
    else return a == b;
  }
  template <class I>
  __device__ static bool pair_beats(K a, I ia, K b, I ib) { return beats(a, b) || (same(a, b) && ia < ib); }
};

template <class T, class K>
__device__ __forceinline__ K load_key(const T* q) {
  if constexpr (std::is_same_v<T, bf16_t>) return bf16_bits_to_float(*reinterpret_cast<const uint16_t*>(q));
  else if constexpr (std::is_same_v<T, f16_t>)
    return static_cast<float>(__builtin_bit_cast(_Float16, *reinterpret_cast<const uint16_t*>(q)));
  else return *q;
}

template <class T, class K>
__device__ __forceinline__ T key_to_elem(K v) {
  if constexpr (std::is_same_v<T, bf16_t>) return bf16_t{float_to_bf16_bits(v)};  // exact: v came from a bf16
  else if constexpr (std::is_same_v<T, f16_t>) return f16_t{float_to_f16_bits(v)};
  else return v;
}

template <class K>
__device__ __forceinline__ uint64_t key_bits(K v) {
  uint64_t b = 0;
  __builtin_memcpy(&b, &v, sizeof(K));
  return b;
}

template <class K>
__device__ __forceinline__ K bits_key(uint64_t b) {
  K v;
  __builtin_memcpy(&v, &b, sizeof(K));
  return v;
}

struct ArgArgs {
  const void* in;
  uint64_t rows, cols;
  uint64_t splits;    // workgroups per row (long rows)
  int lpr;            // short rows: lanes per row
  void* out_value;
  int64_t* out_index;
  uint64_t* partials; // [rows * splits][2]: value bits, index (splits > 1)
  unsigned* tickets;  // [rows] (splits > 1)
};

template <class T>
__device__ T g_arg_dummy;  // readable target of the short-row loads past a row's end

// Pair fold across the lanes of a wave (xor butterfly over offsets < width).
template <bool MAX, class K, class I = int64_t>
__device__ __forceinline__ void wave_fold(K& v, I& i, int width) {
  using C = ArgCmp<MAX, K>;
  for (int off = width >> 1; off > 0; off >>= 1) {
    const K ov = __shfl_xor(v, off, 64);
    const I oi = __shfl_xor(i, off, 64);
    if (C::pair_beats(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
}

// Pair fold across the workgroup; the result is valid in thread 0.
template <bool MAX, class K>
__device__ __forceinline__ void block_fold(K& v, int64_t& i, K* lv, int64_t* li) {
  using C = ArgCmp<MAX, K>;
  constexpr int kWaves = kArgBlock / 64;
  const int tid = threadIdx.x;
  wave_fold<MAX, K>(v, i, 64);
  if ((tid & 63) == 0) {
    lv[tid >> 6] = v;
    li[tid >> 6] = i;
  }
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int w = 1; w < kWaves; ++w)
      if (C::pair_beats(lv[w], li[w], v, i)) {
        v = lv[w];
        i = li[w];
      }
  }
}

template <class V>
__device__ V g_arg_dummy_vec;  // readable 16 bytes for predicated-off vector loads

// Row batches per wave trip of the 16-byte short-row kernel: M x batches vectors in flight per lane.
constexpr int short_vec_batches(int m) { return m >= 4 ? 4 : kArgUnroll; }

// Long rows: the `splits` workgroups of a row interleave over its tiles of kArgUnroll x kArgBlock
// vectors (workgroup s takes tiles s, s + splits, ...), so at any moment the grid streams one
// contiguous window of the array — the access order of the full reduction. The last, partial tile
// is loaded predicated (lanes past the end read a dummy) by the workgroup whose turn it is.
template <bool MAX, class T, int U>
__global__ __launch_bounds__(kArgBlock) void arg_rows_kernel(ArgArgs a) {
  using K = typename ArgKey<T>::type;
  using C = ArgCmp<MAX, K>;
  using V = typename Vec16<T>::type;
  constexpr int N = Vec16<T>::N;
  constexpr uint64_t kTile = static_cast<uint64_t>(U) * kArgBlock;  // vectors per tile
  constexpr int P = N >= 8 ? 1 : (8 / N < U ? 8 / N : U);  // slot groups: P * N running bests per lane
  static_assert(U % P == 0, "slot groups must divide the unroll");
  constexpr int kWaves = kArgBlock / 64;
  __shared__ K lv[kWaves];
  __shared__ int64_t li[kWaves];
  __shared__ int last;
  const int tid = threadIdx.x;
  const uint64_t S = a.splits;
  const uint64_t nseg = a.rows * S;
  const T* base = static_cast<const T*>(a.in);
  for (uint64_t seg = blockIdx.x; seg < nseg; seg += gridDim.x) {  // workgroup-uniform
    const uint64_t r = seg / S;
    const uint64_t s = seg % S;
    const T* p = base + r * a.cols;
    const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
    uint64_t head = addr % 16 ? (16 - addr % 16) / sizeof(T) : 0;
    if (head > a.cols) head = a.cols;
    const uint64_t nvec = (a.cols - head) / N;
    const uint64_t tb = head + nvec * N;  // scalar tail [tb, cols)
    const uint64_t nfull = nvec / kTile, ntiles = (nvec + kTile - 1) / kTile;
    const V* vp = reinterpret_cast<const V*>(p + head);
    K bv = C::identity();
    int64_t bi = kNoIndex;
    if (s == 0 && static_cast<uint64_t>(tid) < head) {
      bv = load_key<T, K>(p + tid);
      bi = tid;
    }
    K best[P][N];
    uint32_t trip[P][N];  // q = m * U + u: the u-th vector of this workgroup's m-th tile
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
      for (int k = 0; k < N; ++k) {
        best[q][k] = C::identity();
        trip[q][k] = kNoTrip;
      }
    uint64_t tile = s;
    uint32_t m = 0;
    for (; tile < nfull; tile += S, ++m) {
      const V* tp = vp + tile * kTile + tid;
      V v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(tp + static_cast<uint64_t>(u) * kArgBlock);
      __builtin_amdgcn_sched_barrier(0);  // all loads out before the first compare
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const K x = elem<T, K>(v[u], k);
          const bool w = C::beats(x, best[u % P][k]);
          best[u % P][k] = w ? x : best[u % P][k];
          trip[u % P][k] = w ? m * U + u : trip[u % P][k];
        }
      }
    }
    if (tile < ntiles) {  // the partial last tile is this workgroup's turn
      const uint64_t j0 = tile * kTile + tid;
      V v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t j = j0 + static_cast<uint64_t>(u) * kArgBlock;
        v[u] = __builtin_nontemporal_load(j < nvec ? vp + j : &g_arg_dummy_vec<V>);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = j0 + static_cast<uint64_t>(u) * kArgBlock < nvec;
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const K x = elem<T, K>(v[u], k);
          const bool w = ok && C::beats(x, best[u % P][k]);
          best[u % P][k] = w ? x : best[u % P][k];
          trip[u % P][k] = w ? m * U + u : trip[u % P][k];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
      for (int k = 0; k < N; ++k) {
        if (trip[q][k] == kNoTrip) continue;
        const uint64_t mt = trip[q][k] / U, u = trip[q][k] % U;
        const uint64_t j = (s + mt * S) * kTile + u * kArgBlock + tid;
        const int64_t idx = static_cast<int64_t>(head + j * N + k);
        if (C::pair_beats(best[q][k], idx, bv, bi)) {
          bv = best[q][k];
          bi = idx;
        }
      }
    if (s == S - 1 && static_cast<uint64_t>(tid) < a.cols - tb) {
      const K x = load_key<T, K>(p + tb + tid);
      const int64_t idx = static_cast<int64_t>(tb + tid);
      if (C::pair_beats(x, idx, bv, bi)) {
        bv = x;
        bi = idx;
      }
    }
    block_fold<MAX, K>(bv, bi, lv, li);
    if (S == 1) {
      if (tid == 0) {
        // no element registered: every element of the row equals the identity -> index 0
        static_cast<T*>(a.out_value)[r] = key_to_elem<T, K>(bv);
        a.out_index[r] = bi == kNoIndex ? 0 : bi;
      }
    } else {
      if (tid == 0) {
        store_sc1(&a.partials[2 * seg], key_bits(bv));
        store_sc1(&a.partials[2 * seg + 1], static_cast<uint64_t>(bi));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(&a.tickets[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == S - 1;
        if (last) __hip_atomic_store(&a.tickets[r], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (last) {  // last workgroup of row r: every lane folds a share of the row's partials
        K fv = C::identity();
        int64_t fi = kNoIndex;
        const uint64_t* part = a.partials + 2 * r * S;
        for (uint64_t j = tid; j < S; j += kArgBlock) {
          const K v = bits_key<K>(load_sc1(&part[2 * j]));
          const int64_t ix = static_cast<int64_t>(load_sc1(&part[2 * j + 1]));
          if (C::pair_beats(v, ix, fv, fi)) {
            fv = v;
            fi = ix;
          }
        }
        block_fold<MAX, K>(fv, fi, lv, li);
        if (tid == 0) {
          static_cast<T*>(a.out_value)[r] = key_to_elem<T, K>(fv);
          a.out_index[r] = fi == kNoIndex ? 0 : fi;
        }
      }
    }
    __syncthreads();  // lv/li/last are rewritten by the next segment
  }
}

// Medium rows (a few KB to tens of KB): one wave per row, no LDS and no barriers — tiles of
// U x 64 vectors, the same slot/trip bookkeeping as the long-row kernel, a 64-lane butterfly.
template <bool MAX, class T, int U>
__global__ __launch_bounds__(kArgBlock) void arg_wave_rows_kernel(ArgArgs a) {
  using K = typename ArgKey<T>::type;
  using C = ArgCmp<MAX, K>;
  using V = typename Vec16<T>::type;
  constexpr int N = Vec16<T>::N;
  constexpr uint64_t kTile = static_cast<uint64_t>(U) * 64;
  constexpr int P = N >= 8 ? 1 : (8 / N < U ? 8 / N : U);
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (static_cast<uint64_t>(blockIdx.x) * kArgBlock + threadIdx.x) / 64;
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kArgBlock / 64);
  const T* base = static_cast<const T*>(a.in);
  for (uint64_t r = wave; r < a.rows; r += nwaves) {  // wave-uniform
    const T* p = base + r * a.cols;
    const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
    uint64_t head = addr % 16 ? (16 - addr % 16) / sizeof(T) : 0;
    if (head > a.cols) head = a.cols;
    const uint64_t nvec = (a.cols - head) / N;
    const uint64_t tb = head + nvec * N;
    const uint64_t nfull = nvec / kTile;
    const V* vp = reinterpret_cast<const V*>(p + head);
    K bv = C::identity();
    int64_t bi = kNoIndex;
    if (static_cast<uint64_t>(lane) < head) {
      bv = load_key<T, K>(p + lane);
      bi = lane;
    }
    K best[P][N];
    uint32_t trip[P][N];  // q = tile * U + u: vector q * 64 + lane
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
      for (int k = 0; k < N; ++k) {
        best[q][k] = C::identity();
        trip[q][k] = kNoTrip;
      }
    uint32_t tile = 0;
    for (; tile < nfull; ++tile) {
      const V* tp = vp + tile * kTile + lane;
      V v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(tp + u * 64);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const K x = elem<T, K>(v[u], k);
          const bool w = C::beats(x, best[u % P][k]);
          best[u % P][k] = w ? x : best[u % P][k];
          trip[u % P][k] = w ? tile * U + u : trip[u % P][k];
        }
      }
    }
    if (static_cast<uint64_t>(tile) * kTile < nvec) {  // partial last tile, predicated
      const uint64_t j0 = static_cast<uint64_t>(tile) * kTile + lane;
      V v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t j = j0 + static_cast<uint64_t>(u) * 64;
        v[u] = __builtin_nontemporal_load(j < nvec ? vp + j : &g_arg_dummy_vec<V>);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = j0 + static_cast<uint64_t>(u) * 64 < nvec;
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const K x = elem<T, K>(v[u], k);
          const bool w = ok && C::beats(x, best[u % P][k]);
          best[u % P][k] = w ? x : best[u % P][k];
          trip[u % P][k] = w ? tile * U + u : trip[u % P][k];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
      for (int k = 0; k < N; ++k) {
        if (trip[q][k] == kNoTrip) continue;
        const int64_t idx = static_cast<int64_t>(head + (static_cast<uint64_t>(trip[q][k]) * 64 + lane) * N + k);
        if (C::pair_beats(best[q][k], idx, bv, bi)) {
          bv = best[q][k];
          bi = idx;
        }
      }
    if (static_cast<uint64_t>(lane) < a.cols - tb) {
      const K x = load_key<T, K>(p + tb + lane);
      const int64_t idx = static_cast<int64_t>(tb + lane);
      if (C::pair_beats(x, idx, bv, bi)) {
        bv = x;
        bi = idx;
      }
    }
    wave_fold<MAX, K>(bv, bi, 64);
    if (lane == 0) {
      static_cast<T*>(a.out_value)[r] = key_to_elem<T, K>(bv);
      a.out_index[r] = bi == kNoIndex ? 0 : bi;
    }
  }
}

// Short 16-byte-aligned rows (cols * sizeof(T) a multiple of 16, at most lpr * M vectors): lpr
// lanes per row, each lane M 16-byte vectors per row, kArgUnroll batches of (64 / lpr) rows per
// wave trip, all loads issued before the first compare.
template <bool MAX, class T, int M>
__global__ __launch_bounds__(kArgBlock) void arg_short_vec_kernel(ArgArgs a) {
  using K = typename ArgKey<T>::type;
  using C = ArgCmp<MAX, K>;
  using V = typename Vec16<T>::type;
  constexpr int N = Vec16<T>::N;
  constexpr int U = short_vec_batches(M);
  const int lane = threadIdx.x & 63;
  const int lpr = a.lpr;
  const int per_wave = 64 / lpr;
  const int sub = lane / lpr, sl = lane % lpr;
  const uint64_t vecs = a.cols / N;
  const uint64_t wave = (static_cast<uint64_t>(blockIdx.x) * kArgBlock + threadIdx.x) / 64;
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kArgBlock / 64);
  const uint64_t per_trip = static_cast<uint64_t>(per_wave) * U;
  const V* base = static_cast<const V*>(a.in);
  for (uint64_t r0 = wave * per_trip; r0 < a.rows; r0 += nwaves * per_trip) {  // wave-uniform
    V v[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t r = r0 + static_cast<uint64_t>(u) * per_wave + sub;
#pragma unroll
      for (int mm = 0; mm < M; ++mm) {
        const uint64_t c = static_cast<uint64_t>(sl) + static_cast<uint64_t>(mm) * lpr;
        const bool ok = r < a.rows && c < vecs;
        v[u][mm] = __builtin_nontemporal_load(ok ? base + r * vecs + c : &g_arg_dummy_vec<V>);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // all loads out before the first compare
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t r = r0 + static_cast<uint64_t>(u) * per_wave + sub;
      K bv = C::identity();
      uint32_t bi = kNoIndex32;
#pragma unroll
      for (int mm = 0; mm < M; ++mm) {
        const uint64_t c = static_cast<uint64_t>(sl) + static_cast<uint64_t>(mm) * lpr;
        const bool ok = c < vecs;
#pragma unroll
        for (int k = 0; k < N; ++k) {  // indices increase with mm and k: strict keeps the first
          const K x = elem<T, K>(v[u][mm], k);
          if (ok && C::beats(x, bv)) {
            bv = x;
            bi = static_cast<uint32_t>(c * N + k);
          }
        }
      }
      wave_fold<MAX, K, uint32_t>(bv, bi, lpr);
      if (sl == 0 && r < a.rows) {
        static_cast<T*>(a.out_value)[r] = key_to_elem<T, K>(bv);
        a.out_index[r] = bi == kNoIndex32 ? 0 : static_cast<int64_t>(bi);
      }
    }
  }
}

// Short rows: cols <= lpr * M. A wave covers (64 / lpr) rows per batch and kArgUnroll batches per
// trip; lane sl of a row group reads columns sl, sl + lpr, ... (M of them).
template <bool MAX, class T, int M>
__global__ __launch_bounds__(kArgBlock) void arg_short_kernel(ArgArgs a) {
  using K = typename ArgKey<T>::type;
  using C = ArgCmp<MAX, K>;
  constexpr int U = kArgUnroll;
  const int lane = threadIdx.x & 63;
  const int lpr = a.lpr;
  const int per_wave = 64 / lpr;
  const int sub = lane / lpr, sl = lane % lpr;
  const uint64_t wave = (static_cast<uint64_t>(blockIdx.x) * kArgBlock + threadIdx.x) / 64;
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * (kArgBlock / 64);
  const uint64_t per_trip = static_cast<uint64_t>(per_wave) * U;
  const T* base = static_cast<const T*>(a.in);
  for (uint64_t r0 = wave * per_trip; r0 < a.rows; r0 += nwaves * per_trip) {  // wave-uniform
    K x[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t r = r0 + static_cast<uint64_t>(u) * per_wave + sub;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const uint64_t c = static_cast<uint64_t>(sl) + static_cast<uint64_t>(m) * lpr;
        const bool ok = r < a.rows && c < a.cols;
        x[u][m] = load_key<T, K>(ok ? base + r * a.cols + c : &g_arg_dummy<T>);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // all loads out before the first compare
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t r = r0 + static_cast<uint64_t>(u) * per_wave + sub;
      K bv = C::identity();
      uint32_t bi = kNoIndex32;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const uint64_t c = static_cast<uint64_t>(sl) + static_cast<uint64_t>(m) * lpr;
        if (c < a.cols && C::beats(x[u][m], bv)) {  // columns increase with m: strict keeps the first
          bv = x[u][m];
          bi = static_cast<uint32_t>(c);
        }
      }
      wave_fold<MAX, K, uint32_t>(bv, bi, lpr);
      if (sl == 0 && r < a.rows) {
        static_cast<T*>(a.out_value)[r] = key_to_elem<T, K>(bv);
        a.out_index[r] = bi == kNoIndex32 ? 0 : static_cast<int64_t>(bi);
      }
    }
  }
}

// Cross-rank MAXLOC / MINLOC pairs (arg_reduce.hpp loc_pack / loc_pick): one thread each.
template <class T>
__global__ void loc_pack_kernel(const T* __restrict__ value, const int64_t* __restrict__ index, int64_t offset,
                                uint64_t* __restrict__ pair) {
  using K = typename ArgKey<T>::type;
  pair[0] = key_bits(load_key<T, K>(value));
  pair[1] = static_cast<uint64_t>(index[0] + offset);
}

template <bool MAX, class T>
__global__ void loc_pick_kernel(const uint64_t* __restrict__ pairs, int world, int64_t* __restrict__ out_index,
                                T* __restrict__ out_value) {
  using K = typename ArgKey<T>::type;
  using C = ArgCmp<MAX, K>;
  K bv = bits_key<K>(pairs[0]);
  int64_t bi = static_cast<int64_t>(pairs[1]);
  for (int r = 1; r < world; ++r) {
    const K v = bits_key<K>(pairs[2 * r]);
    const int64_t i = static_cast<int64_t>(pairs[2 * r + 1]);
    if (C::pair_beats(v, i, bv, bi)) {
      bv = v;
      bi = i;
    }
  }
  out_index[0] = bi;
  if (out_value) out_value[0] = key_to_elem<T, K>(bv);
}

}  // namespace kern

namespace {

constexpr int kMaxResident = 8;
constexpr uint64_t kMaxArgSplits = 4096;
constexpr uint64_t kShortCols = 256;        // scalar lane-group rows (any alignment)
constexpr uint64_t kShortVecBytes = 4096;   // 16-byte lane-group rows (aligned)
constexpr uint64_t kWaveRowBytes = 65536;   // wave-per-row rows

uint64_t next_pow2_u(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

// Kernel variants: 0 long rows; 1, 2, 4 scalar short rows (M columns per lane); 11, 12 vector
// short rows (M = 1, 2, 4 vectors per lane); 20 medium rows (a wave per row).
enum Variant : int { kLong = 0, kScalar1 = 1, kScalar2 = 2, kScalar4 = 4, kVec1 = 11, kVec2 = 12, kVec4 = 14, kWave = 20 };

int variant_of(const void* in, uint64_t cols, DType t) {
  const uint64_t es = dtype_size(t), bytes = cols * es;
  if (reinterpret_cast<uintptr_t>(in) % 16 == 0 && bytes % 16 == 0 && bytes <= kShortVecBytes)
    return bytes / 16 <= 64 ? kVec1 : bytes / 16 <= 128 ? kVec2 : kVec4;
  if (cols <= kShortCols) return cols <= 64 ? kScalar1 : cols <= 128 ? kScalar2 : kScalar4;
  return bytes <= kWaveRowBytes ? kWave : kLong;
}

struct ArgLayout {
  int lpr = kern::kArgBlock;  // short rows: lanes per row
  uint64_t splits = 1;        // long rows: workgroups per row
  int grid = 1;
};

ArgLayout arg_layout(int variant, uint64_t rows, uint64_t cols, DType t, int num_cus, int resident, int unroll) {
  ArgLayout L;
  const uint64_t N = 16 / dtype_size(t);
  const uint64_t target = static_cast<uint64_t>(num_cus) * resident;  // resident workgroups
  uint64_t blocks;
  if (variant == kWave) {
    blocks = (rows + 3) / 4;
  } else if (variant != kLong) {
    const uint64_t units = variant >= kVec1 ? cols / N : cols;  // vectors or elements per row
    const uint64_t m = variant >= kVec1 ? variant - 10 : variant;
    L.lpr = static_cast<int>(std::min<uint64_t>(64, next_pow2_u(std::max<uint64_t>((units + m - 1) / m, 1))));
    const uint64_t batches = variant >= kVec1 ? kern::short_vec_batches(static_cast<int>(m)) : kern::kArgUnroll;
    const uint64_t per_trip = static_cast<uint64_t>(64 / L.lpr) * batches;
    const uint64_t waves = (rows + per_trip - 1) / per_trip;
    blocks = (waves + 3) / 4;
  } else {
    const uint64_t tiles = std::max<uint64_t>(1, (cols / N) / (static_cast<uint64_t>(unroll) * kern::kArgBlock));
    const uint64_t want = (target + rows - 1) / rows;
    L.splits = std::max<uint64_t>(1, std::min({want, tiles, kMaxArgSplits}));
    blocks = rows * L.splits;
  }
  L.grid = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(blocks, target)));
  return L;
}

template <class Kern>
int resident_of(Kern k) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kern::kArgBlock, 0) != hipSuccess || n < 1) n = 1;
  return std::min(n, kMaxResident);
}

using ArgFn = void (*)(const kern::ArgArgs&, int variant, int unroll, int grid, hipStream_t);
using ArgOccFn = int (*)(int variant, int unroll);

template <bool MAX, class T>
void launch_arg(const kern::ArgArgs& a, int variant, int unroll, int grid, hipStream_t s) {
  const dim3 g(grid), b(kern::kArgBlock);
  switch (variant) {
    case kLong:
      if (unroll == 2) hipLaunchKernelGGL((kern::arg_rows_kernel<MAX, T, 2>), g, b, 0, s, a);
      else if (unroll == 8) hipLaunchKernelGGL((kern::arg_rows_kernel<MAX, T, 8>), g, b, 0, s, a);
      else hipLaunchKernelGGL((kern::arg_rows_kernel<MAX, T, 4>), g, b, 0, s, a);
      break;
    case kScalar1: hipLaunchKernelGGL((kern::arg_short_kernel<MAX, T, 1>), g, b, 0, s, a); break;
    case kScalar2: hipLaunchKernelGGL((kern::arg_short_kernel<MAX, T, 2>), g, b, 0, s, a); break;
    case kScalar4: hipLaunchKernelGGL((kern::arg_short_kernel<MAX, T, 4>), g, b, 0, s, a); break;
    case kVec1: hipLaunchKernelGGL((kern::arg_short_vec_kernel<MAX, T, 1>), g, b, 0, s, a); break;
    case kWave:
      if (unroll == 2) hipLaunchKernelGGL((kern::arg_wave_rows_kernel<MAX, T, 2>), g, b, 0, s, a);
      else if (unroll == 8) hipLaunchKernelGGL((kern::arg_wave_rows_kernel<MAX, T, 8>), g, b, 0, s, a);
      else hipLaunchKernelGGL((kern::arg_wave_rows_kernel<MAX, T, 4>), g, b, 0, s, a);
      break;
    case kVec2: hipLaunchKernelGGL((kern::arg_short_vec_kernel<MAX, T, 2>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((kern::arg_short_vec_kernel<MAX, T, 4>), g, b, 0, s, a); break;
  }
}

template <bool MAX, class T>
int arg_resident(int variant, int unroll) {
  static const int occ_long[3] = {resident_of(kern::arg_rows_kernel<MAX, T, 2>), resident_of(kern::arg_rows_kernel<MAX, T, 4>),
                                  resident_of(kern::arg_rows_kernel<MAX, T, 8>)};
  static const int occ_wave[3] = {resident_of(kern::arg_wave_rows_kernel<MAX, T, 2>),
                                  resident_of(kern::arg_wave_rows_kernel<MAX, T, 4>),
                                  resident_of(kern::arg_wave_rows_kernel<MAX, T, 8>)};
  static const int occ_vec4 = resident_of(kern::arg_short_vec_kernel<MAX, T, 4>);
  static const int occ[6] = {0,
                             resident_of(kern::arg_short_kernel<MAX, T, 1>),
                             resident_of(kern::arg_short_kernel<MAX, T, 2>),
                             resident_of(kern::arg_short_kernel<MAX, T, 4>),
                             resident_of(kern::arg_short_vec_kernel<MAX, T, 1>),
                             resident_of(kern::arg_short_vec_kernel<MAX, T, 2>)};
  switch (variant) {
    case kLong: return occ_long[unroll == 2 ? 0 : unroll == 8 ? 2 : 1];
    case kWave: return occ_wave[unroll == 2 ? 0 : unroll == 8 ? 2 : 1];
    case kScalar1: return occ[1];
    case kScalar2: return occ[2];
    case kScalar4: return occ[3];
    case kVec1: return occ[4];
    case kVec2: return occ[5];
    default: return occ_vec4;
  }
}

struct ArgEntry {
  ArgFn fn;
  ArgOccFn occ;
};

template <bool MAX, class T>
constexpr ArgEntry arg_entry() {
  return {launch_arg<MAX, T>, arg_resident<MAX, T>};
}

template <bool MAX>
ArgEntry arg_lookup_dtype(DType t) {
  switch (t) {
    case DType::Int32: return arg_entry<MAX, int32_t>();
    case DType::Int64: return arg_entry<MAX, int64_t>();
    case DType::Float32: return arg_entry<MAX, float>();
    case DType::Float64: return arg_entry<MAX, double>();
    case DType::BFloat16: return arg_entry<MAX, bf16_t>();
    case DType::Float16: return arg_entry<MAX, f16_t>();
  }
  throw Error("arg_reduce: unsupported element type");
}

ArgEntry arg_lookup(Op op, DType t) {
  MIREDUCE_REQUIRE(op == Op::Max || op == Op::Min, "arg_reduce: the operator must be MAX or MIN");
  return op == Op::Max ? arg_lookup_dtype<true>(t) : arg_lookup_dtype<false>(t);
}

template <class T>
void launch_loc_pack(const void* value, const int64_t* index, int64_t offset, uint64_t* pair, hipStream_t s) {
  hipLaunchKernelGGL(kern::loc_pack_kernel<T>, dim3(1), dim3(1), 0, s, static_cast<const T*>(value), index, offset, pair);
}

template <class T>
void launch_loc_pick(const uint64_t* pairs, int world, bool max, int64_t* out_index, void* out_value, hipStream_t s) {
  if (max) hipLaunchKernelGGL((kern::loc_pick_kernel<true, T>), dim3(1), dim3(1), 0, s, pairs, world, out_index,
                              static_cast<T*>(out_value));
  else hipLaunchKernelGGL((kern::loc_pick_kernel<false, T>), dim3(1), dim3(1), 0, s, pairs, world, out_index,
                          static_cast<T*>(out_value));
}

size_t ticket_bytes(uint64_t rows) { return (rows * sizeof(unsigned) + 255) / 256 * 256; }

// Split rows have rows < target = num_cus x resident <= num_cus x kMaxResident (arg_layout), so
// the per-row tickets of EVERY split launch fit one fixed region at the start of the scratch and
// the partials always start after it. A row-count-dependent boundary would let a later call with
// more rows read an earlier call's partial bits as tickets (the kernels leave only tickets zero).
size_t ticket_region_bytes(int num_cus) {
  return ticket_bytes(static_cast<uint64_t>(num_cus) * kMaxResident);
}

}  // namespace

size_t arg_reduce_scratch_bytes(size_t rows, size_t cols, DType t, int num_cus) {
  // Only long rows split, and the most splits any occupancy gives bounds every launch (rows short
  // enough for the lane-group kernels have a single tile, hence no splits either way).
  const ArgLayout L = arg_layout(kLong, rows, cols, t, num_cus, kMaxResident, 2);
  if (L.splits <= 1) return 0;
  return ticket_region_bytes(num_cus) + rows * L.splits * 16;
}

ArgPlan arg_reduce_rows(const void* in, size_t rows, size_t cols, DType t, Op op, void* out_value, int64_t* out_index,
                        void* scratch, int num_cus, hipStream_t stream, ArgTune tune) {
  const ArgEntry e = arg_lookup(op, t);
  MIREDUCE_REQUIRE(cols >= 1, "arg_reduce: rows must have at least one element");
  MIREDUCE_REQUIRE(out_value != nullptr && out_index != nullptr, "arg_reduce: output pointer is null");
  MIREDUCE_REQUIRE(reinterpret_cast<uintptr_t>(in) % dtype_size(t) == 0, "arg_reduce: misaligned input");
  MIREDUCE_REQUIRE(num_cus >= 1, "arg_reduce: num_cus must be >= 1");
  ArgPlan plan;
  if (rows == 0) return plan;
  const int variant = variant_of(in, cols, t);
  MIREDUCE_REQUIRE(tune.unroll == 0 || tune.unroll == 2 || tune.unroll == 4 || tune.unroll == 8,
                   "arg_reduce: unroll must be 2, 4 or 8");
  // Defaults from tools/arg_reduce_bw.py --sweep (profiles/r1_session3/arg_reduce/): a row split
  // over many workgroups (whole arrays) streams best with ONE workgroup per CU and 8 vectors in
  // flight per lane (f64 7.37, f32 7.13, i32 7.28 TB/s; bf16 wants 2 x 4: 7.08) — more resident
  // workgroups are more concurrent DRAM streams and lose 5-15 %; one workgroup per row wants 4 x 4.
  int unroll = tune.unroll, cap = tune.wg_per_cu;
  if (variant == kLong && rows < static_cast<size_t>(num_cus)) {
    if (!unroll) unroll = dtype_size(t) >= 4 ? 8 : 4;
    if (!cap) cap = dtype_size(t) >= 4 ? 1 : 2;
  } else if (variant == kLong) {
    if (!unroll) unroll = 4;
    if (!cap) cap = 4;
  } else if (variant == kWave) {  // 16 KB rows: 2 x 4 (6.6 TB/s); 32 KB rows: 4 x 3-5 (6.1-6.2)
    const uint64_t vecs = cols * dtype_size(t) / 16;
    if (!unroll) unroll = vecs <= 1024 ? 2 : 4;
    if (!cap) cap = 4;
  }
  if (!unroll) unroll = kern::kArgLongUnroll;
  int resident = e.occ(variant, unroll);
  if (cap > 0) resident = std::min(resident, cap);
  const ArgLayout L = arg_layout(variant, rows, cols, t, num_cus, resident, unroll);
  kern::ArgArgs a{};
  a.in = in;
  a.rows = rows;
  a.cols = cols;
  a.splits = L.splits;
  a.lpr = L.lpr;
  a.out_value = out_value;
  a.out_index = out_index;
  if (L.splits > 1) {
    MIREDUCE_REQUIRE(scratch != nullptr, "arg_reduce: this shape needs scratch (arg_reduce_scratch_bytes)");
    MIREDUCE_REQUIRE(rows < static_cast<size_t>(num_cus) * kMaxResident, "arg_reduce: split rows exceed the ticket region");
    a.tickets = static_cast<unsigned*>(scratch);
    a.partials = reinterpret_cast<uint64_t*>(static_cast<char*>(scratch) + ticket_region_bytes(num_cus));
  }
  e.fn(a, variant, unroll, L.grid, stream);
  MIREDUCE_HIP_THROW(hipGetLastError());
  plan.grid = L.grid;
  plan.lanes_per_row = L.lpr;
  plan.splits = L.splits;
  plan.unroll = variant == kLong || variant == kWave ? unroll : kern::kArgUnroll;
  plan.wg_per_cu = resident;
  return plan;
}

void loc_pack(const void* value, const int64_t* index, int64_t index_offset, DType t, uint64_t* pair,
              hipStream_t stream) {
  MIREDUCE_REQUIRE(value != nullptr && index != nullptr && pair != nullptr, "loc_pack: null pointer");
  switch (t) {
    case DType::Int32: launch_loc_pack<int32_t>(value, index, index_offset, pair, stream); break;
    case DType::Int64: launch_loc_pack<int64_t>(value, index, index_offset, pair, stream); break;
    case DType::Float32: launch_loc_pack<float>(value, index, index_offset, pair, stream); break;
    case DType::Float64: launch_loc_pack<double>(value, index, index_offset, pair, stream); break;
    case DType::BFloat16: launch_loc_pack<bf16_t>(value, index, index_offset, pair, stream); break;
    case DType::Float16: launch_loc_pack<f16_t>(value, index, index_offset, pair, stream); break;
  }
  MIREDUCE_HIP_THROW(hipGetLastError());
}

void loc_pick(const uint64_t* pairs, int world, DType t, Op op, int64_t* out_index, void* out_value,
              hipStream_t stream) {
  MIREDUCE_REQUIRE(op == Op::Max || op == Op::Min, "loc_pick: the operator must be MAX or MIN");
  MIREDUCE_REQUIRE(world >= 1 && pairs != nullptr && out_index != nullptr, "loc_pick: bad arguments");
  const bool mx = op == Op::Max;
  switch (t) {
    case DType::Int32: launch_loc_pick<int32_t>(pairs, world, mx, out_index, out_value, stream); break;
    case DType::Int64: launch_loc_pick<int64_t>(pairs, world, mx, out_index, out_value, stream); break;
    case DType::Float32: launch_loc_pick<float>(pairs, world, mx, out_index, out_value, stream); break;
    case DType::Float64: launch_loc_pick<double>(pairs, world, mx, out_index, out_value, stream); break;
    case DType::BFloat16: launch_loc_pick<bf16_t>(pairs, world, mx, out_index, out_value, stream); break;
    case DType::Float16: launch_loc_pick<f16_t>(pairs, world, mx, out_index, out_value, stream); break;
  }
  MIREDUCE_HIP_THROW(hipGetLastError());
}

}  // namespace mireduce
