// Streaming reduction kernels for gfx950 (MI355X, CDNA4).
//
// Capability parity: the reference's block-reduction kernels sumreduce6/minreduce6/maxreduce6
// (cuda/C/src/reduction/reduction_kernel.cu:74-253), their 20-way launch switch per (op, T)
// (reduction_kernel.cu:263-524) and the second in-place finalisation launch
// (reduction.cpp:344-357). Design:
//   * one templated kernel, op functors (ops.hpp), operator identity instead of g_idata[i] (B2);
//   * 16-byte non-temporal vector loads, UNROLL independent loads in flight per lane, grid-stride
//     over BLOCK*UNROLL-vector tiles with 64-bit indices (B4);
//   * wave64 butterfly (__shfl_xor over 64 lanes) instead of the 32-lane volatile tail
//     (reduction_kernel.cu:110-122 assumes warp lockstep — wrong on CDNA), then one LDS slot per
//     wave;
//   * single launch: each workgroup publishes its partial write-through (sc1), drains, and takes
//     an agent-scope ticket on one of G sharded counters; the last arriver of each group takes a
//     ticket on the top counter and the last of those folds every partial in one parallel sc1
//     load round (threadFenceReduction_kernel.cu:116-171 idea, but with the gfx950
//     release/acquire forms and a sharded fan-in: one counter for 2048 arrivals costs ~25 us,
//     eight counters ~3 us). MIREDUCE_FANIN=tree selects the older two-level fold (each group's
//     last arriver folds and republishes its group first).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mireduce/check.hpp"
#include "mireduce/half.hpp"
#include "mireduce/ops.hpp"
#include "mireduce/vec16.hpp"
#include "mireduce/reduce.hpp"
#include "mireduce/xrank.hpp"

namespace mireduce {
namespace kern {

template <class OpT, class AccT>
__device__ __forceinline__ AccT wave_reduce(AccT v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = OpT::apply(v, __shfl_xor(v, off, 64));
  return v;
}

// Result is valid in wave 0 (all lanes). Caller must barrier before reusing `lds`.
template <class OpT, class AccT, int BLOCK>
__device__ __forceinline__ AccT block_reduce(AccT v, AccT* lds) {
  constexpr int kWaves = BLOCK / 64;
  v = wave_reduce<OpT>(v);
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  if (wave == 0) {
    v = lane < kWaves ? lds[lane] : OpT::template identity<AccT>();
    v = wave_reduce<OpT>(v);
  }
  return v;
}

struct Args {
  const void* body;      // 16-byte aligned start of the vector body
  const void* head_ptr;  // original pointer (head elements live here)
  uint64_t head;         // scalar elements before `body`
  uint64_t nvec;         // 16-byte vectors
  uint64_t tail;         // scalar elements after the body
  void* partials;        // [gridDim.x] AccT
  void* group_partials;  // [groups] AccT
  unsigned* tickets;     // [(groups + 1) * kTicketStride]
  void* out;             // AccT[1]
  int groups;            // 0: two-pass mode (write partials only)
  int flat;              // 1: group last-arrivers only count; the final arriver folds every partial
  int contig;            // 1: workgroup b streams one contiguous run of tiles; 0: tiles b, b+grid, ...
  const XrankDesc* xrank;  // non-null: fold the ranks' partials in-kernel before writing out (xrank.hpp)
  uint64_t* slots;         // non-null: polled fan-in (no tickets), [gridDim.x][2] flag-tagged words
  int balance;             // 1 (interleaved split): whole rounds of tiles, then the leftover < grid
                           // tiles split evenly over ALL workgroups (no one-tile tail on a few)
};

// Polled fan-in: a published partial is two 8-byte words (tag << 32 | 32 data bits); a cleared
// slot is 0. The finisher clears every slot it consumed, so each launch starts from zeros.
constexpr uint64_t kSlotTag = 0xA5C3E1F7ull << 32;
constexpr int kPollSlots = 4;  // slots one finisher lane polls per round (grid <= 4 x BLOCK)

template <class T>
__device__ __forceinline__ uint64_t to_bits64(T v) {
  if constexpr (sizeof(T) == 8) {
    return __builtin_bit_cast(uint64_t, v);
  } else {
    return static_cast<uint64_t>(__builtin_bit_cast(uint32_t, v));
  }
}

template <class T>
__device__ __forceinline__ T from_bits64(uint64_t b) {
  if constexpr (sizeof(T) == 8) {
    return __builtin_bit_cast(T, b);
  } else {
    return __builtin_bit_cast(T, static_cast<uint32_t>(b));
  }
}

// Cross-rank finish (xrank.hpp), run by the 64 lanes of the finishing workgroup's wave 0 with
// this rank's partial `t` in every lane; returns the fold over all ranks in every lane.
// Lane p pushes to rank p's mailbox and then polls slot p of its own: the world pushes leave in
// one store round and the polls overlap. Words are (epoch << 32 | 32 data bits), written and
// read with system-scope atomics (8-byte single-copy atomic over xGMI), so a matching epoch in
// both words of a slot means the whole partial of this launch has landed.
//
// The descriptor fields a lane needs are read by xrank_prefetch: in the polled fan-in the
// finisher is known up front and issues these loads before it waits for the other workgroups'
// partials, so their latency (a descriptor miss, ~0.5 us at N=1) is off the critical path.
struct XrankLane {
  uint64_t* peer;       // rank `lane`'s mailbox (lane < world, lane != rank)
  const uint64_t* own;  // this rank's mailbox
  uint64_t limit;       // wait bound in wall-clock ticks (0 after a sticky error: look once)
  unsigned e;           // this launch's epoch
  int world, rank;
};

__device__ __forceinline__ XrankLane xrank_prefetch(const XrankDesc* d, unsigned e, unsigned err) {
  const int lane = threadIdx.x & 63;
  XrankLane x;
  x.world = d->world;
  x.rank = d->rank;
  x.peer = d->peer_mbox[lane < kMaxXrankRanks ? lane : 0];
  x.own = d->own_mbox;
  x.limit = err ? 0 : d->timeout_ticks;  // a sticky error means a peer is gone: do not wait
  x.e = e;
  return x;
}

template <class OpT, class AccT>
__device__ __forceinline__ AccT xrank_finish(const XrankDesc* d, const XrankLane& x, AccT t) {
  const int lane = threadIdx.x & 63;
  const unsigned e = x.e;
  const uint64_t parity = static_cast<uint64_t>(e & 1u) * kMaxXrankRanks;
  const uint64_t tag = static_cast<uint64_t>(e) << 32;
  const uint64_t bits = to_bits64(t);
  AccT v = OpT::template identity<AccT>();
  if (lane < x.world && lane != x.rank) {
    uint64_t* dst = x.peer + (parity + x.rank) * 2;
    __hip_atomic_store(dst, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t* src = x.own + (parity + lane) * 2;
    const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
    for (;;) {
      const uint64_t lo = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint64_t hi = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((lo >> 32) == e && (hi >> 32) == e) {
        v = from_bits64<AccT>((lo & 0xffffffffull) | (hi << 32));
        break;
      }
      if (static_cast<uint64_t>(wall_clock64()) - t0 > x.limit) {
        __hip_atomic_fetch_or(d->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  } else if (lane == x.rank) {
    v = t;  // this rank's own partial never leaves the register file
  }
  if (lane == 0) __hip_atomic_store(d->epoch, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return wave_reduce<OpT>(v);
}

template <class V, int BLOCK, int UNROLL, bool NT>
__device__ __forceinline__ void load_tile(V (&v)[UNROLL], const V* p) {
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    if constexpr (NT) v[u] = __builtin_nontemporal_load(p + u * BLOCK);
    else v[u] = p[u * BLOCK];
  }
}

template <class OpT, class T, class AccT, class V, int N, int UNROLL>
__device__ __forceinline__ void consume_tile(AccT (&acc)[UNROLL], const V (&v)[UNROLL]) {
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
    for (int k = 0; k < N; ++k) acc[u] = OpT::apply(acc[u], OpT::pre(elem<T, AccT>(v[u], k)));
  }
}

// PIPE: software-pipelined body — tile t+grid's loads are issued before tile t is consumed, so
// a wave always has UNROLL loads in flight while it computes (two register sets). The loop has
// no per-load condition (the last tile is peeled), see cdna_hip_programming.md §5 trap (c).
template <class OpT, class T, class AccT, int BLOCK, int UNROLL, bool NT, bool PIPE>
__global__ __launch_bounds__(BLOCK) void reduce_stream(Args a) {
  using V = typename Vec16<T>::type;
  constexpr int N = Vec16<T>::N;
  __shared__ AccT lds[BLOCK / 64];
  __shared__ int is_last;

  AccT acc[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) acc[u] = OpT::template identity<AccT>();

  const V* __restrict__ vin = static_cast<const V*>(a.body);
  constexpr uint64_t kTile = static_cast<uint64_t>(BLOCK) * UNROLL;
  const uint64_t ntiles = a.nvec / kTile;
  // This workgroup's full tiles: t0, t0 + step, ... < t1 (interleaved over the grid, or one
  // contiguous run of ntiles / grid tiles each).
  const uint64_t grid = gridDim.x;
  const bool balanced = a.balance && !a.contig;
  const uint64_t full = balanced ? ntiles / grid * grid : ntiles;  // tiles streamed in whole rounds
  const uint64_t t0 = a.contig ? blockIdx.x * ntiles / grid : blockIdx.x;
  const uint64_t t1 = a.contig ? (blockIdx.x + 1) * ntiles / grid : full;
  const uint64_t step = a.contig ? 1 : grid;
  if constexpr (PIPE) {
    if (t0 < t1) {
      V cur[UNROLL];
      load_tile<V, BLOCK, UNROLL, NT>(cur, vin + t0 * kTile + threadIdx.x);
      for (uint64_t tn = t0 + step; tn < t1; tn += step) {
        V nxt[UNROLL];
        load_tile<V, BLOCK, UNROLL, NT>(nxt, vin + tn * kTile + threadIdx.x);
        consume_tile<OpT, T, AccT, V, N, UNROLL>(acc, cur);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) cur[u] = nxt[u];
      }
      consume_tile<OpT, T, AccT, V, N, UNROLL>(acc, cur);
    }
  } else {
    for (uint64_t t = t0; t < t1; t += step) {
      V v[UNROLL];
      load_tile<V, BLOCK, UNROLL, NT>(v, vin + t * kTile + threadIdx.x);
      consume_tile<OpT, T, AccT, V, N, UNROLL>(acc, v);
    }
  }
  if (balanced) {
    // The leftover after the whole rounds (< grid tiles + the sub-tile remainder) as one even,
    // contiguous piece per workgroup (< one tile each): every load issued unconditionally (an
    // out-of-piece lane re-reads its piece's first vector and discards it), so no per-load branch
    // serialises the wave (cdna_hip_programming.md §5 trap (c)).
    const uint64_t l0 = full * kTile, left = a.nvec - l0;
    const uint64_t s0 = l0 + left * blockIdx.x / grid, s1 = l0 + left * (blockIdx.x + 1) / grid;
    for (uint64_t base = s0 + threadIdx.x; base < s1; base += kTile) {
      V v[UNROLL];
      bool ok[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const uint64_t idx = base + static_cast<uint64_t>(u) * BLOCK;
        ok[u] = idx < s1;
        const V* p = vin + (ok[u] ? idx : base);
        if constexpr (NT) v[u] = __builtin_nontemporal_load(p);
        else v[u] = *p;
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        if (ok[u]) {
#pragma unroll
          for (int k = 0; k < N; ++k) acc[u] = OpT::apply(acc[u], OpT::pre(elem<T, AccT>(v[u], k)));
        }
      }
    }
  } else {
    // Vectors past the last full tile, grid-strided.
    for (uint64_t i = ntiles * kTile + static_cast<uint64_t>(blockIdx.x) * BLOCK + threadIdx.x;
         i < a.nvec; i += static_cast<uint64_t>(gridDim.x) * BLOCK) {
      const V v = vin[i];
#pragma unroll
      for (int k = 0; k < N; ++k) acc[0] = OpT::apply(acc[0], OpT::pre(elem<T, AccT>(v, k)));
    }
  }
  // Unaligned head and sub-vector tail (< N elements each), folded by the last workgroup.
  if (blockIdx.x == gridDim.x - 1) {
    const T* hp = static_cast<const T*>(a.head_ptr);
    if (threadIdx.x < a.head) acc[0] = OpT::apply(acc[0], OpT::pre(static_cast<AccT>(hp[threadIdx.x])));
    const T* tp = static_cast<const T*>(a.body) + a.nvec * N;
    if (threadIdx.x < a.tail) acc[0] = OpT::apply(acc[0], OpT::pre(static_cast<AccT>(tp[threadIdx.x])));
  }
#pragma unroll
  for (int u = 1; u < UNROLL; ++u) acc[0] = OpT::apply(acc[0], acc[u]);

  // Fused cross-rank finish: this launch's epoch (counter + 1; only the finishing workgroup bumps
  // the counter, and it runs last) and the sticky error word, loaded by every workgroup after its
  // streaming body (not before: extra live values there change hipcc's load scheduling of the
  // body — 76 -> 60 VGPRs and 7.3 -> 5.1 TB/s at 512 x 16) so the finisher pays no atomic round trip.
  unsigned xr_epoch = 0, xr_err = 0;
  if (a.xrank) {
    xr_epoch = __hip_atomic_load(a.xrank->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    xr_err = __hip_atomic_load(a.xrank->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  AccT v = block_reduce<OpT, AccT, BLOCK>(acc[0], lds);
  AccT* partials = static_cast<AccT*>(a.partials);
  if (a.groups == 0) {  // two-pass mode: the finalize kernel (kernel boundary) reads these
    if (threadIdx.x == 0) partials[blockIdx.x] = v;
    return;
  }

  // ---- one workgroup (small n): it is the last arriver by construction — no partial publish,
  //      no tickets, no second load round.
  if (gridDim.x == 1) {
    if (threadIdx.x < 64) {
      if (a.xrank) v = xrank_finish<OpT, AccT>(a.xrank, xrank_prefetch(a.xrank, xr_epoch, xr_err), v);
      if (threadIdx.x == 0) *static_cast<AccT*>(a.out) = v;
    }
    return;
  }

  // ---- polled fan-in (default): no tickets, no publish-then-drain wait. Every workgroup stores
  // its partial as two tagged words (the data carries its own validity, as in the cross-rank
  // mailbox) and exits; the last-indexed workgroup — with interleaved tiles one of the first to
  // run out of work — polls all slots, folds them in slot order (deterministic), clears them and
  // finishes. The finisher's path after the last partial lands is one store + one poll round,
  // instead of store, drain, ticket (x2) and a load round. Slots live in uncached memory, so
  // polls always see the other XCDs' stores.
  if (a.slots) {
    if (threadIdx.x == 0) {
      const uint64_t bits = to_bits64(v);
      uint64_t* sl = a.slots + 2 * static_cast<uint64_t>(blockIdx.x);
      __hip_atomic_store(sl, kSlotTag | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sl + 1, kSlotTag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (blockIdx.x != gridDim.x - 1) return;
    // The finisher: start the cross-rank descriptor loads now, they land while it polls.
    XrankLane xl{};
    if (a.xrank && threadIdx.x < 64) xl = xrank_prefetch(a.xrank, xr_epoch, xr_err);
    AccT t = OpT::template identity<AccT>();
    // Bounded like every device-side wait here (all workgroups of this launch always publish, so
    // the bound is never reached by a correct launch; it only keeps a misuse from hanging the GPU).
    const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
    constexpr uint64_t kBound = 1ull << 30;  // ~10 s of the 100 MHz wall clock
    if (gridDim.x <= kPollSlots * BLOCK) {
      // Each lane polls ALL its slots (<= kPollSlots) every round, so the finish costs one poll
      // round trip after the last store lands, not one per slot.
      uint64_t lo[kPollSlots], hi[kPollSlots];
      unsigned pending = 0;
#pragma unroll
      for (int k = 0; k < kPollSlots; ++k)
        if (threadIdx.x + k * BLOCK < gridDim.x) pending |= 1u << k;
      while (pending) {
#pragma unroll
        for (int k = 0; k < kPollSlots; ++k) {
          if (pending & (1u << k)) {
            const uint64_t* sl = a.slots + 2 * static_cast<uint64_t>(threadIdx.x + k * BLOCK);
            lo[k] = __hip_atomic_load(sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            hi[k] = __hip_atomic_load(sl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
#pragma unroll
        for (int k = 0; k < kPollSlots; ++k)
          if ((pending & (1u << k)) && (lo[k] & ~0xffffffffull) == kSlotTag && (hi[k] & ~0xffffffffull) == kSlotTag)
            pending &= ~(1u << k);
        if (!pending || static_cast<uint64_t>(wall_clock64()) - t0 > kBound) break;
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int k = 0; k < kPollSlots; ++k) {  // fold in slot order (deterministic), then clear
        if (threadIdx.x + k * BLOCK < gridDim.x) {
          t = OpT::apply(t, from_bits64<AccT>((lo[k] & 0xffffffffull) | (hi[k] << 32)));
          uint64_t* sl = a.slots + 2 * static_cast<uint64_t>(threadIdx.x + k * BLOCK);
          __hip_atomic_store(sl, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(sl + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    } else {  // very large grids (user --maxblocks / wg-per-cu): slot by slot
      for (unsigned i = threadIdx.x; i < gridDim.x; i += BLOCK) {
        uint64_t* sl = a.slots + 2 * static_cast<uint64_t>(i);
        uint64_t l, h;
        for (;;) {
          l = __hip_atomic_load(sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          h = __hip_atomic_load(sl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((l & ~0xffffffffull) == kSlotTag && (h & ~0xffffffffull) == kSlotTag) break;
          if (static_cast<uint64_t>(wall_clock64()) - t0 > kBound) break;
          __builtin_amdgcn_s_sleep(1);
        }
        t = OpT::apply(t, from_bits64<AccT>((l & 0xffffffffull) | (h << 32)));
        __hip_atomic_store(sl, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sl + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    t = block_reduce<OpT, AccT, BLOCK>(t, lds);
    if (threadIdx.x < 64) {
      if (a.xrank) t = xrank_finish<OpT, AccT>(a.xrank, xl, t);
      if (threadIdx.x == 0) *static_cast<AccT*>(a.out) = t;
    }
    return;
  }

  // ---- ticketed finalisation (MIREDUCE_FANIN=flat|tree; cdna_hip_programming.md §6 G16, sc1 form)
  // Ordering rests on the gfx950 code hipcc emits for these relaxed agent-scope atomics (the full
  // acq_rel form would add an L2 write-back per arrival). Generated for <SumOp,double,512,16,nt>
  // and pinned by tests/test_isa_ordering.py:
  //   global_store_dwordx2 v4, v[2:3], s[30:31] sc1     ; partial, write-through past L2
  //   s_waitcnt vmcnt(0)                                ; ... acknowledged before
  //   global_atomic_add v6, v4, v6, s[34:35] sc0        ; the (returning) ticket
  //   s_barrier                                         ; is_last broadcast
  //   global_load_dwordx2 v[8:9], v[8:9], off sc1       ; last arriver reads partials past L1
  const unsigned G = static_cast<unsigned>(a.groups);
  const unsigned g = blockIdx.x % G;  // group label only; correctness is placement-independent
  if (threadIdx.x == 0) {
    store_sc1(&partials[blockIdx.x], v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned members = gridDim.x / G + (g < gridDim.x % G ? 1u : 0u);
    const unsigned prev = __hip_atomic_fetch_add(&a.tickets[g * kTicketStride], 1u,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (prev == members - 1);
  }
  __syncthreads();
  if (!is_last) return;

  if (a.flat) {
    // Flat fan-in: the group's last arriver only takes a ticket on the top counter; the last of
    // those folds all gridDim.x partials at once (one parallel sc1 load round instead of a
    // group fold + group-partial publish + second fold: two memory round trips shorter).
    // (One group — small grids — has no top counter: its last arriver is the finisher.)
    if (G > 1) {
      if (threadIdx.x == 0) {
        __hip_atomic_store(&a.tickets[g * kTicketStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned prev = __hip_atomic_fetch_add(&a.tickets[G * kTicketStride], 1u,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (prev == G - 1);
      }
      __syncthreads();
      if (!is_last) return;
    }
    AccT t = OpT::template identity<AccT>();
    for (unsigned i = threadIdx.x; i < gridDim.x; i += BLOCK) t = OpT::apply(t, load_sc1(&partials[i]));
    t = block_reduce<OpT, AccT, BLOCK>(t, lds);
    if (threadIdx.x < 64) {
      if (a.xrank) t = xrank_finish<OpT, AccT>(a.xrank, xrank_prefetch(a.xrank, xr_epoch, xr_err), t);
      if (threadIdx.x == 0) {
        *static_cast<AccT*>(a.out) = t;
        // reset: the top counter, or (one group) the group counter itself
        __hip_atomic_store(&a.tickets[(G > 1 ? G : 0) * kTicketStride], 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }

  // Last arriver of group g: fold partials g, g+G, g+2G, ... (sc1 loads: L1 never holds them).
  AccT s = OpT::template identity<AccT>();
  for (unsigned i = g + threadIdx.x * G; i < gridDim.x; i += BLOCK * G)
    s = OpT::apply(s, load_sc1(&partials[i]));
  s = block_reduce<OpT, AccT, BLOCK>(s, lds);
  AccT* gpart = static_cast<AccT*>(a.group_partials);
  if (threadIdx.x == 0) {
    store_sc1(&gpart[g], s);
    __hip_atomic_store(&a.tickets[g * kTicketStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&a.tickets[G * kTicketStride], 1u,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (prev == G - 1);
  }
  __syncthreads();
  if (!is_last) return;

  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    AccT t = lane < static_cast<int>(G) ? load_sc1(&gpart[lane]) : OpT::template identity<AccT>();
    t = wave_reduce<OpT>(t);
    if (a.xrank) t = xrank_finish<OpT, AccT>(a.xrank, xrank_prefetch(a.xrank, xr_epoch, xr_err), t);
    if (lane == 0) {
      *static_cast<AccT*>(a.out) = t;
      __hip_atomic_store(&a.tickets[G * kTicketStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Second level of the two-pass path (and the on-device fold for reduce_finalize): one
// workgroup folds `count` values. Launched after a kernel boundary, so plain loads are fine.
template <class OpT, class AccT>
__global__ __launch_bounds__(256) void finalize(const AccT* __restrict__ partials, uint64_t count,
                                                AccT* __restrict__ out) {
  __shared__ AccT lds[4];
  AccT s = OpT::template identity<AccT>();
  for (uint64_t i = threadIdx.x; i < count; i += 256) s = OpT::apply(s, partials[i]);
  s = block_reduce<OpT, AccT, 256>(s, lds);
  if (threadIdx.x == 0) *out = s;
}

template <class OpT, class T>
__global__ __launch_bounds__(256) void combine(T* __restrict__ inout, const T* __restrict__ other,
                                               uint64_t n) {
  using V = typename Vec16<T>::type;
  constexpr int N = Vec16<T>::N;
  const uint64_t nvec = n / N;
  V* vio = reinterpret_cast<V*>(inout);
  const V* vo = reinterpret_cast<const V*>(other);
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < nvec; i += stride) {
    V x = __builtin_nontemporal_load(vio + i);
    const V y = __builtin_nontemporal_load(vo + i);
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = OpT::apply(x[k], y[k]);
    __builtin_nontemporal_store(x, vio + i);
  }
  const uint64_t rem = n - nvec * N;
  if (blockIdx.x == 0 && threadIdx.x < rem) {
    const uint64_t i = nvec * N + threadIdx.x;
    inout[i] = OpT::apply(inout[i], other[i]);
  }
}

}  // namespace kern

// ----------------------------------------------------------------------------------------------
// Host-side dispatch: a table keyed by (op, dtype, acc, block, unroll, policy) replaces the
// reference's runtime switch over 20 template instantiations per (op, T).
// ----------------------------------------------------------------------------------------------
namespace {

using LaunchFn = void (*)(const kern::Args&, int grid, hipStream_t);

template <class OpT, class T, class AccT, int BLOCK, int UNROLL, bool NT, bool PIPE>
void launch_stream(const kern::Args& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((kern::reduce_stream<OpT, T, AccT, BLOCK, UNROLL, NT, PIPE>), dim3(grid), dim3(BLOCK),
                     0, s, a);
}

constexpr int kBlocks[] = {256, 512, 1024};
constexpr int kUnrolls[] = {2, 4, 8, 16};
constexpr int kNumBlocks = 3;
constexpr int kNumUnrolls = 4;

int block_index(int b) { return b == 256 ? 0 : (b == 512 ? 1 : (b == 1024 ? 2 : -1)); }
int unroll_index(int u) { return u == 2 ? 0 : (u == 4 ? 1 : (u == 8 ? 2 : (u == 16 ? 3 : -1))); }

// combo index: (op, dtype, acc) → 0..28
int combo_index(Op op, DType t, DType acc) {
  if (op == Op::SumSq) {  // 20..24
    switch (t) {
      case DType::Float32: return acc == DType::Float64 ? 20 : (acc == DType::Float32 ? 21 : -1);
      case DType::Float64: return acc == DType::Float64 ? 22 : -1;
      case DType::BFloat16: return acc == DType::Float32 ? 23 : -1;
      case DType::Float16: return acc == DType::Float32 ? 24 : -1;
      default: return -1;
    }
  }
  if (op == Op::AbsMax) {  // 25..28
    switch (t) {
      case DType::Float32: return acc == DType::Float32 ? 25 : -1;
      case DType::Float64: return acc == DType::Float64 ? 26 : -1;
      case DType::BFloat16: return acc == DType::Float32 ? 27 : -1;
      case DType::Float16: return acc == DType::Float32 ? 28 : -1;
      default: return -1;
    }
  }
  const int o = static_cast<int>(op);
  switch (t) {
    case DType::Int32:
      if (op == Op::Sum) return acc == DType::Int64 ? 0 : (acc == DType::Int32 ? 1 : -1);
      return acc == DType::Int32 ? 1 + o : -1;  // 2 (min), 3 (max)
    case DType::Int64:
      return acc == DType::Int64 ? 4 + o : -1;  // 4..6
    case DType::Float32:
      if (op == Op::Sum) return acc == DType::Float64 ? 7 : (acc == DType::Float32 ? 8 : -1);
      return acc == DType::Float32 ? 8 + o : -1;  // 9 (min), 10 (max)
    case DType::Float64:
      return acc == DType::Float64 ? 11 + o : -1;  // 11..13
    case DType::BFloat16:
      return acc == DType::Float32 ? 14 + o : -1;  // 14..16
    case DType::Float16:
      return acc == DType::Float32 ? 17 + o : -1;  // 17..19
  }
  return -1;
}
constexpr int kCombos = 29;

struct Table {
  LaunchFn fn[kCombos][kNumBlocks][kNumUnrolls][2][2];  // [..][policy nt][pipelined]
};

// Pipelined variants need two register sets of UNROLL 16-byte vectors: only where the
// per-SIMD register budget allows it (BLOCK * UNROLL <= 8192); elsewhere the plain body.
constexpr bool pipe_ok(int b, int u) { return b * u <= 8192; }

template <class OpT, class T, class AccT, int BI, int UI>
void fill_one(Table& tb, int c) {
  constexpr int B = kBlocks[BI];
  constexpr int U = kUnrolls[UI];
  constexpr bool P = pipe_ok(B, U);
  tb.fn[c][BI][UI][0][0] = launch_stream<OpT, T, AccT, B, U, false, false>;
  tb.fn[c][BI][UI][1][0] = launch_stream<OpT, T, AccT, B, U, true, false>;
  tb.fn[c][BI][UI][0][1] = launch_stream<OpT, T, AccT, B, U, false, P>;
  tb.fn[c][BI][UI][1][1] = launch_stream<OpT, T, AccT, B, U, true, P>;
}

template <class OpT, class T, class AccT, int BI>
void fill_block(Table& tb, int c) {
  fill_one<OpT, T, AccT, BI, 0>(tb, c);
  fill_one<OpT, T, AccT, BI, 1>(tb, c);
  fill_one<OpT, T, AccT, BI, 2>(tb, c);
  fill_one<OpT, T, AccT, BI, 3>(tb, c);
}

template <class OpT, class T, class AccT>
void fill_combo(Table& tb, int c) {
  fill_block<OpT, T, AccT, 0>(tb, c);
  fill_block<OpT, T, AccT, 1>(tb, c);
  fill_block<OpT, T, AccT, 2>(tb, c);
}

const Table& table() {
  static const Table tb = [] {
    Table t{};
    fill_combo<SumOp, int32_t, int64_t>(t, 0);
    fill_combo<SumOp, int32_t, int32_t>(t, 1);
    fill_combo<MinOp, int32_t, int32_t>(t, 2);
    fill_combo<MaxOp, int32_t, int32_t>(t, 3);
    fill_combo<SumOp, int64_t, int64_t>(t, 4);
    fill_combo<MinOp, int64_t, int64_t>(t, 5);
    fill_combo<MaxOp, int64_t, int64_t>(t, 6);
    fill_combo<SumOp, float, double>(t, 7);
    fill_combo<SumOp, float, float>(t, 8);
    fill_combo<MinOp, float, float>(t, 9);
    fill_combo<MaxOp, float, float>(t, 10);
    fill_combo<SumOp, double, double>(t, 11);
    fill_combo<MinOp, double, double>(t, 12);
    fill_combo<MaxOp, double, double>(t, 13);
    fill_combo<SumOp, bf16_t, float>(t, 14);
    fill_combo<MinOp, bf16_t, float>(t, 15);
    fill_combo<MaxOp, bf16_t, float>(t, 16);
    fill_combo<SumOp, f16_t, float>(t, 17);
    fill_combo<MinOp, f16_t, float>(t, 18);
    fill_combo<MaxOp, f16_t, float>(t, 19);
    fill_combo<SumSqOp, float, double>(t, 20);
    fill_combo<SumSqOp, float, float>(t, 21);
    fill_combo<SumSqOp, double, double>(t, 22);
    fill_combo<SumSqOp, bf16_t, float>(t, 23);
    fill_combo<SumSqOp, f16_t, float>(t, 24);
    fill_combo<AbsMaxOp, float, float>(t, 25);
    fill_combo<AbsMaxOp, double, double>(t, 26);
    fill_combo<AbsMaxOp, bf16_t, float>(t, 27);
    fill_combo<AbsMaxOp, f16_t, float>(t, 28);
    return t;
  }();
  return tb;
}

// Tuned gfx950 defaults, measured on MI355X with tools/tune.py (interleaved rounds in one
// process; profiles/r1_tuning/). Median read bandwidth of the chosen point:
//   8 GB f64 sum / min  512 x 16, 1 WG/CU, nt   7.29 / 7.38 TB/s (best point for both)
//   1 GB f64 sum        256 x  2, 3 WG/CU, nt   7.12 TB/s (best)
//   8 GB i64 max        256 x  2, 3 WG/CU, nt   7.30 TB/s (best; 512 x 16 x 1 is not in the top 8)
//   8 GB f32 sum / max  256 x  2, 3 WG/CU, nt   7.20 / 7.25 TB/s (best 7.21 / 7.25)
//   8 GB i32 sum        256 x  2, 3 WG/CU, nt   7.20 TB/s (best 7.25)
//   192-384 MB          256 x  2, 3 WG/CU, nt   256 MB: 6.33 TB/s warm, 5.93 cold (--cold). The
//                       earlier warm-only pick (512 x 16 x 1, default policy: 6.25 warm) fell to
//                       2.69 TB/s when the array was not already in the Infinity Cache
//                       (profiles/r1_bench/plan_256mb.csv): non-nt loads are never the safe choice.
//   128 MB              256 x  4, 3 WG/CU, nt   6.10 TB/s (best; launch + tail dominate)
//   8 GB / 1 GB bf16 sum 256 x  4, 2 WG/CU, nt   7.18 / 7.01 TB/s (best at both; 256 x 2 x 3: 7.10 / 6.97);
//   8 GB f16 max        512 x 4 x 1 7.18, 256 x 4 x 2 7.14 (profiles/r1_session3/tune_half.txt)
// Fewer, fatter workgroups beat the "fill every wave slot" grid (8 WG/CU: 6.91 TB/s at 8 GB).
struct Defaults {
  int block, unroll, wg_per_cu, policy, pipeline;
};
Defaults tuned_defaults(size_t bytes, DType t) {
  constexpr size_t MB = 1ull << 20;
  // >= 3 GB: one 512-thread workgroup per CU (tools/tune_types.sh, profiles/r1_session3/tune_types.txt):
  // 8-byte types 16 vectors in flight per lane (f64 7.30, i64 7.30 TB/s vs 7.16 at 256x2x3),
  // 4-byte types 4 (f32 7.17, i32 7.19 vs 7.14).
  if (dtype_size(t) == 8 && bytes >= 3072 * MB) return {512, 16, 1, 1, 0};
  if (dtype_size(t) == 4 && bytes >= 3072 * MB) return {512, 4, 1, 1, 0};
  if (dtype_is_half(t) && bytes > 192 * MB) return {256, 4, 2, 1, 0};
  if (bytes > 192 * MB) return {256, 2, 3, 1, 0};
  return {256, 4, 3, 1, 0};
}
constexpr int kDefaultGroups = 8;
constexpr int kOneGroupGrid = 64;

// Fan-in shape of the single-pass finalisation: 0 tree, 1 flat (ticketed), 2 poll (default);
// MIREDUCE_FANIN=poll|flat|tree overrides (A/B runs).
int fanin_mode() {
  static const int v = [] {
    const char* e = std::getenv("MIREDUCE_FANIN");
    if (e && std::strcmp(e, "tree") == 0) return 0;
    if (e && std::strcmp(e, "flat") == 0) return 1;
    return 2;
  }();
  return v;
}

// Balanced leftover: MIREDUCE_BALANCE=1 opts in (read per plan). Off by default: measured equal
// within noise at 128 MiB - 4 GB for four plans (profiles/r2_small/balance_ab.txt) — the
// bandwidth the idle workgroups free up already lets the few with an extra tile finish early.
bool balance_leftover() {
  const char* e = std::getenv("MIREDUCE_BALANCE");
  return e && std::strcmp(e, "1") == 0;
}

// Work split of the streaming body; MIREDUCE_SPLIT=stride|contig overrides (A/B runs; read per
// plan so one process can compare both).
bool split_contiguous() {
  const char* e = std::getenv("MIREDUCE_SPLIT");
  if (e && std::strcmp(e, "contig") == 0) return true;
  if (e && std::strcmp(e, "stride") == 0) return false;
  return false;
}

template <class OpT, class AccT>
void launch_finalize(const void* partials, uint64_t count, void* out, hipStream_t s) {
  hipLaunchKernelGGL((kern::finalize<OpT, AccT>), dim3(1), dim3(256), 0, s,
                     static_cast<const AccT*>(partials), count, static_cast<AccT*>(out));
}

template <class OpT>
void finalize_by_acc(DType acc, const void* partials, uint64_t count, void* out, hipStream_t s) {
  switch (acc) {
    case DType::Int32: launch_finalize<OpT, int32_t>(partials, count, out, s); break;
    case DType::Int64: launch_finalize<OpT, int64_t>(partials, count, out, s); break;
    case DType::Float32: launch_finalize<OpT, float>(partials, count, out, s); break;
    case DType::Float64: launch_finalize<OpT, double>(partials, count, out, s); break;
    default: MIREDUCE_REQUIRE(false, "finalize: accumulator must be int32, int64, float32 or float64");
  }
}

template <class OpT, class T>
void launch_combine(void* inout, const void* other, uint64_t n, hipStream_t s) {
  constexpr int N = kern::Vec16<T>::N;
  uint64_t blocks = (n / N + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL((kern::combine<OpT, T>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s,
                     static_cast<T*>(inout), static_cast<const T*>(other), n);
}

template <class OpT>
void combine_by_type(DType t, void* inout, const void* other, uint64_t n, hipStream_t s) {
  switch (t) {
    case DType::Int32: launch_combine<OpT, int32_t>(inout, other, n, s); break;
    case DType::Int64: launch_combine<OpT, int64_t>(inout, other, n, s); break;
    case DType::Float32: launch_combine<OpT, float>(inout, other, n, s); break;
    case DType::Float64: launch_combine<OpT, double>(inout, other, n, s); break;
    default: MIREDUCE_REQUIRE(false, "combine_elementwise: int32, int64, float32 or float64 only");
  }
}

}  // namespace

// ----------------------------------------------------------------------------------------------

Workspace::Workspace(int device, int max_grid) : max_grid_(max_grid) {
  MIREDUCE_REQUIRE(max_grid >= 1, "Workspace: max_grid must be positive");
  if (device < 0) MIREDUCE_HIP_THROW(hipGetDevice(&device));
  device_ = device;
  int cus = 0;
  MIREDUCE_HIP_THROW(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  num_cus_ = cus > 0 ? cus : 256;
  int prev = 0;
  MIREDUCE_HIP_THROW(hipGetDevice(&prev));
  MIREDUCE_HIP_THROW(hipSetDevice(device));
  MIREDUCE_HIP_THROW(hipMalloc(&partials_, static_cast<size_t>(max_grid) * 8));
  MIREDUCE_HIP_THROW(hipMalloc(&group_partials_, static_cast<size_t>(kMaxGroups) * 8));
  const size_t tbytes = static_cast<size_t>(kMaxGroups + 1) * kTicketStride * sizeof(unsigned);
  MIREDUCE_HIP_THROW(hipMalloc(reinterpret_cast<void**>(&tickets_), tbytes));
  MIREDUCE_HIP_THROW(hipMemset(tickets_, 0, tbytes));
  // polled fan-in slots: uncached, so the finisher's polls see every XCD's stores
  MIREDUCE_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&slots_), static_cast<size_t>(max_grid) * 16,
                                           hipDeviceMallocUncached));
  MIREDUCE_HIP_THROW(hipMemset(slots_, 0, static_cast<size_t>(max_grid) * 16));
  MIREDUCE_HIP_THROW(hipDeviceSynchronize());
  MIREDUCE_HIP_THROW(hipSetDevice(prev));
}

Workspace::~Workspace() {
  (void)hipFree(partials_);
  (void)hipFree(group_partials_);
  (void)hipFree(tickets_);
  (void)hipFree(slots_);
}

void Workspace::reset(hipStream_t stream) {
  const size_t tbytes = static_cast<size_t>(kMaxGroups + 1) * kTicketStride * sizeof(unsigned);
  MIREDUCE_HIP_THROW(hipMemsetAsync(tickets_, 0, tbytes, stream));
  MIREDUCE_HIP_THROW(hipMemsetAsync(slots_, 0, static_cast<size_t>(max_grid_) * 16, stream));
}

LaunchPlan plan_reduce(const void* in, size_t n, DType t, const ReduceConfig& cfg, int num_cus,
                       int max_grid) {
  LaunchPlan p;
  const size_t es = dtype_size(t);
  const Defaults d = tuned_defaults(n * es, t);
  p.block = cfg.block ? cfg.block : d.block;
  p.unroll = cfg.unroll ? cfg.unroll : d.unroll;
  p.nontemporal = cfg.policy < 0 ? d.policy == 1 : cfg.policy == 1;
  p.single_pass = cfg.single_pass;
  MIREDUCE_REQUIRE(cfg.xrank == nullptr || cfg.single_pass,
                   "the fused cross-rank finish needs the single-pass kernel");
  p.pipelined = (cfg.pipeline < 0 ? d.pipeline == 1 : cfg.pipeline == 1) && p.block * p.unroll <= 8192;
  MIREDUCE_REQUIRE(block_index(p.block) >= 0, "block must be 256, 512 or 1024");
  MIREDUCE_REQUIRE(unroll_index(p.unroll) >= 0, "unroll must be 2, 4, 8 or 16");
  const size_t vec = 16 / es;
  const uintptr_t addr = reinterpret_cast<uintptr_t>(in);
  MIREDUCE_REQUIRE(n == 0 || addr % es == 0, "input pointer is not aligned to its element size");
  uint64_t head = 0;
  if (addr % 16 != 0) head = (16 - addr % 16) / es;
  if (head > n) head = n;
  p.head = head;
  p.nvec = (n - head) / vec;
  p.tail = (n - head) - p.nvec * vec;
  // wg_per_cu given without block: keep the thread count per CU of the tuned point.
  int wg_per_cu = cfg.wg_per_cu;
  if (!wg_per_cu) wg_per_cu = cfg.block ? std::max(1, d.wg_per_cu * d.block / p.block) : d.wg_per_cu;
  const uint64_t tile = static_cast<uint64_t>(p.block) * p.unroll;
  uint64_t want = (p.nvec + tile - 1) / tile;
  const uint64_t cap = static_cast<uint64_t>(num_cus) * wg_per_cu;
  if (want > cap) want = cap;
  if (cfg.max_blocks > 0 && want > static_cast<uint64_t>(cfg.max_blocks)) want = cfg.max_blocks;
  if (want > static_cast<uint64_t>(max_grid)) want = max_grid;
  if (want < 1) want = 1;
  p.grid = static_cast<int>(want);
  // Arrival counters: one for small grids (<= kOneGroupGrid arrivals contend little, and the
  // finisher then skips the second ticket round trip), kDefaultGroups shards above.
  int groups = cfg.groups ? cfg.groups : (static_cast<int>(want) <= kOneGroupGrid ? 1 : kDefaultGroups);
  if (groups > kMaxGroups) groups = kMaxGroups;
  if (groups > p.grid) groups = p.grid;
  p.groups = p.single_pass ? groups : 0;
  p.poll = p.single_pass && fanin_mode() == 2;
  p.flat = p.single_pass && fanin_mode() == 1;
  p.contiguous = split_contiguous();
  p.balanced = !p.contiguous && balance_leftover();
  return p;
}

static kern::Args make_args(const void* in, const LaunchPlan& p, DType t) {
  kern::Args a{};
  a.head_ptr = in;
  a.body = static_cast<const char*>(in) + p.head * dtype_size(t);
  a.head = p.head;
  a.nvec = p.nvec;
  a.tail = p.tail;
  a.contig = p.contiguous ? 1 : 0;
  a.balance = p.balanced ? 1 : 0;
  return a;
}

LaunchPlan reduce(const void* in, size_t n, DType t, Op op, DType acc, void* out, Workspace& ws,
                  hipStream_t stream, const ReduceConfig& cfg) {
  const int c = combo_index(op, t, acc);
  MIREDUCE_REQUIRE(c >= 0, "unsupported (dtype, op, accumulator) combination");
  MIREDUCE_REQUIRE(out != nullptr, "output pointer is null");
  LaunchPlan p = plan_reduce(in, n, t, cfg, ws.num_cus(), ws.max_grid());
  kern::Args a = make_args(in, p, t);
  a.partials = ws.partials();
  a.group_partials = ws.group_partials();
  a.tickets = ws.tickets();
  a.out = out;
  a.groups = p.groups;
  a.flat = p.flat ? 1 : 0;
  a.slots = p.poll ? ws.slots() : nullptr;
  a.xrank = static_cast<const XrankDesc*>(cfg.xrank);
  const LaunchFn fn = table().fn[c][block_index(p.block)][unroll_index(p.unroll)][p.nontemporal ? 1 : 0][p.pipelined ? 1 : 0];
  fn(a, p.grid, stream);
  MIREDUCE_HIP_THROW(hipGetLastError());
  if (!p.single_pass) reduce_finalize(ws.partials(), p.grid, acc, op, out, stream);
  return p;
}

struct BoundReduce::Impl {
  kern::Args args;
  LaunchFn fn;
  LaunchPlan plan;
  Op op;
  DType acc;
};

BoundReduce::BoundReduce(const void* in, size_t n, DType t, Op op, DType acc, void* out, Workspace& ws,
                         const ReduceConfig& cfg)
    : impl_(nullptr) {
  const int c = combo_index(op, t, acc);
  MIREDUCE_REQUIRE(c >= 0, "unsupported (dtype, op, accumulator) combination");
  MIREDUCE_REQUIRE(out != nullptr, "output pointer is null");
  const LaunchPlan p = plan_reduce(in, n, t, cfg, ws.num_cus(), ws.max_grid());
  kern::Args a = make_args(in, p, t);
  a.partials = ws.partials();
  a.group_partials = ws.group_partials();
  a.tickets = ws.tickets();
  a.out = out;
  a.groups = p.groups;
  a.flat = p.flat ? 1 : 0;
  a.slots = p.poll ? ws.slots() : nullptr;
  a.xrank = static_cast<const XrankDesc*>(cfg.xrank);
  impl_ = new Impl{a, table().fn[c][block_index(p.block)][unroll_index(p.unroll)][p.nontemporal ? 1 : 0][p.pipelined ? 1 : 0],
                   p, op, acc};
}

BoundReduce::~BoundReduce() { delete impl_; }

void BoundReduce::launch(hipStream_t stream, void* out) const {
  kern::Args a = impl_->args;
  if (out) a.out = out;
  impl_->fn(a, impl_->plan.grid, stream);
  MIREDUCE_HIP_THROW(hipGetLastError());
  if (!impl_->plan.single_pass) reduce_finalize(a.partials, impl_->plan.grid, impl_->acc, impl_->op, a.out, stream);
}

const LaunchPlan& BoundReduce::plan() const { return impl_->plan; }

LaunchPlan reduce_partials(const void* in, size_t n, DType t, Op op, DType acc, void* partials,
                           int max_grid, int num_cus, hipStream_t stream, const ReduceConfig& cfg) {
  const int c = combo_index(op, t, acc);
  MIREDUCE_REQUIRE(c >= 0, "unsupported (dtype, op, accumulator) combination");
  ReduceConfig c2 = cfg;
  c2.single_pass = false;
  c2.xrank = nullptr;
  LaunchPlan p = plan_reduce(in, n, t, c2, num_cus, max_grid);
  kern::Args a = make_args(in, p, t);
  a.partials = partials;
  a.groups = 0;
  const LaunchFn fn = table().fn[c][block_index(p.block)][unroll_index(p.unroll)][p.nontemporal ? 1 : 0][p.pipelined ? 1 : 0];
  fn(a, p.grid, stream);
  MIREDUCE_HIP_THROW(hipGetLastError());
  return p;
}

ReducePasses reduce_passes(const void* in, size_t n, DType t, Op op, DType acc, void* scratch, int max_grid,
                           int num_cus, uint64_t cpu_thresh, bool cpu_final, hipStream_t stream,
                           const ReduceConfig& cfg) {
  ReducePasses r;
  char* a = static_cast<char*>(scratch);
  char* b = a + static_cast<size_t>(max_grid) * 8;
  r.plan = reduce_partials(in, n, t, op, acc, a, max_grid, num_cus, stream, cfg);
  r.passes = 1;
  uint64_t left = static_cast<uint64_t>(r.plan.grid);
  // Later passes fold already-transformed partials: SUMSQ folds like SUM, AMAX like MAX.
  const Op fold = op == Op::SumSq ? Op::Sum : (op == Op::AbsMax ? Op::Max : op);
  ReduceConfig c2 = cfg;
  c2.max_blocks = 0;  // the partial passes use the planner's own grid
  while (!cpu_final && left > std::max<uint64_t>(cpu_thresh, 1)) {
    const LaunchPlan p = reduce_partials(a, left, acc, fold, acc, b, max_grid, num_cus, stream, c2);
    left = static_cast<uint64_t>(p.grid);
    ++r.passes;
    std::swap(a, b);
  }
  r.left = left;
  r.partials = a;
  return r;
}

void reduce_finalize(const void* partials, size_t count, DType acc, Op op, void* out,
                     hipStream_t stream) {
  switch (op) {  // partials are already transformed: SUMSQ folds like SUM, AMAX like MAX
    case Op::Sum:
    case Op::SumSq: finalize_by_acc<SumOp>(acc, partials, count, out, stream); break;
    case Op::Min: finalize_by_acc<MinOp>(acc, partials, count, out, stream); break;
    case Op::Max:
    case Op::AbsMax: finalize_by_acc<MaxOp>(acc, partials, count, out, stream); break;
  }
  MIREDUCE_HIP_THROW(hipGetLastError());
}

void combine_elementwise(void* inout, const void* other, size_t n, DType t, Op op,
                         hipStream_t stream) {
  if (n == 0) return;
  MIREDUCE_REQUIRE(reinterpret_cast<uintptr_t>(inout) % 16 == 0 &&
                       reinterpret_cast<uintptr_t>(other) % 16 == 0,
                   "combine_elementwise needs 16-byte aligned buffers");
  switch (op) {
    case Op::Sum: combine_by_type<SumOp>(t, inout, other, n, stream); break;
    case Op::Min: combine_by_type<MinOp>(t, inout, other, n, stream); break;
    case Op::Max: combine_by_type<MaxOp>(t, inout, other, n, stream); break;
    default: MIREDUCE_REQUIRE(false, "combine_elementwise: SUM, MIN or MAX");
  }
  MIREDUCE_HIP_THROW(hipGetLastError());
}

std::vector<std::string> compiled_variants() {
  std::vector<std::string> v;
  for (int b : kBlocks)
    for (int u : kUnrolls)
      for (int nt = 0; nt < 2; ++nt)
        for (int pp = 0; pp < 2; ++pp)
          if (!pp || b * u <= 8192)
            v.push_back("block=" + std::to_string(b) + " unroll=" + std::to_string(u) +
                        (nt ? " policy=nt" : " policy=default") + (pp ? " pipelined" : ""));
  return v;
}

}  // namespace mireduce
