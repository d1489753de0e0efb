// Streaming reduction kernels for gfx950 (MI355X, CDNA4): the kernel templates and the
// dispatch-table machinery shared by reduce.hip (host side: planner, launches) and the
// reduce_tab_*.hip translation units, each of which instantiates the table entries of a few
// (op, dtype, acc) combos (one TU held all ~1,400 instantiations and took ~9 min to compile).
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
//   * single launch with a polled fan-in: every workgroup stores its partial as two epoch-tagged
//     words (no ticket, no drain) and the last-indexed workgroup polls them all, folds them in slot
//     order and finishes (threadFenceReduction_kernel.cu:116-171 idea, without its atomic ticket:
//     one counter for 2048 arrivals costs ~25 us, the polled finish ~1.5 us); a two-pass mode
//     (partials, then a one-workgroup finalize) serves the reference's multi-pass / --cpufinal paths.
// Round 6 pruned the bodies measured as no gain (docs/TUNING.md): the software-pipelined body, the
// strict load window (tools/window_ab.hip keeps it as a control), the contiguous and balanced-leftover
// splits and the ticketed flat / tree fan-ins. One body per plan ships: hipcc's schedule of the plain
// loop (<= 192 MB) or the explicit load window (above), over the interleaved (XCD-weighted) split.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
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
  void* partials;        // two-pass mode: [gridDim.x] AccT
  void* out;             // AccT[1]
  int two_pass;          // 1: write partials only (the finalize kernel folds them after a kernel boundary)
  const XrankDesc* xrank;  // non-null: fold the ranks' partials in-kernel before writing out (xrank.hpp)
  uint64_t* slots;         // single pass: the polled fan-in's [gridDim.x][2] epoch-tagged words (Workspace)
  unsigned* fan;           // polled fan-in state (Workspace): [0] epoch = finished launches, [1] sticky error,
                           // [2..3] the XCD anchor of the weighted split (XcdAnchor)
  uint64_t fan_bound;      // polled fan-in: finisher's wait bound in wall-clock ticks
  unsigned fan_slots;      // polled fan-in: slots in the workspace (all zeroed when the epoch wraps)
  int delay_wg;            // test hook (ReduceConfig::debug_delay_wg): this workgroup sleeps
  uint64_t delay_ticks;    // delay_ticks before publishing its partial; -1 = none
  uint64_t anchor_delay;   // test hook (ReduceConfig::debug_delay_anchor_ticks): workgroup 0 sleeps this
                           // long before publishing the XCD anchor; 0 = none
  uint64_t* wg_stamps;     // diagnostic (ReduceConfig::debug_wg_stamps): per-workgroup end stamps
  int xskew;               // XCD-weighted split (window bodies): |xskew| extra rounds of tiles for the
                           // workgroups on odd (xskew > 0) or even (< 0) XCCs; 0 = equal
  uint64_t x_ra;           // weighted split, precomputed on the host: common rounds (ntiles / grid at 0)
  uint64_t x_dd;           // extra rounds actually given to the favoured parity
  int two_pass_epoch;      // two-pass launch whose finalize ends the fan-in epoch (fan[0]; XcdAnchor)
  const void* carry;       // segmented launches (polled fan-in): AccT[ncarry] results of the earlier
  unsigned ncarry;         // segments (written by earlier kernels), folded in by this launch's finisher
};

// Polled fan-in: a published partial is two 8-byte words (epoch << 32 | 32 data bits), where the
// epoch is this launch's number (Workspace fan[0] + 1, read by every workgroup at its start and
// advanced by the finisher after it has consumed every slot): a slot is valid for exactly one
// launch, so nothing needs clearing, and a late store from an earlier (timed-out) launch never
// matches. Reaching the bound sets the sticky error fan[1] and poisons the result instead of
// folding unpublished slots; Workspace::error() reports it, Workspace::reset() clears it.
// The epoch is 32 bits: when it wraps (every 2^32 launches of one workspace) the finisher first
// zeroes every slot of the workspace (Args::fan_slots), so a slot last written a whole cycle ago —
// beyond the grid of the launches since — cannot carry the new cycle's tag.
constexpr int kPollSlots = 4;  // slots one finisher lane polls per round (grid <= 4 x BLOCK)
constexpr uint64_t kFanBoundTicks = 1ull << 30;  // ~10.7 s of the 100 MHz wall clock

// The value a launch writes when its fan-in or cross-rank finish failed: NaN for floating types;
// for integers no in-range value can signal an error, so they get the operator's identity — neutral
// in any later fold — and the error WORDS (Workspace::error(), XrankChannel::error()) are the signal.
template <class OpT, class AccT>
__device__ __forceinline__ AccT poisoned() {
  if constexpr (std::is_floating_point_v<AccT>) return __builtin_nan("");
  else return OpT::template identity<AccT>();
}

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
// Mailbox word tags: a 31-bit epoch plus the poison flag (bit 63 of the word): a rank whose own
// result is poisoned pushes its (neutral) partial with the flag set, and every peer that folds it
// sets error value 2 (bit 1) on its own channel and poisons its result too — a failure on one rank is never
// a plausible-looking value on another.
constexpr unsigned kXrankEpochMask = 0x7fffffffu;
constexpr uint64_t kXrankPoisonBit = 1ull << 63;
constexpr unsigned kXrankErrTimeout = 1u;    // a peer's partial missed the timeout
constexpr unsigned kXrankErrPeerPoison = 2u; // a peer pushed a poisoned partial

// Next launch's epoch from the channel counter: 31 bits, 0 skipped (a zeroed mailbox word) and the
// parity kept alternating across the wrap (0x7fffffff -> 2), which the double buffer relies on.
__device__ __forceinline__ unsigned xrank_next_epoch(unsigned cur) {
  const unsigned e = (cur + 1u) & kXrankEpochMask;
  return e ? e : 2u;
}

struct XrankLane {
  uint64_t* peer;       // rank `lane`'s mailbox (lane < world, lane != rank)
  const uint64_t* own;  // this rank's mailbox
  uint64_t limit;       // wait bound in wall-clock ticks (0 after a sticky error: look once)
  uint64_t* stamps;     // exchange timing (XrankDesc::stamps; null: off)
  unsigned stamp_mask;
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
  x.stamps = d->stamps;
  x.stamp_mask = d->stamp_mask;
  x.e = e;
  return x;
}

// `poison`: this rank's partial `t` is already poisoned (its fan-in failed): it is pushed with the
// poison flag. `failed` (wave-uniform) returns whether this launch's global value is unusable: a
// peer's partial missed the timeout or arrived poisoned (the caller then writes poisoned<>()).
template <class OpT, class AccT>
__device__ __forceinline__ AccT xrank_finish(const XrankDesc* d, const XrankLane& x, AccT t, bool poison,
                                             bool& failed) {
  const int lane = threadIdx.x & 63;
  const unsigned e = x.e;
  const uint64_t parity = static_cast<uint64_t>(e & 1u) * kMaxXrankRanks;
  const uint64_t tag = (static_cast<uint64_t>(e) << 32) | (poison ? kXrankPoisonBit : 0ull);
  const uint64_t bits = to_bits64(t);
  AccT v = OpT::template identity<AccT>();
  bool bad = false;
  const uint64_t t_push = x.stamps ? static_cast<uint64_t>(wall_clock64()) : 0;
  if (lane < x.world && lane != x.rank) {
    uint64_t* dst = x.peer + (parity + x.rank) * 2;
    __hip_atomic_store(dst, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t* src = x.own + (parity + lane) * 2;
    const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
    for (;;) {
      const uint64_t lo = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint64_t hi = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (((lo >> 32) & kXrankEpochMask) == e && ((hi >> 32) & kXrankEpochMask) == e) {
        v = from_bits64<AccT>((lo & 0xffffffffull) | (hi << 32));
        if ((lo | hi) & kXrankPoisonBit) {
          __hip_atomic_fetch_or(d->error, kXrankErrPeerPoison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          bad = true;
        }
        break;
      }
      if (static_cast<uint64_t>(wall_clock64()) - t0 > x.limit) {
        __hip_atomic_fetch_or(d->error, kXrankErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bad = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  } else if (lane == x.rank) {
    v = t;  // this rank's own partial never leaves the register file
  }
  if (lane == 0) __hip_atomic_store(d->epoch, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  failed = __ballot(bad) != 0;  // (also: every lane's poll has ended)
  if (x.stamps && lane == 0) {
    uint64_t* st = x.stamps + 2 * static_cast<uint64_t>(e & x.stamp_mask);
    st[0] = t_push;
    st[1] = static_cast<uint64_t>(wall_clock64());
  }
  return wave_reduce<OpT>(v);
}

template <class V, bool NT>
__device__ __forceinline__ V ld16(const V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
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

// Explicit load window (stream_window_seq below): the thread's loads over its tiles form one sequence
// held in WIN registers — each step issues the load WIN ahead and then consumes the oldest (so
// WIN + 1 are in flight at each issue, WIN after each wait; the strict form that consumes first,
// WIN at most, is kept as a control in tools/window_ab.hip);
// a sched_barrier between steps pins the interleave (hipcc's own grouping of the plain body moves
// with unrelated code in the kernel: profiles/r3_regress). Measured (profiles/r3_window/): the
// loose form with ~18-20 loads in flight per CU is fastest (256x8x1 with 4: 8 GB 1092 vs 1112 us
// for hipcc's schedule, 1 GB 141.0 vs 144.5 us for 256x2x3), the strict form 1-70 % slower. The loads are raw buffer loads:
// the tile base rides in a wave-uniform descriptor (SGPRs), the lane's byte offset in one VGPR and
// each load's tile offset in soffset, so a load costs no address arithmetic, and the non-temporal
// bit is part of the instruction (aux = 2: a plain-pointer nontemporal load lost it under this
// interleave, profiles/r3_window/).
constexpr int kAuxNT = 2;  // buffer-load cache policy: nt

template <class V>
__device__ __forceinline__ V ld_buf_nt(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, kAuxNT));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

// The tiles one workgroup streams as up to three arithmetic runs (the XCD-weighted split): run 0
// `n0` tiles from `s0` by `st0`, run 1 `n1` tiles from `s1` by `st1`, run 2 `n2` tiles from `s2`
// by `st0`. Workgroups are dispatched to the 8 XCDs round-robin (XCD = blockIdx % 8), and the
// XCDs do not stream equally fast: with equal tiles, the even XCDs' workgroups end ~1.5-2 % later
// than the odd ones' in every run (tools/xcd_balance.py, profiles/r4_suite/), and the kernel ends
// with the slowest. The weighted split gives one parity a few more rounds so both end together.
struct TileSeq {
  uint64_t s0, st0, s1, st1, s2;
  uint32_t n0, n1, n2;  // tile counts fit 32 bits (2^32 tiles of 4 KB+ = 16 TB+)
  __device__ __forceinline__ uint32_t count() const { return n0 + n1 + n2; }
};

// Runs 1 and 2 of the weighted split of workgroup b, the blockIdx parity `fpar` taking the extra
// rounds: after the `ra` common rounds (run 0: b, b + grid, ...), the favoured workgroups take `dd`
// more rounds interleaved among themselves, and the leftover (< grid tiles) goes one tile each to
// the favoured workgroups first. A bijection onto [0, ntiles) for either parity.
__device__ __forceinline__ void weighted_tail(TileSeq& q, uint64_t ntiles, uint64_t grid, unsigned fpar, uint64_t ra,
                                              uint64_t dd, uint64_t b) {
  const uint64_t half = grid >> 1, base1 = ra * grid;
  const bool favoured = (b & 1u) == fpar;
  q.s1 = base1 + (b >> 1);
  q.st1 = half;
  q.n1 = favoured ? static_cast<uint32_t>(dd) : 0u;
  const uint64_t base2 = base1 + dd * half, left = ntiles - base2;  // < grid
  const uint64_t rank2 = favoured ? (b >> 1) : half + (b >> 1);   // favoured workgroups first
  q.s2 = base2 + rank2;
  q.n2 = rank2 < left ? 1 : 0;
}

// Workgroup b's tiles of the interleaved split of `ntiles` over `grid` workgroups with the blockIdx
// parity `fpar` favoured (skewed: even grid, `ra` / `dd` precomputed on the host — no 64-bit
// division on the device). Unskewed: tiles b, b + grid, ... (run 0 over the ra = ntiles / grid
// whole rounds, run 2 = the leftover tile of the first ntiles % grid workgroups).
// GPU test: tests/test_kernels_gpu.py::test_xcd_weighted_split.
__device__ __forceinline__ TileSeq weighted_tiles(uint64_t ntiles, uint64_t grid, bool skewed, unsigned fpar,
                                                  uint64_t ra, uint64_t dd, uint64_t b) {
  TileSeq q{};
  q.s0 = b;
  q.st0 = grid;
  q.n0 = static_cast<uint32_t>(ra);
  if (!skewed) {
    q.s2 = ra * grid + b;
    q.n2 = b < ntiles - ra * grid ? 1 : 0;
    return q;
  }
  weighted_tail(q, ntiles, grid, fpar, ra, dd, b);
  return q;
}

// Which XCD runs workgroup b is (b + the XCD of workgroup 0) % 8, and that start is not fixed:
// tools/xcd_balance.py always saw workgroup 0 on XCC 0, but the reduction app's launches were
// dealt otherwise (favouring odd blockIdx slowed it, odd XCCs speed it up; profiles/r4_ab/), so
// the favoured blockIdx parity cannot be chosen on the host.
// The launch's workgroup 0 publishes its XCC's parity, tagged with the launch's fan-in epoch, into
// Workspace fan[2..3] (uncached); every workgroup loads it some tiles before its common rounds end
// and derives the same favoured parity from it — the split stays a bijection whatever the deal.
struct XcdAnchor {
  uint64_t* word;     // null: the split is complete up front (q); else q is run 0 (>= 1 tile) only
  unsigned favour;    // XCC parity taking the extra rounds (xskew > 0: odd)
  bool publish;       // workgroup 0
  unsigned* err;      // sticky error word (Workspace fan[1]); value 2 (bit 1): the anchor never arrived
  uint64_t bound;     // wait bound in wall-clock ticks
  uint64_t delay;     // test hook: workgroup 0 sleeps this long before publishing (0: none)
  uint64_t ntiles, grid, ra, dd, b;
};

constexpr uint32_t kAnchorLead = 8;

// this launch's fan-in epoch (fan[0] + 1, never 0: the tag of a zeroed slot)
__device__ __forceinline__ unsigned fan_epoch(unsigned fan_raw) {
  const unsigned e = __builtin_amdgcn_readfirstlane(fan_raw) + 1u;
  return e == 0 ? 1u : e;
}  // tiles before the common rounds end that the anchor is loaded

__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v))) |
         static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32))) << 32;
}

// The anchored runs 1 and 2: `w` is the anchor as loaded; re-polled (bounded) while it is an earlier
// launch's. Returns true (uniform) if the anchor never arrived within the bound: this workgroup then
// streams the parity-0 tail, which need not match the other workgroups' — the split is no longer a
// bijection, so the caller must poison the launch's result (sticky value 2 (bit 1) of fan[1] is set here).
__device__ __forceinline__ bool resolve_anchor(TileSeq& q, const XcdAnchor& x, unsigned fan_raw, uint64_t w) {
  const uint64_t tag = static_cast<uint64_t>(fan_epoch(fan_raw)) << 32;
  bool late = false;
  w = rfl64(w);
  if ((w & ~0xffffffffull) != tag) {
    const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
    for (;;) {
      __builtin_amdgcn_s_sleep(1);
      w = rfl64(__hip_atomic_load(x.word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if ((w & ~0xffffffffull) == tag) break;
      if (static_cast<uint64_t>(wall_clock64()) - t0 > x.bound) {  // reported, never silent
        if (threadIdx.x == 0) __hip_atomic_fetch_or(x.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        w = tag;
        late = true;
        break;
      }
    }
  }
  // favoured blockIdx parity: the one that lands on XCCs of parity `favour`
  weighted_tail(q, x.ntiles, x.grid, x.favour ^ static_cast<unsigned>(w & 1u), x.ra, x.dd, x.b);
  q.s1 = rfl64(q.s1), q.st1 = rfl64(q.st1), q.s2 = rfl64(q.s2);
  q.n1 = __builtin_amdgcn_readfirstlane(q.n1), q.n2 = __builtin_amdgcn_readfirstlane(q.n2);
  if (q.n1 == 0) q.s1 = q.s2, q.n1 = q.n2, q.n2 = 0;
  return late;
}

// 8-byte integer MIN / MAX: gfx950 has no 64-bit integer min / max, so each element costs a compare
// (into VCC) and two selects, and folding a vector's two elements into one accumulator chains two
// such steps with a VCC wait state between them. Folded alternately into two accumulators, the two
// chains interleave (round 6, VERDICT r5 item 5: +0.24 % for int64 MIN, profiles/r6_ops/). The same
// split of the widening sums (int32 into int64, fp32 into fp64) measured 0-0.9 % SLOWER
// (profiles/r6_fold/), so they keep the single chain.
template <class OpT, class T, class AccT>
inline constexpr bool kSplitFold = std::is_integral_v<AccT> && sizeof(AccT) == 8 && !std::is_same_v<OpT, SumOp>;

template <class OpT, class T, class AccT, class V, int N>
__device__ __forceinline__ void consume_vec(AccT& a, AccT& b, const V& v) {
  if constexpr (kSplitFold<OpT, T, AccT>) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if (k & 1) b = OpT::apply(b, OpT::pre(elem<T, AccT>(v, k)));
      else a = OpT::apply(a, OpT::pre(elem<T, AccT>(v, k)));
    }
  } else {
#pragma unroll
    for (int k = 0; k < N; ++k) a = OpT::apply(a, OpT::pre(elem<T, AccT>(v, k)));
  }
}

// The window body over a TileSeq. The next tile is found incrementally with 32-bit uniform counters
// (scalar compares and branches: gfx950's SALU has no 64-bit less-than, and a first version that
// indexed the runs with 64-bit compares put them on the VALU in front of every tile's loads, 0.15-0.4 %
// slower than the single-run loop, profiles/r4_ab/). With an anchor, runs 1 and 2 are resolved when
// run 0 ends; the loop is split where the anchor's load issues (no load under a branch in the loop:
// hipcc's wait counts would turn conservative for every tile).
// `anchor_late` is set (uniform) when the anchor wait reached its bound (resolve_anchor).
template <class OpT, class T, class AccT, class V, int N, int BLOCK, int UNROLL, int WIN>
__device__ __forceinline__ uint32_t stream_window_seq(AccT (&acc)[UNROLL], const V* __restrict__ vin, TileSeq q,
                                                      const XcdAnchor& x, unsigned fan_raw, bool& anchor_late) {
  static_assert(UNROLL % WIN == 0, "the window must divide the unroll");
  constexpr uint64_t kTile = static_cast<uint64_t>(BLOCK) * UNROLL;
  constexpr uint32_t kStride = BLOCK * 16;
  // every field is uniform over the workgroup; say so, or the divergence analysis may keep them in
  // VGPRs and wrap each tile's loads in a readfirstlane waterfall loop
  q.s0 = rfl64(q.s0), q.st0 = rfl64(q.st0), q.s1 = rfl64(q.s1), q.st1 = rfl64(q.st1), q.s2 = rfl64(q.s2);
  q.n0 = __builtin_amdgcn_readfirstlane(q.n0), q.n1 = __builtin_amdgcn_readfirstlane(q.n1);
  q.n2 = __builtin_amdgcn_readfirstlane(q.n2);
  const bool anchored = x.word != nullptr;
  // runs in order, empty ones dropped: (start, step, count) of the current run, then the rest
  if (q.n0 == 0) {
    q.s0 = q.s1, q.st0 = q.st1, q.n0 = q.n1;
    q.s1 = q.s2, q.n1 = q.n2, q.n2 = 0;
    if (q.n0 == 0) q.s0 = q.s1, q.n0 = q.n1, q.n1 = 0;
  } else if (q.n1 == 0) {
    q.s1 = q.s2, q.n1 = q.n2, q.n2 = 0;
  }
  const bool pending = anchored;  // runs 1 and 2 resolved when run 0 (>= 1 tile when anchored) ends
  uint32_t n = q.count();  // tiles left, the current one included (run 0's only while pending)
  if (n == 0) return 0;
  uint32_t total = n;
  uint64_t t = q.s0, st = q.st0;
  uint32_t left = q.n0;  // tiles of the current run from t on
  const uint32_t voff = threadIdx.x * 16;
  __amdgpu_buffer_rsrc_t rp = tile_rsrc(vin + t * kTile);
  AccT acc2[kSplitFold<OpT, T, AccT> ? UNROLL : 1];  // the second accumulators of a split fold
#pragma unroll
  for (int u = 0; u < (kSplitFold<OpT, T, AccT> ? UNROLL : 1); ++u) acc2[u] = OpT::template identity<AccT>();
  V buf[WIN];
#pragma unroll
  for (int j = 0; j < WIN; ++j) buf[j] = ld_buf_nt<V>(rp, voff, j * kStride);
  // Workgroup 0 publishes its XCC's parity for this launch, after the first loads: the tag's wait
  // (the fan-in epoch, loaded at the kernel's start) is then no later than the first consume's.
  if (anchored && x.publish && threadIdx.x == 0) {
    if (x.delay) {  // test hook: a late anchor
      const uint64_t d0 = static_cast<uint64_t>(wall_clock64());
      while (static_cast<uint64_t>(wall_clock64()) - d0 < x.delay) __builtin_amdgcn_s_sleep(127);
    }
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint64_t tag = static_cast<uint64_t>(fan_epoch(fan_raw)) << 32;
    __hip_atomic_store(x.word, tag | (xcc & 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  auto step = [&]() {  // the next tile's loads under this one's consume: the loose window of stream_window
    if (left > 1) {
      t += st;
      --left;
    } else {  // the next run (runs 1 and 2 share run 1's step; run 2 holds at most one tile)
      t = q.s1;
      st = q.st1;
      left = q.n1;
      q.s1 = q.s2;
      q.n1 = q.n2;
      q.n2 = 0;
    }
    const __amdgpu_buffer_rsrc_t rq = tile_rsrc(vin + t * kTile);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      consume_vec<OpT, T, AccT, V, N>(acc[u], acc2[u], buf[u % WIN]);
      const int j = u + WIN;
      buf[u % WIN] = j < UNROLL ? ld_buf_nt<V>(rp, voff, j * kStride) : ld_buf_nt<V>(rq, voff, (j - UNROLL) * kStride);
      __builtin_amdgcn_sched_barrier(0);
    }
    rp = rq;
  };
  // (no unrolling: a constant-trip copy is straight-line code, where hipcc hoists every tile's loads
  // to the top — the window gone)
  if (pending) {
    if (n > kAnchorLead) {
#pragma nounroll
      for (; n > kAnchorLead; --n) step();
      // the anchor's load, then one straight-line tile: every path to its use has >= WIN loads
      // issued after it, so its wait is vmcnt(WIN), not a drain of the window
      const uint64_t w = __hip_atomic_load(x.word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      step();
#pragma nounroll
      for (--n; n > 1; --n) step();
      anchor_late = resolve_anchor(q, x, fan_raw, w);
    } else {
#pragma nounroll
      for (; n > 1; --n) step();
      anchor_late = resolve_anchor(q, x, fan_raw, __hip_atomic_load(x.word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    n += q.n1 + q.n2;
    total += q.n1 + q.n2;
  }
#pragma nounroll
  for (; n > 1; --n) step();
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {  // the last tile: no loads of a next one
    consume_vec<OpT, T, AccT, V, N>(acc[u], acc2[u], buf[u % WIN]);
    const int j = u + WIN;
    if (j < UNROLL) buf[u % WIN] = ld_buf_nt<V>(rp, voff, j * kStride);
  }
  if constexpr (kSplitFold<OpT, T, AccT>) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc[u] = OpT::apply(acc[u], acc2[u]);
  }
  return total;
}

// One streaming body per plan: WIN > 0 the explicit load window over the (XCD-weighted) interleaved
// split, WIN == 0 hipcc's schedule of the plain loop over tiles b, b + grid, ... The loop has no
// per-load condition (cdna_hip_programming.md §5 trap (c)).
template <class OpT, class T, class AccT, int BLOCK, int UNROLL, bool NT, int WIN = 0>
__global__ __launch_bounds__(BLOCK) void reduce_stream(Args a) {
  using V = typename Vec16<T>::type;
  constexpr int N = Vec16<T>::N;
  __shared__ AccT lds[BLOCK / 64];

  AccT acc[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) acc[u] = OpT::template identity<AccT>();

  // Polled fan-in epoch of this launch: the load is issued before the streaming body and its value
  // first used after it, so its latency hides under the body's first loads (one VGPR; the ISA test
  // pins that no wait sits between it and the body). Every workgroup reads it before the finisher
  // can advance it: the finisher advances fan[0] only after every slot holds this epoch.
  const bool polled = a.slots && gridDim.x > 1;
  // the launch's fan-in epoch: the polled fan-in's, or a two-pass launch's (its finalize ends it)
  const bool epoch = (polled || a.two_pass_epoch) && gridDim.x > 1;
  const unsigned fan_raw = epoch ? __hip_atomic_load(a.fan, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;

  const V* __restrict__ vin = static_cast<const V*>(a.body);
  constexpr uint64_t kTile = static_cast<uint64_t>(BLOCK) * UNROLL;
  const uint64_t ntiles = a.nvec / kTile;
  const uint64_t grid = gridDim.x;
  uint32_t streamed = 0;  // full tiles of the window body (diagnostic stamps)
  bool anchor_late = false;  // the XCD anchor missed its bound: this workgroup's tiles may overlap others
  if constexpr (WIN > 0) {
    TileSeq q{};
    XcdAnchor x{};
    if (a.xskew != 0 && epoch && (grid & 1u) == 0 && a.x_ra > 0) {  // weighted, anchored to the XCDs
      q.s0 = blockIdx.x;
      q.st0 = grid;
      q.n0 = static_cast<uint32_t>(a.x_ra);
      x.word = reinterpret_cast<uint64_t*>(a.fan + 2);
      x.favour = a.xskew > 0 ? 1u : 0u;
      x.publish = blockIdx.x == 0;
      x.err = a.fan + 1;
      x.bound = a.fan_bound;
      x.delay = a.anchor_delay;
      x.ntiles = ntiles, x.grid = grid, x.ra = a.x_ra, x.dd = a.x_dd, x.b = blockIdx.x;
    } else {  // unskewed, or skewed by blockIdx parity (no fan-in epoch to tag an anchor with)
      q = weighted_tiles(ntiles, grid, a.xskew != 0 && (grid & 1u) == 0, a.xskew > 0 ? 1u : 0u, a.x_ra, a.x_dd,
                         blockIdx.x);
    }
    // fan_raw (the launch's fan-in epoch, the anchor's tag) passed as is: a copy into the struct
    // would be a VGPR move that waits for its load before the first tile's loads issue
    streamed = stream_window_seq<OpT, T, AccT, V, N, BLOCK, UNROLL, WIN>(acc, vin, q, x, fan_raw, anchor_late);
  } else {
    for (uint64_t t = blockIdx.x; t < ntiles; t += grid) {
      V v[UNROLL];
      load_tile<V, BLOCK, UNROLL, NT>(v, vin + t * kTile + threadIdx.x);
      consume_tile<OpT, T, AccT, V, N, UNROLL>(acc, v);
    }
  }
  // Vectors past the last full tile, grid-strided.
  for (uint64_t i = ntiles * kTile + static_cast<uint64_t>(blockIdx.x) * BLOCK + threadIdx.x; i < a.nvec;
       i += static_cast<uint64_t>(gridDim.x) * BLOCK) {
    const V v = vin[i];
#pragma unroll
    for (int k = 0; k < N; ++k) acc[0] = OpT::apply(acc[0], OpT::pre(elem<T, AccT>(v, k)));
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
  if (a.wg_stamps && threadIdx.x == 0) {  // diagnostic: when this workgroup's streaming ended
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t_end = static_cast<uint64_t>(wall_clock64());
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uint64_t* st = a.wg_stamps + 3 * static_cast<uint64_t>(blockIdx.x);
    st[0] = t_end;
    st[1] = xcc & 0xfu;
    st[2] = WIN > 0 ? streamed : (ntiles > blockIdx.x ? (ntiles - blockIdx.x + grid - 1) / grid : 0);
  }

  // Fused cross-rank finish: this launch's epoch (counter + 1; only the finishing workgroup bumps
  // the counter, and it runs last) and the sticky error word. Only the finisher loads them, where
  // their latency hides: the polled fan-in's finisher (known up front) right after publishing its
  // own partial, under its poll of the others'; a one-workgroup launch just before the exchange.
  // (Loading them in every workgroup cost each workgroup the loads' round trip before its block
  // barrier, ~1.4 us per fused step, bench.py decomposition, round 4; loading them before the body
  // changed hipcc's load scheduling of it: 76 -> 60 VGPRs and 7.3 -> 5.1 TB/s at 512 x 16.)
  unsigned xr_epoch = 0, xr_err = 0;
  auto load_xr = [&]() {
    xr_epoch = xrank_next_epoch(__hip_atomic_load(a.xrank->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    xr_err = __hip_atomic_load(a.xrank->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  AccT v = block_reduce<OpT, AccT, BLOCK>(acc[0], lds);
  if (a.two_pass) {  // two-pass mode: the finalize kernel (kernel boundary) reads these
    // (a late anchor: the finalize sees fan[1] value 2 (bit 1) after the kernel boundary and poisons the result)
    if (threadIdx.x == 0) static_cast<AccT*>(a.partials)[blockIdx.x] = anchor_late ? poisoned<OpT, AccT>() : v;
    return;
  }

  // ---- one workgroup (small n): it is the finisher by construction — no partial publish, no poll.
  if (gridDim.x == 1) {
    if (threadIdx.x < 64) {
      bool xf = false;
      if (a.xrank) load_xr();
      if (a.xrank) v = xrank_finish<OpT, AccT>(a.xrank, xrank_prefetch(a.xrank, xr_epoch, xr_err), v, false, xf);
      if (threadIdx.x == 0) *static_cast<AccT*>(a.out) = xf ? poisoned<OpT, AccT>() : v;
    }
    return;
  }

  // ---- polled fan-in (every single-pass launch of more than one workgroup): no tickets, no
  // publish-then-drain wait. Every workgroup stores its partial as two tagged words (the data
  // carries its own validity, as in the cross-rank mailbox) and exits; the last-indexed workgroup —
  // with interleaved tiles one of the first to run out of work — polls all slots, folds them in slot
  // order (deterministic), and finishes. The finisher's path after the last partial lands is one
  // store + one poll round. Slots live in uncached memory, so polls always see the other XCDs' stores.
  const unsigned fan_e = fan_epoch(fan_raw);
  const uint64_t tag = static_cast<uint64_t>(fan_e) << 32;
  // A workgroup whose XCD anchor was late (its tiles may double-count or skip others') does not
  // publish: the finisher then reaches its bound and poisons the launch — never a plausible sum of
  // the wrong tiles. (Publishing a flag instead would cost the finisher a load round trip after its
  // poll on every launch, to order it after the slot stores.)
  if (anchor_late && blockIdx.x != gridDim.x - 1) return;
  if (threadIdx.x == 0) {
    if (static_cast<int>(blockIdx.x) == a.delay_wg) {  // test hook: a slow workgroup
      const uint64_t d0 = static_cast<uint64_t>(wall_clock64());
      while (static_cast<uint64_t>(wall_clock64()) - d0 < a.delay_ticks) __builtin_amdgcn_s_sleep(127);
    }
    const uint64_t bits = to_bits64(v);
    uint64_t* sl = a.slots + 2 * static_cast<uint64_t>(blockIdx.x);
    __hip_atomic_store(sl, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sl + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (blockIdx.x != gridDim.x - 1) return;
  // Segmented launches: the earlier segments' results (kernel boundaries ago: plain loads), one per
  // lane, issued before the poll so their latency hides under it.
  AccT carried = OpT::template identity<AccT>();
  if (threadIdx.x < a.ncarry) carried = static_cast<const AccT*>(a.carry)[threadIdx.x];
  // The finisher: start the cross-rank descriptor loads and the sticky-error load now, they land
  // while it polls.
  XrankLane xl{};
  if (a.xrank && threadIdx.x < 64) {
    load_xr();
    xl = xrank_prefetch(a.xrank, xr_epoch, xr_err);
  }
  const unsigned fan_err = __hip_atomic_load(a.fan + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  AccT t = OpT::template identity<AccT>();
  // Bounded like every device-side wait here (all workgroups of this launch always publish, so a
  // correct launch never reaches the bound; it keeps a stalled or misused launch from hanging the
  // GPU, and reaching it is reported, never folded into a plausible-looking result).
  const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
  const uint64_t kBound = a.fan_bound;
  bool late = false;
  if (gridDim.x <= kPollSlots * BLOCK) {
    // Each lane polls ALL its slots (<= kPollSlots) every round, so the finish costs one poll round
    // trip after the last store lands, not one per slot.
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
        if ((pending & (1u << k)) && (lo[k] & ~0xffffffffull) == tag && (hi[k] & ~0xffffffffull) == tag)
          pending &= ~(1u << k);
      if (!pending) break;
      if (static_cast<uint64_t>(wall_clock64()) - t0 > kBound) {
        late = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int k = 0; k < kPollSlots; ++k)  // fold in slot order (deterministic)
      if (threadIdx.x + k * BLOCK < gridDim.x)
        t = OpT::apply(t, from_bits64<AccT>((lo[k] & 0xffffffffull) | (hi[k] << 32)));
  } else {  // very large grids (user --maxblocks / wg-per-cu): slot by slot
    for (unsigned i = threadIdx.x; i < gridDim.x; i += BLOCK) {
      const uint64_t* sl = a.slots + 2 * static_cast<uint64_t>(i);
      uint64_t l, h;
      for (;;) {
        l = __hip_atomic_load(sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        h = __hip_atomic_load(sl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((l & ~0xffffffffull) == tag && (h & ~0xffffffffull) == tag) break;
        if (late || static_cast<uint64_t>(wall_clock64()) - t0 > kBound) {
          late = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      t = OpT::apply(t, from_bits64<AccT>((l & 0xffffffffull) | (h << 32)));
    }
  }
  // Any lane past the bound (or an earlier launch's sticky error) poisons this launch's result.
  const bool bad = __syncthreads_or(late) || fan_err != 0 || anchor_late;
  t = block_reduce<OpT, AccT, BLOCK>(OpT::apply(t, carried), lds);
  if (fan_e == 0xffffffffu) {  // the epoch wraps after this launch: invalidate every slot first
    __syncthreads();
    for (unsigned i = threadIdx.x; i < 2u * a.fan_slots; i += BLOCK)
      __hip_atomic_store(a.slots + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0)  // and the XCD anchor (XcdAnchor), tagged with the same epochs
      __hip_atomic_store(reinterpret_cast<uint64_t*>(a.fan + 2), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
  }
  if (threadIdx.x < 64) {
    bool xf = false;
    if (a.xrank) t = xrank_finish<OpT, AccT>(a.xrank, xl, bad ? poisoned<OpT, AccT>() : t, bad, xf);
    if (threadIdx.x == 0) {
      *static_cast<AccT*>(a.out) = (bad || xf) ? poisoned<OpT, AccT>() : t;
      if (bad) __hip_atomic_fetch_or(a.fan + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // every slot of this launch has been read (or abandoned): the next launch's epoch
      __hip_atomic_store(a.fan, fan_e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Second level of the two-pass path (and the on-device fold for reduce_finalize): one
// workgroup folds `count` values. Launched after a kernel boundary, so plain loads are fine.
// `fan` (two-pass launches of reduce_stream; null otherwise): this launch then also ends the first
// level's fan-in epoch, as the polled fan-in's finisher does (the first level's workgroups tag
// the XCD anchor with it), zeroing the workspace's `fan_slots` polled slots and the anchor first
// when the epoch wraps.
template <class OpT, class AccT>
__global__ __launch_bounds__(256) void finalize(const AccT* __restrict__ partials, uint64_t count,
                                                AccT* __restrict__ out, unsigned* fan, uint64_t* slots,
                                                unsigned fan_slots) {
  __shared__ AccT lds[4];
  AccT s = OpT::template identity<AccT>();
  for (uint64_t i = threadIdx.x; i < count; i += 256) s = OpT::apply(s, partials[i]);
  s = block_reduce<OpT, AccT, 256>(s, lds);
  // a first-level workgroup's XCD anchor was late (sticky value 2, bit 1): its tiles were not the split's
  const bool anchor_err = fan && (__hip_atomic_load(fan + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2u);
  if (threadIdx.x == 0) *out = anchor_err ? poisoned<OpT, AccT>() : s;
  if (fan) {
    const unsigned e = fan_epoch(__hip_atomic_load(fan, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (e == 0xffffffffu) {  // the epoch wraps after this launch: invalidate every tag first
      for (unsigned i = threadIdx.x; i < 2u * fan_slots; i += 256)
        __hip_atomic_store(slots + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<uint64_t*>(fan + 2), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
    }
    if (threadIdx.x == 0) __hip_atomic_store(fan, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
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
// Dispatch table keyed by (op, dtype, acc, block, unroll, policy, body); replaces the reference's
// runtime switch over 20 template instantiations per (op, T).
// ----------------------------------------------------------------------------------------------
namespace detail {

using LaunchFn = void (*)(const kern::Args&, int grid, hipStream_t);

template <class OpT, class T, class AccT, int BLOCK, int UNROLL, bool NT, int WIN = 0>
void launch_stream(const kern::Args& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((kern::reduce_stream<OpT, T, AccT, BLOCK, UNROLL, NT, WIN>), dim3(grid), dim3(BLOCK), 0, s, a);
}

constexpr int kBlocks[] = {256, 512, 1024};
constexpr int kUnrolls[] = {2, 4, 8, 16};
constexpr int kNumBlocks = 3;
constexpr int kNumUnrolls = 4;

constexpr int kCombos = 29;

// Body schedules: 0 = hipcc's own schedule of the plain loop, 1 / 2 = explicit load window of 2 / 4
// registers per thread (stream_window_seq; nt only).
constexpr int kNumBodies = 3;
struct Table {
  LaunchFn fn[kCombos][kNumBlocks][kNumUnrolls][2][kNumBodies];  // [..][policy nt][body]
};

// Explicit windows are instantiated for the non-temporal policy, 256- and 512-thread blocks and
// unroll 2..8 (profiles/r3_window/: the measured winners and their neighbours); elsewhere null.
constexpr bool window_ok(int b, int u, int w) { return (b == 256 || b == 512) && u <= 8 && u % w == 0; }

template <class OpT, class T, class AccT, int BI, int UI>
void fill_one(Table& tb, int c) {
  constexpr int B = kBlocks[BI];
  constexpr int U = kUnrolls[UI];
  tb.fn[c][BI][UI][0][0] = launch_stream<OpT, T, AccT, B, U, false>;
  tb.fn[c][BI][UI][1][0] = launch_stream<OpT, T, AccT, B, U, true>;
  if constexpr (window_ok(B, U, 2)) tb.fn[c][BI][UI][1][1] = launch_stream<OpT, T, AccT, B, U, true, 2>;
  if constexpr (window_ok(B, U, 4)) tb.fn[c][BI][UI][1][2] = launch_stream<OpT, T, AccT, B, U, true, 4>;
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

// One filler per TU (reduce_tab_<group>.hip): sets tb.fn[c] for its combos c.
void fill_table_int32(Table& tb);  // combos 0..3
void fill_table_int64(Table& tb);  // combos 4..6
void fill_table_f32(Table& tb);  // combos 7..10
void fill_table_f64(Table& tb);  // combos 11..13
void fill_table_bf16(Table& tb);  // combos 14..16
void fill_table_f16(Table& tb);  // combos 17..19
void fill_table_sumsq(Table& tb);  // combos 20..24
void fill_table_absmax(Table& tb);  // combos 25..28

}  // namespace detail
}  // namespace mireduce
