// Diagnostic: per-workgroup timeline of the streaming reduction body on gfx950.
//
// Question it answers: at the 1 GB per-GPU shard of the 8-GPU run, where do the ~2 % between the
// 1 GB rate (7.12 TB/s) and the 8 GB rate (7.29 TB/s) go — launch ramp, end-of-kernel skew
// between workgroups (static grid-stride assignment: the kernel ends with its slowest CU), or
// the steady-state rate of the plan?
//
// Variants (float64 SUM body, 16-byte nt loads, as csrc/kernels/reduce.hip's reduce_stream):
//   static  grid-stride over BLOCK*UNROLL-vector tiles (the production body);
//   dynamic tiles handed out by a device-scope counter: big chunks of CHUNK tiles first, single
//           tiles for the last ~TAILPCT % (guided self-scheduling), next chunk prefetched one
//           chunk ahead so the atomic's latency hides behind the current chunk's loads.
// Each variant runs without stamps for timing (hipEvents, interleaved rounds, median) and once
// with stamps (s_memrealtime, 100 MHz, at entry and after the last consumed load; XCC id) to get
// the start/end distribution. Partials are folded by a second tiny kernel: the fan-in is not
// what is measured here (profiles/r1_session3/fanin_groups_sweep.txt).
//
//   build/bin/wg_timeline [--n=125000000] [--rounds=7] [--iters=20] [--set=mlp|sched]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                    \
    }                                                                                  \
  } while (0)

using V = double __attribute__((ext_vector_type(2)));

struct TArgs {
  const V* v;
  uint64_t nvec;
  double* partials;
  unsigned long long* ctr;   // dynamic: monotonically increasing across launches
  unsigned long long base;   // dynamic: counter value at this launch's start
  uint64_t nbig;             // dynamic: number of big chunks
  uint64_t chunk;            // dynamic: tiles per big chunk
  uint64_t nchunks;          // dynamic: big chunks + single-tile chunks
  uint64_t* stamps;          // [grid * 4] start, end, xcc, tiles (nullptr: no stamps)
  unsigned long long* qctr;  // tail-steal: 8 queue counters, 16 words apart (zeroed by fold)
};

__device__ __forceinline__ uint64_t now_rt() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xf;
}

// MODE 0: as written (the compiler's scheduler decides how many loads stay in flight — it
// interleaves them with the adds to save registers); MODE 1: all UNROLL loads issued before the
// first add (sched_barrier); MODE 2: software-pipelined with barriers — the next tile's loads are
// issued before this tile's adds (two register sets).
template <int BLOCK, int UNROLL, int MODE>
__device__ __forceinline__ void tile(double (&acc)[UNROLL], const V* p) {
  V v[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(p + u * BLOCK);
  if constexpr (MODE == 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) acc[u] += v[u][0] + v[u][1];
}

template <int UNROLL>
__device__ __forceinline__ void consume(double (&acc)[UNROLL], const V (&v)[UNROLL]) {
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) acc[u] += v[u][0] + v[u][1];
}

template <int BLOCK, int UNROLL>
__device__ __forceinline__ void issue(V (&v)[UNROLL], const V* p) {
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(p + u * BLOCK);
}

template <int BLOCK>
__device__ __forceinline__ double block_sum(double s, double* lds) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = s;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x < 64) {
    t = threadIdx.x < BLOCK / 64 ? lds[threadIdx.x] : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
  }
  return t;
}

template <int BLOCK, int UNROLL, bool DYN, int MODE>
__global__ __launch_bounds__(BLOCK) void body(TArgs a) {
  __shared__ double lds[BLOCK / 64];
  __shared__ unsigned long long next_k[2];
  const uint64_t t0 = a.stamps ? now_rt() : 0;
  double acc[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) acc[u] = 0.0;
  constexpr uint64_t kTile = static_cast<uint64_t>(BLOCK) * UNROLL;
  const uint64_t ntiles = a.nvec / kTile;
  uint64_t done = 0;
  if constexpr (!DYN && MODE == 2) {
    if (blockIdx.x < ntiles) {
      V cur[UNROLL];
      issue<BLOCK, UNROLL>(cur, a.v + blockIdx.x * kTile + threadIdx.x);
      for (uint64_t t = blockIdx.x + gridDim.x; t < ntiles; t += gridDim.x, ++done) {
        V nxt[UNROLL];
        issue<BLOCK, UNROLL>(nxt, a.v + t * kTile + threadIdx.x);
        __builtin_amdgcn_sched_barrier(0);
        consume<UNROLL>(acc, cur);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) cur[u] = nxt[u];
      }
      consume<UNROLL>(acc, cur);
      ++done;
    }
  } else if constexpr (!DYN && MODE == 5) {
    // rotated grid-stride: in round k workgroup b takes tile k*grid + (b + k*a.chunk) % grid, so
    // the tiles an XCD reads (b % 8 under round-robin dispatch) cycle through every address
    // residue instead of always sitting at offset (b % 8) * tile within each 8-tile stripe.
    const uint64_t g = gridDim.x;
    for (uint64_t k = 0;; ++k) {
      const uint64_t t = k * g + (blockIdx.x + k * a.chunk) % g;
      if (t >= ntiles) {
        if (k * g >= ntiles) break;
        continue;
      }
      tile<BLOCK, UNROLL, 0>(acc, a.v + t * kTile + threadIdx.x);
      ++done;
    }
  } else if constexpr (!DYN && MODE == 6) {
    // XCD-residue shift: within each stripe of 8 consecutive tiles, workgroup b takes tile
    // (b + a.chunk) % 8 instead of b % 8, so under round-robin dispatch (XCD = b % 8) XCD x reads
    // the tiles of address residue (x + shift) % 8 — shifts 0..7 measure every (XCD, residue) pair.
    const uint64_t g = gridDim.x;
    const uint64_t b = (blockIdx.x & ~7ull) | ((blockIdx.x + a.chunk) & 7ull);
    for (uint64_t t = b; t < ntiles; t += g, ++done) tile<BLOCK, UNROLL, 0>(acc, a.v + t * kTile + threadIdx.x);
  } else if constexpr (!DYN && MODE >= 100) {
    // Explicit load window (MODE = 100 + D, D | UNROLL): the thread's loads form one sequence over its
    // interleaved tiles; exactly D are in flight — each step consumes the load issued D steps earlier
    // and issues the next one, and a sched_barrier between steps keeps hipcc's scheduler from
    // regrouping them (its own grouping moves with unrelated code: round 3 found a 2.5 % swing).
    constexpr int D = MODE - 100;
    static_assert(UNROLL % D == 0, "window must divide the unroll");
    const uint64_t g = gridDim.x;
    const V* base = a.v + threadIdx.x;
    uint64_t t = blockIdx.x;
    if (t < ntiles) {
      V buf[D];
#pragma unroll
      for (int j = 0; j < D; ++j) buf[j] = __builtin_nontemporal_load(base + t * kTile + j * BLOCK);
      for (; t + g < ntiles; t += g, ++done) {
        const V* p = base + t * kTile;
        const V* q = base + (t + g) * kTile;
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
          acc[u] += buf[u % D][0] + buf[u % D][1];
          const int j = u + D;
          buf[u % D] = __builtin_nontemporal_load(j < UNROLL ? p + j * BLOCK : q + (j - UNROLL) * BLOCK);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      const V* p = base + t * kTile;  // last tile: no next-tile loads
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        acc[u] += buf[u % D][0] + buf[u % D][1];
        const int j = u + D;
        if (j < UNROLL) buf[u % D] = __builtin_nontemporal_load(p + j * BLOCK);
      }
      ++done;
    }
  } else if constexpr (!DYN && MODE == 7) {
    // Static rounds over tiles [0, a.nbig) (a.nbig a multiple of the grid), then every remaining
    // vector as WAVE granules of a.chunk wave-tiles (64 lanes x UNROLL vectors each), dealt from 8
    // heads (a.qctr + 16 h, head h owning a contiguous range of a.nchunks granules): lane 0 takes a
    // granule with one returning device-scope atomic, issued one granule AHEAD (before the current
    // granule's loads, so the in-order vmcnt wait of those loads covers it), broadcast with
    // readfirstlane — no LDS, no barrier. A wave starts at head (wave id % 8) and moves on when a
    // head runs dry, so fast XCDs simply take more granules.
    for (uint64_t t = blockIdx.x; t < a.nbig; t += gridDim.x, ++done) tile<BLOCK, UNROLL, 0>(acc, a.v + t * kTile + threadIdx.x);
    const unsigned lane = threadIdx.x & 63;
    const uint64_t v0 = a.nbig * kTile;
    const uint64_t gsz = 64ull * UNROLL * a.chunk;
    const uint64_t ng = a.nvec > v0 ? (a.nvec - v0 + gsz - 1) / gsz : 0;
    const uint64_t per = a.nchunks;  // granules per head
    unsigned h = (blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6)) & 7u;
    unsigned tried = 0;
    auto grab = [&](unsigned hh) -> uint64_t {
      unsigned long long r = 0;
      if (lane == 0) r = __hip_atomic_fetch_add(a.qctr + 16 * hh, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned lo = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(r));
      const unsigned hi = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(r >> 32));
      return (static_cast<uint64_t>(hi) << 32) | lo;
    };
    auto head_size = [&](unsigned hh) -> uint64_t {
      const uint64_t b0 = hh * per;
      return b0 >= ng ? 0 : (b0 + per <= ng ? per : ng - b0);
    };
    uint64_t g = ng ? grab(h) : 0;
    while (ng) {
      while (g >= head_size(h)) {  // this head is dry: the next one
        if (++tried == 8) break;
        h = (h + 1) & 7u;
        g = grab(h);
      }
      if (tried == 8) break;
      const uint64_t cur = h * per + g;
      const uint64_t nxt = grab(h);  // one granule ahead
      const uint64_t base = v0 + cur * gsz + lane;
      for (uint64_t c = 0; c < a.chunk; ++c) {
        V v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
          const uint64_t i = base + (c * UNROLL + u) * 64;
          v[u] = __builtin_nontemporal_load(a.v + (i < a.nvec ? i : a.nvec - 1));
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
          if (base + (c * UNROLL + u) * 64 < a.nvec) acc[u] += v[u][0] + v[u][1];
      }
      ++done;
      g = nxt;
    }
  } else if constexpr (!DYN && MODE == 4) {
    // static grid-stride over the first a.nbig tiles, then the tail [a.nbig, ntiles) as 8 queues
    // of a.nchunks granules (a.chunk tiles each); a workgroup drains its own XCD's queue first,
    // then the others. A plain sc1 read skips exhausted queues without an atomic.
    __shared__ unsigned long long grab[2];
    for (uint64_t t = blockIdx.x; t < a.nbig; t += gridDim.x, ++done) tile<BLOCK, UNROLL, 0>(acc, a.v + t * kTile + threadIdx.x);
    const unsigned x = xcc_id();
    int slot = 0;
    for (unsigned j = 0; j < 8; ++j) {
      const unsigned q = (x + j) & 7u;
      unsigned long long* c = a.qctr + 16 * q;
      while (true) {
        if (threadIdx.x == 0) {
          unsigned long long g = a.nchunks;
          if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.nchunks)
            g = __hip_atomic_fetch_add(c, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          grab[slot] = g;
        }
        __syncthreads();
        const unsigned long long g = grab[slot];
        slot ^= 1;
        if (g >= a.nchunks) break;
        const uint64_t first = a.nbig + (q * a.nchunks + g) * a.chunk;
        const uint64_t last = first + a.chunk < ntiles ? first + a.chunk : ntiles;
        for (uint64_t t = first; t < last; ++t, ++done) tile<BLOCK, UNROLL, 0>(acc, a.v + t * kTile + threadIdx.x);
      }
    }
  } else if constexpr (!DYN && MODE == 3) {
    // static, but in runs of a.chunk consecutive tiles (the dynamic variant's access window)
    const uint64_t runs = ntiles / a.chunk;
    for (uint64_t r = blockIdx.x; r < runs; r += gridDim.x)
      for (uint64_t t = r * a.chunk; t < (r + 1) * a.chunk; ++t, ++done) tile<BLOCK, UNROLL, 1>(acc, a.v + t * kTile + threadIdx.x);
    for (uint64_t t = runs * a.chunk + blockIdx.x; t < ntiles; t += gridDim.x, ++done)
      tile<BLOCK, UNROLL, 1>(acc, a.v + t * kTile + threadIdx.x);
  } else if constexpr (!DYN) {
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x, ++done) tile<BLOCK, UNROLL, MODE>(acc, a.v + t * kTile + threadIdx.x);
  } else {
    // chunk k -> tiles [first, first + count)
    auto range = [&](uint64_t k, uint64_t& first, uint64_t& count) {
      if (k < a.nbig) {
        first = k * a.chunk;
        count = a.chunk;
      } else {
        first = a.nbig * a.chunk + (k - a.nbig);
        count = 1;
      }
    };
    if (threadIdx.x == 0) next_k[0] = atomicAdd(a.ctr, 1ull) - a.base;
    __syncthreads();
    unsigned long long k = next_k[0];
    int slot = 1;
    while (k < a.nchunks) {
      // prefetch the next chunk index while this chunk's loads are in flight
      if (threadIdx.x == 0) next_k[slot] = atomicAdd(a.ctr, 1ull) - a.base;
      uint64_t first, count;
      range(k, first, count);
      for (uint64_t t = first; t < first + count; ++t, ++done) tile<BLOCK, UNROLL, MODE>(acc, a.v + t * kTile + threadIdx.x);
      __syncthreads();
      k = next_k[slot];
      slot ^= 1;
    }
  }
  // vectors past the last full tile (MODE 7 covers them in its dynamic part)
  if constexpr (MODE != 7)
    for (uint64_t i = ntiles * kTile + static_cast<uint64_t>(blockIdx.x) * BLOCK + threadIdx.x; i < a.nvec;
         i += static_cast<uint64_t>(gridDim.x) * BLOCK)
      acc[0] += a.v[i][0] + a.v[i][1];
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) s += acc[u];
  if (a.stamps && threadIdx.x == 0) {
    const uint64_t t1 = now_rt();
    uint64_t* st = a.stamps + 4 * static_cast<uint64_t>(blockIdx.x);
    st[0] = t0;
    st[1] = t1;
    st[2] = xcc_id();
    st[3] = done;
  }
  s = block_sum<BLOCK>(s, lds);
  if (threadIdx.x == 0) a.partials[blockIdx.x] = s;
}

__global__ void fold(const double* p, int n, double* out, unsigned long long* qctr) {
  if (threadIdx.x < 8) qctr[16 * threadIdx.x] = 0;  // tail-steal queues: ready for the next launch
  __shared__ double lds[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += p[i];
  s = block_sum<256>(s, lds);
  if (threadIdx.x == 0) *out = s;
}

__global__ void fill(V* v, uint64_t nvec) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < nvec; i += static_cast<uint64_t>(gridDim.x) * 256) {
    const double a = static_cast<double>((i * 2654435761ull) & 1023) / 1024.0;
    v[i] = V{a, 1.0 - a};  // each pair sums to exactly 1
  }
}

struct Variant {
  std::string name;
  int block, unroll, wpc;
  bool dyn;
  int chunk;      // tiles per big chunk
  double tailpct; // share of tiles handed out one by one
  void (*kern)(TArgs);
};

template <int B, int U, bool D, int M>
Variant mk(const char* name, int wpc, int chunk = 0, double tail = 0.0) {
  return {name, B, U, wpc, D, chunk, tail, body<B, U, D, M>};
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  uint64_t n = 125000000;
  int rounds = 7, iters = 20;
  std::string set = "sched";
  for (int i = 1; i < argc; ++i) {
    if (!std::strncmp(argv[i], "--n=", 4)) n = static_cast<uint64_t>(std::atof(argv[i] + 4));
    else if (!std::strncmp(argv[i], "--rounds=", 9)) rounds = std::atoi(argv[i] + 9);
    else if (!std::strncmp(argv[i], "--iters=", 8)) iters = std::atoi(argv[i] + 8);
    else if (!std::strncmp(argv[i], "--set=", 6)) set = argv[i] + 6;
    else {
      std::fprintf(stderr, "usage: wg_timeline [--n=N] [--rounds=R] [--iters=I] [--set=mlp|sched|rotate|steal|shift|wavetail|window]\n");
      return 1;
    }
  }
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t nvec = n / 2;
  V* v;
  double *partials, *out;
  unsigned long long *ctr, *qctr;
  uint64_t* stamps;
  CK(hipMalloc(&v, nvec * sizeof(V)));
  CK(hipMalloc(&partials, 8192 * sizeof(double)));
  CK(hipMalloc(&out, sizeof(double)));
  CK(hipMalloc(&ctr, sizeof(unsigned long long)));
  CK(hipMalloc(&qctr, 8 * 16 * sizeof(unsigned long long)));
  CK(hipMemset(qctr, 0, 8 * 16 * sizeof(unsigned long long)));
  CK(hipMalloc(&stamps, 8192 * 4 * sizeof(uint64_t)));
  CK(hipMemset(ctr, 0, sizeof(unsigned long long)));
  fill<<<4096, 256>>>(v, nvec);
  CK(hipDeviceSynchronize());
  const double expect = static_cast<double>(nvec);

  // --set=mlp: how many loads the scheduler keeps in flight; --set=sched: static-chunked and
  // dynamic assignment (profiles/r1_session3/wg_timeline/).
  std::vector<Variant> vars;
  if (set == "rotate") {
    vars = {
        mk<256, 2, false, 0>("s 256x2x3", 3),
        mk<256, 2, false, 5>("rot1 256x2x3", 3, 1),
        mk<256, 2, false, 5>("rot3 256x2x3", 3, 3),
        mk<256, 2, false, 5>("rot8 256x2x3", 3, 8),
        mk<512, 16, false, 0>("s 512x16x1", 1),
        mk<512, 16, false, 5>("rot1 512x16x1", 1, 1),
        mk<256, 4, false, 0>("s 256x4x2", 2),
        mk<256, 4, false, 5>("rot1 256x4x2", 2, 1),
    };
  } else if (set == "shift") {
    // (XCD, address residue) affinity: every shift for the production plans (grids are multiples of 8)
    vars = {
        mk<256, 2, false, 6>("sh0 256x2x3", 3, 0), mk<256, 2, false, 6>("sh1 256x2x3", 3, 1),
        mk<256, 2, false, 6>("sh2 256x2x3", 3, 2), mk<256, 2, false, 6>("sh3 256x2x3", 3, 3),
        mk<256, 2, false, 6>("sh4 256x2x3", 3, 4), mk<256, 2, false, 6>("sh5 256x2x3", 3, 5),
        mk<256, 2, false, 6>("sh6 256x2x3", 3, 6), mk<256, 2, false, 6>("sh7 256x2x3", 3, 7),
        mk<256, 8, false, 6>("sh0 256x8x1", 1, 0), mk<256, 8, false, 6>("sh1 256x8x1", 1, 1),
        mk<256, 8, false, 6>("sh2 256x8x1", 1, 2), mk<256, 8, false, 6>("sh3 256x8x1", 1, 3),
        mk<256, 8, false, 6>("sh4 256x8x1", 1, 4), mk<256, 8, false, 6>("sh5 256x8x1", 1, 5),
        mk<256, 8, false, 6>("sh6 256x8x1", 1, 6), mk<256, 8, false, 6>("sh7 256x8x1", 1, 7),
        mk<512, 8, false, 6>("sh0 512x8x1", 1, 0), mk<512, 8, false, 6>("sh1 512x8x1", 1, 1),
        mk<512, 8, false, 6>("sh2 512x8x1", 1, 2), mk<512, 8, false, 6>("sh3 512x8x1", 1, 3),
        mk<512, 8, false, 6>("sh4 512x8x1", 1, 4), mk<512, 8, false, 6>("sh5 512x8x1", 1, 5),
        mk<512, 8, false, 6>("sh6 512x8x1", 1, 6), mk<512, 8, false, 6>("sh7 512x8x1", 1, 7),
    };
  } else if (set == "window") {
    // explicit in-flight window per thread (MODE 100 + D) against hipcc's own schedule (MODE 0)
    vars = {
        mk<512, 16, false, 0>("s 512x16x1", 1),
        mk<512, 16, false, 102>("w2 512x16x1", 1), mk<512, 16, false, 104>("w4 512x16x1", 1),
        mk<512, 16, false, 108>("w8 512x16x1", 1), mk<512, 16, false, 116>("w16 512x16x1", 1),
        mk<256, 8, false, 0>("s 256x8x1", 1),
        mk<256, 8, false, 102>("w2 256x8x1", 1), mk<256, 8, false, 104>("w4 256x8x1", 1),
        mk<256, 8, false, 108>("w8 256x8x1", 1),
        mk<256, 16, false, 0>("s 256x16x1", 1),
        mk<256, 16, false, 104>("w4 256x16x1", 1), mk<256, 16, false, 108>("w8 256x16x1", 1),
        mk<256, 16, false, 116>("w16 256x16x1", 1),
        mk<512, 8, false, 0>("s 512x8x1", 1),
        mk<512, 8, false, 104>("w4 512x8x1", 1), mk<512, 8, false, 108>("w8 512x8x1", 1),
        mk<256, 2, false, 0>("s 256x2x3", 3), mk<256, 2, false, 102>("w2 256x2x3", 3),
        mk<256, 4, false, 104>("w4 256x4x2", 2), mk<256, 4, false, 102>("w2 256x4x2", 2),
    };
  } else if (set == "wavetail") {
    // static rounds + a dynamic per-wave tail (MODE 7): chunk = wave-tiles per granule, tail = % of tiles
    vars = {
        mk<256, 8, false, 0>("s 256x8x1", 1),
        mk<256, 8, false, 7>("wt 256x8x1 c4 t4", 1, 4, 4), mk<256, 8, false, 7>("wt 256x8x1 c4 t8", 1, 4, 8),
        mk<256, 8, false, 7>("wt 256x8x1 c8 t8", 1, 8, 8), mk<256, 8, false, 7>("wt 256x8x1 c2 t8", 1, 2, 8),
        mk<256, 8, false, 7>("wt 256x8x1 c4 t15", 1, 4, 15),
        mk<256, 2, false, 0>("s 256x2x3", 3),
        mk<256, 2, false, 7>("wt 256x2x3 c8 t8", 3, 8, 8), mk<256, 2, false, 7>("wt 256x2x3 c16 t8", 3, 16, 8),
        mk<256, 2, false, 7>("wt 256x2x3 c8 t15", 3, 8, 15),
        mk<512, 16, false, 0>("s 512x16x1", 1),
        mk<512, 16, false, 7>("wt 512x16x1 c2 t8", 1, 2, 8),
    };
  } else if (set == "steal") {
    vars = {
        mk<256, 2, false, 0>("s 256x2x3", 3),
        mk<256, 2, false, 4>("steal 256x2x3 g4 t8", 3, 4, 8),
        mk<256, 2, false, 4>("steal 256x2x3 g8 t8", 3, 8, 8),
        mk<256, 2, false, 4>("steal 256x2x3 g2 t5", 3, 2, 5),
        mk<256, 2, false, 4>("steal 256x2x3 g8 t15", 3, 8, 15),
        mk<512, 16, false, 0>("s 512x16x1", 1),
        mk<512, 16, false, 4>("steal 512x16x1 g1 t8", 1, 1, 8),
        mk<256, 4, false, 0>("s 256x4x2", 2),
        mk<256, 4, false, 4>("steal 256x4x2 g4 t8", 2, 4, 8),
    };
  } else if (set == "mlp") {
    vars = {
        mk<256, 2, false, 0>("s 256x2x3 compiler", 3),
        mk<512, 16, false, 0>("s 512x16x1 compiler", 1),
        mk<256, 2, false, 1>("s 256x2x3 forced", 3),
        mk<256, 4, false, 1>("s 256x4x3 forced", 3),
        mk<256, 8, false, 1>("s 256x8x2 forced", 2),
        mk<256, 16, false, 1>("s 256x16x1 forced", 1),
        mk<512, 4, false, 1>("s 512x4x2 forced", 2),
        mk<512, 8, false, 1>("s 512x8x1 forced", 1),
        mk<512, 16, false, 1>("s 512x16x1 forced", 1),
        mk<1024, 4, false, 1>("s 1024x4x1 forced", 1),
        mk<256, 4, false, 2>("s 256x4x2 pipe", 2),
        mk<256, 8, false, 2>("s 256x8x1 pipe", 1),
        mk<512, 4, false, 2>("s 512x4x1 pipe", 1),
        mk<512, 8, false, 2>("s 512x8x1 pipe", 1),
    };
  } else {
    vars = {
        mk<256, 2, false, 0>("s 256x2x3 compiler", 3),
        mk<512, 8, false, 1>("s 512x8x1 forced", 1),
        mk<512, 8, false, 3>("sc 512x8x1 run8", 1, 8),
        mk<256, 2, false, 3>("sc 256x2x3 run16", 3, 16),
        mk<256, 2, false, 3>("sc 256x2x3 run4", 3, 4),
        mk<512, 16, true, 1>("d 512x16x1 c1", 1, 1, 0),
        mk<512, 8, true, 1>("d 512x8x1 c2", 1, 2, 0),
        mk<512, 8, true, 1>("d 512x8x1 c8 t5", 1, 8, 5),
        mk<512, 16, true, 1>("d 512x16x1 c4 t10", 1, 4, 10),
        mk<256, 16, true, 1>("d 256x16x2 c1", 2, 1, 0),
    };
  }
  unsigned long long counter = 0;  // host mirror of the device counter
  auto launch = [&](const Variant& x, uint64_t* st) {
    const uint64_t tile = static_cast<uint64_t>(x.block) * x.unroll;
    const uint64_t ntiles = nvec / tile;
    uint64_t grid = std::min<uint64_t>(static_cast<uint64_t>(cus) * x.wpc, std::max<uint64_t>(ntiles, 1));
    TArgs a{v, nvec, partials, ctr, counter, 0, 0, 0, st, qctr};
    if (x.kern == body<256, 8, false, 7> || x.kern == body<256, 2, false, 7> || x.kern == body<512, 16, false, 7>) {
      // wave tail: whole static rounds for the first (100 - tailpct) % of tiles, the rest dynamic
      const uint64_t rounds = static_cast<uint64_t>(std::floor(ntiles * (1.0 - x.tailpct / 100.0))) / grid;
      a.nbig = rounds * grid;
      a.chunk = x.chunk;
      const uint64_t gsz = 64ull * x.unroll * x.chunk;
      const uint64_t v0 = a.nbig * tile;
      const uint64_t ng = nvec > v0 ? (nvec - v0 + gsz - 1) / gsz : 0;
      a.nchunks = (ng + 7) / 8;
    } else if (!x.dyn && x.tailpct > 0) {  // tail-steal: chunk = granule tiles, tail = tailpct % of tiles
      const uint64_t tail = static_cast<uint64_t>(std::ceil(ntiles * x.tailpct / 100.0));
      a.nbig = ntiles - std::min(tail, ntiles);
      a.chunk = x.chunk;
      const uint64_t granules = (ntiles - a.nbig + x.chunk - 1) / x.chunk;
      a.nchunks = (granules + 7) / 8;
    }
    if (!x.dyn && x.chunk && !a.nchunks) a.chunk = x.chunk;  // MODE 3: run length; MODE 5: rotation step; MODE 6: shift
    if (x.dyn) {
      const uint64_t tail = static_cast<uint64_t>(std::ceil(ntiles * x.tailpct / 100.0));
      a.chunk = x.chunk;
      a.nbig = (ntiles - std::min(tail, ntiles)) / x.chunk;
      a.nchunks = a.nbig + (ntiles - a.nbig * x.chunk);
      counter += a.nchunks + grid;  // every workgroup draws exactly one index past the end
    }
    hipLaunchKernelGGL(x.kern, dim3(static_cast<unsigned>(grid)), dim3(x.block), 0, 0, a);
    fold<<<1, 256>>>(partials, static_cast<int>(grid), out, qctr);
    return grid;
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> ms(vars.size());
  for (int r = 0; r < rounds; ++r) {
    std::vector<size_t> order(vars.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::srand(r + 1);
    for (size_t i = order.size(); i > 1; --i) std::swap(order[i - 1], order[std::rand() % i]);
    for (size_t i : order) {
      launch(vars[i], nullptr);
      CK(hipEventRecord(e0));
      for (int it = 0; it < iters; ++it) launch(vars[i], nullptr);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[i].push_back(t / iters);
      double got = 0;
      CK(hipMemcpy(&got, out, sizeof(double), hipMemcpyDeviceToHost));
      if (got != expect) {
        std::fprintf(stderr, "WRONG RESULT %s: %.17g vs %.17g\n", vars[i].name.c_str(), got, expect);
        return 3;
      }
    }
  }
  std::printf("n=%llu doubles (%.3f GB), %d CUs, %d rounds x %d launches (+ fold kernel each)\n",
              static_cast<unsigned long long>(n), n * 8e-9, cus, rounds, iters);
  std::printf("%-22s %9s %8s | stamped: %8s %8s %8s %8s %8s %8s %6s\n", "variant", "ms(med)", "TB/s", "start90", "end_min",
              "end_p50", "end_p99", "end_max", "busy%", "tiles");
  std::vector<uint64_t> h(8192 * 4);
  for (size_t i = 0; i < vars.size(); ++i) {
    const double m = median(ms[i]);
    // stamped run (own launch; its duration is not quoted)
    const uint64_t grid = launch(vars[i], stamps);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), stamps, grid * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    uint64_t s0 = UINT64_MAX;
    for (uint64_t g = 0; g < grid; ++g) s0 = std::min(s0, h[4 * g]);
    std::vector<double> starts, ends;
    double busy = 0, endmax = 0;
    uint64_t tmin = UINT64_MAX, tmax = 0;
    std::vector<double> xsum(16, 0.0), xcnt(16, 0.0);
    for (uint64_t g = 0; g < grid; ++g) {
      const double st = (h[4 * g] - s0) * 0.01, en = (h[4 * g + 1] - s0) * 0.01;  // us (100 MHz)
      starts.push_back(st);
      ends.push_back(en);
      busy += en - st;
      endmax = std::max(endmax, en);
      tmin = std::min(tmin, h[4 * g + 3]);
      tmax = std::max(tmax, h[4 * g + 3]);
      xsum[h[4 * g + 2] & 15] += en;
      xcnt[h[4 * g + 2] & 15] += 1;
    }
    std::sort(starts.begin(), starts.end());
    std::sort(ends.begin(), ends.end());
    const auto pct = [](const std::vector<double>& a, double p) { return a[static_cast<size_t>(p * (a.size() - 1))]; };
    std::printf("%-22s %9.4f %8.3f | %8.2f %8.2f %8.2f %8.2f %8.2f %8.1f %3llu-%llu\n", vars[i].name.c_str(), m,
                n * 8.0 / (m * 1e-3) / 1e12, pct(starts, 0.9), ends.front(), pct(ends, 0.5), pct(ends, 0.99), endmax,
                100.0 * busy / (grid * endmax), static_cast<unsigned long long>(tmin), static_cast<unsigned long long>(tmax));
    std::printf("%-22s   mean end by XCC (us):", "");
    for (int x = 0; x < 16; ++x)
      if (xcnt[x] > 0) std::printf(" %d:%.1f", x, xsum[x] / xcnt[x]);
    std::printf("\n");
  }
  return 0;
}
