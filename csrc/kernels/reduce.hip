// Streaming reduction, host side: tuned launch planner, dispatch table (filled by the
// reduce_tab_*.hip translation units), single-/two-pass launches, bound (prepared) launches and
// the two-pass finalize / element-wise combine kernels. The kernel templates and their design
// notes live in reduce_kernels.hpp.
#include "reduce_kernels.hpp"

namespace mireduce {

// ----------------------------------------------------------------------------------------------
// Host-side dispatch: a table keyed by (op, dtype, acc, block, unroll, policy) replaces the
// reference's runtime switch over 20 template instantiations per (op, T) (reduce_kernels.hpp).
// ----------------------------------------------------------------------------------------------
namespace {

using namespace detail;

int block_index(int b) { return b == 256 ? 0 : (b == 512 ? 1 : (b == 1024 ? 2 : -1)); }
// Table body slot of a plan: 0 hipcc's schedule, 1 / 2 explicit window 2 / 4.
int body_index(const LaunchPlan& p) { return p.window == 2 ? 1 : (p.window == 4 ? 2 : 0); }
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
const Table& table() {
  static const Table tb = [] {
    Table t{};
    fill_table_int32(t);
    fill_table_int64(t);
    fill_table_f32(t);
    fill_table_f64(t);
    fill_table_bf16(t);
    fill_table_f16(t);
    fill_table_sumsq(t);
    fill_table_absmax(t);
    return t;
  }();
  return tb;
}

// Tuned gfx950 defaults, measured on MI355X with tools/tune.py (interleaved rounds in one
// process; profiles/r1_tuning/). Median read bandwidth of the chosen point:
//   8 GB f64 sum / min  512 x 16, 1 WG/CU, nt   7.29 / 7.38 TB/s (round 1; round 2: 256 x 8 x 1, below)
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
  int block, unroll, wg_per_cu, policy, window;
};
Defaults tuned_defaults(size_t bytes, DType t, Op op) {
  constexpr size_t MB = 1ull << 20;
  // >= 3 GB, 8-byte types: one 256-thread workgroup per CU, 8 vectors in flight per lane. Round 1
  // picked 512 x 16 x 1 (f64 7.29 vs 7.23 for 256 x 8 x 1, profiles/r1_tuning/); on round 2's boxes
  // 512 x 16 x 1 ran 0.8-2.0 % behind 256 x 8 x 1, which was first or second on every box measured
  // for f64 SUM and int64 MAX (8 GB: 7.21 / 7.22 vs 7.07 / 7.17, profiles/r2_plan/, r2_tune/).
  // (Its compiled body issues 4 loads then interleaves waits and adds, ~9 in flight at 86 VGPRs;
  // forcing all 16 up front with a sched_barrier was slower still: 6.95 TB/s, r2_plan/run2.sh.)
  // (Rounds 1-2 ran 4-byte types >= 3 GB as 512 x 4 x 1 and other types above 192 MB as 256 x 2 x 3 /
  // 256 x 4 x 2 for 16-bit, all with hipcc's schedule: profiles/r1_session3/tune_types.txt.)
  // Round 3 (profiles/r3_window/, production kernel, same box, 7 interleaved rounds): 8-byte types
  // above 192 MB stream fastest as 256 threads x 8 vectors x 1 WG per CU with an explicit load
  // window of 4 (~18 loads in flight per CU): 8 GB 1092.1 vs 1112.4 us for hipcc's schedule of
  // the same plan, 1 GB 141.0 vs 144.5 us for 256x2x3. (hipcc's own schedule of a plan moves with
  // unrelated kernel code, profiles/r3_regress/; the explicit window does not.)
  // 4- and 2-byte types (profiles/r3_types/, tools/tune.py, 5 interleaved rounds per sweep, 1 / 2 /
  // 8 GB): the window-4 plan is first for f32 SUM at all three sizes (8 GB 7.26 vs 7.23 TB/s for the
  // old 512x4x1; 1 GB 7.14 vs 7.09 for 256x2x3), for int32 MAX and bf16 SUM (8 GB 7.38 vs 7.21 for
  // 256x4x2) and within 0.2 % of first for f32 MAX. Two exceptions: int32 SUM/SUMSQ, whose int64
  // accumulation doubles the VALU work per load, collapses with it (6.06-6.22 TB/s) and streams
  // best as 256x8x2 with a window of 2 (7.15-7.27, first at every size); 16-bit MIN/MAX run the
  // window-4 plan at 7.13 and 256x8x2 window 2 at 7.25 (8 GB f16 MAX; the old 256x4x2: 7.16).
  // (Rechecked in round 6 on two boxes, profiles/r6_plan/: no consistent int32 SUM winner, and the
  // 256x8x2 window-2 plan first for all four 16-bit MIN / MAX pairs at 1-4 GB.)
  const bool widening_int = t == DType::Int32 && (op == Op::Sum || op == Op::SumSq);
  const bool half_cmp = dtype_is_half(t) && op != Op::Sum && op != Op::SumSq;
  if (dtype_size(t) == 8 && bytes > 192 * MB) return {256, 8, 1, 1, 4};
  if ((widening_int || half_cmp) && bytes > 192 * MB) return {256, 8, 2, 1, 2};
  if (dtype_size(t) <= 4 && bytes > 192 * MB) return {256, 8, 1, 1, 4};
  // <= 192 MB: 256x4x3 with hipcc's schedule. (256x8x2 window 2 led tune.py's back-to-back launches
  // at 64-192 MiB by 0.5-4 %, but not the reduction app's per-iteration timing at the reference's
  // 2^24 doubles, warm or cold: profiles/r3_types/small/.)
  return {256, 4, 3, 1, 0};
}
// (Round 6 removed the measured-null plan options: the software-pipelined body, the ticketed
// flat / tree fan-ins, the balanced leftover and the contiguous split — docs/TUNING.md keeps their
// measurements: profiles/r1_bench/fanin_ab.txt, r2_small/balance_ab.txt, r1_session4/split_ab/.)

// XCD-weighted split default (permille of the rounds per workgroup given extra to the workgroups
// on odd XCCs; see plan_reduce, weighted_tiles and XcdAnchor). Measured per plan with the anchored
// split (profiles/r4_skew/, 8 GB, 0 / 10 / 20 / 30): 20 is the best for every window-4 plan of 8-
// and 4-byte elements (f64 MAX 1096.5 -> 1090.1 us, int64 MIN 1108.1 -> 1101.4, fp32 SUM 1107.8 ->
// 1101.1, int32 MAX 1095.9 -> 1090.4; f64 SUM 1092.6 -> 1087.5, profiles/r4_ab/), 0 for bf16 (1089.5
// at 0, 1105+ with any) and the window-2 int32 SUM plan (1102.5 at 0, 1105.7+). bench.py re-measures
// 0 / default / 2x on the node for the headline's shards.
// The measured asymmetry is between the XCDs of a whole MI355X in SPX mode (8 XCDs, 256 CUs, workgroups
// dealt round-robin): a partition with one XCD (CPX, 32 CUs) has no parity to balance, and one of 2-4
// XCDs (DPX / QPX) was never measured, so the default skew is 0 there (an explicit skew still applies).
constexpr int kSpxCus = 256;
// The tuned default's extra rounds for the favoured XCD parity (arrays of >= kSkewOffsetMinRounds
// rounds per workgroup): kSkewOffsetRounds + kSkewSharePermille of the rounds.
constexpr uint64_t kSkewOffsetMinRounds = 64;
constexpr int64_t kSkewOffsetRounds = 2;
constexpr int64_t kSkewSharePermille = 18;

int tuned_xcd_skew(DType t, const LaunchPlan& p, int num_cus) {
  const size_t es = dtype_size(t);
  if (num_cus < kSpxCus) return 0;
  return (es == 8 || es == 4) && p.window == 4 ? 20 : 0;
}

// `fan` non-null: the second level of a two-pass reduce_stream launch, which ends its fan-in epoch
// (kern::finalize).
struct FanEnd {
  unsigned* fan = nullptr;
  uint64_t* slots = nullptr;
  unsigned fan_slots = 0;
};

template <class OpT, class AccT>
void launch_finalize(const void* partials, uint64_t count, void* out, hipStream_t s, const FanEnd& f) {
  hipLaunchKernelGGL((kern::finalize<OpT, AccT>), dim3(1), dim3(256), 0, s,
                     static_cast<const AccT*>(partials), count, static_cast<AccT*>(out), f.fan, f.slots,
                     f.fan_slots);
}

template <class OpT>
void finalize_by_acc(DType acc, const void* partials, uint64_t count, void* out, hipStream_t s,
                     const FanEnd& f = FanEnd{}) {
  switch (acc) {
    case DType::Int32: launch_finalize<OpT, int32_t>(partials, count, out, s, f); break;
    case DType::Int64: launch_finalize<OpT, int64_t>(partials, count, out, s, f); break;
    case DType::Float32: launch_finalize<OpT, float>(partials, count, out, s, f); break;
    case DType::Float64: launch_finalize<OpT, double>(partials, count, out, s, f); break;
    default: MIREDUCE_REQUIRE(false, "finalize: accumulator must be int32, int64, float32 or float64");
  }
}

void fold_partials(const void* partials, uint64_t count, DType acc, Op op, void* out, hipStream_t stream,
                   const FanEnd& f) {
  switch (op) {  // partials are already transformed: SUMSQ folds like SUM, AMAX like MAX
    case Op::Sum:
    case Op::SumSq: finalize_by_acc<SumOp>(acc, partials, count, out, stream, f); break;
    case Op::Min: finalize_by_acc<MinOp>(acc, partials, count, out, stream, f); break;
    case Op::Max:
    case Op::AbsMax: finalize_by_acc<MaxOp>(acc, partials, count, out, stream, f); break;
  }
  MIREDUCE_HIP_THROW(hipGetLastError());
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

Workspace::Workspace(int device, int max_grid, SlotMemory slot_memory) : max_grid_(max_grid) {
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
  // polled fan-in slots: uncached, so the finisher's polls see every XCD's stores. SlotMemory::Coarse
  // (experiments only, tools/launch_floor.hip): ordinary device memory instead, relying on the
  // agent-scope atomics alone for cross-XCD visibility.
  const unsigned flags = slot_memory == SlotMemory::Coarse ? hipDeviceMallocDefault : hipDeviceMallocUncached;
  MIREDUCE_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&slots_), static_cast<size_t>(max_grid) * 16,
                                           flags));
  MIREDUCE_HIP_THROW(hipMemset(slots_, 0, static_cast<size_t>(max_grid) * 16));
  MIREDUCE_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&fan_), 256, flags));
  MIREDUCE_HIP_THROW(hipMemset(fan_, 0, 256));
  MIREDUCE_HIP_THROW(hipDeviceSynchronize());
  MIREDUCE_HIP_THROW(hipSetDevice(prev));
}

Workspace::~Workspace() {
  (void)hipFree(partials_);
  (void)hipFree(slots_);
  (void)hipFree(fan_);
}

unsigned Workspace::error() const {
  unsigned v = 0;
  int prev = 0;
  MIREDUCE_HIP_THROW(hipGetDevice(&prev));
  MIREDUCE_HIP_THROW(hipSetDevice(device_));
  const hipError_t e = hipMemcpy(&v, fan_ + 1, sizeof v, hipMemcpyDeviceToHost);
  (void)hipSetDevice(prev);
  MIREDUCE_HIP_THROW(e);
  return v;
}

void Workspace::reset(hipStream_t stream) {
  MIREDUCE_HIP_THROW(hipMemsetAsync(slots_, 0, static_cast<size_t>(max_grid_) * 16, stream));
  // the epoch may stay: every slot is 0 now, and epochs start at 1
  MIREDUCE_HIP_THROW(hipMemsetAsync(fan_ + 1, 0, sizeof(unsigned), stream));
}

LaunchPlan plan_reduce(const void* in, size_t n, DType t, const ReduceConfig& cfg, int num_cus,
                       int max_grid, Op op) {
  LaunchPlan p;
  const size_t es = dtype_size(t);
  const Defaults d = tuned_defaults(n * es, t, op);
  p.block = cfg.block ? cfg.block : d.block;
  p.unroll = cfg.unroll ? cfg.unroll : d.unroll;
  p.nontemporal = cfg.policy < 0 ? d.policy == 1 : cfg.policy == 1;
  p.single_pass = cfg.single_pass;
  MIREDUCE_REQUIRE(cfg.xrank == nullptr || cfg.single_pass,
                   "the fused cross-rank finish needs the single-pass kernel");
  MIREDUCE_REQUIRE(block_index(p.block) >= 0, "block must be 256, 512 or 1024");
  MIREDUCE_REQUIRE(unroll_index(p.unroll) >= 0, "unroll must be 2, 4, 8 or 16");
  MIREDUCE_REQUIRE(cfg.window == -1 || cfg.window == 0 || cfg.window == 2 || cfg.window == 4,
                   "window must be 0, 2 or 4");
  {  // an explicit window where one is instantiated (non-temporal), else hipcc's schedule
    const int w = cfg.window < 0 ? d.window : cfg.window;
    const bool explicit_plan = cfg.block || cfg.unroll;  // a window tuned for the default plan only
    const int wd = cfg.window < 0 && explicit_plan ? 0 : w;
    p.window = (wd > 0 && p.nontemporal && window_ok(p.block, p.unroll, wd)) ? wd : 0;
  }
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
  // XCD-weighted split (window bodies, interleaved, even grids): permille of the rounds per
  // workgroup -> extra rounds for one parity. MIREDUCE_XCD_SKEW=<permille> overrides the tuned
  // default (A/B runs).
  // Launches with a fan-in epoch only (the polled fan-in, or two-pass: its finalize ends the epoch):
  // the kernel anchors the favoured parity to the XCDs with it.
  if (p.window > 0 && p.grid % 2 == 0 && p.grid > 1) {
    // (the env override replaces the tuned default only: a caller's explicit skew — e.g. bench.py's
    // plan-tuning candidates — is what it says)
    bool tuned = cfg.xcd_skew == (-2147483647 - 1);
    int permille = tuned ? tuned_xcd_skew(t, p, num_cus) : cfg.xcd_skew;
    if (const char* e = std::getenv("MIREDUCE_XCD_SKEW"); e && tuned) {
      permille = std::atoi(e);
      tuned = false;
    }
    const uint64_t tile = static_cast<uint64_t>(p.block) * static_cast<uint64_t>(p.unroll);
    const uint64_t rounds = tile ? p.nvec / tile / static_cast<uint64_t>(p.grid) : 0;
    int64_t d = (static_cast<int64_t>(rounds) * permille + (permille >= 0 ? 500 : -500)) / 1000;
    if (tuned && permille > 0 && rounds >= kSkewOffsetMinRounds)
      // The tuned default is a fixed offset plus a share of the rounds, not a flat share: the
      // optimum measured 4-5 extra rounds at the 1 GB N=8 shard (119 rounds: 20 permille gives 2,
      // 0.3-0.6 % slower), ~6 at 2 GB and 19 at 8 GB (profiles/r5_skew/).
      d = (static_cast<int64_t>(rounds) * kSkewSharePermille + 500) / 1000 + kSkewOffsetRounds;
    // the common rounds must stay >= 1 (the kernel resolves the anchor at their end)
    const uint64_t ad = static_cast<uint64_t>(d < 0 ? -d : d), ntiles = tile ? p.nvec / tile : 0;
    const uint64_t g = static_cast<uint64_t>(p.grid);
    p.xskew = ad * (g / 2) + g <= ntiles ? static_cast<int>(d) : 0;
  }
  return p;
}

static kern::Args make_args(const void* in, const LaunchPlan& p, DType t, const ReduceConfig& cfg) {
  kern::Args a{};
  a.fan_bound = cfg.fanin_bound_ticks ? cfg.fanin_bound_ticks : kern::kFanBoundTicks;
  a.delay_wg = cfg.debug_delay_wg;
  a.delay_ticks = cfg.debug_delay_ticks;
  a.anchor_delay = cfg.debug_delay_anchor_ticks;
  a.wg_stamps = cfg.debug_wg_stamps;
  a.head_ptr = in;
  a.body = static_cast<const char*>(in) + p.head * dtype_size(t);
  a.head = p.head;
  a.nvec = p.nvec;
  a.tail = p.tail;
  a.xskew = p.xskew;
  {  // the weighted split's common / extra rounds (weighted_tiles), precomputed here
    const uint64_t tile = static_cast<uint64_t>(p.block) * static_cast<uint64_t>(p.unroll);
    const uint64_t ntiles = tile ? p.nvec / tile : 0, grid = static_cast<uint64_t>(p.grid > 0 ? p.grid : 1);
    const uint64_t half = grid / 2, d = static_cast<uint64_t>(p.xskew < 0 ? -static_cast<int64_t>(p.xskew) : p.xskew);
    if (p.xskew == 0 || half == 0) {
      a.xskew = 0;
      a.x_ra = ntiles / grid;
      a.x_dd = 0;
    } else {  // plan_reduce keeps d * half + grid <= ntiles: >= 1 common round
      a.x_ra = (ntiles - d * half) / grid;
      a.x_dd = d;
    }
  }
  return a;
}

// The two-pass launch's finalize ends the first level's fan-in epoch (grid > 1: a one-workgroup
// first level reads no epoch).
static FanEnd fan_end(const kern::Args& a, const Workspace& ws) {
  FanEnd f;
  if (a.two_pass_epoch) {
    f.fan = a.fan;
    f.slots = ws.slots();
    f.fan_slots = a.fan_slots;
  }
  return f;
}

// Segmented launches (ReduceConfig::segment_bytes): how many consecutive segments of how many
// elements; {1, 0} = one launch. Polled single-pass launches only (the last segment's finisher folds
// the earlier segments' results, one per lane of its first wave: at most `max_carry` of them).
struct Segments {
  int count = 1;
  uint64_t elems = 0;
};
static Segments plan_segments(size_t n, size_t es, const ReduceConfig& cfg, const LaunchPlan& whole, int max_carry) {
  Segments sg;
  if (!whole.single_pass || cfg.segment_bytes < 0 || n == 0) return sg;
  const uint64_t bytes = static_cast<uint64_t>(n) * es;
  if (cfg.segment_bytes == 0 && bytes <= 2 * static_cast<uint64_t>(kSegmentBytes)) return sg;
  constexpr uint64_t kMiB = 1ull << 20;
  const uint64_t want = cfg.segment_bytes > 0 ? static_cast<uint64_t>(cfg.segment_bytes) : kSegmentBytes;
  const uint64_t quantum = kMiB / es;  // segments start on 1 MiB boundaries of the array
  uint64_t elems = std::max<uint64_t>(1, want / kMiB) * quantum;
  uint64_t count = (n + elems - 1) / elems;
  if (count > static_cast<uint64_t>(max_carry) + 1) count = static_cast<uint64_t>(max_carry) + 1;  // larger ones
  if (count <= 1) return sg;
  // equal segments (whole MiB each, the last one the rest): no short tail segment, so the last launch
  // — whose finisher folds the carried results — always has a multi-workgroup polled plan
  elems = ((n + count - 1) / count + quantum - 1) / quantum * quantum;
  count = (n + elems - 1) / elems;
  if (count <= 1) return sg;
  sg.count = static_cast<int>(count);
  sg.elems = elems;
  return sg;
}

namespace {

// One launch of the streaming kernel over [in, in + n): its plan, arguments and table entry.
struct Launch {
  LaunchPlan plan;
  kern::Args args;
  LaunchFn fn = nullptr;
};

Launch make_launch(const void* in, size_t n, DType t, Op op, int c, void* out, Workspace& ws, const ReduceConfig& cfg,
                   const void* xrank, const void* carry, unsigned ncarry) {
  Launch L;
  L.plan = plan_reduce(in, n, t, cfg, ws.num_cus(), ws.max_grid(), op);
  const LaunchPlan& p = L.plan;
  kern::Args a = make_args(in, p, t, cfg);
  a.partials = ws.partials();
  a.out = out;
  a.two_pass = p.single_pass ? 0 : 1;
  a.slots = p.single_pass ? ws.slots() : nullptr;
  a.fan = ws.fan();
  a.fan_slots = static_cast<unsigned>(ws.max_grid());
  a.two_pass_epoch = p.single_pass ? 0 : 1;
  a.xrank = static_cast<const XrankDesc*>(xrank);
  a.carry = carry;
  a.ncarry = ncarry;
  L.args = a;
  L.fn = table().fn[c][block_index(p.block)][unroll_index(p.unroll)][p.nontemporal ? 1 : 0][body_index(p)];
  return L;
}

// Every launch of a reduction: one, or (segmented) one per segment — the earlier segments write
// their results into the workspace's partials (unused by the polled fan-in), the last one carries
// them in, writes `out` and does the fused cross-rank finish. The returned plans' first entry
// describes the first launch, with `segments` / `segment_elems` set.
std::vector<Launch> make_launches(const void* in, size_t n, DType t, Op op, DType acc, void* out, Workspace& ws,
                                  const ReduceConfig& cfg) {
  const int c = combo_index(op, t, acc);
  MIREDUCE_REQUIRE(c >= 0, "unsupported (dtype, op, accumulator) combination");
  MIREDUCE_REQUIRE(out != nullptr, "output pointer is null");
  std::vector<Launch> v;
  v.push_back(make_launch(in, n, t, op, c, out, ws, cfg, cfg.xrank, nullptr, 0));
  const size_t es = dtype_size(t);
  const Segments sg = plan_segments(n, es, cfg, v[0].plan, std::min(256, ws.max_grid()));
  if (sg.count == 1) return v;
  v.clear();
  const size_t as = dtype_size(acc);
  char* carry = static_cast<char*>(ws.partials());
  for (int k = 0; k < sg.count; ++k) {
    const uint64_t off = static_cast<uint64_t>(k) * sg.elems;
    const uint64_t nk = std::min<uint64_t>(sg.elems, n - off);
    const void* ink = static_cast<const char*>(in) + off * es;
    const bool last = k == sg.count - 1;
    v.push_back(make_launch(ink, nk, t, op, c, last ? out : carry + k * as, ws, cfg, last ? cfg.xrank : nullptr,
                            last ? carry : nullptr, last ? static_cast<unsigned>(sg.count - 1) : 0u));
  }
  // the carried results are folded by the last launch's polled finisher only
  MIREDUCE_REQUIRE(v.back().plan.single_pass && v.back().plan.grid > 1, "segmented reduction: the last segment's "
                   "plan has no polled multi-workgroup fan-in (segment too small)");
  v[0].plan.segments = sg.count;
  v[0].plan.segment_elems = sg.elems;
  return v;
}

void run_launches(const std::vector<Launch>& v, void* out, Op op, DType acc, const Workspace& ws,
                  hipStream_t stream) {
  for (size_t k = 0; k < v.size(); ++k) {
    kern::Args a = v[k].args;
    if (out && k + 1 == v.size()) a.out = out;
    v[k].fn(a, v[k].plan.grid, stream);
    MIREDUCE_HIP_THROW(hipGetLastError());
    if (!v[k].plan.single_pass) fold_partials(a.partials, v[k].plan.grid, acc, op, a.out, stream, fan_end(a, ws));
  }
}

}  // namespace

void plan_segmentation(size_t n, DType t, const ReduceConfig& cfg, LaunchPlan& whole, int max_carry) {
  const Segments sg = plan_segments(n, dtype_size(t), cfg, whole, max_carry);
  whole.segments = sg.count;
  whole.segment_elems = sg.elems;
}

LaunchPlan reduce(const void* in, size_t n, DType t, Op op, DType acc, void* out, Workspace& ws,
                  hipStream_t stream, const ReduceConfig& cfg) {
  const std::vector<Launch> v = make_launches(in, n, t, op, acc, out, ws, cfg);
  run_launches(v, nullptr, op, acc, ws, stream);
  return v[0].plan;
}

unsigned reduce_checked(const void* in, size_t n, DType t, Op op, DType acc, void* out, Workspace& ws,
                        hipStream_t stream, const ReduceConfig& cfg, LaunchPlan* plan) {
  const LaunchPlan p = reduce(in, n, t, op, acc, out, ws, stream, cfg);
  if (plan) *plan = p;
  MIREDUCE_HIP_THROW(hipStreamSynchronize(stream));
  unsigned err = ws.error();
  if (cfg.xrank) {  // the fused finish's own error word (a peer's partial late or poisoned)
    unsigned xe = 0;
    const auto* d = static_cast<const XrankDesc*>(cfg.xrank);
    unsigned* word = nullptr;
    MIREDUCE_HIP_THROW(hipMemcpy(&word, &d->error, sizeof word, hipMemcpyDeviceToHost));
    MIREDUCE_HIP_THROW(hipMemcpy(&xe, word, sizeof xe, hipMemcpyDeviceToHost));
    err |= xe << 8;
  }
  return err;
}

struct BoundReduce::Impl {
  std::vector<Launch> launches;  // one, or one per segment (make_launches)
  Op op;
  DType acc;
  const Workspace* ws;
};

BoundReduce::BoundReduce(const void* in, size_t n, DType t, Op op, DType acc, void* out, Workspace& ws,
                         const ReduceConfig& cfg)
    : impl_(new Impl{make_launches(in, n, t, op, acc, out, ws, cfg), op, acc, &ws}) {}

BoundReduce::~BoundReduce() { delete impl_; }

void BoundReduce::launch(hipStream_t stream, void* out) const {
  run_launches(impl_->launches, out, impl_->op, impl_->acc, *impl_->ws, stream);
}

const LaunchPlan& BoundReduce::plan() const { return impl_->launches[0].plan; }

unsigned BoundReduce::error() const { return impl_->ws->error(); }

LaunchPlan reduce_partials(const void* in, size_t n, DType t, Op op, DType acc, void* partials,
                           int max_grid, int num_cus, hipStream_t stream, const ReduceConfig& cfg) {
  const int c = combo_index(op, t, acc);
  MIREDUCE_REQUIRE(c >= 0, "unsupported (dtype, op, accumulator) combination");
  ReduceConfig c2 = cfg;
  c2.single_pass = false;
  c2.xrank = nullptr;
  LaunchPlan p = plan_reduce(in, n, t, c2, num_cus, max_grid, op);
  p.xskew = 0;  // no workspace, so no fan-in epoch to anchor the XCD-weighted split with: equal rounds
  kern::Args a = make_args(in, p, t, c2);
  a.partials = partials;
  a.two_pass = 1;
  const LaunchFn fn = table().fn[c][block_index(p.block)][unroll_index(p.unroll)][p.nontemporal ? 1 : 0][body_index(p)];
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
  fold_partials(partials, count, acc, op, out, stream, FanEnd{});
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
      for (int nt = 0; nt < 2; ++nt) {
        v.push_back("block=" + std::to_string(b) + " unroll=" + std::to_string(u) +
                    (nt ? " policy=nt" : " policy=default"));
        for (int w : {2, 4})
          if (nt && window_ok(b, u, w))
            v.push_back("block=" + std::to_string(b) + " unroll=" + std::to_string(u) + " policy=nt window=" +
                        std::to_string(w));
      }
  return v;
}

}  // namespace mireduce
