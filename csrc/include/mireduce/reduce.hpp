// Public C++ API of the single-GPU reduction library.
//
// Reference parity: replaces `template<class T> void {sum,min,max}reduce(int size, int threads,
// int blocks, int whichKernel, T* d_idata, T* d_odata)` (cuda/C/src/reduction/reduction.h:15-25)
// and the launch-geometry planner getNumBlocksAndThreads (reduction.cpp:272-291).
// Differences by design: 64-bit sizes (bug B4), an explicit accumulator dtype, a
// one-launch finalisation (reference: second in-place launch, reduction.cpp:344-357), and a
// persistent grid sized for 256 CUs instead of the fixed 64 blocks (reduction.cpp:668).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "mireduce/rng.hpp"
#include "mireduce/types.hpp"

namespace mireduce {

// Tunables of the streaming kernel. 0 (or -1 for `policy`) means "use the tuned gfx950 default",
// which depends on the array size (docs/TUNING.md, profiles/r1_tuning/).
struct ReduceConfig {
  int block = 0;          // threads per workgroup: 256 | 512 | 1024
  int unroll = 0;         // independent 16-byte loads in flight per thread: 2 | 4 | 8 | 16
  int wg_per_cu = 0;      // persistent-grid occupancy target
  int max_blocks = 0;     // hard cap on the grid (reference --maxblocks)
  int policy = -1;        // streaming-load cache policy: -1 auto, 0 default, 1 non-temporal (nt)
  // Streaming body's load schedule: -1 auto (tuned), 0 hipcc's own, 2 or 4 = an explicit window of
  // that many 16-byte loads per thread, the next one issued before the oldest is consumed
  // (non-temporal policy, 256/512 threads, unroll 2..8 divisible by it; otherwise hipcc's).
  // profiles/r3_window/.
  int window = -1;
  // XCD-weighted split of the interleaved window body, in permille of the rounds per workgroup:
  // > 0 gives the workgroups on odd XCCs that many more rounds, < 0 those on even ones; 0 equal
  // rounds; INT_MIN = tuned default. Launches with a fan-in epoch only (polled single-pass or
  // two-pass): the kernel anchors the parity on the device. (profiles/r4_xcd/, r4_ab/, r4_skew/)
  int xcd_skew = -2147483647 - 1;
  bool single_pass = true;   // last-arriver finalisation vs a second finalize launch
  // Segmented launches (polled single-pass only): an array of more than 2 x kSegmentBytes bytes is
  // reduced as a sequence of launches over consecutive segments of about this many bytes on the
  // same stream, each segment's result carried into the last launch, which folds them with its own
  // (and does the fused cross-rank finish). One launch over ~292 GB streamed 2.4 % slower than the
  // same bytes as 8 GB launches (profiles/r5_hbmfill/): 0 = auto (kSegmentBytes above
  // 2 x kSegmentBytes), < 0 = one launch, > 0 = this segment size (bytes, rounded to 1 MiB).
  int64_t segment_bytes = 0;
  // Fused cross-rank finish: XrankChannel::device_desc() (xrank.hpp). The launch then writes the
  // fold over every rank's partial into out (single-pass only).
  const void* xrank = nullptr;
  // Polled fan-in wait bound in wall-clock ticks (0: ~10.7 s). Reaching it sets the workspace's
  // sticky error and poisons the result (Workspace::error()).
  uint64_t fanin_bound_ticks = 0;
  // Test hook (failure-path tests only): workgroup `debug_delay_wg` sleeps `debug_delay_ticks`
  // wall-clock ticks before publishing its partial (-1: none).
  int debug_delay_wg = -1;
  uint64_t debug_delay_ticks = 0;
  // Test hook: workgroup 0 of an XCD-weighted launch sleeps this many wall-clock ticks before it
  // publishes the XCD anchor (0: none); past fanin_bound_ticks every other workgroup gives up on
  // it, the launch is poisoned and Workspace::error() has value 2 (bit 1) set.
  uint64_t debug_delay_anchor_ticks = 0;
  // Diagnostic hook (tools/xcd_balance.py): workgroup b writes [3b] the wall clock after its last
  // streamed tile was consumed, [3b+1] its XCC id, [3b+2] its tile count (device pointer; null: off).
  uint64_t* debug_wg_stamps = nullptr;
};

// What the planner chose (printed by the apps, recorded in JSON sidecars).
struct LaunchPlan {
  int block = 0;
  int unroll = 0;
  int grid = 0;
  bool nontemporal = true;
  int window = 0;      // explicit load window per thread (0: hipcc's schedule)
  bool single_pass = true;  // polled single-pass fan-in vs a second finalize launch (two-pass)
  int xskew = 0;            // window body: extra rounds for odd (> 0) / even (< 0) workgroups
  uint64_t head = 0;   // scalar elements before the first 16-B aligned vector
  uint64_t nvec = 0;   // 16-byte vectors in the streaming body
  uint64_t tail = 0;   // scalar elements after the body
  // Segmented launches (ReduceConfig::segment_bytes): the fields above describe the first segment.
  int segments = 1;
  uint64_t segment_elems = 0;  // elements per segment (the last one holds the rest); 0 = not segmented
};

// Auto segment size of ReduceConfig::segment_bytes (8 GiB).
constexpr int64_t kSegmentBytes = int64_t{8} << 30;

// Fill `whole.segments` / `segment_elems` for a reduction of n elements planned as `whole`
// (plan_reduce over the whole array): the segmentation reduce() / BoundReduce would use with a
// workspace allowing `max_carry` carried results (min(256, max_grid)).
void plan_segmentation(size_t n, DType t, const ReduceConfig& cfg, LaunchPlan& whole, int max_carry = 256);

// Device scratch for one reduction stream: per-workgroup partials (two-pass mode, segmented
// launches' carried results), the polled fan-in's epoch-tagged slots and its state words (epoch,
// sticky error, XCD anchor) in uncached memory. One Workspace must not be used by two concurrently
// running reductions. `slot_memory` is for experiments only (tools/launch_floor.hip): the fan-in
// words in ordinary (coarse-grained) device memory instead of uncached.
enum class SlotMemory { Uncached, Coarse };
class Workspace {
 public:
  explicit Workspace(int device = -1, int max_grid = 16384, SlotMemory slot_memory = SlotMemory::Uncached);
  ~Workspace();
  Workspace(const Workspace&) = delete;
  Workspace& operator=(const Workspace&) = delete;

  int device() const { return device_; }
  int num_cus() const { return num_cus_; }
  int max_grid() const { return max_grid_; }
  void* partials() const { return partials_; }
  uint64_t* slots() const { return slots_; }
  unsigned* fan() const { return fan_; }
  // Sticky error word of the launches on this workspace (synchronous read: call after they
  // completed). Bit 0: some launch's polled fan-in finisher reached its wait bound. Bit 1: the
  // XCD anchor of a weighted split (XcdAnchor) was late: some workgroup waited past the bound
  // for workgroup 0's publish, so its tiles were not the split's (it then withholds its partial,
  // and in two-pass mode the finalize poisons the result). Non-zero: that launch and every later
  // one wrote a poisoned result (NaN, or the operator's identity for integers — for which this
  // word, not the value, is the signal) until reset(). (Value 2 (bit 1): a late XCD anchor.)
  unsigned error() const;
  // Re-zero the fan-in slots and the sticky error (after an error or an aborted launch;
  // stream-ordered: no launch on this workspace may be running on another stream).
  void reset(hipStream_t stream);

 private:
  int device_ = 0;
  int num_cus_ = 256;
  int max_grid_ = 0;
  void* partials_ = nullptr;
  uint64_t* slots_ = nullptr;  // polled fan-in: [max_grid][2] tagged words, uncached
  unsigned* fan_ = nullptr;    // polled fan-in: [0] epoch, [1] sticky error, uncached
};

// The tuned plan depends on the element type, the size and (for 4- and 2-byte types) the operator:
// see tuned_defaults in reduce.hip.
LaunchPlan plan_reduce(const void* in, size_t n, DType t, const ReduceConfig& cfg, int num_cus,
                       int max_grid, Op op = Op::Sum);

// Enqueue a full reduction of n elements at device pointer `in` into out[0] (device pointer,
// element type `acc`). Asynchronous on `stream`; safe to capture into a hipGraph.
// Throws mireduce::Error on invalid arguments.
// Error state: a launch whose fan-in (or fused cross-rank finish) failed writes a poisoned value —
// NaN for floating accumulators, the operator's IDENTITY for integers (no in-range integer can
// signal an error, and the identity stays neutral in a later cross-rank fold) — and sets a sticky
// error word. The value therefore does not tell an integer caller anything: read the word
// (Workspace::error() after the stream completed, XrankChannel::error() for the fused finish), or
// use reduce_checked() below.
LaunchPlan reduce(const void* in, size_t n, DType t, Op op, DType acc, void* out, Workspace& ws,
                  hipStream_t stream, const ReduceConfig& cfg = {});

// Synchronous form: reduce(), wait for `stream`, and return the error state of this and every
// earlier launch on `ws` since its last reset(): 0 = out[0] is valid; bit 0 = the polled fan-in
// reached its wait bound; bit 1 = an XCD anchor was late (Workspace::error()); bits 8.. = the
// fused finish's channel error (<< 8: 1 a peer's partial
// timed out, 2 a peer pushed a poisoned partial). Non-zero: out[0] is poisoned; reset() the
// workspace (and XrankChannel::clear_error()) before relying on later launches.
unsigned reduce_checked(const void* in, size_t n, DType t, Op op, DType acc, void* out, Workspace& ws,
                        hipStream_t stream, const ReduceConfig& cfg = {}, LaunchPlan* plan = nullptr);

// A reduction whose plan, kernel variant and arguments are resolved once. launch() is a single
// kernel launch (plus the finalize launch in two-pass mode) with no planning or argument
// marshalling: the per-step path of bench loops and hipGraph capture. The buffers and the
// workspace must outlive the object; same concurrency rule as Workspace.
class BoundReduce {
 public:
  BoundReduce(const void* in, size_t n, DType t, Op op, DType acc, void* out, Workspace& ws,
              const ReduceConfig& cfg = {});
  ~BoundReduce();
  BoundReduce(const BoundReduce&) = delete;
  BoundReduce& operator=(const BoundReduce&) = delete;
  // `out` (optional) redirects the result to another accumulator slot for this launch.
  void launch(hipStream_t stream, void* out = nullptr) const;
  const LaunchPlan& plan() const;
  // The bound workspace's sticky fan-in error (Workspace::error()).
  unsigned error() const;

 private:
  struct Impl;
  Impl* impl_;
};

// First level only: writes plan.grid partials (element type `acc`) to `partials`.
LaunchPlan reduce_partials(const void* in, size_t n, DType t, Op op, DType acc, void* partials,
                           int max_grid, int num_cus, hipStream_t stream,
                           const ReduceConfig& cfg = {});

// The reference's timed multi-pass reduction (benchmarkReduce*, reduction.cpp:319-374) on the
// streaming kernel: first level into partials, then the same first-level kernel relaunched on
// the partials (ping-pong, never in place) while more than `cpu_thresh` remain; `cpu_final`:
// first level only (--cpufinal, reduction.cpp:328-340). The `left` partials (acc type; 1 = the
// result) are at `partials`, inside `scratch` (>= 2 * max_grid * 8 bytes), for a host fold.
struct ReducePasses {
  LaunchPlan plan;          // first level
  int passes = 0;           // kernel launches
  uint64_t left = 0;
  const void* partials = nullptr;
};
ReducePasses reduce_passes(const void* in, size_t n, DType t, Op op, DType acc, void* scratch, int max_grid,
                           int num_cus, uint64_t cpu_thresh, bool cpu_final, hipStream_t stream,
                           const ReduceConfig& cfg = {});

// Fold `count` partials on the device with one workgroup.
void reduce_finalize(const void* partials, size_t count, DType acc, Op op, void* out,
                     hipStream_t stream);

// Element-wise combine: inout[i] = op(inout[i], other[i]) for n elements (vector mode).
void combine_elementwise(void* inout, const void* other, size_t n, DType t, Op op,
                         hipStream_t stream);

// Fill n elements with a synthetic pattern (bit-identical with fill_host).
void fill_device(void* ptr, size_t n, DType t, const FillSpec& spec, hipStream_t stream);
void fill_host(void* ptr, size_t n, DType t, const FillSpec& spec);

// Human-readable list of compiled kernel variants ("block x unroll x policy").
std::vector<std::string> compiled_variants();

}  // namespace mireduce
