// Fused cross-rank finalisation of a scalar reduction over xGMI (no RCCL launch).
//
// A global reduction of a sharded array is "local reduce, then a 1-element all-reduce"
// (SURVEY.md §5.8 mode scalar; the vendored simpleMPI does MPI_Reduce of one float after a local
// reduce, cuda/C/src/simpleMPI/simpleMPI.cpp:92-98). With RCCL that second step is a separate
// kernel on a separate stream plus the stream/event bookkeeping around it. Here the single-pass
// kernel's last workgroup (reduce.hip; the last-block-done idea of
// threadFenceReduction_kernel.cu:116-171, stretched across devices) does it in place:
//
//   1. it pushes its rank's partial into slot [rank] of EVERY rank's mailbox (one 8-byte system-
//      scope store per 32 bits, each word carrying the launch's epoch in its upper half — the
//      "LL" flag-in-data form: a word is valid iff its epoch matches, no separate flag or fence);
//   2. it polls its own mailbox until all `world` slots hold this epoch, and
//   3. folds the `world` partials with the same wave64 butterfly on every rank (bit-identical
//      results everywhere), then writes `out`.
//
// Mailboxes are uncached device memory (every access bypasses the caches) mapped into each peer
// through HIP IPC, so a peer's store over xGMI is what the poller reads. Epochs come from a
// device-resident counter bumped by the finishing workgroup, so a captured hipGraph replays
// without host involvement; the mailbox is double-buffered by epoch parity (a rank can run at
// most one epoch ahead of the slowest peer: it needs that peer's partial to finish). A poll that
// exceeds `timeout` sets a sticky error word instead of hanging (later launches then do not wait),
// which XrankChannel::error() reports. A rank whose own fan-in failed pushes its partial with a
// poison flag in the tag; its peers then set error value 2 (bit 1) and poison their results too, so the
// failure is visible on every rank (integers are poisoned to the operator's identity, so the
// error word is their only signal). Epochs are 31 bits (the 32nd tag bit is the flag) and wrap
// keeping their parity.
//
// Every rank must launch the bound reductions of a channel in the same order; one channel per
// concurrently running reduction (stream lane).
#pragma once

#include <hip/hip_runtime_api.h>

#include <array>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace mireduce {

constexpr int kMaxXrankRanks = 16;
// [parity 2][source rank kMaxXrankRanks][2 words]
constexpr size_t kXrankMailboxWords = 2 * kMaxXrankRanks * 2;

// Device-resident descriptor read by the finishing workgroup (reduce.hip).
struct XrankDesc {
  uint64_t* peer_mbox[kMaxXrankRanks];  // rank p's mailbox as mapped in this process ([rank] = own)
  uint64_t* own_mbox;
  unsigned* epoch;          // finished launches on this channel
  unsigned* error;          // sticky bits: 1 = a peer's partial missed the timeout,
                            // 2 = a peer pushed a poisoned partial (its own fan-in failed)
  int rank;
  int world;
  uint64_t timeout_ticks;   // wall_clock64() ticks
  // Exchange timing (set_stamps; null = off): the finisher records, per launch e, the wall clock
  // at its first push and when every peer's partial had landed, at stamps[2 * (e & stamp_mask)].
  uint64_t* stamps;
  unsigned stamp_mask;
};

using IpcHandleBytes = std::array<char, sizeof(hipIpcMemHandle_t)>;

class XrankChannel {
 public:
  // Allocates this rank's mailbox (uncached device memory) on `device` (-1: current).
  explicit XrankChannel(int device = -1, double timeout_s = 2.0);
  ~XrankChannel();
  XrankChannel(const XrankChannel&) = delete;
  XrankChannel& operator=(const XrankChannel&) = delete;

  // IPC handle of this rank's mailbox (exchange it with every peer, e.g. an all-gather).
  IpcHandleBytes handle() const;
  // Map every peer's mailbox (handles[r] = rank r's handle(); handles[rank] is ignored).
  void connect(int rank, int world, const std::vector<IpcHandleBytes>& handles);
  bool connected() const { return connected_; }
  const XrankDesc* device_desc() const { return desc_dev_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  // Synchronous reads (after the launches have completed).
  unsigned error() const;
  unsigned epoch() const;
  void clear_error();
  // Exchange timing: `stamps` (device, 2 * cap uint64, cap a power of two; nullptr = off) receives
  // (push, all peers landed) wall-clock ticks of launch e at [2 * (e % cap)]. Synchronous; no launch
  // on this channel may be running.
  void set_stamps(uint64_t* stamps, unsigned cap);
  // Ticks per microsecond of the device wall clock (wall_clock64()).
  double ticks_per_us() const { return ticks_per_us_; }

 private:
  int device_ = 0;
  int rank_ = 0, world_ = 1;
  bool connected_ = false;
  double timeout_s_ = 2.0;
  double ticks_per_us_ = 100.0;
  uint64_t* mbox_ = nullptr;     // own mailbox (uncached)
  unsigned* counters_ = nullptr; // [0] epoch, [1] error
  XrankDesc* desc_dev_ = nullptr;
  std::vector<void*> opened_;    // peer mappings to close
};

}  // namespace mireduce
