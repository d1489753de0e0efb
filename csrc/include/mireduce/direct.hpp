// Direct peer-to-peer element-wise reductions over xGMI (no RCCL), one kernel per collective.
//
// Reference pattern: the vendored simpleP2P sample (peer access + a kernel on GPU0 reading GPU1's
// buffer, cuda/C/src/simpleP2P/simpleP2P.cu:164,250-330) — SURVEY.md §2.2 last row, P11, §7.4
// step 9 — applied to mpi/reduce.c's element-wise MPI_Reduce (reduce.c:76,90).
//
// MI355X design: 8 fully connected GPUs, 7 xGMI links each. A ring all-reduce moves each byte over
// one link per step; here every rank pulls its 1/world chunk from ALL peers at once (reduce-
// scatter), then pulls the other reduced chunks from their owners (all-gather), so all 7 links of
// every GPU carry traffic in both phases. Every rank maps every peer's input / output / signal
// buffers through HIP IPC once (connect); a collective is then ONE kernel launch with no host
// involvement — capturable into a hipGraph:
//
//   barrier 0 (inputs ready) -> reduce-scatter -> barrier 1 (chunks reduced) -> all-gather
//   -> barrier 2 (nobody still reads this rank's buffers)
//
// The barriers are per workgroup: workgroup b of every rank handles the same sub-range of every
// chunk, so it only has to meet workgroup b of the other ranks (flags in uncached signal memory,
// written with system-scope stores into every peer's array, polled locally; producers release at
// system scope first, consumers acquire after). Flags carry the launch's epoch from a device
// counter (so graph replays need no host reset). Every wait is bounded: a timeout sets a sticky
// error word (later launches then do not wait) instead of hanging — error() reports it.
// All ranks must use the same grid (checked in connect) and launch the same sequence of collectives.
#pragma once

#include <hip/hip_runtime_api.h>

#include <array>
#include <cstddef>
#include <cstdint>
#include <vector>

#include "mireduce/types.hpp"
#include "mireduce/xrank.hpp"

namespace mireduce {

constexpr int kMaxDirectRanks = 16;
constexpr int kMaxDirectBlocks = 1024;
constexpr int kDirectBlock = 512;  // threads per workgroup
constexpr int kDirectPhases = 3;

// Device-resident descriptor read by the kernel.
struct DirectDesc {
  const char* in[kMaxDirectRanks];  // rank r's input buffer as mapped here ([rank] = own)
  char* out[kMaxDirectRanks];       // rank r's output buffer
  unsigned* sig[kMaxDirectRanks];   // rank r's flags [phase][block][source rank]
  unsigned* ctl;                    // own: [0] epoch, [1] error, [2] arrival ticket
  int rank;
  int world;
  uint64_t timeout_ticks;
};

class DirectAllreduce {
 public:
  // Registers `bytes` of input and output on `device` (-1: current); `grid` workgroups per
  // collective (0: one per CU), identical on every rank.
  DirectAllreduce(int device, size_t bytes, int grid = 0, double timeout_s = 10.0);
  ~DirectAllreduce();
  DirectAllreduce(const DirectAllreduce&) = delete;
  DirectAllreduce& operator=(const DirectAllreduce&) = delete;

  // This rank's IPC handles (input, output, signals) + grid, to all-gather over the ranks.
  static constexpr size_t kHandleBytes = 3 * sizeof(IpcHandleBytes) + sizeof(int32_t);
  std::vector<char> handles() const;
  void connect(int rank, int world, const std::vector<std::vector<char>>& all);

  void* in() const { return in_; }
  void* out() const { return out_; }
  size_t bytes() const { return bytes_; }
  int grid() const { return grid_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  bool connected() const { return connected_; }

  // out[i] = op over ranks of in[i] on every rank.
  void allreduce(size_t count, DType t, Op op, hipStream_t s);
  // out[i] = op over ranks of in[i] on `root` only (reduce-scatter + gather to the root).
  void reduce(size_t count, DType t, Op op, int root, hipStream_t s);
  // Fabric probe (no reduction): one kernel reads `bytes_each` (<= bytes()) of every peer's input
  // buffer at once over xGMI (own buffer when world == 1) — this rank's ingress roofline next to
  // the collectives that run on the same buffers.
  void read_peers(size_t bytes_each, hipStream_t s);
  // Synchronous reads (after the launches have completed).
  unsigned error() const;
  unsigned epoch() const;

 private:
  void launch(size_t count, DType t, Op op, int gather_rank, hipStream_t s);
  int device_ = 0, rank_ = 0, world_ = 1, grid_ = 0;
  size_t bytes_ = 0;
  double timeout_s_ = 10.0;
  bool connected_ = false;
  void* in_ = nullptr;
  void* out_ = nullptr;
  unsigned* sig_ = nullptr;
  unsigned* ctl_ = nullptr;
  DirectDesc* desc_ = nullptr;
  uint32_t* sink_ = nullptr;
  std::vector<void*> opened_;
  std::vector<const void*> peer_in_;  // peers' input buffers as mapped here
};

// Chunk r of `count` elements split over `world` ranks, aligned to 16-byte vectors.
void direct_chunk(size_t count, size_t elem_size, int world, int r, size_t* begin, size_t* end);

}  // namespace mireduce
