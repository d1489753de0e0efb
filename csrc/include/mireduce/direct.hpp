// Direct peer-to-peer reductions over xGMI (no RCCL): every rank maps every peer's buffers
// through HIP IPC handles and reduces by reading them with its own kernels.
//
// Reference pattern: the vendored simpleP2P sample (peer access + a kernel on GPU0 reading GPU1's
// buffer, cuda/C/src/simpleP2P/simpleP2P.cu:164,250-330) — SURVEY.md §2.2 last row, P11, §7.4
// step 9. MI355X design: 8 fully connected GPUs with 7 xGMI links each; a ring all-reduce moves
// each byte over one link per step, while this one-shot scheme has every rank pull its chunk
// from all 7 peers at once (reduce-scatter), then pull the other 7 reduced chunks (all-gather):
// all 7 links of every GPU are busy in both phases.
//
// Synchronisation is host-side (stream sync + TCP-bootstrap barrier between phases), so no
// kernel ever waits on another GPU — nothing can hang on a missing peer. Cross-device
// visibility: buffers are fine-grained device memory (hipDeviceMallocFinegrained); producing
// kernels end with a system-scope release, consuming kernels start with a system-scope acquire.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <vector>

#include "mireduce/comm.hpp"
#include "mireduce/types.hpp"

namespace mireduce {

constexpr int kMaxDirectPeers = 16;

class DirectPeers {
 public:
  // Collective over `boot`: allocates `bytes` for in and out on this rank, exchanges IPC handles.
  DirectPeers(TcpBootstrap& boot, int device, size_t bytes, bool finegrained = true);
  ~DirectPeers();
  DirectPeers(const DirectPeers&) = delete;
  DirectPeers& operator=(const DirectPeers&) = delete;

  void* in() const { return in_; }
  void* out() const { return out_; }
  size_t bytes() const { return bytes_; }
  bool finegrained() const { return finegrained_; }
  int device() const { return device_; }

  // out[i] = op over ranks of in[i], on every rank (one-shot reduce-scatter + all-gather).
  void allreduce(size_t count, DType t, Op op, hipStream_t s);
  // out[i] = op over ranks of in[i] on `root` only (reduce-scatter + gather to root).
  void reduce(size_t count, DType t, Op op, int root, hipStream_t s);

 private:
  void reduce_scatter(size_t count, DType t, Op op, hipStream_t s);
  void gather_chunks(size_t count, DType t, hipStream_t s);
  TcpBootstrap& boot_;
  int rank_ = 0, world_ = 1, device_ = 0;
  size_t bytes_ = 0;
  bool finegrained_ = true;
  void* in_ = nullptr;
  void* out_ = nullptr;
  std::vector<void*> peer_in_, peer_out_;  // [world]; own entries are in_/out_
};

// Chunk r of `count` elements split over `world` ranks, aligned to 16-byte vectors.
void direct_chunk(size_t count, size_t elem_size, int world, int r, size_t* begin, size_t* end);

}  // namespace mireduce
