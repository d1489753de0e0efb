// One launch, many tensors: out[i] = op over tensor i (csrc/kernels/reduce_many.hip).
//
// Not in the reference (one array per run: cuda/C/src/reduction/reduction.cpp:661-783). The
// MI355X use is the per-step reduction of a whole list of same-typed tensors — e.g. the L2 norms
// of every gradient shard of a data-parallel step (SUMSQ), or the amax of every tensor an FP8
// recipe scales (AMAX) — without one launch (and one tail) per tensor.
//
// The list is bound once (its segment table is built on the host and uploaded to the device);
// launch() is then a single kernel launch, capturable into a hipGraph. Tensors may have any length
// and alignment (scalar head/tail per segment); long tensors are cut into segments reduced by
// different waves and finished single-pass by their last segment (per-tensor tickets, fold in
// segment order: deterministic).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "mireduce/types.hpp"

namespace mireduce {

class BoundReduceMany {
 public:
  // ptrs[i] / counts[i]: device pointer and element count of tensor i (element type t).
  // out: device array of ptrs.size() values of type acc. stream: where the table upload goes.
  BoundReduceMany(const std::vector<const void*>& ptrs, const std::vector<uint64_t>& counts, DType t, Op op,
                  DType acc, void* out, int device, int num_cus, hipStream_t stream);
  ~BoundReduceMany();
  BoundReduceMany(const BoundReduceMany&) = delete;
  BoundReduceMany& operator=(const BoundReduceMany&) = delete;

  // `out` (optional) redirects this launch's results to another device array of ptrs.size() values.
  void launch(hipStream_t stream, void* out = nullptr) const;
  size_t tensors() const { return tensors_; }
  size_t segments() const { return segments_; }
  int grid() const { return grid_; }

 private:
  size_t tensors_ = 0, segments_ = 0;
  int grid_ = 1;
  DType t_, acc_;
  Op op_;
  void* out_ = nullptr;
  void* table_ = nullptr;     // device: segment descriptors + per-tensor first/count
  void* partials_ = nullptr;  // device: one AccT per segment
  unsigned* tickets_ = nullptr;
};

}  // namespace mireduce
