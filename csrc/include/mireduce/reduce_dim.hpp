// Reductions along one axis of a row-major [rows, cols] matrix (csrc/kernels/reduce_dim.hip).
//
// Not in the reference, whose reductions always collapse a whole array to one value
// (cuda/C/src/reduction/reduction_kernel.cu:74-253) or combine whole vectors element-wise across
// ranks (mpi/reduce.c:76,90). A framework on MI355X also needs the per-row / per-column forms
// (torch.sum(x, dim)); they share the element types, operators, accumulators and 16-byte loads of
// the full reduction.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

#include "mireduce/types.hpp"

namespace mireduce {

// How a dimension reduction was laid out (recorded by the Python layer; printed by the tools).
struct DimPlan {
  int grid = 0;             // workgroups
  int block = 256;          // threads per workgroup
  int lanes_per_row = 64;   // rows mode: lanes cooperating on one row segment (1..64)
  uint64_t splits = 1;      // rows mode: segments per row (> 1: per-row tickets, last arriver folds)
                            // cols mode: row ranges per column block (> 1: second fold launch)
};

// Scratch (device bytes) a dimension reduction of this shape needs; 0 if none. The buffer must be
// zero-filled once before its first use (the kernels leave the ticket words zero again).
size_t reduce_rows_scratch_bytes(size_t rows, size_t cols, DType t, int num_cus);
size_t reduce_cols_scratch_bytes(size_t outer, size_t rows, size_t cols, DType t, DType acc, int num_cus);

// out[r] = op over c of in[r * cols + c]   (out: `rows` values of type acc)
DimPlan reduce_rows(const void* in, size_t rows, size_t cols, DType t, Op op, DType acc, void* out,
                    void* scratch, int num_cus, hipStream_t stream);

// out[o * cols + c] = op over r of in[(o * rows + r) * cols + c]   (out: outer * cols values of
// type acc) — the middle axis of a contiguous [outer, rows, cols] tensor; outer = 1 is the
// column reduction of a matrix.
DimPlan reduce_cols(const void* in, size_t outer, size_t rows, size_t cols, DType t, Op op, DType acc, void* out,
                    void* scratch, int num_cus, hipStream_t stream);

}  // namespace mireduce
