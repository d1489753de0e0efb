// Arg-reductions: the position (and value) of the maximum or minimum (csrc/kernels/arg_reduce.hip).
//
// Not in the reference, whose MIN/MAX reductions return the extreme value only
// (cuda/C/src/reduction/reduction_kernel.cu:128-253, mpi/reduce.c:21-28). torch.argmax / argmin /
// max(dim) semantics: the FIRST index of the extreme; NaN counts as the extreme for both
// (the first NaN wins); -0.0 == +0.0. Whole arrays are the rows = 1 case.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

#include "mireduce/types.hpp"

namespace mireduce {

struct ArgPlan {
  int grid = 0;              // workgroups
  int block = 256;           // threads per workgroup
  int lanes_per_row = 256;   // < 64: short rows, a group of this many lanes per row
  uint64_t splits = 1;       // long rows: workgroups per row (> 1: per-row tickets, the last one folds)
  int unroll = 0;            // 16-byte vectors in flight per lane (long rows) / row batches (short)
  int wg_per_cu = 0;         // resident workgroups per CU the grid was sized for
};

// Long-row tunables (0 = the gfx950 default; tools/arg_reduce_bw.py --sweep measures them).
struct ArgTune {
  int unroll = 0;     // 2, 4 or 8
  int wg_per_cu = 0;  // cap on resident workgroups per CU
};

// Scratch (device bytes) an arg-reduction of this shape needs; 0 if none. Zero-fill it once before
// its first use (the kernel leaves the ticket words zero again).
size_t arg_reduce_scratch_bytes(size_t rows, size_t cols, DType t, int num_cus);

// For every row r of the row-major [rows, cols] matrix `in` (cols >= 1):
//   out_index[r] = first c with in[r, c] the maximum (op = Max) or minimum (op = Min),
//   out_value[r] = in[r, out_index[r]]   (element type t).
ArgPlan arg_reduce_rows(const void* in, size_t rows, size_t cols, DType t, Op op, void* out_value,
                        int64_t* out_index, void* scratch, int num_cus, hipStream_t stream,
                        ArgTune tune = {});

// Cross-rank MAXLOC / MINLOC combine of one (value, index) pair per rank, device-side and
// graph-capturable (models/loc.py): loc_pack writes this rank's pair — the value's comparison key
// bits (16-bit floats widened to fp32) and index + index_offset — as 2 uint64 words; after an
// all-gather of the pairs, loc_pick folds `world` of them with arg_reduce's rules (the extreme
// wins, NaN being the extreme; equal values: the smaller index) and writes the winning global index
// to out_index[0] (and, when out_value is not null, its value in element type t). One thread each.
void loc_pack(const void* value, const int64_t* index, int64_t index_offset, DType t, uint64_t* pair,
              hipStream_t stream);
void loc_pick(const uint64_t* pairs, int world, DType t, Op op, int64_t* out_index, void* out_value,
              hipStream_t stream);

// Host reference with the same semantics (multi-threaded over rows).
void cpu_arg_reduce_rows(const void* in, size_t rows, size_t cols, DType t, Op op, void* out_value,
                         int64_t* out_index);

}  // namespace mireduce
