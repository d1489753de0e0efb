// Dispatch-table entries of the int32 combos (0..3): every (block, unroll, policy, pipelined)
// reduce_stream variant of each (op, dtype, acc) (reduce_kernels.hpp; split out of reduce.hip so the
// ~1,400 instantiations compile in parallel).
#include "reduce_kernels.hpp"

namespace mireduce {
namespace detail {

void fill_table_int32(Table& tb) {
  fill_combo<SumOp, int32_t, int64_t>(tb, 0);
  fill_combo<SumOp, int32_t, int32_t>(tb, 1);
  fill_combo<MinOp, int32_t, int32_t>(tb, 2);
  fill_combo<MaxOp, int32_t, int32_t>(tb, 3);
}

}  // namespace detail
}  // namespace mireduce
