// Dispatch-table entries of the int64 combos (4..6): every (block, unroll, policy, pipelined)
// reduce_stream variant of each (op, dtype, acc) (reduce_kernels.hpp; split out of reduce.hip so the
// ~1,400 instantiations compile in parallel).
#include "reduce_kernels.hpp"

namespace mireduce {
namespace detail {

void fill_table_int64(Table& tb) {
  fill_combo<SumOp, int64_t, int64_t>(tb, 4);
  fill_combo<MinOp, int64_t, int64_t>(tb, 5);
  fill_combo<MaxOp, int64_t, int64_t>(tb, 6);
}

}  // namespace detail
}  // namespace mireduce
