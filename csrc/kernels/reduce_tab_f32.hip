// Dispatch-table entries of the f32 combos (7..10): every (block, unroll, policy, pipelined)
// reduce_stream variant of each (op, dtype, acc) (reduce_kernels.hpp; split out of reduce.hip so the
// ~1,400 instantiations compile in parallel).
#include "reduce_kernels.hpp"

namespace mireduce {
namespace detail {

void fill_table_f32(Table& tb) {
  fill_combo<SumOp, float, double>(tb, 7);
  fill_combo<SumOp, float, float>(tb, 8);
  fill_combo<MinOp, float, float>(tb, 9);
  fill_combo<MaxOp, float, float>(tb, 10);
}

}  // namespace detail
}  // namespace mireduce
