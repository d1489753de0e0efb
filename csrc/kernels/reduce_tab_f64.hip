// Dispatch-table entries of the f64 combos (11..13): every (block, unroll, policy, pipelined)
// reduce_stream variant of each (op, dtype, acc) (reduce_kernels.hpp; split out of reduce.hip so the
// ~1,400 instantiations compile in parallel).
#include "reduce_kernels.hpp"

namespace mireduce {
namespace detail {

void fill_table_f64(Table& tb) {
  fill_combo<SumOp, double, double>(tb, 11);
  fill_combo<MinOp, double, double>(tb, 12);
  fill_combo<MaxOp, double, double>(tb, 13);
}

}  // namespace detail
}  // namespace mireduce
