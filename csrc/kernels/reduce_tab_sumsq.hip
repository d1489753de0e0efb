// Dispatch-table entries of the sumsq combos (20..24): every (block, unroll, policy, pipelined)
// reduce_stream variant of each (op, dtype, acc) (reduce_kernels.hpp; split out of reduce.hip so the
// ~1,400 instantiations compile in parallel).
#include "reduce_kernels.hpp"

namespace mireduce {
namespace detail {

void fill_table_sumsq(Table& tb) {
  fill_combo<SumSqOp, float, double>(tb, 20);
  fill_combo<SumSqOp, float, float>(tb, 21);
  fill_combo<SumSqOp, double, double>(tb, 22);
  fill_combo<SumSqOp, bf16_t, float>(tb, 23);
  fill_combo<SumSqOp, f16_t, float>(tb, 24);
}

}  // namespace detail
}  // namespace mireduce
