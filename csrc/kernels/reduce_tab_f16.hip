// Dispatch-table entries of the f16 combos (17..19): every (block, unroll, policy, pipelined)
// reduce_stream variant of each (op, dtype, acc) (reduce_kernels.hpp; split out of reduce.hip so the
// ~1,400 instantiations compile in parallel).
#include "reduce_kernels.hpp"

namespace mireduce {
namespace detail {

void fill_table_f16(Table& tb) {
  fill_combo<SumOp, f16_t, float>(tb, 17);
  fill_combo<MinOp, f16_t, float>(tb, 18);
  fill_combo<MaxOp, f16_t, float>(tb, 19);
}

}  // namespace detail
}  // namespace mireduce
