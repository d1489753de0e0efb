// Dispatch-table entries of the bf16 combos (14..16): every (block, unroll, policy, pipelined)
// reduce_stream variant of each (op, dtype, acc) (reduce_kernels.hpp; split out of reduce.hip so the
// ~1,400 instantiations compile in parallel).
#include "reduce_kernels.hpp"

namespace mireduce {
namespace detail {

void fill_table_bf16(Table& tb) {
  fill_combo<SumOp, bf16_t, float>(tb, 14);
  fill_combo<MinOp, bf16_t, float>(tb, 15);
  fill_combo<MaxOp, bf16_t, float>(tb, 16);
}

}  // namespace detail
}  // namespace mireduce
