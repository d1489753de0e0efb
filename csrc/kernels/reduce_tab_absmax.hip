// Dispatch-table entries of the absmax combos (25..28): every (block, unroll, policy, pipelined)
// reduce_stream variant of each (op, dtype, acc) (reduce_kernels.hpp; split out of reduce.hip so the
// ~1,400 instantiations compile in parallel).
#include "reduce_kernels.hpp"

namespace mireduce {
namespace detail {

void fill_table_absmax(Table& tb) {
  fill_combo<AbsMaxOp, float, float>(tb, 25);
  fill_combo<AbsMaxOp, double, double>(tb, 26);
  fill_combo<AbsMaxOp, bf16_t, float>(tb, 27);
  fill_combo<AbsMaxOp, f16_t, float>(tb, 28);
}

}  // namespace detail
}  // namespace mireduce
