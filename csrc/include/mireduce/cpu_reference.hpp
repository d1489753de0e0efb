// Host reference reducers (SURVEY.md §2.1 C8 → host/cpu_reference).
//
// Reference: sumreduceCPU (Kahan, reduction.cpp:214-227), minreduceCPU / maxreduceCPU
// (reduction.cpp:228-249). Here: compensated (Neumaier) sums in the accumulator type, exact
// modular integer sums, optional multi-threading for multi-GB arrays, and the tolerance policy
// used by every verifier in the framework.
#pragma once

#include <cstddef>
#include <cstdint>

#include "mireduce/types.hpp"

namespace mireduce {

// Reduce n host elements of type t with op into *out (element type acc). threads <= 0: auto.
void cpu_reduce(const void* in, size_t n, DType t, Op op, DType acc, void* out, int threads = 0);

// Σ|x| in fp64 (scale for the relative sum tolerance).
double cpu_abs_sum(const void* in, size_t n, DType t, int threads = 0);

// Fold `count` partials (element type acc) on the host — the reference's --cpufinal path
// (reduction.cpp:328-340), with the MIN/MAX fold fixed to use the operator (bug B3).
void cpu_fold(const void* partials, size_t count, DType acc, Op op, void* out);

// Absolute tolerance for comparing a device result against cpu_reduce. Exact (0) for integer
// types and for MIN/MAX; for floating sums a bound proportional to Σ|x|.
double sum_tolerance(DType t, DType acc, size_t n, double abs_sum);

// Value of the first element of an accumulator-typed buffer as double / int64 (for printing).
// Closed-form result of reducing n elements of the IotaMod pattern (x[i] = i mod 1024, i from
// `offset`) — an oracle for arrays too large to copy to the host that shares no code with any
// device kernel. Exact for integer accumulators and for fp64; returns
// false for 16-bit element types (their elements above 256 are rounded). Writes `acc` bytes.
bool analytic_iotamod(uint64_t n, uint64_t offset, DType t, Op op, DType acc, void* out);

double acc_as_double(const void* p, DType acc);
int64_t acc_as_int64(const void* p, DType acc);

}  // namespace mireduce
