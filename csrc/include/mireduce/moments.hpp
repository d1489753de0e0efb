// Fused one-pass statistics (count, mean, variance, min, max) of a float32/float64 array;
// see csrc/kernels/moments.hip.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>

#include "mireduce/types.hpp"

namespace mireduce {

// out5 (device, 5 doubles) <- [K = x[0], Σ(x-K), Σ(x-K)², min, max]. `partials` must hold
// moments_partials_bytes(max_grid) bytes. Input must be 16-byte aligned.
void moments_device(const void* in, size_t n, DType t, double* out5, void* partials, int max_grid, int num_cus,
                    hipStream_t stream);
size_t moments_partials_bytes(int max_grid);

}  // namespace mireduce
