// Minimal C++ use of the mireduce library: fill 2^28 doubles on the device, reduce them with the
// single-pass streaming kernel, print the sum and the plan (the C++ counterpart of
// examples/01_single_gpu.py; reference entry point: cuda/C/src/reduction/reduction.cpp:84-204).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "mireduce/reduce.hpp"
#include "mireduce/rng.hpp"

int main() {
  using namespace mireduce;
  const size_t n = size_t{1} << 28;
  double *x = nullptr, *out = nullptr;
  if (hipMalloc(&x, n * sizeof(double)) != hipSuccess || hipMalloc(&out, sizeof(double)) != hipSuccess) {
    std::fprintf(stderr, "no usable HIP device\n");
    return 1;
  }
  FillSpec spec;
  spec.pattern = Pattern::IotaMod;  // x[i] = i mod 1024: the exact sum is known in closed form
  fill_device(x, n, DType::Float64, spec, nullptr);
  Workspace ws(-1, 16384);
  const LaunchPlan p = reduce(x, n, DType::Float64, Op::Sum, DType::Float64, out, ws, nullptr, ReduceConfig{});
  double got = 0;
  (void)hipMemcpy(&got, out, sizeof got, hipMemcpyDeviceToHost);
  const double expect = static_cast<double>(n / 1024) * (1023.0 * 1024.0 / 2.0);
  std::printf("sum = %.1f (expected %.1f), grid %d x %d threads, unroll %d\n", got, expect, p.grid, p.block, p.unroll);
  (void)hipFree(x);
  (void)hipFree(out);
  return got == expect ? 0 : 2;
}
