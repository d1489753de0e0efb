// Reduction operator functors, usable from host and device code.
//
// One functor per operator replaces the reference's three copy-pasted kernels
// (sumreduce6/minreduce6/maxreduce6, cuda/C/src/reduction/reduction_kernel.cu:74-253).
// The identity element is the operator's neutral value (0, +max, lowest) rather than
// g_idata[i] as in reduction_kernel.cu:140,204 — that read is the out-of-bounds bug B2.
#pragma once

#include <cmath>
#include <cstdint>
#include <limits>
#include <type_traits>

#if defined(__HIPCC__)
#define MIREDUCE_HD __host__ __device__ __forceinline__
#else
#define MIREDUCE_HD inline
#endif

namespace mireduce {

// Integer sums wrap modulo 2^bits (two's complement) instead of invoking signed-overflow UB.
template <class T>
MIREDUCE_HD T wrap_add(T a, T b) {
  if constexpr (std::is_integral_v<T>) {
    using U = std::make_unsigned_t<T>;
    return static_cast<T>(static_cast<U>(a) + static_cast<U>(b));
  } else {
    return a + b;
  }
}

struct SumOp {
  template <class T> MIREDUCE_HD static T identity() { return T(0); }
  template <class T> MIREDUCE_HD static T apply(T a, T b) { return wrap_add(a, b); }
};

// MIN/MAX on floats follow IEEE-754 minNum/maxNum (a NaN operand is ignored), which is what
// v_min_f64 / v_max_f32 implement and what std::fmin/std::fmax do on the host.
struct MinOp {
  template <class T> MIREDUCE_HD static T identity() {
    if constexpr (std::is_floating_point_v<T>) return std::numeric_limits<T>::infinity();
    else return std::numeric_limits<T>::max();
  }
  template <class T> MIREDUCE_HD static T apply(T a, T b) {
    if constexpr (std::is_floating_point_v<T>) return std::fmin(a, b);
    else return b < a ? b : a;
  }
};

struct MaxOp {
  template <class T> MIREDUCE_HD static T identity() {
    if constexpr (std::is_floating_point_v<T>) return -std::numeric_limits<T>::infinity();
    else return std::numeric_limits<T>::lowest();
  }
  template <class T> MIREDUCE_HD static T apply(T a, T b) {
    if constexpr (std::is_floating_point_v<T>) return std::fmax(a, b);
    else return a < b ? b : a;
  }
};

}  // namespace mireduce
