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

// Every functor has `identity`, `apply` (the associative combine of two accumulators) and `pre`
// (the per-element transform applied once when an input element enters an accumulator: the
// identity for SUM/MIN/MAX, x*x for SUMSQ, |x| for AMAX). Partials are combined with `apply`
// only, so a fused transform never runs twice.
struct SumOp {
  template <class T> MIREDUCE_HD static T identity() { return T(0); }
  template <class T> MIREDUCE_HD static T apply(T a, T b) { return wrap_add(a, b); }
  template <class T> MIREDUCE_HD static T pre(T x) { return x; }
};

// Σ x² (squared L2 norm) — fused: the square is taken in the accumulator type as the element is
// loaded, no intermediate array. Floating types only.
struct SumSqOp {
  template <class T> MIREDUCE_HD static T identity() { return T(0); }
  template <class T> MIREDUCE_HD static T apply(T a, T b) { return a + b; }
  template <class T> MIREDUCE_HD static T pre(T x) { return x * x; }
};

// MIN/MAX on floats follow IEEE-754 minNum/maxNum (a NaN operand is ignored), which is what
// v_min_f64 / v_max_f32 implement and what std::fmin/std::fmax do on the host.
//
// On the device the instructions are emitted directly: llvm.minnum in IEEE mode makes hipcc
// canonicalise every operand first (an extra `v_max_f64 x, x, x` per element, which doubled the
// VALU work of the MIN/MAX streaming loop). The hardware ops already return the non-NaN operand
// for quiet NaNs; only signalling-NaN inputs (never produced by arithmetic) would differ.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ double hw_min(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double hw_max(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float hw_min(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float hw_max(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
#endif

struct MinOp {
  template <class T> MIREDUCE_HD static T identity() {
    if constexpr (std::is_floating_point_v<T>) return std::numeric_limits<T>::infinity();
    else return std::numeric_limits<T>::max();
  }
  template <class T> MIREDUCE_HD static T apply(T a, T b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (std::is_floating_point_v<T>) return hw_min(a, b);
#else
    if constexpr (std::is_floating_point_v<T>) return std::fmin(a, b);
#endif
    else return b < a ? b : a;
  }
  template <class T> MIREDUCE_HD static T pre(T x) { return x; }
};

struct MaxOp {
  template <class T> MIREDUCE_HD static T identity() {
    if constexpr (std::is_floating_point_v<T>) return -std::numeric_limits<T>::infinity();
    else return std::numeric_limits<T>::lowest();
  }
  template <class T> MIREDUCE_HD static T apply(T a, T b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (std::is_floating_point_v<T>) return hw_max(a, b);
#else
    if constexpr (std::is_floating_point_v<T>) return std::fmax(a, b);
#endif
    else return a < b ? b : a;
  }
  template <class T> MIREDUCE_HD static T pre(T x) { return x; }
};

// max |x| (the amax of FP8 scaling, the inf-norm): |x| on load, MAX to combine (identity 0 since
// every transformed value is >= 0; a NaN input is ignored like in MaxOp). Floating types only.
struct AbsMaxOp {
  template <class T> MIREDUCE_HD static T identity() { return T(0); }
  template <class T> MIREDUCE_HD static T apply(T a, T b) { return MaxOp::apply(a, b); }
#if defined(__HIP_DEVICE_COMPILE__)
  template <class T> MIREDUCE_HD static T pre(T x) { return __builtin_fabs(x); }
#else
  template <class T> MIREDUCE_HD static T pre(T x) { return std::fabs(x); }
#endif
};

}  // namespace mireduce
