// 16-byte vector loads for the streaming kernels (device code; included by .hip sources only).
//
// Every element type is read 16 bytes per lane — one global_load_dwordx4 — whatever its width:
// int32x4, int64x2, float4, double2, or eight bf16/f16 carried as four 32-bit words. elem() returns
// element k of such a vector in the accumulator type. store_sc1 / load_sc1 are the write-through /
// L1-bypassing accesses the single-pass finalisations publish and read partials with.
#pragma once

#include <cstdint>
#include <type_traits>

#include "mireduce/half.hpp"

namespace mireduce {
namespace kern {

template <class T> struct Vec16;
template <> struct Vec16<int32_t> { using type = int32_t __attribute__((ext_vector_type(4))); static constexpr int N = 4; };
template <> struct Vec16<int64_t> { using type = int64_t __attribute__((ext_vector_type(2))); static constexpr int N = 2; };
template <> struct Vec16<float>   { using type = float __attribute__((ext_vector_type(4)));   static constexpr int N = 4; };
template <> struct Vec16<double>  { using type = double __attribute__((ext_vector_type(2)));  static constexpr int N = 2; };
// 16-bit floats: 8 elements per 16-byte load, carried as four 32-bit words (half.hpp)
template <> struct Vec16<bf16_t>  { using type = uint32_t __attribute__((ext_vector_type(4))); static constexpr int N = 8; };
template <> struct Vec16<f16_t>   { using type = uint32_t __attribute__((ext_vector_type(4))); static constexpr int N = 8; };

// Element k of a loaded 16-byte vector, converted to the accumulator type. bf16 -> fp32 is a
// shift or a mask of the containing word; fp16 -> fp32 is one v_cvt_f32_f16.
template <class T, class AccT, class V>
__device__ __forceinline__ AccT elem(const V& v, int k) {
  if constexpr (std::is_same_v<T, bf16_t>) {
    const uint32_t w = v[k >> 1];
    return bits_to_float((k & 1) ? (w & 0xffff0000u) : (w << 16));
  } else if constexpr (std::is_same_v<T, f16_t>) {
    const uint32_t w = v[k >> 1];
    const uint16_t h = static_cast<uint16_t>((k & 1) ? (w >> 16) : (w & 0xffffu));
    return static_cast<float>(__builtin_bit_cast(_Float16, h));
  } else {
    return static_cast<AccT>(v[k]);
  }
}


template <class T> struct Bits { using type = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>; };

// Write-through (sc1) store / L1-bypassing (sc1) load of one accumulator value: the
// agent-scope relaxed atomic forms lower to global_store/load ... sc1 on gfx950.
template <class T>
__device__ __forceinline__ void store_sc1(T* p, T v) {
  using B = typename Bits<T>::type;
  B b;
  __builtin_memcpy(&b, &v, sizeof(T));
  __hip_atomic_store(reinterpret_cast<B*>(p), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class T>
__device__ __forceinline__ T load_sc1(const T* p) {
  using B = typename Bits<T>::type;
  B b = __hip_atomic_load(reinterpret_cast<const B*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  T v;
  __builtin_memcpy(&v, &b, sizeof(T));
  return v;
}

}  // namespace kern
}  // namespace mireduce
