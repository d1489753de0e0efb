// 16-bit floating element types: bfloat16 and IEEE binary16 (half).
//
// Not in the reference (its element types are int, float and double:
// cuda/C/src/reduction/reduction_kernel.cu:527-564; MPI_INT / MPI_DOUBLE in mpi/reduce.c:76,90).
// They are the native storage types of the MI355X matrix cores and of most data a framework on
// this GPU reduces, so the streaming kernel reads them at the same 16 bytes per lane (8 elements)
// and accumulates in fp32.
//
// Storage is a 16-bit pattern wrapped in a struct (no arithmetic on the storage type: every
// operation converts to float first). Conversions are plain bit manipulation, identical on host
// and device, so host- and device-generated data are bit-for-bit the same; float -> 16-bit rounds
// to nearest even and keeps NaNs quiet.
#pragma once

#include <cstdint>

#include "mireduce/ops.hpp"

namespace mireduce {

MIREDUCE_HD float bits_to_float(uint32_t u) {
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}

MIREDUCE_HD uint32_t float_to_bits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return u;
}

MIREDUCE_HD float bf16_bits_to_float(uint16_t b) { return bits_to_float(static_cast<uint32_t>(b) << 16); }

MIREDUCE_HD uint16_t float_to_bf16_bits(float f) {
  const uint32_t u = float_to_bits(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);  // quiet NaN
  const uint32_t rounding = 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>((u + rounding) >> 16);
}

MIREDUCE_HD float f16_bits_to_float(uint16_t h) {
  const uint32_t sign = static_cast<uint32_t>(h & 0x8000u) << 16;
  const uint32_t exp = (h >> 10) & 0x1fu;
  uint32_t man = h & 0x3ffu;
  if (exp == 0x1fu) return bits_to_float(sign | 0x7f800000u | (man << 13));  // inf / nan
  if (exp != 0) return bits_to_float(sign | ((exp + 112u) << 23) | (man << 13));
  if (man == 0) return bits_to_float(sign);  // +-0
  // subnormal: value = man * 2^-24
  int e = -1;
  do {
    man <<= 1;
    ++e;
  } while ((man & 0x400u) == 0);
  return bits_to_float(sign | ((112u - static_cast<uint32_t>(e)) << 23) | ((man & 0x3ffu) << 13));
}

MIREDUCE_HD uint16_t float_to_f16_bits(float f) {
  const uint32_t u = float_to_bits(f);
  const uint16_t sign = static_cast<uint16_t>((u >> 16) & 0x8000u);
  const uint32_t a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return static_cast<uint16_t>(sign | 0x7e00u | ((a >> 13) & 0x3ffu));  // quiet NaN
  if (a >= 0x477ff000u) return static_cast<uint16_t>(sign | 0x7c00u);  // rounds to >= 65520: inf
  if (a >= 0x38800000u) {  // normal half (>= 2^-14)
    const uint32_t rounding = 0xfffu + ((a >> 13) & 1u);
    return static_cast<uint16_t>(sign | ((a - 0x38000000u + rounding) >> 13));
  }
  if (a < 0x33000000u) return sign;  // < 2^-25: rounds to zero
  // subnormal half: shift the 24-bit significand right, round to nearest even
  const uint32_t e = a >> 23;
  const uint32_t m = (a & 0x7fffffu) | 0x800000u;
  const uint32_t shift = 126u - e;  // 14..24 (value = m * 2^(e-150), half ulp = 2^-24)
  const uint32_t q = m >> shift, rem = m & ((1u << shift) - 1u), half = 1u << (shift - 1u);
  return static_cast<uint16_t>(sign | (q + ((rem > half || (rem == half && (q & 1u))) ? 1u : 0u)));
}

struct bf16_t {
  uint16_t bits;
  MIREDUCE_HD static bf16_t from_float(float f) { return bf16_t{float_to_bf16_bits(f)}; }
  MIREDUCE_HD explicit operator float() const { return bf16_bits_to_float(bits); }
  MIREDUCE_HD explicit operator double() const { return bf16_bits_to_float(bits); }
};

struct f16_t {
  uint16_t bits;
  MIREDUCE_HD static f16_t from_float(float f) { return f16_t{float_to_f16_bits(f)}; }
  MIREDUCE_HD explicit operator float() const { return f16_bits_to_float(bits); }
  MIREDUCE_HD explicit operator double() const { return f16_bits_to_float(bits); }
};

template <class T> struct is_half16 { static constexpr bool value = false; };
template <> struct is_half16<bf16_t> { static constexpr bool value = true; };
template <> struct is_half16<f16_t> { static constexpr bool value = true; };
template <class T> inline constexpr bool is_half16_v = is_half16<T>::value;

// Significand bits (incl. the implicit one): uniform fills use exactly this many random bits so
// every generated value is representable.
template <class T> struct half_precision;
template <> struct half_precision<bf16_t> { static constexpr int value = 8; };
template <> struct half_precision<f16_t> { static constexpr int value = 11; };

}  // namespace mireduce
