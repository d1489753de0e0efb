// Counter-based synthetic data generation, bit-identical on host and device.
//
// The reference fills its inputs on the host: rand()&0xFF in the CUDA sample
// (cuda/C/src/reduction/reduction.cpp:698-705) and MT19937 genrand_int32 / genrand_res53 in the
// MPI benchmark (mpi/reduce.c:51-57). A host generator cannot fill 288 GB of HBM in reasonable
// time, so element i here is a pure function of (seed, global index i):
// any rank, any GPU count, any chunking produces the same logical array, and the host can
// recompute any element to verify a device result.
#pragma once

#include <cstdint>

#include "mireduce/half.hpp"
#include "mireduce/ops.hpp"
#include "mireduce/types.hpp"

namespace mireduce {

enum class Pattern : int {
  Uniform = 0,    // floats: U[0,1) (53/24 random mantissa bits); ints: full-range random bits
  SmallInt = 1,   // reference CUDA sample data: (r & 0xFF) for ints, (r & 0xFF)/RAND_MAX for floats
  FullRange = 2,  // reduce.c data: int32 = (int)genrand_int32-like bits, doubles = U[0,1)
  IotaMod = 3,    // x[i] = i mod 1024 — closed-form sum/min/max for huge-array checks
  Constant = 4,   // x[i] = value
};

constexpr double kRandMax = 2147483647.0;  // glibc RAND_MAX, reduction.cpp:702

MIREDUCE_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Random 64 bits for global element index `i` of stream `seed`.
MIREDUCE_HD uint64_t element_bits(uint64_t seed, uint64_t i) {
  return splitmix64(i ^ splitmix64(seed));
}

template <class T>
MIREDUCE_HD T pattern_value(Pattern p, uint64_t seed, uint64_t i, double value) {
  switch (p) {
    case Pattern::Constant: return static_cast<T>(value);
    case Pattern::IotaMod: return static_cast<T>(i & 1023u);
    default: break;
  }
  const uint64_t h = element_bits(seed, i);
  if constexpr (std::is_floating_point_v<T>) {
    if (p == Pattern::SmallInt) return static_cast<T>(static_cast<double>(h & 0xFFu) / kRandMax);
    if constexpr (sizeof(T) == 8) return static_cast<T>((h >> 11) * 0x1.0p-53);
    else return static_cast<T>((h >> 40) * 0x1.0p-24f);
  } else {
    if (p == Pattern::SmallInt) return static_cast<T>(h & 0xFFu);
    if constexpr (sizeof(T) == 8) return static_cast<T>(h);
    else return static_cast<T>(static_cast<uint32_t>(h >> 32));
  }
}

// 16-bit floats (half.hpp): the value is produced in fp32 and rounded to nearest even; the uniform
// patterns draw exactly as many random bits as the type's significand holds, so U[0,1) values are
// exact and never round up to 1.0.
template <class H>
MIREDUCE_HD uint16_t pattern_half_bits(Pattern p, uint64_t seed, uint64_t i, double value) {
  float f;
  switch (p) {
    case Pattern::Constant: f = static_cast<float>(value); break;
    case Pattern::IotaMod: f = static_cast<float>(i & 1023u); break;
    default: {
      const uint64_t h = element_bits(seed, i);
      constexpr int P = half_precision<H>::value;
      if (p == Pattern::SmallInt) f = static_cast<float>(static_cast<double>(h & 0xFFu) / kRandMax);
      else f = static_cast<float>(h >> (64 - P)) * (1.0f / static_cast<float>(1u << P));
      break;
    }
  }
  return H::from_float(f).bits;
}

struct FillSpec {
  Pattern pattern = Pattern::Uniform;
  uint64_t seed = 0x5EED;
  uint64_t offset = 0;  // global index of element 0 (rank shard offset)
  double value = 0.0;   // Pattern::Constant
};

}  // namespace mireduce
