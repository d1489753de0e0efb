// MT19937 (Matsumoto & Nishimura, 1998), as used by the reference MPI benchmark to fill its
// per-rank buffers (mpi/externalfunctions.h:45-179; seeding at mpi/reduce.c:38-41). Implemented
// from the published algorithm as a re-entrant class (the reference keeps global state) so that
// CPU-rank runs of apps/reduce_mpi reproduce reduce.c's data bit for bit.
#pragma once

#include <cstddef>
#include <cstdint>

namespace mireduce {

class Mt19937 {
 public:
  static constexpr int kN = 624;
  static constexpr int kM = 397;

  Mt19937() { init_genrand(5489u); }
  explicit Mt19937(uint32_t seed) { init_genrand(seed); }

  void init_genrand(uint32_t seed);
  // Keys are truncated to 32 bits, as the reference's `unsigned long` keys are masked.
  void init_by_array(const uint64_t* key, size_t len);

  uint32_t genrand_int32();
  int32_t genrand_int31() { return static_cast<int32_t>(genrand_int32() >> 1); }
  double genrand_real1() { return genrand_int32() * (1.0 / 4294967295.0); }  // [0,1]
  double genrand_real2() { return genrand_int32() * (1.0 / 4294967296.0); }  // [0,1)
  double genrand_real3() { return (static_cast<double>(genrand_int32()) + 0.5) * (1.0 / 4294967296.0); }  // (0,1)
  double genrand_res53();                                                   // [0,1), 53-bit

 private:
  void refill();
  uint32_t mt_[kN];
  int mti_ = kN + 1;
};

}  // namespace mireduce
