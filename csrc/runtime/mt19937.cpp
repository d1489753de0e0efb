// MT19937 implementation (see mt19937.hpp; parity target mpi/externalfunctions.h:60-174).
#include "mireduce/mt19937.hpp"

namespace mireduce {

namespace {
constexpr uint32_t kMatrixA = 0x9908b0dfu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7fffffffu;
inline uint32_t twist(uint32_t a, uint32_t b) {
  const uint32_t y = (a & kUpper) | (b & kLower);
  return (y >> 1) ^ ((y & 1u) ? kMatrixA : 0u);
}
}  // namespace

void Mt19937::init_genrand(uint32_t seed) {
  mt_[0] = seed;
  for (int i = 1; i < kN; ++i) mt_[i] = 1812433253u * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + static_cast<uint32_t>(i);
  mti_ = kN;
}

void Mt19937::init_by_array(const uint64_t* key, size_t len) {
  init_genrand(19650218u);
  int i = 1;
  size_t j = 0;
  for (size_t k = (static_cast<size_t>(kN) > len ? kN : len); k > 0; --k) {
    mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1664525u)) + static_cast<uint32_t>(key[j]) +
             static_cast<uint32_t>(j);
    ++i;
    ++j;
    if (i >= kN) { mt_[0] = mt_[kN - 1]; i = 1; }
    if (j >= len) j = 0;
  }
  for (int k = kN - 1; k > 0; --k) {
    mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1566083941u)) - static_cast<uint32_t>(i);
    ++i;
    if (i >= kN) { mt_[0] = mt_[kN - 1]; i = 1; }
  }
  mt_[0] = 0x80000000u;
  mti_ = kN;
}

void Mt19937::refill() {
  int k = 0;
  for (; k < kN - kM; ++k) mt_[k] = mt_[k + kM] ^ twist(mt_[k], mt_[k + 1]);
  for (; k < kN - 1; ++k) mt_[k] = mt_[k + (kM - kN)] ^ twist(mt_[k], mt_[k + 1]);
  mt_[kN - 1] = mt_[kM - 1] ^ twist(mt_[kN - 1], mt_[0]);
  mti_ = 0;
}

uint32_t Mt19937::genrand_int32() {
  if (mti_ >= kN) {
    if (mti_ == kN + 1) init_genrand(5489u);
    refill();
  }
  uint32_t y = mt_[mti_++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

double Mt19937::genrand_res53() {
  const uint32_t a = genrand_int32() >> 5;
  const uint32_t b = genrand_int32() >> 6;
  return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

}  // namespace mireduce
