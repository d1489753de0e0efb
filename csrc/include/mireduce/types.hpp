// mireduce — MI355X-native parallel reduction framework.
//
// Element types and reduction operators shared by host and device code.
//
// Reference parity: the reference supports {int, float, double} x {SUM, MIN, MAX} on one GPU
// (cuda/C/src/reduction/reduction_kernel.cu:527-564) and {MPI_INT, MPI_DOUBLE} x
// {MPI_MAX, MPI_MIN, MPI_SUM} across ranks (mpi/reduce.c:21-28). We add int64 (BASELINE config 3)
// and make the accumulator type explicit so that int32 SUM does not silently wrap
// (SURVEY.md §8 B7/B11). bfloat16 / half (half.hpp) are MI355X additions: read at 16 bytes per
// lane like every other type, accumulated in fp32.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace mireduce {

enum class DType : int { Int32 = 0, Int64 = 1, Float32 = 2, Float64 = 3, BFloat16 = 4, Float16 = 5 };
enum class Op : int { Sum = 0, Min = 1, Max = 2, SumSq = 3, AbsMax = 4 };

constexpr int kNumDTypes = 6;
constexpr int kNumOps = 5;

inline size_t dtype_size(DType t) {
  switch (t) {
    case DType::Int32: return 4;
    case DType::Int64: return 8;
    case DType::Float32: return 4;
    case DType::Float64: return 8;
    case DType::BFloat16: return 2;
    case DType::Float16: return 2;
  }
  return 0;
}

inline bool dtype_is_half(DType t) { return t == DType::BFloat16 || t == DType::Float16; }
inline bool dtype_is_float(DType t) { return t == DType::Float32 || t == DType::Float64 || dtype_is_half(t); }

// Names as they appear in the reference's GNUPlot lines ("INT", "DOUBLE"; mpi/reduce.c:81,95)
// plus the two new element types.
inline const char* dtype_gnuplot_name(DType t) {
  switch (t) {
    case DType::Int32: return "INT";
    case DType::Int64: return "LONG";
    case DType::Float32: return "FLOAT";
    case DType::Float64: return "DOUBLE";
    case DType::BFloat16: return "BF16";
    case DType::Float16: return "HALF";
  }
  return "?";
}

// Lower-case names as accepted by `--type=` in the CUDA sample (reduction.cpp:96-109).
inline const char* dtype_cli_name(DType t) {
  switch (t) {
    case DType::Int32: return "int";
    case DType::Int64: return "int64";
    case DType::Float32: return "float";
    case DType::Float64: return "double";
    case DType::BFloat16: return "bf16";
    case DType::Float16: return "half";
  }
  return "?";
}

inline const char* op_name(Op o) {
  switch (o) {
    case Op::Sum: return "SUM";
    case Op::Min: return "MIN";
    case Op::Max: return "MAX";
    case Op::SumSq: return "SUMSQ";
    case Op::AbsMax: return "AMAX";
  }
  return "?";
}

// Case-insensitive dtype parser. Accepts the reference spellings and common aliases.
// Returns false when the string is not recognised.
bool parse_dtype(const std::string& s, DType* out);
// Case-SENSITIVE op parser ("SUM" | "MIN" | "MAX", plus the fused "SUMSQ" | "AMAX"), mirroring
// reduction.cpp:165-199's strcmp.
bool parse_op_strict(const std::string& s, Op* out);
// Case-insensitive op parser used by the new apps' list flags (`--ops=max,min,sum`).
bool parse_op(const std::string& s, Op* out);

// Default accumulator: widen int32 SUM to int64 and fp32 SUM to fp64; MIN/MAX keep the
// element type (they cannot overflow or lose precision). The 16-bit float types always
// accumulate (and return) fp32: every 16-bit value is exact in fp32.
// The fused ops (SUMSQ, AMAX) are for floating types; SUMSQ accumulates like SUM.
inline bool op_is_fused(Op o) { return o == Op::SumSq || o == Op::AbsMax; }

inline DType default_acc(DType t, Op o) {
  if (dtype_is_half(t)) return DType::Float32;
  if (o == Op::SumSq) o = Op::Sum;
  if (o != Op::Sum) return t;
  if (t == DType::Int32) return DType::Int64;
  if (t == DType::Float32) return DType::Float64;
  return t;
}

// Accumulator types we instantiate: same as input, or the widened type for SUM.
inline bool acc_supported(DType t, Op o, DType acc) {
  if (op_is_fused(o) && !dtype_is_float(t)) return false;
  if (o == Op::SumSq) o = Op::Sum;
  if (dtype_is_half(t)) return acc == DType::Float32;
  if (acc == t) return true;
  if (o != Op::Sum) return false;
  return (t == DType::Int32 && acc == DType::Int64) || (t == DType::Float32 && acc == DType::Float64);
}

}  // namespace mireduce
