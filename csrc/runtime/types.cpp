// Parsing of dtype / op names (reduction.cpp:93-109 case-insensitive --type; reduction.cpp:165-199
// case-sensitive --method). Host-only, no HIP dependency (linked into the CPU MPI app too).
#include <strings.h>

#include <string>

#include "mireduce/types.hpp"

namespace mireduce {

bool parse_dtype(const std::string& s, DType* out) {
  const char* c = s.c_str();
  if (!strcasecmp(c, "int") || !strcasecmp(c, "int32") || !strcasecmp(c, "i32")) { *out = DType::Int32; return true; }
  if (!strcasecmp(c, "int64") || !strcasecmp(c, "long") || !strcasecmp(c, "i64")) { *out = DType::Int64; return true; }
  if (!strcasecmp(c, "float") || !strcasecmp(c, "float32") || !strcasecmp(c, "fp32") || !strcasecmp(c, "f32")) { *out = DType::Float32; return true; }
  if (!strcasecmp(c, "double") || !strcasecmp(c, "float64") || !strcasecmp(c, "fp64") || !strcasecmp(c, "f64")) { *out = DType::Float64; return true; }
  if (!strcasecmp(c, "bf16") || !strcasecmp(c, "bfloat16")) { *out = DType::BFloat16; return true; }
  if (!strcasecmp(c, "half") || !strcasecmp(c, "float16") || !strcasecmp(c, "fp16") || !strcasecmp(c, "f16")) { *out = DType::Float16; return true; }
  return false;
}

bool parse_op_strict(const std::string& s, Op* out) {
  if (s == "SUM") { *out = Op::Sum; return true; }
  if (s == "MIN") { *out = Op::Min; return true; }
  if (s == "MAX") { *out = Op::Max; return true; }
  if (s == "SUMSQ") { *out = Op::SumSq; return true; }
  if (s == "AMAX") { *out = Op::AbsMax; return true; }
  return false;
}

bool parse_op(const std::string& s, Op* out) {
  const char* c = s.c_str();
  if (!strcasecmp(c, "sum")) { *out = Op::Sum; return true; }
  if (!strcasecmp(c, "min")) { *out = Op::Min; return true; }
  if (!strcasecmp(c, "max")) { *out = Op::Max; return true; }
  if (!strcasecmp(c, "sumsq")) { *out = Op::SumSq; return true; }
  if (!strcasecmp(c, "amax") || !strcasecmp(c, "absmax")) { *out = Op::AbsMax; return true; }
  return false;
}

}  // namespace mireduce
