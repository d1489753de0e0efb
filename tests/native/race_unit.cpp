// Race detection for the host code that runs threads: the multi-threaded CPU
// reference reducers and arg-reductions (csrc/runtime/cpu_reference.cpp, arg_reduce_cpu.cpp) —
// the oracles every GPU result is checked against — built with ThreadSanitizer (`make tsan`).
// Each threaded call is compared with the single-threaded result of the same input: integers
// exactly, floating sums within the association tolerance, MIN/MAX and arg-reductions exactly.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "mireduce/arg_reduce.hpp"
#include "mireduce/cpu_reference.hpp"
#include "mireduce/half.hpp"
#include "mireduce/types.hpp"

using namespace mireduce;

static int g_fail = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

// xorshift64*: deterministic, no shared state between threads
static uint64_t next(uint64_t& s) {
  s ^= s >> 12;
  s ^= s << 25;
  s ^= s >> 27;
  return s * 2685821657736338717ull;
}

static std::vector<unsigned char> make(DType t, size_t n, uint64_t seed) {
  std::vector<unsigned char> b(n * dtype_size(t));
  uint64_t s = seed | 1;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t r = next(s);
    const double u = static_cast<double>(r >> 11) * 0x1.0p-53 - 0.5;
    switch (t) {
      case DType::Int32: { int32_t v = static_cast<int32_t>(r); std::memcpy(&b[i * 4], &v, 4); break; }
      case DType::Int64: { int64_t v = static_cast<int64_t>(r >> 8); std::memcpy(&b[i * 8], &v, 8); break; }
      case DType::Float32: { float v = static_cast<float>(u); std::memcpy(&b[i * 4], &v, 4); break; }
      case DType::Float64: { std::memcpy(&b[i * 8], &u, 8); break; }
      case DType::BFloat16: { bf16_t v = bf16_t::from_float(static_cast<float>(u)); std::memcpy(&b[i * 2], &v, 2); break; }
      case DType::Float16: { f16_t v = f16_t::from_float(static_cast<float>(u)); std::memcpy(&b[i * 2], &v, 2); break; }
    }
  }
  return b;
}

int main() {
  const DType types[] = {DType::Int32, DType::Int64, DType::Float32, DType::Float64, DType::BFloat16, DType::Float16};
  const Op ops[] = {Op::Sum, Op::Min, Op::Max, Op::SumSq, Op::AbsMax};
  const DType accs[] = {DType::Int32, DType::Int64, DType::Float32, DType::Float64};
  const size_t sizes[] = {1, 7, 1000, 100003};
  int combos = 0;
  for (DType t : types)
    for (size_t n : sizes) {
      const auto buf = make(t, n, 0x9e3779b97f4a7c15ull ^ n ^ static_cast<uint64_t>(t));
      for (Op op : ops)
        for (DType acc : accs) {
          if (!acc_supported(t, op, acc)) continue;
          unsigned char ref[8] = {}, got[8] = {};
          cpu_reduce(buf.data(), n, t, op, acc, ref, 1);
          for (int threads : {3, 7, 16}) {
            cpu_reduce(buf.data(), n, t, op, acc, got, threads);
            if (!dtype_is_float(acc) || op == Op::Min || op == Op::Max || op == Op::AbsMax) {
              CHECK(std::memcmp(ref, got, dtype_size(acc)) == 0);
            } else {
              const double a = acc_as_double(ref, acc), b = acc_as_double(got, acc);
              const double tol = sum_tolerance(t, acc, n, cpu_abs_sum(buf.data(), n, t, 5)) * (op == Op::SumSq ? 2 : 1);
              CHECK(std::fabs(a - b) <= tol + 1e-300);
            }
          }
          ++combos;
        }
      const double s1 = cpu_abs_sum(buf.data(), n, t, 1), s7 = cpu_abs_sum(buf.data(), n, t, 7);
      CHECK(std::fabs(s1 - s7) <= 1e-9 * (s1 + 1));
    }
  // arg-reductions: many rows (one thread per row stripe) and one long row (the row split over
  // threads, >= 2^22 columns), with the extreme planted twice so the FIRST index must win.
  for (DType t : {DType::Float32, DType::Int64, DType::BFloat16}) {
    for (size_t rows : {size_t{64}, size_t{1}}) {
      const size_t cols = rows == 1 ? (size_t{1} << 22) + 123 : 4099;
      auto buf = make(t, rows * cols, 77 + rows);
      const size_t es = dtype_size(t);
      unsigned char big[8] = {};
      switch (t) {
        case DType::Float32: { float v = 1e30f; std::memcpy(big, &v, 4); break; }
        case DType::Int64: { int64_t v = INT64_MAX; std::memcpy(big, &v, 8); break; }
        default: { bf16_t v = bf16_t::from_float(1e30f); std::memcpy(big, &v, 2); break; }
      }
      auto c0 = [&](size_t r) { return (r * 131 + cols / 3) % cols; };
      auto c1 = [&](size_t r) { return cols - 1 - (r % 5); };
      for (size_t r = 0; r < rows; ++r) {  // the maximum at two columns of every row
        std::memcpy(&buf[(r * cols + c0(r)) * es], big, es);
        std::memcpy(&buf[(r * cols + c1(r)) * es], big, es);
      }
      std::vector<unsigned char> val(rows * es);
      std::vector<int64_t> idx(rows, -1);
      cpu_arg_reduce_rows(buf.data(), rows, cols, t, Op::Max, val.data(), idx.data());
      for (size_t r = 0; r < rows; ++r) {
        CHECK(idx[r] == static_cast<int64_t>(c0(r) < c1(r) ? c0(r) : c1(r)));
        CHECK(std::memcmp(&val[r * es], big, es) == 0);
      }
    }
  }
  std::printf("race_unit: %d reduce combos, %s\n", combos, g_fail ? "FAILED" : "ok");
  return g_fail ? 1 : 0;
}
