// Host reference reducers; see cpu_reference.hpp.
#include "mireduce/cpu_reference.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <type_traits>
#include <vector>

#include "mireduce/check.hpp"
#include "mireduce/half.hpp"
#include "mireduce/ops.hpp"

namespace mireduce {

namespace {

// Neumaier-compensated accumulator (Kahan variant that also handles |x| > |sum|).
template <class A>
struct Compensated {
  A sum = 0, c = 0;
  void add(A x) {
    const A t = sum + x;
    if (std::fabs(sum) >= std::fabs(x)) c += (sum - t) + x;
    else c += (x - t) + sum;
    sum = t;
  }
  A value() const { return sum + c; }
};

// Floating sums are compensated in fp64 whatever the accumulator type (per-thread partials stay
// fp64 too) and rounded to it once at the end: a float-typed Neumaier sum saturates once its
// compensation term stops absorbing the addends (4e9 bf16 values of ~6e-8 summed to 64.0 instead
// of 237.5). W is the working type of a range: fp64 for floating sums, the accumulator otherwise.
// The fused ops transform each element once (OpT::pre) and combine like SUM (SUMSQ) or MAX (AMAX);
// partial results are folded with the combining op only.
template <class OpT>
using Combine = std::conditional_t<std::is_same_v<OpT, SumSqOp>, SumOp,
                                   std::conditional_t<std::is_same_v<OpT, AbsMaxOp>, MaxOp, OpT>>;

template <class OpT>
inline constexpr bool kIsSum = std::is_same_v<Combine<OpT>, SumOp>;

template <class OpT, class A>
using Work = std::conditional_t<kIsSum<OpT> && std::is_floating_point_v<A>, double, A>;

template <class OpT, class T, class A>
Work<OpT, A> reduce_range(const T* p, size_t n) {
  if constexpr (kIsSum<OpT> && std::is_floating_point_v<A>) {
    Compensated<double> k;  // squares (SUMSQ) are taken in fp64 here: the exact reference
    for (size_t i = 0; i < n; ++i) k.add(OpT::pre(static_cast<double>(static_cast<A>(p[i]))));
    return k.value();
  } else {
    A a = OpT::template identity<A>();
    for (size_t i = 0; i < n; ++i) a = OpT::apply(a, OpT::pre(static_cast<A>(p[i])));
    return a;
  }
}

int pick_threads(size_t n, int threads) {
  if (threads > 0) return threads;
  if (n < (1u << 22)) return 1;
  unsigned hc = std::thread::hardware_concurrency();
  if (hc == 0) hc = 1;
  return static_cast<int>(std::min<unsigned>(hc, 16));
}

template <class OpT, class T, class A>
A reduce_parallel(const T* p, size_t n, int threads) {
  using W = Work<OpT, A>;
  threads = pick_threads(n, threads);
  if (threads <= 1) return static_cast<A>(reduce_range<OpT, T, A>(p, n));
  std::vector<W> part(threads);
  std::vector<std::thread> pool;
  const size_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t] {
      const size_t b = std::min(n, t * chunk), e = std::min(n, b + chunk);
      part[t] = reduce_range<OpT, T, A>(p + b, e - b);
    });
  }
  for (auto& th : pool) th.join();
  return static_cast<A>(reduce_range<Combine<OpT>, W, W>(part.data(), part.size()));
}

template <class OpT, class T>
void dispatch_acc(const void* in, size_t n, DType acc, void* out, int threads) {
  const T* p = static_cast<const T*>(in);
  if constexpr (is_half16_v<T>) {  // 16-bit floats accumulate in fp32 only (acc_supported)
    float r = reduce_parallel<OpT, T, float>(p, n, threads);
    std::memcpy(out, &r, 4);
  } else {
    switch (acc) {
      case DType::Int32: { int32_t r = reduce_parallel<OpT, T, int32_t>(p, n, threads); std::memcpy(out, &r, 4); break; }
      case DType::Int64: { int64_t r = reduce_parallel<OpT, T, int64_t>(p, n, threads); std::memcpy(out, &r, 8); break; }
      case DType::Float32: { float r = reduce_parallel<OpT, T, float>(p, n, threads); std::memcpy(out, &r, 4); break; }
      case DType::Float64: { double r = reduce_parallel<OpT, T, double>(p, n, threads); std::memcpy(out, &r, 8); break; }
      default: MIREDUCE_REQUIRE(false, "accumulator must be int32, int64, float32 or float64");
    }
  }
}

template <class OpT>
void dispatch_t(const void* in, size_t n, DType t, DType acc, void* out, int threads) {
  switch (t) {
    case DType::Int32: dispatch_acc<OpT, int32_t>(in, n, acc, out, threads); break;
    case DType::Int64: dispatch_acc<OpT, int64_t>(in, n, acc, out, threads); break;
    case DType::Float32: dispatch_acc<OpT, float>(in, n, acc, out, threads); break;
    case DType::Float64: dispatch_acc<OpT, double>(in, n, acc, out, threads); break;
    case DType::BFloat16: dispatch_acc<OpT, bf16_t>(in, n, acc, out, threads); break;
    case DType::Float16: dispatch_acc<OpT, f16_t>(in, n, acc, out, threads); break;
  }
}

}  // namespace

void cpu_reduce(const void* in, size_t n, DType t, Op op, DType acc, void* out, int threads) {
  MIREDUCE_REQUIRE(acc_supported(t, op, acc), "unsupported (dtype, op, accumulator) combination");
  switch (op) {
    case Op::Sum: dispatch_t<SumOp>(in, n, t, acc, out, threads); break;
    case Op::Min: dispatch_t<MinOp>(in, n, t, acc, out, threads); break;
    case Op::Max: dispatch_t<MaxOp>(in, n, t, acc, out, threads); break;
    case Op::SumSq: dispatch_t<SumSqOp>(in, n, t, acc, out, threads); break;
    case Op::AbsMax: dispatch_t<AbsMaxOp>(in, n, t, acc, out, threads); break;
  }
}

namespace {
template <class T>
double abs_sum_range(const T* p, size_t n) {
  Compensated<double> k;
  for (size_t i = 0; i < n; ++i) k.add(std::fabs(static_cast<double>(p[i])));
  return k.value();
}
template <class T>
double abs_sum_t(const void* in, size_t n, int threads) {
  const T* p = static_cast<const T*>(in);
  threads = pick_threads(n, threads);
  if (threads <= 1) return abs_sum_range(p, n);
  std::vector<double> part(threads);
  std::vector<std::thread> pool;
  const size_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      const size_t b = std::min(n, t * chunk), e = std::min(n, b + chunk);
      part[t] = abs_sum_range(p + b, e - b);
    });
  for (auto& th : pool) th.join();
  return abs_sum_range(part.data(), part.size());
}
}  // namespace

double cpu_abs_sum(const void* in, size_t n, DType t, int threads) {
  switch (t) {
    case DType::Int32: return abs_sum_t<int32_t>(in, n, threads);
    case DType::Int64: return abs_sum_t<int64_t>(in, n, threads);
    case DType::Float32: return abs_sum_t<float>(in, n, threads);
    case DType::Float64: return abs_sum_t<double>(in, n, threads);
    case DType::BFloat16: return abs_sum_t<bf16_t>(in, n, threads);
    case DType::Float16: return abs_sum_t<f16_t>(in, n, threads);
  }
  return 0.0;
}

void cpu_fold(const void* partials, size_t count, DType acc, Op op, void* out) {
  // partials of the fused ops are already transformed: fold them with the combining op
  const Op combine = op == Op::SumSq ? Op::Sum : (op == Op::AbsMax ? Op::Max : op);
  cpu_reduce(partials, count, acc, combine, acc, out, 1);
}

double sum_tolerance(DType t, DType acc, size_t n, double abs_sum) {
  if (!dtype_is_float(acc)) return 0.0;
  // Device summation is blocked: per-lane sequential runs plus a log-depth tree. A generous
  // bound: (per-lane run + tree depth + margin) * eps(acc) * Σ|x|, floored at the reference's
  // absolute thresholds (1e-12 for double, reduction.cpp:760; 1e-8*n for float, :765).
  const double eps = (acc == DType::Float64) ? 1.1102230246251565e-16 : 5.960464477539063e-8;
  const double depth = std::log2(static_cast<double>(n) + 2.0);
  double tol = (4096.0 + 4.0 * depth) * eps * abs_sum;
  const double floor_abs = (t == DType::Float32 && acc == DType::Float32) ? 1e-8 * static_cast<double>(n) : 1e-12;
  return std::max(tol, floor_abs);
}

double acc_as_double(const void* p, DType acc) {
  switch (acc) {
    case DType::Int32: { int32_t v; std::memcpy(&v, p, 4); return v; }
    case DType::Int64: { int64_t v; std::memcpy(&v, p, 8); return static_cast<double>(v); }
    case DType::Float32: { float v; std::memcpy(&v, p, 4); return v; }
    case DType::Float64: { double v; std::memcpy(&v, p, 8); return v; }
    case DType::BFloat16: { bf16_t v; std::memcpy(&v, p, 2); return static_cast<float>(v); }
    case DType::Float16: { f16_t v; std::memcpy(&v, p, 2); return static_cast<float>(v); }
  }
  return 0.0;
}

int64_t acc_as_int64(const void* p, DType acc) {
  switch (acc) {
    case DType::Int32: { int32_t v; std::memcpy(&v, p, 4); return v; }
    case DType::Int64: { int64_t v; std::memcpy(&v, p, 8); return v; }
    case DType::Float32: { float v; std::memcpy(&v, p, 4); return static_cast<int64_t>(v); }
    case DType::Float64: { double v; std::memcpy(&v, p, 8); return static_cast<int64_t>(v); }
    case DType::BFloat16:
    case DType::Float16: return static_cast<int64_t>(acc_as_double(p, acc));
  }
  return 0;
}

bool analytic_iotamod(uint64_t n, uint64_t offset, DType t, Op op, DType acc, void* out) {
  if (dtype_is_half(t)) return false;
  // Σ and Σ² over one index range [a, b) of the 1024-periodic pattern, as exact integers
  // (n < 2^64 elements: Σ x <= 1023 n and Σ x² <= 1023² n fit in unsigned __int128).
  using U = unsigned __int128;
  auto prefix = [](uint64_t m, int pw) -> U {  // Σ_{k<m} (k mod 1024)^pw
    const uint64_t c = m / 1024, r = m % 1024;
    U full = 0, part = 0;
    for (uint64_t k = 0; k < 1024; ++k) {
      const U v = pw == 1 ? U(k) : U(k) * k;
      full += v;
      if (k < r) part += v;
    }
    return full * c + part;
  };
  const U s1 = prefix(offset + n, 1) - prefix(offset, 1);
  const U s2 = prefix(offset + n, 2) - prefix(offset, 2);
  uint64_t mn = 1023, mx = 0;
  if (n >= 1024) {
    mn = 0;
    mx = 1023;
  } else {
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t v = (offset + i) & 1023u;
      mn = std::min(mn, v);
      mx = std::max(mx, v);
    }
  }
  long double v = 0;
  uint64_t iv = 0;
  switch (op) {
    case Op::Sum: v = static_cast<long double>(s1); iv = static_cast<uint64_t>(s1); break;
    case Op::SumSq: v = static_cast<long double>(s2); iv = static_cast<uint64_t>(s2); break;
    case Op::Min: v = mn; iv = mn; break;
    case Op::Max:
    case Op::AbsMax: v = mx; iv = mx; break;
  }
  switch (acc) {
    case DType::Int32: { const int32_t x = static_cast<int32_t>(static_cast<uint32_t>(iv)); std::memcpy(out, &x, 4); break; }
    case DType::Int64: { const int64_t x = static_cast<int64_t>(iv); std::memcpy(out, &x, 8); break; }
    case DType::Float32: { const float x = static_cast<float>(v); std::memcpy(out, &x, 4); break; }
    case DType::Float64: { const double x = static_cast<double>(v); std::memcpy(out, &x, 8); break; }
    default: return false;
  }
  return true;
}

}  // namespace mireduce
