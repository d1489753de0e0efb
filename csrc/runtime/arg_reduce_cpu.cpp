// Host reference of the arg-reductions (arg_reduce.hpp): first index of the max / min per row,
// NaN the extreme (first NaN wins), -0.0 == +0.0. Rows are split over threads; a single long row
// (the whole-array case) is split into column chunks whose (value, index) winners fold in order.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <type_traits>
#include <vector>

#include "mireduce/arg_reduce.hpp"
#include "mireduce/check.hpp"
#include "mireduce/half.hpp"

namespace mireduce {
namespace {

template <class T> struct HostKey { using type = T; };
template <> struct HostKey<bf16_t> { using type = float; };
template <> struct HostKey<f16_t> { using type = float; };

template <class T, class K>
K key_of(const T& x) {
  if constexpr (is_half16_v<T>) return static_cast<float>(x);
  else return x;
}

// a strictly beats b (NaN beats numbers; a NaN b is never beaten)
template <bool MAX, class K>
bool beats(K a, K b) {
  if constexpr (std::is_floating_point_v<K>) {
    if (std::isnan(b)) return false;
    if (std::isnan(a)) return true;
  }
  return MAX ? a > b : a < b;
}

template <bool MAX, class T>
size_t first_best(const T* p, size_t b, size_t e) {  // first index of the extreme over [b, e)
  using K = typename HostKey<T>::type;
  size_t bi = b;
  K bv = key_of<T, K>(p[b]);
  for (size_t c = b + 1; c < e; ++c) {
    const K x = key_of<T, K>(p[c]);
    if (beats<MAX, K>(x, bv)) {
      bv = x;
      bi = c;
    }
  }
  return bi;
}

template <bool MAX, class T>
size_t row_argbest(const T* p, size_t cols, int threads) {
  using K = typename HostKey<T>::type;
  if (threads <= 1 || cols < (size_t{1} << 22)) return first_best<MAX, T>(p, 0, cols);
  std::vector<size_t> win(threads);
  std::vector<std::thread> pool;
  const size_t chunk = (cols + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const size_t b = std::min(cols, t * chunk), e = std::min(cols, b + chunk);
    pool.emplace_back([&, t, b, e] { win[t] = b < e ? first_best<MAX, T>(p, b, e) : cols; });
  }
  for (auto& th : pool) th.join();
  size_t bi = win[0];
  for (int t = 1; t < threads; ++t)  // chunks in order: only a strict improvement moves the index
    if (win[t] < cols && beats<MAX, K>(key_of<T, K>(p[win[t]]), key_of<T, K>(p[bi]))) bi = win[t];
  return bi;
}

template <bool MAX, class T>
void arg_rows(const T* in, size_t rows, size_t cols, T* out_value, int64_t* out_index) {
  unsigned hc = std::thread::hardware_concurrency();
  const int threads = static_cast<int>(std::max(1u, std::min(hc ? hc : 1u, 32u)));
  auto one = [&](size_t r, int th) {
    const size_t c = row_argbest<MAX, T>(in + r * cols, cols, th);
    out_index[r] = static_cast<int64_t>(c);
    out_value[r] = in[r * cols + c];
  };
  if (rows == 1 || threads == 1) {
    for (size_t r = 0; r < rows; ++r) one(r, threads);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (size_t r = t; r < rows; r += threads) one(r, 1);
    });
  for (auto& th : pool) th.join();
}

template <bool MAX>
void arg_dispatch(const void* in, size_t rows, size_t cols, DType t, void* ov, int64_t* oi) {
  switch (t) {
    case DType::Int32: arg_rows<MAX>(static_cast<const int32_t*>(in), rows, cols, static_cast<int32_t*>(ov), oi); break;
    case DType::Int64: arg_rows<MAX>(static_cast<const int64_t*>(in), rows, cols, static_cast<int64_t*>(ov), oi); break;
    case DType::Float32: arg_rows<MAX>(static_cast<const float*>(in), rows, cols, static_cast<float*>(ov), oi); break;
    case DType::Float64: arg_rows<MAX>(static_cast<const double*>(in), rows, cols, static_cast<double*>(ov), oi); break;
    case DType::BFloat16: arg_rows<MAX>(static_cast<const bf16_t*>(in), rows, cols, static_cast<bf16_t*>(ov), oi); break;
    case DType::Float16: arg_rows<MAX>(static_cast<const f16_t*>(in), rows, cols, static_cast<f16_t*>(ov), oi); break;
  }
}

}  // namespace

void cpu_arg_reduce_rows(const void* in, size_t rows, size_t cols, DType t, Op op, void* out_value,
                         int64_t* out_index) {
  MIREDUCE_REQUIRE(op == Op::Max || op == Op::Min, "arg_reduce: the operator must be MAX or MIN");
  MIREDUCE_REQUIRE(cols >= 1, "arg_reduce: rows must have at least one element");
  if (op == Op::Max) arg_dispatch<true>(in, rows, cols, t, out_value, out_index);
  else arg_dispatch<false>(in, rows, cols, t, out_value, out_index);
}

}  // namespace mireduce
