// reduce_mpi — CPU-rank MPI_Reduce benchmark with reduce.c's semantics and output.
//
// Reference: mpi/reduce.c:9-108 (+ constants.h:1-5, externalfunctions.h). What is kept:
//   * per-rank MT19937 seeded with {rank, 0x123, 0x234, 0x345, 0x456, 0x789} (reduce.c:38-41),
//     int32 data = (int)genrand_int32(), doubles = genrand_res53() (reduce.c:51-57);
//   * one warm-up SUM per dtype (reduce.c:61-64), RETRY_COUNT x {MAX, MIN, SUM} per dtype,
//     element-wise MPI_Reduce of the N/P shard to root 0 (reduce.c:71-99);
//   * output "# DATATYPE OP NODES GB/sec" + "%s %s %d %10.3lf" rows printed by rank 0, GB = 2^30
//     B of total data (reduce.c:67-69,79-82,93-96) — byte-compatible with getAvgs.sh/makePlots.gp.
// What is fixed / added: counts, dtypes, ops, retries, root and collective are
// runtime flags (defaults = constants.h); a barrier before each timed collective and the MAX
// over ranks as the time (B8; --timing=root restores reduce.c's root-only clock); a monotonic
// clock instead of rdtsc/CLOCK_RATE (B9); GB/s is computed from the bytes actually reduced,
// N/P*P, instead of N (B10); --verify checks the reduced vector at sampled indices (B11); int SUM keeps MPI_INT's
// wrap-around semantics (documented, checked modulo 2^32).
#include <mpi.h>

#include <algorithm>
#include <cinttypes>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <set>
#include <string>
#include <type_traits>
#include <vector>
#include <cmath>

#include "mireduce/version.hpp"
#include "mireduce/cli.hpp"
#include "mireduce/fault.hpp"
#include "mireduce/mt19937.hpp"
#include "mireduce/report.hpp"
#include "mireduce/timer.hpp"
#include "mireduce/types.hpp"

using namespace mireduce;

namespace {

constexpr uint64_t kNumInts = 512ull * 1024 * 1024;     // constants.h:1
constexpr uint64_t kNumDoubles = 256ull * 1024 * 1024;  // constants.h:2
constexpr int kRetryCount = 5;                          // constants.h:5

#define MPI_CHECK(call)                                                                   \
  do {                                                                                    \
    int e_ = (call);                                                                      \
    if (e_ != MPI_SUCCESS) {                                                              \
      char s_[MPI_MAX_ERROR_STRING];                                                      \
      int l_ = 0;                                                                         \
      MPI_Error_string(e_, s_, &l_);                                                      \
      std::fprintf(stderr, "%s(%d) : MPI error : %s : %s\n", __FILE__, __LINE__, #call, s_); \
      MPI_Abort(MPI_COMM_WORLD, 1);                                                       \
    }                                                                                     \
  } while (0)

MPI_Datatype mpi_type(DType t) {
  switch (t) {
    case DType::Int32: return MPI_INT;
    case DType::Int64: return MPI_LONG_LONG;
    case DType::Float32: return MPI_FLOAT;
    case DType::Float64: return MPI_DOUBLE;
    default: break;
  }
  return MPI_DATATYPE_NULL;
}

MPI_Op mpi_op(Op o) {
  switch (o) {
    case Op::Sum: return MPI_SUM;
    case Op::Min: return MPI_MIN;
    case Op::Max: return MPI_MAX;
    default: break;
  }
  return MPI_OP_NULL;
}

// reduce.c's generator per dtype (int32: genrand_int32 wrapped into int; fp: genrand_res53).
void generate(Mt19937& g, DType t, void* buf, uint64_t n) {
  switch (t) {
    case DType::Int32: { auto* p = static_cast<int32_t*>(buf); for (uint64_t i = 0; i < n; ++i) p[i] = static_cast<int32_t>(g.genrand_int32()); break; }
    case DType::Int64: { auto* p = static_cast<int64_t*>(buf); for (uint64_t i = 0; i < n; ++i) { uint64_t hi = g.genrand_int32(); p[i] = static_cast<int64_t>((hi << 32) | g.genrand_int32()); } break; }
    case DType::Float32: { auto* p = static_cast<float*>(buf); for (uint64_t i = 0; i < n; ++i) p[i] = static_cast<float>(g.genrand_res53()); break; }
    case DType::Float64: { auto* p = static_cast<double*>(buf); for (uint64_t i = 0; i < n; ++i) p[i] = g.genrand_res53(); break; }
    default: break;
  }
}

template <class T>
T combine(Op o, T a, T b) {
  if (o == Op::Sum) {
    if constexpr (std::is_integral_v<T>) {
      using U = std::make_unsigned_t<T>;
      return static_cast<T>(static_cast<U>(a) + static_cast<U>(b));
    } else {
      return a + b;
    }
  }
  if (o == Op::Min) return b < a ? b : a;
  return a < b ? b : a;
}

// Root gathers every rank's sample values and checks the reduced vector at those indices.
template <class T>
bool verify_samples(Op o, const T* send, const T* recv, uint64_t count, int rank, int size, int root,
                    MPI_Datatype dt) {
  const int kSamples = 16;
  std::vector<uint64_t> idx(kSamples);
  for (int s = 0; s < kSamples; ++s) idx[s] = count ? (static_cast<uint64_t>(s) * 2654435761ull) % count : 0;
  std::vector<T> mine(kSamples), all(static_cast<size_t>(kSamples) * size);
  for (int s = 0; s < kSamples; ++s) mine[s] = count ? send[idx[s]] : T(0);
  MPI_CHECK(MPI_Gather(mine.data(), kSamples, dt, all.data(), kSamples, dt, root, MPI_COMM_WORLD));
  int ok = 1;
  if (rank == root && count) {
    for (int s = 0; s < kSamples; ++s) {
      T e = all[s];
      for (int r = 1; r < size; ++r) e = combine(o, e, all[static_cast<size_t>(r) * kSamples + s]);
      if constexpr (std::is_floating_point_v<T>) {
        const double tol = (o == Op::Sum) ? 1e-12 * size * (std::abs(static_cast<double>(e)) + 1.0) : 0.0;
        if (std::abs(static_cast<double>(e) - static_cast<double>(recv[idx[s]])) > tol) ok = 0;
      } else if (e != recv[idx[s]]) {
        ok = 0;
      }
    }
  }
  MPI_CHECK(MPI_Bcast(&ok, 1, MPI_INT, root, MPI_COMM_WORLD));
  return ok != 0;
}

bool verify(DType t, Op o, const void* send, const void* recv, uint64_t count, int rank, int size, int root) {
  switch (t) {
    case DType::Int32: return verify_samples(o, static_cast<const int32_t*>(send), static_cast<const int32_t*>(recv), count, rank, size, root, MPI_INT);
    case DType::Int64: return verify_samples(o, static_cast<const int64_t*>(send), static_cast<const int64_t*>(recv), count, rank, size, root, MPI_LONG_LONG);
    case DType::Float32: return verify_samples(o, static_cast<const float*>(send), static_cast<const float*>(recv), count, rank, size, root, MPI_FLOAT);
    case DType::Float64: return verify_samples(o, static_cast<const double*>(send), static_cast<const double*>(recv), count, rank, size, root, MPI_DOUBLE);
    default: break;
  }
  return false;
}

template <class T>
void corrupt_first_t(Op o, T* p) {
  if (o == Op::Sum) p[0] = static_cast<T>(p[0] + T(1));
  else p[0] = o == Op::Min ? std::numeric_limits<T>::lowest() : std::numeric_limits<T>::max();
}

void corrupt_first(DType t, Op o, void* p) {
  switch (t) {
    case DType::Int32: {  // wrap like MPI_INT instead of signed overflow
      auto* q = static_cast<int32_t*>(p);
      if (o == Op::Sum) q[0] = static_cast<int32_t>(static_cast<uint32_t>(q[0]) + 1u);
      else corrupt_first_t(o, q);
      break;
    }
    case DType::Int64: {
      auto* q = static_cast<int64_t*>(p);
      if (o == Op::Sum) q[0] = static_cast<int64_t>(static_cast<uint64_t>(q[0]) + 1u);
      else corrupt_first_t(o, q);
      break;
    }
    case DType::Float32: corrupt_first_t(o, static_cast<float*>(p)); break;
    case DType::Float64: corrupt_first_t(o, static_cast<double*>(p)); break;
    default: break;
  }
}

void usage() {
  std::printf(
      "reduce_mpi — element-wise MPI_Reduce benchmark (reduce.c semantics)\n"
      "  --ints=N          global int32 count   (default 512M = NUM_INTS)\n"
      "  --doubles=N       global double count  (default 256M = NUM_DOUBLES)\n"
      "  --longs=N --floats=N   counts for the LONG / FLOAT dtypes (default = ints / doubles)\n"
      "  --dtypes=INT,DOUBLE    order of dtypes (INT, LONG, FLOAT, DOUBLE)\n"
      "  --ops=MAX,MIN,SUM      order of ops\n"
      "  --retries=5  --warmup=1  --root=0  --collective=reduce|allreduce\n"
      "  --timing=max|root      max over ranks after a barrier (default) or reduce.c's root clock\n"
      "  --verify               check the reduced vector at sampled indices\n"
      "  --json=PATH            append one JSON record per measurement\n"
      "  --inject-fault=KIND[@RANK][:STEP]  exit|hang|corrupt|delay=<ms> before timed collective STEP\n");
}

}  // namespace

int main(int argc, char** argv) {
  MPI_CHECK(MPI_Init(&argc, &argv));
  int rank = 0, size = 1;
  MPI_CHECK(MPI_Comm_rank(MPI_COMM_WORLD, &rank));
  MPI_CHECK(MPI_Comm_size(MPI_COMM_WORLD, &size));

  CmdArgs args;
  try {
    args = CmdArgs(argc, argv);
  } catch (const CliError& e) {
    if (rank == 0) std::fprintf(stderr, "%s\n", e.what());
    MPI_Finalize();
    return EXIT_FAILURE;
  }
  if (args.has("version")) {  // build provenance (version.hpp)
    std::printf("reduce_mpi (mireduce) native source %s\n", mireduce::source_hash());
    return 0;
  }
  if (args.has("help")) {
    if (rank == 0) usage();
    MPI_Finalize();
    return EXIT_SUCCESS;
  }
  const std::set<std::string> known = {"ints", "doubles", "longs", "floats", "dtypes", "ops", "retries", "warmup",
                                       "root", "collective", "timing", "verify", "json", "help", "version", "inject-fault"};
  for (const auto& u : args.unknown(known))
    if (rank == 0) std::fprintf(stderr, "warning: unknown flag --%s ignored\n", u.c_str());

  uint64_t n_ints = kNumInts, n_doubles = kNumDoubles;
  std::vector<DType> dtypes = {DType::Int32, DType::Float64};
  std::vector<Op> ops = {Op::Max, Op::Min, Op::Sum};  // reduce.c:26-28 order
  int retries = kRetryCount, warmup = 1, root = 0;
  std::string collective = "reduce", timing = "max", json_path;
  try {
    args.get_uint("ints", &n_ints);
    args.get_uint("doubles", &n_doubles);
    uint64_t n_longs = n_ints, n_floats = n_doubles;
    args.get_uint("longs", &n_longs);
    args.get_uint("floats", &n_floats);
    std::vector<std::string> list;
    if (args.get_list("dtypes", &list)) {
      dtypes.clear();
      for (auto& s : list) {
        DType t;
        if (!parse_dtype(s, &t)) throw CliError("unknown dtype " + s);
        if (dtype_is_half(t)) throw CliError("--dtypes=" + s + ": MPI has no 16-bit float datatype (reduce.c types: INT, DOUBLE; plus LONG, FLOAT)");
        dtypes.push_back(t);
      }
    }
    if (args.get_list("ops", &list)) {
      ops.clear();
      for (auto& s : list) {
        Op o;
        if (!parse_op(s, &o)) throw CliError("unknown op " + s);
        if (op_is_fused(o)) throw CliError("--ops=" + s + ": the element-wise cross-rank benchmark keeps reduce.c's MAX/MIN/SUM");
        ops.push_back(o);
      }
    }
    retries = args.int_or<int>("retries", retries);
    warmup = args.int_or<int>("warmup", warmup);
    root = args.int_or<int>("root", root);
    collective = args.str_or("collective", collective);
    timing = args.str_or("timing", timing);
    json_path = args.str_or("json", "");
    if (collective != "reduce" && collective != "allreduce") throw CliError("--collective must be reduce|allreduce");
    if (timing != "max" && timing != "root") throw CliError("--timing must be max|root");
    if (root < 0 || root >= size) throw CliError("--root out of range");
    FaultInjector fault;
    try {
      fault = FaultInjector::from_flag_or_env(args.str_or("inject-fault", ""));
    } catch (const std::invalid_argument& e) {
      throw CliError(e.what());
    }
    long fault_step = 0;

    // per-dtype global counts
    auto global_count = [&](DType t) -> uint64_t {
      switch (t) {
        case DType::Int32: return n_ints;
        case DType::Int64: return n_longs;
        case DType::Float32: return n_floats;
        case DType::Float64: return n_doubles;
        default: break;
      }
      return 0;
    };

    Mt19937 gen;
    const uint64_t seeds[6] = {static_cast<uint64_t>(rank), 0x123, 0x234, 0x345, 0x456, 0x789};
    gen.init_by_array(seeds, 6);

    struct Buf {
      DType t;
      uint64_t count;  // this rank's count: N/P on every rank (reduce.c:43-44; the remainder is not reduced)
      uint64_t total;  // elements actually reduced = sum of counts
      std::vector<unsigned char> send, recv;
    };
    std::vector<Buf> bufs;
    for (DType t : dtypes) {
      const uint64_t n = global_count(t);
      // Element-wise reduction needs equal vectors on every rank: N/P each, as reduce.c:43-44.
      // Bandwidth is computed from the bytes actually reduced (count * P), not from N (B10).
      const uint64_t count = std::max<uint64_t>(1, n / static_cast<uint64_t>(size));
      if (count > static_cast<uint64_t>(INT32_MAX)) throw CliError("per-rank count exceeds MPI int count");
      Buf b{t, count, count * static_cast<uint64_t>(size), {}, {}};
      b.send.resize(count * dtype_size(t));
      b.recv.resize(count * dtype_size(t));
      generate(gen, t, b.send.data(), count);
      bufs.push_back(std::move(b));
    }

    auto run_one = [&](Buf& b, Op o) -> double {
      std::memset(b.recv.data(), 0, b.recv.size());  // bzero(reduced_*) (reduce.c:74,88)
      if (timing == "max") MPI_CHECK(MPI_Barrier(MPI_COMM_WORLD));
      const double t0 = StopWatch::now_s();
      if (collective == "reduce")
        MPI_CHECK(MPI_Reduce(b.send.data(), b.recv.data(), static_cast<int>(b.count), mpi_type(b.t), mpi_op(o), root, MPI_COMM_WORLD));
      else
        MPI_CHECK(MPI_Allreduce(b.send.data(), b.recv.data(), static_cast<int>(b.count), mpi_type(b.t), mpi_op(o), MPI_COMM_WORLD));
      double dt = StopWatch::now_s() - t0;
      if (timing == "max") MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, &dt, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD));
      return dt;
    };

    for (int w = 0; w < warmup; ++w)
      for (auto& b : bufs) run_one(b, Op::Sum);

    if (rank == root) std::printf("%s\n", gnuplot_header().c_str());
    bool all_ok = true;
    for (int x = 0; x < retries; ++x) {
      for (auto& b : bufs) {
        for (Op o : ops) {
          // fault injection: a wrong contribution at element 0 (a sampled index) for this collective
          unsigned char saved[8];
          const bool corrupt = fault.at(rank, fault_step++, "MPI collective") && b.count;
          if (corrupt) {
            std::memcpy(saved, b.send.data(), dtype_size(b.t));
            corrupt_first(b.t, o, b.send.data());
          }
          const double dt = run_one(b, o);
          if (corrupt) std::memcpy(b.send.data(), saved, dtype_size(b.t));
          const double bytes = static_cast<double>(b.total) * dtype_size(b.t);
          const double gib = bytes / dt / kGiB;
          if (rank == root) {
            std::printf("%s\n", gnuplot_line(dtype_gnuplot_name(b.t), op_name(o), size, gib).c_str());
            std::fflush(stdout);
          }
          bool ok = true;
          if (args.has("verify")) {
            ok = verify(b.t, o, b.send.data(), b.recv.data(), b.count, rank, size, root);
            all_ok = all_ok && ok;
          }
          if (rank == root && !json_path.empty()) {
            Json j;
            j.set("app", "reduce_mpi").set("dtype", dtype_gnuplot_name(b.t)).set("op", op_name(o))
                .set("ranks", size).set("count_per_rank", b.count).set("elements_total", b.total)
                .set("bytes_total", static_cast<uint64_t>(bytes)).set("seconds", dt)
                .set("gib_per_s", gib).set("gb_per_s", bytes / dt / kGB).set("bytes_per_GB", kGiB)
                .set("collective", collective).set("timing", timing).set("retry", x);
            if (args.has("verify")) j.set("verified", ok);
            j.write_file(json_path);
          }
        }
      }
    }
    if (args.has("verify") && rank == root)
      std::fprintf(stderr, "[reduce_mpi] verification %s\n", all_ok ? "PASSED" : "FAILED");
    MPI_Finalize();
    return all_ok ? EXIT_SUCCESS : EXIT_FAILURE;
  } catch (const CliError& e) {
    if (rank == 0) std::fprintf(stderr, "error: %s\n", e.what());
    MPI_Finalize();
    return EXIT_FAILURE;
  }
}
