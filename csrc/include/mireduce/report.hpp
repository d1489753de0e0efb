// Output formats and statistics.
//
// Compatibility contract:
//  * reduce.c GNUPlot lines: header "# DATATYPE OP NODES GB/sec" and rows "%s %s %d %10.3lf"
//    (mpi/reduce.c:67-69,80-82,94-96), GB = 2^30 B of total data, consumed unchanged by
//    getAvgs.sh (mpi/getAvgs.sh:3-14) and makePlots.gp (`using 3:4`).
//  * CUDA-sample throughput line (cuda/C/src/reduction/reduction.cpp:744-745), GB = 1e9 B,
//    with a 64-bit Size and the real device count.
// New: a tiny JSON writer for the per-run sidecars (all parameters, per-iteration times, units).
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace mireduce {

constexpr double kGiB = 1073741824.0;  // reduce.c's "GB" (mpi/reduce.c:79)
constexpr double kGB = 1.0e9;          // reduction.cpp's "GB" (reduction.cpp:745)

std::string gnuplot_header();
std::string gnuplot_line(const std::string& dtype, const std::string& op, int nodes, double gib_per_s);
std::string throughput_line(double gb_per_s, double seconds, uint64_t elements, int num_devs,
                            unsigned workgroup);

struct Stats {
  int count = 0;
  double mean = 0, median = 0, min = 0, max = 0, stddev = 0;
};
Stats compute_stats(const std::vector<double>& v);

// Minimal ordered JSON object builder (strings escaped; numbers printed with %.17g).
class Json {
 public:
  Json& set(const std::string& k, const std::string& v);
  Json& set(const std::string& k, const char* v) { return set(k, std::string(v)); }
  Json& set(const std::string& k, double v);
  Json& set(const std::string& k, int64_t v);
  Json& set(const std::string& k, uint64_t v);
  Json& set(const std::string& k, int v) { return set(k, static_cast<int64_t>(v)); }
  Json& set(const std::string& k, unsigned v) { return set(k, static_cast<uint64_t>(v)); }
  Json& set(const std::string& k, bool v);
  Json& set(const std::string& k, const std::vector<double>& v);
  Json& set(const std::string& k, const Json& obj);
  Json& set_null(const std::string& k);
  std::string str() const;
  bool write_file(const std::string& path) const;

 private:
  std::vector<std::pair<std::string, std::string>> kv_;  // value already serialised
};

std::string json_escape(const std::string& s);

// Peer (xGMI) bandwidth test (bandwidth_test --peer): the ordered (src, dst) device pairs, src !=
// dst, row-major — the simpleP2P copy of cuda/C/src/simpleP2P/simpleP2P.cu:314-329 for every pair.
std::vector<std::pair<int, int>> peer_pairs(int ndev);
// Matrix table of per-pair values (rows = src, columns = dst, ndev x ndev row-major; "-" on the
// diagonal), one line per source device.
std::string peer_matrix(int ndev, const std::vector<double>& values, const char* unit);

}  // namespace mireduce
