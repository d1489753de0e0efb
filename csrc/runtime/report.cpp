// Output formats and statistics; see report.hpp.
#include "mireduce/report.hpp"
#include "mireduce/version.hpp"

#include <algorithm>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <fstream>

namespace mireduce {

std::string gnuplot_header() { return "# DATATYPE OP NODES GB/sec"; }

std::string gnuplot_line(const std::string& dtype, const std::string& op, int nodes, double gib_per_s) {
  char buf[256];
  std::snprintf(buf, sizeof buf, "%s %s %d %10.3lf", dtype.c_str(), op.c_str(), nodes, gib_per_s);
  return buf;
}

std::string throughput_line(double gb_per_s, double seconds, uint64_t elements, int num_devs,
                            unsigned workgroup) {
  char buf[256];
  std::snprintf(buf, sizeof buf,
                "Reduction, Throughput = %.4f GB/s, Time = %.5f s, Size = %" PRIu64
                " Elements, NumDevsUsed = %d, Workgroup = %u",
                gb_per_s, seconds, elements, num_devs, workgroup);
  return buf;
}

Stats compute_stats(const std::vector<double>& v) {
  Stats s;
  s.count = static_cast<int>(v.size());
  if (v.empty()) return s;
  std::vector<double> t = v;
  std::sort(t.begin(), t.end());
  double sum = 0;
  for (double x : t) sum += x;
  s.mean = sum / t.size();
  s.min = t.front();
  s.max = t.back();
  const size_t m = t.size() / 2;
  s.median = (t.size() % 2) ? t[m] : 0.5 * (t[m - 1] + t[m]);
  double var = 0;
  for (double x : t) var += (x - s.mean) * (x - s.mean);
  s.stddev = t.size() > 1 ? std::sqrt(var / (t.size() - 1)) : 0.0;
  return s;
}

std::string json_escape(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  return o + "\"";
}

static std::string num(double v) {
  if (!std::isfinite(v)) return "null";
  char b[64];
  std::snprintf(b, sizeof b, "%.17g", v);
  return b;
}

Json& Json::set(const std::string& k, const std::string& v) { kv_.emplace_back(k, json_escape(v)); return *this; }
Json& Json::set(const std::string& k, double v) { kv_.emplace_back(k, num(v)); return *this; }
Json& Json::set(const std::string& k, int64_t v) { kv_.emplace_back(k, std::to_string(v)); return *this; }
Json& Json::set(const std::string& k, uint64_t v) { kv_.emplace_back(k, std::to_string(v)); return *this; }
Json& Json::set(const std::string& k, bool v) { kv_.emplace_back(k, v ? "true" : "false"); return *this; }
Json& Json::set_null(const std::string& k) { kv_.emplace_back(k, "null"); return *this; }
Json& Json::set(const std::string& k, const std::vector<double>& v) {
  std::string s = "[";
  for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + num(v[i]);
  kv_.emplace_back(k, s + "]");
  return *this;
}
Json& Json::set(const std::string& k, const Json& obj) { kv_.emplace_back(k, obj.str()); return *this; }

std::string Json::str() const {
  std::string s = "{";
  for (size_t i = 0; i < kv_.size(); ++i) s += (i ? ", " : "") + json_escape(kv_[i].first) + ": " + kv_[i].second;
  return s + "}";
}

bool Json::write_file(const std::string& path) const {
  std::ofstream f(path, std::ios::app);
  if (!f) return false;
  // every sidecar record carries the build provenance (version.hpp)
  bool has_hash = false;
  for (const auto& kv : kv_) has_hash = has_hash || kv.first == "native_source_hash";
  if (has_hash) {
    f << str() << "\n";
  } else {
    Json j = *this;
    j.set("native_source_hash", std::string(source_hash()));
    f << j.str() << "\n";
  }
  return static_cast<bool>(f);
}


std::vector<std::pair<int, int>> peer_pairs(int ndev) {
  std::vector<std::pair<int, int>> v;
  for (int s = 0; s < ndev; ++s)
    for (int d = 0; d < ndev; ++d)
      if (s != d) v.emplace_back(s, d);
  return v;
}

std::string peer_matrix(int ndev, const std::vector<double>& values, const char* unit) {
  std::string out = std::string("   src\\dst (") + unit + ")";
  char buf[64];
  out += "\n      ";
  for (int d = 0; d < ndev; ++d) {
    std::snprintf(buf, sizeof buf, "%9d", d);
    out += buf;
  }
  out += "\n";
  for (int s = 0; s < ndev; ++s) {
    std::snprintf(buf, sizeof buf, "%6d", s);
    out += buf;
    for (int d = 0; d < ndev; ++d) {
      const size_t k = static_cast<size_t>(s) * ndev + d;
      if (s == d || k >= values.size()) std::snprintf(buf, sizeof buf, "%9s", "-");
      else std::snprintf(buf, sizeof buf, "%9.1f", values[k]);
      out += buf;
    }
    out += "\n";
  }
  return out;
}

}  // namespace mireduce
