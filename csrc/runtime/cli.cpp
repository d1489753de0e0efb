// Command-line grammar; see cli.hpp.
#include "mireduce/cli.hpp"

#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <sstream>

namespace mireduce {

CmdArgs::CmdArgs(int argc, const char* const* argv) {
  if (argc > 0 && argv[0]) {
    std::string p = argv[0];
    const auto slash = p.find_last_of("/\\");
    program_ = slash == std::string::npos ? p : p.substr(slash + 1);
  }
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i] ? argv[i] : "";
    if (a.empty() || a[0] != '-')
      throw CliError("Invalid command line argument: '" + a + "' (arguments must start with - or --)");
    const size_t dashes = (a.size() > 1 && a[1] == '-') ? 2 : 1;
    const size_t eq = a.find('=');
    if (eq == std::string::npos) {
      args_[a.substr(dashes)] = kFlag;
    } else {
      args_[a.substr(dashes, eq - dashes)] = a.substr(eq + 1);
    }
  }
}

bool CmdArgs::has(const std::string& name) const { return args_.count(name) != 0; }

bool CmdArgs::get_str(const std::string& name, std::string* out) const {
  auto it = args_.find(name);
  if (it == args_.end() || it->second == kFlag) return false;
  *out = it->second;
  return true;
}

bool CmdArgs::get_int(const std::string& name, int64_t* out) const {
  std::string s;
  if (!get_str(name, &s)) return false;
  uint64_t u = 0;
  if (!s.empty() && s[0] == '-') {
    if (!parse_count(s.substr(1), &u)) throw CliError("--" + name + ": not an integer: " + s);
    *out = -static_cast<int64_t>(u);
    return true;
  }
  if (!parse_count(s, &u)) throw CliError("--" + name + ": not an integer: " + s);
  *out = static_cast<int64_t>(u);
  return true;
}

bool CmdArgs::get_uint(const std::string& name, uint64_t* out) const {
  std::string s;
  if (!get_str(name, &s)) return false;
  if (!parse_count(s, out)) throw CliError("--" + name + ": not a non-negative integer: " + s);
  return true;
}

bool CmdArgs::get_double(const std::string& name, double* out) const {
  std::string s;
  if (!get_str(name, &s)) return false;
  char* end = nullptr;
  errno = 0;
  const double v = std::strtod(s.c_str(), &end);
  if (errno || end == s.c_str() || *end) throw CliError("--" + name + ": not a number: " + s);
  *out = v;
  return true;
}

bool CmdArgs::get_list(const std::string& name, std::vector<std::string>* out) const {
  std::string s;
  if (!get_str(name, &s)) return false;
  out->clear();
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, ','))
    if (!item.empty()) out->push_back(item);
  return true;
}

std::vector<std::string> CmdArgs::unknown(const std::set<std::string>& known) const {
  std::vector<std::string> u;
  for (const auto& kv : args_)
    if (!known.count(kv.first)) u.push_back(kv.first);
  return u;
}

bool parse_count(const std::string& s, uint64_t* out) {
  if (s.empty()) return false;
  size_t pos = 0;
  while (pos < s.size() && (std::isdigit(static_cast<unsigned char>(s[pos])))) ++pos;
  if (pos == 0) return false;
  if (pos == s.size()) {
    errno = 0;
    *out = std::strtoull(s.c_str(), nullptr, 10);
    return errno == 0;
  }
  const std::string num = s.substr(0, pos);
  const std::string suf = s.substr(pos);
  uint64_t base = std::strtoull(num.c_str(), nullptr, 10);
  if (suf == "k" || suf == "K") { *out = base << 10; return true; }
  if (suf == "m" || suf == "M") { *out = base << 20; return true; }
  if (suf == "g" || suf == "G") { *out = base << 30; return true; }
  if (suf[0] == 'e' || suf[0] == 'E') {
    char* end = nullptr;
    const double v = std::strtod(s.c_str(), &end);
    if (*end || v < 0 || v > 1.8e19 || v != std::floor(v)) return false;
    *out = static_cast<uint64_t>(v);
    return true;
  }
  return false;
}

}  // namespace mireduce
