// Command-line grammar shared by all apps.
//
// Same grammar as the SDK's CmdArgReader (cuda/C/common/src/cmd_arg_reader.cpp:119-151):
// every token must start with '-' (otherwise an error), `-name` / `--name` set a flag, and
// `-name=value` / `--name=value` set a value; values are converted on lookup
// (cmd_arg_reader.h:39-48). Lookups mirror cutCheckCmdLineFlag / cutGetCmdLineArgumenti /
// cutGetCmdLineArgumentstr (cuda/C/common/src/cutil.cpp:1135,1168,1250).
#pragma once

#include <cstdint>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

namespace mireduce {

struct CliError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class CmdArgs {
 public:
  CmdArgs() = default;
  CmdArgs(int argc, const char* const* argv);  // throws CliError

  bool has(const std::string& name) const;  // flag or value given
  bool get_str(const std::string& name, std::string* out) const;
  bool get_int(const std::string& name, int64_t* out) const;  // throws CliError on junk
  bool get_uint(const std::string& name, uint64_t* out) const;
  bool get_double(const std::string& name, double* out) const;
  // Comma-separated list value ("--ops=MAX,MIN,SUM").
  bool get_list(const std::string& name, std::vector<std::string>* out) const;

  template <class T>
  T int_or(const std::string& name, T def) const {
    int64_t v;
    return get_int(name, &v) ? static_cast<T>(v) : def;
  }
  std::string str_or(const std::string& name, const std::string& def) const {
    std::string v;
    return get_str(name, &v) ? v : def;
  }

  // Names given on the command line that are not in `known`.
  std::vector<std::string> unknown(const std::set<std::string>& known) const;
  const std::map<std::string, std::string>& raw() const { return args_; }
  const std::string& program() const { return program_; }

  static constexpr const char* kFlag = "\x01FLAG";

 private:
  std::map<std::string, std::string> args_;
  std::string program_;
};

// Element counts accept plain integers and k/M/G (2^10/2^20/2^30) or e-notation ("1e9").
bool parse_count(const std::string& s, uint64_t* out);

}  // namespace mireduce
