// Logging: console + per-run log file + optional append-only master CSV.
//
// Reference: shrLog / shrLogEx(LOGBOTH|MASTER) and shrSetLogFileName("reduction.txt")
// (cuda/shared/src/shrUtils.cpp:157-565; used at reduction.cpp:88,744). LOGBOTH writes the
// console and the log file; MASTER also appends to SdkMasterLog.csv, which is truncated once it
// exceeds 50,000 bytes (shrUtils.cpp:274).
#pragma once

#include <cstdio>
#include <string>

namespace mireduce {

enum LogTarget : unsigned { kLogConsole = 1u, kLogFile = 2u, kLogBoth = 3u, kLogMaster = 4u };

class Logger {
 public:
  static Logger& instance();
  // Opening a log file truncates it (one file per run, like shrSetLogFileName).
  void set_log_file(const std::string& path);
  void set_master_file(const std::string& path) { master_path_ = path; }
  void set_quiet(bool q) { quiet_ = q; }
  void log(unsigned targets, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
  void close();
  ~Logger() { close(); }

  static constexpr long kMasterLimit = 50000;

 private:
  std::FILE* file_ = nullptr;
  std::string master_path_;
  bool quiet_ = false;
};

#define MIREDUCE_LOG(...) ::mireduce::Logger::instance().log(::mireduce::kLogBoth, __VA_ARGS__)

}  // namespace mireduce
