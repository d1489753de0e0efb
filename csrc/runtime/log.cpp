// Logging; see log.hpp.
#include "mireduce/log.hpp"

#include <cstdarg>
#include <sys/stat.h>

namespace mireduce {

Logger& Logger::instance() {
  static Logger l;
  return l;
}

void Logger::set_log_file(const std::string& path) {
  close();
  if (!path.empty()) file_ = std::fopen(path.c_str(), "w");
}

void Logger::close() {
  if (file_) std::fclose(file_);
  file_ = nullptr;
}

void Logger::log(unsigned targets, const char* fmt, ...) {
  char buf[4096];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if ((targets & kLogConsole) && !quiet_) {
    std::fputs(buf, stdout);
    std::fflush(stdout);
  }
  if ((targets & kLogFile) && file_) {
    std::fputs(buf, file_);
    std::fflush(file_);
  }
  if ((targets & kLogMaster) && !master_path_.empty()) {
    struct stat st;
    const bool too_big = stat(master_path_.c_str(), &st) == 0 && st.st_size > kMasterLimit;
    if (std::FILE* m = std::fopen(master_path_.c_str(), too_big ? "w" : "a")) {
      std::fputs(buf, m);
      std::fclose(m);
    }
  }
}

}  // namespace mireduce
