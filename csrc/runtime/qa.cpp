// QA protocol; see qa.hpp.
#include "mireduce/qa.hpp"

#include <strings.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace mireduce {

namespace {
const char* exe_name(const char* argv0) {
  const char* s = std::strrchr(argv0, '/');
  return s ? s + 1 : argv0;
}
bool has_flag(int argc, const char* const* argv, const char* name) {
  for (int i = 1; i < argc; ++i) {
    const char* a = argv[i];
    while (*a == '-') ++a;
    const char* eq = std::strchr(a, '=');
    const size_t len = eq ? static_cast<size_t>(eq - a) : std::strlen(a);
    if (len == std::strlen(name) && !strncasecmp(a, name, len)) return true;
  }
  return false;
}
void print_cmd(const char* tag, int argc, const char* const* argv) {
  std::fprintf(stderr, "&&&& %s %s", tag, exe_name(argv[0]));
  for (int i = 1; i < argc; ++i) std::fprintf(stderr, " %s", argv[i]);
  std::fprintf(stderr, "\n");
}
}  // namespace

const char* qa_status_name(QaStatus s) {
  switch (s) {
    case QaStatus::Failed: return "FAILED";
    case QaStatus::Passed: return "PASSED";
    case QaStatus::Waived: return "WAIVED";
  }
  return "?";
}

void qa_start(int argc, const char* const* argv) {
  std::fflush(stdout);
  if (has_flag(argc, argv, "qatest")) print_cmd("RUNNING", argc, argv);
  else std::fprintf(stderr, "[%s] starting...\n", exe_name(argv[0]));
  std::fflush(stderr);
  std::printf("\n");
  std::fflush(stdout);
}

void qa_finish(int argc, const char* const* argv, QaStatus status) {
  if (has_flag(argc, argv, "qatest")) print_cmd(qa_status_name(status), argc, argv);
  else std::fprintf(stderr, "[%s] test results...\n%s\n", exe_name(argv[0]), qa_status_name(status));
  std::fflush(stderr);
  std::printf("\n");
  std::fflush(stdout);
  if (has_flag(argc, argv, "countdown")) {
    std::fprintf(stderr, "> exiting in 3 seconds: ");
    for (int i = 3; i > 0; --i) { std::fprintf(stderr, "%d...", i); std::fflush(stderr); sleep(1); }
    std::fprintf(stderr, "done!\n");
  } else if (has_flag(argc, argv, "prompt")) {
    std::fprintf(stderr, "\nPress <Enter> to exit...\n");
    std::getchar();
  }
}

void qa_finish_exit(int argc, const char* const* argv, QaStatus status) {
  qa_finish(argc, argv, status);
  std::exit(status == QaStatus::Failed ? EXIT_FAILURE : EXIT_SUCCESS);
}

}  // namespace mireduce
