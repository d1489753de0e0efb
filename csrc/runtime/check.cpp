// Fatal-error path behind HIP_CHECK / RCCL_CHECK (cutil_inline_runtime.h:267-273 parity).
#include <cstdio>
#include <cstdlib>
#include <string>

#include "mireduce/check.hpp"

namespace mireduce {

namespace {
FatalHook g_fatal_hook = nullptr;
}

void set_fatal_hook(FatalHook hook) { g_fatal_hook = hook; }

void fatal(const char* file, int line, const std::string& msg, int code) {
  std::fprintf(stderr, "%s(%d) : fatal error : %s\n", file, line, msg.c_str());
  std::fflush(stderr);
  if (g_fatal_hook) g_fatal_hook(code);
  std::exit(code);
}

std::string hip_error_string(hipError_t e, const char* expr, const char* file, int line) {
  return std::string(file) + "(" + std::to_string(line) + "): " + expr + " failed: " +
         hipGetErrorString(e);
}

}  // namespace mireduce
