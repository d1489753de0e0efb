// Error-checking macros.
//
// Replaces the cutil pattern cutilSafeCallNoSync / cutilCheckMsg
// (cuda/C/common/inc/cutil_inline_runtime.h:267-273,352-359): print `file(line)` and the error
// string, then exit non-zero. In a multi-rank job the fatal path also aborts the communicator
//  via the hook installed by comm/rccl_comm.cpp.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace mireduce {

// Called before exit() on a fatal error; the comm layer installs ncclCommAbort / MPI_Abort here.
using FatalHook = void (*)(int code);
void set_fatal_hook(FatalHook hook);
[[noreturn]] void fatal(const char* file, int line, const std::string& msg, int code = EXIT_FAILURE);

// Library code throws (so the Python binding can turn errors into exceptions); apps use the
// *_FATAL forms which print and exit like the reference.
struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

std::string hip_error_string(hipError_t e, const char* expr, const char* file, int line);

}  // namespace mireduce

#define MIREDUCE_HIP_THROW(expr)                                                              \
  do {                                                                                        \
    hipError_t mireduce_e_ = (expr);                                                          \
    if (mireduce_e_ != hipSuccess)                                                            \
      throw ::mireduce::Error(::mireduce::hip_error_string(mireduce_e_, #expr, __FILE__, __LINE__)); \
  } while (0)

#define HIP_CHECK(expr)                                                                       \
  do {                                                                                        \
    hipError_t mireduce_e_ = (expr);                                                          \
    if (mireduce_e_ != hipSuccess)                                                            \
      ::mireduce::fatal(__FILE__, __LINE__,                                                   \
                        std::string(#expr) + ": " + hipGetErrorString(mireduce_e_));          \
  } while (0)

#define MIREDUCE_REQUIRE(cond, msg)                                                           \
  do {                                                                                        \
    if (!(cond)) throw ::mireduce::Error(std::string(msg) + " [" #cond "]");                  \
  } while (0)
