// roctx ranges; see trace.hpp.
#include "mireduce/trace.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace mireduce {

namespace {
bool g_tracing = false;
}

void set_tracing(bool on) { g_tracing = on; }
bool tracing() { return g_tracing; }
void trace_push(const char* name) { roctxRangePushA(name); }
void trace_pop() { roctxRangePop(); }
void trace_mark(const char* name) {
  if (g_tracing) roctxMarkA(name);
}

}  // namespace mireduce
