// roctx ranges for rocprofv3 --marker-trace (SURVEY.md §5.1 "`--trace` emits roctx ranges").
// Disabled unless set_tracing(true) (apps: --trace); a disabled range costs one branch.
#pragma once

namespace mireduce {

void set_tracing(bool on);
bool tracing();
void trace_push(const char* name);
void trace_pop();
void trace_mark(const char* name);

class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(tracing()) {
    if (on_) trace_push(name);
  }
  ~TraceRange() {
    if (on_) trace_pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

}  // namespace mireduce
