// Host timers; see timer.hpp.
#include "mireduce/timer.hpp"

namespace mireduce {

double StopWatch::stop() {
  if (!running_) return 0.0;
  const double ms = std::chrono::duration<double, std::milli>(clock::now() - t0_).count();
  running_ = false;
  total_ms_ += ms;
  ++sessions_;
  laps_.push_back(ms);
  return ms;
}

double StopWatch::now_s() {
  return std::chrono::duration<double>(clock::now().time_since_epoch()).count();
}

}  // namespace mireduce
