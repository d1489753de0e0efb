// Host timers.
//
// Reference: StopWatchLinux (gettimeofday, averaged over sessions; stopwatch_linux.h:86-157)
// in the CUDA sample and rdtsc()/CLOCK_RATE with a hard-coded clock in reduce.c
// (externalfunctions.h:5-43, constants.h:3-4 — wrong on any other machine, bug B9). Here a
// monotonic steady clock with the same start/stop/average-over-sessions semantics; device-side
// intervals use hipEvents (gpu_timer.hpp).
#pragma once

#include <chrono>
#include <cstdint>
#include <vector>

namespace mireduce {

class StopWatch {
 public:
  void start() { t0_ = clock::now(); running_ = true; }
  // Ends a session and returns its length in ms.
  double stop();
  void reset() { total_ms_ = 0; sessions_ = 0; laps_.clear(); running_ = false; }
  double total_ms() const { return total_ms_; }
  double average_ms() const { return sessions_ ? total_ms_ / sessions_ : 0.0; }
  int sessions() const { return sessions_; }
  const std::vector<double>& laps_ms() const { return laps_; }

  static double now_s();

 private:
  using clock = std::chrono::steady_clock;
  clock::time_point t0_{};
  double total_ms_ = 0;
  int sessions_ = 0;
  bool running_ = false;
  std::vector<double> laps_;
};

}  // namespace mireduce
