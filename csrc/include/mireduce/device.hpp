// Device helpers: properties, hipEvent timing, RAII device buffers.
//
// Reference: cutilDeviceInit / cudaChooseDevice / cudaGetDeviceProperties (reduction.cpp:130-155,
// cutil_inline_runtime.h:388-417) and the cutil timers. Device-side intervals are measured with
// hipEvents on the stream instead of a host clock around device syncs.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <string>

#include "mireduce/check.hpp"

namespace mireduce {

struct DeviceInfo {
  int id = 0;
  std::string name;
  std::string arch;
  int cus = 0;
  size_t total_mem = 0;
  int clock_khz = 0;
};

DeviceInfo device_info(int dev);
int device_count();

class EventTimer {
 public:
  EventTimer();
  ~EventTimer();
  EventTimer(const EventTimer&) = delete;
  EventTimer& operator=(const EventTimer&) = delete;
  void start(hipStream_t s);
  void stop(hipStream_t s);
  float elapsed_ms();  // synchronises on the stop event

 private:
  hipEvent_t a_ = nullptr, b_ = nullptr;
};

class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t bytes) { allocate(bytes); }
  ~DeviceBuffer() { release(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
  void allocate(size_t bytes);
  void release();
  void* get() const { return p_; }
  template <class T> T* as() const { return static_cast<T*>(p_); }
  size_t bytes() const { return n_; }

 private:
  void* p_ = nullptr;
  size_t n_ = 0;
};

}  // namespace mireduce
