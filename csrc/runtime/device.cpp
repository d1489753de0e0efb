// Device helpers; see device.hpp.
#include "mireduce/device.hpp"

namespace mireduce {

DeviceInfo device_info(int dev) {
  hipDeviceProp_t p;
  MIREDUCE_HIP_THROW(hipGetDeviceProperties(&p, dev));
  DeviceInfo d;
  d.id = dev;
  d.name = p.name;
  d.arch = p.gcnArchName;
  d.cus = p.multiProcessorCount;
  d.total_mem = p.totalGlobalMem;
  d.clock_khz = p.clockRate;
  return d;
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

EventTimer::EventTimer() {
  MIREDUCE_HIP_THROW(hipEventCreate(&a_));
  MIREDUCE_HIP_THROW(hipEventCreate(&b_));
}

EventTimer::~EventTimer() {
  if (a_) (void)hipEventDestroy(a_);
  if (b_) (void)hipEventDestroy(b_);
}

void EventTimer::start(hipStream_t s) { MIREDUCE_HIP_THROW(hipEventRecord(a_, s)); }
void EventTimer::stop(hipStream_t s) { MIREDUCE_HIP_THROW(hipEventRecord(b_, s)); }

float EventTimer::elapsed_ms() {
  MIREDUCE_HIP_THROW(hipEventSynchronize(b_));
  float ms = 0;
  MIREDUCE_HIP_THROW(hipEventElapsedTime(&ms, a_, b_));
  return ms;
}

void DeviceBuffer::allocate(size_t bytes) {
  release();
  if (bytes) MIREDUCE_HIP_THROW(hipMalloc(&p_, bytes));
  n_ = bytes;
}

void DeviceBuffer::release() {
  if (p_) (void)hipFree(p_);
  p_ = nullptr;
  n_ = 0;
}

}  // namespace mireduce
