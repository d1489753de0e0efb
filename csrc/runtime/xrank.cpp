// Host side of the fused cross-rank finalisation channel (xrank.hpp): mailbox allocation, IPC
// mapping of every peer's mailbox, and the device descriptor the finishing workgroup reads.
#include "mireduce/xrank.hpp"

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstring>

#include "mireduce/check.hpp"

namespace mireduce {

namespace {
struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int dev) {
    MIREDUCE_HIP_THROW(hipGetDevice(&prev));
    MIREDUCE_HIP_THROW(hipSetDevice(dev));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

constexpr size_t kMailboxBytes = 4096;  // one page: IPC maps whole allocations
}  // namespace

XrankChannel::XrankChannel(int device, double timeout_s) : timeout_s_(timeout_s) {
  MIREDUCE_REQUIRE(timeout_s > 0, "XrankChannel: timeout must be positive");
  if (device < 0) MIREDUCE_HIP_THROW(hipGetDevice(&device));
  device_ = device;
  DeviceGuard g(device_);
  // Uncached: the poller must see a peer's xGMI store, not a line its own L2 holds.
  MIREDUCE_HIP_THROW(hipExtMallocWithFlags(reinterpret_cast<void**>(&mbox_), kMailboxBytes, hipDeviceMallocUncached));
  MIREDUCE_HIP_THROW(hipMemset(mbox_, 0, kMailboxBytes));
  MIREDUCE_HIP_THROW(hipMalloc(reinterpret_cast<void**>(&counters_), 256));
  MIREDUCE_HIP_THROW(hipMemset(counters_, 0, 256));
  MIREDUCE_HIP_THROW(hipMalloc(reinterpret_cast<void**>(&desc_dev_), sizeof(XrankDesc)));
  MIREDUCE_HIP_THROW(hipDeviceSynchronize());
}

XrankChannel::~XrankChannel() {
  DeviceGuard g(device_);
  for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
  (void)hipFree(desc_dev_);
  (void)hipFree(counters_);
  (void)hipFree(mbox_);
  (void)hipGetLastError();  // ignored failures above must not surface at the next launch check
}

IpcHandleBytes XrankChannel::handle() const {
  hipIpcMemHandle_t h;
  MIREDUCE_HIP_THROW(hipIpcGetMemHandle(&h, mbox_));
  IpcHandleBytes b;
  std::memcpy(b.data(), &h, sizeof h);
  return b;
}

void XrankChannel::connect(int rank, int world, const std::vector<IpcHandleBytes>& handles) {
  MIREDUCE_REQUIRE(!connected_, "XrankChannel: already connected");
  MIREDUCE_REQUIRE(world >= 1 && world <= kMaxXrankRanks, "XrankChannel: world must be 1..16");
  MIREDUCE_REQUIRE(rank >= 0 && rank < world, "XrankChannel: rank out of range");
  MIREDUCE_REQUIRE(handles.size() == static_cast<size_t>(world), "XrankChannel: one handle per rank");
  DeviceGuard g(device_);
  XrankDesc d{};
  for (int r = 0; r < world; ++r) {
    if (r == rank) {
      d.peer_mbox[r] = mbox_;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof h);
    void* p = nullptr;
    MIREDUCE_HIP_THROW(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    opened_.push_back(p);
    d.peer_mbox[r] = static_cast<uint64_t*>(p);
  }
  d.own_mbox = mbox_;
  d.epoch = counters_;
  d.error = counters_ + 1;
  d.rank = rank;
  d.world = world;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_) != hipSuccess || khz <= 0)
    khz = 100000;  // gfx950: 100 MHz
  d.timeout_ticks = static_cast<uint64_t>(timeout_s_ * 1e3 * khz);
  ticks_per_us_ = khz * 1e-3;
  d.stamps = nullptr;
  d.stamp_mask = 0;
  MIREDUCE_HIP_THROW(hipMemcpy(desc_dev_, &d, sizeof d, hipMemcpyHostToDevice));
  MIREDUCE_HIP_THROW(hipDeviceSynchronize());
  rank_ = rank;
  world_ = world;
  connected_ = true;
}

unsigned XrankChannel::error() const {
  unsigned v = 0;
  DeviceGuard g(device_);
  MIREDUCE_HIP_THROW(hipMemcpy(&v, counters_ + 1, sizeof v, hipMemcpyDeviceToHost));
  return v;
}

unsigned XrankChannel::epoch() const {
  unsigned v = 0;
  DeviceGuard g(device_);
  MIREDUCE_HIP_THROW(hipMemcpy(&v, counters_, sizeof v, hipMemcpyDeviceToHost));
  return v;
}

void XrankChannel::set_stamps(uint64_t* stamps, unsigned cap) {
  MIREDUCE_REQUIRE(connected_, "XrankChannel::set_stamps: not connected");
  MIREDUCE_REQUIRE(stamps == nullptr || (cap > 0 && (cap & (cap - 1)) == 0),
                   "XrankChannel::set_stamps: capacity must be a power of two");
  DeviceGuard g(device_);
  struct {
    uint64_t* p;
    unsigned m;
  } f{stamps, stamps ? cap - 1 : 0u};
  static_assert(offsetof(XrankDesc, stamp_mask) == offsetof(XrankDesc, stamps) + sizeof(uint64_t*),
                "stamp fields must be adjacent");
  MIREDUCE_HIP_THROW(hipDeviceSynchronize());
  MIREDUCE_HIP_THROW(hipMemcpy(reinterpret_cast<char*>(desc_dev_) + offsetof(XrankDesc, stamps), &f,
                               sizeof(uint64_t*) + sizeof(unsigned), hipMemcpyHostToDevice));
  MIREDUCE_HIP_THROW(hipDeviceSynchronize());
}

void XrankChannel::clear_error() {
  DeviceGuard g(device_);
  MIREDUCE_HIP_THROW(hipMemset(counters_ + 1, 0, sizeof(unsigned)));
  MIREDUCE_HIP_THROW(hipDeviceSynchronize());
}

}  // namespace mireduce
