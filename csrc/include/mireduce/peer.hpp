// Peer-read kernel for the xGMI roofline (bandwidth_test --peer).
//
// Reference: the vendored simpleP2P sample enables peer access and has a kernel on one GPU read
// another GPU's buffer (cuda/C/src/simpleP2P/simpleP2P.cu:164,250-275). Here one launch on the
// reading device streams 16-byte non-temporal loads from up to 16 peer buffers at once (workgroup
// b reads source b % nsrc), so a single kernel exercises every xGMI link of the device together.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace mireduce {

constexpr int kMaxPeerSources = 16;

struct PeerSources {
  const void* p[kMaxPeerSources];
};

// Read `bytes_each` from each of the `nsrc` sources (device pointers valid on the current device:
// local or peer-mapped). `sink` (>= grid uint32) only keeps the loads alive. grid: workgroups,
// rounded up to a multiple of nsrc (0: 128 per source).
void peer_read(const PeerSources& srcs, int nsrc, size_t bytes_each, uint32_t* sink, int grid, hipStream_t s);

}  // namespace mireduce
