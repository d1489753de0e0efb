// Peer-read kernel; see peer.hpp.
#include <hip/hip_runtime.h>

#include "mireduce/check.hpp"
#include "mireduce/peer.hpp"

namespace mireduce {
namespace kern {

constexpr int kPeerBlock = 256;
constexpr int kPeerUnroll = 4;

__global__ __launch_bounds__(kPeerBlock) void peer_read_kernel(PeerSources srcs, int nsrc, uint64_t nvec,
                                                                uint32_t* sink) {
  using V = uint32_t __attribute__((ext_vector_type(4)));
  const int src = blockIdx.x % nsrc;
  const uint64_t part = blockIdx.x / nsrc;
  const uint64_t parts = gridDim.x / nsrc;
  const V* p = static_cast<const V*>(srcs.p[src]);
  const uint64_t stride = parts * kPeerBlock;
  uint32_t acc = 0;
  uint64_t i = part * kPeerBlock + threadIdx.x;
  for (; i + (kPeerUnroll - 1) * stride < nvec; i += kPeerUnroll * stride) {
    V v[kPeerUnroll];
#pragma unroll
    for (int u = 0; u < kPeerUnroll; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
    for (int u = 0; u < kPeerUnroll; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < nvec; i += stride) {
    const V v = __builtin_nontemporal_load(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;  // data-dependent: the loads cannot be dropped
}

}  // namespace kern

void peer_read(const PeerSources& srcs, int nsrc, size_t bytes_each, uint32_t* sink, int grid, hipStream_t s) {
  MIREDUCE_REQUIRE(nsrc >= 1 && nsrc <= kMaxPeerSources, "peer_read: 1..16 sources");
  if (grid <= 0) grid = 128 * nsrc;
  grid = (grid + nsrc - 1) / nsrc * nsrc;
  (void)hipGetLastError();  // the check below must see this launch only, not an earlier ignored call
  hipLaunchKernelGGL(kern::peer_read_kernel, dim3(grid), dim3(kern::kPeerBlock), 0, s, srcs, nsrc,
                     static_cast<uint64_t>(bytes_each / 16), sink);
  MIREDUCE_HIP_THROW(hipGetLastError());
}

}  // namespace mireduce
