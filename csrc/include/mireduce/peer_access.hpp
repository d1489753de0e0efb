// Peer-access preflight of the IPC-mapped xGMI paths (the fused cross-rank finish, the direct
// collective): before any rank opens a peer's IPC handle, every rank must know that every pair of
// distinct GPUs in the job can map each other's memory — a rank that went ahead without it would
// fault the GPU instead of failing a host call.
//
// Reference: the vendored simpleP2P checks cudaDeviceCanAccessPeer both ways before it enables or
// maps anything (cuda/C/src/simpleP2P/simpleP2P.cu:250-251,273-275). Same rules as the Python
// preflight (cuda_mpi_reductions_amd/parallel/topology.py peer_verdict): one host, distinct
// physical devices at distinct indices, and peer access for every distinct pair. Ranks that share
// one physical GPU (the one-GPU rehearsals) need no peer access between them.
#pragma once

#include <functional>
#include <string>
#include <vector>

namespace mireduce {

struct PeerKey {
  std::string host;  // hostname
  std::string gpu;   // physical device identity (UUID, else PCI bus id)
  int index = 0;     // local device index of the rank
};

// This rank's verdict (pure): "" when rank `me` can map every peer's memory, else why not.
// can_access(my_index, peer_index) answers hipDeviceCanAccessPeer.
std::string peer_verdict(const std::vector<PeerKey>& keys, int me, const std::function<bool(int, int)>& can_access);

// Combine every rank's verdict into the job's (identical on every rank): "" or
// "rank r: why; rank s: why".
std::string agree_verdicts(const std::vector<std::string>& verdicts);

class TcpBootstrap;
class FaultInjector;

// Collective over `boot`: all-gather (host, GPU, index) and every rank's verdict; returns the
// agreed verdict ("" = every rank may map every peer). `fault` (kind nopeer) makes its rank's
// access query answer no. A rank whose own device query fails reports that as its verdict (it
// still takes part in both gathers, so no rank is left waiting).
std::string peer_preflight(TcpBootstrap& boot, int device, const FaultInjector* fault = nullptr);

}  // namespace mireduce
