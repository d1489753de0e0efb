// Collective peer-access preflight over the TCP bootstrap (peer_access.hpp).
#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <array>
#include <cstring>

#include "mireduce/comm.hpp"
#include "mireduce/fault.hpp"
#include "mireduce/peer_access.hpp"

namespace mireduce {

namespace {

constexpr size_t kField = 128;  // fixed-width fields of the all-gathered records

struct KeyRecord {
  char host[kField];
  char gpu[kField];
  int index;
  int ok;             // 0: this rank's own device query failed (err holds why)
  char err[kField];
};

void put(char (&dst)[kField], const std::string& s) {
  std::memset(dst, 0, kField);
  std::memcpy(dst, s.data(), std::min(s.size(), kField - 1));
}

std::string device_identity(int device, std::string* err) {
  hipUUID uuid{};
  if (hipDeviceGetUuid(&uuid, device) == hipSuccess) {
    static const char* hex = "0123456789abcdef";
    std::string s;
    for (unsigned char c : uuid.bytes) {
      s += hex[c >> 4];
      s += hex[c & 15];
    }
    if (s.find_first_not_of('0') != std::string::npos) return s;
  }
  char bus[64] = {0};
  const hipError_t e = hipDeviceGetPCIBusId(bus, sizeof bus, device);
  if (e != hipSuccess) {
    *err = std::string("cannot identify device ") + std::to_string(device) + ": " + hipGetErrorString(e);
    return "";
  }
  return bus;
}

}  // namespace

std::string peer_preflight(TcpBootstrap& boot, int device, const FaultInjector* fault) {
  const int world = boot.world(), rank = boot.rank();
  KeyRecord mine{};
  std::string err;
  char host[kField] = {0};
  if (gethostname(host, kField - 1) != 0) std::strcpy(host, "?");
  put(mine.host, host);
  put(mine.gpu, device_identity(device, &err));
  mine.index = device;
  mine.ok = err.empty() ? 1 : 0;
  put(mine.err, err);
  std::vector<KeyRecord> all(world);
  boot.allgather(&mine, all.data(), sizeof(KeyRecord));
  std::vector<PeerKey> keys(world);
  for (int r = 0; r < world; ++r) keys[r] = PeerKey{all[r].host, all[r].gpu, all[r].index};
  std::string verdict;
  if (!mine.ok) {
    verdict = err;
  } else {
    verdict = peer_verdict(keys, rank, [](int a, int b) {
      int can = 0;
      return hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can != 0;
    });
    // injected (--inject-fault nopeer): this rank reports no peer access even where none is needed
    // (ranks sharing one GPU), so the decline path runs in one-GPU rehearsals too
    if (fault && fault->no_peer(rank) && verdict.empty())
      verdict = "device " + std::to_string(device) + " cannot access its peers (injected: --inject-fault nopeer)";
  }
  char vbuf[2 * kField] = {0};
  std::memcpy(vbuf, verdict.data(), std::min(verdict.size(), sizeof vbuf - 1));
  std::vector<std::array<char, 2 * kField>> vs(world);
  boot.allgather(vbuf, vs.data(), sizeof vbuf);
  std::vector<std::string> verdicts(world);
  for (int r = 0; r < world; ++r) verdicts[r] = std::string(vs[r].data());
  return agree_verdicts(verdicts);
}

}  // namespace mireduce
