// Pure peer-access verdicts (host code; no HIP): see peer_access.hpp.
#include "mireduce/peer_access.hpp"

namespace mireduce {

std::string peer_verdict(const std::vector<PeerKey>& keys, int me, const std::function<bool(int, int)>& can_access) {
  if (me < 0 || me >= static_cast<int>(keys.size())) return "rank index out of range";
  const PeerKey& mine = keys[me];
  for (int r = 0; r < static_cast<int>(keys.size()); ++r) {
    const PeerKey& k = keys[r];
    if (r == me || (k.gpu == mine.gpu && k.host == mine.host)) continue;  // itself, or the same physical GPU
    if (k.host != mine.host)
      return "rank " + std::to_string(r) + " runs on host " + k.host + ", not " + mine.host +
             " (IPC handles do not cross hosts)";
    if (k.index == mine.index)
      return "rank " + std::to_string(r) + " reports device " + std::to_string(k.index) +
             " = mine but a different GPU (" + k.gpu + " vs " + mine.gpu + ")";
    if (!can_access(mine.index, k.index))
      return "device " + std::to_string(mine.index) + " cannot access peer device " + std::to_string(k.index) +
             " (rank " + std::to_string(r) + ")";
  }
  return "";
}

std::string agree_verdicts(const std::vector<std::string>& verdicts) {
  std::string out;
  for (size_t r = 0; r < verdicts.size(); ++r) {
    if (verdicts[r].empty()) continue;
    if (!out.empty()) out += "; ";
    out += "rank " + std::to_string(r) + ": " + verdicts[r];
  }
  return out;
}

}  // namespace mireduce
