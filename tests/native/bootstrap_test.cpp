// Multi-process test of the TCP bootstrap used to share the ncclUniqueId (csrc/comm/bootstrap.cpp).
// Launch: torchrun --nproc-per-node=N --no-python build/bin/bootstrap_test
#include <cstdio>
#include <cstring>
#include <vector>

#include "mireduce/check.hpp"
#include "mireduce/comm.hpp"
#include "mireduce/fault.hpp"

using namespace mireduce;

int run(const LaunchEnv& env);

int main() {
  LaunchEnv env = launch_env_from_environment();
  try {
    return run(env);
  } catch (const Error& e) {  // failure detection: a missing peer is an error, never a hang
    std::fprintf(stderr, "bootstrap_test rank %d: %s\n", env.rank, e.what());
    return 2;
  }
}

// MIREDUCE_INJECT_FAULT=KIND@RANK:STEP fires before exchange STEP (0..4) on RANK: the other
// ranks must fail with a bootstrap error (peer closed / timed out), never hang.
int run(const LaunchEnv& env) {
  FaultInjector fault = FaultInjector::from_flag_or_env("");
  TcpBootstrap boot(env, 60.0);
  fault.at(env.rank, 0, "bootstrap");
  int ok = 1;
  char id[128];
  for (int i = 0; i < 128; ++i) id[i] = env.rank == 0 ? static_cast<char>(i * 7 + 3) : 0;
  boot.broadcast(id, sizeof id, 0);
  for (int i = 0; i < 128; ++i) ok &= id[i] == static_cast<char>(i * 7 + 3);
  fault.at(env.rank, 1, "bootstrap");
  int last = env.world - 1;
  double payload = env.rank == last ? 42.5 : 0.0;
  boot.broadcast(&payload, sizeof payload, last);  // non-zero root is relayed through rank 0
  ok &= payload == 42.5;
  fault.at(env.rank, 2, "bootstrap");
  std::vector<int> all(env.world);
  int mine = env.rank * 10;
  boot.allgather(&mine, all.data(), sizeof mine);
  for (int r = 0; r < env.world; ++r) ok &= all[r] == r * 10;
  fault.at(env.rank, 3, "bootstrap");
  boot.barrier();
  fault.at(env.rank, 4, "bootstrap");
  ok &= boot.max_double(static_cast<double>(env.rank)) == static_cast<double>(env.world - 1);
  std::vector<int> oks(env.world);
  boot.allgather(&ok, oks.data(), sizeof ok);
  int all_ok = 1;
  for (int v : oks) all_ok &= v;
  if (env.rank == 0) std::printf("bootstrap_test world=%d launcher=%s %s\n", env.world, env.launcher.c_str(), all_ok ? "PASSED" : "FAILED");
  return all_ok ? 0 : 1;
}
