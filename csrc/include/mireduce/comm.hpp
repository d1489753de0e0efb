// Cross-rank communication for GPU ranks: RCCL over xGMI, bootstrapped over TCP.
//
// Reference: MPI_Init/Comm_rank/Comm_size + blocking MPI_Reduce on MPI_COMM_WORLD
// (mpi/reduce.c:32-34,62-63,76,90), with return codes ignored (errors fatal by default, §5.3).
// MI355X design: one process per GPU, hipSetDevice(local_rank), an
// ncclUniqueId created by rank 0 and shared with the others, then ncclCommInitRank; collectives
// are ncclAllReduce / ncclReduce / ncclBroadcast with ncclSum/Min/Max on int32/int64/f32/f64.
// The id is exchanged over a small TCP star instead of MPI_Bcast so the same binary runs under
// torchrun (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR), mpirun (PMI_RANK/PMI_SIZE/MPI_LOCALRANKID)
// or any launcher that exports those variables — and needs no MPI library.
#pragma once

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "mireduce/types.hpp"

namespace mireduce {

struct LaunchEnv {
  int rank = 0;
  int world = 1;
  int local_rank = 0;
  std::string addr = "127.0.0.1";
  int port = 29517;
  std::string launcher = "none";  // torchrun | mpich | openmpi | slurm | none
};

// Read rank/world/local-rank/rendezvous address from the environment. The bootstrap port is
// MIREDUCE_BOOTSTRAP_PORT, else MASTER_PORT + 17 (torchrun's own store owns MASTER_PORT), else
// 29517.
LaunchEnv launch_env_from_environment();

// Star-topology TCP exchange through rank 0. Blocking; every call is collective.
class TcpBootstrap {
 public:
  TcpBootstrap(const LaunchEnv& env, double timeout_s = 300.0);
  ~TcpBootstrap();
  TcpBootstrap(const TcpBootstrap&) = delete;
  TcpBootstrap& operator=(const TcpBootstrap&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  void broadcast(void* data, size_t bytes, int root = 0);
  void allgather(const void* mine, void* all, size_t bytes);  // all = world * bytes
  void barrier();
  double max_double(double v);

 private:
  int rank_ = 0, world_ = 1;
  double timeout_s_ = 300.0;  // every exchange fails after this long without progress
  int listen_fd_ = -1;
  int root_fd_ = -1;            // non-root: connection to rank 0
  std::vector<int> peer_fds_;   // rank 0: fd of rank r at [r]
};

ncclDataType_t nccl_type(DType t);
ncclRedOp_t nccl_op(Op o);
std::string nccl_error_string(ncclResult_t r);

class RcclComm {
 public:
  // Collective over all ranks of `boot`; device must already be current.
  RcclComm(TcpBootstrap& boot, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  void allreduce(const void* send, void* recv, size_t count, DType t, Op o, hipStream_t s);
  void reduce(const void* send, void* recv, size_t count, DType t, Op o, int root, hipStream_t s);
  void broadcast(const void* send, void* recv, size_t count, DType t, int root, hipStream_t s);
  // Block until `s` drains, polling ncclCommGetAsyncError; abort the communicator and throw
  // after `timeout_s` (SURVEY.md §5.3 per-collective timeout).
  void synchronize(hipStream_t s, double timeout_s = 300.0);
  void abort();
  ncclComm_t raw() const { return comm_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  static int version();

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, world_ = 1;
};

// Single-process multi-GPU communicator set (ncclCommInitAll over `devices`): the
// simpleMultiGPU / P9 layout (cuda/C/src/simpleMultiGPU/simpleMultiGPU.cpp:185-310), with the
// per-device collectives issued inside one ncclGroupStart/End.
class RcclGroup {
 public:
  explicit RcclGroup(const std::vector<int>& devices);
  ~RcclGroup();
  RcclGroup(const RcclGroup&) = delete;
  RcclGroup& operator=(const RcclGroup&) = delete;
  int size() const { return static_cast<int>(devices_.size()); }
  int device(int i) const { return devices_[i]; }
  void allreduce(const std::vector<const void*>& send, const std::vector<void*>& recv, size_t count, DType t, Op o,
                 const std::vector<hipStream_t>& streams);
  void reduce(const std::vector<const void*>& send, const std::vector<void*>& recv, size_t count, DType t, Op o,
              int root, const std::vector<hipStream_t>& streams);

 private:
  std::vector<int> devices_;
  std::vector<ncclComm_t> comms_;
};

// Register `comm` for the fatal-error hook: HIP_CHECK failures abort it before exiting.
void install_comm_abort_hook(RcclComm* comm);

}  // namespace mireduce
