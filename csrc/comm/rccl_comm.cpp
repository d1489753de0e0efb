// RCCL communicator wrapper; see comm.hpp.
#include <hip/hip_runtime_api.h>

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <string>
#include <thread>

#include "mireduce/check.hpp"
#include "mireduce/comm.hpp"

namespace mireduce {

namespace {
RcclComm* g_abort_comm = nullptr;
void abort_hook(int) {
  if (g_abort_comm) g_abort_comm->abort();
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error(std::string(what) + ": " + nccl_error_string(r));
}
}  // namespace

std::string nccl_error_string(ncclResult_t r) { return ncclGetErrorString(r); }

ncclDataType_t nccl_type(DType t) {
  switch (t) {
    case DType::Int32: return ncclInt32;
    case DType::Int64: return ncclInt64;
    case DType::Float32: return ncclFloat32;
    case DType::Float64: return ncclFloat64;
    case DType::BFloat16: return ncclBfloat16;
    case DType::Float16: return ncclFloat16;
  }
  return ncclFloat64;
}

ncclRedOp_t nccl_op(Op o) {
  switch (o) {
    case Op::Sum: return ncclSum;
    case Op::Min: return ncclMin;
    case Op::Max: return ncclMax;
    // fused ops: ranks exchange already-transformed partials (sum of x^2, max |x|), combined like SUM / MAX
    case Op::SumSq: return ncclSum;
    case Op::AbsMax: return ncclMax;
  }
  return ncclSum;
}

namespace {
// RCCL prints a version banner on stdout when a communicator is created; our stdout carries
// reduce.c-format data lines, so the banner is sent to stderr instead.
class StdoutToStderr {
 public:
  StdoutToStderr() {
    std::fflush(stdout);
    saved_ = dup(1);
    if (saved_ >= 0) dup2(2, 1);
  }
  ~StdoutToStderr() {
    std::fflush(stdout);
    if (saved_ >= 0) {
      dup2(saved_, 1);
      close(saved_);
    }
  }

 private:
  int saved_ = -1;
};
}  // namespace

RcclComm::RcclComm(TcpBootstrap& boot, int device) : rank_(boot.rank()), world_(boot.world()) {
  (void)device;
  ncclUniqueId id;
  StdoutToStderr quiet;
  if (rank_ == 0) check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  boot.broadcast(&id, sizeof id, 0);
  check(ncclCommInitRank(&comm_, world_, id, rank_), "ncclCommInitRank");
}

RcclComm::~RcclComm() {
  if (g_abort_comm == this) g_abort_comm = nullptr;
  if (comm_) ncclCommDestroy(comm_);
}

void RcclComm::allreduce(const void* send, void* recv, size_t count, DType t, Op o, hipStream_t s) {
  check(ncclAllReduce(send, recv, count, nccl_type(t), nccl_op(o), comm_, s), "ncclAllReduce");
}

void RcclComm::reduce(const void* send, void* recv, size_t count, DType t, Op o, int root, hipStream_t s) {
  check(ncclReduce(send, recv, count, nccl_type(t), nccl_op(o), root, comm_, s), "ncclReduce");
}

void RcclComm::broadcast(const void* send, void* recv, size_t count, DType t, int root, hipStream_t s) {
  check(ncclBroadcast(send, recv, count, nccl_type(t), root, comm_, s), "ncclBroadcast");
}

void RcclComm::synchronize(hipStream_t s, double timeout_s) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (true) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) throw Error(std::string("stream error: ") + hipGetErrorString(q));
    ncclResult_t async = ncclSuccess;
    check(ncclCommGetAsyncError(comm_, &async), "ncclCommGetAsyncError");
    if (async != ncclSuccess && async != ncclInProgress) {
      abort();
      throw Error("RCCL async error: " + nccl_error_string(async));
    }
    if (std::chrono::steady_clock::now() > deadline) {
      abort();
      throw Error("RCCL collective timed out");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

void RcclComm::abort() {
  if (comm_) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

int RcclComm::version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

RcclGroup::RcclGroup(const std::vector<int>& devices) : devices_(devices), comms_(devices.size(), nullptr) {
  StdoutToStderr quiet;
  check(ncclCommInitAll(comms_.data(), static_cast<int>(devices_.size()), devices_.data()), "ncclCommInitAll");
}

RcclGroup::~RcclGroup() {
  for (ncclComm_t c : comms_)
    if (c) ncclCommDestroy(c);
}

void RcclGroup::allreduce(const std::vector<const void*>& send, const std::vector<void*>& recv, size_t count, DType t,
                          Op o, const std::vector<hipStream_t>& streams) {
  check(ncclGroupStart(), "ncclGroupStart");
  for (size_t i = 0; i < comms_.size(); ++i)
    check(ncclAllReduce(send[i], recv[i], count, nccl_type(t), nccl_op(o), comms_[i], streams[i]), "ncclAllReduce");
  check(ncclGroupEnd(), "ncclGroupEnd");
}

void RcclGroup::reduce(const std::vector<const void*>& send, const std::vector<void*>& recv, size_t count, DType t,
                       Op o, int root, const std::vector<hipStream_t>& streams) {
  check(ncclGroupStart(), "ncclGroupStart");
  for (size_t i = 0; i < comms_.size(); ++i)
    check(ncclReduce(send[i], recv[i], count, nccl_type(t), nccl_op(o), root, comms_[i], streams[i]), "ncclReduce");
  check(ncclGroupEnd(), "ncclGroupEnd");
}

void install_comm_abort_hook(RcclComm* comm) {
  g_abort_comm = comm;
  set_fatal_hook(comm ? abort_hook : nullptr);
}

}  // namespace mireduce
