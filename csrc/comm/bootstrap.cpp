// TCP bootstrap + launcher environment detection; see comm.hpp.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#include "mireduce/check.hpp"
#include "mireduce/comm.hpp"

namespace mireduce {

namespace {

const char* env(const char* k) {
  const char* v = std::getenv(k);
  return (v && *v) ? v : nullptr;
}

int env_int(const char* k, int def) {
  const char* v = env(k);
  return v ? std::atoi(v) : def;
}

void send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) throw Error(std::string("bootstrap send failed: ") + std::strerror(errno));
    c += k;
    n -= static_cast<size_t>(k);
  }
}

void recv_all(int fd, void* p, size_t n, double timeout_s) {
  char* c = static_cast<char*>(p);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (n) {
    pollfd pfd{fd, POLLIN, 0};
    const int left = static_cast<int>(std::chrono::duration<double, std::milli>(deadline - std::chrono::steady_clock::now()).count());
    if (left <= 0) throw Error("bootstrap recv timed out");
    const int pr = ::poll(&pfd, 1, left);
    if (pr < 0 && errno == EINTR) continue;
    if (pr <= 0) throw Error("bootstrap recv timed out");
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) throw Error(std::string("bootstrap peer closed: ") + (k < 0 ? std::strerror(errno) : "EOF"));
    c += k;
    n -= static_cast<size_t>(k);
  }
}

void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

}  // namespace

LaunchEnv launch_env_from_environment() {
  LaunchEnv e;
  if (env("RANK") && env("WORLD_SIZE")) {
    e.rank = env_int("RANK", 0);
    e.world = env_int("WORLD_SIZE", 1);
    e.local_rank = env_int("LOCAL_RANK", e.rank);
    e.launcher = "torchrun";
  } else if (env("PMI_RANK") && env("PMI_SIZE")) {
    e.rank = env_int("PMI_RANK", 0);
    e.world = env_int("PMI_SIZE", 1);
    e.local_rank = env_int("MPI_LOCALRANKID", e.rank);
    e.launcher = "mpich";
  } else if (env("OMPI_COMM_WORLD_RANK")) {
    e.rank = env_int("OMPI_COMM_WORLD_RANK", 0);
    e.world = env_int("OMPI_COMM_WORLD_SIZE", 1);
    e.local_rank = env_int("OMPI_COMM_WORLD_LOCAL_RANK", e.rank);
    e.launcher = "openmpi";
  } else if (env("SLURM_PROCID") && env("SLURM_NTASKS")) {
    e.rank = env_int("SLURM_PROCID", 0);
    e.world = env_int("SLURM_NTASKS", 1);
    e.local_rank = env_int("SLURM_LOCALID", e.rank);
    e.launcher = "slurm";
  }
  if (const char* a = env("MASTER_ADDR")) e.addr = a;
  if (const char* p = env("MIREDUCE_BOOTSTRAP_PORT")) e.port = std::atoi(p);
  else if (const char* p2 = env("MASTER_PORT")) e.port = std::atoi(p2) + 17;
  return e;
}

TcpBootstrap::TcpBootstrap(const LaunchEnv& env_, double timeout_s) : rank_(env_.rank), world_(env_.world) {
  if (world_ <= 1) return;
  if (const char* t = env("MIREDUCE_BOOTSTRAP_TIMEOUT")) timeout_s = std::atof(t);  // failure detection knob
  timeout_s_ = timeout_s;
  addrinfo hints{};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  const std::string port = std::to_string(env_.port);
  if (getaddrinfo(env_.addr.c_str(), port.c_str(), &hints, &res) != 0 || !res)
    throw Error("bootstrap: cannot resolve " + env_.addr);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  if (rank_ == 0) {
    listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(static_cast<uint16_t>(env_.port));
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0 || ::listen(listen_fd_, world_) != 0) {
      freeaddrinfo(res);
      throw Error("bootstrap: cannot listen on port " + port + ": " + std::strerror(errno));
    }
    peer_fds_.assign(world_, -1);
    for (int got = 1; got < world_;) {
      pollfd pfd{listen_fd_, POLLIN, 0};
      const int left = static_cast<int>(std::chrono::duration<double, std::milli>(deadline - std::chrono::steady_clock::now()).count());
      if (left <= 0 || ::poll(&pfd, 1, left) <= 0) {
        freeaddrinfo(res);
        throw Error("bootstrap: timed out waiting for peers");
      }
      const int fd = ::accept(listen_fd_, nullptr, nullptr);
      if (fd < 0) continue;
      set_nodelay(fd);
      int32_t r = -1;
      recv_all(fd, &r, sizeof r, timeout_s);
      if (r <= 0 || r >= world_ || peer_fds_[r] != -1) {
        ::close(fd);
        freeaddrinfo(res);
        throw Error("bootstrap: bad or duplicate rank " + std::to_string(r));
      }
      peer_fds_[r] = fd;
      ++got;
    }
  } else {
    while (true) {
      root_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
      if (::connect(root_fd_, res->ai_addr, res->ai_addrlen) == 0) break;
      ::close(root_fd_);
      root_fd_ = -1;
      if (std::chrono::steady_clock::now() > deadline) {
        freeaddrinfo(res);
        throw Error("bootstrap: cannot connect to " + env_.addr + ":" + port);
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    set_nodelay(root_fd_);
    const int32_t r = rank_;
    send_all(root_fd_, &r, sizeof r);
  }
  freeaddrinfo(res);
}

TcpBootstrap::~TcpBootstrap() {
  for (int fd : peer_fds_)
    if (fd >= 0) ::close(fd);
  if (root_fd_ >= 0) ::close(root_fd_);
  if (listen_fd_ >= 0) ::close(listen_fd_);
}

void TcpBootstrap::broadcast(void* data, size_t bytes, int root) {
  if (world_ <= 1) return;
  if (root != 0) {  // relay through rank 0
    if (rank_ == root) send_all(root_fd_, data, bytes);
    if (rank_ == 0) recv_all(peer_fds_[root], data, bytes, timeout_s_);
  }
  if (rank_ == 0) {
    for (int r = 1; r < world_; ++r) send_all(peer_fds_[r], data, bytes);
  } else {
    recv_all(root_fd_, data, bytes, timeout_s_);
  }
}

void TcpBootstrap::allgather(const void* mine, void* all, size_t bytes) {
  char* out = static_cast<char*>(all);
  std::memcpy(out + static_cast<size_t>(rank_) * bytes, mine, bytes);
  if (world_ <= 1) return;
  if (rank_ == 0) {
    for (int r = 1; r < world_; ++r) recv_all(peer_fds_[r], out + static_cast<size_t>(r) * bytes, bytes, timeout_s_);
    for (int r = 1; r < world_; ++r) send_all(peer_fds_[r], out, bytes * world_);
  } else {
    send_all(root_fd_, mine, bytes);
    recv_all(root_fd_, out, bytes * world_, timeout_s_);
  }
}

void TcpBootstrap::barrier() {
  char c = 0;
  std::vector<char> all(world_);
  allgather(&c, all.data(), 1);
}

double TcpBootstrap::max_double(double v) {
  std::vector<double> all(world_);
  allgather(&v, all.data(), sizeof v);
  double m = all[0];
  for (double x : all) m = x > m ? x : m;
  return m;
}

}  // namespace mireduce
