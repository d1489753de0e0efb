// One result line, printed exactly once (final_line.hpp).
#include "mireduce/final_line.hpp"

#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <mutex>

namespace mireduce {

namespace {

constexpr size_t kMaxLine = 256 * 1024;
char g_buf[2][kMaxLine + 1];        // double buffer: the handler reads one while arm() fills the other
size_t g_len[2] = {0, 0};
std::atomic<int> g_cur{-1};         // buffer holding the armed line, -1: none
std::atomic<bool> g_emitted{false}; // the once-guard
std::mutex g_arm_mu;                // serialises arm / disarm (not taken in the handler)
std::atomic<bool> g_installed{false};

void write_all(const char* p, size_t n) {
  while (n > 0) {
    const ssize_t w = ::write(1, p, n);
    if (w <= 0) return;
    p += w;
    n -= static_cast<size_t>(w);
  }
}

void on_signal(int sig) {
  const int c = g_cur.load(std::memory_order_acquire);
  if (c >= 0 && !g_emitted.exchange(true)) write_all(g_buf[c], g_len[c]);
  ::signal(sig, SIG_DFL);
  ::raise(sig);
}

void install() {
  if (g_installed.exchange(true)) return;
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_signal;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESETHAND;
  for (int s : {SIGTERM, SIGINT, SIGHUP, SIGABRT, SIGSEGV, SIGBUS, SIGFPE}) ::sigaction(s, &sa, nullptr);
}

}  // namespace

void arm_final_line(const std::string& line) {
  std::lock_guard<std::mutex> lk(g_arm_mu);
  install();
  const int next = g_cur.load() == 0 ? 1 : 0;
  const size_t n = line.size() < kMaxLine ? line.size() : kMaxLine;
  std::memcpy(g_buf[next], line.data(), n);
  g_buf[next][n] = '\n';
  g_len[next] = n + 1;
  g_cur.store(next, std::memory_order_release);
}

void disarm_final_line() {
  std::lock_guard<std::mutex> lk(g_arm_mu);
  g_cur.store(-1, std::memory_order_release);
}

bool emit_final_line(const std::string& line) {
  if (g_emitted.exchange(true)) return false;
  std::string s = line;
  s += '\n';
  write_all(s.data(), s.size());
  return true;
}

bool final_line_emitted() { return g_emitted.load(); }

}  // namespace mireduce
