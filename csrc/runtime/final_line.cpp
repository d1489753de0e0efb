// One result line, printed exactly once (final_line.hpp).
#include "mireduce/final_line.hpp"

#include <fcntl.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <mutex>

namespace mireduce {

namespace {

constexpr size_t kMaxLine = 256 * 1024;
constexpr int kSignals[] = {SIGTERM, SIGINT, SIGHUP, SIGABRT, SIGSEGV, SIGBUS, SIGFPE};
constexpr int kNumSignals = sizeof(kSignals) / sizeof(kSignals[0]);

char g_buf[2][kMaxLine + 1];        // double buffer: the handler reads one while arm() fills the other
size_t g_len[2] = {0, 0};
std::atomic<int> g_cur{-1};         // buffer holding the armed line, -1: none
std::atomic<bool> g_emitted{false}; // the once-guard: some thread or handler owns the line
std::atomic<bool> g_written{false}; // ... and has finished writing it
std::mutex g_arm_mu;                // serialises arm / disarm (not taken in the handler)
struct sigaction g_prev[kNumSignals];  // the handler each signal had before ours (chained to)
// The process's stdout as it was at the first arm: a later phase may route fd 1 elsewhere for a
// while (dist.stdout_to_stderr keeps RCCL's banner off stdout during the rendezvous), and the line
// must still reach the real stdout if the process dies then.
std::atomic<int> g_fd{-1};

void write_all(const char* p, size_t n) {
  const int fd = g_fd.load(std::memory_order_acquire);
  while (n > 0) {
    const ssize_t w = ::write(fd >= 0 ? fd : 1, p, n);
    if (w <= 0) return;
    p += w;
    n -= static_cast<size_t>(w);
  }
}

int slot_of(int sig) {
  for (int i = 0; i < kNumSignals; ++i)
    if (kSignals[i] == sig) return i;
  return -1;
}

void on_signal(int sig, siginfo_t* info, void* uctx);

bool is_ours(const struct sigaction& sa) {
  return (sa.sa_flags & SA_SIGINFO) && sa.sa_sigaction == on_signal;
}

// The armed line (once), then whatever handled the signal before us: Python's SIGINT handler
// (KeyboardInterrupt), faulthandler / a crash reporter, or the default action (re-raised).
void on_signal(int sig, siginfo_t* info, void* uctx) {
  const int k = slot_of(sig);
  struct sigaction prev{};
  if (k >= 0) prev = g_prev[k];
  // A signal the process ignored before us stays ignored: it must not take the once-guard (the
  // process lives on and its real line must still print), ADVICE r5. (install() skips ignored
  // signals; this covers a disposition recorded otherwise.)
  if (k >= 0 && !(prev.sa_flags & SA_SIGINFO) && prev.sa_handler == SIG_IGN) return;
  const int c = g_cur.load(std::memory_order_acquire);
  if (!g_emitted.exchange(true)) {
    if (c >= 0) write_all(g_buf[c], g_len[c]);
    g_written.store(true, std::memory_order_release);
  } else {
    // another thread is printing the line right now (emit_final_line, or a watchdog): let it
    // finish before the process can die, for at most ~2 s (nanosleep is async-signal-safe)
    const struct timespec ts = {0, 1000000};
    for (int i = 0; i < 2000 && !g_written.load(std::memory_order_acquire); ++i) ::nanosleep(&ts, nullptr);
  }
  if (k < 0 || (!(prev.sa_flags & SA_SIGINFO) && prev.sa_handler == SIG_DFL)) {
    ::signal(sig, SIG_DFL);
    ::raise(sig);
    return;
  }
  // chain: the previous handler runs as it would have (it stays installed for the next signal)
  ::sigaction(sig, &prev, nullptr);
  if (prev.sa_flags & SA_SIGINFO) prev.sa_sigaction(sig, info, uctx);
  else prev.sa_handler(sig);
}

// (Re)install: a handler someone installed after ours (e.g. a library initialised since the last
// arm) becomes the one we chain to, and ours goes back on top.
void install() {
  for (int i = 0; i < kNumSignals; ++i) {
    struct sigaction cur;
    if (::sigaction(kSignals[i], nullptr, &cur) != 0 || is_ours(cur)) continue;
    // ignored (SIGHUP under nohup, SIGINT of a background job): not a termination, leave it so
    if (!(cur.sa_flags & SA_SIGINFO) && cur.sa_handler == SIG_IGN) continue;
    g_prev[i] = cur;
    struct sigaction sa;
    std::memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_signal;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_SIGINFO;
    ::sigaction(kSignals[i], &sa, nullptr);
  }
}

}  // namespace

void arm_final_line(const std::string& line) {
  std::lock_guard<std::mutex> lk(g_arm_mu);
  if (g_fd.load() < 0) g_fd.store(::fcntl(1, F_DUPFD_CLOEXEC, 3), std::memory_order_release);
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
  g_written.store(true, std::memory_order_release);
  return true;
}

bool final_line_emitted() { return g_emitted.load(); }

}  // namespace mireduce
