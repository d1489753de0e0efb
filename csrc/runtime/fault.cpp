// Fault injection; see fault.hpp.
#include "mireduce/fault.hpp"

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <thread>

namespace mireduce {

namespace {

long to_long(const std::string& s, const std::string& spec) {
  if (s.empty()) throw std::invalid_argument("bad fault spec '" + spec + "': empty number");
  char* end = nullptr;
  const long v = std::strtol(s.c_str(), &end, 10);
  if (*end != '\0' || v < 0) throw std::invalid_argument("bad fault spec '" + spec + "': '" + s + "' is not a count");
  return v;
}

}  // namespace

FaultSpec parse_fault_spec(const std::string& spec) {
  FaultSpec f;
  if (spec.empty() || spec == "none") return f;
  std::string kind = spec, rank, step;
  const size_t colon = kind.find(':');
  if (colon != std::string::npos) {
    step = kind.substr(colon + 1);
    kind = kind.substr(0, colon);
  }
  const size_t at = kind.find('@');
  if (at != std::string::npos) {
    rank = kind.substr(at + 1);
    kind = kind.substr(0, at);
  }
  if (kind == "exit") f.kind = FaultSpec::Kind::Exit;
  else if (kind == "hang") f.kind = FaultSpec::Kind::Hang;
  else if (kind == "corrupt") f.kind = FaultSpec::Kind::Corrupt;
  else if (kind == "nopeer") f.kind = FaultSpec::Kind::NoPeer;
  else if (kind.rfind("delay=", 0) == 0) {
    f.kind = FaultSpec::Kind::Delay;
    f.delay_ms = static_cast<int>(to_long(kind.substr(6), spec));
  } else {
    throw std::invalid_argument("bad fault spec '" + spec + "': kind must be exit, hang, corrupt, delay=<ms> or nopeer");
  }
  if (at != std::string::npos) f.rank = static_cast<int>(to_long(rank, spec));
  if (colon != std::string::npos) f.step = to_long(step, spec);
  return f;
}

FaultInjector FaultInjector::from_flag_or_env(const std::string& flag) {
  if (!flag.empty()) return FaultInjector(parse_fault_spec(flag));
  const char* e = std::getenv("MIREDUCE_INJECT_FAULT");
  return FaultInjector(parse_fault_spec(e ? e : ""));
}

bool FaultInjector::at(int rank, long step, const char* site) {
  if (fired_ || spec_.kind == FaultSpec::Kind::None || spec_.kind == FaultSpec::Kind::NoPeer || rank != spec_.rank ||
      step != spec_.step)
    return false;
  fired_ = true;
  switch (spec_.kind) {
    case FaultSpec::Kind::Exit:
      std::fprintf(stderr, "[fault] rank %d exits at %s step %ld\n", rank, site, step);
      std::fflush(stderr);
      std::fflush(stdout);
      ::_exit(3);
    case FaultSpec::Kind::Hang:
      std::fprintf(stderr, "[fault] rank %d hangs at %s step %ld\n", rank, site, step);
      std::fflush(stderr);
      for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
    case FaultSpec::Kind::Delay:
      std::fprintf(stderr, "[fault] rank %d delays %d ms at %s step %ld\n", rank, spec_.delay_ms, site, step);
      std::this_thread::sleep_for(std::chrono::milliseconds(spec_.delay_ms));
      return false;
    case FaultSpec::Kind::Corrupt:
      std::fprintf(stderr, "[fault] rank %d corrupts its result at %s step %ld\n", rank, site, step);
      return true;
    case FaultSpec::Kind::NoPeer:  // not a step fault (no_peer())
    case FaultSpec::Kind::None:
      break;
  }
  return false;
}

}  // namespace mireduce
