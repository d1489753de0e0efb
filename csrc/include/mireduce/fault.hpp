// Fault injection for failure-detection tests ("--inject-fault").
//
// The reference has no failure handling at all: MPI return codes are ignored (mpi/reduce.c:32-106,
// default MPI_ERRORS_ARE_FATAL) and a stuck rank simply stalls the job until the SLURM walltime
// (mpi/submit_all.sh:4). Here every cross-rank wait has a deadline; this module lets tests
// provoke the failures those deadlines exist for.
//
// Spec grammar (flag --inject-fault=SPEC or env MIREDUCE_INJECT_FAULT=SPEC):
//   KIND[@RANK][:STEP]      KIND = exit | hang | corrupt | delay=<ms>
// RANK defaults to 1 (0 when the job has one rank is handled by the caller), STEP to 0.
//   exit     the rank leaves with status 3 (a crashed peer)
//   hang     the rank stops making progress (sleeps; killed by the launcher or a deadline)
//   corrupt  at() returns true once: the caller perturbs its local result (verification must fail)
//   delay    the rank sleeps <ms> once (a straggler; results stay correct)
//   nopeer   the rank's peer-access query answers "no" for every peer device (the IPC-mapped
//            paths must then decline on every rank before mapping anything; STEP ignored)
#pragma once

#include <string>

namespace mireduce {

struct FaultSpec {
  enum class Kind { None, Exit, Hang, Corrupt, Delay, NoPeer };
  Kind kind = Kind::None;
  int rank = 1;
  long step = 0;
  int delay_ms = 0;
};

// Throws std::invalid_argument on a malformed spec (host-only: also linked into reduce_mpi). Empty spec -> Kind::None.
FaultSpec parse_fault_spec(const std::string& spec);

class FaultInjector {
 public:
  FaultInjector() = default;
  explicit FaultInjector(const FaultSpec& s) : spec_(s) {}
  // Spec from `flag` if non-empty, else from MIREDUCE_INJECT_FAULT.
  static FaultInjector from_flag_or_env(const std::string& flag);
  bool enabled() const { return spec_.kind != FaultSpec::Kind::None; }
  const FaultSpec& spec() const { return spec_; }
  // Call at each numbered step; fires once when (rank, step) match. Returns true iff the caller
  // must corrupt its local result now. `site` names the call site in the log line.
  bool at(int rank, long step, const char* site);
  // Whether `rank` must report no peer access (Kind::NoPeer; every query, not once).
  bool no_peer(int rank) const { return spec_.kind == FaultSpec::Kind::NoPeer && rank == spec_.rank; }

 private:
  FaultSpec spec_;
  bool fired_ = false;
};

}  // namespace mireduce
