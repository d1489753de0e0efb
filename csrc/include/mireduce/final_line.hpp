// The benchmark's one result line, printed exactly once even when the process is killed.
//
// bench.py's contract is ONE JSON line from rank 0. After the headline is measured, the run goes
// on (extras, teardown); if it then dies — torchrun SIGTERMs every rank when one rank fails, a GPU
// memory fault aborts the process (SIGABRT), a segfault — a line printed only at the end would be
// lost with it. `arm_final_line` keeps the line to print in that case (updated as the run
// progresses, e.g. with the extras finished so far); signal handlers for SIGTERM, SIGINT, SIGHUP,
// SIGABRT, SIGSEGV, SIGBUS and SIGFPE write the armed line to fd 1 with write(2) (async-signal-
// safe) and then hand the signal to whatever handled it before (Python's SIGINT handler, a
// faulthandler, ...) or, if that was the default action, re-raise it. Every arm re-installs the
// handlers if a library replaced them since (the replacement becomes the one chained to).
// `emit_final_line` is the normal path; a process-wide once-guard makes sure that whichever comes
// first is the only line printed, and a handler that finds another thread mid-way through printing
// waits (bounded, ~2 s) for it to finish before the process can die. The line goes to stdout as it
// was at the first arm (a duplicate of fd 1 taken then), even if fd 1 is routed elsewhere later.
#pragma once

#include <string>

namespace mireduce {

// Install the handlers (idempotent) and make `line` (without the trailing newline) the line to
// print if the process is terminated before emit_final_line(). Lines longer than 256 KiB are
// truncated. Thread-safe; the previous armed line stays valid until replaced.
void arm_final_line(const std::string& line);

// Forget the armed line (the process may now die silently: e.g. non-final phases).
void disarm_final_line();

// Print `line` + "\n" unless a line was already printed (by a signal handler or an earlier call);
// returns whether this call printed it.
bool emit_final_line(const std::string& line);

// Whether some line has been printed.
bool final_line_emitted();

}  // namespace mireduce
