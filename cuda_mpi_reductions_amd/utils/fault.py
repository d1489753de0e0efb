"""Fault injection for failure-detection tests — the Python twin of csrc/include/mireduce/fault.hpp.

The reference has no failure handling (MPI return codes ignored, mpi/reduce.c:32-106; a stuck
rank stalls until the SLURM walltime, mpi/submit_all.sh:4). Here every cross-rank wait has a
deadline (process-group timeout, bootstrap deadline, RCCL async-error polling) and results are
verified; ``--inject-fault`` provokes the failures those mechanisms exist for.

Spec: ``KIND[@RANK][:STEP][/SITE]`` with KIND = exit | hang | raise | corrupt | delay=<ms> | mailbox;
RANK defaults to 1, STEP to 0, SITE to ``step`` (also read from ``MIREDUCE_INJECT_FAULT``).

* SITE ``step``: the measured steps of the headline (bench.py counts warm-up steps first);
  ``extras``: the steps of bench.py's after-headline candidates (pipelined / RCCL measurements) —
  a hang there must still leave a printed, verified headline (the extras watchdog);
  ``teardown``: just before the process-group teardown that follows the printed line (STEP is
  ignored) — a hang there must end within the teardown deadline with the headline's status;
  ``capture``: inside bench.py's replay probe of captured collective steps (STEP ignored) — a
  probe that misses its deadline on one rank must send every rank to eager issue, and the
  headline must still be measured and verified.
  ``init``: before the rank arms its result line or joins the process group (STEP ignored) — a
  rank that hangs there must still end the job within the headline deadline with exactly one
  diagnostic line (rank 0's, or the self-spawning parent's when rank 0 itself dies there).
  ``canary`` / ``selfcheck`` / ``tune`` (STEP ignored): bench.py's optional headline stages — the
  fused finish's canary (after this rank's helper ended, before the verdicts are agreed), its
  self-check (before the three checked steps) and the per-rank plan tuning (before the candidates
  are measured). A failure there on any rank must become an agreed fallback (RCCL combine / the
  tuned default plan) with the headline still measured, or — for a rank that dies or hangs — one
  diagnostic line naming the stage (bench.py, parallel.dist.agree).
* KIND ``raise``: the rank raises :class:`InjectedFault` (a Python-level failure of that stage,
  e.g. a plan the native layer rejects or an IPC error) instead of exiting or hanging.
* KIND ``mailbox``: rank RANK fails to create its fused-finish mailbox
  (:func:`parallel.xrank.open_channel`); every rank must then agree on the RCCL fallback.
"""
from __future__ import annotations

import os
import sys
import time
from dataclasses import dataclass
from typing import Optional

__all__ = ["FaultSpec", "FaultInjector", "InjectedFault", "parse_fault_spec"]

KINDS = ("none", "exit", "hang", "raise", "corrupt", "delay", "mailbox")
SITES = ("step", "extras", "teardown", "capture", "init", "canary", "selfcheck", "tune")
# sites that fire once per run wherever they are reached (their STEP is ignored)
_STEPLESS = ("capture", "init", "teardown", "canary", "selfcheck", "tune")


class InjectedFault(RuntimeError):
    """The exception a ``raise`` fault throws."""


@dataclass(frozen=True)
class FaultSpec:
    kind: str = "none"
    rank: int = 1
    step: int = 0
    delay_ms: int = 0
    site: str = "step"


def _count(s: str, spec: str) -> int:
    if not s.isdigit():
        raise ValueError(f"bad fault spec {spec!r}: {s!r} is not a count")
    return int(s)


def parse_fault_spec(spec: Optional[str]) -> FaultSpec:
    if not spec or spec == "none":
        return FaultSpec()
    kind, step, rank, site = spec, None, None, "step"
    if "/" in kind:
        kind, site = kind.split("/", 1)
        if site not in SITES:
            raise ValueError(f"bad fault spec {spec!r}: site must be one of {', '.join(SITES)}")
    if ":" in kind:
        kind, step = kind.split(":", 1)
    if "@" in kind:
        kind, rank = kind.split("@", 1)
    delay = 0
    if kind.startswith("delay="):
        delay = _count(kind[len("delay="):], spec)
        kind = "delay"
    if kind not in KINDS[1:]:
        raise ValueError(f"bad fault spec {spec!r}: kind must be exit, hang, raise, corrupt, delay=<ms> or mailbox")
    return FaultSpec(kind, 1 if rank is None else _count(rank, spec), 0 if step is None else _count(step, spec), delay,
                     site)


class FaultInjector:
    def __init__(self, spec: Optional[FaultSpec] = None):
        self.spec = spec or FaultSpec()
        self.fired = False

    @classmethod
    def from_flag_or_env(cls, flag: Optional[str]) -> "FaultInjector":
        return cls(parse_fault_spec(flag if flag else os.environ.get("MIREDUCE_INJECT_FAULT")))

    @property
    def enabled(self) -> bool:
        return self.spec.kind != "none"

    def on(self, site: str = "step") -> bool:
        """Whether a step fault is armed at ``site`` (the bench issues such steps eagerly)."""
        return self.spec.kind not in ("none", "mailbox") and self.spec.site == site

    def mailbox(self, rank: int) -> bool:
        """Whether ``rank`` must fail to create its fused-finish mailbox (every attempt)."""
        return self.spec.kind == "mailbox" and rank == self.spec.rank

    def at(self, rank: int, step: int, site: str = "step", label: str = "") -> bool:
        """Fire once at (rank, step) of ``site``. Returns True iff the caller must corrupt its local
        result."""
        s = self.spec
        if self.fired or not self.on(site) or rank != s.rank or (step != s.step and site not in _STEPLESS):
            return False
        self.fired = True
        print(f"[fault] rank {rank} {s.kind} at {label or site} {step}", file=sys.stderr, flush=True)
        if s.kind == "exit":
            sys.stdout.flush()
            os._exit(3)
        if s.kind == "hang":
            while True:
                time.sleep(1)
        if s.kind == "raise":
            raise InjectedFault(f"injected fault at {label or site} (rank {rank})")
        if s.kind == "delay":
            time.sleep(s.delay_ms / 1000.0)
            return False
        return s.kind == "corrupt"
