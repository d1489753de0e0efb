"""Fault injection for failure-detection tests — the Python twin of csrc/include/mireduce/fault.hpp.

The reference has no failure handling (MPI return codes ignored, mpi/reduce.c:32-106; a stuck
rank stalls until the SLURM walltime, mpi/submit_all.sh:4). Here every cross-rank wait has a
deadline (process-group timeout, bootstrap deadline, RCCL async-error polling) and results are
verified; ``--inject-fault`` provokes the failures those mechanisms exist for.

Spec: ``KIND[@RANK][:STEP]`` with KIND = exit | hang | corrupt | delay=<ms>; RANK defaults to 1,
STEP to 0 (also read from ``MIREDUCE_INJECT_FAULT``).
"""
from __future__ import annotations

import os
import sys
import time
from dataclasses import dataclass
from typing import Optional

__all__ = ["FaultSpec", "FaultInjector", "parse_fault_spec"]

KINDS = ("none", "exit", "hang", "corrupt", "delay")


@dataclass(frozen=True)
class FaultSpec:
    kind: str = "none"
    rank: int = 1
    step: int = 0
    delay_ms: int = 0


def _count(s: str, spec: str) -> int:
    if not s.isdigit():
        raise ValueError(f"bad fault spec {spec!r}: {s!r} is not a count")
    return int(s)


def parse_fault_spec(spec: Optional[str]) -> FaultSpec:
    if not spec or spec == "none":
        return FaultSpec()
    kind, step, rank = spec, None, None
    if ":" in kind:
        kind, step = kind.split(":", 1)
    if "@" in kind:
        kind, rank = kind.split("@", 1)
    delay = 0
    if kind.startswith("delay="):
        delay = _count(kind[len("delay="):], spec)
        kind = "delay"
    if kind not in KINDS[1:]:
        raise ValueError(f"bad fault spec {spec!r}: kind must be exit, hang, corrupt or delay=<ms>")
    return FaultSpec(kind, 1 if rank is None else _count(rank, spec), 0 if step is None else _count(step, spec), delay)


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

    def at(self, rank: int, step: int, site: str = "step") -> bool:
        """Fire once at (rank, step). Returns True iff the caller must corrupt its local result."""
        s = self.spec
        if self.fired or s.kind == "none" or rank != s.rank or step != s.step:
            return False
        self.fired = True
        print(f"[fault] rank {rank} {s.kind} at {site} {step}", file=sys.stderr, flush=True)
        if s.kind == "exit":
            sys.stdout.flush()
            os._exit(3)
        if s.kind == "hang":
            while True:
                time.sleep(1)
        if s.kind == "delay":
            time.sleep(s.delay_ms / 1000.0)
            return False
        return s.kind == "corrupt"
