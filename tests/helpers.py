"""Shared helpers for the CPU test suite."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")
MPIRUN = "/opt/conda/bin/mpirun"

_built = False


def ensure_built():
    """Build the native tree once per session (no-op when up to date)."""
    global _built
    if not _built:
        subprocess.run(["make", "-C", ROOT, "-j8", "all"], check=True, stdout=subprocess.DEVNULL)
        _built = True


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(cmd, timeout=300, cwd=None, env=None):
    e = dict(os.environ)
    if env:
        e.update(env)
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=cwd, env=e)


def torchrun(nproc, script_args, timeout=600, cwd=None, env=None):
    master = free_port()
    boot = free_port()
    while boot == master:
        boot = free_port()
    # The native TCP bootstrap (csrc/comm/bootstrap.cpp) would otherwise listen on MASTER_PORT + 17,
    # which nobody checked was free (a busy port there failed a run on the GPU box).
    e = {"MIREDUCE_BOOTSTRAP_PORT": str(boot)}
    if env:
        e.update(env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(master)] + script_args
    return run(cmd, timeout=timeout, cwd=cwd, env=e)


def bench_record(stdout: str) -> dict:
    """bench.py's result as tests read it: the (first) JSON line on stdout, merged with the extras
    sidecar the line names (``summary.extras_file``, same ``summary.run``): the line's keys win, and
    the sidecar's ``config_detail`` (long descriptions, kernel plan, topology) is folded into
    ``config`` so both can be asserted on in one place."""
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    d = json.loads(lines[0])
    path = (d.get("summary") or {}).get("extras_file")
    if not path or not os.path.exists(path):
        return d
    with open(path) as f:
        side = json.load(f)
    if (side.get("summary") or {}).get("run") != d["summary"].get("run"):
        return d
    merged = dict(side)
    merged.update(d)
    merged["config"] = {**(side.get("config_detail") or {}), **d.get("config", {})}
    return merged
