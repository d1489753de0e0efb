"""Canary run of the fused cross-rank finish in throw-away child processes.

The fused finish (:mod:`.xrank`) stores into and polls peers' IPC-mapped GPU memory from inside the
reduction kernel. Every rank agrees on peer access before mapping (:mod:`.topology`), device waits
are bounded and results are self-checked — but a fault of the mapping itself (a GPU memory-access
fault) would abort the process, and with it the measurement it was meant to serve. So before a
benchmark process touches a peer's memory, :func:`fused_canary` has one helper process per rank
run the same exchange end to end: a private gloo group over a TCPStore that rank 0 serves for the
canary on a free port, a channel, three fused launches of a 1-element-per-rank-distinguishable array, and a
check of every result, the error words and a final barrier (nobody unmaps while a peer still
polls). Each rank waits for its helper (bounded), and the verdicts are agreed over the real
process group: any failure — a crash, a timeout, a wrong value — makes every rank decline the
fused finish together (bench.py then combines over RCCL). The helpers never share a process with
the benchmark, so whatever faults in them cannot take the benchmark down.

Reference: the vendored simpleP2P checks peer access and then actually exercises the peer path
(a kernel reading the other GPU's buffer, verified) before reporting bandwidth
(cuda/C/src/simpleP2P/simpleP2P.cu:250-275,330-350).

``python -m cuda_mpi_reductions_amd.parallel.canary`` is the helper (its parameters come from
``MIREDUCE_CANARY_*`` environment variables set by :func:`fused_canary`). Ranks sharing one GPU map
no other GPU's memory, so there the canary is skipped unless ``MIREDUCE_CANARY_FORCE=1``.
"""
from __future__ import annotations

import datetime
import os
import secrets
import subprocess
import sys
from typing import Optional

__all__ = ["fused_canary", "direct_canary"]

_ENV = "MIREDUCE_CANARY_"


def _helper_fault(rank: int) -> None:
    """Test hook: MIREDUCE_CANARY_FAULT = abort@R | hang@R | wrong@R (the helper of rank R)."""
    spec = os.environ.get(_ENV + "FAULT", "")
    if not spec or "@" not in spec:
        return
    kind, r = spec.split("@", 1)
    if int(r) != rank:
        return
    if kind == "abort":
        print(f"[canary] rank {rank}: injected abort", file=sys.stderr, flush=True)
        os.abort()
    if kind == "hang":
        import time
        while True:
            time.sleep(1)


def _helper() -> int:
    rank, world = int(os.environ[_ENV + "RANK"]), int(os.environ[_ENV + "WORLD"])
    host, port = os.environ[_ENV + "ADDR"], int(os.environ[_ENV + "PORT"])
    prefix, dry = os.environ[_ENV + "PREFIX"], os.environ.get(_ENV + "DRY") == "1"
    timeout = datetime.timedelta(seconds=float(os.environ.get(_ENV + "TIMEOUT", "60")))
    import torch
    import torch.distributed as dist
    store = dist.PrefixStore(prefix, dist.TCPStore(host, port, is_master=False, timeout=timeout,
                                                   wait_for_workers=False))
    dist.init_process_group("gloo", store=store, rank=rank, world_size=world, timeout=timeout)
    _helper_fault(rank)
    wrong = os.environ.get(_ENV + "FAULT", "") == f"wrong@{rank}"
    if dry:  # no GPU: the orchestration only (CPU tests)
        t = torch.tensor([float(rank + 1) + (1.0 if wrong else 0.0)], dtype=torch.float64)
        dist.all_reduce(t)
        ok = t.item() == world * (world + 1) / 2
        msg = None if ok else f"gloo all-reduce gave {t.item()}"
    elif os.environ.get(_ENV + "KIND", "fused") == "direct":
        # the direct one-kernel collective (parallel/direct.py): registered buffers mapped by every
        # rank, an all-reduce and a reduce to root 0, a peer-read pass, error words, close
        from .direct import DirectComm
        idx = int(os.environ[_ENV + "DEVICE"])
        dev = torch.device("cuda", idx)
        torch.cuda.set_device(dev)
        n = int(os.environ.get(_ENV + "ELEMENTS", str(1 << 20)))
        t = torch.full((n,), float(rank + 1), dtype=torch.float64, device=dev)
        if wrong:
            t[0] += 1.0
        comm = DirectComm(dev, n * 8, timeout_s=5.0)
        expect = world * (world + 1) / 2
        a = comm.allreduce(t.clone(), "sum")
        r0 = comm.reduce(t.clone(), "sum", root=0)
        comm.read_peers(n * 8)
        torch.cuda.synchronize(dev)
        err = comm.check()  # collective
        ok = err is None and bool((a == expect).all().item()) and (rank != 0 or bool((r0 == expect).all().item()))
        msg = None if ok else f"direct all-reduce / reduce wrong or device error ({err})"
        comm.close()  # collective
    else:
        from ..ops import Reducer
        from .xrank import close_channels, open_channel
        idx = int(os.environ[_ENV + "DEVICE"])
        dev = torch.device("cuda", idx)
        torch.cuda.set_device(dev)
        n = int(os.environ.get(_ENV + "ELEMENTS", str(1 << 20)))
        x = torch.full((n,), float(rank + 1), dtype=torch.float64, device=dev)
        if wrong:
            x[0] += 1.0
        out = torch.zeros(3, dtype=torch.float64, device=dev)
        ch = open_channel(dev, timeout_s=5.0)  # collective over the helpers' group
        red = Reducer(dev)
        b = red.bind(x, "sum", torch.float64, out=out[:1], xrank=ch)
        s = torch.cuda.current_stream(dev).cuda_stream
        for i in range(3):  # epochs 1..3: both mailbox parities
            b.launch(s, out[i:i + 1].data_ptr())
        torch.cuda.synchronize(dev)
        expect = float(n) * world * (world + 1) / 2
        got = out.tolist()
        errs = (int(ch.error()), int(red.ws.error()))
        ok = errs == (0, 0) and all(v == expect for v in got)
        msg = None if ok else f"results {got} (expected {expect}), channel / fan-in error words {errs}"
        del b
        close_channels([ch], dev)  # collective: nobody unmaps a mailbox a peer still polls
    dist.barrier()
    dist.destroy_process_group()
    if msg:
        print(f"[canary] rank {rank}: {msg}", file=sys.stderr, flush=True)
    return 0 if ok else 1


def fused_canary(ctx, timeout_s: float = 90.0, dry: bool = False, elements: int = 1 << 20,
                 kind: str = "fused", fault=None, agree_timeout_s: float = 100.0) -> Optional[str]:
    """Collective over the default process group: None if every rank's helper ran the exchange
    correctly, else the agreed reason ("rank r: ..." for each failing rank). ``kind``: ``fused``
    (the fused cross-rank finish) or ``direct`` (the direct one-kernel collective and the peer-read
    probe, parallel/direct.py). World 1 maps no peer memory: None without a helper. ``dry`` (CPU
    tests): helpers rendezvous and all-reduce over gloo only.

    The verdicts are agreed through :func:`.dist.agree` (bounded by ``agree_timeout_s``, which must
    outlast ``timeout_s``: a rank whose helper failed at once arrives up to ``timeout_s`` before one
    whose helper waited for it): a rank whose own part failed in Python still reports (its verdict is
    the error), and a rank that died or hangs raises :class:`.dist.PeerLost` on the others instead of
    holding them in a collective.
    ``fault`` (utils.fault, site ``canary``) fires after this rank's helper ended."""
    from .dist import agree
    import torch.distributed as dist
    if ctx.world_size == 1 or not dist.is_initialized():
        return None
    if not dry and os.environ.get(_ENV + "FORCE") != "1":
        # The canary guards the mapping of ANOTHER GPU's memory. Ranks that share one GPU (the
        # one-GPU rehearsals) map their own device's memory only — and a helper per rank would
        # double the processes holding that GPU (the pool allows 16 per GPU; 8 ranks + 8 helpers
        # + the test runner is 17). MIREDUCE_CANARY_FORCE=1 runs it anyway (its GPU tests).
        from .topology import peer_map  # collective; cached, open_channel asks the same
        idx = ctx.device.index if ctx.device.index is not None else 0
        if peer_map(idx).ranks_per_gpu > 1:
            return None
    # The helpers' rendezvous: a fresh TCPStore that rank 0 serves on a free port for the duration
    # of this call (not the job's own store, which need not be a TCPStore on MASTER_PORT — file or
    # custom-port rendezvous — and would then cost every helper its full timeout).
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    server, where = None, [None]
    if ctx.rank == 0:
        try:
            server = dist.TCPStore(host, 0, is_master=True, wait_for_workers=False,
                                   timeout=datetime.timedelta(seconds=max(10.0, timeout_s)))
            where = [(host, int(server.port), secrets.token_hex(8))]
        except Exception as e:  # noqa: BLE001 - every rank then declines together
            where = [("", f"rank 0 could not serve the canary's store: {type(e).__name__}: {e}"[:200], "")]
    dist.broadcast_object_list(where, src=0)
    addr, port, token = where[0]
    env = dict(os.environ)
    env.update({_ENV + "RANK": str(ctx.rank), _ENV + "WORLD": str(ctx.world_size),
                _ENV + "ADDR": addr, _ENV + "PORT": str(port) if addr else "",
                _ENV + "PREFIX": f"mireduce_canary/{token}/",
                _ENV + "DEVICE": str(ctx.device.index if ctx.device.index is not None else 0),
                _ENV + "TIMEOUT": str(max(10.0, timeout_s - 10.0)), _ENV + "ELEMENTS": str(elements),
                _ENV + "KIND": kind})
    if dry:
        env[_ENV + "DRY"] = "1"
    mine = None
    if not addr:
        mine = str(port)
    else:
        try:
            p = subprocess.Popen([sys.executable, "-m", "cuda_mpi_reductions_amd.parallel.canary"], env=env,
                                 stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                                 cwd=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
            try:
                _, err = p.communicate(timeout=timeout_s)
                if p.returncode != 0:
                    lines = [ln for ln in (err or "").strip().splitlines() if ln and not ln.startswith("[W")]
                    tail = " | ".join(lines[-2:])
                    how = (f"crashed (signal {-p.returncode})" if p.returncode < 0 else
                           f"exited with {p.returncode}")
                    mine = f"helper {how}: {tail}"[:300]
            except subprocess.TimeoutExpired:
                p.kill()
                p.communicate()
                mine = f"helper did not finish within {timeout_s:g} s"
        except OSError as e:
            mine = f"could not start the helper: {e}"[:300]
    try:
        if fault is not None:
            fault.at(ctx.rank, fault.spec.step, "canary", "fused-finish canary")
    except Exception as e:  # noqa: BLE001 - this rank's part failed: its verdict says so
        mine = f"{type(e).__name__}: {e}"[:300]
    # (every helper has ended: rank 0's store may go)
    verdicts = [row["verdict"] for row in agree(ctx, f"canary ({kind})", {"verdict": mine}, agree_timeout_s)]
    del server
    # the root causes first: helpers that crashed or hung, then the ones that only lost a peer
    first = [f"rank {r}: {m}" for r, m in enumerate(verdicts) if m and ("crashed" in m or "did not finish" in m)]
    rest = [f"rank {r}: {m}" for r, m in enumerate(verdicts) if m and not ("crashed" in m or "did not finish" in m)]
    bad = first + rest
    return "; ".join(bad)[:600] if bad else None


def direct_canary(ctx, timeout_s: float = 90.0, dry: bool = False) -> Optional[str]:
    """:func:`fused_canary` for the direct one-kernel collective (bench.py runs it before its
    reduce.c table's direct rows and the xGMI peer-read probe)."""
    return fused_canary(ctx, timeout_s=timeout_s, dry=dry, kind="direct", agree_timeout_s=timeout_s + 10.0)


if __name__ == "__main__":
    sys.exit(_helper())
