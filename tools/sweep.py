#!/usr/bin/env python3
"""Experiment orchestration: the reference's submit_all.sh + ccni_vn.sh + manual collection
(mpi/submit_all.sh:3-5, mpi/ccni_vn.sh:7-9) as one resumable script.

For every rank count P it launches one job (torchrun for GPU apps, mpirun for reduce_mpi), writes
``<out>/stdout-<name>-P<P>.txt`` (+ ``.rc``), and skips points whose ``.rc`` already says 0 —
an interrupted sweep resumes where it stopped. Afterwards it concatenates every
reduce.c-format line into ``<out>/collected.txt``, averages them (tools/getAvgs.sh semantics) into
``<out>/results/`` and, for bench.py, collects the JSON lines into ``<out>/bench.jsonl``.

    python tools/sweep.py --app reduce_xgmi --ranks 1,2,4,8 --out runs/vector -- --mode=vector
    python tools/sweep.py --app bench --ranks 1,2,4,8 --out runs/bench -- --steps 50 --warmup 10
    python tools/sweep.py --app reduce_mpi --ranks 2,4 --out runs/mpi -- --ints=1M --doubles=1M
    python tools/sweep.py --preset node --out runs/node      # the whole 1/2/4/8-GPU matrix below

``--rccl-knobs`` sweeps RCCL's tuning knobs over reduce.c's element-wise table (the
algorithm / protocol / channel count decide how much of the 7 xGMI links a collective uses):
``NCCL_ALGO`` x ``NCCL_PROTO`` x ``NCCL_MIN_NCHANNELS`` (``--knob-grid``, default Ring|Tree x
Simple|LL128 x default|16|32), one sub-directory per setting (``rccl-<algo>-<proto>-ch<n>/``, with
``knobs.json`` and getAvgs-format ``collected.txt`` / ``results/``), every other NCCL_* knob unset,
and ``<out>/rccl_knobs.md``: GiB/s per setting x N for each DATATYPE x OP, best setting per N marked.

    python tools/sweep.py --rccl-knobs --ranks 2,4,8 --out runs/knobs            # reduce_xgmi, reduce
    python tools/sweep.py --rccl-knobs --ranks 2,4,8 --out runs/knobs --rccl-collective allreduce

``--preset node`` runs, resumable point by point: the xGMI roofline (``bandwidth_test --peer``, once);
reduce.c's vector benchmark over every collective — RCCL ``reduce`` / ``allreduce`` and the one-kernel
direct ``direct-reduce`` / ``direct`` (csrc/kernels/direct.hip), each graph-replayed — at every rank
count; and the north-star bench.py at every rank count. Each entry gets its own collected.txt /
results/ (getAvgs format) under ``<out>/<name>/``.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from cuda_mpi_reductions_amd.utils import getavgs  # noqa: E402

MPIRUN = "/opt/conda/bin/mpirun"


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _port_taken(stderr) -> bool:
    text = (stderr if isinstance(stderr, str) else (stderr or b"").decode(errors="replace")).lower()
    return "eaddrinuse" in text or "address already in use" in text


def command(app: str, p: int, extra: list[str]) -> list[str]:
    if app == "reduce_mpi":
        return [MPIRUN, "-np", str(p), os.path.join(ROOT, "build", "bin", "reduce_mpi")] + extra
    target = os.path.join(ROOT, "bench.py") if app == "bench" else os.path.join(ROOT, "build", "bin", app)
    tr = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={p}",
          "--master-addr", "127.0.0.1", "--master-port", str(free_port())]
    if app != "bench":
        tr.append("--no-python")
    args = list(extra)
    if app == "bench":
        args = ["--gpus", str(p)] + args
    return tr + [target] + args


VECTOR_COLLECTIVES = ("reduce", "allreduce", "direct-reduce", "direct")


def node_preset(extra: list[str]) -> list[tuple]:
    """(app, name, ranks or None for one single-process run, args) of ``--preset node``."""
    entries = [("bandwidth_test", "fabric", None, ["--peer", "--json=fabric.json"])]
    for coll in VECTOR_COLLECTIVES:
        entries.append(("reduce_xgmi", f"vector-{coll}", "ranks",
                        ["--mode=vector", f"--collective={coll}", "--graph", "--dtypes=INT,DOUBLE"] + extra))
    for coll in ("allreduce", "fused"):  # simpleMPI's scalar combine: RCCL vs the in-kernel fused finish
        entries.append(("reduce_xgmi", f"scalar-{coll}", "ranks",
                        ["--mode=scalar", f"--collective={coll}", "--graph", "--dtypes=INT,DOUBLE"] + extra))
    entries.append(("bench", "bench", "ranks", ["--steps", "50", "--warmup", "10"]))
    return entries


KNOB_GRID = "NCCL_ALGO=Ring,Tree;NCCL_PROTO=Simple,LL128;NCCL_MIN_NCHANNELS=default,16,32"
KNOB_VARS = ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_BUFFSIZE",
             "NCCL_NTHREADS", "RCCL_MSCCL_ENABLE", "RCCL_MSCCLPP_ENABLE")


def knob_settings(grid: str = KNOB_GRID) -> list:
    """Every combination of ``VAR=v1,v2;VAR=...`` (``default`` = leave the variable unset), as
    (name, {VAR: value or None})."""
    import itertools
    axes = []
    for part in (p for p in grid.split(";") if p.strip()):
        var, vals = part.split("=", 1)
        axes.append([(var.strip(), None if v.strip() == "default" else v.strip()) for v in vals.split(",")])
    out = []
    for combo in itertools.product(*axes):
        short = {"NCCL_ALGO": "", "NCCL_PROTO": "", "NCCL_MIN_NCHANNELS": "ch"}
        name = "rccl-" + "-".join(f"{short.get(k, k.lower() + '_')}{v if v is not None else 'default'}".lower()
                                  for k, v in combo)
        out.append((name, dict(combo)))
    return out


def knob_env(setting: dict) -> dict:
    """The process environment of one knob setting: every known knob unset, then the setting's."""
    env = {k: v for k, v in os.environ.items() if k not in KNOB_VARS}
    env.update({k: v for k, v in setting.items() if v is not None})
    return env


def run_knobs(a) -> int:
    """``--rccl-knobs``: reduce.c's table over RCCL for every knob setting (resumable per point)."""
    ranks = [int(x) for x in a.ranks.split(",") if x]
    app = a.app or "reduce_xgmi"
    failures, table = 0, []
    for name, setting in knob_settings(a.knob_grid):
        sub = os.path.join(a.out, name)
        os.makedirs(sub, exist_ok=True)
        with open(os.path.join(sub, "knobs.json"), "w") as f:
            json.dump({k: v for k, v in setting.items()}, f)
        args = list(a.extra)
        if app == "reduce_xgmi":
            args = ["--mode=vector", f"--collective={a.rccl_collective}", "--graph", "--dtypes=INT,DOUBLE",
                    "--json=points.jsonl"] + args
        failures += run_points(app, name, ranks, args, os.path.abspath(sub), a.timeout, a.force,
                               env=knob_env(setting))
        collect(sub, name)
        table.append((name, setting, _results_means(os.path.join(sub, "results"))))
    with open(os.path.join(a.out, "rccl_knobs.md"), "w") as f:
        f.write(knob_table(table))
    print(knob_table(table), end="")
    return 1 if failures else 0


def _results_means(results_dir: str) -> dict:
    """{(DT, OP, N): GiB/s} from a getAvgs results directory (missing -> {})."""
    out = {}
    if not os.path.isdir(results_dir):
        return out
    for fn in sorted(os.listdir(results_dir)):
        for line in open(os.path.join(results_dir, fn)):
            f = line.split()
            if len(f) == 4:
                out[(f[0], f[1], int(f[2]))] = float(f[3])
    return out


def knob_table(table: list) -> str:
    """Markdown: one row per (DATATYPE, OP, N) x setting, the best setting per (DATATYPE, OP, N) in bold."""
    keys = sorted({k for _, _, m in table for k in m})
    lines = ["| DATATYPE | OP | N | setting | GiB/s |", "|---|---|---|---|---|"]
    for k in keys:
        vals = [(name, m[k]) for name, _, m in table if k in m]
        best = max(v for _, v in vals)
        for name, v in vals:
            cell = f"**{v:.3f}**" if v == best else f"{v:.3f}"
            lines.append(f"| {k[0]} | {k[1]} | {k[2]} | {name} | {cell} |")
    return "\n".join(lines) + "\n"


def run_points(app: str, name: str, ranks: list, extra: list[str], out: str, timeout: float, force: bool,
               env: "dict | None" = None) -> int:
    failures = 0
    for p in ranks:
        base = os.path.join(out, f"stdout-{name}-P{p}")
        rc_path = base + ".rc"
        if not force and os.path.exists(rc_path) and open(rc_path).read().strip() == "0":
            print(f"[sweep] {name} P={p}: done, skipping ({base}.txt)")
            continue
        if p is None:  # one single-process run (all visible GPUs)
            cmd = [os.path.join(ROOT, "build", "bin", app)] + extra
        else:
            cmd = command(app, p, extra)
        t0 = time.time()
        for attempt in range(2):
            print(f"[sweep] {name} P={p}: {' '.join(cmd)}", flush=True)
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=out, env=env)
                rc, stdout, err = r.returncode, r.stdout, r.stderr
            except subprocess.TimeoutExpired as e:
                rc, stdout, err = 124, e.stdout or "", (e.stderr or "") + "\n[sweep] timeout"
            # free_port() closes the port before the launcher binds it: another process can take it
            # in between. That is a launch failure, not a result: one retry on a new port.
            if attempt == 0 and rc != 0 and p is not None and app != "reduce_mpi" and _port_taken(err):
                print(f"[sweep] {name} P={p}: rendezvous port taken, retrying on a new port", flush=True)
                cmd = command(app, p, extra)
                continue
            break
        with open(base + ".txt", "w") as f:
            f.write(stdout if isinstance(stdout, str) else stdout.decode())
        with open(base + ".err", "w") as f:
            f.write(err if isinstance(err, str) else err.decode())
        with open(rc_path, "w") as f:
            f.write(f"{rc}\n")
        print(f"[sweep] {name} P={p}: rc={rc} in {time.time() - t0:.1f} s", flush=True)
        failures += rc != 0
    return failures


def run_preset(a) -> int:
    ranks = [int(x) for x in a.ranks.split(",") if x]
    failures = 0
    for app, name, rk, args in node_preset(a.extra):
        sub = os.path.join(a.out, name)
        os.makedirs(sub, exist_ok=True)
        failures += run_points(app, name, [None] if rk is None else ranks, args, sub, a.timeout, a.force)
        collect(sub, name)
    return 1 if failures else 0


def collect(out: str, name: str) -> None:
    collected, jsonl = [], []
    for fn in sorted(os.listdir(out)):
        if fn.startswith(f"stdout-{name}-P") and fn.endswith(".txt"):
            for line in open(os.path.join(out, fn)):
                if line.startswith("{"):
                    jsonl.append(line.strip())
                elif not line.startswith("#") and len(line.split()) == 4:
                    collected.append(line)
    if collected:
        cpath = os.path.join(out, "collected.txt")
        with open(cpath, "w") as f:
            f.writelines(collected)
        getavgs.write_results(cpath, os.path.join(out, "results"))
    if jsonl:
        with open(os.path.join(out, "bench.jsonl"), "w") as f:
            f.write("\n".join(jsonl) + "\n")
        rows = [json.loads(j) for j in jsonl]
        base1 = next((r["value"] for r in rows if r.get("n_gpus") == 1), None)
        for r in sorted(rows, key=lambda r: r.get("n_gpus", 0)):
            eff = (r["value"] / (r["n_gpus"] * base1)) if base1 else float("nan")
            print(f"[sweep] N={r['n_gpus']}: {r['value']:.1f} {r['unit']}  ms/step {r['ms_per_step']}  "
                  f"scaling efficiency {eff:.3f}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--app", choices=["bench", "reduce_xgmi", "reduce_mpi", "reduction"])
    ap.add_argument("--preset", choices=["node"], help="run a predefined matrix instead of one --app")
    ap.add_argument("--rccl-knobs", action="store_true",
                    help="sweep RCCL's NCCL_ALGO / NCCL_PROTO / NCCL_MIN_NCHANNELS over reduce.c's table "
                         "(--app: reduce_xgmi by default)")
    ap.add_argument("--knob-grid", default=KNOB_GRID, help="VAR=v1,v2;VAR=... (default: %(default)s)")
    ap.add_argument("--rccl-collective", default="reduce", choices=["reduce", "allreduce"],
                    help="--rccl-knobs with reduce_xgmi: MPI_Reduce-like (reduce.c) or all-reduce")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--out", required=True)
    ap.add_argument("--name", default="")
    ap.add_argument("--timeout", type=float, default=900)
    ap.add_argument("--force", action="store_true", help="re-run points that already completed")
    ap.add_argument("extra", nargs="*")
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    if a.rccl_knobs:
        return run_knobs(a)
    if a.preset:
        return run_preset(a)
    if not a.app:
        ap.error("--app or --preset is required")
    name = a.name or a.app
    ranks = [int(x) for x in a.ranks.split(",") if x]
    failures = run_points(a.app, name, ranks, a.extra, os.path.abspath(a.out), a.timeout, a.force)
    collect(a.out, name)
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
