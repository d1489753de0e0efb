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


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--app", required=True, choices=["bench", "reduce_xgmi", "reduce_mpi", "reduction"])
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--out", required=True)
    ap.add_argument("--name", default="")
    ap.add_argument("--timeout", type=float, default=900)
    ap.add_argument("--force", action="store_true", help="re-run points that already completed")
    ap.add_argument("extra", nargs="*")
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    name = a.name or a.app
    failures = 0
    for p in [int(x) for x in a.ranks.split(",") if x]:
        base = os.path.join(a.out, f"stdout-{name}-P{p}")
        rc_path = base + ".rc"
        if not a.force and os.path.exists(rc_path) and open(rc_path).read().strip() == "0":
            print(f"[sweep] P={p}: done, skipping ({base}.txt)")
            continue
        cmd = command(a.app, p, a.extra)
        print(f"[sweep] P={p}: {' '.join(cmd)}", flush=True)
        t0 = time.time()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout)
            rc, out, err = r.returncode, r.stdout, r.stderr
        except subprocess.TimeoutExpired as e:
            rc, out, err = 124, e.stdout or "", (e.stderr or "") + "\n[sweep] timeout"
        with open(base + ".txt", "w") as f:
            f.write(out if isinstance(out, str) else out.decode())
        with open(base + ".err", "w") as f:
            f.write(err if isinstance(err, str) else err.decode())
        with open(rc_path, "w") as f:
            f.write(f"{rc}\n")
        print(f"[sweep] P={p}: rc={rc} in {time.time() - t0:.1f} s", flush=True)
        failures += rc != 0
    # collect
    collected, jsonl = [], []
    for fn in sorted(os.listdir(a.out)):
        if fn.startswith(f"stdout-{name}-P") and fn.endswith(".txt"):
            for line in open(os.path.join(a.out, fn)):
                if line.startswith("{"):
                    jsonl.append(line.strip())
                elif not line.startswith("#") and len(line.split()) == 4:
                    collected.append(line)
    if collected:
        cpath = os.path.join(a.out, "collected.txt")
        with open(cpath, "w") as f:
            f.writelines(collected)
        getavgs.write_results(cpath, os.path.join(a.out, "results"))
    if jsonl:
        with open(os.path.join(a.out, "bench.jsonl"), "w") as f:
            f.write("\n".join(jsonl) + "\n")
        rows = [json.loads(j) for j in jsonl]
        base1 = next((r["value"] for r in rows if r["n_gpus"] == 1), None)
        for r in sorted(rows, key=lambda r: r["n_gpus"]):
            eff = (r["value"] / (r["n_gpus"] * base1)) if base1 else float("nan")
            print(f"[sweep] N={r['n_gpus']}: {r['value']:.1f} {r['unit']}  ms/step {r['ms_per_step']}  "
                  f"scaling efficiency {eff:.3f}")
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
