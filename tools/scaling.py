#!/usr/bin/env python3
"""Scaling curve from bench.py JSON lines -> the reference's results format and a scaling table.

The reference's pipeline is: per-run stdout rows ``DATATYPE OP NODES GB/sec`` (mpi/reduce.c:81,95)
-> mpi/getAvgs.sh:3-14 (mean of column 4 per DATATYPE x OP x NODES into results/<DT>_<OP>.txt,
starting with a blank line) -> mpi/makePlots.gp:1-40 (``using 3:4``). This tool feeds the headline
benchmark into the same pipeline: it collects every bench.py result object (one JSON line per run,
or any JSON document holding such objects, e.g. the driver's scaling file), groups them by
(config, n_gpus), averages repeated runs like getAvgs.sh, and writes

* ``<out>/<DT>_<OP>.txt``      rows ``DOUBLE SUM <N> <GB/s>`` (GB = 1e9 B, bench.py's unit),
                               readable by tools/plot.py and tools/makePlots.gp unchanged;
* ``<out>/scaling.md``         N, GB/s, ms/step, speed-up over N=1 and efficiency;
* ``<out>/vector_<impl>/<DT>_<OP>.txt``  reduce.c's own table from the north-star runs'
                               ``reduce_c_vector.table`` (INT / DOUBLE x MAX / MIN / SUM element-wise
                               to root 0, GiB/s of total data, impl = rccl | direct), averaged per N
                               like getAvgs.sh: the counterpart of mpi/results/<DT>_<OP>.txt, plus
                               ``<out>/vector.md`` (N > 1 only: one rank has no cross-rank reduction);
* ``<out>/vector_<impl>/collected.txt``  every run's reduce.c-format stdout rows (``reduce_c_vector.
                               rows[impl]``, N > 1), the input mpi/getAvgs.sh / utils/getavgs.py expect.

Efficiency = value(N) / (N * value(1)): the whole-node bandwidth of N GPUs against N copies of the
1-GPU run (bench.py's headline is strong scaling, so this is also t(1) / (N * t(N))).

Where an N-GPU step's time goes (bench.py's ``decomposition``, averaged like the headline): the
slowest rank's local reduce (ms/step, the same kernel without the combine), the cross-rank
exchange (us/step = headline - local), the inter-GPU skew of the local work (us/step) and
``vs local`` = local time / step time (1.0 = the combine is free) and, for the fused finish, the
device-timed wait from a rank's push to all partials landed (the least waiting rank ~ the local
poll, the most waiting ~ skew + xGMI latency). So a loss of efficiency at N=8
splits into the per-GPU rate at the smaller shard (local ms vs N=1), the exchange and the skew.

    python tools/scaling.py SCALE_r01.json bench_*.json --out results/scaling
    python tools/scaling.py --from SCALE_r06.json --out results/scaling --update-writeup docs/WRITEUP.md

``--from`` is the one command for the driver's scaling record: results files, scaling.md, the
reduce.c vector tables, the WRITEUP table (measured next to the one-GPU projection) and both report
figures (tools/report.py); a skipped record, a missing rank count or an unverified N fails it
(rc 2, nothing written) — a curve is never interpolated.

Round 5+ lines are compact: each names its extras sidecar (``summary.extras_file``, bench.py's
``--extras-file``), which is merged in when found (as named or next to the input file); a
sidecar may also be passed directly (it holds the line too). A line and its sidecar count once.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from collections import defaultdict

_DT = {"fp64": "DOUBLE", "float64": "DOUBLE", "fp32": "FLOAT", "float32": "FLOAT",
       "int32": "INT", "int64": "LONG", "bf16": "BF16", "bfloat16": "BF16", "fp16": "HALF"}


def _walk(obj):
    """Yield every dict in a JSON document that looks like a bench.py result — also the whole JSON
    lines inside string values (the driver's records keep the printed line in a stdout tail, and
    only the contract keys of it in ``parsed``)."""
    if isinstance(obj, dict):
        if "n_gpus" in obj and "value" in obj and "metric" in obj:
            yield obj
        else:
            for v in obj.values():
                yield from _walk(v)
    elif isinstance(obj, list):
        for v in obj:
            yield from _walk(v)
    elif isinstance(obj, str) and '"metric"' in obj:
        for line in obj.splitlines():
            line = line.strip()
            if line.startswith("{"):
                try:
                    yield from _walk(json.loads(line))
                except ValueError:
                    continue


def parse_text(text: str):
    """Bench results from a whole-file JSON document, or from JSON lines mixed with other output."""
    try:
        return list(_walk(json.loads(text)))
    except ValueError:
        pass
    out = []
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                out.extend(_walk(json.loads(line)))
            except ValueError:
                continue
    return out


def with_sidecar(r: dict, base_dir: "str | None" = None) -> dict:
    """A bench.py line (round 5+) carries only the headline and a summary; the full extras record
    (decomposition, reduce.c table, per-rank plans, ...) is the sidecar named in
    ``summary.extras_file``. Merge it in when it exists (as named, or by file name next to
    ``base_dir``) and belongs to the same run (``summary.run``); the line's keys win."""
    s = r.get("summary")
    if not isinstance(s, dict) or not s.get("extras_file"):
        return r
    for path in (s["extras_file"], os.path.join(base_dir or ".", os.path.basename(s["extras_file"]))):
        try:
            with open(path) as f:
                side = json.load(f)
        except (OSError, ValueError):
            continue
        if isinstance(side, dict) and (side.get("summary") or {}).get("run") == s.get("run"):
            merged = dict(side)
            merged.update(r)
            return merged
    return r


def dedupe(results):
    """One result per bench run: a line and its sidecar (or the same line in two files) share
    ``summary.run``; the record with more keys (the merged one) is kept. Results without a run id
    (older rounds) are all kept."""
    out, seen = [], {}
    for r in results:
        run = (r.get("summary") or {}).get("run") if isinstance(r.get("summary"), dict) else None
        if run is None:
            out.append(r)
        elif run not in seen:
            seen[run] = len(out)
            out.append(r)
        elif len(r) > len(out[seen[run]]):
            out[seen[run]] = r
    # a record without a run id that repeats a run's headline (the driver's ``parsed`` copy of a
    # line also found whole in its stdout tail) is the same run
    ided = {_headline(r) for r in out if (r.get("summary") or {}).get("run") if isinstance(r.get("summary"), dict)}
    return [r for r in out if (isinstance(r.get("summary"), dict) and r["summary"].get("run"))
            or _headline(r) not in ided]


def _combine(r) -> str:
    """The cross-rank combine a run used, with why the fused finish was not it (bench.py's
    ``config.collective_reason``, shortened)."""
    c = r.get("config") or {}
    why = c.get("collective_reason")
    return str(c.get("collective", "")) + (f" ({str(why)[:60]})" if why else "")


def _headline(r) -> tuple:
    return (r.get("metric"), r.get("n_gpus"), r.get("value"), r.get("ms_per_step"))


def key_of(r):
    cfg = r.get("config") or {}
    model = str(cfg.get("model", "")).split(":")[0] or "bench"
    dt = _DT.get(str(r.get("dtype", "")).lower(), str(r.get("dtype", "")).upper() or "DOUBLE")
    op = str(cfg.get("op", "SUM")).upper()
    return model, dt, op


def summarise(results):
    """{(model, DT, OP): {N: {"gbps": mean value, "ms": mean ms/step, "runs": k}}}."""
    acc = defaultdict(lambda: defaultdict(list))
    for r in results:
        if r.get("value") is None:
            continue
        acc[key_of(r)][int(r["n_gpus"])].append(r)
    out = {}
    for k, per_n in acc.items():
        out[k] = {}
        for n, rs in sorted(per_n.items()):
            ms = [float(r["ms_per_step"]) for r in rs if r.get("ms_per_step") is not None]
            out[k][n] = {"gbps": sum(float(r["value"]) for r in rs) / len(rs),
                         "ms": sum(ms) / len(ms) if ms else None, "runs": len(rs),
                         "verified": (False if any(r.get("verified") is False for r in rs) else
                                      True if all(r.get("verified") is True for r in rs) else None),
                         "combine": "/".join(sorted({_combine(r) for r in rs})),
                         "plans": "; ".join(sorted({str((r.get("summary") or {}).get("plans"))
                                                     for r in rs if (r.get("summary") or {}).get("plans")}))}
            out[k][n].update(_decomposition(rs))
    return out


DECOMP = (("local_ms", "local_ms_per_step"), ("exchange_us", "exchange_us_per_step"),
          ("skew_us", "skew_us_per_step"), ("vs_local", "scaling_efficiency_vs_local"))


def _decomp_of(r) -> dict:
    """A run's decomposition: the sidecar's ``decomposition``, or — for a bare printed line (the
    driver's records keep no sidecar) — the same fields rebuilt from the line's ``summary``
    (``local_gbps``, ``exchange_us``, ``skew_us``, ``efficiency_vs_local``, ``wait_us`` = [min, max])."""
    d = r.get("decomposition")
    if isinstance(d, dict) and d:
        return d
    s = r.get("summary") if isinstance(r.get("summary"), dict) else {}
    cfg = r.get("config") or {}
    out = {}
    nbytes = cfg.get("bytes_per_step")
    if s.get("local_gbps") and nbytes:
        out["local_ms_per_step"] = float(nbytes) / (float(s["local_gbps"]) * 1e9) * 1e3
    for field, key in (("exchange_us_per_step", "exchange_us"), ("skew_us_per_step", "skew_us"),
                       ("scaling_efficiency_vs_local", "efficiency_vs_local")):
        if s.get(key) is not None:
            out[field] = s[key]
    w = s.get("wait_us")
    if isinstance(w, (list, tuple)) and len(w) == 2:
        out["exchange_wait_us"] = {"min_rank_median": w[0], "max_rank_median": w[1]}
    return out


def _decomposition(rs) -> dict:
    """Mean of each bench.py ``decomposition`` field over the runs that carry it (None if none do),
    plus the device-timed fused exchange wait (``exchange_wait_us``: least / most waiting rank)."""
    out = {}
    decs = [_decomp_of(r) for r in rs]
    decs = [d for d in decs if d]
    for name, field in DECOMP:
        vals = [float(d[field]) for d in decs if d.get(field) is not None]
        out[name] = sum(vals) / len(vals) if vals else None
    for name, field in (("wait_min_us", "min_rank_median"), ("wait_max_us", "max_rank_median")):
        vals = [float(d["exchange_wait_us"][field]) for d in decs
                if isinstance(d.get("exchange_wait_us"), dict) and d["exchange_wait_us"].get(field) is not None]
        out[name] = sum(vals) / len(vals) if vals else None
    return out


def _rows_from_summary(rows) -> list:
    """bench.py's ``summary.reduce_c_rows`` ({impl: "INT MAX 12.345; ...; DOUBLE SUM 9.876"}, each the
    mean over the retries, ``!`` = a retry failed verification) as table entries."""
    out = []
    for impl, text in (rows or {}).items():
        for item in str(text).split(";"):
            parts = item.split()
            if len(parts) == 3:
                out.append({"impl": impl, "dtype": parts[0], "op": parts[1], "gibps": float(parts[2].rstrip("!")),
                            "verified": not parts[2].endswith("!")})
    return out


def summarise_vector(results):
    """{(impl, DT, OP): {N: {"gibps": mean, "runs": k}}} from every result's reduce_c_vector.table
    (one entry per timed collective, RETRY_COUNT per (dtype, op), averaged like getAvgs.sh).
    Skipped: entries without a number (errors; RCCL at world 1) and every N=1 entry — one rank has
    no cross-rank reduction (RCCL's 1-rank in-place reduce does no work, direct is a local copy),
    so an N=1 point next to the N>1 ones in results/<DT>_<OP>.txt would be unphysical."""
    acc = defaultdict(lambda: defaultdict(list))
    for r in results:
        if int(r.get("n_gpus", 0)) <= 1:
            continue
        table = (r.get("reduce_c_vector") or {}).get("table")
        if not table:  # a bare printed line (e.g. the driver's record): its summary's getAvgs-style means
            table = _rows_from_summary((r.get("summary") or {}).get("reduce_c_rows"))
        for row in table or []:
            if row.get("gibps") is None:
                continue
            acc[(row["impl"], row["dtype"], row["op"])][int(r["n_gpus"])].append(float(row["gibps"]))
    return {k: {n: {"gibps": sum(v) / len(v), "runs": len(v)} for n, v in sorted(per_n.items())}
            for k, per_n in acc.items()}


def write_vector(vsummary, out_dir):
    """results/vector_<impl>/<DT>_<OP>.txt (getAvgs.sh format) and vector.md; returns the markdown."""
    md = ["| impl | DATATYPE | OP | N | GiB/s (total data) | runs |", "|---|---|---|---|---|---|"]
    for (impl, dt, op), per_n in sorted(vsummary.items()):
        d = os.path.join(out_dir, f"vector_{impl}")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"{dt}_{op}.txt"), "w") as f:
            f.write("\n")
            for n, v in per_n.items():
                f.write(f"{dt} {op} {n} {v['gibps']:.5f}\n")
        for n, v in per_n.items():
            md.append(f"| {impl} | {dt} | {op} | {n} | {v['gibps']:.3f} | {v['runs']} |")
    text = "\n".join(md) + "\n"
    if vsummary:
        with open(os.path.join(out_dir, "vector.md"), "w") as f:
            f.write(text)
    return text


def write_collected(results, out_dir):
    """<out>/vector_<impl>/collected.txt: the concatenated reduce.c stdout of every N > 1 run (the
    reference's mpi/collected.txt, which getAvgs.sh reads). Returns {impl: path}."""
    by_impl = defaultdict(list)
    for r in results:
        if int(r.get("n_gpus", 0)) <= 1:
            continue
        rows = (r.get("reduce_c_vector") or {}).get("rows")
        if isinstance(rows, dict):
            for impl, lines in rows.items():
                by_impl[impl].extend(lines)
    paths = {}
    for impl, lines in by_impl.items():
        d = os.path.join(out_dir, f"vector_{impl}")
        os.makedirs(d, exist_ok=True)
        paths[impl] = os.path.join(d, "collected.txt")
        with open(paths[impl], "w") as f:
            f.write("".join(ln + "\n" for ln in lines))
    return paths


def efficiency(per_n):
    """{N: (speed-up over N=1, efficiency)}; None where there is no N=1 point."""
    base = per_n.get(1, {}).get("gbps")
    return {n: ((v["gbps"] / base, v["gbps"] / (n * base)) if base else (None, None))
            for n, v in per_n.items()}


def write(summary, out_dir):
    os.makedirs(out_dir, exist_ok=True)
    md = ["| config | dtype | op | N | GB/s (whole node) | ms/step | speed-up | efficiency | runs "
          "| local ms/step | exchange us/step | skew us/step | vs local | fused wait us (min-max rank) "
          "| combine | verified | plans (per rank) |",
          "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for (model, dt, op), per_n in sorted(summary.items()):
        with open(os.path.join(out_dir, f"{dt}_{op}.txt"), "w") as f:
            f.write("\n")  # getAvgs.sh:5-6 starts each results file with a blank line
            for n, v in per_n.items():
                f.write(f"{dt} {op} {n} {v['gbps']:.5f}\n")
        eff = efficiency(per_n)
        for n, v in per_n.items():
            s, e = eff[n]
            ms = "" if v["ms"] is None else "%.4f" % v["ms"]
            sp = "" if s is None else "%.2fx" % s
            ef = "" if e is None else "%.1f %%" % (100 * e)
            dec = ["" if v.get(f) is None else fmt % v[f] for f, fmt in
                   (("local_ms", "%.4f"), ("exchange_us", "%.2f"), ("skew_us", "%.2f"), ("vs_local", "%.3f"))]
            wait = "" if v.get("wait_min_us") is None else "%.2f-%.2f" % (v["wait_min_us"], v["wait_max_us"])
            md.append(f"| {model} | {dt} | {op} | {n} | {v['gbps']:.1f} | {ms} | {sp} | {ef} | {v['runs']} | "
                      + " | ".join(dec) + f" | {wait} | {v.get('combine', '')} | "
                      + {True: "yes", False: "**NO**"}.get(v.get("verified"), "?") + f" | {v.get('plans', '')} |")
    text = "\n".join(md) + "\n"
    with open(os.path.join(out_dir, "scaling.md"), "w") as f:
        f.write(text)
    return text


# ---------------------------------------------------------------- --from: a driver's SCALE record
HEADLINE_MODEL = "xgmi_1b_double_sum"
HEADLINE_BYTES = 8e9
# docs/WRITEUP.md §2's projection, from one-GPU measurements only: a shard of G GB streams in
# G x 135.56 us plus ~1.9 us per launch (profiles/r5_floor/), plus the exchange t_x per step
PROJ_US_PER_GB, PROJ_LAUNCH_US = 135.56, 1.9


def projection(n: int, t_x_us: float = 0.0) -> float:
    """Projected whole-node GB/s of the headline at N GPUs (8 GB over N shards) with exchange t_x."""
    return HEADLINE_BYTES / ((HEADLINE_BYTES / 1e9 / n * PROJ_US_PER_GB + PROJ_LAUNCH_US + t_x_us) * 1e-6) / 1e9


class ScalingError(RuntimeError):
    pass


def check_curve(per_n: dict, require, failed: "dict | None" = None) -> None:
    """Refuse a partial or unverified curve (never interpolate): every required N measured, every
    measured N verified. ``failed``: {N: error} of the runs that printed no number (their
    diagnostic lines), quoted for the missing rank counts."""
    missing = [n for n in require if n not in per_n]
    bad = [f"N={n} ({'unverified' if v.get('verified') is None else 'verification FAILED'})"
           for n, v in sorted(per_n.items()) if v.get("verified") is not True]
    msgs = []
    if missing:
        msgs.append("no headline result for " + ", ".join(
            f"N={n}" + (f" (its run: {str((failed or {})[n])[:160]})" if n in (failed or {}) else "") for n in missing))
    if bad:
        msgs.append("not verified: " + ", ".join(bad))
    if msgs:
        raise ScalingError("; ".join(msgs))


def writeup_table(per_n: dict) -> str:
    """The WRITEUP §2 table with the measured values next to the projection they replace."""
    rows = ["| N | shard | measured GB/s | ms/step | efficiency | projection t_x = 0 | projection t_x = measured wait "
            "| measured / projection | local us/step | exchange us/step | skew us/step | combine |",
            "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    eff = efficiency(per_n)
    for n, v in sorted(per_n.items()):
        p0 = projection(n)
        tx = v.get("wait_max_us")
        px = projection(n, tx) if tx is not None else None
        e = eff[n][1]
        f = lambda x, fmt: "" if x is None else fmt % x  # noqa: E731
        rows.append(f"| {n} | {8 / n:g} GB | {v['gbps']:.1f} | {f(v['ms'], '%.5f')} | {f(None if e is None else 100 * e, '%.1f %%')} "
                    f"| {p0:.0f} | {f(px, '%.0f')} | {v['gbps'] / p0:.3f} | {f(None if v.get('local_ms') is None else 1e3 * v['local_ms'], '%.1f')} "
                    f"| {f(v.get('exchange_us'), '%.2f')} | {f(v.get('skew_us'), '%.2f')} | {v.get('combine', '')} |")
    return "\n".join(rows) + "\n"


def bgl_ranks_to_match(gbps: float, dt: str = "DOUBLE", op: str = "SUM", at: int = 1024) -> float:
    """The reference's cross-processor comparison (writeup.tex:19: BG/L's INT reduction overtakes one
    2012 GPU at ~500-600 ranks), restated for a measured MI355X number: how many BG/L VN ranks, each
    at the per-rank rate of the reference's own ``at``-rank run (mpi/results/<DT>_<OP>.txt), would
    match ``gbps`` (GB/s). Like the reference, this sets an element-wise reduction against a whole-
    array one: each moves every input byte once."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from reference_data import BGL_VN, GIB_PER_GB
    per_rank_gibps = BGL_VN[(dt, op)][at] / at
    return gbps * GIB_PER_GB / per_rank_gibps


def crossover_text(per_n: dict) -> str:
    """One sentence per measured N: the BG/L ranks that would match it (DOUBLE SUM and INT SUM rates)."""
    parts = [f"N={n}: {bgl_ranks_to_match(v['gbps']):,.0f} (DOUBLE SUM rate) / "
             f"{bgl_ranks_to_match(v['gbps'], 'INT'):,.0f} (INT SUM rate)" for n, v in sorted(per_n.items())]
    return ("The reference's cross-processor conclusion (`writeup.tex:19`: BG/L's INT reduction overtakes one "
            "2012 GPU at ~500-600 ranks), restated: BG/L VN ranks, each at the per-rank rate of the reference's "
            "1024-rank run, needed to match the measured node — " + "; ".join(parts) + ".\n")


WRITEUP_BEGIN, WRITEUP_END = "<!-- scaling:begin -->", "<!-- scaling:end -->"


def update_writeup(path: str, table: str, source: str, crossover: str = "") -> bool:
    """Replace the text between the scaling markers of docs/WRITEUP.md with the measured table."""
    text = open(path).read()
    if WRITEUP_BEGIN not in text or WRITEUP_END not in text:
        return False
    head, rest = text.split(WRITEUP_BEGIN, 1)
    _, tail = rest.split(WRITEUP_END, 1)
    body = (f"\nMeasured by the driver's scaling run (`{source}`, via `tools/scaling.py --from`), next to the "
            "one-GPU projection it replaces:\n\n" + table + ("\n" + crossover if crossover else ""))
    with open(path, "w") as f:
        f.write(head + WRITEUP_BEGIN + body + WRITEUP_END + tail)
    return True


def from_driver(paths, out_dir: str, require=(1, 2, 4, 8), writeup: "str | None" = None) -> dict:
    """A driver's scaling record(s) (SCALE_r*.json: per-N bench.py runs, their printed lines kept in
    stdout tails) -> the results files, scaling.md, the reduce.c vector tables, the WRITEUP table
    (writeup_scaling.md; docs/WRITEUP.md's marked section too with ``writeup``) and both report
    figures (tools/report.py). Raises ScalingError — writing nothing — when a record was skipped, a
    required rank count is missing or any N is unverified."""
    results = []
    for p in paths:
        text = open(p).read()
        try:
            doc = json.loads(text)
        except ValueError:
            doc = None
        if isinstance(doc, dict) and doc.get("skipped"):
            raise ScalingError(f"{p}: the driver skipped the scaling run ({doc.get('reason', 'no reason given')})")
        results.extend(with_sidecar(r, os.path.dirname(os.path.abspath(p))) for r in parse_text(text))
    results = dedupe(results)
    head = [r for r in results if key_of(r)[0] == HEADLINE_MODEL]
    summ = summarise(head)
    per_n = next((v for k, v in summ.items() if k[0] == HEADLINE_MODEL), {})
    # (a run that printed only its diagnostic line carries the metric but no config)
    failed = {int(r["n_gpus"]): r.get("error") or "no value" for r in results
              if r.get("value") is None and (key_of(r)[0] == HEADLINE_MODEL or "1B-double" in str(r.get("metric")))}
    check_curve(per_n, require, failed)
    os.makedirs(out_dir, exist_ok=True)
    md = write(summ, out_dir)
    vs = summarise_vector(results)
    write_vector(vs, out_dir)
    write_collected(results, out_dir)
    table = writeup_table(per_n)
    with open(os.path.join(out_dir, "writeup_scaling.md"), "w") as f:
        f.write(table)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import report
    figs = report.make_figures(os.path.join(out_dir, "figures"), bench_path=paths[0],
                               vector_dir=os.path.join(out_dir, "vector_direct"))
    cross = crossover_text(per_n)
    with open(os.path.join(out_dir, "writeup_scaling.md"), "a") as f:
        f.write("\n" + cross)
    updated = update_writeup(writeup, table, ", ".join(os.path.basename(p) for p in paths), cross) if writeup else False
    return {"scaling_md": md, "writeup_table": table, "crossover": cross, "figures": figs, "writeup_updated": updated,
            "vector": sorted(vs)}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("inputs", nargs="*", help="files with bench.py JSON (default: stdin)")
    ap.add_argument("--out", default="results/scaling")
    ap.add_argument("--from", dest="from_", nargs="+", default=None, metavar="SCALE_rNN.json",
                    help="the driver's scaling record(s): results files, tables, the WRITEUP table and both "
                         "figures; fails (rc 2, nothing written) on a skipped run, a missing rank count "
                         "(--require) or an unverified N")
    ap.add_argument("--require", default="1,2,4,8", help="rank counts the curve must have (--from)")
    ap.add_argument("--update-writeup", default=None, metavar="docs/WRITEUP.md",
                    help="--from: also replace the marked scaling section of this file")
    a = ap.parse_args(argv)
    if a.from_:
        try:
            r = from_driver(a.from_, a.out, tuple(int(v) for v in a.require.split(",") if v), a.update_writeup)
        except ScalingError as e:
            print(f"[scaling] refusing to build the scaling curve: {e}", file=sys.stderr)
            return 2
        print(r["scaling_md"], end="")
        print(r["writeup_table"], end="")
        print(r["crossover"], end="")
        for p in r["figures"]:
            print(p)
        return 0
    results = []
    if a.inputs:
        for p in a.inputs:
            with open(p) as f:
                results.extend(with_sidecar(r, os.path.dirname(os.path.abspath(p))) for r in parse_text(f.read()))
    else:
        results.extend(with_sidecar(r) for r in parse_text(sys.stdin.read()))
    results = dedupe(results)
    if not results:
        print("[scaling] no bench.py results found", file=sys.stderr)
        return 1
    print(write(summarise(results), a.out), end="")
    vs = summarise_vector(results)
    if vs:
        print(write_vector(vs, a.out), end="")
    write_collected(results, a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
