"""tools/scaling.py: bench.py JSON -> reference results format (getAvgs.sh / makePlots.gp)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import scaling  # noqa: E402


def _line(n, value, ms, model="xgmi_1b_double_sum: 1B double sum", op="SUM", dtype="fp64"):
    return {"metric": "reduction bandwidth (GB/s, whole node), 1B-double sum at 1/2/4/8 MI355X",
            "value": value, "unit": "GB/s", "n_gpus": n, "steps": 50, "warmup": 10,
            "ms_per_step": ms, "dtype": dtype, "config": {"model": model, "op": op}}


def test_parse_jsonl_mixed_with_logs_and_nested_documents():
    text = "RCCL version : x\n" + json.dumps(_line(1, 7300.0, 1.0959)) + "\nnoise {not json\n"
    assert [r["n_gpus"] for r in scaling.parse_text(text)] == [1]
    doc = {"runs": [{"n": 2, "result": _line(2, 14000.0, 0.5714)}, _line(4, 27000.0, 0.2963)]}
    assert sorted(r["n_gpus"] for r in scaling.parse_text(json.dumps(doc))) == [2, 4]


def test_summary_averages_repeats_and_efficiency():
    rs = [_line(1, 7300.0, 1.0), _line(1, 7100.0, 1.2), _line(2, 14000.0, 0.57), _line(8, 50400.0, 0.16)]
    s = scaling.summarise(rs)
    per_n = s[("xgmi_1b_double_sum", "DOUBLE", "SUM")]
    assert per_n[1]["gbps"] == 7200.0 and per_n[1]["runs"] == 2 and abs(per_n[1]["ms"] - 1.1) < 1e-12
    eff = scaling.efficiency(per_n)
    assert abs(eff[8][0] - 7.0) < 1e-12 and abs(eff[8][1] - 0.875) < 1e-12
    assert scaling.efficiency({2: {"gbps": 1.0}})[2] == (None, None)


def test_cli_writes_results_files_readable_by_plot_and_getavgs(tmp_path):
    src = tmp_path / "scale.jsonl"
    src.write_text("\n".join(json.dumps(_line(n, 7300.0 * n * 0.95 ** (n > 1), 8.0 / (7.3 * n)))
                             for n in (1, 2, 4, 8)) + "\n")
    out = tmp_path / "res"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling.py"), str(src), "--out", str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "| 8 |" in r.stdout and "95.0 %" in r.stdout
    rows = (out / "DOUBLE_SUM.txt").read_text().split("\n")
    assert rows[0] == ""  # getAvgs.sh writes a leading blank line
    assert rows[1].split()[:3] == ["DOUBLE", "SUM", "1"] and len(rows[1].split()) == 4
    import plot  # the unchanged reader used for the reference-style figures
    assert [n for n, _ in plot.read_results(str(out / "DOUBLE_SUM.txt"))] == [1, 2, 4, 8]


def test_decomposition_columns(tmp_path):
    # bench.py's per-N decomposition (local / exchange / skew) reaches the table
    a = _line(8, 50000.0, 0.16)
    a["decomposition"] = {"local_ms_per_step": 0.14, "exchange_us_per_step": 20.0, "skew_us_per_step": 1.5,
                          "scaling_efficiency_vs_local": 0.875}
    b = _line(8, 52000.0, 0.154)
    b["decomposition"] = {"local_ms_per_step": 0.142, "exchange_us_per_step": 12.0, "skew_us_per_step": 2.5,
                          "scaling_efficiency_vs_local": 0.922}
    c = _line(1, 7300.0, 1.0959)  # an older line without the field
    per_n = scaling.summarise([a, b, c])[("xgmi_1b_double_sum", "DOUBLE", "SUM")]
    assert abs(per_n[8]["local_ms"] - 0.141) < 1e-12 and per_n[8]["exchange_us"] == 16.0
    assert per_n[8]["skew_us"] == 2.0 and abs(per_n[8]["vs_local"] - 0.8985) < 1e-12
    assert per_n[1]["local_ms"] is None
    text = scaling.write({("xgmi_1b_double_sum", "DOUBLE", "SUM"): per_n}, str(tmp_path))
    assert "exchange us/step" in text and "| 0.1410 | 16.00 | 2.00 | 0.899 |  |" in text


def test_cli_without_results_fails(tmp_path):
    empty = tmp_path / "e.txt"
    empty.write_text("nothing here\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling.py"), str(empty),
                        "--out", str(tmp_path / "o")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no bench.py results" in r.stderr


def test_reduce_c_vector_table_becomes_results_files(tmp_path):
    # bench.py's reduce_c_vector.table (reduce.c's INT/DOUBLE x MAX/MIN/SUM) per N -> one getAvgs-format
    # file per (impl, DATATYPE, OP), the counterpart of the reference's mpi/results/<DT>_<OP>.txt.
    def with_table(n, scale):
        d = _line(n, 7300.0 * n, 8.0 / (7.3 * n))
        d["reduce_c_vector"] = {"table": [
            {"dtype": dt, "op": op, "impl": impl, "gibps": scale * n * (2 if impl == "direct" else 1)}
            for dt in ("INT", "DOUBLE") for op in ("MAX", "MIN", "SUM") for impl in ("rccl", "direct")]
            + [{"dtype": "INT", "op": "SUM", "impl": "rccl", "error": "RuntimeError: x"}]}
        return d
    src = tmp_path / "scale.jsonl"
    src.write_text("\n".join(json.dumps(with_table(n, s)) for n in (1, 2, 8) for s in (100.0, 300.0)) + "\n")
    out = tmp_path / "res"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling.py"), str(src), "--out", str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rows = (out / "vector_rccl" / "INT_SUM.txt").read_text().split("\n")
    # N=1 is left out (one rank has no cross-rank reduction to report)
    assert rows[0] == "" and rows[1:3] == ["INT SUM 2 400.00000", "INT SUM 8 1600.00000"] and rows[3] == ""
    assert (out / "vector_direct" / "DOUBLE_MAX.txt").read_text().split("\n")[2] == "DOUBLE MAX 8 3200.00000"
    assert "| direct | DOUBLE | MIN | 2 | 800.000 | 2 |" in (out / "vector.md").read_text()
    assert "| 1 |" not in (out / "vector.md").read_text()
    import plot
    assert [n for n, _ in plot.read_results(str(out / "vector_rccl" / "DOUBLE_MIN.txt"))] == [2, 8]


def test_bench_reduce_c_rows_through_getavgs_match_the_reference_shape(tmp_path):
    # bench.py's reduce_c_vector.rows[impl] are reduce.c's own stdout (header +
    # RETRY_COUNT retry-major rounds of INT/DOUBLE x MAX/MIN/SUM, "%s %s %d %10.3lf"); tools/scaling.py
    # concatenates the N > 1 runs into collected.txt and utils/getavgs.py (getAvgs.sh) turns that into
    # results/<DT>_<OP>.txt with exactly the shape of the reference's mpi/results/*.txt.
    import re
    from cuda_mpi_reductions_amd.utils import getavgs

    def bench_line(n):
        d = _line(n, 7300.0 * n, 8.0 / (7.3 * n))
        lines, table = ["# DATATYPE OP NODES GB/sec"], []
        for x in range(5):
            for dt in ("INT", "DOUBLE"):
                for op in ("MAX", "MIN", "SUM"):
                    g = 100.0 * n + x + (0.5 if dt == "DOUBLE" else 0.0)
                    lines.append("%s %s %d %10.3lf" % (dt, op, n, g))
                    table.append({"retry": x, "dtype": dt, "op": op, "impl": "direct", "gibps": g})
        d["reduce_c_vector"] = {"table": table, "rows": {"direct": lines}}
        return d
    src = tmp_path / "scale.jsonl"
    src.write_text("\n".join(json.dumps(bench_line(n)) for n in (1, 2, 4, 8)) + "\n")
    out = tmp_path / "res"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling.py"), str(src), "--out", str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    collected = out / "vector_direct" / "collected.txt"
    text = collected.read_text().splitlines()
    assert text.count("# DATATYPE OP NODES GB/sec") == 3  # the N = 2, 4, 8 runs; N = 1 left out
    assert len(text) == 3 * 31 and not [ln for ln in text if ln.startswith("INT MAX 1 ")]
    res = tmp_path / "results"
    getavgs.write_results(str(collected), str(res))
    ref_dir = "/root/reference/mpi/results"
    line_rx = re.compile(r"^(INT|DOUBLE) (SUM|MIN|MAX) \d+ \d+\.\d{5}$")
    for dt in ("INT", "DOUBLE"):
        for op in ("SUM", "MIN", "MAX"):
            got = (res / f"{dt}_{op}.txt").read_text().split("\n")
            assert got[0] == "" and got[-1] == "" and len(got) == 5, got  # blank line + N = 2, 4, 8
            assert all(line_rx.match(ln) for ln in got[1:-1]), got
            assert sorted(int(ln.split()[2]) for ln in got[1:-1]) == [2, 4, 8]
            mean8 = float([ln for ln in got[1:-1] if ln.split()[2] == "8"][0].split()[3])
            assert abs(mean8 - (800.0 + 2.0 + (0.5 if dt == "DOUBLE" else 0.0))) < 1e-4  # mean of retries 0..4
            ref_path = os.path.join(ref_dir, f"{dt}_{op}.txt")
            if os.path.exists(ref_path):  # the reference's own file has the same shape
                ref = open(ref_path).read().split("\n")
                assert ref[0] == "" and all(line_rx.match(ln) for ln in ref[1:] if ln)


def test_compact_lines_merge_their_sidecars(tmp_path):
    # round 5: the printed line carries a summary and names its sidecar (the full extras record);
    # the tool merges it (found by name next to the input when the recorded path is elsewhere), and
    # a line passed together with its own sidecar counts once
    side_dir = tmp_path / "out"
    side_dir.mkdir()
    lines = []
    for n, run in ((1, "r1"), (8, "r8")):
        ln = _line(n, 7300.0 * n * (0.95 if n > 1 else 1), 8.0 / (7.3 * n))
        ln["summary"] = {"run": run, "extras_file": f"/elsewhere/bench_extras_n{n}.json",
                         "plans": "0-7: tuned default" if n == 8 else "0: tuned default"}
        ln["verified"] = True
        ln["config"]["collective"] = "fused"
        full = dict(ln)
        full["decomposition"] = {"local_ms_per_step": 0.14 if n == 8 else 1.09, "exchange_us_per_step": 4.0,
                                 "skew_us_per_step": 1.0, "scaling_efficiency_vs_local": 0.97}
        (side_dir / f"bench_extras_n{n}.json").write_text(json.dumps(full))
        lines.append(json.dumps(ln))
    src = side_dir / "lines.jsonl"
    src.write_text("\n".join(lines) + "\n")
    rs = [scaling.with_sidecar(r, str(side_dir)) for r in scaling.parse_text(src.read_text())]
    assert all("decomposition" in r for r in rs)
    stale = dict(json.loads(lines[0]))
    stale["summary"] = {"run": "other", "extras_file": str(side_dir / "bench_extras_n1.json")}
    assert "decomposition" not in scaling.with_sidecar(stale)  # a different run's sidecar is not merged
    out = tmp_path / "res"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling.py"), str(src),
                        str(side_dir / "bench_extras_n8.json"), "--out", str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    row8 = [ln for ln in (out / "scaling.md").read_text().splitlines() if "| 8 |" in ln]
    cells = [c.strip() for c in row8[0].strip("|").split("|")] if len(row8) == 1 else []
    assert cells[8] == "1" and cells[9] == "0.1400", row8  # one run (line + sidecar), local ms merged
    assert cells[-3:] == ["fused", "yes", "0-7: tuned default"], row8  # combine, verified, per-rank plans


def test_bare_lines_give_the_vector_table_from_their_summary(tmp_path):
    # the driver keeps only the printed lines: reduce.c's per-N table comes from summary.reduce_c_rows
    lines = []
    for n in (1, 2, 8):
        ln = _line(n, 7300.0 * n, 8.0 / (7.3 * n))
        ln["summary"] = {"reduce_c_rows": {"direct": f"INT MAX {10.0 * n:.3f}; DOUBLE SUM {5.0 * n:.3f}!",
                                           "rccl": f"INT MAX {8.0 * n:.3f}"}}
        lines.append(json.dumps(ln))
    src = tmp_path / "scale.jsonl"
    src.write_text("\n".join(lines) + "\n")
    v = scaling.summarise_vector(scaling.parse_text(src.read_text()))
    assert v[("direct", "INT", "MAX")] == {2: {"gibps": 20.0, "runs": 1}, 8: {"gibps": 80.0, "runs": 1}}
    assert v[("direct", "DOUBLE", "SUM")][8]["gibps"] == 40.0 and v[("rccl", "INT", "MAX")][2]["gibps"] == 16.0
    out = tmp_path / "res"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling.py"), str(src), "--out", str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert (out / "vector_direct" / "INT_MAX.txt").read_text() == "\nINT MAX 2 20.00000\nINT MAX 8 80.00000\n"


def test_driver_record_line_in_the_stdout_tail(tmp_path):
    # the driver keeps the contract keys in `parsed` and the printed line whole in `run.stdout_tail`:
    # the tool reads the line (summary included) and counts the run once
    ln = _line(8, 57000.0, 0.14)
    ln["summary"] = {"run": "abc", "reduce_c_rows": {"direct": "INT MAX 2500.000"}}
    parsed = {k: v for k, v in ln.items() if k != "summary"}
    rec = {"n": 5, "runs": [{"n_gpus": 8, "parsed": parsed,
                             "run": {"stdout_tail": "[bench] x\n" + json.dumps(ln) + "\n"}}]}
    src = tmp_path / "SCALE.json"
    src.write_text(json.dumps(rec))
    rs = scaling.dedupe(scaling.parse_text(src.read_text()))
    assert len(rs) == 1 and rs[0]["summary"]["run"] == "abc"
    assert scaling.summarise_vector(rs)[("direct", "INT", "MAX")][8]["gibps"] == 2500.0


# ---------------------------------------------------------------- --from: the driver's SCALE record
def _scale_record(tmp_path, ns=(1, 2, 4, 8), unverified=(), reason_at=None):
    """A synthetic driver scaling record: per-N runs whose printed line sits in a stdout tail (as in
    BENCH_r*.json), every field bench.py's line carries."""
    runs = []
    for n in ns:
        line = _line(n, 7300.0 * n * (0.97 if n > 1 else 1.0), 8.0 / (7.3 * n * (0.97 if n > 1 else 1.0)))
        line["verified"] = n not in unverified
        line["config"]["collective"] = "fused"
        if n == reason_at:
            line["config"].update(collective="rccl", collective_reason="self-check: rank 2: InjectedFault: ...")
        line["summary"] = {"plans": f"tuned default x{n}", "reduce_c_rows": {
            "direct": "INT MAX 100.0; INT MIN 90.0; INT SUM 95.0; DOUBLE MAX 80.0; DOUBLE MIN 81.0; DOUBLE SUM 82.0"}}
        line["decomposition"] = {"local_ms_per_step": 1.0 / n, "exchange_us_per_step": 3.0, "skew_us_per_step": 1.0,
                                 "scaling_efficiency_vs_local": 0.99, "exchange_wait_us": {"min_rank_median": 0.5,
                                                                                          "max_rank_median": 2.0}}
        runs.append({"n": n, "rc": 0, "tail": "RCCL version : x\n" + json.dumps(line) + "\n---- stderr ----\n"})
    p = tmp_path / "SCALE_r06.json"
    p.write_text(json.dumps({"runs": runs}))
    return p


def test_from_driver_record_builds_everything(tmp_path):
    # one command turns the driver's scaling record into the results files, the
    # tables, the WRITEUP section (measured next to the projection it replaces) and both figures
    src = _scale_record(tmp_path, reason_at=4)
    writeup = tmp_path / "WRITEUP.md"
    writeup.write_text("# x\n\nbefore\n" + scaling.WRITEUP_BEGIN + "\nprojection table\n" + scaling.WRITEUP_END + "\nafter\n")
    out = tmp_path / "res"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling.py"), "--from", str(src), "--out", str(out),
                        "--update-writeup", str(writeup)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = [ln.split() for ln in (out / "DOUBLE_SUM.txt").read_text().splitlines() if ln]
    assert [int(x[2]) for x in rows] == [1, 2, 4, 8]
    table = (out / "writeup_scaling.md").read_text()
    assert "| 8 | 1 GB |" in table and "projection t_x = 0" in table
    eight = [ln for ln in table.splitlines() if ln.startswith("| 8 |")][0].split("|")
    assert abs(float(eight[6]) - scaling.projection(8)) < 1.0  # the projection kept alongside
    assert "rccl (self-check: rank 2" in table  # the fallback is named where it happened
    text = writeup.read_text()
    assert "projection table" not in text and "Measured by the driver's scaling run" in text and "after" in text
    assert (out / "figures" / "int.png").stat().st_size > 10000 and (out / "figures" / "double.png").exists()
    assert (out / "vector_direct" / "DOUBLE_SUM.txt").exists()  # reduce.c's own table, N > 1
    assert "decomposition" not in table and "| 3.00 |" in table  # exchange us/step column
    # the reference's cross-processor conclusion (writeup.tex:19), restated for the measured node
    assert "writeup.tex:19" in table and "N=8: " in table and "writeup.tex:19" in text


def test_bgl_ranks_to_match():
    # mpi/results/DOUBLE_SUM.txt: 60.9754 GiB/s at 1024 ranks -> 0.059546 GiB/s per rank; one GiB/s of
    # MI355X needs 1/0.059546 = 16.79 such ranks; the reference's own INT SUM at 1024 ranks matches itself
    assert abs(scaling.bgl_ranks_to_match(1 / scaling_gib()) - 1024 / 60.9754) < 1e-6
    assert abs(scaling.bgl_ranks_to_match(146.818 / scaling_gib(), "INT") - 1024) < 1e-6


def scaling_gib():
    return 1e9 / 2 ** 30


def test_from_driver_record_refuses_partial_or_unverified_curves(tmp_path):
    tool = os.path.join(ROOT, "tools", "scaling.py")
    for kw, want in (({"ns": (1, 2, 8)}, "no headline result for N=4"),
                     ({"unverified": (8,)}, "not verified: N=8 (verification FAILED)")):
        src = _scale_record(tmp_path, **kw)
        out = tmp_path / "res_bad"
        r = subprocess.run([sys.executable, tool, "--from", str(src), "--out", str(out)], capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 2 and want in r.stderr, (r.stdout, r.stderr)
        assert not out.exists()  # nothing written, nothing interpolated
    # a rank count whose run printed only its diagnostic line: the refusal quotes it
    src = _scale_record(tmp_path, ns=(1, 2, 4))
    doc = json.loads(src.read_text())
    diag = {"metric": doc["runs"][0]["tail"].split('"metric": "')[1].split('"')[0], "value": None, "n_gpus": 8,
            "error": "headline phase did not finish within 155 s (stage: canary); no measurement"}
    doc["runs"].append({"n": 8, "rc": 2, "tail": json.dumps(diag)})
    src.write_text(json.dumps(doc))
    r = subprocess.run([sys.executable, tool, "--from", str(src), "--out", str(tmp_path / "x")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2 and "N=8 (its run: headline phase did not finish" in r.stderr, r.stderr
    skipped = tmp_path / "SCALE_skip.json"
    skipped.write_text(json.dumps({"skipped": True, "reason": "no 8-GPU node"}))
    r = subprocess.run([sys.executable, tool, "--from", str(skipped), "--out", str(tmp_path / "s")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "skipped the scaling run (no 8-GPU node)" in r.stderr


def test_projection_matches_the_writeup_model():
    # docs/WRITEUP.md §2: shard G GB in G x 135.56 us + 1.9 us per launch (+ t_x)
    assert abs(scaling.projection(8) - 8e9 / (137.46e-6) / 1e9) < 1.0 and round(scaling.projection(8)) == 58199
    assert scaling.projection(8, 5.0) < scaling.projection(8) < 8 * scaling.projection(1)


def test_report_figures_regenerate_from_committed_data(tmp_path):
    # the reference's two figures (mpi/makePlots.gp), regenerated from data in the
    # repo: BG/L VN curves, the CUDA constants, the 8-CPU MPICH curve, the MI355X lines
    import report
    paths = report.make_figures(str(tmp_path), bench_path=os.path.join(ROOT, "BENCH_r05.json"))
    assert sorted(os.path.basename(p) for p in paths) == ["double.png", "int.png"]
    assert all(os.path.getsize(p) > 10000 for p in paths)
    s = report.series({"INT SUM": {"gbps": 7200.0}}, report.bench_vector_n1(os.path.join(ROOT, "BENCH_r05.json")),
                      "", report.DEFAULT_MPICH)
    labels = {lab: data for lab, _, data in s["INT"]}
    assert abs(labels["BG/L VN SUM"][1024] - 146.818 / report.GIB_PER_GB) < 1e-6  # mpi/results/INT_SUM.txt
    assert labels["ref CUDA SUM"] == 90.8413 and labels["MI355X 1 GPU SUM"] == 7200.0
    assert 1 in labels["reduce.c, 8-CPU MPICH SUM"] and 8 in labels["reduce.c, 8-CPU MPICH SUM"]
    assert labels["MI355X reduce.c (direct) SUM"][1] > 1000  # BENCH_r05's N=1 direct row (GiB/s -> GB/s)


def test_bare_driver_line_decomposition_from_its_summary(tmp_path):
    # the driver's records keep the printed line only (its sidecar stays on the GPU box): the table's
    # decomposition columns come from the line's summary (local GB/s, exchange, skew, fused wait)
    out = tmp_path / "r"
    r = scaling.from_driver([os.path.join(ROOT, "BENCH_r05.json")], str(out), require=(1,))
    row = [ln for ln in r["writeup_table"].splitlines() if ln.startswith("| 1 |")][0].split("|")
    assert row[9].strip() == "1091.1" and row[10].strip() == "3.81"  # local us/step, exchange us/step
    v = scaling.summarise(scaling.dedupe(scaling.parse_text(open(os.path.join(ROOT, "BENCH_r05.json")).read())))
    per_n = v[("xgmi_1b_double_sum", "DOUBLE", "SUM")][1]
    assert per_n["verified"] is True and per_n["wait_min_us"] == 0.24 and per_n["runs"] == 1
