"""Native C++ unit tests (host code), the TCP bootstrap under torchrun and mpirun, host
sanitizers (ASan/UBSan on host code), and the resumable sweep orchestration."""
import json
import os
import re
import sys
import subprocess

import pytest

from helpers import BIN, MPIRUN, ROOT, ensure_built, free_port, run, torchrun


@pytest.fixture(scope="module", autouse=True)
def built():
    ensure_built()


def test_host_unit():
    r = run([os.path.join(BIN, "host_unit")])
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout


@pytest.mark.parametrize("nproc", [2, 4])
def test_bootstrap_torchrun(nproc):
    r = torchrun(nproc, ["--no-python", os.path.join(BIN, "bootstrap_test")], timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    assert f"bootstrap_test world={nproc} launcher=torchrun PASSED" in r.stdout


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="MPICH not available")
def test_bootstrap_mpirun():
    r = run([MPIRUN, "-np", "3", os.path.join(BIN, "bootstrap_test")], timeout=180,
            env={"MIREDUCE_BOOTSTRAP_PORT": str(free_port())})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "bootstrap_test world=3 launcher=mpich PASSED" in r.stdout


def test_host_sanitizers():
    subprocess.run(["make", "-C", ROOT, "asan"], check=True, stdout=subprocess.DEVNULL)
    r = run([os.path.join(ROOT, "build", "asan", "host_unit")], env={"ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0, r.stderr
    if os.path.exists(MPIRUN):
        r = run([MPIRUN, "-np", "2", os.path.join(ROOT, "build", "asan", "reduce_mpi"), "--ints=64k",
                 "--doubles=64k", "--retries=1", "--verify"], timeout=300, env={"ASAN_OPTIONS": "detect_leaks=0"})
        assert r.returncode == 0, r.stderr[-3000:]
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_experiment_tools_build():
    # tools/window_ab.hip, dyntail_ab.hip and i32sum_ab.hip include the production kernel header directly
    # (their A/Bs run the real kern::reduce_stream): they must keep compiling as it changes.
    subprocess.run(["make", "-C", ROOT, "-j8", "window_ab", "dyntail_ab", "i32sum_ab"], check=True, stdout=subprocess.DEVNULL)
    for b in ("window_ab", "dyntail_ab", "i32sum_ab"):
        assert os.path.exists(os.path.join(BIN, b))


def test_threaded_host_references_race_free():
    # SURVEY.md §5.2 race detection: the multi-threaded CPU oracles under ThreadSanitizer agree
    # with their single-threaded results, and TSan reports nothing (it exits 66 on a report).
    subprocess.run(["make", "-C", ROOT, "tsan"], check=True, stdout=subprocess.DEVNULL)
    r = run([os.path.join(ROOT, "build", "tsan", "race_unit")], timeout=300,
            env={"TSAN_OPTIONS": "halt_on_error=1 exitcode=66"})
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "ThreadSanitizer" not in r.stderr and "ok" in r.stdout


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="MPICH not available")
def test_sweep_resume_and_collect(tmp_path):
    out = tmp_path / "sweep"
    cmd = ["python", os.path.join(ROOT, "tools", "sweep.py"), "--app", "reduce_mpi", "--ranks", "1,2",
           "--out", str(out), "--", "--ints=16k", "--doubles=16k", "--retries=2"]
    r = run(cmd, timeout=300)
    assert r.returncode == 0, r.stderr
    assert (out / "stdout-reduce_mpi-P2.txt").exists() and (out / "results" / "DOUBLE_MAX.txt").exists()
    res = (out / "results" / "INT_SUM.txt").read_text().splitlines()
    assert res[0] == "" and [ln.split()[2] for ln in res[1:]] == ["1", "2"]
    r2 = run(cmd, timeout=300)
    assert "P=1: done, skipping" in r2.stdout and "P=2: done, skipping" in r2.stdout


def test_sweep_knob_grid_settings():
    # the RCCL knob grid (default 2 x 2 x 3 settings), named per setting, with
    # "default" meaning the variable is left unset and every other knob removed from the environment
    import importlib.util
    spec = importlib.util.spec_from_file_location("sweep_knobs", os.path.join(ROOT, "tools", "sweep.py"))
    sw = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sw)
    st = sw.knob_settings()
    assert len(st) == 12 and len({n for n, _ in st}) == 12
    names = dict(st)
    assert names["rccl-ring-simple-chdefault"] == {"NCCL_ALGO": "Ring", "NCCL_PROTO": "Simple",
                                                   "NCCL_MIN_NCHANNELS": None}
    assert names["rccl-tree-ll128-ch32"]["NCCL_MIN_NCHANNELS"] == "32"
    os.environ["NCCL_PROTO"] = "LL"
    try:
        env = sw.knob_env({"NCCL_ALGO": "Tree", "NCCL_MIN_NCHANNELS": None})
    finally:
        os.environ.pop("NCCL_PROTO")
    assert env["NCCL_ALGO"] == "Tree" and "NCCL_PROTO" not in env and "NCCL_MIN_NCHANNELS" not in env


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="MPICH not available")
def test_sweep_rccl_knobs_writes_getavgs_results_per_setting(tmp_path):
    # the knob sweep's orchestration on CPU ranks (reduce_mpi: the same reduce.c rows; MPICH ignores
    # the NCCL_* variables): one getAvgs results directory per setting and the comparison table
    out = tmp_path / "knobs"
    r = run(["python", os.path.join(ROOT, "tools", "sweep.py"), "--rccl-knobs", "--app", "reduce_mpi", "--ranks", "2",
             "--knob-grid", "NCCL_ALGO=Ring,Tree;NCCL_PROTO=Simple", "--out", str(out), "--",
             "--ints=16k", "--doubles=16k", "--retries=2"], timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    for name, algo in (("rccl-ring-simple", "Ring"), ("rccl-tree-simple", "Tree")):
        sub = out / name
        assert json.loads((sub / "knobs.json").read_text()) == {"NCCL_ALGO": algo, "NCCL_PROTO": "Simple"}
        res = (sub / "results" / "DOUBLE_SUM.txt").read_text().splitlines()
        assert res[0] == "" and res[1].split()[:3] == ["DOUBLE", "SUM", "2"]
    md = (out / "rccl_knobs.md").read_text()
    rows = [ln for ln in md.splitlines() if ln.startswith("| DOUBLE | SUM | 2 |")]
    assert len(rows) == 2 and sum("**" in ln for ln in rows) >= 1, md


def test_sweep_rccl_knobs_env_reaches_the_json(tmp_path):
    # env passthrough: bench.py's reduce.c config on two gloo CPU ranks records the knobs it ran with
    out = tmp_path / "knobs_bench"
    r = run(["python", os.path.join(ROOT, "tools", "sweep.py"), "--rccl-knobs", "--app", "bench", "--ranks", "2",
             "--knob-grid", "NCCL_ALGO=Tree;NCCL_MIN_NCHANNELS=default,16", "--out", str(out), "--",
             "--config", "mpi_1m_int32_sum_cpu2", "--steps", "2", "--warmup", "1"], timeout=600,
            env={"NCCL_PROTO": "LL"})
    assert r.returncode == 0, r.stderr[-2000:]
    got = {}
    for name in ("rccl-tree-chdefault", "rccl-tree-ch16"):
        d = json.loads((out / name / "bench.jsonl").read_text().splitlines()[0])
        assert d["verified"] is True
        got[name] = d["config"]["rccl_env"]
    assert got == {"rccl-tree-chdefault": "NCCL_ALGO=Tree", "rccl-tree-ch16": "NCCL_ALGO=Tree NCCL_MIN_NCHANNELS=16"}


def test_sweep_node_preset_matrix():
    # --preset node: fabric roofline once, reduce.c vector mode over RCCL AND the direct one-kernel
    # collectives (graph-replayed), then the north-star bench — VERDICT r1 item 3/4.
    import importlib.util
    spec = importlib.util.spec_from_file_location("sweep", os.path.join(ROOT, "tools", "sweep.py"))
    sw = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sw)
    plan = sw.node_preset([])
    names = [e[1] for e in plan]
    assert names[0] == "fabric" and plan[0][0] == "bandwidth_test" and "--peer" in plan[0][3] and plan[0][2] is None
    for coll in ("reduce", "allreduce", "direct-reduce", "direct"):
        e = plan[names.index(f"vector-{coll}")]
        assert e[0] == "reduce_xgmi" and f"--collective={coll}" in e[3] and "--graph" in e[3]
    for coll in ("allreduce", "fused"):
        e = plan[names.index(f"scalar-{coll}")]
        assert "--mode=scalar" in e[3] and f"--collective={coll}" in e[3] and "--graph" in e[3]
    assert names[-1] == "bench"


def test_sweep_retries_a_taken_rendezvous_port(tmp_path, monkeypatch):
    # A launcher that loses its port to another process between free_port() and its bind fails with
    # EADDRINUSE: the point is relaunched once on a new port; any other failure is recorded as is.
    import importlib.util
    import sys
    spec = importlib.util.spec_from_file_location("sweep_retry", os.path.join(ROOT, "tools", "sweep.py"))
    sw = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sw)
    marker = tmp_path / "launched_once"
    script = ("import os, sys\n"
              f"m = {str(marker)!r}\n"
              "if not os.path.exists(m):\n"
              "    open(m, 'w').close()\n"
              "    sys.stderr.write('RuntimeError: EADDRINUSE: address already in use\\n'); sys.exit(1)\n"
              "print('INT SUM 2   1.000')\n")
    calls = []

    def fake_command(app, p, extra):
        calls.append(p)
        return [sys.executable, "-c", script]
    monkeypatch.setattr(sw, "command", fake_command)
    assert sw.run_points("reduce_xgmi", "x", [2], [], str(tmp_path), 60, False) == 0
    assert calls == [2, 2] and (tmp_path / "stdout-x-P2.rc").read_text().strip() == "0"
    assert "INT SUM 2" in (tmp_path / "stdout-x-P2.txt").read_text()
    monkeypatch.setattr(sw, "command", lambda app, p, extra: [sys.executable, "-c", "import sys; sys.exit(5)"])
    assert sw.run_points("reduce_xgmi", "y", [2], [], str(tmp_path), 60, False) == 1
    assert (tmp_path / "stdout-y-P2.rc").read_text().strip() == "5"
    assert not sw._port_taken("some other failure") and sw._port_taken(b"bind: Address already in use")


def test_plot_tool(tmp_path):
    res = tmp_path / "results"
    res.mkdir()
    (res / "INT_SUM.txt").write_text("\nINT SUM 1 100.0\nINT SUM 2 190.0\n")
    r = run(["python", os.path.join(ROOT, "tools", "plot.py"), "--results", str(res), "--out", str(tmp_path / "p"),
             "--reference-cuda"], timeout=300)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "p" / "int.png").exists()


@pytest.mark.parametrize("rank", [0, 1])
def test_bootstrap_missing_peer_fails_fast(rank):
    # SURVEY §5.3 failure detection: a rank whose peer never shows up gets an error after the
    # bootstrap timeout instead of hanging.
    import time
    t0 = time.time()
    r = run([os.path.join(BIN, "bootstrap_test")], timeout=60,
            env={"RANK": str(rank), "WORLD_SIZE": "2", "LOCAL_RANK": str(rank), "MASTER_ADDR": "127.0.0.1",
                 "MIREDUCE_BOOTSTRAP_PORT": str(free_port()), "MIREDUCE_BOOTSTRAP_TIMEOUT": "2"})
    assert r.returncode == 2, (r.returncode, r.stderr)
    assert ("timed out" in r.stderr) or ("cannot connect" in r.stderr)
    assert time.time() - t0 < 30


def _spawn_bootstrap_ranks(world, fault, timeout_s="3"):
    import subprocess
    port = str(free_port())
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MIREDUCE_BOOTSTRAP_PORT=port, MIREDUCE_BOOTSTRAP_TIMEOUT=timeout_s,
                   MIREDUCE_INJECT_FAULT=fault)
        procs.append(subprocess.Popen([os.path.join(BIN, "bootstrap_test")], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    return procs


@pytest.mark.parametrize("step", [0, 2, 4])
def test_bootstrap_peer_crash_detected(step):
    # Injected crash of rank 1 mid-exchange: every other rank fails with a bootstrap error quickly
    # (the reference's MPI job would hang or die with MPI_ERRORS_ARE_FATAL, mpi/reduce.c:32-106).
    import time
    t0 = time.time()
    procs = _spawn_bootstrap_ranks(3, f"exit@1:{step}")
    outs = [p.communicate(timeout=60) for p in procs]
    codes = [p.returncode for p in procs]
    assert codes[1] == 3, outs[1]
    assert "[fault] rank 1 exits" in outs[1][1]
    for r in (0, 2):
        assert codes[r] == 2, (r, codes, outs[r])
        assert "bootstrap" in outs[r][1]
    assert time.time() - t0 < 30


def test_bootstrap_peer_hang_detected():
    # Injected hang of rank 2: the others hit the bootstrap deadline (3 s) and exit with an error;
    # the hung rank is then killed, as a launcher would.
    import time
    t0 = time.time()
    procs = _spawn_bootstrap_ranks(3, "hang@2:3", timeout_s="3")
    try:
        for r in (0, 1):
            out, err = procs[r].communicate(timeout=60)
            assert procs[r].returncode == 2, (r, err)
            assert "timed out" in err or "peer closed" in err, err
        assert time.time() - t0 < 30
        assert procs[2].poll() is None  # still hung
    finally:
        procs[2].kill()
        procs[2].communicate()


def test_slurm_scripts_dry_run():
    # tools/slurm/ plays the role of mpi/submit_all.sh + mpi/ccni_vn.sh (SLURM job orchestration).
    env = dict(os.environ, DRY_RUN="1", PARTITION="mi355x", EXTRA="--dtypes=INT,DOUBLE --retries=2")
    r = run(["bash", os.path.join(ROOT, "tools", "slurm", "submit_all.sh"), "1", "8"], env=env, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 2 and lines[1].startswith("sbatch -p mi355x --nodes 1 --ntasks-per-node 8 --gpus-per-node 8")
    env.update(SLURM_NTASKS="8", SLURM_JOB_ID="42", MODE="scalar")
    r = run(["bash", os.path.join(ROOT, "tools", "slurm", "mi355x_sweep.sbatch")], env=env, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1].endswith("reduce_xgmi --mode=scalar --dtypes=INT,DOUBLE --retries=2")
    bad = run(["bash", os.path.join(ROOT, "tools", "slurm", "submit_all.sh"), "16"], env=env, timeout=60)
    assert bad.returncode == 2


def test_plot_shmoo_tool(tmp_path):
    csv = os.path.join(ROOT, "profiles", "r1_bench", "shmoo_double_sum_r1.csv")
    out = tmp_path / "shmoo.png"
    r = run(["python", os.path.join(ROOT, "tools", "plot_shmoo.py"), csv, "-o", str(out), "--title", "t"], timeout=300)
    assert r.returncode == 0, r.stderr
    assert out.exists() and out.stat().st_size > 1000


def test_cmake_build_and_ctest(tmp_path):
    """The CMake build configures, builds the CPU-only targets and passes
    their ctest entries (the HIP targets are the Makefile's, built by ensure_built)."""
    b = tmp_path / "cmake"
    r = run(["cmake", "-S", ROOT, "-B", str(b), "-G", "Ninja", "-DMIREDUCE_ASAN=ON"], timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    targets = ["host_unit"] + (["reduce_mpi"] if os.path.exists(MPIRUN) else [])
    r = run(["cmake", "--build", str(b), "-j4", "--target"] + targets, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    r = run(["ctest", "--test-dir", str(b), "-R", "host_unit|reduce_mpi", "--output-on-failure"], timeout=300,
            env={"ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "tests passed" in r.stdout


def test_prof_db_summary_and_steady_overlap(tmp_path):
    """tools/prof_db.py on a synthetic rocpd-style SQLite file: per-kernel table, and --steady's
    period / overlap of back-to-back kernels (two lanes overlapping vs one lane with gaps)."""
    import sqlite3
    db = tmp_path / "t_results.db"
    c = sqlite3.connect(db)
    c.execute("create table kernels (name text, start integer, end integer)")
    # lane-overlapped run: a kernel every 100 us lasting 150 us; then idle; then a gapped run
    rows = [("reduce_stream<x>", i * 100_000, i * 100_000 + 150_000) for i in range(20)]
    rows += [("reduce_stream<x>", 10_000_000 + i * 200_000, 10_000_000 + i * 200_000 + 150_000) for i in range(5)]
    rows += [("fill_kernel", 50_000_000, 50_010_000)]
    c.executemany("insert into kernels values (?, ?, ?)", rows)
    c.commit()
    c.close()
    r = run([sys.executable, os.path.join(ROOT, "tools", "prof_db.py"), str(db), "--steady", "reduce_stream"])
    assert r.returncode == 0, r.stderr
    assert "25 x     150.00 us" in r.stdout and "fill_kernel" in r.stdout
    m = re.search(r"steady: 20 x 'reduce_stream' back to back: period ([0-9.]+) us per kernel, mean duration "
                  r"150.00 us, >= 2 running ([0-9.]+) %", r.stdout)
    assert m and abs(float(m.group(1)) - 102.5) < 0.01 and float(m.group(2)) > 40, r.stdout
