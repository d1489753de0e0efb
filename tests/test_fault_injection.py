"""Failure detection under injected faults, on CPU ranks over gloo.

The reference had none: MPI return codes ignored (mpi/reduce.c:32-106), no result check
(B11), a stuck rank stalls until the SLURM walltime (mpi/submit_all.sh:4). Here a wrong
contribution must fail verification, and a crashed or hung rank must end the job with an error
within the process-group deadline — never a silent pass or an endless hang. The native twin
(bootstrap deadlines) is covered in tests/test_native_unit.py.
"""
import json
import os
import time

import pytest

from helpers import ROOT, torchrun

from cuda_mpi_reductions_amd.utils.fault import FaultInjector, FaultSpec, parse_fault_spec

BENCH = os.path.join(ROOT, "bench.py")
SCALAR = ["--gpus", "2", "--device", "cpu", "--elements", "200003", "--steps", "6", "--warmup", "2"]
VECTOR = ["--gpus", "2", "--config", "mpi_1m_int32_sum_cpu2", "--steps", "4", "--warmup", "1"]


def _json(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return json.loads(lines[0]) if lines else None


REHEARSE = ["--gpus", "4", "--device", "cpu", "--elements", "200003", "--steps", "6", "--warmup", "2",
            "--rehearse-stages", "--canary-timeout", "20", "--agree-timeout", "8", "--xrank-timeout", "2",
            "--no-decompose"]
STAGE = {"canary": "canary", "selfcheck": "fused self-check", "tune": "plan tuning"}


@pytest.mark.parametrize("site", ["canary", "selfcheck", "tune"])
@pytest.mark.parametrize("kind", ["raise", "hang", "exit"])
def test_optional_headline_stage_failure_on_one_of_four_ranks(tmp_path, site, kind):
    # the optional headline stages (the fused finish's canary and self-check, the
    # per-rank plan tuning) fail on rank 2 of 4 (gloo CPU ranks; --rehearse-stages runs them in their
    # CPU form). Whatever the failure, the job prints exactly one line within the budget:
    #   raise -> an agreed fallback (RCCL combine / the tuned default plan), named, and a verified number;
    #   hang  -> the bounded agreement names the stage and the lost rank, no number, rc != 0;
    #   exit  -> torchrun tears the job down and rank 0's armed line names the stage, rc != 0.
    t0 = time.time()
    r = torchrun(4, [BENCH, *REHEARSE, "--inject-fault", f"{kind}@2/{site}"], cwd=tmp_path, timeout=300)
    took = time.time() - t0
    lines = [ln for ln in r.stdout.splitlines() if "{" in ln]
    assert len(lines) == 1, (r.stdout, r.stderr[-3000:])
    d = json.loads(lines[0][lines[0].index("{"):])
    assert d["n_gpus"] == 4 and took < 120, (took, d)
    assert f"[fault] rank 2 {kind} at" in r.stderr
    if kind == "raise":
        assert r.returncode == 0, r.stderr[-3000:]
        assert d["verified"] is True and d["value"] > 0
        if site == "tune":
            assert d["config"]["collective"] == "fused"
            assert "rank 2: InjectedFault" in d["config"]["plan_reason"], d["config"]
            assert d["summary"]["plans"] == "tuned default x4"
        else:
            assert d["config"]["collective"] == "rccl"
            reason = d["config"]["collective_reason"]
            assert reason.startswith("canary: rank 2: InjectedFault" if site == "canary" else
                                     "self-check: rank 2: InjectedFault"), reason
    else:
        assert r.returncode != 0
        assert d["value"] is None and f"(stage: {STAGE[site]})" in d["error"], d
        if kind == "hang":  # (the canary's bound outlasts the helpers' wait, --canary-timeout + 10 s; a
            # hang before the self-check's steps is caught by its readiness agreement, --agree-timeout)
            want = {"canary": "within 30 s"}.get(site, "within 8 s")
            assert f"rank(s) 2 did not report {want}" in d["error"], d
        else:
            assert "terminated" in d["error"] or "rank(s) 2 did not report" in d["error"], d


def test_rehearsed_stages_pass_cleanly_on_four_ranks(tmp_path):
    # no fault: the CPU forms of the canary, the fused self-check (store mailboxes) and plan tuning
    # all pass; the headline runs over the fused finish's twin and verifies
    from helpers import bench_record
    r = torchrun(4, [BENCH, *REHEARSE], cwd=tmp_path, timeout=300,
                 env={"MIREDUCE_EXTRAS_DIR": str(tmp_path)})
    assert r.returncode == 0, r.stderr[-3000:]
    d = bench_record(r.stdout)
    assert d["verified"] is True and d["config"]["collective"] == "fused" and "plan_reason" not in d["config"]
    pt = d["plan_tuning"]
    assert len(pt["plan_by_rank"]) == 4 and all(len(t) == 5 for t in pt["gbps_by_rank"]) and "error" not in pt


def test_agree_is_bounded_and_names_the_missing_rank(tmp_path):
    # parallel.dist.agree: payloads in rank order; a rank that never reports is named after the
    # timeout (PeerLost) instead of holding the others in a collective
    script = tmp_path / "ag.py"
    script.write_text(
        "import sys, time\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "from cuda_mpi_reductions_amd.parallel import dist as pdist\n"
        "ctx = pdist.init(backend='gloo', device_type='cpu')\n"
        "out = open(f'r{ctx.rank}.txt', 'w')\n"
        "rows = pdist.agree(ctx, 'one', {'r': ctx.rank * 10})\n"
        "out.write(f\"rows {[x['r'] for x in rows]}\\n\"); out.flush()\n"
        "if ctx.rank == 2:\n"
        "    time.sleep(8); sys.exit(0)\n"
        "try:\n"
        "    pdist.agree(ctx, 'two', {}, timeout_s=2)\n"
        "except pdist.PeerLost as e:\n"
        "    out.write(f'lost {e.missing} {e.stage}\\n')\n"
        "out.close()\n")
    torchrun(3, [str(script)], cwd=tmp_path, timeout=120)
    got = [(tmp_path / f"r{r}.txt").read_text().splitlines() for r in range(3)]
    assert got[0] == got[1] == ["rows [0, 10, 20]", "lost [2] two"] and got[2] == ["rows [0, 10, 20]"], got


def test_parse_fault_spec():
    assert parse_fault_spec(None) == FaultSpec()
    assert parse_fault_spec("exit") == FaultSpec("exit", 1, 0, 0)
    assert parse_fault_spec("hang@3:17") == FaultSpec("hang", 3, 17, 0)
    assert parse_fault_spec("delay=250@0:2") == FaultSpec("delay", 0, 2, 250)
    assert parse_fault_spec("corrupt:5") == FaultSpec("corrupt", 1, 5, 0)
    assert parse_fault_spec("hang@1/teardown") == FaultSpec("hang", 1, 0, 0, "teardown")
    assert parse_fault_spec("delay=500@0/capture") == FaultSpec("delay", 0, 0, 500, "capture")
    assert parse_fault_spec("raise@2/tune") == FaultSpec("raise", 2, 0, 0, "tune")
    for site in ("canary", "selfcheck"):
        assert parse_fault_spec(f"hang@3/{site}").site == site
    from cuda_mpi_reductions_amd.utils.fault import InjectedFault
    inj = FaultInjector(parse_fault_spec("raise@1/selfcheck"))
    assert not inj.at(1, 0, "tune")
    with pytest.raises(InjectedFault):
        inj.at(1, 7, "selfcheck")  # (stepless site: any step)
    assert not inj.at(1, 7, "selfcheck")  # fires once
    for bad in ("boom", "exit@", "exit@x", "hang:-1", "delay=", "corrupt@1:2x"):
        with pytest.raises(ValueError):
            parse_fault_spec(bad)
    inj = FaultInjector(parse_fault_spec("corrupt@2:4"))
    assert not inj.at(1, 4) and not inj.at(2, 3) and inj.at(2, 4) and not inj.at(2, 4)


@pytest.mark.parametrize("args", [SCALAR, VECTOR], ids=["scalar", "vector"])
@pytest.mark.parametrize("step", [1, 4])
def test_corrupt_contribution_fails_verification(tmp_path, args, step):
    r = torchrun(2, [BENCH, *args, "--inject-fault", f"corrupt@1:{step}"], cwd=tmp_path, timeout=300)
    assert r.returncode == 1, r.stderr[-2000:]
    d = _json(r)
    assert d is not None and d["verified"] is False
    assert "[fault] rank 1 corrupt" in r.stderr


@pytest.mark.parametrize("args", [SCALAR, VECTOR], ids=["scalar", "vector"])
def test_straggler_delay_still_verifies(tmp_path, args):
    r = torchrun(2, [BENCH, *args, "--inject-fault", "delay=300@0:3"], cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json(r)
    assert d["verified"] is True


def test_crashed_rank_fails_job_fast(tmp_path):
    # rank 1 dies inside the timed loop; torchrun tears the job down (SIGTERM to rank 0), and rank 0's
    # armed diagnostic line is what gets printed: no number, the stage named (final_line.hpp)
    t0 = time.time()
    r = torchrun(2, [BENCH, *SCALAR, "--inject-fault", "exit@1:3", "--pg-timeout", "20"], cwd=tmp_path, timeout=300)
    assert r.returncode != 0
    d = _json(r)
    assert d is None or (d["value"] is None and "terminated" in d["error"] and "stage: timed steps" in d["error"]), d
    assert len([ln for ln in r.stdout.splitlines() if ln.startswith("{")]) <= 1
    assert time.time() - t0 < 120


def test_rank_killed_during_extras_keeps_the_verified_headline(tmp_path):
    # the headline is final, then rank 1 dies in the first extra: torchrun SIGTERMs rank 0, whose
    # signal handler prints the armed line — the measured, verified headline — exactly once
    r = torchrun(2, [BENCH, *SCALAR, "--inject-fault", "exit@1:0/extras"], cwd=tmp_path, timeout=300)
    assert r.returncode != 0  # the job did fail
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["verified"] is True and d["n_gpus"] == 2
    assert "terminated (signal) during the extras" in d["summary"]["extras_error"]


def test_hung_rank_hits_deadline(tmp_path):
    # rank 1 stops making progress inside the timed loop; rank 0's all-reduce times out after
    # --pg-timeout and the launcher tears the job down.
    t0 = time.time()
    r = torchrun(2, [BENCH, *SCALAR, "--inject-fault", "hang@1:4", "--pg-timeout", "8"], cwd=tmp_path, timeout=300)
    assert r.returncode != 0
    d = _json(r)
    assert d is None or d["value"] is None, d  # at most the diagnostic line, never a number
    assert "[fault] rank 1 hang" in r.stderr
    assert time.time() - t0 < 150


def test_hang_in_teardown_keeps_the_line_and_status(tmp_path):
    # rank 1 hangs after the line is printed (e.g. stuck destroying its communicator): the teardown
    # deadline ends every rank with the headline's status, well before the process-group timeout.
    t0 = time.time()
    r = torchrun(2, [BENCH, *SCALAR, "--inject-fault", "hang@1/teardown", "--teardown-deadline", "5",
                     "--pg-timeout", "300"], cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json(r)
    assert d is not None and d["verified"] is True
    assert "[fault] rank 1 hang at teardown" in r.stderr and "teardown exceeded 5 s" in r.stderr
    assert time.time() - t0 < 120


def test_rank_hung_before_init_ends_within_the_headline_deadline(tmp_path):
    # rank 1 never joins the process group (fault site "init"). Rank 0 armed its
    # diagnostic line and started the headline deadline BEFORE the rendezvous, so the job ends with
    # exactly one line (no number, stage "init") long before the process-group timeout.
    t0 = time.time()
    r = torchrun(2, [BENCH, *SCALAR, "--inject-fault", "hang@1/init", "--headline-deadline", "15",
                     "--pg-timeout", "120"], cwd=tmp_path, timeout=300)
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    d = json.loads(lines[0])
    assert d["value"] is None and "stage: init" in d["error"] and d["n_gpus"] == 2, d
    assert "[fault] rank 1 hang at process-group init" in r.stderr
    assert time.time() - t0 < 100


def test_self_spawned_rank0_dead_before_arming_parent_prints_the_line(tmp_path):
    # without a launcher, bench.py starts the ranks as a child and relays their
    # stdout; rank 0 dies before it armed anything, so no rank prints a line: the parent does (one
    # diagnostic line, rc != 0), within the run budget.
    from helpers import run as run_cmd
    import sys
    t0 = time.time()
    r = run_cmd([sys.executable, BENCH, *SCALAR, "--inject-fault", "exit@0/init", "--pg-timeout", "20"],
                cwd=tmp_path, timeout=300)
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    d = json.loads(lines[0])
    assert d["value"] is None and "without printing a result line" in d["error"] and d["n_gpus"] == 2, d
    assert time.time() - t0 < 120


def test_parent_enforces_the_run_budget(capsys):
    # the self-spawning parent's backstop: a child that outlives budget + grace is terminated (its
    # whole process group) and, having printed nothing, gets one diagnostic line from the parent
    import importlib.util
    import subprocess
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    b.PARENT_GRACE_S = 0.5
    child = subprocess.Popen(["sleep", "100"], stdout=subprocess.PIPE, start_new_session=True)
    t0 = time.time()
    rc = b._relay_child(child, time.time() + 1.0, 4)
    out = capsys.readouterr().out
    assert time.time() - t0 < 20 and rc != 0
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] is None and "exceeded the run budget" in d["error"] and d["n_gpus"] == 4


def test_child_line_is_relayed_once(capsys):
    # a child that prints its own result line: the parent relays it and adds nothing
    import importlib.util
    import subprocess
    import sys
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    code = "import json; print('noise'); print(json.dumps({'metric': 'm', 'value': 2.0, 'n_gpus': 2}))"
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, start_new_session=True)
    rc = b._relay_child(child, time.time() + 60, 2)
    out = capsys.readouterr().out
    assert rc == 0 and out.count("{") == 1 and "noise" in out and '"value": 2.0' in out


# ---------------------------------------------------------------- native apps on CPU ranks (MPICH)

from helpers import BIN, MPIRUN, ensure_built, run  # noqa: E402

needs_mpi = pytest.mark.skipif(not os.path.exists(MPIRUN), reason="MPICH not available")


@needs_mpi
@pytest.mark.parametrize("op", ["SUM", "MIN", "MAX"])
@pytest.mark.parametrize("dtypes", ["INT", "LONG", "FLOAT", "DOUBLE"])
def test_reduce_mpi_corrupt_detected(op, dtypes):
    ensure_built()
    r = run([MPIRUN, "-np", "3", os.path.join(BIN, "reduce_mpi"), "--ints=30001", "--doubles=30001", f"--dtypes={dtypes}",
             f"--ops={op}", "--retries=1", "--verify", "--inject-fault=corrupt@2:0"], timeout=120)
    assert r.returncode != 0
    assert "[fault] rank 2 corrupts" in r.stderr and "verification FAILED" in r.stderr


@needs_mpi
def test_reduce_mpi_crashed_rank_ends_job():
    ensure_built()
    t0 = time.time()
    r = run([MPIRUN, "-np", "2", os.path.join(BIN, "reduce_mpi"), "--ints=30001", "--doubles=30001", "--retries=3",
             "--inject-fault=exit@1:2"], timeout=120)
    assert r.returncode != 0
    assert time.time() - t0 < 60


def test_replay_probe_miss_on_one_rank_goes_eager_and_still_measures(tmp_path):
    # rank 1 misses the replay probe's deadline (injected delay past it); every
    # rank must agree to issue the headline eagerly, and the headline is still measured and
    # verified with rc 0 — the JSON names the rank and the reason.
    r = torchrun(2, [BENCH, *SCALAR, "--replay-probe", "on", "--probe-deadline", "1",
                     "--inject-fault", "delay=2500@1/capture"], cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json(r)
    assert d["verified"] is True and d["value"] > 0
    launch = d["config"]["launch"]
    assert launch.startswith("eager (replay probe failed: ") and "rank 1: 3 steps took" in launch, launch
    assert "[fault] rank 1 delay at replay probe" in r.stderr


def _final_line_child(code: str):
    import subprocess
    import sys
    pre = (f"import os, sys, signal, time\nsys.path.insert(0, {ROOT!r})\n"
           "from cuda_mpi_reductions_amd._native import native\nC = native()\n")
    return subprocess.run([sys.executable, "-c", pre + code], capture_output=True, text=True, timeout=60)


def test_final_line_chains_to_python_sigint_handler():
    # the once-guard prints the armed line and then hands SIGINT to the handler that was
    # there before (Python's: KeyboardInterrupt), instead of killing the process with SIG_DFL
    r = _final_line_child(
        "C.arm_final_line('{\"value\": 1}')\n"
        "try:\n"
        "    os.kill(os.getpid(), signal.SIGINT)\n"
        "    time.sleep(5)\n"
        "except KeyboardInterrupt:\n"
        "    print('KI', flush=True)\n"
        "print('emitted-again' if C.emit_final_line('{\"value\": 2}') else 'once', flush=True)\n")
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"value": 1}', "KI", "once"], r.stdout


def test_final_line_reaches_stdout_while_fd1_is_redirected():
    # fd 1 routed to stderr for a while (dist.stdout_to_stderr during the rendezvous): the line armed
    # before goes to the real stdout when the process is terminated then
    r = _final_line_child(
        "C.arm_final_line('{\"value\": 3}')\n"
        "os.dup2(2, 1)\n"
        "os.kill(os.getpid(), signal.SIGTERM)\n"
        "time.sleep(5)\n")
    assert r.returncode == -15
    assert r.stdout.strip() == '{"value": 3}' and '{"value": 3}' not in r.stderr, (r.stdout, r.stderr)


def test_final_line_reinstalls_over_a_later_handler():
    # a library that installs its own SIGTERM handler after the first arm: the next arm puts the guard
    # back on top and chains to that handler
    r = _final_line_child(
        "C.arm_final_line('{\"value\": 4}')\n"
        "signal.signal(signal.SIGTERM, lambda s, f: print('lib-handler', flush=True))\n"
        "C.arm_final_line('{\"value\": 5}')\n"
        "os.kill(os.getpid(), signal.SIGTERM)\n"
        "time.sleep(0.5)\n"
        "print('alive', flush=True)\n")
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"value": 5}', "lib-handler", "alive"], r.stdout


def test_final_line_leaves_an_ignored_signal_ignored():
    # SIGHUP ignored before the first arm (nohup) stays ignored — it must not print the
    # armed line and take the once-guard; the process goes on and its real line is the one printed
    r = _final_line_child(
        "signal.signal(signal.SIGHUP, signal.SIG_IGN)\n"
        "C.arm_final_line('{\"value\": null}')\n"
        "os.kill(os.getpid(), signal.SIGHUP)\n"
        "time.sleep(0.3)\n"
        "print('emitted' if C.emit_final_line('{\"value\": 6}') else 'lost', flush=True)\n")
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"value": 6}', "emitted"], r.stdout


def test_relayed_line_behind_a_fragment_counts_as_the_result(capsys):
    # a rank's line written on the signal path (write(2)) can follow an unterminated piece
    # of Python's buffered stdout on the same line; the self-spawning parent must still see a result
    # (and print no diagnostic line of its own after it)
    import importlib.util
    import subprocess
    import sys
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    code = ("import os, sys, json\nsys.stdout.write('[progress] half a li'); sys.stdout.flush()\n"
            "os.write(1, (json.dumps({'metric': 'm', 'value': 3.0, 'n_gpus': 2}) + '\\n').encode())\n")
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, start_new_session=True)
    rc = b._relay_child(child, time.time() + 60, 2)
    out = capsys.readouterr().out
    assert rc == 0 and out.count('"metric"') == 1 and '"value": 3.0' in out, out
    assert b._is_result_line('noise {"metric": "m", "value": null}') and not b._is_result_line("{not json")


@pytest.mark.parametrize("test_mode", [False, True])
def test_plan_for_rank_hook_only_in_test_runs(tmp_path, test_mode):
    # MIREDUCE_PLAN_FOR_RANK (forces a rank onto a plan candidate) is honoured only with
    # MIREDUCE_TEST=1, and the record then says so (plan_tuning.forced_by_env)
    from helpers import bench_record
    env = {"MIREDUCE_EXTRAS_DIR": str(tmp_path), "MIREDUCE_PLAN_FOR_RANK": "1=256x4x2 window 2"}
    if test_mode:
        env["MIREDUCE_TEST"] = "1"
    r = torchrun(2, [BENCH, "--gpus", "2", "--device", "cpu", "--elements", "200003", "--steps", "4", "--warmup", "1",
                     "--rehearse-stages", "--canary-timeout", "20", "--no-decompose"], cwd=tmp_path, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    pt = bench_record(r.stdout)["plan_tuning"]
    if test_mode:
        assert pt["plan_by_rank"][1] == "256x4x2 window 2" and pt["forced_by_env"] == {"1": "256x4x2 window 2"}
    else:
        assert "forced_by_env" not in pt
