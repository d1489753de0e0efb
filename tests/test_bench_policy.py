"""bench.py's measurement policies (pure functions, CPU): graph chunking and tuning length."""
import importlib.util
import os

from helpers import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_graph_chunk_auto():
    b = _bench()
    assert b._graph_chunk(0, 1000, issues_collective=False) == 1000  # kernel-only steps: one graph
    assert b._graph_chunk(0, 10000, issues_collective=False) == 4096
    assert b._graph_chunk(0, 1000, issues_collective=True) == 128  # RCCL in every step
    assert b._graph_chunk(16, 1000, issues_collective=False) == 16  # explicit wins


def test_auto_tune_steps_covers_about_30ms():
    b = _bench()
    assert b._auto_tune_steps(1e9) == 210  # the N=8 shard: 143 us per step at 7 TB/s
    assert b._auto_tune_steps(8e9) == 27
    assert b._auto_tune_steps(1e6) == 400 and b._auto_tune_steps(1e12) == 20  # clamps


def _watchdog_child(deadline, work_s, rc, side):
    import subprocess
    import sys
    code = (
        "import importlib.util, os, sys, time\n"
        f"spec = importlib.util.spec_from_file_location('b', os.path.join({ROOT!r}, 'bench.py'))\n"
        "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
        f"rec = b._Record({{'metric': 'm', 'value': 1.0}}, {{}}, {side!r})\n"
        f"g = b._ExtrasWatchdog(rec, {deadline}, {rc})\n"
        f"time.sleep({work_s})\n"
        "print('finished' if g.finish() else 'late', flush=True)\n"
        "sys.exit(7)\n")
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)


def test_extras_watchdog_prints_headline_and_exits_on_deadline(tmp_path):
    import json
    r = _watchdog_child(0.3, 30, 0, str(tmp_path / "x.json"))
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1 and "finished" not in r.stdout, (r.stdout, r.stderr)
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and "did not finish" in d["summary"]["extras_error"]
    assert "exceeded" in r.stderr


def test_extras_watchdog_stays_quiet_when_extras_finish(tmp_path):
    r = _watchdog_child(30, 0.1, 0, str(tmp_path / "x.json"))
    assert r.returncode == 7 and r.stdout.strip() == "finished", (r.stdout, r.stderr)


def test_plan_candidates_only_for_the_headline_shards():
    b = _bench()
    GB = 1 << 30
    # the tuned default (its XCD skew), equal rounds per XCD, twice the skew, the skew favouring the
    # even XCCs, the window runner-up
    cands = [(0, 0, 0, -1, None), (0, 0, 0, -1, 0), (0, 0, 0, -1, 40), (0, 0, 0, -1, -20), (256, 4, 2, 2, None)]
    assert b._plan_candidates(8e9, 8) == cands  # N=1 / N=2 shards
    assert b._plan_candidates(1e9, 8) == cands  # N=8 shard
    assert b._plan_candidates(0.5 * GB, 8) == [(0, 0, 0, -1, None)]
    assert b._plan_candidates(8e9, 4) == [(0, 0, 0, -1, None)] and b._plan_candidates(8e9, 2) == [(0, 0, 0, -1, None)]
    assert b._plan_key((256, 4, 2, 2, None)) == "256x4x2 window 2"
    assert b._plan_key((256, 8, 1, 0, None)) == "256x8x1 hipcc schedule"
    assert b._plan_key((0, 0, 0, -1, None)) == "tuned default" and b._plan_key((0, 0, 0, -1, 0)) == "tuned default, XCD skew 0"


def test_extras_watchdog_reports_the_extras_completed_so_far(tmp_path):
    # a hang mid-way through the extras (e.g. an RCCL collective at N>1) must still publish the rows
    # measured before it: their summary in the line, all of them in the sidecar it names
    import json
    side = tmp_path / "extras.json"
    import subprocess
    import sys
    code = (
        "import importlib.util, os, sys, time\n"
        f"spec = importlib.util.spec_from_file_location('b', os.path.join({ROOT!r}, 'bench.py'))\n"
        "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
        f"rec = b._Record({{'metric': 'm', 'value': 1.0}}, {{}}, {str(side)!r})\n"
        "g = b._ExtrasWatchdog(rec, 0.5, 0)\n"
        "rec.extras['reduce_c_vector'] = {'rows': {'direct': ['# DATATYPE OP NODES GB/sec', 'INT MAX 8   1.000']},\n"
        "                                 'reduce_direct': {'gibps': 3.5, 'verified': True}}\n"
        "time.sleep(30)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.stdout, r.stderr)
    d = json.loads(lines[0])
    assert "did not finish" in d["summary"]["extras_error"] and d["value"] == 1.0
    assert d["summary"]["reduce_c_gibps"]["direct"] == 3.5 and d["summary"]["extras_verified"] is True
    assert d["summary"]["extras_file"] == str(side)
    full = json.loads(side.read_text())
    v = full["reduce_c_vector"]
    assert v["rows"]["direct"][1] == "INT MAX 8   1.000" and "did not finish" in v["error"]
    assert full["value"] == 1.0 and full["summary"]["run"] == d["summary"]["run"]


def test_reduce_c_rows_summary_averages_retries_in_reduce_c_order():
    # the driver keeps the printed line: reduce.c's table rides in it as getAvgs-style means
    b = _bench()
    tab = [{"impl": "direct", "error": "x"}]
    for x, g in enumerate((1.0, 2.0)):
        for dt in ("INT", "DOUBLE"):
            for op in ("MAX", "MIN", "SUM"):
                tab.append({"retry": x, "dtype": dt, "op": op, "impl": "direct", "gibps": g, "verified": True})
    tab.append({"dtype": "INT", "op": "SUM", "impl": "rccl", "gibps": None})
    tab[3]["verified"] = False  # INT SUM, retry 0
    rows = b._reduce_c_means(tab)
    assert list(rows) == ["direct"]
    assert rows["direct"] == ("INT MAX 1.500; INT MIN 1.500; INT SUM 1.500!; "
                              "DOUBLE MAX 1.500; DOUBLE MIN 1.500; DOUBLE SUM 1.500")
    s = b._summarise({"reduce_c_vector": {"table": tab, "reduce_direct": {"gibps": 1.5}}})
    assert s["reduce_c_rows"] == rows and s["reduce_c_gibps"]["direct"] == 1.5


def test_summary_carries_the_decomposition_skew_and_exchange_wait():
    b = _bench()
    dec = {"local_gbps": 7300.0, "scaling_efficiency_vs_local": 0.97, "exchange_us_per_step": 4.2,
           "skew_us_per_step": 1.5, "exchange_wait_us": {"min_rank_median": 2.1, "max_rank_median": 3.4}}
    s = b._summarise({"decomposition": dec})
    assert s["skew_us"] == 1.5 and s["wait_us"] == [2.1, 3.4] and s["exchange_us"] == 4.2
    assert "wait_us" not in b._summarise({"decomposition": {"local_gbps": 1.0}})


class _StubWorkload:
    """Just what bench._selfcheck_slots reads: the op, slot allocation and the channel-free launch."""

    def __init__(self, op, value, dtype):
        import torch
        from types import SimpleNamespace
        self.cfg = SimpleNamespace(op=op)
        self._value, self._dtype = value, dtype
        self._torch = torch

    def new_slots(self, k):
        return self._torch.empty(k, dtype=self._dtype)

    def local(self, out):
        out.fill_(self._value)
        return out


def test_fused_selfcheck_compares_with_the_local_partials():
    # The fused finish's self-check (no torch pass over the array before the timed steps,
    # profiles/r3_selfcheck/): every slot must equal the channel-free launch's value, combined over
    # the group — exactly for MIN/MAX and integers, within a few ulps of the accumulator for SUM.
    import torch
    from types import SimpleNamespace
    b = _bench()
    ctx = SimpleNamespace(world_size=1, backend="gloo", device=torch.device("cpu"))
    wl = _StubWorkload("sum", 1000.0, torch.float32)
    eps = torch.finfo(torch.float32).eps
    ok, ref = b._selfcheck_slots(wl, torch.tensor([1000.0, 1000.0 + 2 * eps * 1000, 1000.0]), ctx)
    assert ok and ref["expected"] == 1000.0 and ref["tolerance"] > 0
    ok, _ = b._selfcheck_slots(wl, torch.tensor([1000.0, 1000.1, 1000.0]), ctx)
    assert not ok
    wl = _StubWorkload("max", 7.5, torch.float64)
    assert b._selfcheck_slots(wl, torch.tensor([7.5, 7.5, 7.5], dtype=torch.float64), ctx)[0]
    assert not b._selfcheck_slots(wl, torch.tensor([7.5, 7.5, 7.5 + 1e-12], dtype=torch.float64), ctx)[0]
    wl = _StubWorkload("sum", 123456789012, torch.int64)
    assert b._selfcheck_slots(wl, torch.tensor([123456789012] * 3), ctx)[0]
    assert not b._selfcheck_slots(wl, torch.tensor([123456789012, 123456789013, 123456789012]), ctx)[0]


def test_fused_selfcheck_two_ranks_gloo(tmp_path):
    # world 2 (gloo, CPU): the partials are combined over the group and the verdict is agreed; a
    # slot that matches only this rank's own partial (a broken exchange) fails on every rank.
    from helpers import torchrun
    script = tmp_path / "sc.py"
    script.write_text(
        "import importlib.util, os, sys, torch\n"
        f"sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r})\n"
        "from test_bench_policy import _StubWorkload, _bench\n"
        "from cuda_mpi_reductions_amd.parallel import dist as pdist\n"
        "b = _bench()\n"
        "ctx = pdist.init(backend='gloo', device_type='cpu')\n"
        "wl = _StubWorkload('sum', float(ctx.rank + 1), torch.float64)\n"
        "good = b._selfcheck_slots(wl, torch.tensor([3.0, 3.0], dtype=torch.float64), ctx)[0]\n"
        "own = float(ctx.rank + 1) if ctx.rank == 1 else 3.0\n"
        "bad = b._selfcheck_slots(wl, torch.tensor([own, own], dtype=torch.float64), ctx)[0]\n"
        "print(f'rank {ctx.rank} good={good} bad={bad}', flush=True)\n"
        "pdist.shutdown(ctx)\n")
    r = torchrun(2, [str(script)], timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "rank 0 good=True bad=False" in r.stdout and "rank 1 good=True bad=False" in r.stdout, r.stdout
