"""The native apps on a real MI355X: QA protocol, CLI parity paths, verification, output formats."""
import json
import os
import re
import sys

import pytest

from helpers import BIN, ensure_built, run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def built():
    ensure_built()


def reduction(tmp_path, *args, timeout=600):
    r = run([os.path.join(BIN, "reduction"), "--qatest", "--log=none", *args], cwd=tmp_path, timeout=timeout)
    return r


@pytest.mark.parametrize("method", ["SUM", "MIN", "MAX"])
@pytest.mark.parametrize("type_", ["int", "int64", "float", "double"])
def test_reduction_app_methods_types(tmp_path, method, type_):
    r = reduction(tmp_path, f"--method={method}", f"--type={type_}", "--n=3000017", "--iterations=5")
    assert r.returncode == 0, r.stdout + r.stderr
    assert re.search(r"&&&& PASSED reduction", r.stderr)
    assert re.search(r"Reduction, Throughput = [0-9.]+ GB/s, Time = [0-9.]+ s, Size = 3000017 Elements, "
                     r"NumDevsUsed = 1, Workgroup = \d+", r.stdout)
    assert "GPU result = " in r.stdout and "CPU result = " in r.stdout


@pytest.mark.parametrize("kernel", range(9))
def test_reduction_app_every_kernel(tmp_path, kernel):
    r = reduction(tmp_path, "--method=SUM", "--type=double", f"--kernel={kernel}", "--n=1000001", "--iterations=3")
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("flags", [["--cpufinal"], ["--cputhresh=100000"], ["--maxblocks=7"],
                                   ["--threads=1024", "--unroll=16"], ["--policy=default", "--unroll=2"],
                                   ["--acc=int"], ["--fill=device", "--pattern=iotamod"]])
def test_reduction_app_paths(tmp_path, flags):
    r = reduction(tmp_path, "--method=MAX" if "--acc=int" not in flags else "--method=SUM", "--n=2000003",
                  "--iterations=3", *flags)
    assert r.returncode == 0, r.stdout + r.stderr


# ---- C6 parity: the reference's timed multi-pass loop (reduction.cpp:319-374). n = 2^24 doubles
# (the reference default): kernel 6 makes 64 partials (maxblocks 64); kernels 7/8 make their
# persistent grid of partials. (kernel, cputhresh|cpufinal) -> (passes, partials folded on host).
C6_CASES = [
    (6, "--cpufinal", 1, 64), (6, "--cputhresh=1", 2, 0), (6, "--cputhresh=2", 2, 0),
    (6, "--cputhresh=33", 2, 0), (6, "--cputhresh=1000", 1, 64),
    (7, "--cputhresh=1", 1, 0), (8, "--cputhresh=1", 2, 0),
    (7, "--cputhresh=2", 2, 0), (7, "--cputhresh=33", 2, 0), (8, "--cputhresh=1000", 1, "grid"),
    (7, "--cpufinal", 1, "grid"), (2, "--cputhresh=1000", 2, 256), (0, "--cputhresh=33", None, None),
]


@pytest.mark.parametrize("kernel,flag,passes,folded", C6_CASES, ids=lambda v: str(v))
@pytest.mark.parametrize("method", ["SUM", "MIN"])
def test_reduction_multipass_cputhresh(tmp_path, kernel, flag, passes, folded, method):
    js = tmp_path / "c6.json"
    r = reduction(tmp_path, f"--method={method}", "--type=double", f"--kernel={kernel}", flag,
                  "--iterations=3", f"--json={js}")
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(js.read_text().splitlines()[-1])
    assert d["verified"] is True
    if passes is not None:
        assert d["passes"] == passes, d
    if folded == "grid":
        assert d["host_folded"] == d["grid"] > 1, d
    elif folded is not None:
        assert d["host_folded"] == folded, d
    if kernel == 0:  # kernel 0: 2^24 / 256 partials, relaunched until <= 33 remain
        assert d["passes"] >= 2 and d["host_folded"] <= 33


@pytest.mark.parametrize("kernel,threads", [(6, 32), (6, 1), (0, 32), (4, 16), (5, 8), (3, 128), (7, 128)])
def test_reduction_threads_reference_range(tmp_path, kernel, threads):
    # the reference accepts any power of two up to 512 (reduction.cpp:272-291)
    r = reduction(tmp_path, "--method=SUM", "--type=int", f"--kernel={kernel}", f"--threads={threads}",
                  "--n=1000003", "--iterations=2")
    assert r.returncode == 0, r.stdout + r.stderr
    if kernel == 7:
        assert "using 256" in r.stderr


@pytest.mark.parametrize("type_,method", [("int64", "SUM"), ("double", "MAX"), ("int", "MIN")])
def test_reduction_huge_device_fill_closed_form_oracle(tmp_path, type_, method):
    # > 2^30 elements, device fill, no host copy: the closed-form iotamod result is the oracle
    js = tmp_path / "huge.json"
    r = reduction(tmp_path, f"--method={method}", f"--type={type_}", "--n=3000000000", "--fill=device",
                  "--pattern=iotamod", "--iterations=2", f"--json={js}")
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(js.read_text().splitlines()[-1])
    assert d["verified"] is True and d["oracle"] == "closed-form iotamod", d


def test_reduction_huge_device_fill_ladder_oracle(tmp_path):
    js = tmp_path / "huge.json"
    r = reduction(tmp_path, "--method=SUM", "--type=double", "--n=1200000000", "--fill=device", "--pattern=uniform",
                  "--iterations=2", f"--json={js}")
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(js.read_text().splitlines()[-1])
    assert d["verified"] is True and d["oracle"] == "ladder kernel 6", d


@pytest.mark.parametrize("method,type_,pattern", [("MAX", "double", "uniform"), ("MIN", "int", "smallint"),
                                                    ("MAX", "bf16", "uniform"), ("MIN", "int64", "fullrange")])
def test_reduction_app_arg(tmp_path, method, type_, pattern):
    out = tmp_path / "arg.json"
    r = reduction(tmp_path, f"--method={method}", f"--type={type_}", "--arg", "--n=30000017", f"--pattern={pattern}",
                  "--iterations=5", f"--json={out}")
    assert r.returncode == 0, r.stdout + r.stderr
    assert re.search(r"&&&& PASSED reduction", r.stderr)
    gi = re.search(r"GPU result = index (\d+)", r.stdout).group(1)
    ci = re.search(r"CPU result = index (\d+)", r.stdout).group(1)
    assert gi == ci
    import json
    j = json.loads(out.read_text())
    assert j["method"] == "ARG" + method and j["passed"] and j["verified"] and j["index"] == int(gi)
    assert len(j["iteration_ms"]) == 5 and j["min_ms"] <= j["median_ms"] <= j["max_ms"] and j["bytes_per_GB"] == 1e9
    assert j["arch"].startswith("gfx950") and j["cus"] > 0


def test_reduction_app_json_and_log(tmp_path):
    r = run([os.path.join(BIN, "reduction"), "--method=SUM", "--type=double", "--n=1M", "--iterations=4",
             "--json=out.jsonl", "--master-log=master.csv"], cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "reduction.txt").exists()           # shrSetLogFileName("reduction.txt")
    assert "Reduction, Throughput" in (tmp_path / "master.csv").read_text()
    d = json.loads((tmp_path / "out.jsonl").read_text().splitlines()[0])
    assert d["verified"] is True and len(d["iteration_ms"]) == 4 and d["bytes_per_GB"] == 1e9


def test_reduction_shmoo(tmp_path):
    r = run([os.path.join(BIN, "reduction"), "--method=SUM", "--type=float", "--shmoo", "--shmoo-max=65536",
             "--iterations=2", "--log=none"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr
    rows = [ln for ln in r.stdout.splitlines() if re.match(r"^\d+,", ln)]
    assert len(rows) == 17 * 9   # n = 1..65536 (powers of two) x kernels {0..6, 8, 7}


def test_reduce_xgmi_single_rank_scalar_and_graph(tmp_path):
    for extra in ([], ["--graph"]):
        r = run([os.path.join(BIN, "reduce_xgmi"), "--mode=scalar", "--n=6000007", "--dtypes=INT,LONG,FLOAT,DOUBLE",
                 "--retries=1", "--iters=3", *extra], timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        assert "verification PASSED" in r.stderr
        rows = [ln for ln in r.stdout.splitlines() if re.match(r"^(INT|LONG|FLOAT|DOUBLE) (MAX|MIN|SUM) 1 +[0-9.]+$", ln)]
        assert len(rows) == 12


def test_reduce_xgmi_single_rank_vector_mt19937(tmp_path):
    r = run([os.path.join(BIN, "reduce_xgmi"), "--mode=vector", "--ints=1M", "--doubles=1M", "--retries=2",
             "--mt19937", f"--json={tmp_path / 'x.jsonl'}"], timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.splitlines()[0] == "# DATATYPE OP NODES GB/sec"
    recs = [json.loads(x) for x in (tmp_path / "x.jsonl").read_text().splitlines()]
    assert len(recs) == 12 and all(x.get("verified", True) for x in recs)


def test_bandwidth_test_app():
    r = run([os.path.join(BIN, "bandwidth_test"), "--size=256M", "--iters=5"], timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Device to Device copy" in r.stdout and "Read stream" in r.stdout
    assert "peer_read kernel, local" in r.stdout


def test_bandwidth_peer_on_this_box(tmp_path):
    # One GPU on the test box: WAIVED; on a node with >= 2 GPUs: every ordered pair measured.
    js = tmp_path / "peer.json"
    r = run([os.path.join(BIN, "bandwidth_test"), "--peer", "--size=16M", "--iters=5", f"--json={js}"], timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    if "WAIVED" in r.stdout:
        assert "1 visible device(s)" in r.stdout
    else:
        d = json.loads(js.read_text().splitlines()[-1])
        assert d["node_ingress_gbps"] > 0 and d["all_pairs_peer_access"] is True


def test_cpp_consumer_example():
    """examples/cpp_consumer: a plain C++ program linked against libmireduce (closed-form sum)."""
    r = run([os.path.join(BIN, "cpp_consumer")], timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "expected" in r.stdout


# ---------------------------------------------------------------------------------------------
# Multi-rank paths rehearsed on the 1-GPU box (every rank on GPU 0).
from helpers import ROOT, bench_record, torchrun  # noqa: E402


@pytest.mark.parametrize("collective", ["direct", "direct-reduce"])
@pytest.mark.parametrize("nproc", [2, 3])
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_reduce_xgmi_direct_peer_reads(collective, nproc, graph):
    # One-kernel peer-read all-reduce through HIP IPC handles with device-side per-workgroup
    # barriers (csrc/kernels/direct.hip), also replayed from a captured hipGraph; all ranks share
    # one GPU here, so this checks the protocol, chunking and kernels — not xGMI speed.
    r = torchrun(nproc, ["--no-python", os.path.join(BIN, "reduce_xgmi"), "--mode=vector",
                         f"--collective={collective}", "--ints=1000003", "--doubles=999999", "--longs=77777",
                         "--floats=123457", "--dtypes=INT,LONG,FLOAT,DOUBLE", "--retries=1", "--iters=3",
                         "--direct-grid=64", "--timeout=20"] + (["--graph"] if graph else []), timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "verification PASSED" in r.stderr
    rows = [ln for ln in r.stdout.splitlines() if re.match(rf"^(INT|LONG|FLOAT|DOUBLE) (MAX|MIN|SUM) {nproc} ", ln)]
    assert len(rows) == 12


@pytest.mark.parametrize("nproc", [1, 3])
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_reduce_xgmi_scalar_fused(nproc, graph):
    # scalar mode with the fused in-kernel cross-rank finish (no RCCL): every rank's result is
    # checked against the host fold of all ranks' local results (+ the ladder oracle per rank)
    r = torchrun(nproc, ["--no-python", os.path.join(BIN, "reduce_xgmi"), "--mode=scalar", "--collective=fused",
                         "--doubles=30000001", "--ints=20000003", "--dtypes=INT,DOUBLE", "--retries=2", "--iters=5",
                         "--timeout=20"] + (["--graph"] if graph else []), timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "verification PASSED" in r.stderr
    rows = [ln for ln in r.stdout.splitlines() if re.match(rf"^(INT|DOUBLE) (MAX|MIN|SUM) {nproc} ", ln)]
    assert len(rows) == 12


@pytest.mark.parametrize("count", ["1", "2", "3", "5", "17", "65", "4099"])
def test_reduce_xgmi_direct_tiny_counts(count):
    # chunks shorter than a vector, empty chunks, sub-vector tails in the last chunk
    r = torchrun(3, ["--no-python", os.path.join(BIN, "reduce_xgmi"), "--mode=vector", "--collective=direct",
                     f"--ints={count}", f"--doubles={count}", "--dtypes=INT,DOUBLE", "--retries=1", "--iters=2",
                     "--direct-grid=8",
                     "--timeout=20"], timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "verification PASSED" in r.stderr


@pytest.mark.parametrize("args", [["--kernel=0", "--threads=64"], ["--kernel=3", "--n=1e8"]])
def test_reduction_cpufinal_more_partials_than_the_pinned_default(tmp_path, args):
    # kernels 0..5 have no --maxblocks cap, so --cpufinal can leave more partials
    # than the default 64 Ki-entry pinned landing zone; it must grow, not overflow the host heap.
    js = tmp_path / "cf.json"
    r = reduction(tmp_path, "--method=SUM", "--type=double", "--cpufinal", "--iterations=2", f"--json={js}", *args)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(js.read_text().splitlines()[-1])
    assert d["verified"] is True and d["passes"] == 1 and d["host_folded"] > 65536, d
    assert d["fanin_error"] == 0 and d["native_source_hash"] != "unknown"


def test_bench_rehearsal_two_ranks_one_gpu(tmp_path):
    env_before = os.environ.get("MIREDUCE_FORCE_DEVICE")
    os.environ["MIREDUCE_FORCE_DEVICE"] = "0"
    try:
        r = torchrun(2, [os.path.join(ROOT, "bench.py"), "--no-vector-extras", "--gpus", "2", "--backend", "gloo", "--steps", "5",
                         "--warmup", "1", "--elements", "20000003"], cwd=tmp_path, timeout=600)
    finally:
        if env_before is None:
            os.environ.pop("MIREDUCE_FORCE_DEVICE")
        else:
            os.environ["MIREDUCE_FORCE_DEVICE"] = env_before
    assert r.returncode == 0, r.stderr[-3000:]
    d = bench_record(r.stdout)
    assert d["verified"] is True and d["n_gpus"] == 2 and d["config"]["backend"] == "gloo"


def test_bench_graph_capture_failure_falls_back_on_all_ranks(tmp_path, monkeypatch):
    # gloo collectives on GPU tensors cannot be captured: every rank must agree on the failure
    # and fall back to eager issue (never some ranks replaying graphs and others not).
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    # (the extras are not this test's subject: without them it takes ~5 s instead of ~30 s)
    r = torchrun(2, [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "6",
                     "--warmup", "2", "--elements", "20000003", "--launch", "graph", "--collective", "rccl",
                     "--no-vector-extras", "--no-candidates"],
                 cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = bench_record(r.stdout)
    assert d["verified"] is True
    assert d["config"]["launch"].startswith("eager (graph capture failed"), d["config"]["launch"]


@pytest.mark.parametrize("launch", ["graph", "eager"])
def test_bench_launch_modes(tmp_path, launch):
    # Default launch on a GPU is graph replay of the timed steps; both modes verify every slot.
    r = run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-vector-extras", "--steps", "37", "--warmup", "3", "--elements",
             "50000017", "--launch", launch, "--graph-chunk", "16"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = bench_record(r.stdout)
    assert d["verified"] is True and d["steps"] == 37
    assert d["config"]["launch"].startswith(launch)
    if launch == "graph":
        assert d["config"]["launch"] == "graph (chunk 16, 2 replays + 1 of 5)"


@pytest.mark.parametrize("collective", ["allreduce", "host"])
def test_reduce_xgmi_single_process(collective):
    # simpleMultiGPU / P9: one process drives every visible GPU (one on this box).
    r = run([os.path.join(BIN, "reduce_xgmi"), "--single-process", "--mode=scalar", f"--collective={collective}",
             "--n=30000001", "--dtypes=INT,DOUBLE", "--retries=2", "--iters=3"], timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "verification PASSED" in r.stderr
    rows = [ln for ln in r.stdout.splitlines() if re.match(r"^(INT|DOUBLE) (MAX|MIN|SUM) \d+ +[0-9.]+$", ln)]
    assert len(rows) == 12 and r.stdout.splitlines()[0] == "# DATATYPE OP NODES GB/sec"


# ---------------------------------------------------------------- failure detection

def test_reduce_xgmi_scalar_corrupt_detected():
    r = run([os.path.join(BIN, "reduce_xgmi"), "--mode=scalar", "--n=10000019", "--dtypes=DOUBLE", "--ops=SUM",
             "--retries=2", "--iters=3", "--inject-fault=corrupt@0:0"], timeout=300)
    assert r.returncode != 0
    assert "[fault] rank 0 corrupts" in r.stderr and "verification FAILED" in r.stderr


@pytest.mark.parametrize("collective", ["direct", "direct-reduce"])
def test_reduce_xgmi_direct_corrupt_detected(collective):
    r = torchrun(2, ["--no-python", os.path.join(BIN, "reduce_xgmi"), "--mode=vector", f"--collective={collective}",
                     "--ints=1000003", "--doubles=999999", "--retries=1", "--iters=2", "--inject-fault=corrupt@1:4"],
                 timeout=300)
    assert r.returncode != 0
    assert "verification FAILED" in r.stderr


@pytest.mark.parametrize("mode,collective", [("scalar", "fused"), ("vector", "direct"), ("vector", "direct-reduce")])
def test_reduce_xgmi_peer_preflight_declines_on_every_rank(mode, collective):
    # the IPC-mapped paths agree on peer access BEFORE any hipIpcOpenMemHandle;
    # rank 1 reporting "no peer access" (injected) makes every rank exit non-zero with the agreed
    # message — no GPU fault, no hang, no collective started (no header row printed).
    r = torchrun(2, ["--no-python", os.path.join(BIN, "reduce_xgmi"), f"--mode={mode}", f"--collective={collective}",
                     "--ints=100003", "--doubles=100003", "--retries=1", "--iters=1", "--timeout=5",
                     "--inject-fault=nopeer@1"], timeout=240)
    assert r.returncode != 0
    for k in range(2):
        assert f"[rank {k}] error: --collective={collective} needs peer access" in r.stderr, r.stderr[-3000:]
    assert "rank 1: device" in r.stderr and "injected" in r.stderr
    assert "# DATATYPE" not in r.stdout


# "hang" only: a peer that EXITS frees its registered buffers, and the survivor's kernel would
# then store its barrier flag into unmapped peer memory — a GPU fault by construction, not a test.
@pytest.mark.parametrize("kind", ["hang"])
def test_reduce_xgmi_direct_lost_peer_fails_fast(kind, monkeypatch):
    # A crashed or hung peer: the survivor's kernel waits at its device-side barrier for at most
    # --timeout, flags the error and returns (nothing hangs on the device); the survivor reports it
    # and exits non-zero; torchrun then tears down the hung rank.
    import time
    monkeypatch.setenv("MIREDUCE_BOOTSTRAP_TIMEOUT", "5")
    t0 = time.time()
    r = torchrun(2, ["--no-python", os.path.join(BIN, "reduce_xgmi"), "--mode=vector", "--collective=direct",
                     "--ints=1000003", "--doubles=999999", "--retries=2", "--iters=2", "--timeout=2",
                     f"--inject-fault={kind}@1:2"], timeout=240)
    assert r.returncode != 0
    assert f"[fault] rank 1 {'exits' if kind == 'exit' else 'hangs'}" in r.stderr
    assert ("[rank 0] error: direct: a peer's barrier flag never arrived" in r.stderr
            or "[rank 0] error: bootstrap" in r.stderr), r.stderr[-2000:]
    assert time.time() - t0 < 180


def test_reduction_cold_cache_mode(tmp_path):
    # --cold evicts the array from L2 / Infinity Cache before each timed iteration (per-iter timing).
    js = tmp_path / "cold.jsonl"
    r = reduction(tmp_path, "--method=SUM", "--type=double", "--n=16777216", "--iterations=5", "--cold",
                  f"--json={js}")
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(js.read_text().splitlines()[-1])
    assert d["cold"] is True and d["timing"] == "per-iter" and d["verified"] is True


@pytest.mark.parametrize("launch", ["graph", "eager"])
def test_bench_maxloc_config(tmp_path, launch):
    r = run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "xgmi_1b_double_maxloc", "--steps", "20",
             "--warmup", "3", "--elements", "50000017", "--launch", launch], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    d = bench_record(r.stdout)
    assert d["verified"] is True and d["config"]["op"] == "MAXLOC"
    assert d["config"]["launch"].startswith(launch)
    assert d["config"]["kernel_plan"]["splits"] > 1


def test_sweep_node_preset_on_one_gpu(tmp_path):
    """tools/sweep.py --preset node end to end at P=1: fabric probe (WAIVED on one GPU), reduce.c
    vector mode over RCCL and direct, scalar mode over RCCL and the fused finish, the bench; every
    point's rc file, the getAvgs results and the bench JSONL."""
    out = tmp_path / "node"
    r = run([sys.executable, os.path.join(ROOT, "tools", "sweep.py"), "--preset", "node", "--ranks", "1",
             "--out", str(out), "--timeout", "300", "--", "--ints=1000003", "--doubles=1000003", "--retries=1"],
            timeout=1200)
    if r.returncode != 0:  # name the failing point's own stderr, not only the sweep's summary
        errs = sorted(out.glob("*/stdout-*.rc"))
        bad = [p for p in errs if p.read_text().strip() != "0"]
        detail = "".join(f"\n--- {p.name}\n" + p.with_suffix(".err").read_text()[-3000:] for p in bad)
        raise AssertionError(r.stdout[-2000:] + r.stderr[-2000:] + detail)
    for name in ("vector-reduce", "vector-allreduce", "vector-direct-reduce", "vector-direct", "scalar-allreduce",
                 "scalar-fused", "bench"):
        assert (out / name / f"stdout-{name}-P1.rc").read_text().strip() == "0", name
    assert (out / "fabric" / "stdout-fabric-PNone.rc").read_text().strip() == "0"
    assert "WAIVED" in (out / "fabric" / "stdout-fabric-PNone.txt").read_text()
    assert (out / "scalar-fused" / "results" / "DOUBLE_SUM.txt").read_text().startswith("\nDOUBLE SUM 1 ")
    assert "scaling efficiency" in r.stdout and (out / "bench" / "bench.jsonl").exists()
