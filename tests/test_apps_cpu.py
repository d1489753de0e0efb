"""The native apps' CPU-visible behaviour: CLI grammar, QA protocol, MPI app (BASELINE config 1)
on 2 CPU ranks with byte-compatible output, getAvgs round trip."""
import os
import re
import shutil

import pytest

from cuda_mpi_reductions_amd.utils import formats, getavgs
from helpers import BIN, MPIRUN, ensure_built, run

pytestmark = pytest.mark.filterwarnings("ignore")


@pytest.fixture(scope="module", autouse=True)
def built():
    ensure_built()


def test_reduction_requires_method(tmp_path):
    r = run([os.path.join(BIN, "reduction"), "--type=double"], cwd=tmp_path)
    assert r.returncode == 1
    assert "MISSING --method FLAG." in r.stderr


def test_reduction_method_is_case_sensitive(tmp_path):
    r = run([os.path.join(BIN, "reduction"), "--method=sum"], cwd=tmp_path)
    assert r.returncode == 1 and "No --method specified!" in r.stderr


def test_reduction_rejects_non_dash_token(tmp_path):
    r = run([os.path.join(BIN, "reduction"), "--method=SUM", "foo"], cwd=tmp_path)
    assert r.returncode == 1 and "Invalid command line argument" in r.stderr


def test_reduction_waives_without_gpu_and_qa_lines(tmp_path):
    r = run([os.path.join(BIN, "reduction"), "--method=SUM", "--qatest"], cwd=tmp_path,
            env={"HIP_VISIBLE_DEVICES": "-1"})
    assert r.returncode == 0
    assert "&&&& RUNNING reduction --method=SUM --qatest" in r.stderr
    assert "&&&& WAIVED reduction --method=SUM --qatest" in r.stderr


def test_bandwidth_peer_waives_below_two_devices():
    # bandwidth_test --peer (xGMI roofline, simpleP2P parity) on a host with fewer than two visible
    # devices: a clear WAIVED line, QA protocol, exit 0 (HIP_VISIBLE_DEVICES=-1 also hides any GPU).
    r = run([os.path.join(BIN, "bandwidth_test"), "--peer", "--qatest"], env={"HIP_VISIBLE_DEVICES": "-1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert re.search(r"Peer-to-peer \(xGMI\) bandwidth: \d visible device\(s\), needs >= 2 -> WAIVED", r.stdout)
    assert "&&&& WAIVED bandwidth_test --peer --qatest" in r.stderr


def test_reduction_help(tmp_path):
    r = run([os.path.join(BIN, "reduction"), "--help"], cwd=tmp_path)
    assert r.returncode == 0 and "--cpufinal" in r.stdout and "--shmoo" in r.stdout


def test_reduce_xgmi_help():
    r = run([os.path.join(BIN, "reduce_xgmi"), "--help"])
    assert r.returncode == 0 and "--mode=vector|scalar" in r.stdout


needs_mpi = pytest.mark.skipif(not os.path.exists(MPIRUN), reason="MPICH not available")


@needs_mpi
def test_reduce_mpi_config1_two_cpu_ranks(tmp_path):
    # BASELINE.json config 1: 1M int32 SUM via MPI_Reduce on 2 CPU ranks.
    out = tmp_path / "run.json"
    r = run([MPIRUN, "-np", "2", os.path.join(BIN, "reduce_mpi"), "--ints=1M", "--dtypes=INT", "--ops=SUM",
             "--retries=3", "--verify", f"--json={out}"], timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "# DATATYPE OP NODES GB/sec"
    assert len(lines) == 4
    for ln in lines[1:]:
        assert re.fullmatch(r"INT SUM 2 +[0-9]+\.[0-9]{3}", ln), ln
    assert "verification PASSED" in r.stderr
    recs = out.read_text().splitlines()
    assert len(recs) == 3 and '"bytes_per_GB": 1073741824' in recs[0]


@needs_mpi
def test_reduce_mpi_default_order_and_getavgs(tmp_path):
    # reduce.c order per retry: INT MAX, INT MIN, INT SUM, DOUBLE MAX, DOUBLE MIN, DOUBLE SUM.
    r = run([MPIRUN, "-np", "2", os.path.join(BIN, "reduce_mpi"), "--ints=64k", "--doubles=32k", "--retries=2",
             "--verify", "--collective=allreduce"], timeout=300)
    assert r.returncode == 0, r.stderr
    rows = list(formats.parse_gnuplot(r.stdout.splitlines()))
    assert [(x.dtype, x.op) for x in rows[:6]] == [("INT", "MAX"), ("INT", "MIN"), ("INT", "SUM"),
                                                  ("DOUBLE", "MAX"), ("DOUBLE", "MIN"), ("DOUBLE", "SUM")]
    assert all(x.nodes == 2 and x.value > 0 for x in rows) and len(rows) == 12
    collected = tmp_path / "collected.txt"
    collected.write_text(r.stdout)
    getavgs.write_results(str(collected), str(tmp_path / "results"))
    res = (tmp_path / "results" / "INT_SUM.txt").read_text().splitlines()
    assert res[0] == "" and res[1].startswith("INT SUM 2 ")


@needs_mpi
def test_reduce_mpi_all_dtypes_verify():
    r = run([MPIRUN, "-np", "3", os.path.join(BIN, "reduce_mpi"), "--ints=30001", "--doubles=30001",
             "--longs=30001", "--floats=30001", "--dtypes=INT,LONG,FLOAT,DOUBLE", "--retries=1", "--verify",
             "--timing=root"], timeout=300)
    assert r.returncode == 0, r.stderr
    rows = list(formats.parse_gnuplot(r.stdout.splitlines()))
    assert {x.dtype for x in rows} == {"INT", "LONG", "FLOAT", "DOUBLE"} and len(rows) == 12
    assert "verification PASSED" in r.stderr


@needs_mpi
def test_reduce_mpi_rejects_bad_flags():
    r = run([MPIRUN, "-np", "1", os.path.join(BIN, "reduce_mpi"), "--dtypes=CHAR"], timeout=120)
    assert r.returncode != 0 and "unknown dtype" in r.stderr


def test_reduce_xgmi_bootstrap_env_parsing():
    # Without a GPU the app stops at device discovery, after parsing flags.
    r = run([os.path.join(BIN, "reduce_xgmi"), "--mode=scalar", "--n=1000"], env={"HIP_VISIBLE_DEVICES": "-1"})
    assert r.returncode == 1 and "no HIP device" in r.stderr
    r = run([os.path.join(BIN, "reduce_xgmi"), "--mode=bogus"])
    assert r.returncode == 1 and "--mode must be" in r.stderr


def test_reduction_arg_needs_min_or_max(tmp_path):
    r = run([os.path.join(BIN, "reduction"), "--method=SUM", "--arg"], cwd=tmp_path)
    assert r.returncode != 0 and "--arg needs --method=MIN or MAX" in r.stderr
    r = run([os.path.join(BIN, "reduction"), "--method=MAX", "--arg", "--kernel=3"], cwd=tmp_path)
    assert r.returncode != 0 and "arg-reduction kernel only" in r.stderr
