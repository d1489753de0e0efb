"""Examples and the Python CLI front-end."""
import os
import re
import sys

import pytest

from helpers import ROOT, run, torchrun


def test_example_distributed_sum_cpu(tmp_path):
    r = torchrun(2, [os.path.join(ROOT, "examples", "02_distributed_sum.py"), "--cpu"], cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert re.search(r"2 ranks: sum = [0-9.]+  verified=True", r.stdout)


def test_example_vector_reduce_cpu(tmp_path):
    r = torchrun(2, [os.path.join(ROOT, "examples", "03_vector_reduce.py")], cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("verified=True") == 3


def test_python_cli_grammar_errors(tmp_path):
    r = run([sys.executable, "-m", "cuda_mpi_reductions_amd", "--type=double"], cwd=ROOT)
    assert r.returncode == 1 and "MISSING --method FLAG." in r.stderr
    r = run([sys.executable, "-m", "cuda_mpi_reductions_amd", "--method=sum"], cwd=ROOT)
    assert r.returncode == 1 and "No --method specified!" in r.stderr
    r = run([sys.executable, "-m", "cuda_mpi_reductions_amd", "--method=SUM", "oops"], cwd=ROOT)
    assert r.returncode == 1 and "Invalid command line argument" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("method,type_", [("SUM", "double"), ("MIN", "int64"), ("MAX", "float"), ("SUM", "int")])
def test_python_cli_gpu(method, type_):
    r = run([sys.executable, "-m", "cuda_mpi_reductions_amd", f"--method={method}", f"--type={type_}",
             "--n=4000037", "--iterations=5", "--qatest"], cwd=ROOT, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "&&&& PASSED" in r.stderr
    assert re.search(r"Reduction, Throughput = [0-9.]+ GB/s, Time = [0-9.]+ s, Size = 4000037 Elements", r.stdout)


@pytest.mark.gpu
@pytest.mark.parametrize("method,type_", [("MAX", "double"), ("MIN", "bf16")])
def test_python_cli_gpu_arg(method, type_):
    r = run([sys.executable, "-m", "cuda_mpi_reductions_amd", f"--method={method}", f"--type={type_}", "--arg",
             "--n=4000037", "--iterations=5", "--pattern=uniform", "--qatest"], cwd=ROOT, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "&&&& PASSED" in r.stderr and "GPU result = index" in r.stdout


@pytest.mark.gpu
def test_example_single_gpu():
    r = run([sys.executable, os.path.join(ROOT, "examples", "01_single_gpu.py")], cwd=ROOT, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "GB/s" in r.stdout


@pytest.mark.gpu
def test_example_norms_dims_many():
    r = run([sys.executable, os.path.join(ROOT, "examples", "04_norms_dims_many.py")], timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "per-tensor sum of squares" in r.stdout and "total grad-norm-style L2" in r.stdout


def test_example_argmax_maxloc_cpu(tmp_path):
    r = torchrun(2, [os.path.join(ROOT, "examples", "05_argmax_maxloc.py"), "--cpu"], cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("match torch: True") == 2
    assert r.stdout.count("arg_reduce agrees: True") == 2


@pytest.mark.gpu
def test_example_argmax_maxloc():
    r = run([sys.executable, os.path.join(ROOT, "examples", "05_argmax_maxloc.py")], cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "match torch: True" in r.stdout and "arg_reduce agrees: True" in r.stdout


@pytest.mark.gpu
def test_example_xgmi_collectives_single():
    r = run([sys.executable, os.path.join(ROOT, "examples", "06_xgmi_collectives.py")], cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"\[rank 0\] fused global sum ([0-9.]+) \(torch: ([0-9.]+), epoch 10, channel ok\)", r.stdout)
    assert m and abs(float(m.group(1)) - float(m.group(2))) <= 1e-9 * float(m.group(2)), r.stdout
    assert "matches the gathered sum; no timeouts" in r.stdout


@pytest.mark.gpu
def test_example_xgmi_collectives_three_ranks_one_gpu(tmp_path):
    """Three ranks sharing the one GPU of the box (gloo for the host-side agreement)."""
    r = torchrun(3, [os.path.join(ROOT, "examples", "06_xgmi_collectives.py"), "--backend", "gloo"],
                 cwd=tmp_path, timeout=300, env={"MIREDUCE_FORCE_DEVICE": "0"})
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    sums = re.findall(r"\[rank (\d)\] fused global sum ([0-9.]+) \(torch: ([0-9.]+), epoch 10, channel ok\)", r.stdout)
    assert len(sums) == 3, r.stdout
    assert len({s[1] for s in sums}) == 1  # bit-identical on every rank
    assert abs(float(sums[0][1]) - float(sums[0][2])) <= 1e-9 * float(sums[0][2])
    assert "matches the gathered sum; no timeouts" in r.stdout
