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
