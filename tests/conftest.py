import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _own_bench_sidecar_dir(tmp_path, monkeypatch):
    """bench.py's default sidecar (bench_extras_n<N>.json) goes to this test's own directory:
    concurrent tests (pytest -n) must not overwrite each other's, nor the repo's gpurun_out/."""
    monkeypatch.setenv("MIREDUCE_EXTRAS_DIR", str(tmp_path))
