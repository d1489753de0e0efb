"""Every argparse-driven tool under tools/ keeps a working command line on a CPU host: `--help`
must import the tool (and whatever it imports at module level) and exit 0 without touching a GPU.
The tools' measurements themselves run on the GPU box (profiles/r*_scripts/)."""
import glob
import os
import sys

import pytest

from helpers import ROOT, run

TOOLS = sorted(p for p in glob.glob(os.path.join(ROOT, "tools", "*.py")) if "argparse" in open(p).read())


@pytest.mark.parametrize("path", TOOLS, ids=[os.path.basename(p) for p in TOOLS])
def test_tool_help(path):
    r = run([sys.executable, path, "--help"], timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "usage" in r.stdout.lower()
