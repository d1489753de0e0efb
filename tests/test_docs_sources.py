"""Every record the report documents cite exists in the repo (no number without a
traceable source). Checks the backticked paths of docs/WRITEUP.md, README.md and BASELINE.md —
`profiles/...`, `BENCH_rNN.json` / `GPUTEST_rNN.json` / `SCALE_rNN.json`, `tools/...`, `tests/...`,
`docs/...` — and that the WRITEUP's figures and its scaling markers are in place."""
import os
import re

from helpers import ROOT

DOCS = ("docs/WRITEUP.md", "README.md", "BASELINE.md")
PREFIXES = ("profiles/", "tools/", "tests/", "docs/", "BENCH_r", "GPUTEST_r", "SCALE_r")


def _cited(text: str) -> set:
    out = set()
    for tok in re.findall(r"`([^`\s]+)`", text):
        tok = tok.split(":")[0].rstrip(",;")
        if tok.startswith(PREFIXES):
            out.add(tok)
    return out


def _exists(path: str) -> bool:
    m = re.match(r"^(BENCH|GPUTEST|SCALE)_r(\d\d)-(\d\d)\.json$", path)
    if m:  # a range of driver records: BENCH_r01-04.json
        return all(os.path.exists(os.path.join(ROOT, f"{m.group(1)}_r{i:02d}.json"))
                   for i in range(int(m.group(2)), int(m.group(3)) + 1))
    if "*" in path or "<" in path or "{" in path:
        return True  # a pattern, not a file
    return os.path.exists(os.path.join(ROOT, path.rstrip("/")))


def test_cited_records_exist():
    missing = []
    for doc in DOCS:
        text = open(os.path.join(ROOT, doc)).read()
        for p in sorted(_cited(text)):
            if not _exists(p):
                missing.append(f"{doc}: {p}")
    assert not missing, missing


def test_writeup_figures_and_scaling_section():
    text = open(os.path.join(ROOT, "docs", "WRITEUP.md")).read()
    for fig in ("figures/int.png", "figures/double.png"):
        assert f"]({fig})" in text and os.path.getsize(os.path.join(ROOT, "docs", fig)) > 10000
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scaling
    assert text.count(scaling.WRITEUP_BEGIN) == 1 and text.count(scaling.WRITEUP_END) == 1
    assert len(text.splitlines()) <= 170  # a report, not a lab notebook (docs/CHANGELOG.md)
