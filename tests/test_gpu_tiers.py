"""The GPU test tiers (tests/conftest.py): the default `-m gpu` set is a subset in
which every value of every parameter of each subsampled sweep still appears, and the whole-test moves
name real tests. CPU only (collection, no GPU)."""
import json
import os
import subprocess
import sys

from helpers import ROOT

PLUGIN = '''
import json, os
import conftest as cf
def pytest_collection_finish(session):
    cf._INDICES.update(cf._param_indices(session.items))  # (this module object may not be pytest's conftest)
    rows = []
    for it in session.items:
        if "gpu" not in it.keywords:
            continue
        cs = getattr(it, "callspec", None)
        rows.append({"name": getattr(it, "originalname", it.name), "file": it.nodeid.split("::")[0],
                     "params": {k: repr(v) for k, v in cs.params.items()} if cs else {}, "tier": cf._tier(it)})
    with open(os.environ["TIERS_OUT"], "w") as f:
        json.dump(rows, f)
'''


def _collect(tmp_path):
    (tmp_path / "tiers_plugin.py").write_text(PLUGIN)
    out = tmp_path / "tiers.json"
    env = dict(os.environ, TIERS_OUT=str(out), PYTHONPATH=f"{tmp_path}:{os.path.join(ROOT, 'tests')}")
    r = subprocess.run([sys.executable, "-m", "pytest", "tests", "--collect-only", "-q", "-p", "tiers_plugin"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(out.read_text())


def test_default_tier_keeps_every_parameter_value(tmp_path):
    import conftest as cf
    rows = _collect(tmp_path)
    names = {r["name"] for r in rows}
    assert set(cf.GPU_FULL_ONLY) <= names and set(cf.GPU_FULL_SUBSAMPLE) <= names
    for fn in cf.GPU_FULL_SUBSAMPLE:
        cases = [r for r in rows if r["name"] == fn]
        kept = [r for r in cases if r["tier"] is None]
        assert 0 < len(kept) < len(cases), fn
        cols = {p: tuple(r["params"][p] for r in cases) for p in cases[0]["params"]}
        if len(set(cols.values())) == 1 or any(len(set(c)) == len(cases) for c in cols.values()):
            # one parameter group (a list of cases): a k-fold subset of it by construction
            assert len(kept) == -(-len(cases) // cf.GPU_FULL_SUBSAMPLE[fn]), fn
            continue
        for p in cases[0]["params"]:  # several groups: every value of every parameter is still run
            assert {r["params"][p] for r in kept} == {r["params"][p] for r in cases}, (fn, p)
    full = [r for r in rows if r["tier"] == "full"]
    assert {r["name"] for r in full} >= set(cf.GPU_FULL_ONLY)
    assert {c.split("[")[0] for c in cf.GPU_FULL_CASES} <= names
    # the protocol tests stay in the default tier
    for fn in ("test_bench_eight_ranks_fused_on_one_gpu", "test_reduce_xgmi_direct_eight_ranks_on_one_gpu",
               "test_segmented_launches_match_the_reference", "test_fused_poison_reaches_every_rank",
               "test_every_variant", "test_xcd_weighted_split"):
        assert any(r["name"] == fn and r["tier"] is None for r in rows), fn
