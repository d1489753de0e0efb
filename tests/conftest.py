import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "gpu_full: the full GPU tier (MIREDUCE_GPU_FULL=1 -m gpu): the long "
                                       "orchestration rehearsals and every case of the combinatorial sweeps")
    config.addinivalue_line("markers", "slow: long-running test")


# ---- GPU tiers. The default `-m gpu` set stays within ~300 s on one MI355X and
# still covers every shipped plan, every op x dtype x acc combo, the size edges, segmented launches and
# the fused / direct / xrank protocols; MIREDUCE_GPU_FULL=1 runs everything (round 5: 3301 tests,
# 473 s). Durations: gpurun_out/r6_gpu_all.log -> profiles/r6_tiers/.
#
# Whole tests in the full tier only, with what keeps their subject covered by default:
GPU_FULL_ONLY = {
    # 53 s: the driver's default command at N=8 on one GPU (gloo). Default tier: the 8-rank fused
    # finish (test_bench_eight_ranks_fused_on_one_gpu), the W=8 direct collective
    # (test_reduce_xgmi_direct_eight_ranks_on_one_gpu), the reduce.c extras at 1 rank
    # (test_bench_vector_extras_in_headline) and the 2-rank auto path (test_bench_rehearsal_two_ranks_one_gpu)
    "test_bench_eight_ranks_auto_on_one_gpu",
    # 32 s: tools/sweep.py's node preset (orchestration; its resume logic is CPU-tested, tests/test_tools_cli.py)
    "test_sweep_node_preset_on_one_gpu",
    # 29 s: a 25 s extras deadline (the extras watchdog is CPU-tested at 2 and 4 ranks,
    # tests/test_fault_injection.py, tests/test_bench_policy.py)
    "test_bench_extras_hang_in_rccl_candidate_keeps_the_headline",
    # 4 s: examples/06 at world 1 (the default tier runs the same example at three ranks,
    # test_example_xgmi_collectives_three_ranks_one_gpu, and the world-1 fused finish in test_xrank_gpu.py)
    "test_example_xgmi_collectives_single",
}
# Single cases in the full tier only:
GPU_FULL_CASES = {
    # 10 s: the hang of a rank in plan tuning, GPU form (the bounded agreement that names it is the same
    # store exchange as on CPU ranks, tested there at 4 ranks for every stage; the GPU tier keeps the
    # raise cases, which run the GPU code of both stages)
    "test_bench_optional_stage_failure_two_ranks_one_gpu[hang@1/tune]",
}
# Parametrized sweeps: the default tier keeps the cases whose parameter indices sum to 0 mod k — a
# Latin-style subset in which every value of every parameter still appears (every combo, every size,
# every window plan, ...), k-fold fewer cases.
GPU_FULL_SUBSAMPLE = {
    "test_all_combos_sizes": 4, "test_window_variants": 3, "test_ladder_kernels": 3, "test_cols": 3,
    "test_rows": 3, "test_gpu_half_sizes": 3, "test_device_whole": 3, "test_device_rows": 3,
    "test_gpu_full_reduction": 2, "test_fused_world1_matches_torch": 2,
    # subprocess-heavy app sweeps (each case starts ranks)
    "test_reduce_xgmi_direct_peer_reads": 2, "test_reduce_xgmi_direct_tiny_counts": 2,
    "test_reduce_xgmi_scalar_fused": 2, "test_reduction_multipass_cputhresh": 2,
    "test_reduction_app_methods_types": 2,
    "test_bench_ranks_hold_different_plans_and_verify": 3, "test_python_cli_gpu": 2,
    # multi-rank rehearsals by rank count: the default tier keeps the 2-rank case (the 8-rank fused and
    # direct tests cover the wide worlds), and one of maxloc's launch modes
    "test_bench_fused_ranks_share_one_gpu": 2, "test_bench_vector_direct_ranks_share_one_gpu": 2,
    "test_bench_maxloc_config": 2, "test_reduce_xgmi_peer_preflight_declines_on_every_rank": 2,
}


def _name(item) -> str:
    return item.originalname if hasattr(item, "originalname") else item.name


def _param_indices(items) -> dict:
    """{item nodeid: [index of each parameter group's value]} for the subsampled sweeps: a value's
    index is its rank among the distinct values of that argument over the function's cases, and
    arguments that always vary together (one parametrize over "dt,op,acc") count as one group."""
    by_fn = {}
    for it in items:
        if _name(it) in GPU_FULL_SUBSAMPLE and getattr(it, "callspec", None) is not None:
            by_fn.setdefault((str(it.path), _name(it)), []).append(it)
    out = {}
    for its in by_fn.values():
        names = list(its[0].callspec.params)
        cols = {}
        for a in names:
            order = {}
            cols[a] = tuple(order.setdefault(repr(it.callspec.params[a]), len(order)) for it in its)
        groups = list(dict.fromkeys(cols.values()))  # co-varying arguments collapse into one column
        key = [g for g in groups if len(set(g)) == len(its)]
        if key:  # one argument tells every case apart: the sweep is a list of cases
            groups = key[:1]
        for i, it in enumerate(its):
            out[it.nodeid] = [g[i] for g in groups]
    return out


_INDICES: dict = {}


def _tier(item) -> "str | None":
    """'full' if the item belongs to the full GPU tier only."""
    name = _name(item)
    if name in GPU_FULL_ONLY or item.name in GPU_FULL_CASES:
        return "full"
    k = GPU_FULL_SUBSAMPLE.get(name)
    idx = _INDICES.get(item.nodeid)
    if k and idx is not None and sum(idx) % k:
        return "full"
    return None


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    _INDICES.update(_param_indices(items))
    full = os.environ.get("MIREDUCE_GPU_FULL") == "1"
    tier_skip = pytest.mark.skip(reason="gpu_full tier (MIREDUCE_GPU_FULL=1 runs it; tests/conftest.py)")
    for item in items:
        if "gpu" in item.keywords and _tier(item) == "full":
            item.add_marker(pytest.mark.gpu_full)
            if has_gpu and not full:
                item.add_marker(tier_skip)
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
