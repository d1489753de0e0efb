"""Fused cross-rank finish (csrc/include/mireduce/xrank.hpp) and the exact N-GPU bench step run on
one GPU: the cross-rank combine is issued (and graph-captured) even at world 1, serial and
pipelined; several ranks share the one GPU of the box through HIP IPC for the multi-rank protocol
(not xGMI speed)."""
import json
import os
import sys
import time

import pytest
import torch

from helpers import ROOT, bench_record, run, torchrun

pytestmark = pytest.mark.gpu

BENCH = os.path.join(ROOT, "bench.py")


def _json(r):
    return bench_record(r.stdout)


# ---------------------------------------------------------------- kernel numerics at world 1

@pytest.mark.parametrize("dt,op", [(torch.float64, "sum"), (torch.float64, "min"), (torch.int64, "min"),
                                   (torch.int64, "sum"), (torch.int32, "sum"), (torch.int32, "max"),
                                   (torch.float32, "sum"), (torch.float32, "max"), (torch.bfloat16, "sum"),
                                   (torch.float64, "sumsq"), (torch.float32, "amax")])
@pytest.mark.parametrize("n", [1, 1000, 3_000_017])
def test_fused_world1_matches_torch(dt, op, n):
    from cuda_mpi_reductions_amd.ops import Reducer, default_acc_dtype
    from cuda_mpi_reductions_amd.parallel.xrank import open_channel
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(n)
    if dt.is_floating_point:
        x = (torch.rand(n, generator=g, dtype=torch.float64) * 2 - 1).to(dt).to(dev)
    else:
        x = torch.randint(-1000, 1000, (n,), generator=g).to(dt).to(dev)
    acc = default_acc_dtype(dt, op)
    out = torch.empty(1, dtype=acc, device=dev)
    ch = open_channel(dev)
    b = Reducer(dev).bind(x, op, acc, out=out, xrank=ch)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):  # epochs 1..3: both mailbox parities
        out.fill_(0)
        b.launch(s)
    torch.cuda.synchronize()
    xd = x.double()
    ref = {"sum": lambda: xd.sum(), "min": lambda: xd.min(), "max": lambda: xd.max(),
           "sumsq": lambda: (xd * xd).sum(), "amax": lambda: xd.abs().max()}[op]().item()
    got = out.item()
    assert ch.error() == 0 and ch.epoch() == 3
    if op in ("sum", "sumsq") and dt.is_floating_point:
        from cuda_mpi_reductions_amd.ops import sum_tolerance
        tol = sum_tolerance(dt, acc, n, (xd * xd).sum().item() if op == "sumsq" else xd.abs().sum().item())
        assert abs(got - ref) <= tol, (got, ref, tol)
    else:
        assert got == ref


# ---------------------------------------------------------------- bench: exact N-GPU step at N=1

@pytest.mark.parametrize("collective", ["rccl", "fused"])
def test_bench_torchrun_one_rank_graphs_both_modes(tmp_path, collective):
    # the cross-rank combine is issued at world 1 and captured into graphs for both
    # the pipelined headline and the serial measurement.
    r = torchrun(1, [BENCH, "--no-vector-extras", "--gpus", "1", "--steps", "8", "--warmup", "2", "--elements", "50000017",
                     "--collective", collective], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["n_gpus"] == 1 and d["config"]["collective"] == collective
    assert d["config"]["launch"].startswith("graph"), d["config"]["launch"]
    # the headline IS the per-reduction (serial, one lane) measurement
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["streams"] == 1 and d["config"]["overlap"].startswith("serial")
    combine = d["config"]["cross_rank_combine"]
    assert combine.startswith("none at world 1")  # the JSON says the combine is a no-op at world 1
    assert ("RCCL" in combine) if collective == "rccl" else ("fused" in combine)
    assert d["native_source_hash"] and d["native_source_hash"] != "unknown"
    assert d["config"]["topology"] == {"hosts": 1, "gpus": 1, "ranks_per_gpu": 1, "peer_access": "n/a (one GPU)"}
    dec = d["decomposition"]  # round 4: the step without its combine, and (fused) the device-timed exchange
    assert dec["consistent"] is True and dec["local_ms_per_step"] > 0
    if collective == "fused":
        w = dec["exchange_wait_us"]
        assert w["launches"] >= 8 and w["errors"] is None and 0 <= w["min_rank_median"] < 50, w
    else:
        assert "exchange_wait_us" not in dec


def test_bench_fused_two_lanes(tmp_path):
    r = run([sys.executable, BENCH, "--no-vector-extras", "--steps", "24", "--warmup", "2", "--elements", "50000017", "--collective",
             "fused", "--pipelined", "--streams", "2", "--graph-chunk", "8"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["config"]["streams"] == 2
    assert d["config"]["launch"].startswith("graph")


# ---------------------------------------------------------------- several ranks on the one GPU

@pytest.mark.parametrize("nproc", [2, 4])
def test_bench_fused_ranks_share_one_gpu(tmp_path, nproc, monkeypatch):
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    r = torchrun(nproc, [BENCH, "--no-vector-extras", "--gpus", str(nproc), "--backend", "gloo", "--collective", "fused", "--steps", "10",
                         "--warmup", "2", "--elements", "20000003", "--graph-chunk", "5"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["n_gpus"] == nproc
    assert d["config"]["launch"].startswith("graph")


@pytest.mark.parametrize("dt,op", [(torch.int64, "min"), (torch.float64, "sum")])
def test_fused_poison_reaches_every_rank(tmp_path, dt, op):
    # rank 1's polled fan-in misses its bound, so its partial is poisoned (the
    # MIN identity for int64, NaN for fp64) and pushed with the poison flag: rank 0 must flag its own
    # channel (bit 2) and poison its result too — never fold a neutral partial into a plausible
    # value with a clean error word. Then, after resets, a clean launch is exact on both ranks.
    script = tmp_path / "xp.py"
    script.write_text(
        "import math, os, sys, torch\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch.distributed as dist\n"
        "from cuda_mpi_reductions_amd._native import native\n"
        "from cuda_mpi_reductions_amd.ops import Reducer, default_acc_dtype, dtype_code, op_code\n"
        "from cuda_mpi_reductions_amd.parallel.xrank import open_channel\n"
        "dist.init_process_group('gloo')\n"
        "r = dist.get_rank(); C = native()\n"
        "dev = torch.device('cuda', 0); torch.cuda.set_device(dev)\n"
        f"dt, op = {dt}, {op!r}\n"
        "x = torch.full((1 << 22,), 3 + r, dtype=dt, device=dev)\n"
        "acc = default_acc_dtype(dt, op)\n"
        "out = torch.zeros(1, dtype=acc, device=dev)\n"
        "ch = open_channel(dev, timeout_s=5.0)\n"
        "red = Reducer(dev)\n"
        "s = torch.cuda.current_stream().cuda_stream\n"
        "def launch(**kw):\n"
        "    return C.reduce(red.ws, x.data_ptr(), x.numel(), dtype_code(dt), op_code(op), dtype_code(acc),\n"
        "                    out.data_ptr(), s, xrank=ch.desc_ptr, **kw)\n"
        "kw = dict(fanin_bound_ticks=100_000, debug_delay_wg=0, debug_delay_ticks=5_000_000) if r == 1 else {}\n"
        "launch(**kw); torch.cuda.synchronize()\n"
        "v = out.item(); fan, xr = red.ws.error(), ch.error()\n"
        "dist.barrier()\n"
        "red.ws.reset(s); ch.clear_error(); torch.cuda.synchronize(); dist.barrier()\n"
        "launch(); torch.cuda.synchronize()\n"
        "import json\n"
        f"open(os.path.join({str(tmp_path)!r}, 'r%d' % r), 'w').write(json.dumps((v, fan, xr, out.item(), ch.error())))\n"
        "dist.destroy_process_group()\n")
    r = torchrun(2, [str(script)], timeout=240, env={"MIREDUCE_FORCE_DEVICE": "0"})
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    import math
    ident = torch.iinfo(dt).max if op == "min" else 0
    clean = 3 if op == "min" else (3.0 + 4.0) * (1 << 22)
    res = {k: json.loads((tmp_path / f"r{k}").read_text()) for k in range(2)}
    for k, (v, fan, xr, v2, xr2) in res.items():
        assert (math.isnan(v) if dt.is_floating_point else v == ident), (k, v)
        assert v2 == clean and xr2 == 0, (k, v2, xr2)
    assert res[1][1] != 0 and res[1][2] == 0   # rank 1: its own fan-in failed; its channel saw clean peers
    assert res[0][1] == 0 and res[0][2] == 2   # rank 0: clean fan-in, a poisoned partial from rank 1


def test_fused_missing_peer_times_out_not_hangs(tmp_path):
    # Rank 1 never launches: rank 0's kernel must give up after its timeout, flag the channel
    # (sticky: the next launch does not wait again) and the collective check must report it.
    script = tmp_path / "xr.py"
    script.write_text(
        "import os, sys, time, torch\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch.distributed as dist\n"
        "from cuda_mpi_reductions_amd.ops import Reducer\n"
        "from cuda_mpi_reductions_amd.parallel.xrank import open_channel, check_channel\n"
        "dist.init_process_group('gloo')\n"
        "r = dist.get_rank()\n"
        "dev = torch.device('cuda', 0); torch.cuda.set_device(dev)\n"
        "x = torch.ones(1 << 20, dtype=torch.float64, device=dev)\n"
        "out = torch.zeros(1, dtype=torch.float64, device=dev)\n"
        "ch = open_channel(dev, timeout_s=0.5)\n"
        "b = Reducer(dev).bind(x, 'sum', out=out, xrank=ch)\n"
        "s = torch.cuda.current_stream().cuda_stream\n"
        "t0 = time.time()\n"
        "if r == 0:\n"
        "    b.launch(s); torch.cuda.synchronize()\n"
        "    t1 = time.time() - t0\n"
        "    b.launch(s); torch.cuda.synchronize()\n"
        "    t2 = time.time() - t0 - t1\n"
        f"    open(os.path.join({str(tmp_path)!r}, 'res'), 'w').write('%d %.3f %.3f' % (ch.error(), t1, t2))\n"
        "msg = check_channel([ch])\n"
        f"open(os.path.join({str(tmp_path)!r}, 'msg%d' % r), 'w').write(str(msg))\n"
        "dist.destroy_process_group()\n")
    r = torchrun(2, [str(script)], timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    err, t1, t2 = (tmp_path / "res").read_text().split()
    assert int(err) == 1 and 0.4 < float(t1) < 10 and float(t2) < 0.3
    for k in range(2):
        assert "timed out" in (tmp_path / f"msg{k}").read_text()


def test_bench_auto_falls_back_to_rccl_on_every_rank(tmp_path, monkeypatch):
    # One rank cannot create its mailbox (fault injector, kind mailbox): every rank must agree and run
    # the RCCL/gloo combine.
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    r = torchrun(2, [BENCH, "--no-vector-extras", "--gpus", "2", "--backend", "gloo", "--steps", "4", "--warmup", "1",
                     "--elements", "20000003", "--inject-fault", "mailbox@1"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["config"]["collective"] == "rccl"
    assert d["config"]["collective_choice"].startswith("auto; fused unavailable"), d["config"]["collective_choice"]
    assert "injected mailbox failure" in d["config"]["collective_choice"]


def test_bench_auto_headline_is_serial_fused_extras_after(tmp_path):
    # value = the serial one-lane fused measurement; the pipelined 2-lane number is
    # an extra measured after the line is final; at world 1 there is no RCCL combine to measure.
    r = run([sys.executable, BENCH, "--no-vector-extras", "--steps", "12", "--warmup", "2", "--elements", "50000017"],
            cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["config"]["collective"] == "fused"
    assert d["config"]["streams"] == 1 and d["config"]["launch"].startswith("graph")
    c = d["candidates"]
    assert c["fused_2lane_pipelined"]["verified"] is True and c["fused_2lane_pipelined"]["gbps"] > 0
    assert d["summary"]["pipelined_gbps"] == c["fused_2lane_pipelined"]["gbps"]
    assert d["summary"]["rccl_serial_gbps"] is None and "world 1" in c["rccl_serial"]["note"]


# ---------------------------------------------------------------- direct collective from Python

def test_direct_comm_world1_views_and_staging():
    from cuda_mpi_reductions_amd.parallel import DirectComm
    dev = torch.device("cuda", 0)
    comm = DirectComm(dev, 1 << 20)
    t = torch.arange(1000, dtype=torch.float64, device=dev)
    ref = t.clone()
    comm.allreduce(t, "sum")
    torch.cuda.synchronize()
    assert torch.equal(t, ref) and comm.check() is None and comm.epoch == 1
    iv, ov = comm.in_view(77, torch.int32), comm.out_view(77, torch.int32)
    iv.copy_(torch.arange(77, dtype=torch.int32, device=dev) - 30)
    comm.launch_reduce(77, torch.int32, "max", root=0)
    torch.cuda.synchronize()
    assert torch.equal(ov, iv) and comm.epoch == 2
    comm.read_peers()  # fabric probe at world 1 reads the own buffer: no barrier, no epoch change
    torch.cuda.synchronize()
    assert comm.epoch == 2 and comm.check() is None
    with pytest.raises(Exception, match="beyond the registered"):
        comm.read_peers((1 << 20) + 4096)


def test_direct_comm_registration_fault():
    # --inject-fault mailbox: this rank fails to register its buffers; the collective constructor
    # reports it (on every rank) instead of leaving a peer blocked
    from cuda_mpi_reductions_amd.parallel import DirectComm
    from cuda_mpi_reductions_amd.utils.fault import FaultInjector, parse_fault_spec
    with pytest.raises(RuntimeError, match="direct collective unavailable: rank 0: .*injected registration failure"):
        DirectComm(torch.device("cuda", 0), 1 << 20, fault=FaultInjector(parse_fault_spec("mailbox@0")))
    comm = DirectComm(torch.device("cuda", 0), 1 << 20)  # world 1: one workgroup per CU
    assert comm.grid == torch.cuda.get_device_properties(0).multi_processor_count
    print("device uuid:", getattr(torch.cuda.get_device_properties(0), "uuid", None),
          "pci_bus_id:", getattr(torch.cuda.get_device_properties(0), "pci_bus_id", None))


@pytest.mark.parametrize("nproc", [2, 3])
def test_bench_vector_direct_ranks_share_one_gpu(tmp_path, nproc, monkeypatch):
    # reduce.c semantics through bench.py with the direct one-kernel collective (verified against the
    # gathered inputs), and the same over the torch.distributed path for comparison.
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    for impl in ("direct",):  # (gloo cannot reduce GPU tensors; RCCL refuses 2 ranks on 1 GPU)
        r = torchrun(nproc, [BENCH, "--gpus", str(nproc), "--backend", "gloo", "--device", "cuda", "--config",
                             "xgmi_2g_double_sum_reduce", "--elements", "3000017", "--steps", "4", "--warmup", "1",
                             "--vector-impl", impl],
                     cwd=tmp_path, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        d = _json(r)
        assert d["verified"] is True and d["config"]["impl"] == impl and d["unit"] == "GiB/s"


def test_bench_vector_extras_in_headline(tmp_path):
    r = run([sys.executable, BENCH, "--steps", "4", "--warmup", "1", "--elements", "50000017", "--no-candidates"],
            cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    ex = d["reduce_c_vector"]
    for k in ("reduce_direct", "allreduce_direct"):
        assert ex[k].get("verified") is True and ex[k]["gibps"] > 0, (k, ex[k])
    # world 1: RCCL's 1-rank in-place reduce does no work -> null rows, never a number
    assert ex["reduce_rccl"]["gibps"] is None and ex["allreduce_rccl"]["gibps"] is None
    assert "peer_read" not in ex  # one rank: no peers to read
    tab = ex["table"]
    rccl = [t for t in tab if t["impl"] == "rccl"]
    assert len(rccl) == 6 and all(t["gibps"] is None for t in rccl)
    # reduce.c's table over the direct collective: RETRY_COUNT rounds of INT / DOUBLE x MAX / MIN / SUM,
    # retry-major, each collective timed on its own and verified (retry 0) / checksum-reproduced
    direct = [t for t in tab if t["impl"] == "direct"]
    order = [(dt, op) for dt in ("INT", "DOUBLE") for op in ("MAX", "MIN", "SUM")]
    assert [(t["retry"], t["dtype"], t["op"]) for t in direct] == [(x, dt, op) for x in range(5) for dt, op in order]
    assert all(t.get("verified") is True and t["gibps"] > 0 for t in direct), direct
    rows = ex["rows"]["direct"]
    assert rows[0] == "# DATATYPE OP NODES GB/sec" and len(rows) == 31 and rows[1].startswith("INT MAX 1 ")
    assert "rccl" not in ex["rows"]


def test_bench_fused_corrupt_rank_fails_verification(tmp_path, monkeypatch):
    # fault injection through the fused finish: rank 1's result is perturbed; the AND over ranks
    # of the per-slot verification must fail the run.
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    r = torchrun(2, [BENCH, "--no-vector-extras", "--gpus", "2", "--backend", "gloo", "--collective", "fused", "--steps", "6",
                     "--warmup", "2", "--elements", "20000003", "--inject-fault", "corrupt@1:3"], cwd=tmp_path,
                 timeout=600)
    assert r.returncode != 0
    d = _json(r)
    assert d["verified"] is False


def test_bench_auto_remeasures_over_rccl_when_fused_fails_the_headline(tmp_path, monkeypatch):
    # --collective auto: the fused finish passes its canary and self-check, then rank 1's result is
    # wrong on a timed step (the injected fault fires once). The headline is re-measured over the
    # process group's all-reduce, verifies, and the sidecar says why.
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    r = torchrun(2, [BENCH, "--no-vector-extras", "--gpus", "2", "--backend", "gloo", "--steps", "6",
                     "--warmup", "2", "--elements", "20000003", "--inject-fault", "corrupt@1:3"], cwd=tmp_path,
                 timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "fused finish failed on the headline steps" in r.stderr
    d = bench_record(r.stdout)
    assert d["verified"] is True and d["config"]["collective"] == "rccl"
    assert "fused finish failed on the headline steps" in d["config"]["collective_choice"]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    # the reason rides in the printed line's config (the driver's record keeps config values)
    assert line["config"]["collective_reason"].startswith("fused finish failed on the headline steps")


# ---------------------------------------------------------------- the N=8 shapes, rehearsed
# Eight ranks share the one GPU of the test box: the world-8 mailbox indexing of the fused finish,
# the W=8 instantiation of the direct kernel and bench.py's 8-rank flow (not xGMI speed).

def test_bench_eight_ranks_fused_on_one_gpu(tmp_path, monkeypatch):
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    r = torchrun(8, [BENCH, "--gpus", "8", "--backend", "gloo", "--collective", "fused", "--steps", "12",
                     "--warmup", "2", "--elements", "40000003", "--graph-chunk", "6", "--no-vector-extras"],
                 cwd=tmp_path, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["n_gpus"] == 8 and d["config"]["parallelism"] == "dp8"
    assert d["config"]["launch"].startswith("graph")
    lo, hi = d["summary"]["wait_us"]  # the device-timed exchange wait, min / max rank median
    assert 0 <= lo <= hi and d["config"]["peer_access"]


def test_bench_eight_ranks_auto_on_one_gpu(tmp_path, monkeypatch):
    # the driver's default command at N=8 (auto-tuned combine), rehearsed with gloo on one GPU
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    r = torchrun(8, [BENCH, "--gpus", "8", "--backend", "gloo", "--steps", "12", "--warmup", "2",
                     "--elements", "40000003", "--tune-steps", "4"], cwd=tmp_path, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["n_gpus"] == 8
    assert d["config"]["collective"] == "fused" and "reduce_c_vector" in d
    assert d["rccl_ranks_seen"] is None and d["ranks_seen"] == 8  # gloo here
    # peer_map: eight ranks, one physical GPU, nothing to map across devices
    assert d["config"]["topology"] == {"hosts": 1, "gpus": 1, "ranks_per_gpu": 8, "peer_access": "n/a (one GPU)"}
    ex = d["reduce_c_vector"]
    bad = [t for t in ex["table"] if t.get("verified") is not True]
    assert not bad and len(ex["table"]) == 30, (bad, r.stderr[-2000:])
    assert ex["reduce_direct"].get("verified") is True, (ex["reduce_direct"], ex.get("allreduce_direct"))
    # eight ranks on one GPU split its CUs, so every rank's barrier kernel can be co-resident
    assert ex["direct_grid"] == torch.cuda.get_device_properties(0).multi_processor_count // 8, ex["direct_grid"]
    assert len(ex["rows"]["direct"]) == 31 and ex["rows"]["direct"][1].startswith("INT MAX 8 ")
    pr = ex["peer_read"]  # fabric probe: 8 ranks reading each other's buffers (here all on one GPU)
    assert "error" not in pr and 0 < pr["ingress_gbps_min"] <= pr["ingress_gbps_max"] and pr["node_gbps"] > 0, pr


def test_reduce_xgmi_direct_eight_ranks_on_one_gpu():
    # Two hardware queues per rank (HIP's default here is 4): 8 ranks x 4 plus the test process's own
    # can exceed the queues the scheduler keeps mapped at once, and a rank whose queue is swapped out
    # leaves its peers spinning at the device-side barrier until the next time slice (one box: 50 s
    # instead of 3 s). Each rank runs one stream, so nothing of its own waits behind the barrier.
    from helpers import BIN
    r = torchrun(8, env={"GPU_MAX_HW_QUEUES": "2"}, script_args=["--no-python", os.path.join(BIN, "reduce_xgmi"), "--mode=vector", "--collective=direct",
                     "--ints=4000037", "--doubles=2000003", "--dtypes=INT,DOUBLE", "--retries=1", "--iters=3",
                     "--direct-grid=16", "--timeout=30", "--graph"], timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "verification PASSED" in r.stderr


def test_bench_extras_deadline_keeps_the_headline(tmp_path):
    # reduce.c extras past their deadline: the headline line is still printed (extras marked as
    # timed out) and the run ends with the headline's status.
    r = run([sys.executable, BENCH, "--steps", "4", "--warmup", "1", "--elements", "50000017",
             "--extras-deadline", "0.05"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = _json(r)
    assert d["verified"] is True and "did not finish" in d["summary"]["extras_error"]
    assert "extras_skipped" not in d["summary"]  # an explicit short deadline cuts the extras, not skips them
    if "reduce_c_vector" in d:  # (the deadline may pass before the table starts)
        assert "did not finish" in d["reduce_c_vector"]["error"]


def test_bench_extras_hang_in_rccl_candidate_keeps_the_headline(tmp_path, monkeypatch):
    # a hang inside an after-headline RCCL candidate (fault site "extras") still
    # ends the run with the verified headline printed and rc 0 (the extras watchdog), on every rank.
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    r = torchrun(2, [BENCH, "--no-vector-extras", "--gpus", "2", "--backend", "gloo", "--collective", "rccl",
                     "--steps", "4", "--warmup", "1", "--elements", "20000003", "--extras-deadline", "25",
                     "--inject-fault", "hang@1:0/extras"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["verified"] is True and d["value"] > 0 and "did not finish" in d["summary"]["extras_error"]
    assert "hang at bench extras 0" in r.stderr


def test_bench_plan_tuning_at_the_eight_gpu_shard(tmp_path):
    # auto at the 1 GB shard: the tuned default plan is measured against 256x8x1 and the faster
    # is the one the headline runs.
    r = run([sys.executable, BENCH, "--steps", "8", "--warmup", "2", "--elements", "125000000",
             "--no-vector-extras", "--tune-steps", "8"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True
    pt = d["plan_tuning"]
    table = pt["gbps_by_rank"][0]  # per rank: one rank here
    assert set(table) == {"tuned default", "tuned default, XCD skew 0", "tuned default, XCD skew 40",
                          "tuned default, XCD skew -20", "256x4x2 window 2"}
    assert pt["chosen"] == max(table, key=table.get) == pt["plan_by_rank"][0]
    assert d["summary"]["plans"] == pt["chosen"]
    plan = d["config"]["kernel_plan"]
    # (block, unroll, window, xskew): 119 rounds per workgroup at the 1 GB shard; the tuned default
    # gives the favoured XCD parity 2 + 1.8 % of the rounds = 4 (round 5, profiles/r5_skew/)
    want = {"tuned default": (256, 8, 4, 4), "tuned default, XCD skew 0": (256, 8, 4, 0),
            "tuned default, XCD skew 40": (256, 8, 4, 5), "tuned default, XCD skew -20": (256, 8, 4, -2),
            "256x4x2 window 2": (256, 4, 2, 0)}
    assert (plan["block"], plan["unroll"], plan["window"], plan["xskew"]) == want[pt["chosen"]]


def test_bench_maxloc_config_skips_plan_tuning(tmp_path):
    # MAXLOC runs the arg-reduction kernel (no streaming plan to re-bind): auto must not plan-tune it.
    r = run([sys.executable, BENCH, "--config", "xgmi_1b_double_maxloc", "--steps", "4", "--warmup", "1",
             "--elements", "125000000", "--no-vector-extras"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and "plan_tuning" not in d


# ---------------------------------------------------------------- bench: replay probe, decomposition

def test_bench_replay_probe_and_decomposition_one_gpu(tmp_path):
    # VERDICT r3 items 2 and 4 on the GPU path: the RCCL combine captured at world 1 runs the replay
    # probe (forced on) and passes it; the decomposition's local time is the same kernel without
    # the combine, so at world 1 the exchange costs little.
    r = run([sys.executable, BENCH, "--no-vector-extras", "--no-candidates", "--steps", "40", "--warmup", "2",
             "--elements", "50000017", "--collective", "rccl", "--replay-probe", "on"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["config"]["launch"].startswith("graph") and "replay probe ok" in d["config"]["launch"]
    dec = d["decomposition"]
    assert dec["consistent"] is True and dec["local_launch"].startswith("graph")
    assert 0 < dec["local_ms_per_step"] <= d["ms_per_step"] * 1.5
    assert dec["local_ms_min"] <= dec["local_ms_max"] and dec["skew_us_per_step"] == 0.0  # one rank
    assert d["launcher"] == "single process" and d["rccl_ranks_seen"] == 1


def test_bench_replay_probe_failure_goes_eager_one_gpu(tmp_path):
    # a probe that misses its deadline (injected 1.5 s delay vs a 0.5 s deadline) sends the headline to
    # eager issue; it is still measured and verified (rc 0)
    r = run([sys.executable, BENCH, "--no-vector-extras", "--no-candidates", "--steps", "10", "--warmup", "2",
             "--elements", "50000017", "--collective", "rccl", "--replay-probe", "on", "--probe-deadline", "0.5",
             "--inject-fault", "delay=1500@0/capture"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True
    assert d["config"]["launch"].startswith("eager (captured replay probe failed: rank 0: "), d["config"]["launch"]


@pytest.mark.parametrize("fault", [None, "abort@1"])
def test_bench_fused_canary_two_ranks_one_gpu(tmp_path, monkeypatch, fault):
    # the fused finish's canary (parallel/canary.py) with real GPU helpers (two ranks sharing the
    # GPU): clean -> fused chosen; a helper that aborts -> every rank declines the fused finish and
    # the headline is still measured and verified over the other combine
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    monkeypatch.setenv("MIREDUCE_CANARY_FORCE", "1")  # ranks share the GPU: the canary would be skipped
    if fault:
        monkeypatch.setenv("MIREDUCE_CANARY_FAULT", fault)
    r = torchrun(2, [BENCH, "--no-vector-extras", "--no-candidates", "--gpus", "2", "--backend", "gloo", "--steps", "6",
                     "--warmup", "2", "--elements", "20000003", "--canary-timeout", "40"], cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["n_gpus"] == 2
    if fault:
        assert d["config"]["collective"] == "rccl"
        assert "canary: rank 1: helper crashed (signal 6)" in d["config"]["collective_choice"], \
            d["config"]["collective_choice"]
    else:
        assert d["config"]["collective"] == "fused", d["config"]["collective_choice"]


@pytest.mark.parametrize("plan", ["tuned default, XCD skew 0", "tuned default, XCD skew -20", "256x4x2 window 2"])
def test_bench_ranks_hold_different_plans_and_verify(tmp_path, monkeypatch, plan):
    # plan tuning is per rank. Two ranks sharing the GPU, each with a 1 GB shard
    # (so the candidates are timed); rank 1 is made to hold another plan than rank 0 would pick —
    # every candidate the tuner can choose (the self-check ran with the default plan before tuning)
    # must combine with the fused finish, next to a rank of another plan, and verify every step.
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    monkeypatch.setenv("MIREDUCE_TEST", "1")  # the hook is honoured in test runs only
    monkeypatch.setenv("MIREDUCE_PLAN_FOR_RANK", f"1={plan}")
    side = tmp_path / "x.json"
    r = torchrun(2, [BENCH, "--no-vector-extras", "--no-candidates", "--gpus", "2", "--backend", "gloo", "--steps", "8",
                     "--warmup", "2", "--elements", "250000000", "--tune-steps", "6", "--extras-file", str(side)],
                 cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r)
    assert d["verified"] is True and d["config"]["collective"] == "fused"
    pt = d["plan_tuning"]
    assert len(pt["plan_by_rank"]) == 2 and pt["plan_by_rank"][1] == plan, pt
    assert all(len(t) == 5 for t in pt["gbps_by_rank"])
    assert d["summary"]["plans"].count(" x") == (1 if pt["plan_by_rank"][0] == pt["plan_by_rank"][1] else 2)


# ---------------------------------------------------------------- fail-soft optional stages (round 6)
@pytest.mark.parametrize("fault", ["raise@1/tune", "raise@1/selfcheck", "hang@1/tune"])
def test_bench_optional_stage_failure_two_ranks_one_gpu(tmp_path, monkeypatch, fault):
    # VERDICT r5 item 1 on the GPU path: plan tuning (local launches on fresh workspaces, one bounded
    # agreement) and the fused self-check (real fused launches, local error words) fail on rank 1 of
    # two ranks sharing the GPU. raise -> every rank falls back (tuned default plan / RCCL), the
    # headline is measured and verified, the reason named; hang -> the agreement names the stage and
    # the lost rank within --agree-timeout, one line, no number.
    monkeypatch.setenv("MIREDUCE_FORCE_DEVICE", "0")
    r = torchrun(2, [BENCH, "--no-vector-extras", "--no-candidates", "--gpus", "2", "--backend", "gloo", "--steps", "6",
                     "--warmup", "2", "--elements", "250000000", "--tune-steps", "6", "--agree-timeout", "5",
                     "--xrank-timeout", "3", "--inject-fault", fault], cwd=tmp_path, timeout=600)
    lines = [ln for ln in r.stdout.splitlines() if "{" in ln]
    assert len(lines) == 1, (r.stdout, r.stderr[-3000:])
    d = json.loads(lines[0][lines[0].index("{"):])
    if fault.startswith("raise"):
        assert r.returncode == 0, r.stderr[-3000:]
        assert d["verified"] is True and d["value"] > 0
        if fault.endswith("tune"):
            assert d["config"]["collective"] == "fused" and "rank 1: InjectedFault" in d["config"]["plan_reason"]
        else:
            assert d["config"]["collective"] == "rccl"
            assert d["config"]["collective_reason"].startswith("self-check: rank 1: InjectedFault")
    else:
        assert r.returncode != 0 and d["value"] is None
        assert "plan tuning: rank(s) 1 did not report within 5 s" in d["error"], d


def test_use_kernel_rebinds_locally_and_keeps_the_channel():
    # bench.py binds each rank's tuned plan with ScalarReduction.use_kernel: local (no collective),
    # the lane keeps its fused channel, whose epoch counter runs on across the re-bind, and the
    # steps stay exact under the new plan
    from dataclasses import replace
    from cuda_mpi_reductions_amd.models import CONFIGS, scalar_workload
    from cuda_mpi_reductions_amd.ops import KernelConfig
    from cuda_mpi_reductions_amd.parallel import dist as pdist
    ctx = pdist.init(backend="gloo", device_type="cuda")  # (the fused finish needs no RCCL)
    try:
        cfg = replace(CONFIGS["xgmi_1b_double_sum"], n_total=30_000_017)
        wl = scalar_workload(cfg, ctx, collective="fused").setup()
        ch = wl.channels[0]
        slots = wl.new_slots(6)
        for i in range(3):
            wl.step(slots[i:i + 1])
        torch.cuda.synchronize()
        assert ch.epoch() == 3
        plan0 = dict(wl.reducer.last_plan)
        wl.use_kernel(KernelConfig(block=256, unroll=4, wg_per_cu=2, window=2), streams=1)
        assert wl.channels[0] is ch and wl.lanes[0][3] is ch
        assert wl.reducer.last_plan["unroll"] == 4 and wl.reducer.last_plan != plan0
        for i in range(3, 6):
            wl.step(slots[i:i + 1])
        torch.cuda.synchronize()
        assert ch.epoch() == 6 and ch.error() == 0 and wl.error_counts() == [0, 0, 0, 0]
        ref = wl.x.sum(dtype=torch.float64).item()
        for v in slots.cpu().tolist():
            assert abs(v - ref) <= 1e-9 * abs(ref), (v, ref)
    finally:
        pdist.shutdown(ctx)
