"""arg_reduce / argmax / argmin (csrc/kernels/arg_reduce.hip, csrc/runtime/arg_reduce_cpu.cpp)
against torch.argmax / argmin on the host (first occurrence, NaN the extreme). Data is drawn from
a small integer range so ties are everywhere and the first-occurrence rule is what is tested;
shapes cover the short-row lane groups (1..256 columns), long split rows, whole arrays split into
thousands of segments, misaligned bases and every element type."""
import os
import sys

import pytest
import torch

from cuda_mpi_reductions_amd.ops import arg_reduce, argmax, argmin

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

DTYPES = [torch.float64, torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.int64]


def _data(shape, dt, seed=0, lo=-60, hi=60, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(lo, hi, shape, generator=g).to(dt)
    return x.to(device)


def _torch_ref(x: torch.Tensor, op: str, dim=None):
    h = x.cpu()
    if h.dtype in (torch.bfloat16, torch.float16):
        h = h.float()  # exact; host argmax over halves compares the same values
    return (h.argmax(dim) if op == "max" else h.argmin(dim)) if dim is not None else (h.argmax() if op == "max" else h.argmin())


def _check(x, op, dim=None):
    v, i = arg_reduce(x, op, dim)
    exp = _torch_ref(x, op, dim)
    assert torch.equal(i.cpu(), exp), (i.cpu()[:8], exp[:8] if exp.dim() else exp)
    # value = the element at the index (exact, NaN included)
    if dim is None:
        ref_v = x.reshape(-1)[exp].cpu()
    else:
        ref_v = torch.gather(x.cpu(), dim % x.dim(), exp.unsqueeze(dim % x.dim())).squeeze(dim % x.dim())
    got_v = v.cpu()
    if got_v.is_floating_point():
        assert torch.equal(torch.isnan(got_v), torch.isnan(ref_v))
        got_v, ref_v = got_v.nan_to_num(), ref_v.nan_to_num()
    assert torch.equal(got_v, ref_v)


# ---- host path (native reference) ----------------------------------------------------------

@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("op", ["max", "min"])
def test_host_rows_and_whole(dt, op):
    x = _data((33, 517), dt, seed=1)
    _check(x, op, 1)
    _check(x, op, 0)
    _check(x, op)


def test_host_nan_zero_inf_rules():
    x = torch.tensor([1.0, float("nan"), 3.0, float("nan")])
    assert int(argmax(x)) == 1 and int(argmin(x)) == 1
    x = torch.tensor([-0.0, 0.0, -0.0])
    assert int(argmax(x)) == 0 and int(argmin(x)) == 0
    assert int(argmax(torch.full((9,), float("-inf")))) == 0
    assert int(argmin(torch.full((9,), float("inf")))) == 0
    i = torch.iinfo(torch.int32)
    assert int(argmax(torch.full((5,), i.min, dtype=torch.int32))) == 0
    assert int(argmin(torch.full((5,), i.max, dtype=torch.int32))) == 0


def test_host_long_row_threads():
    x = torch.zeros(1 << 23)
    x[6_000_000] = 2
    x[6_000_001] = 2
    x[7_000_000] = float("nan")
    assert int(argmax(x[:7_000_000])) == 6_000_000
    assert int(argmax(x)) == 7_000_000


def test_keepdim_and_errors():
    x = _data((4, 6, 5), torch.float32)
    v, i = arg_reduce(x, "max", 1, keepdim=True)
    assert i.shape == (4, 1, 5) and torch.equal(i.squeeze(1), x.argmax(1))
    v, i = arg_reduce(x, "min", keepdim=True)
    assert i.shape == (1, 1, 1)
    with pytest.raises(ValueError):
        arg_reduce(torch.empty(0), "max")
    with pytest.raises(ValueError):
        arg_reduce(x, "sum")
    with pytest.raises(TypeError):
        arg_reduce(torch.zeros(4, dtype=torch.uint8), "max")


def test_global_two_cpu_ranks(tmp_path):
    from helpers import torchrun
    script = tmp_path / "argd.py"
    script.write_text(
        "import os, sys, torch\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch.distributed as dist\n"
        "from cuda_mpi_reductions_amd.ops import arg_reduce\n"
        "dist.init_process_group('gloo')\n"
        "r = dist.get_rank()\n"
        "x = torch.zeros(1000 + 7 * r)\n"
        "x[100 + r] = 5.0   # tie across ranks: rank 0's copy is first\n"
        "x[900] = -3.0 if r == 1 else 0.0\n"
        "v, i = arg_reduce(x, 'max', group=dist.group.WORLD)\n"
        "v2, i2 = arg_reduce(x, 'min', group=dist.group.WORLD)\n"
        f"open(os.path.join({str(tmp_path)!r}, 'res%d' % r), 'w').write('%r %d %r %d' % (float(v), int(i), float(v2), int(i2)))\n"
        "dist.destroy_process_group()\n")
    r = torchrun(2, [str(script)], timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    for rank in range(2):  # (ranks' stdout interleaves: each writes its own file)
        v, i, v2, i2 = (tmp_path / f"res{rank}").read_text().split()
        assert float(v) == 5.0 and int(i) == 100  # rank 0's element 100
        assert float(v2) == -3.0 and int(i2) == 1000 + 900  # rank 1's element 900 after rank 0's 1000


def test_rank_local_without_group_in_a_job(tmp_path):
    # without group=, a whole-array arg_reduce stays rank-local even when a
    # world>1 process group exists (a rank-local argmax in a DDP job must not become a collective).
    from helpers import torchrun
    script = tmp_path / "argl.py"
    script.write_text(
        "import os, sys, torch\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch.distributed as dist\n"
        "from cuda_mpi_reductions_amd.ops import arg_reduce\n"
        "dist.init_process_group('gloo')\n"
        "r = dist.get_rank()\n"
        "x = torch.zeros(50)\n"
        "x[10 + r] = 1.0\n"
        "if r == 0:\n"
        "    v, i = arg_reduce(x, 'max')  # only rank 0 calls it: must not hang\n"
        "    open(os.path.join(%r, 'res'), 'w').write('%%d' %% int(i))\n" % str(tmp_path) +
        "dist.barrier()\n"
        "dist.destroy_process_group()\n")
    r = torchrun(2, [str(script)], timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert int((tmp_path / "res").read_text()) == 10


# ---- device kernels ------------------------------------------------------------------------

ROW_SHAPES = [(1, 1), (3, 5), (1000, 64), (513, 65), (77, 128), (300, 129), (64, 256), (5, 257), (8, 4096),
              (3, 100_003), (1, 3_000_001), (4096, 1000), (2, 8192 + 3), (100, 2048), (77, 1000), (33, 1536)]


@pytest.mark.gpu
@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("op", ["max", "min"])
@pytest.mark.parametrize("shape", ROW_SHAPES, ids=lambda s: f"{s[0]}x{s[1]}")
def test_device_rows(dt, op, shape):
    x = _data(shape, dt, seed=shape[0] * 7 + shape[1], device="cuda")
    _check(x, op, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("op", ["max", "min"])
@pytest.mark.parametrize("n", [1, 7, 255, 4096, 65_537, (1 << 20) + 3, 50_000_017])
@pytest.mark.parametrize("off", [0, 1, 3])
def test_device_whole(dt, op, n, off):
    base = _data((n + off,), dt, seed=n + off, lo=-1000, hi=1000, device="cuda")
    x = base[off:]
    _check(x, op)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.float64, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(1, 5_000_000), (200, 3000), (4096, 64), (1000, 200)], ids=str)
def test_device_nan_and_infinities(dt, shape):
    x = _data(shape, dt, seed=5, device="cuda")
    rows, cols = shape
    g = torch.Generator().manual_seed(9)
    for _ in range(max(1, rows // 3)):  # scattered NaNs, several in some rows
        r, c = int(torch.randint(rows, (1,), generator=g)), int(torch.randint(cols, (1,), generator=g))
        x[r, c] = float("nan")
    x[0, :] = float("-inf")  # an all -inf row: argmax 0
    if rows > 2:
        x[1, :] = float("inf")  # an all +inf row: argmin 0
        x[2, cols // 2] = float("inf")
        x[2, cols - 1] = float("inf")
    for op in ("max", "min"):
        _check(x, op, 1)
        _check(x, op)


@pytest.mark.gpu
def test_device_first_of_many_ties_in_split_row():
    # one long row split into hundreds of segments; the maximum appears in many segments
    x = torch.zeros(40_000_000, dtype=torch.float32, device="cuda")
    pos = torch.tensor([39_999_999, 12_345_678, 20_000_000, 12_345_679], device="cuda")
    x[pos] = 7.0
    assert int(argmax(x)) == 12_345_678
    x[3] = float("nan")
    assert int(argmax(x)) == 3 and int(argmin(x)) == 3


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [0, 1, 2, -1])
def test_device_other_dims(dim):
    x = _data((6, 70, 33), torch.bfloat16, seed=dim + 4, device="cuda")
    _check(x, "max", dim)
    _check(x, "min", dim)


@pytest.mark.gpu
def test_device_repeat_and_stream_reuse():
    # split rows leave their tickets zero: relaunching the same shapes stays right
    x = _data((4, 1_000_003), torch.float32, seed=3, device="cuda")
    for _ in range(5):
        _check(x, "max", 1)
        _check(x, "min")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        i = argmax(x, 1)
    s.synchronize()
    assert torch.equal(i.cpu(), x.cpu().argmax(1))


@pytest.mark.gpu
def test_device_split_scratch_reuse_with_more_rows():
    # a split launch with few rows followed, on the same stream and scratch, by a
    # split launch with MORE rows must not read the first launch's partials as its tickets.
    x1 = _data((30_000_000,), torch.float32, seed=11, device="cuda")  # 1 row, hundreds of segments
    _check(x1, "max")
    x2 = _data((128, 131072), torch.bfloat16, seed=12, device="cuda")  # 128 rows < CUs: split rows
    for _ in range(3):
        _check(x2, "max", 1)
        _check(x1, "min")
        _check(x2, "min", 1)


@pytest.mark.gpu
def test_device_native_kernel_runs():
    from cuda_mpi_reductions_amd._native import native
    C = native()
    x = _data((1, 20_000_000), torch.float64, device="cuda")
    v = torch.empty(1, dtype=x.dtype, device="cuda")
    i = torch.empty(1, dtype=torch.int64, device="cuda")
    need = C.arg_reduce_scratch_bytes(1, x.numel(), 3, 256)
    scratch = torch.zeros(need, dtype=torch.uint8, device="cuda")
    plan = C.arg_reduce_rows(x.data_ptr(), 1, x.numel(), 3, 2, v.data_ptr(), i.data_ptr(), scratch.data_ptr(), 256,
                             torch.cuda.current_stream().cuda_stream)
    assert plan["splits"] > 1 and plan["grid"] >= 256
    assert int(i) == int(x.cpu().argmax())


@pytest.mark.gpu
@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("op", ["max", "min"])
def test_device_loc_pack_pick(dt, op):
    # the device-side MAXLOC / MINLOC combine (models/loc.py): one (value, index + offset) pair per
    # "rank", folded with arg_reduce's rules — the extreme wins, equal values go to the smaller
    # global index, NaN is the extreme
    from cuda_mpi_reductions_amd._native import native
    from cuda_mpi_reductions_amd.ops.reduce import DTYPE_CODES, op_code
    C = native()
    code, oc = DTYPE_CODES[dt], op_code(op)

    def pick(values, local_idx, offsets):
        w = len(values)
        pairs = torch.empty(2 * w, dtype=torch.int64, device="cuda")
        val = torch.tensor(values, dtype=torch.float64).to(dt).cuda()
        idx = torch.tensor(local_idx, dtype=torch.int64, device="cuda")
        for r in range(w):
            C.loc_pack(val[r:].data_ptr(), idx[r:].data_ptr(), offsets[r], code, pairs[2 * r:].data_ptr())
        out_i = torch.full((1,), -1, dtype=torch.int64, device="cuda")
        out_v = torch.empty(1, dtype=dt, device="cuda")
        C.loc_pick(pairs.data_ptr(), w, code, oc, out_i.data_ptr(), out_v.data_ptr())
        torch.cuda.synchronize()
        return int(out_i), out_v.cpu().double().item()

    # ties on the extreme across ranks: the smallest GLOBAL index wins (offset + local index)
    vals = [3, 7, 7, -2, 7, -2]
    loc = [50, 40, 10, 5, 30, 6]
    offs = [0, 100, 200, 300, 400, 500]
    gi, v = pick(vals, loc, offs)
    assert (gi, v) == ((140, 7.0) if op == "max" else (305, -2.0))
    assert pick([5], [9], [1000]) == (1009, 5.0)  # world 1
    if dt.is_floating_point:
        gi, v = pick([3, float("nan"), 7, float("nan")], [1, 9, 2, 4], [0, 10, 20, 30])
        assert gi == 19 and v != v  # the first NaN (global index 10 + 9) beats every number, max or min
