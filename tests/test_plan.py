"""Launch planning (host side of csrc/kernels/reduce.hip and ladder.hip)."""
import pytest

from cuda_mpi_reductions_amd._native import native

F64 = 3


def test_head_body_tail_split():
    C = native()
    for addr in (0x1000, 0x1008):
        for n in (0, 1, 2, 3, 5, 1001):
            p = C.plan(addr, n, F64)
            head = 0 if addr % 16 == 0 else min(1, n)
            assert p["head"] == head
            assert p["head"] + 2 * p["nvec"] + p["tail"] == n
            assert 0 <= p["tail"] < 2


def test_int32_vector_split():
    C = native()
    p = C.plan(0x1004, 1003, 0)          # int32, 4-byte aligned only
    assert p["head"] == 3 and p["head"] + 4 * p["nvec"] + p["tail"] == 1003


def test_misaligned_element_rejected():
    C = native()
    with pytest.raises(C.NativeError):
        C.plan(0x1001, 10, F64)


@pytest.mark.parametrize("n", [0, 1, 100, 10**6, 10**9, 3 * 10**9])
def test_grid_bounds(n):
    C = native()
    p = C.plan(0, n, F64, num_cus=256)
    assert 1 <= p["grid"] <= 256 * 8
    tile = p["block"] * p["unroll"]
    assert p["grid"] <= max(1, -(-p["nvec"] // tile))


def test_tuned_defaults_by_size():
    C = native()
    big = C.plan(0, 10**9, F64)            # 8 GB of 8-byte elements: explicit load window 4 (profiles/r3_window)
    assert (big["block"], big["unroll"], big["grid"], big["nontemporal"], big["window"]) == (256, 8, 256, True, 4)
    mid = C.plan(0, 125_000_000, F64)      # 1 GB: the 8-GPU shard of the north star
    assert (mid["block"], mid["unroll"], mid["grid"], mid["nontemporal"], mid["window"]) == (256, 8, 256, True, 4)
    l3 = C.plan(0, 1 << 25, F64)           # 256 MB: nt is fast warm and cold (plan_256mb.csv)
    assert (l3["block"], l3["unroll"], l3["grid"], l3["nontemporal"], l3["window"]) == (256, 8, 256, True, 4)
    small = C.plan(0, 1 << 24, F64)        # 128 MB (the reference default): hipcc's schedule
    assert (small["block"], small["unroll"], small["window"]) == (256, 4, 0)
    # no size band picks the default (non-nt) policy: it collapses to 2.7 TB/s on a cold cache
    assert all(C.plan(0, n, F64)["nontemporal"] for n in (1, 1 << 20, 3 << 23, 1 << 25, 3 << 24, 1 << 27))
    i64 = C.plan(0, 10**9, 1)              # 8 GB of int64: like fp64
    assert (i64["block"], i64["unroll"], i64["grid"], i64["window"]) == (256, 8, 256, 4)
    # XCD-weighted split (profiles/r4_xcd/, r4_skew/): 20 permille of the rounds extra for the
    # workgroups on odd XCCs in the 8- and 4-byte window-4 plans; explicit values override; no
    # window -> no skew
    assert big["xskew"] == 19 and mid["xskew"] == 4     # 953 and 119 rounds per workgroup: 2 + 18 permille
    assert C.plan(0, 250_000_000, F64)["xskew"] == 6 and C.plan(0, 1 << 25, F64)["xskew"] == 1  # 238 / 32 rounds
    assert C.plan(0, 10**9, F64, xcd_skew=0)["xskew"] == 0 and C.plan(0, 10**9, F64, xcd_skew=-40)["xskew"] == -38
    assert small["xskew"] == 0
    f32 = C.plan(0, 2 * 10**9, 2)          # fp32 SUM 8 GB: window 4, the same skew (profiles/r4_shard/)
    assert f32["window"] == 4 and f32["xskew"] == 19
    bf16 = C.plan(0, 4 * 10**9, 4)         # bf16 SUM 8 GB: window 4 but no skew (profiles/r4_xcd/)
    assert bf16["window"] == 4 and bf16["xskew"] == 0
    i32 = C.plan(0, 2 * 10**9, 0)          # int32 SUM: the window-2 plan, unmeasured: no skew
    assert i32["window"] == 2 and i32["xskew"] == 0


# op codes: SUM 0, MIN 1, MAX 2, SUMSQ 3, AMAX 4; dtypes: int32 0, int64 1, f32 2, f64 3, bf16 4, f16 5
@pytest.mark.parametrize("dtype,n,op,want", [
    (2, 2 * 10**9, 0, (256, 8, 256, 4)),   # f32 SUM 8 GB: window 4 (profiles/r3_types/)
    (2, 250_000_000, 0, (256, 8, 256, 4)),  # f32 SUM 1 GB
    (2, 2 * 10**9, 2, (256, 8, 256, 4)),   # f32 MAX 8 GB
    (0, 2 * 10**9, 2, (256, 8, 256, 4)),   # int32 MAX 8 GB
    (0, 2 * 10**9, 0, (256, 8, 512, 2)),   # int32 SUM (int64 accumulation): 256x8x2, window 2
    (0, 250_000_000, 0, (256, 8, 512, 2)),  # int32 SUM 1 GB
    (4, 4 * 10**9, 0, (256, 8, 256, 4)),   # bf16 SUM 8 GB
    (4, 5 * 10**8, 0, (256, 8, 256, 4)),   # bf16 SUM 1 GB
    (5, 4 * 10**9, 2, (256, 8, 512, 2)),   # f16 MAX 8 GB: 256x8x2, window 2
    (3, 10**9, 1, (256, 8, 256, 4)),       # f64 MIN: the operator does not move 8-byte plans
    (2, 1 << 24, 0, (256, 4, 768, 0)),     # <= 192 MB: unchanged (256x4x3, hipcc's schedule)
    (4, 1 << 25, 0, (256, 4, 768, 0)),
])
def test_tuned_defaults_by_dtype_and_op(dtype, n, op, want):
    p = native().plan(0, n, dtype, op=op)
    assert (p["block"], p["unroll"], p["grid"], p["window"]) == want and p["nontemporal"]


def test_window_only_where_instantiated():
    C = native()
    # explicit plans keep hipcc's schedule unless a window is asked for
    assert C.plan(0, 10**9, F64, block=256, unroll=8)["window"] == 0
    assert C.plan(0, 10**9, F64, block=256, unroll=8, window=4)["window"] == 4
    # not instantiated: 1024 threads, unroll 16, the default (non-nt) policy
    assert C.plan(0, 10**9, F64, block=1024, unroll=4, window=2)["window"] == 0
    assert C.plan(0, 10**9, F64, block=256, unroll=16, window=4)["window"] == 0
    assert C.plan(0, 10**9, F64, block=256, unroll=4, window=2, policy=0)["window"] == 0
    assert C.plan(0, 10**9, F64, block=256, unroll=2, window=4)["window"] == 0  # 4 does not divide 2
    assert C.plan(0, 10**9, F64, window=0)["window"] == 0  # the tuned plan with hipcc's schedule
    with pytest.raises(C.NativeError):
        C.plan(0, 10, F64, window=3)


def test_overrides_and_caps():
    C = native()
    p = C.plan(0, 10**9, F64, block=1024, unroll=8, wg_per_cu=2, max_blocks=100, policy=0)
    assert (p["block"], p["unroll"], p["grid"], p["nontemporal"]) == (1024, 8, 100, False)
    p = C.plan(0, 10**9, F64, single_pass=False)
    assert p["single_pass"] is False
    with pytest.raises(C.NativeError):
        C.plan(0, 10, F64, block=384)
    with pytest.raises(C.NativeError):
        C.plan(0, 10, F64, unroll=3)


def next_pow2(x):
    return 1 if x <= 1 else 1 << (x - 1).bit_length()


@pytest.mark.parametrize("kernel", range(7))
@pytest.mark.parametrize("n", [1, 2, 33, 64, 1000, 1 << 20, (1 << 24) + 3])
def test_ladder_geometry_matches_reference_planner(kernel, n):
    # getNumBlocksAndThreads (cuda/C/src/reduction/reduction.cpp:272-291) exactly: sub-wave blocks
    # (t < 64) are allowed, their tail reduces over the active lanes only.
    C = native()
    mt, mb = 256, 64
    if kernel < 3:
        t = next_pow2(n) if n < mt else mt
        b = -(-n // t)
    else:
        t = next_pow2((n + 1) // 2) if n < 2 * mt else mt
        b = -(-n // (t * 2))
    if kernel == 6:
        b = min(mb, b)
    assert C.ladder_geometry(kernel, n, mt, mb) == (max(b, 1), t)


def test_compiled_variants_cover_grid():
    v = native().compiled_variants()
    plain = [s for s in v if "window" not in s]
    win = [s for s in v if "window" in s]
    assert len(plain) == 3 * 4 * 2  # block x unroll x policy
    # explicit windows: nt, 256/512 threads, unroll 2..8 divisible by the window
    assert len(win) == 2 * (3 + 2) and "block=256 unroll=4 policy=nt window=2" in v
    assert "block=512 unroll=16 policy=nt" in v
    # round 6: one body per plan ships (no software-pipelined variants)
    assert len(v) == len(plain) + len(win) and not any("pipelined" in s for s in v)


def test_single_hip_runtime_in_process():
    # Regression: importing the package before torch used to load /opt/rocm's libamdhip64 next to
    # torch's own copy (two HIP runtimes -> "no ROCm-capable device" on the GPU box).
    import subprocess
    import sys
    code = ("import cuda_mpi_reductions_amd, torch, re\n"
            "maps = open('/proc/self/maps').read()\n"
            "libs = sorted(set(re.findall(r'(/\\S*libamdhip64\\.so[.0-9]*)', maps)))\n"
            "print(len(libs), libs)\n")
    from helpers import ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("1 "), r.stdout


def test_default_xcd_skew_needs_a_whole_spx_device():
    # the default skew balances the 8 round-robin XCDs of a whole MI355X (SPX, 256 CUs);
    # a one-XCD partition (CPX, 32 CUs) or an unmeasured 2-4 XCD one gets none by default, while an
    # explicit skew still applies there
    C = native()
    assert C.plan(0, 10**9, F64, num_cus=256)["xskew"] == 19
    for cus in (32, 64, 128):
        p = C.plan(0, 10**9, F64, num_cus=cus)
        assert p["window"] == 4 and p["xskew"] == 0, (cus, p)
        assert C.plan(0, 10**9, F64, num_cus=cus, xcd_skew=20)["xskew"] > 0


def test_env_skew_overrides_only_the_default(monkeypatch):
    # MIREDUCE_XCD_SKEW replaces the tuned default, never a caller's explicit skew (bench.py's
    # plan-tuning candidates must run what their labels say)
    C = native()
    monkeypatch.setenv("MIREDUCE_XCD_SKEW", "40")
    assert C.plan(0, 10**9, F64)["xskew"] == 38
    assert C.plan(0, 10**9, F64, xcd_skew=0)["xskew"] == 0
    assert C.plan(0, 10**9, F64, xcd_skew=-20)["xskew"] == -19


def test_segmented_launch_plan():
    # round 5 (profiles/r5_hbmfill/): arrays above 16 GiB run as 8 GiB launches on the polled fan-in;
    # segment_bytes > 0 forces a size (1 MiB multiples), < 0 one launch; two-pass never segments; at
    # most min(256, max_grid) carried results (then the segments grow)
    C = native()
    F32 = 2
    hbm = C.plan(0, 73 * 10**9, F32)                      # the HBM-filling fp32 config: 292 GB
    assert hbm["segments"] == -(-73 * 10**9 // ((8 << 30) // 4)) == 34
    # equal whole-MiB segments of at most 8 GiB (no short tail segment)
    e = hbm["segment_elems"]
    assert e <= (8 << 30) // 4 and (e * 4) % (1 << 20) == 0 and 73 * 10**9 - 33 * e > 0.99 * e
    assert C.plan(0, 10**9, F64)["segments"] == 1         # the 8 GB headline: one launch
    assert C.plan(0, 2 * (8 << 30) // 8, F64)["segments"] == 1   # exactly 16 GiB: still one
    assert C.plan(0, 2 * (8 << 30) // 8 + 1, F64)["segments"] == 3
    forced = C.plan(0, 10**9, F64, segment_bytes=3 << 30)  # 8 GB in (at most) 3 GiB segments: 3 equal ones
    assert forced["segments"] == 3 and forced["segment_elems"] <= (3 << 30) // 8
    assert (forced["segment_elems"] * 8) % (1 << 20) == 0 and forced["segment_elems"] * 3 >= 10**9
    assert C.plan(0, 10**9, F64, segment_bytes=(3 << 30) + 12345)["segment_elems"] == forced["segment_elems"]
    assert C.plan(0, 73 * 10**9, F32, segment_bytes=-1)["segments"] == 1
    assert C.plan(0, 73 * 10**9, F32, single_pass=False)["segments"] == 1
    tiny = C.plan(0, 10**9, F64, segment_bytes=1 << 20)    # 7630 x 1 MiB would carry too many: larger segments
    assert tiny["segments"] <= 257 and tiny["segments"] * tiny["segment_elems"] >= 10**9
    assert C.plan(0, 10**9, F64, segment_bytes=1 << 20, max_grid=64)["segments"] <= 65
